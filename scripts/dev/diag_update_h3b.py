"""Seed sweep of the h3 weight update error (test factors vs diag factors)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from megatron_dion_amd.codec import HipDionCodec
from tests.test_gpu_update_precision import _factors

dev = torch.device("cuda", 0)
codec = HipDionCodec(dev)
m, n, r, s = 512, 384, 64, 0.045
for seed in (3, 4, 960, 977, 5, 100, 1000):
    for src in ("test", "diag"):
        if src == "test":
            P, Q = _factors(m, n, r, seed)
        else:
            g = torch.Generator().manual_seed(seed)
            P = torch.linalg.qr(torch.randn(m, r, generator=g, dtype=torch.float64))[0].float()
            R = torch.randn(n, r, generator=g, dtype=torch.float64) * torch.logspace(0, -3, r, dtype=torch.float64)
            Q = (R / (R.norm(dim=0, keepdim=True) + 1e-8)).float()
        W = torch.zeros(m, n, device=dev)
        codec.ef_apply(None, [W], P[None].to(dev).contiguous(), torch.zeros(1, n, r, device=dev), [Q.to(dev).contiguous()],
                       torch.ones(1, dtype=torch.int32, device=dev), mu=0.95, lr=0.01, wd=0.01, scaled_lr=s,
                       transposed=False)
        torch.cuda.synchronize()
        exact = -s * (P.double() @ Q.double().T)
        E = (W.cpu().double() - exact).abs()
        print(seed, src, float(E.max() / exact.abs().max()), float(P.abs().max()), float(Q.abs().max()),
              float(Q.abs().min()), flush=True)
