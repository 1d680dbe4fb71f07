"""Diagnose the h3 weight update: error of dion_ef_apply(M=None) vs fp64 by input family."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from megatron_dion_amd.codec import HipDionCodec

dev = torch.device("cuda", 0)
codec = HipDionCodec(dev)
out = {}
m, n, r = 512, 384, 64
for B in (1, 2):
    for logsp in (False, True):
        for wd in (0.0, 0.01):
            Ps, Qs = [], []
            for b in range(B):
                g = torch.Generator().manual_seed(3 + b)
                P = torch.linalg.qr(torch.randn(m, r, generator=g, dtype=torch.float64))[0].float()
                R = torch.randn(n, r, generator=g, dtype=torch.float64)
                if logsp:
                    R = R * torch.logspace(0, -3, r, dtype=torch.float64)
                Ps.append(P)
                Qs.append((R / (R.norm(dim=0, keepdim=True) + 1e-8)).float())
            s = 0.045
            Ws = [torch.zeros(m, n, device=dev) for _ in range(B)]
            codec.ef_apply(None, Ws, torch.stack(Ps).to(dev).contiguous(), torch.zeros(B, n, r, device=dev),
                           [q.to(dev).contiguous() for q in Qs], torch.ones(B, dtype=torch.int32, device=dev),
                           mu=0.95, lr=0.01, wd=wd, scaled_lr=s, transposed=False)
            torch.cuda.synchronize()
            errs = []
            for b in range(B):
                exact = -s * (Ps[b].double() @ Qs[b].double().T)
                E = (Ws[b].cpu().double() - exact).abs().numpy()
                mx = np.abs(exact.numpy()).max()
                errs.append(float(E.max() / mx))
                if b == B - 1:
                    key = f"B{B}_log{int(logsp)}_wd{wd}"
                    out[key] = {"err": errs,
                                "col_err": [float(E[:, j].max() / mx) for j in range(0, n, 8)],
                                "qcolnorm_min": float(Qs[b].norm(dim=0).min()),
                                "qmax_col": [float(Qs[b][:, k].abs().max()) for k in range(0, r, 8)]}
            print(key, errs, flush=True)
os.makedirs("gpurun_out", exist_ok=True)
with open("gpurun_out/diag_h3.json", "w") as f:
    json.dump(out, f, indent=1)
