"""Precision of the weight update alone (`pytest -m gpu`).

`dion_ef_apply(M=None, W, P, R, Qn)` is the deferred-EF schedule's weight update,
W <- W (1 - lr wd) - s P Qn^T (transposed: - s Qn P^T), dion/kernels.py:229-276 and
dion/runtime.py:1105-1113.  The full-step tests score W as max|dW| / max|W|, which one
step's update (~1e-3 of W) cannot move; here the update is scored on its own:

  err = max |W1_hip - W1_exact| / max |s P Qn^T|,   W1_exact = fp32(W0 d) - s P Qn^T in fp64

With W0 = 0 the score is the product's own error; with W0 != 0 the final fp32 rounding of
W1 (half an ulp of |W1|) is subtracted per element first, so only the update's error is
left.  Bar: 1e-6 of max |s P Qn^T| (fp32-grade: the reference computes P Qn^T as one fp32
GEMM, whose own error is ~sqrt(r) 2^-24 of the row/column norms).
"""
import json
import os

import numpy as np
import pytest
import torch

from megatron_dion_amd.codec import HipDionCodec

pytestmark = pytest.mark.gpu

TOL_UPDATE = 1e-6
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_RESULTS = {}


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _factors(mp, nq, r, seed):
    """P: orthonormal columns (the RCQR output); Qn: unit columns (the column norm's output)."""
    g = torch.Generator().manual_seed(seed)
    P = torch.linalg.qr(torch.randn(mp, r, generator=g, dtype=torch.float64))[0].float()
    R = torch.randn(nq, r, generator=g, dtype=torch.float64) * torch.logspace(0, -3, r, dtype=torch.float64)
    Qn = (R / (R.norm(dim=0, keepdim=True) + 1e-8)).float()
    return P, Qn


def _ulp_half(x):
    x = np.abs(np.asarray(x, dtype=np.float32))
    return (np.nextafter(x, np.float32(np.inf)) - x).astype(np.float64) / 2


def _record(key, val):
    _RESULTS[key] = val
    out = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "update_precision.json"), "w") as f:
            json.dump(_RESULTS, f, indent=1)


CASES = [
    # (m, n, r, transposed, s, w0)
    (512, 384, 64, False, 0.045, 0.0),
    (512, 384, 64, False, 0.045, 0.02),
    (384, 1024, 64, True, 0.045, 0.0),
    (384, 1024, 64, True, 0.045, 0.02),
    (1024, 512, 128, False, 3.0, 0.0),
    (512, 1024, 128, True, 1e-4, 0.0),
    (4096, 4096, 64, False, 0.128, 0.02),
    (4096, 14336, 64, True, 0.24, 0.0),
    (14336, 4096, 128, False, 0.24, 0.02),
    # r = 128 LDS-DMA update (columns a multiple of 256): a 5-step and a 1-strip-block run; and
    # the register-staged kernel it falls back to (416 columns)
    (160, 768, 128, False, 0.5, 0.02),
    (2048, 256, 128, False, 0.3, 0.02),
    (512, 416, 128, False, 0.5, 0.02),
]


@pytest.mark.parametrize("m,n,r,transposed,s,w0", CASES)
def test_weight_update_alone_vs_fp64(m, n, r, transposed, s, w0):
    dev = _dev()
    codec = HipDionCodec(dev)
    mp, nq = (n, m) if transposed else (m, n)
    B = 2
    Ps, Qs, Ws = [], [], []
    for b in range(B):
        P, Qn = _factors(mp, nq, r, 17 * b + m + n + r)
        Ps.append(P)
        Qs.append(Qn)
        g = torch.Generator().manual_seed(5 + b)
        Ws.append(torch.randn(m, n, generator=g) * w0)
    lr, wd = 0.01, 0.01
    decay = np.float32(1.0 - lr * wd)
    Pd = torch.stack(Ps).to(dev).contiguous()
    Rd = torch.zeros(B, nq, r, device=dev)
    Wd = [w.to(dev).contiguous() for w in Ws]
    Qd = [q.to(dev).contiguous() for q in Qs]
    nz = torch.ones(B, dtype=torch.int32, device=dev)
    codec.ef_apply(None, Wd, Pd, Rd, Qd, nz, mu=0.95, lr=lr, wd=wd, scaled_lr=s, transposed=transposed)
    torch.cuda.synchronize()
    worst = 0.0
    for b in range(B):
        P64, Q64 = Ps[b].double(), Qs[b].double()
        upd = s * (Q64 @ P64.T if transposed else P64 @ Q64.T)
        base = (Ws[b].numpy() * decay).astype(np.float32).astype(np.float64)
        exact = base - upd.numpy()
        got = Wd[b].cpu().numpy().astype(np.float64)
        diff = np.abs(got - exact) - (_ulp_half(exact) if w0 != 0.0 else 0.0)
        err = max(float(diff.max()), 0.0) / float(np.abs(upd.numpy()).max())
        worst = max(worst, err)
    _record(f"{m}x{n}_r{r}_T{int(transposed)}_s{s}_w{w0}", worst)
    assert worst <= TOL_UPDATE, (m, n, r, transposed, s, w0, worst)
