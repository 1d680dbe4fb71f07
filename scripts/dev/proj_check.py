"""Dev check: projection accuracy of the loaded codec library against fp64 (set DION_LIB_PATH for a variant).
usage: python scripts/dev/proj_check.py [pb|pb_T|pa|pa_T] [m n r B]"""
import os, sys, torch
sys.path.insert(0, os.getcwd())
from megatron_dion_amd.codec import HipDionCodec

op = sys.argv[1] if len(sys.argv) > 1 else "pb"
m, n, r, B = (int(x) for x in sys.argv[2:6]) if len(sys.argv) > 5 else ((4096, 14336, 64, 2) if op.endswith("_T") else (28672, 4096, 64, 2))
T = m < n
mp, nq = (n, m) if T else (m, n)
dev = torch.device("cuda", 0)
codec = HipDionCodec(dev)
g = torch.Generator(device=dev).manual_seed(5)
Ms = [torch.randn(m, n, device=dev, generator=g) * 1e-3 for _ in range(B)]
# heterogeneous row/column magnitudes (x 1e3 spread) to stress the scaling
Ms[0].mul_(torch.logspace(-1.5, 1.5, m, device=dev)[:, None])
Ms[-1].mul_(torch.logspace(1.5, -1.5, n, device=dev)[None, :])
Qs = [torch.randn(nq, r, device=dev, generator=g) for _ in range(B)]
P = torch.linalg.qr(torch.randn(B, mp, r, device=dev, generator=g))[0].contiguous()
worst = 0.0
if op.startswith("pb"):
    R = torch.zeros(B, nq, r, device=dev)
    codec.project_r(Ms, P, R, T)
    torch.cuda.synchronize()
    for b in range(B):
        X = Ms[b].double().t() if T else Ms[b].double()
        ref = X.t() @ P[b].double()
        e = ((R[b].double() - ref).abs().max() / ref.abs().max()).item()
        ecol = ((R[b].double() - ref).abs().amax(0) / ref.abs().amax(0)).max().item()
        print(f"{op} b{b}: maxrel {e:.3e}  worst per-column rel {ecol:.3e}")
        worst = max(worst, e)
elif op.startswith("pa_ef"):
    Gs = [(torch.randn(m, n, device=dev, generator=g) * 1e-3).to(torch.bfloat16) for _ in range(B)]
    Pp = [torch.linalg.qr(torch.randn(mp, r, device=dev, generator=g))[0].contiguous() for _ in range(B)]
    Rp = [(torch.randn(nq, r, device=dev, generator=g) * 1e-2).contiguous() for _ in range(B)]
    Rp[0].mul_(torch.logspace(-2, 1, nq, device=dev)[:, None])
    alpha = -0.05
    X0 = [M.double().clone() for M in Ms]
    Pout = torch.zeros(B, mp, r, device=dev)
    nz = torch.zeros(B, dtype=torch.int32, device=dev)
    codec.project_p_ef(Gs, Ms, Qs, Pout, nz, T, Pp, Rp, alpha)
    torch.cuda.synchronize()
    for b in range(B):
        ef = (Rp[b].double() @ Pp[b].double().t()) if T else (Pp[b].double() @ Rp[b].double().t())
        Mref = X0[b] + alpha * ef + Gs[b].double()
        X = Mref.t() if T else Mref
        ref = X @ Qs[b].double()
        em = ((Ms[b].double() - Mref).abs().max() / Mref.abs().max()).item()
        e = ((Pout[b].double() - ref).abs().max() / ref.abs().max()).item()
        print(f"{op} b{b}: P maxrel {e:.3e}  M maxrel {em:.3e}")
        worst = max(worst, e, em)
else:
    Pout = torch.zeros(B, mp, r, device=dev)
    nz = torch.zeros(B, dtype=torch.int32, device=dev)
    X0 = [M.double().clone() for M in Ms]
    codec.project_p(None, Ms, Qs, Pout, nz, T)
    torch.cuda.synchronize()
    for b in range(B):
        X = X0[b].t() if T else X0[b]
        ref = X @ Qs[b].double()
        e = ((Pout[b].double() - ref).abs().max() / ref.abs().max()).item()
        print(f"{op} b{b}: maxrel {e:.3e}")
        worst = max(worst, e)
print(f"WORST {op} {worst:.3e}")
