"""dev: read back the effective EF factor of colproj_efh3_kernel: with R' = [I; 0] the updated
M's first r rows are alpha * P'^T, so every lane's split of P' is visible."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch
import megatron_dion_amd  # noqa: F401
from megatron_dion_amd.codec import HipDionCodec

dev = torch.device("cuda:0")
codec = HipDionCodec(dev)
g = torch.Generator().manual_seed(5)
m, n, r = 384, 1024, 64
mp, nq = n, m
M = torch.randn(m, n, generator=g) * 1e-3
G = (torch.randn(m, n, generator=g) * 1e-3).to(torch.bfloat16)
Q = torch.randn(nq, r, generator=g)
Pp = torch.linalg.qr(torch.randn(mp, r, generator=g))[0].contiguous()
Rp = torch.zeros(nq, r)
Rp[:r] = torch.eye(r)
alpha = -0.05
Md = torch.zeros(m, n, device=dev)
P = torch.zeros(1, mp, r, device=dev)
nz = torch.zeros(1, dtype=torch.int32, device=dev)
codec.project_p_ef([torch.zeros(m, n, dtype=torch.bfloat16, device=dev)], [Md], [Q.to(dev)], P, nz, True,
                   [Pp.to(dev)], [Rp.to(dev)], alpha)
torch.cuda.synchronize()
F = Md[:r].cpu().double().t() / alpha        # (n, r): effective P'
ref = Pp.double()
rel = (F - ref).abs() / ref.abs().clamp_min(1e-30)
bad = (rel > 1e-6).nonzero().tolist()
print("bad (row, k) entries:", len(bad), bad[:20])
for (j, k) in bad[:10]:
    print(f"  P'[{j}][{k}] = {ref[j, k].item():.9e}  kernel {F[j, k].item():.9e}  rel {rel[j, k].item():.2e}")
print("rows with bad:", sorted({j for j, _ in bad})[:40])
print("k with bad:", sorted({k for _, k in bad})[:64])
