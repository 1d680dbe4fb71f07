"""Dev: one r = 128 deferred-EF pass A (fc1 shape, 2 matrices) with the library named by
DION_LIB_PATH; saves M, P and the flags to gpurun_out/diag_<tag>.pt for comparison."""
import os, sys, torch
sys.path.insert(0, os.getcwd())
from megatron_dion_amd.codec import HipDionCodec
tag = sys.argv[1]
dev = torch.device("cuda", 0)
codec = HipDionCodec(dev)
B, m, n, r = 2, 512, 1024, 128
g = torch.Generator().manual_seed(0)
Ms = [(torch.randn(m, n, generator=g) * 1e-3).to(dev) for _ in range(B)]
Gs = [(torch.randn(m, n, generator=g) * 1e-3).to(torch.bfloat16).to(dev) for _ in range(B)]
Qs = [torch.randn(n, r, generator=g).to(dev) for _ in range(B)]
Pp = (torch.randn(B, m, r, generator=g) * 0.01).to(dev)
Rp = (torch.randn(B, n, r, generator=g) * 0.01).to(dev)
P = torch.zeros(B, m, r, device=dev)
nz = torch.zeros(B, dtype=torch.int32, device=dev)
codec.project_p_ef(Gs, Ms, Qs, P, nz, False, [Pp[i] for i in range(B)], [Rp[i] for i in range(B)], -0.05)
torch.cuda.synchronize()
torch.save({"M": [x.cpu() for x in Ms], "P": P.cpu(), "nz": nz.cpu()}, f"gpurun_out/diag_{tag}.pt")
print("saved", tag)
