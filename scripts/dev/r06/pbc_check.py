"""Dev: pass B (project_r) of this tree's library against a variant build (DION_LIB_PATH-style
second library, default: the register kernels) on the same inputs, both orientations, with
and without pass A's max |M| (fixed-scale / per-step-scale paths)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)
from megatron_dion_amd import _lib  # noqa: E402
from megatron_dion_amd.codec import HipDionCodec  # noqa: E402

var = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "megatron-dion_amd/csrc/variants/libdion_codec_pbc0.so")
dev = torch.device("cuda", 0)
a = HipDionCodec(dev)
b = HipDionCodec(dev)
b.lib = _lib.load(var)
for (m, n, r) in [(640, 512, 128), (2048, 1024, 64), (2048, 1024, 128), (1792, 256, 128), (6144, 4096, 64),
                  (1024, 2048, 64), (1024, 2048, 128), (512, 640, 128)]:
    tr = m < n
    mp, nq = (n, m) if tr else (m, n)
    B = 3
    g = torch.Generator().manual_seed(m + n + r)
    Ms = [(torch.randn(m, n, generator=g) * 1e-2).to(dev) for _ in range(B)]
    P = torch.linalg.qr(torch.randn(B, mp, r, generator=g))[0].to(dev).contiguous()
    amax = torch.stack([M.abs().max() for M in Ms]).float().cpu()
    nz = amax.view(torch.int32).clone().to(dev)
    ref = torch.stack([(M.double().t() if tr else M.double()).t() @ P[i].double() for i, M in enumerate(Ms)])
    for fixed in (True, False):
        Ra = torch.zeros(B, nq, r, device=dev)
        Rb = torch.zeros(B, nq, r, device=dev)
        kw = {"nonzero": nz} if fixed else {}
        a.project_r(Ms, P, Ra, tr, **kw)
        b.project_r(Ms, P, Rb, tr, **kw)
        torch.cuda.synchronize()
        ea = ((Ra.double() - ref.cpu().to(dev)).abs().max() / ref.abs().max()).item()
        eb = ((Rb.double() - ref.cpu().to(dev)).abs().max() / ref.abs().max()).item()
        bad = (Ra.double() - ref.to(dev)).abs().amax(dim=2)
        rows = torch.nonzero(bad[0] > 1e-3 * ref.abs().max().item()).flatten().tolist()[:12]
        print(f"{m}x{n} r={r} T={int(tr)} fixed={int(fixed)}: tree {ea:.2e} variant {eb:.2e} bad rows(entry0) {rows}",
              flush=True)
