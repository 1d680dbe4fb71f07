"""dev: where does the transposed h3 pass A (colproj_efh3_kernel) lose precision?
EF only / G only / both, error pattern by row and column."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch
import megatron_dion_amd  # noqa: F401
from megatron_dion_amd.codec import HipDionCodec

dev = torch.device("cuda:0")
codec = HipDionCodec(dev)
g = torch.Generator().manual_seed(5)
for (m, n, r) in ((384, 1024, 64), (512, 384, 64)):
    tr = m < n
    mp, nq = (n, m) if tr else (m, n)
    for case in ("ef_only", "g_only", "both", "m_only"):
        M = torch.randn(m, n, generator=g) * 1e-3
        G = (torch.randn(m, n, generator=g) * 1e-3).to(torch.bfloat16)
        Q = torch.randn(nq, r, generator=g)
        Pp = torch.linalg.qr(torch.randn(mp, r, generator=g))[0].contiguous()
        Rp = torch.randn(nq, r, generator=g) * 1e-2
        if case == "ef_only":
            M.zero_(); G.zero_()
        if case == "g_only":
            M.zero_()
        use_ef = case in ("ef_only", "both")
        alpha = -0.05
        Md = M.clone().to(dev)
        P = torch.zeros(1, mp, r, device=dev)
        nz = torch.zeros(1, dtype=torch.int32, device=dev)
        codec.project_p_ef([G.to(dev)], [Md], [Q.to(dev)], P, nz, tr, [Pp.to(dev) if use_ef else None],
                           [Rp.to(dev) if use_ef else None], alpha)
        torch.cuda.synchronize()
        ef = (Rp.double() @ Pp.double().t()) if tr else (Pp.double() @ Rp.double().t())
        Mref = M.double() + (alpha * ef if use_ef else 0.0) + G.double()
        err = (Md.cpu().double() - Mref).abs()
        den = Mref.abs().max().item()
        print(f"{m}x{n} {case:8s} maxrel {err.max().item() / max(den, 1e-300):.3e}  "
              f"worst row {int(err.amax(1).argmax())} col {int(err.amax(0).argmax())}  "
              f"rows>1e-6: {int((err.amax(1) > 1e-6 * den).sum())}/{m} cols>1e-6: {int((err.amax(0) > 1e-6 * den).sum())}/{n}")
        if case == "ef_only":
            bad = (err.amax(0) > 1e-6 * den).nonzero().flatten().tolist()
            src = Pp if tr else Rp
            print("   bad cols", bad, "their factor-row max", [f"{src[c].abs().max().item():.3e}" for c in bad],
                  "global max", f"{src.abs().max().item():.3e}", "argmax row", int(src.abs().amax(1).argmax()))
            for c in bad[:2]:
                print("   col", c, "err/|ref col|max", f"{err[:, c].max().item() / Mref[:, c].abs().max().item():.3e}",
                      "signed err sample", [f"{v:.2e}" for v in (Md.cpu().double() - Mref)[:4, c].tolist()],
                      "ref", [f"{v:.2e}" for v in Mref[:4, c].tolist()])
            e2 = err[:, :]
            print("   err by row block of 32:", [f"{e2[i:i+32].max().item()/den:.1e}" for i in range(0, m, 32)][:12])
            print("   err by col block of 32:", [f"{e2[:, j:j+32].max().item()/den:.1e}" for j in range(0, n, 32)][:12])
