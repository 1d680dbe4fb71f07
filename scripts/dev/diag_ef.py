import sys, os, torch
sys.path.insert(0, os.getcwd())
from megatron_dion_amd.codec import HipDionCodec
dev = torch.device("cuda", 0)
codec = HipDionCodec(dev)
def mr(a, b):
    a = a.double().cpu(); b = b.double().cpu()
    return (a - b).abs().max().item() / b.abs().max().item()
for (m, n, r, T) in ((512, 384, 64, False), (384, 1024, 64, True)):
    mp, nq = (n, m) if T else (m, n)
    g = torch.Generator().manual_seed(1)
    M = torch.randn(m, n, generator=g).to(dev) * 1e-3
    G = (torch.randn(m, n, generator=g) * 1e-3).to(torch.bfloat16).to(dev)
    Q = torch.randn(nq, r, generator=g).to(dev)
    Pp = torch.linalg.qr(torch.randn(mp, r, generator=g))[0].contiguous().to(dev)
    Rp = (torch.randn(nq, r, generator=g) * 1e-2).to(dev)
    alpha = -0.05
    ef = (Rp.double() @ Pp.double().t()) if T else (Pp.double() @ Rp.double().t())
    base = M.double() + G.double()
    M2 = M.clone(); P2 = torch.zeros(1, mp, r, device=dev); nz = torch.zeros(1, dtype=torch.int32, device=dev)
    codec.project_p_ef([G], [M2], [Q], P2, nz, T, [Pp], [Rp], alpha)
    M3 = M.clone(); P3 = torch.zeros(1, mp, r, device=dev)
    codec.project_p_ef([G], [M3], [Q], P3, nz, T, [None], [None], alpha)
    M1 = M.clone()
    codec.ef_apply([M1], None, Pp[None], Rp[None], [Q], torch.ones(1, dtype=torch.int32, device=dev), 0.95, 0, 0, 0, T)
    torch.cuda.synchronize()
    d = (M2.double() - base)
    print("shape", m, n, T)
    print(" noEF path vs M+G:", mr(M3, base), " eager EF vs M+aEF:", mr(M1, M.double() + alpha * ef))
    print(" fused vs M+G+aEF:", mr(M2, base + alpha * ef), " fused-base vs aEF:", mr(d, alpha * ef))
    dd = d.cpu(); e = (alpha * ef).cpu()
    # locate error pattern
    err = (dd - e).abs()
    idx = torch.nonzero(err > 1e-3 * e.abs().max())
    print(" bad count", idx.shape[0], "of", err.numel(), idx[:8].tolist())
    # rows/cols pattern
    if idx.shape[0]:
        print(" bad rows mod 16:", torch.bincount(idx[:, 0] % 16, minlength=16).tolist())
        print(" bad cols mod 32:", torch.bincount(idx[:, 1] % 32, minlength=32).tolist())
        i, j = idx[0].tolist()
        # is dd[i,j] equal to e at another position in the same 16x32 tile?
        ti, tj = i // 16 * 16, j // 32 * 32
        tile = e[ti:ti + 16, tj:tj + 32]
        w = torch.nonzero((tile - dd[i, j]).abs() < 1e-9 + 1e-4 * abs(dd[i, j].item()))
        print(" value at", (i, j), "found in tile at", (w + torch.tensor([ti, tj])).tolist()[:4])
