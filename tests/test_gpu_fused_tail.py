"""The fused orthonormalisation tail against the unfused calls, through the C ABI (`-m gpu`).

The W = 1 fp32 path calls dion_orthonormalize_fused (the fix-up of P in the last solve, pass
B's fixed-scale split of P written beside it) and dion_project_r_fixup; since round 6 the W > 1
path calls dion_orthonormalize on the owner rank and, after the all-gather, dion_pfix_split
(the fix-up's P half with the local zero test + the same split) and dion_project_r_split.  Here
one batch runs three ways from the same P0 and generated sketch:

  A  orthonormalize_fused(fix, split)  -> project_r_fixup(split)                  (W = 1 path)
  B  orthonormalize -> pfix_split(fix, split) -> project_r(split) -> fixup(P=None) (W > 1 path)
  C  orthonormalize -> project_r (measured-scale split of P) -> fixup_colnorm(P)  (unfused)

A and B must agree bit for bit (P, the split, R, Q): they run the same arithmetic with the
fix-up and the split in other launches.  C differs only in pass B's scale for P (one measured
power of two per matrix instead of the fixed 2^14), so R and Q agree to fp32 level.  Each
batch has an all-zero entry (nonzero 0: P -> 0, R -> nan_to_num(Q)) and an entry whose P has a
zero column, which the Cholesky QR turns into NaN columns (the fix-up zeroes them).  r = 16 has
no fused split (trsm_right_kernel's fix only); r = 128 splits after the last solve.
(the fused FINAL epilogues per r were never compared with the unfused sequence.)
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.mark.parametrize("r", [16, 32, 64, 128])
@pytest.mark.parametrize("transposed", [False, True], ids=["rows", "transposed"])
def test_fused_tail_is_the_unfused_sequence(r, transposed):
    from megatron_dion_amd.codec import HipDionCodec

    dev = _dev()
    m, n = (1024, 2048) if transposed else (2048, 1024)
    mp, nq = (n, m) if transposed else (m, n)
    B = 4
    gen = torch.Generator().manual_seed(r + 7 * int(transposed))
    Ms = [(torch.randn(m, n, generator=gen) * 1e-2).to(dev) for _ in range(B)]
    P0 = torch.randn(B, mp, r, generator=gen) * 1e-2
    P0[2, :, r // 2] = 0.0  # a zero column: the Cholesky QR gives NaN columns from it on
    P0 = P0.to(dev).contiguous()
    Q0 = [torch.randn(nq, r, generator=gen).to(dev) for _ in range(B)]
    amax = torch.stack([M.abs().max() for M in Ms]).float().cpu()
    nz = amax.view(torch.int32).clone()
    nz[1] = 0  # an all-zero momentum by its flag
    nz = nz.to(dev)
    eps, seed = 1e-8, 1234
    codec = HipDionCodec(dev)
    split_a = codec.psplit_buffer(B, m, n, r, transposed)
    split_b = codec.psplit_buffer(B, m, n, r, transposed)
    assert (split_a is None) == (r == 16)

    # A: the W = 1 path
    Pa = P0.clone()
    codec.orthonormalize(Pa, m, n, transposed, seed, fix_nonzero=nz, p_split=split_a)
    Ra = torch.empty(B, nq, r, device=dev)
    Qa = [q.clone() for q in Q0]
    codec.project_r_fixup(Ms, Pa, Ra, Qa, nz, eps, transposed, **({} if split_a is None else {"p_split": split_a}))
    # B: the W > 1 path's calls (owner orthonormalises, every rank fixes and splits)
    Pb = P0.clone()
    codec.orthonormalize(Pb, m, n, transposed, seed)
    raw = Pb.clone()
    codec.pfix_split(Pb, m, n, transposed, nz, split_b)
    Rb = torch.empty(B, nq, r, device=dev)
    Qb = [q.clone() for q in Q0]
    codec.project_r(Ms, Pb, Rb, transposed, nonzero=nz, **({} if split_b is None else {"p_split": split_b}))
    codec.fixup_colnorm(None, Rb, Qb, nz, eps, m, n, transposed)
    # C: unfused, pass B splitting P on its measured scale
    Pc = raw.clone()
    Rc = torch.empty(B, nq, r, device=dev)
    Qc = [q.clone() for q in Q0]
    codec.project_r(Ms, Pc, Rc, transposed, nonzero=nz)
    codec.fixup_colnorm(Pc, Rc, Qc, nz, eps, m, n, transposed)
    torch.cuda.synchronize()

    raw = raw.cpu()
    assert torch.isnan(raw[2]).any(), "the zero column should have produced NaN columns"
    assert not torch.isnan(raw[0]).any() and not torch.isnan(raw[3]).any()
    assert torch.equal(Pa.cpu(), Pb.cpu()) and torch.equal(Pb.cpu(), Pc.cpu())
    assert (Pa[1] == 0).all() and torch.isfinite(Pa).all()
    if split_a is not None:
        assert torch.equal(split_a.cpu(), split_b.cpu())
    assert torch.equal(Ra.cpu(), Rb.cpu())
    for a, b in zip(Qa, Qb):
        assert torch.equal(a.cpu(), b.cpu())
    assert torch.equal(Ra[1].cpu(), Q0[1].cpu())  # R of the zero entry is Q (kernels.py:193)
    scale = Rc.abs().max().item()
    assert (Ra - Rc).abs().max().item() <= 2e-6 * scale
    for a, c in zip(Qa, Qc):
        assert (a - c).abs().max().item() <= 2e-6


@pytest.mark.parametrize("r,transposed", [(64, False), (128, True)])
def test_row_sparse_p_follows_the_header_contract(r, transposed):
    """a row-sparse P (one nonzero row) makes the Cholesky QR overflow (the oracle's
    orthogonalize returns +-inf there; the reference's nan_to_num then feeds FLT_MAX into R and the
    update, which is not finite either).  include/dion_codec.h (dion_pfix_split) states what the
    fused path does instead: the fix-up makes P finite (NaN -> 0, +-inf -> +-FLT_MAX, as
    nan_to_num), the split of an entry past the fixed scale's range is inf / NaN, so its R column
    is fixed to 0 where the unfused pass B would rescale.  Pinned here: the fused and the W > 1
    sequences agree bit for bit, and P, R and Q are finite."""
    from megatron_dion_amd.codec import HipDionCodec

    dev = _dev()
    m, n = (1024, 2048) if transposed else (2048, 1024)
    mp, nq = (n, m) if transposed else (m, n)
    B = 2
    gen = torch.Generator().manual_seed(5 + r)
    Ms = [(torch.randn(m, n, generator=gen) * 1e-2).to(dev) for _ in range(B)]
    P0 = torch.zeros(B, mp, r)
    P0[:, 7] = torch.randn(B, r, generator=gen)  # one nonzero row
    P0 = P0.to(dev).contiguous()
    Q0 = [torch.randn(nq, r, generator=gen).to(dev) for _ in range(B)]
    nz = torch.stack([M.abs().max() for M in Ms]).float().cpu().view(torch.int32).clone().to(dev)
    codec = HipDionCodec(dev)
    sa = codec.psplit_buffer(B, m, n, r, transposed)
    sb = codec.psplit_buffer(B, m, n, r, transposed)
    Pa = P0.clone()
    codec.orthonormalize(Pa, m, n, transposed, 99, fix_nonzero=nz, p_split=sa)
    Ra = torch.empty(B, nq, r, device=dev)
    Qa = [q.clone() for q in Q0]
    codec.project_r_fixup(Ms, Pa, Ra, Qa, nz, 1e-8, transposed, p_split=sa)
    Pb = P0.clone()
    codec.orthonormalize(Pb, m, n, transposed, 99)
    codec.pfix_split(Pb, m, n, transposed, nz, sb)
    Rb = torch.empty(B, nq, r, device=dev)
    Qb = [q.clone() for q in Q0]
    codec.project_r(Ms, Pb, Rb, transposed, nonzero=nz, p_split=sb)
    codec.fixup_colnorm(None, Rb, Qb, nz, 1e-8, m, n, transposed)
    torch.cuda.synchronize()
    assert torch.equal(Pa.cpu(), Pb.cpu()) and torch.equal(sa.cpu(), sb.cpu()) and torch.equal(Ra.cpu(), Rb.cpu())
    assert torch.isfinite(Pa).all() and torch.isfinite(Ra).all()
    for a, b in zip(Qa, Qb):
        assert torch.equal(a.cpu(), b.cpu()) and torch.isfinite(a).all()


@pytest.mark.parametrize("m,n,r", [(256, 800, 64), (544, 256, 128), (256, 544, 128), (800, 256, 128),
                                   (256, 8224, 64), (8224, 256, 128)])
def test_lds_dma_pass_b_ragged_k_chunks(m, n, r):
    """Round 6's LDS-DMA pass-B kernels (rowproj_h3gl transposed at r = 64 / 128, colproj_h3gl
    not transposed at r = 128) on contraction lengths whose split-K chunks end in short runs of
    32-column steps (fewer steps than the staging depth, a last chunk shorter than the others),
    against fp64, in both scale modes (pass A's max |M|: one scale per matrix; none: per-step
    scales)."""
    from megatron_dion_amd.codec import HipDionCodec

    dev = _dev()
    tr = m < n
    mp, nq = (n, m) if tr else (m, n)
    B = 3
    gen = torch.Generator().manual_seed(m * 7 + n + r)
    Ms = [(torch.randn(m, n, generator=gen) * 1e-2).to(dev) for _ in range(B)]
    P = torch.linalg.qr(torch.randn(B, mp, r, generator=gen, dtype=torch.float64))[0].float().to(dev).contiguous()
    nz = torch.stack([M.abs().max() for M in Ms]).float().cpu().view(torch.int32).clone().to(dev)
    ref = torch.stack([(M.double().t() if tr else M.double()).t() @ P[i].double() for i, M in enumerate(Ms)])
    codec = HipDionCodec(dev)
    for kw in ({"nonzero": nz}, {}):
        R = torch.zeros(B, nq, r, device=dev)
        codec.project_r(Ms, P, R, tr, **kw)
        torch.cuda.synchronize()
        err = ((R.double() - ref).abs().max() / ref.abs().max()).item()
        assert err <= 1e-6, (m, n, r, bool(kw), err)
