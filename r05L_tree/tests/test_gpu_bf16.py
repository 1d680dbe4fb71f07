"""GPU parity of the bf16-state Dion step (SURVEY 8c case viii; `pytest -m gpu`).

The speedrun's mixed precision (examples/dion/speedrun_nanogpt_mcore.py:422-431:
--dion-momentum-dtype / --dion-q-dtype bfloat16) keeps M and Q in bf16; P, R, the
error-feedback product and the update carry bf16 between stages (SURVEY Appendix A,
"Dtype propagation").  The HIP path (csrc/dion_bf16.hpp) rounds at the same points.

Evidence, all through MegatronDion.step and the C ABI:
  1. golden: the reference's own bf16 capture c11 (two steps, both orientations),
     replayed with the sketches the reference drew;
  2. oracle: seeded cases (bf16 / fp32 G, ragged shapes, a zero entry, split-K sizes)
     against the pinned CPU oracle run in bf16 (exact on c11/c12,
     tests/test_oracle_golden.py), same explicit sketches, three steps.

Tolerances.  torch's bf16 matmul and the MFMA accumulate the same exact bf16
products in fp32 in a different order, so an output that lands next to a bf16
rounding boundary can round the other way: single elements differ by one bf16 ulp
(2^-8 relative) and such flips propagate into the later stages.  Bars, written as
max |a - b| / max |b|:
  M (bf16)            <= 2^-6   (two ulps of the largest element; measured up to
                                 2^-7 after three steps, flips compound through the EF)
  W - W0 (the update) <= 2e-2
  W                   <= 1e-3
  Q (bf16, unit columns) <= 2e-2
"""
import math

import pytest
import torch

import megatron_dion_amd as mda
from megatron_dion_amd.optimizer import attach_dp_routing
from oracle import dion_oracle as O
from tests._golden import Case

pytestmark = pytest.mark.gpu

TOL_M = 2 ** -6
TOL_DW = 2e-2
TOL_W = 1e-3
TOL_Q = 2e-2
BF16 = mda.DionMixedPrecisionConfig(momentum_dtype=torch.bfloat16, q_dtype=torch.bfloat16)


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def maxrel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


@pytest.mark.parametrize("name", ["c11_bf16_two_steps_mixed", "c13_m32_q16_two_steps", "c14_m16_q32_two_steps"])
def test_bf16_golden_replay_through_optimizer(name):
    """c11: bf16 momentum and Q; c13 / c14: independent momentum / Q dtypes (a bf16 Q rounds
    Qn, so either way a product next to a bf16 rounding boundary may round the other way)."""
    dev = _dev()
    case = Case(name)
    mdt = getattr(torch, case.entry["m_dtype"]) if "m_dtype" in case.entry else torch.bfloat16
    qdt = getattr(torch, case.entry["q_dtype"]) if "q_dtype" in case.entry else torch.bfloat16
    h = case.hyper
    names = [n for n, _, _ in case.mats]
    params = {n: torch.nn.Parameter(case.t(0, 0, f"{n}_W0").to(dev)) for n in names}
    opt = mda.MegatronDion([params[n] for n in names], lr=h["lr"], mu=h["mu"], weight_decay=h["weight_decay"],
                           rank_fraction=case.rank_fraction, epsilon=h["epsilon"],
                           rcqr_oversample=h["rcqr_oversample"], scale_mode=h["scale_mode"],
                           extra_scale_factor=h["extra_scale_factor"], coalesce_local=False,
                           mixed_precision_config=mda.DionMixedPrecisionConfig(momentum_dtype=mdt, q_dtype=qdt))
    attach_dp_routing(opt, [(n, params[n]) for n in names])
    for n in names:
        st = opt.state[params[n]]
        assert st["momentum"].dtype == mdt and st["Q"].dtype == qdt
        assert st["r"] == case.r
        st["Q"].copy_(case.t(0, 0, f"{n}_Q0").to(dev))
    name_of = {id(params[n]): n for n in names}
    worst = {}
    for step in range(case.steps):
        for n in names:
            params[n].grad = case.t(0, step, f"{n}_G").to(dev)
        order = [b["members"][0] for b in case.batches(0, step)]
        calls = case.ortho_calls(0, step)
        sk = {m: calls[i]["S"] for i, m in enumerate(order)}
        opt._sketch_override = lambda batch, _sk=sk: {0: _sk[name_of[id(batch.params[0])]][0].to(dev)}
        w0 = {n: params[n].detach().clone() for n in names}
        opt.step()
        opt.flush_error_feedback()
        torch.cuda.synchronize()
        for n in names:
            p = params[n]
            st = opt.state[p]
            ref_w = case.t(0, step, f"{n}_W1")
            errs = dict(W=maxrel(p, ref_w), dW=maxrel(p - w0[n], ref_w.to(dev) - w0[n]),
                        M=maxrel(st["momentum"].float(), case.t(0, step, f"{n}_M1")),
                        Q=maxrel(st["Q"].float(), case.t(0, step, f"{n}_Q1")))
            for k, v in errs.items():
                worst[k] = max(worst.get(k, 0.0), v)
            assert errs["W"] <= TOL_W and errs["dW"] <= TOL_DW and errs["M"] <= TOL_M and errs["Q"] <= TOL_Q, \
                (step, n, errs)
    print(name, "worst errors", worst)


def _seeded(shapes, r, seed, gdt, zero=()):
    gen = torch.Generator().manual_seed(seed)
    out = []
    for i, (m, n) in enumerate(shapes):
        W = torch.randn(m, n, generator=gen) * 0.02
        qn = m if m < n else n
        Q = torch.randn(qn, r, generator=gen).to(torch.bfloat16)
        Gs = [(torch.randn(m, n, generator=gen) * 1e-3).to(gdt) for _ in range(3)]
        if i in zero:
            for G in Gs:
                G.zero_()
        out.append((W, Q, Gs))
    return out


CASES = [
    ("tall_bf16G", [(512, 384)] * 2, 64, torch.bfloat16, ()),
    ("wide_T_bf16G", [(384, 1024)] * 2, 64, torch.bfloat16, ()),
    ("ragged_f32G_r24", [(330, 203)] * 2, 24, torch.float32, ()),
    ("zero_entry_r16", [(256, 256)] * 3, 16, torch.bfloat16, (1,)),
    ("splitk_T_r32", [(1536, 4096)], 32, torch.bfloat16, ()),
]


@pytest.mark.parametrize("label,shapes,r,gdt,zero", CASES, ids=[c[0] for c in CASES])
def test_bf16_matches_oracle_three_steps(label, shapes, r, gdt, zero):
    dev = _dev()
    mats = _seeded(shapes, r, 11, gdt, zero)
    hyper = O.DionHyper(rank_fraction=r / min(shapes[0]))
    names = [f"w{i}" for i in range(len(mats))]
    params = {n: torch.nn.Parameter(W.to(dev)) for n, (W, _, _) in zip(names, mats)}
    opt = mda.MegatronDion([params[n] for n in names], lr=hyper.lr, mu=hyper.mu, weight_decay=hyper.weight_decay,
                           rank_fraction=hyper.rank_fraction, epsilon=hyper.epsilon, coalesce_local=False,
                           mixed_precision_config=BF16)
    attach_dp_routing(opt, [(n, params[n]) for n in names])
    cpu = {}
    for n, (W, Q, _) in zip(names, mats):
        st = opt.state[params[n]]
        assert st["r"] == r
        st["Q"].copy_(Q.to(dev))
        m, k = W.shape
        cpu[n] = O.DionMatrix(W=W.clone(), M=torch.zeros(m, k, dtype=torch.bfloat16), Q=Q.clone(), G=None,
                              transposed=m < k, rank_fraction=hyper.rank_fraction)
    name_of = {id(params[n]): n for n in names}
    kk = O.sketch_rows(r, hyper.rcqr_oversample)
    worst = {}
    for step in range(3):
        gen = torch.Generator().manual_seed(100 + step)
        sk = {}
        for n, (W, _, Gs) in zip(names, mats):
            m, k = W.shape
            mp = k if m < k else m
            sk[n] = torch.randn(1, kk, mp, generator=gen) * (1.0 / kk) ** 0.5
            params[n].main_grad = Gs[step].to(dev)  # Megatron grad-buffer view (bf16 or fp32)
            cpu[n].G = Gs[step].float()
        opt._sketch_override = lambda batch, _sk=sk: {0: _sk[name_of[id(batch.params[0])]][0].to(dev)}
        w0 = {n: params[n].detach().clone() for n in names}
        opt.step()
        torch.cuda.synchronize()
        for n in names:
            w_ref0 = cpu[n].W.clone()
            O.dion_batch_step_local([cpu[n]], hyper, sketch_fn=lambda i, p, _s=sk[n]: _s)
            p = params[n]
            st = opt.state[p]
            errs = dict(W=maxrel(p, cpu[n].W), dW=maxrel(p - w0[n], (cpu[n].W - w_ref0).to(dev)),
                        M=maxrel(st["momentum"].float(), cpu[n].M.float()),
                        Q=maxrel(st["Q"].float(), cpu[n].Q.float()))
            for k, v in errs.items():
                worst[k] = max(worst.get(k, 0.0), v)
            assert errs["W"] <= TOL_W and errs["dW"] <= TOL_DW and errs["M"] <= TOL_M and errs["Q"] <= TOL_Q, \
                (label, step, n, errs)
            if n in [names[i] for i in zero]:
                # all-zero momentum: M stays zero, W only decays, Q is the normalised old Q
                assert not st["momentum"].any()
    print(label, "bf16 worst errors", worst)


def test_bf16_round_kernel_is_rne():
    """dion_round_bf16 against torch's own fp32 -> bf16 conversion (bit-exact)."""
    dev = _dev()
    x = torch.randn(1 << 16, generator=torch.Generator().manual_seed(5)) * 1e3
    x[:8] = torch.tensor([0.0, -0.0, float("inf"), -float("inf"), 1.00390625, 1.01171875, 3.3895313e38, 1e-40])
    ref = x.to(torch.bfloat16).float()
    y = x.to(dev)
    opt = mda.MegatronDion([torch.nn.Parameter(torch.zeros(2, 2, device=dev))])
    opt.codec.round_bf16(y)
    torch.cuda.synchronize()
    assert torch.equal(y.cpu().view(torch.int32), ref.view(torch.int32))


@pytest.mark.parametrize("m,n", [(28672, 4096), (4096, 14336)])
def test_bf16_llama_shape_properties(m, n):
    """Full Llama-3-8B fc1 / fc2 matrices at r = 64 in the bf16 state mode, through the C ABI:
    exact rounding identities where the kernel's output is determined elementwise
    (M += G, bf16-valued factors), Freivalds probes for the products, orthonormal P."""
    from megatron_dion_amd.codec import HipDionCodec

    dev = _dev()
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.manual_seed(12)
    r = 64
    transposed = m < n
    mp, nq = (n, m) if transposed else (m, n)
    codec = HipDionCodec(dev)
    M = (torch.randn(m, n, device=dev) * 1e-3).to(torch.bfloat16)
    G = (torch.randn(m, n, device=dev) * 1e-3).to(torch.bfloat16)
    W = torch.randn(m, n, device=dev) * 0.02
    Q = torch.randn(nq, r, device=dev).to(torch.bfloat16)
    X0 = (M.float() + G.float()).to(torch.bfloat16)            # runtime.py:1560-1566 in bf16
    W0 = W.clone()
    P = torch.zeros(1, mp, r, device=dev)
    nz = torch.zeros(1, dtype=torch.int32, device=dev)
    codec.project_p([G], [M], [Q], P, nz, transposed)
    torch.cuda.synchronize()
    assert torch.equal(M, X0) and int(nz[0]) != 0
    assert torch.equal(P, P.to(torch.bfloat16).float())
    Xo = (X0.t() if transposed else X0).double()
    v = torch.randn(r, 1, device=dev, dtype=torch.float64)
    assert maxrel(P[0].double() @ v, Xo @ (Q.double() @ v)) <= 1e-2
    codec.orthonormalize(P, m, n, transposed, seed=99, state_dtype=torch.bfloat16)
    assert torch.equal(P, P.to(torch.bfloat16).float())
    I = P[0].double().t() @ P[0].double()
    assert (I - torch.eye(r, device=dev, dtype=torch.float64)).abs().max().item() <= 2e-2
    R = torch.zeros(1, nq, r, device=dev)
    codec.project_r([M], P, R, transposed)
    assert torch.equal(R, R.to(torch.bfloat16).float())
    assert maxrel(R[0].double() @ v, Xo.t() @ (P[0].double() @ v)) <= 1e-2
    Qs = [Q]
    codec.fixup_colnorm(P, R, Qs, nz, 1e-8, m, n, transposed)
    qn_ref = (R[0] / (R[0].square().sum(dim=0, keepdim=True).sqrt() + 1e-8)).to(torch.bfloat16)
    assert maxrel(Q.float(), qn_ref.float()) <= 2 ** -7
    Pb, Rb = P[0].to(torch.bfloat16).float(), R[0]
    s = 0.01 * 0.2 * math.sqrt(max(m, n))
    codec.ef_apply([M], [W], P, R, Qs, nz, 0.95, 0.01, 0.01, s, transposed)
    torch.cuda.synchronize()
    upd = (Rb @ Pb.t()) if transposed else (Pb @ Rb.t())        # kernels.py:54-83 in bf16
    upd = (upd.to(torch.bfloat16).float() * -(1.0 - 0.95)).to(torch.bfloat16)
    m_ref = (X0.float() + upd.float()).to(torch.bfloat16)
    assert maxrel(M.float(), m_ref.float()) <= 2 ** -7
    delta = (Q.float() @ Pb.t()) if transposed else (Pb @ Q.float().t())
    w_ref = W0 * (1 - 0.01 * 0.01) - s * delta.to(torch.bfloat16).float()
    assert maxrel(W, w_ref) <= 5e-3


@pytest.mark.parametrize("shapes,r", [([(512, 384)] * 2, 64), ([(384, 1024)] * 2, 64), ([(1536, 4096)], 32),
                                      ([(256, 512), (512, 256)], 32)],
                         ids=["rows_r64", "cols_T_r64", "splitk_T_r32", "both_r32"])
def test_bf16_deferred_ef_matches_eager(shapes, r):
    """The bf16 deferred-EF pass A (b16_row_ef_kernel / b16_col_ef_kernel) against the eager
    schedule (b16_stream_kernel EF + update) on the same inputs: same rounding points, the EF
    increment's fp32 sums in another MFMA order, so the tolerance bars above."""
    dev = _dev()
    mats = _seeded(shapes, r, 5, torch.bfloat16)
    runs = {}
    for defer in (False, True):
        names = [f"w{i}" for i in range(len(mats))]
        params = {n: torch.nn.Parameter(W.to(dev)) for n, (W, _, _) in zip(names, mats)}
        opt = mda.MegatronDion([params[n] for n in names], lr=0.01, mu=0.95, weight_decay=0.01,
                               rank_fraction=r / min(min(s) for s in shapes), coalesce_local=False,
                               mixed_precision_config=BF16, defer_error_feedback=defer)
        attach_dp_routing(opt, [(n, params[n]) for n in names])
        for n, (_, Q, _) in zip(names, mats):
            opt.state[params[n]]["Q"].copy_(Q.to(dev))
        m0, n0 = shapes[0]
        assert opt.codec.supports_deferred_ef(m0, n0, r, m0 < n0, state_dtype=torch.bfloat16,
                                              grad_dtype=torch.bfloat16)
        name_of = {id(params[n]): n for n in names}
        out = []
        for step in range(3):
            gen = torch.Generator().manual_seed(300 + step)
            sk = {}
            for n, (W, _, Gs) in zip(names, mats):
                mm, kk_ = W.shape
                mp = kk_ if mm < kk_ else mm
                sk[n] = torch.randn(1, O.sketch_rows(r, 1.25), mp, generator=gen) * (1.0 / O.sketch_rows(r, 1.25)) ** 0.5
                params[n].main_grad = Gs[step].to(dev)
            opt._sketch_override = lambda batch, _sk=sk: {0: _sk[name_of[id(batch.params[0])]][0].to(dev)}
            opt.step()
            opt.flush_error_feedback()
            torch.cuda.synchronize()
            out.append({n: (params[n].detach().clone(), opt.state[params[n]]["momentum"].float().clone(),
                            opt.state[params[n]]["Q"].float().clone()) for n in names})
        runs[defer] = out
    worst = {}
    for step in range(3):
        for n, (W, M, Q) in runs[True][step].items():
            We, Me, Qe = runs[False][step][n]
            errs = dict(W=maxrel(W, We), M=maxrel(M, Me), Q=maxrel(Q, Qe))
            for k, v in errs.items():
                worst[k] = max(worst.get(k, 0.0), v)
            assert errs["W"] <= TOL_W and errs["M"] <= TOL_M and errs["Q"] <= TOL_Q, (step, n, errs)
    print("bf16 deferred vs eager worst", worst)
