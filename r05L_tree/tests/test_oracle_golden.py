"""Pin the CPU oracle against the golden vectors captured from the reference.

The oracle (oracle/dion_oracle.py) is the checker for every GPU parity test, so it
must first reproduce the reference's own outputs: it is fed the reference's
inputs and the exact sketch the reference drew, then W1/M1/Q1 and the captured
intermediates (P before/after RCQR, fixed-up R) are compared.  Same torch CPU
primitives on the same image, so the bar is 1e-6 max-relative (observed: 0).
"""
import pytest
import torch

from oracle import dion_oracle as O
from tests._golden import Case, case_names


def _maxrel(a, b):
    a = a.double()
    b = b.double()
    if torch.isnan(a).any() or torch.isnan(b).any():
        assert torch.equal(torch.isnan(a), torch.isnan(b))
        a = a.nan_to_num()
        b = b.nan_to_num()
    den = max(b.abs().max().item(), 1e-30)
    return (a - b).abs().max().item() / den


def _hyper(case):
    h = case.hyper
    return O.DionHyper(lr=h["lr"], mu=h["mu"], weight_decay=h["weight_decay"],
                       epsilon=h["epsilon"], rcqr_oversample=h["rcqr_oversample"],
                       scale_mode=h["scale_mode"], extra_scale_factor=h["extra_scale_factor"],
                       rank_fraction=case.rank_fraction)


def _run_oracle(case, shared_p_buffer=True):
    """Replay every step of the case through the oracle; return final per-rank states."""
    hyper = _hyper(case)
    names = [n for n, _, _ in case.mats]
    shapes = {n: (m, k) for n, m, k in case.mats}
    # case (viii): bf16 momentum and Q (stored as their exact fp32 values)
    sdt = torch.bfloat16 if case.entry.get("bf16") else torch.float32
    # independent momentum / Q dtypes (cases c13, c14; DionMixedPrecisionConfig)
    mdt = getattr(torch, case.entry["m_dtype"]) if "m_dtype" in case.entry else sdt
    qdt = getattr(torch, case.entry["q_dtype"]) if "q_dtype" in case.entry else sdt
    state = {}
    for rank in range(case.world):
        for n in names:
            state[(rank, n)] = dict(W=case.t(rank, 0, f"{n}_W0"), M=case.t(rank, 0, f"{n}_M0").to(mdt),
                                    Q=case.t(rank, 0, f"{n}_Q0").to(qdt))
    traces = {}
    for step in range(case.steps):
        for rank in range(case.world):
            for n in names:
                st = state[(rank, n)]
                # the fixture carries each step's inputs; they must equal our running state
                assert _maxrel(st["W"], case.t(rank, step, f"{n}_W0")) <= 1e-6
                st["G"] = case.t(rank, step, f"{n}_G")
        batches = case.batches(0, step)
        replicated = []
        for bi, b in enumerate(batches):
            real = int(b["real"])
            members = b["members"][:real]
            if case.world == 1:
                mats = []
                for n in members:
                    st = state[(0, n)]
                    m, k = shapes[n]
                    mats.append(O.DionMatrix(W=st["W"], M=st["M"], Q=st["Q"], G=st["G"],
                                             transposed=m < k, rank_fraction=case.rank_fraction))
                O.dion_batch_step_local(
                    mats, hyper,
                    sketch_fn=lambda i, p, _s=step: case.sketch_for(0, _s, p))
                for n, mt in zip(members, mats):
                    traces[(0, step, n)] = mt.trace
            else:
                B = case.world
                per_rank = []
                for rank in range(case.world):
                    row = []
                    for idx in range(B):
                        if idx < real:
                            n = members[idx]
                            st = state[(rank, n)]
                            m, k = shapes[n]
                            row.append(O.DionMatrix(W=st["W"], M=st["M"], Q=st["Q"], G=st["G"],
                                                    transposed=m < k,
                                                    rank_fraction=case.rank_fraction))
                        else:
                            n = members[0]
                            m, k = shapes[n]
                            st = state[(rank, n)]
                            row.append(O.DionMatrix(W=st["W"], M=torch.zeros(m, k, dtype=mdt),
                                                    Q=torch.zeros_like(st["Q"]),
                                                    G=torch.zeros(m, k), transposed=m < k,
                                                    rank_fraction=case.rank_fraction))
                    per_rank.append(row)
                replicated.append((per_rank, real, members))
        if replicated:
            O.dion_step_replicated(
                [(pr, real) for pr, real, _ in replicated], hyper,
                sketch_fn=lambda k, idx, p, _s=step: case.sketch_for(k, _s, p),
                reference_shared_p_buffer=shared_p_buffer)
            for per_rank, real, members in replicated:
                for rank in range(case.world):
                    for idx in range(real):
                        traces[(rank, step, members[idx])] = per_rank[rank][idx].trace
        for rank in range(case.world):
            for n in names:
                st = state[(rank, n)]
                yield step, rank, n, st, traces.get((rank, step, n))


@pytest.mark.parametrize("name", case_names())
def test_oracle_matches_reference_golden(name):
    case = Case(name)
    checked = 0
    for step, rank, n, st, tr in _run_oracle(case):
        for key, ref_key in (("W", "W1"), ("M", "M1"), ("Q", "Q1")):
            err = _maxrel(st[key], case.t(rank, step, f"{n}_{ref_key}"))
            assert err <= 1e-6, f"{name} step{step} rank{rank} {n}.{key} maxrel={err}"
            checked += 1
    assert checked > 0


def test_oracle_rank_and_sketch_rules():
    # state.py:183-188 with the Llama set at rank_fraction 1/64
    for m, n in ((6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)):
        assert O.rank_for_shape(m, n, 1 / 64) == 64
    assert O.rank_for_shape(17, 19, 0.5) == 9
    assert O.rank_for_shape(10, 10, 0.01) == 1
    assert O.rank_for_shape(10, 10, 0.35, rank_multiple_of=4) == 4
    assert O.sketch_rows(16) == 128 and O.sketch_rows(64) == 128
    assert O.sketch_rows(102) == 128 and O.sketch_rows(103) == 256 and O.sketch_rows(128) == 256
    assert O.use_low_rank_sync(4096, 4096, 64, 1 / 64)
    assert not O.use_low_rank_sync(32, 32, 32, 1.0)


def test_oracle_scaled_lr_known_answers():
    # tests/unit_tests/optimizer/test_dion_optimizer_contracts.py:1430-1458
    assert O.scaled_lr_for_shape(lr=1.0, m_global=16, n_global=4, scale_mode="spectral",
                                 rank_fraction=0.25) == pytest.approx(0.8)
    assert O.scaled_lr_for_shape(lr=1.0, m_global=16, n_global=4, scale_mode="unit_rms_norm",
                                 rank_fraction=0.25) == pytest.approx(0.8)
    assert O.scaled_lr_for_shape(lr=1.0, m_global=4, n_global=16, scale_mode="shape_scaling",
                                 rank_fraction=0.25) == pytest.approx(0.4)


def test_oracle_fixup_known_answer():
    # tests/unit_tests/optimizer/test_dion_optimizer_contracts.py:1314-1357
    nan = float("nan")
    P = torch.tensor([[[nan], [2.0]], [[1.0], [3.0]], [[nan], [7.0]]])
    R = torch.tensor([[[nan], [5.0], [6.0]], [[9.0], [10.0], [11.0]], [[nan], [12.0], [13.0]]])
    Q = torch.tensor([[[4.0], [5.0], [6.0]], [[nan], [8.0], [9.0]], [[20.0], [21.0], [nan]]])
    M = torch.ones((3, 2, 3))
    M[1].zero_()
    fp, fr = O.fix_all_zero_or_nan(P, R, Q, M, real_batch_size=2)
    assert torch.equal(fp[0], torch.tensor([[0.0], [2.0]]))
    assert torch.equal(fr[0], torch.tensor([[0.0], [5.0], [6.0]]))
    assert torch.equal(fp[1], torch.zeros((2, 1)))
    assert torch.equal(fr[1], torch.tensor([[0.0], [8.0], [9.0]]))
    assert torch.isnan(fp[2, 0, 0]) and fp[2, 1, 0].item() == 7.0
    assert torch.isnan(fr[2, 0, 0])
    assert torch.equal(fr[2, 1:], torch.tensor([[12.0], [13.0]]))


def test_reference_shared_p_buffer_defect_is_the_only_w2_difference():
    """c4 (W=2, two same-shape batches in flight) depends on the reference's
    unscoped "replicated_p_ortho_full" buffer (runtime.py:1419-1424): with it
    emulated the oracle is exact; with per-batch P (the intended Dion step, what
    the HIP path does) the first batch differs.  Single-batch W=2 (c8) is exact
    either way."""
    case = Case("c4_w2_pad3")
    diff = 0.0
    for step, rank, n, st, tr in _run_oracle(case, shared_p_buffer=False):
        diff = max(diff, _maxrel(st["W"], case.t(rank, step, f"{n}_W1")))
    assert diff > 1e-3
    case = Case("c8_w2_two_steps_T")
    for step, rank, n, st, tr in _run_oracle(case, shared_p_buffer=False):
        for key, ref_key in (("W", "W1"), ("M", "M1"), ("Q", "Q1")):
            assert _maxrel(st[key], case.t(rank, step, f"{n}_{ref_key}")) <= 1e-6


def test_w4_capture_is_the_per_batch_dion_step():
    """c15 (W = 4, one batch per shape): no two same-shape batches are in flight, so the
    reference's shared P buffer never aliases and the per-batch oracle (the HIP path's
    semantics) reproduces the capture exactly, padding on rank 3 included."""
    case = Case("c15_w4_pad_two_steps")
    assert case.world == 4
    for step in range(case.steps):
        # the reference's batch order (sorted batch-key reprs, batches.py:903-968); the padded
        # slot repeats the first member (its G, M, Q read as zero)
        assert [(b["members"], b["real"]) for b in case.batches(0, step)] == [
            (["t0", "t1", "t2", "t0"], 3), (["a0", "a1", "a2", "a3"], 4)]
    n = 0
    for step, rank, name, st, tr in _run_oracle(case, shared_p_buffer=False):
        for key, ref_key in (("W", "W1"), ("M", "M1"), ("Q", "Q1")):
            assert _maxrel(st[key], case.t(rank, step, f"{name}_{ref_key}")) <= 1e-6, (step, rank, name, key)
            n += 1
    assert n == 2 * 4 * 7 * 3
