"""World-size-2 gloo tests of the replicate (DP) exchange schedule on CPU.

The product's batch runtime (megatron_dion_amd/runtime.py) runs unchanged --
batching, padding, reduce-scatter(avg) of P, owner-rank orthonormalisation,
all-gather of P, all-reduce(avg) of R, AsyncRuntime interleave -- with the
test-only oracle codec (tests/_cpu_codec.py) in place of the HIP kernels, so the
N > 1 path is covered without GPUs.  Checked against the reference's own
2-rank golden captures (c8: exact; c4: the intended per-batch-P semantics, see
test_oracle_golden.test_reference_shared_p_buffer_defect_is_the_only_w2_difference).
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.slow


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, name, out_dir, deferred=False):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    import megatron_dion_amd as mda
    from megatron_dion_amd.optimizer import attach_dp_routing
    from tests._cpu_codec import OracleCodec
    from tests._golden import Case

    case = Case(name)
    h = case.hyper
    names = [n for n, _, _ in case.mats]
    params = {n: torch.nn.Parameter(case.t(rank, 0, f"{n}_W0").clone()) for n in names}
    state = {"step": 0}
    codec = OracleCodec(sketch_lookup=lambda P: case.sketch_for(rank, state["step"], P), deferred=deferred)
    # case (viii): the speedrun's bf16 momentum and Q
    mpc = mda.DionMixedPrecisionConfig(momentum_dtype=torch.bfloat16, q_dtype=torch.bfloat16) \
        if case.entry.get("bf16") else None
    opt = mda.MegatronDion([params[n] for n in names], lr=h["lr"], mu=h["mu"], weight_decay=h["weight_decay"],
                           rank_fraction=case.rank_fraction, epsilon=h["epsilon"],
                           rcqr_oversample=h["rcqr_oversample"], codec=codec, defer_error_feedback=deferred,
                           mixed_precision_config=mpc)
    attach_dp_routing(opt, [(n, params[n]) for n in names], replicate_group=dist.group.WORLD)
    for n in names:
        opt.state[params[n]]["Q"].copy_(case.t(rank, 0, f"{n}_Q0"))
    results = {}
    for step in range(case.steps):
        state["step"] = step
        for n in names:
            params[n].grad = case.t(rank, step, f"{n}_G").clone()
        batches, _ = opt._route_step_params()
        results[f"s{step}_schedule"] = [([e.dist_meta.param_name if e.dist_meta else "<pad>"
                                          for e in b.entries], b.real_batch_size) for b in batches]
        opt.step()
        if deferred and step == case.steps - 1:
            opt.flush_error_feedback()
        for n in names:
            results[f"s{step}_{n}_W"] = params[n].detach().clone()
            results[f"s{step}_{n}_M"] = opt.state[params[n]]["momentum"].clone()
            results[f"s{step}_{n}_Q"] = opt.state[params[n]]["Q"].clone()
    torch.save(results, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _run(name, world=2, deferred=False):
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_worker, args=(world, _free_port(), name, tmp, deferred), nprocs=world, join=True,
                           start_method="spawn")
        return [torch.load(os.path.join(tmp, f"rank{r}.pt"), weights_only=True) for r in range(world)]


def _maxrel(a, b):
    return (a.double() - b.double()).abs().max().item() / max(b.double().abs().max().item(), 1e-30)


@pytest.mark.parametrize("deferred", [False, True], ids=["eager_ef", "deferred_ef"])
def test_gloo_w2_matches_reference_single_batch(deferred):
    from tests._golden import Case

    case = Case("c8_w2_two_steps_T")
    res = _run(case.name, deferred=deferred)
    names = [n for n, _, _ in case.mats]
    for rank in range(2):
        for step in range(case.steps):
            assert res[rank][f"s{step}_schedule"] == [(["x", "y"], 2)]
            for n in names:
                keys = (("W", "W1"), ("Q", "Q1"))
                if not deferred or step == case.steps - 1:
                    keys += (("M", "M1"),)
                for k, ref in keys:
                    err = _maxrel(res[rank][f"s{step}_{n}_{k}"], case.t(rank, step, f"{n}_{ref}"))
                    assert err <= 1e-6, (rank, step, n, k, err)
    # replicas agree bit-for-bit on W and Q; momentum stays rank-local
    for n in names:
        assert torch.equal(res[0][f"s1_{n}_W"], res[1][f"s1_{n}_W"])
        assert torch.equal(res[0][f"s1_{n}_Q"], res[1][f"s1_{n}_Q"])
        assert not torch.equal(res[0][f"s1_{n}_M"], res[1][f"s1_{n}_M"])


def test_gloo_w2_bf16_state_matches_reference():
    """Case (viii) at world size 2: bf16 momentum and Q through the product runtime
    (reduce-scatter / all-gather of P, all-reduce of R, each average rounded back to
    bf16) against the reference's 2-rank bf16 capture c12.  The CPU codec's bf16
    products accumulate in another order than the reference's bf16 matmul, so single
    bf16 roundings may differ: bar 1 bf16 ulp of the largest element (2^-8)."""
    from tests._golden import Case

    case = Case("c12_bf16_w2_two_steps_T")
    res = _run(case.name)
    names = [n for n, _, _ in case.mats]
    for rank in range(2):
        for step in range(case.steps):
            for n in names:
                assert res[rank][f"s{step}_{n}_M"].dtype == torch.bfloat16
                assert res[rank][f"s{step}_{n}_Q"].dtype == torch.bfloat16
                for k, ref in (("W", "W1"), ("M", "M1"), ("Q", "Q1")):
                    err = _maxrel(res[rank][f"s{step}_{n}_{k}"].float(), case.t(rank, step, f"{n}_{ref}"))
                    assert err <= 2 ** -8, (rank, step, n, k, err)
    for n in names:
        assert torch.equal(res[0][f"s1_{n}_W"], res[1][f"s1_{n}_W"])
        assert torch.equal(res[0][f"s1_{n}_Q"], res[1][f"s1_{n}_Q"])


def test_gloo_w2_padding_and_per_batch_p():
    from tests._golden import Case
    from tests.test_oracle_golden import _run_oracle

    case = Case("c4_w2_pad3")
    res = _run(case.name)
    # reference schedule: [a, b] then [c, <pad>] (batches.py:903-968)
    assert res[0]["s0_schedule"] == [(["a", "b"], 2), (["c", "<pad>"], 1)]
    assert res[1]["s0_schedule"] == res[0]["s0_schedule"]
    for step, rank, n, st, _ in _run_oracle(case, shared_p_buffer=False):
        for k in ("W", "M", "Q"):
            err = _maxrel(res[rank][f"s{step}_{n}_{k}"], st[k])
            assert err <= 1e-6, (rank, n, k, err)


def _coalesce_worker(rank, world, port, out_dir, deferred):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    import megatron_dion_amd as mda
    from megatron_dion_amd.optimizer import attach_dp_routing
    from tests._cpu_codec import OracleCodec

    shapes = [(f"a{i}", 64, 48) for i in range(6)] + [(f"t{i}", 48, 96) for i in range(4)] + [("odd", 64, 48)]
    sketch_gen = {}

    def fixed_sketch(P):  # one sketch per shape, identical in both schedules
        mp_ = int(P.shape[-2])
        if mp_ not in sketch_gen:
            g = torch.Generator().manual_seed(7 + mp_)
            sketch_gen[mp_] = torch.randn(1, 128, mp_, generator=g) * (1.0 / 128) ** 0.5
        return sketch_gen[mp_]

    runs = {}
    for coalesce in (False, True):
        torch.manual_seed(0)
        params = [(n, torch.nn.Parameter(torch.randn(m, k) * 0.02)) for n, m, k in shapes]
        codec = OracleCodec(sketch_lookup=fixed_sketch, deferred=deferred)
        opt = mda.MegatronDion([p for _, p in params], lr=0.01, mu=0.95, weight_decay=0.01, rank_fraction=0.125,
                               codec=codec, coalesce_local=coalesce, coalesce_max_entries=4,
                               defer_error_feedback=deferred)
        attach_dp_routing(opt, params, replicate_group=dist.group.WORLD)
        chunks = []
        for step in range(3):
            gen = torch.Generator().manual_seed(100 * step + 10 * rank + 1)
            for _, p in params:
                p.grad = (torch.randn(p.shape, generator=gen) * 1e-3).to(torch.bfloat16).float()
            chunks.append([int(getattr(b, "_chunks", 0) or 0) for b in opt._batches()[0]])
            opt.step()
        opt.flush_error_feedback()
        runs[coalesce] = {"chunks": chunks,
                          **{f"{n}_{k}": v.detach().clone() for n, p in params
                             for k, v in (("W", p), ("M", opt.state[p]["momentum"]), ("Q", opt.state[p]["Q"]))}}
    torch.save(runs, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("deferred", [False, True], ids=["eager_ef", "deferred_ef"])
def test_gloo_w2_coalesced_groups_match_per_batch(deferred):
    """coalesce_replicated_batches: one RS / batched ortho / AG / AR per group of full
    batches, rank-major layout -- same entries on the same ranks, same results."""
    world = 2
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_coalesce_worker, args=(world, _free_port(), tmp, deferred), nprocs=world, join=True,
                           start_method="spawn")
        res = [torch.load(os.path.join(tmp, f"rank{r}.pt"), weights_only=True) for r in range(world)]
    for rank in range(world):
        plain, merged = res[rank][False], res[rank][True]
        assert all(c == 0 for step in plain["chunks"] for c in step)
        # 7 (64x48) -> groups of 2 full batches + 1 full + a padded one; 4 (48x96) -> 1 group of 2
        assert max(max(step) for step in merged["chunks"]) == 2
        for key, ref in plain.items():
            if key == "chunks":
                continue
            err = _maxrel(merged[key], ref)
            assert err <= 1e-6, (rank, key, err)
    for key in res[0][True]:
        if key.endswith("_W") or key.endswith("_Q"):
            assert torch.equal(res[0][True][key], res[1][True][key]), key


@pytest.mark.parametrize("deferred", [False, True], ids=["eager_ef", "deferred_ef"])
def test_gloo_w4_matches_reference_capture(deferred):
    """BASELINE config 4's replicated schedule beyond two ranks: the product runtime on 4 gloo
    ranks against the reference's own 4-rank capture c15 (a full batch of 4, a padded batch of
    3 transposed matrices whose fourth slot is rank 3's zero entry; two steps)."""
    from tests._golden import Case

    case = Case("c15_w4_pad_two_steps")
    res = _run(case.name, world=4, deferred=deferred)
    names = [n for n, _, _ in case.mats]
    for rank in range(4):
        for step in range(case.steps):
            assert sorted(res[rank][f"s{step}_schedule"]) == [(["a0", "a1", "a2", "a3"], 4),
                                                             (["t0", "t1", "t2", "<pad>"], 3)]
            for n in names:
                keys = (("W", "W1"), ("Q", "Q1"))
                if not deferred or step == case.steps - 1:
                    keys += (("M", "M1"),)
                for k, ref in keys:
                    err = _maxrel(res[rank][f"s{step}_{n}_{k}"], case.t(rank, step, f"{n}_{ref}"))
                    assert err <= 1e-6, (rank, step, n, k, err)
    for n in names:
        for rank in range(1, 4):
            assert torch.equal(res[0][f"s1_{n}_W"], res[rank][f"s1_{n}_W"])
            assert torch.equal(res[0][f"s1_{n}_Q"], res[rank][f"s1_{n}_Q"])
