"""World-size-2 gloo tests of the TP ("fsdp_tp") kernel kind on CPU.

The product's batch runtime (megatron_dion_amd/runtime.py `_tp_batch_update` and
`distributed_orthonormalize`) runs with the oracle codec (oracle/cpu_codec.py) over a real
2-rank gloo TP group: every matrix sharded on its P-row side, Q sharded by columns, Q
all-gathered, the row-sharded randomised Cholesky QR (reduce-scatter / owner factor /
all-gather of the sketch product and the Gram matrix), R summed over TP, Q re-sharded.  The
batches come from the product's own builder (`attach_dp_routing(..., tp_group=, tp_shards=)`),
the sketch slices are the reference's seeded ones (ortho.py:575-640, restated in the oracle and
pinned by tests/test_oracle_golden_tp.py), and every shard on every rank is checked against
the reference's own TP=2 captures (tests/golden/make_golden_tp.py).
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


def tp_sketch_override(case, rank, state, dev):
    """opt._sketch_override: batch -> {entry: this rank's (k, local rows) slice of its sketch}."""
    from oracle import dion_oracle as O

    def fn(batch):
        out = {}
        real = int(batch.real_batch_size)
        for i, meta in enumerate(list(batch.dist_metas)[:real]):
            n = meta.param_name
            sh = case.shard(rank, n)
            ks = O.sketch_rows(int(sh["r"]), case.hyper["rcqr_oversample"])
            seed = O.distributed_sketch_seed(state["step"] + 1, (n,), n)
            rows = int(sh["end"]) - int(sh["start"])
            out[i] = O.reference_sharded_sketch(seed, ks, case.global_rows(n), int(sh["start"]), rows).to(dev)
        return out
    return fn


def _worker(rank, world, port, name, out_dir, deferred, device):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    import megatron_dion_amd as mda
    from megatron_dion_amd.optimizer import attach_dp_routing
    from oracle.cpu_codec import OracleCodec
    from tests._golden import TpCase

    dev = torch.device(device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    case = TpCase(name)
    h = case.hyper
    names = [n for n, _, _ in case.mats]
    gshape = {n: (m, k) for n, m, k in case.mats}
    params = {n: torch.nn.Parameter(case.t(rank, 0, f"{n}_W0").clone().to(dev)) for n in names}
    state = {"step": 0}
    kw = {}
    if dev.type == "cpu":
        kw["codec"] = OracleCodec(deferred=deferred)
    if case.entry.get("bf16"):  # the speedrun's bf16 momentum and Q
        kw["mixed_precision_config"] = mda.DionMixedPrecisionConfig(momentum_dtype=torch.bfloat16,
                                                                    q_dtype=torch.bfloat16)
    opt = mda.MegatronDion([params[n] for n in names], lr=h["lr"], mu=h["mu"], weight_decay=h["weight_decay"],
                           rank_fraction=case.rank_fraction, epsilon=h["epsilon"],
                           rcqr_oversample=h["rcqr_oversample"], defer_error_feedback=deferred, **kw)
    shards = {n: (gshape[n], case.tp_dim(n), case.shard(rank, n)["start"], case.shard(rank, n)["end"])
              for n in names}
    attach_dp_routing(opt, [(n, params[n]) for n in names], tp_group=dist.group.WORLD, tp_shards=shards)
    for n in names:
        sh = case.shard(rank, n)
        assert opt.state[params[n]]["r"] == sh["r"]                       # rank rule on the global shape
        assert tuple(opt.state[params[n]]["Q"].shape) == tuple(case.t(rank, 0, f"{n}_Q0").shape)
        opt.state[params[n]]["Q"].copy_(case.t(rank, 0, f"{n}_Q0"))
    opt._sketch_override = tp_sketch_override(case, rank, state, dev)
    results = {}
    for step in range(case.steps):
        state["step"] = step
        for n in names:
            params[n].grad = case.t(rank, step, f"{n}_G").clone().to(dev)
        batches, _ = opt._route_step_params()
        results[f"s{step}_kinds"] = [(b.batch_group.kernel_kind, int(b.real_batch_size), len(b.entries))
                                     for b in batches]
        opt.step()
        if deferred and step == case.steps - 1:
            opt.flush_error_feedback()
        for n in names:
            results[f"s{step}_{n}_W"] = params[n].detach().cpu().clone()
            results[f"s{step}_{n}_M"] = opt.state[params[n]]["momentum"].cpu().clone()
            results[f"s{step}_{n}_Q"] = opt.state[params[n]]["Q"].cpu().clone()
    torch.save(results, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def run_tp(name, deferred=False, device="cpu"):
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_worker, args=(2, _free_port(), name, tmp, deferred, device), nprocs=2, join=True,
                           start_method="spawn")
        return [torch.load(os.path.join(tmp, f"rank{r}.pt"), weights_only=True) for r in range(2)]


def _maxrel(a, b):
    return (a.double() - b.double()).abs().max().item() / max(b.double().abs().max().item(), 1e-30)


def check_tp_results(res, name, deferred, tol, bf16_tols=None):
    from tests._golden import TpCase

    case = TpCase(name)
    names = [n for n, _, _ in case.mats]
    worst = 0.0
    for rank in range(2):
        for step in range(case.steps):
            assert all(k == "fsdp_tp" for k, _, _ in res[rank][f"s{step}_kinds"])
            assert [(r_, b) for _, r_, b in res[rank][f"s{step}_kinds"]] == \
                [(int(b["real"]), len(b["members"])) for b in case.batches(rank, step)]
            for n in names:
                keys = [("W", "W1"), ("Q", "Q1")]
                if not deferred or step == case.steps - 1:
                    keys.append(("M", "M1"))
                for k, ref in keys:
                    err = _maxrel(res[rank][f"s{step}_{n}_{k}"].float(), case.t(rank, step, f"{n}_{ref}"))
                    worst = max(worst, err)
                    bar = bf16_tols[k] if (bf16_tols and case.entry.get("bf16")) else tol
                    assert err <= bar, (name, rank, step, n, k, err)
    return worst


@pytest.mark.parametrize("name", ["t1_tp2_rows", "t2_tp2_cols_T", "t3_tp2_odd_r_mixed", "t4_tp2_plain_qr",
                                  "t5_tp2_bf16_rows", "t6_tp2_bf16_odd_mixed"])
@pytest.mark.parametrize("deferred", [False, True], ids=["eager_ef", "deferred_ef"])
def test_gloo_tp2_matches_reference(name, deferred):
    res = run_tp(name, deferred=deferred)
    check_tp_results(res, name, deferred, 1e-5)
