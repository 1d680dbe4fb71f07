"""World-size-2 gloo tests of the FS ("fsdp") kernel kind on CPU.

The product's batch runtime (megatron_dion_amd/runtime.py `_fs_batch_update`) runs with the
oracle codec (oracle/cpu_codec.py) over a real 2-rank gloo FS group: every matrix sharded
along its fs_shard_dim, reduce-scatter(sum) of the partial P, owner-rank orthonormalisation,
all-gather, shard-local R / fix-up / error feedback, column sums all-reduced over the FS
group, weight update with the global shape's LR.  The batches come from the product's own
builder (`attach_dp_routing(..., fs_group=, fs_shards=)`), and every shard on every rank is
checked against the reference's own FS=2 captures (tests/golden/make_golden_fs.py).
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


def _worker(rank, world, port, name, out_dir, deferred, device):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    import megatron_dion_amd as mda
    from megatron_dion_amd.optimizer import attach_dp_routing
    from oracle.cpu_codec import OracleCodec
    from tests._golden import FsCase

    dev = torch.device(device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    case = FsCase(name)
    h = case.hyper
    names = [n for n, _, _ in case.mats]
    gshape = {n: (m, k) for n, m, k in case.mats}
    params = {n: torch.nn.Parameter(case.t(rank, 0, f"{n}_W0").clone().to(dev)) for n in names}
    state = {"step": 0}
    kw = {}
    if dev.type == "cpu":
        kw["codec"] = OracleCodec(sketch_lookup=lambda P: case.sketch_for(rank, state["step"], P.cpu()),
                                  deferred=deferred)
    if case.entry.get("bf16"):  # the speedrun's bf16 momentum and Q
        kw["mixed_precision_config"] = mda.DionMixedPrecisionConfig(momentum_dtype=torch.bfloat16,
                                                                    q_dtype=torch.bfloat16)
    opt = mda.MegatronDion([params[n] for n in names], lr=h["lr"], mu=h["mu"], weight_decay=h["weight_decay"],
                           rank_fraction=case.rank_fraction, epsilon=h["epsilon"],
                           rcqr_oversample=h["rcqr_oversample"], defer_error_feedback=deferred, **kw)
    shards = {n: (gshape[n], case.fs_dim(n), case.shard(rank, n)["start"], case.shard(rank, n)["end"])
              for n in names}
    attach_dp_routing(opt, [(n, params[n]) for n in names], fs_group=dist.group.WORLD, fs_shards=shards)
    for n in names:
        assert opt.state[params[n]]["r"] == case.shard(rank, n)["r"]        # rank rule on the global shape
        opt.state[params[n]]["Q"].copy_(case.t(rank, 0, f"{n}_Q0"))
    results = {}
    for step in range(case.steps):
        state["step"] = step
        for n in names:
            params[n].grad = case.t(rank, step, f"{n}_G").clone().to(dev)
        batches, _ = opt._route_step_params()
        results[f"s{step}_kinds"] = [(b.batch_group.kernel_kind, int(b.real_batch_size), len(b.entries))
                                     for b in batches]
        if dev.type == "cuda":
            opt._sketch_override = _owned_sketches(case, rank, step, dev)
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


def _owned_sketches(case, rank, step, dev):
    """The sketch the reference drew on this rank for the entry it owns in each batch (ortho calls
    run in batch order, one per batch whose owned entry is real)."""
    calls = case.ortho_calls(rank, step)
    it = iter(calls)
    per_batch = []
    for b in case.batches(rank, step):
        owned_real = rank < int(b["real"])
        per_batch.append(next(it)["S"] if owned_real else None)
    order = {}

    def fn(batch, _pb=per_batch, _order=order):
        key = id(batch)
        if key not in _order:
            _order[key] = len(_order)
        S = _pb[_order[key]]
        return None if S is None else {rank: S[0].to(dev)}
    return fn


def run_fs(name, deferred=False, device="cpu"):
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_worker, args=(2, _free_port(), name, tmp, deferred, device), nprocs=2, join=True,
                           start_method="spawn")
        return [torch.load(os.path.join(tmp, f"rank{r}.pt"), weights_only=True) for r in range(2)]


def _maxrel(a, b):
    return (a.double() - b.double()).abs().max().item() / max(b.double().abs().max().item(), 1e-30)


# bf16 state on the GPU: the HIP kernels accumulate in another order than torch's CPU bf16
# matmuls, so a product next to a bf16 rounding boundary can round the other way: one bf16
# ulp of the largest element (tests/test_gpu_bf16.py explains the bars)
BF16_GPU_TOLS = {"W": 1e-3, "M": 2 ** -6, "Q": 2e-2}


def check_fs_results(res, name, deferred, tol, bf16_tols=None):
    from tests._golden import FsCase

    case = FsCase(name)
    names = [n for n, _, _ in case.mats]
    worst = 0.0
    for rank in range(2):
        for step in range(case.steps):
            assert all(k == "fsdp" for k, _, _ in res[rank][f"s{step}_kinds"])
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


@pytest.mark.parametrize("name", ["f1_fs2_cols", "f2_fs2_rows_pad", "f3_fs2_uneven_mixed", "f4_fs2_bf16_cols",
                                  "f5_fs2_bf16_mixed"])
@pytest.mark.parametrize("deferred", [False, True], ids=["eager_ef", "deferred_ef"])
def test_gloo_fs2_matches_reference(name, deferred):
    res = run_fs(name, deferred=deferred)
    check_fs_results(res, name, deferred, 1e-6)
