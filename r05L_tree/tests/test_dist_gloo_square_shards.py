"""Deferred error feedback on square FS / TP shards, on CPU over gloo W = 2.

The orientation of a pending error feedback cannot be told from the shapes when the local
shard is square: a (2048, 1024)-style global matrix FS-sharded on dim 0 over 2 ranks has a
(1024, 1024)-style local shard and is transposed (the FS shard dim sits on the contraction
side, dion/state.py:304-310), and so is a TP shard of a wide matrix on dim 1.  The pending
entry records the orientation; here the deferred schedule's momentum -- applied late by
flush_error_feedback(), by a `state["momentum"]` read and by `dict(state)` (ADVICE r2, low:
CPython's dict fast path) -- must equal the eager schedule's after every step count.  The
product runtime runs with the test-only oracle codec, so both schedules do the same
arithmetic and agree to fp32 rounding.
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.slow

# name -> (global shape, shard dim); 2 ranks -> square 64 x 64 local shards
FS_MATS = {"fs_rows": ((128, 64), 0), "fs_rows_b": ((128, 64), 0)}
TP_MATS = {"tp_cols": ((64, 128), 1), "tp_cols_b": ((64, 128), 1)}
STEPS = 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _tp_sketches(rank, step):
    """TP batches take this rank's rows of one seeded global sketch per entry."""
    def fn(batch):
        out = {}
        for i, p in enumerate(batch.params):
            g = torch.Generator().manual_seed(1000 * step + i)
            S = torch.randn(128, 128, generator=g) / 128 ** 0.5  # k x global P rows (n = 128)
            out[i] = S[:, rank * 64:(rank + 1) * 64].contiguous()
        return out
    return fn


def _run(rank, kind, deferred):
    import megatron_dion_amd as mda
    from megatron_dion_amd.optimizer import attach_dp_routing
    from oracle.cpu_codec import OracleCodec

    mats = FS_MATS if kind == "fs" else TP_MATS
    params, shards = {}, {}
    for i, (name, ((m, n), dim)) in enumerate(mats.items()):
        full = torch.randn(m, n, generator=torch.Generator().manual_seed(i)) * 0.02
        lo, hi = (rank * (m // 2), (rank + 1) * (m // 2)) if dim == 0 else (rank * (n // 2), (rank + 1) * (n // 2))
        local = full[lo:hi] if dim == 0 else full[:, lo:hi]
        params[name] = torch.nn.Parameter(local.contiguous())
        shards[name] = ((m, n), dim, lo, hi)
    opt = mda.MegatronDion(list(params.values()), lr=0.01, mu=0.95, weight_decay=0.01, rank_fraction=0.25,
                           codec=OracleCodec(deferred=True), defer_error_feedback=deferred)
    kw = dict(fs_group=dist.group.WORLD, fs_shards=shards) if kind == "fs" else \
        dict(tp_group=dist.group.WORLD, tp_shards=shards)
    attach_dp_routing(opt, list(params.items()), **kw)
    for name, p in params.items():
        assert tuple(p.shape) == (64, 64)  # square local shard
    out = {}
    for step in range(STEPS):
        if kind == "tp":
            opt._sketch_override = _tp_sketches(rank, step)
        for i, (name, p) in enumerate(params.items()):
            p.grad = torch.randn(p.shape, generator=torch.Generator().manual_seed(50 * step + 10 * i + rank)) * 1e-3
        opt.step()
        names = list(params)
        if deferred:
            # three ways a pending error feedback reaches the momentum from outside the step
            out[f"s{step}_{names[0]}_M"] = dict(opt.state[params[names[0]]])["momentum"].clone()
            out[f"s{step}_{names[1]}_M"] = opt.state[params[names[1]]]["momentum"].clone()
            opt.flush_error_feedback()
        else:
            for name in names:
                out[f"s{step}_{name}_M"] = opt.state[params[name]]["momentum"].clone()
        for name, p in params.items():
            out[f"s{step}_{name}_W"] = p.detach().clone()
    return out


def _worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    res = {}
    for kind in ("fs", "tp"):
        for deferred in (False, True):
            for k, v in _run(rank, kind, deferred).items():
                res[f"{kind}_{int(deferred)}_{k}"] = v
    torch.save(res, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_deferred_ef_on_square_shards_equals_eager():
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_worker, args=(2, _free_port(), tmp), nprocs=2, join=True, start_method="spawn")
        res = [torch.load(os.path.join(tmp, f"rank{r}.pt"), weights_only=True) for r in range(2)]
    for rank in range(2):
        for kind, mats in (("fs", FS_MATS), ("tp", TP_MATS)):
            for step in range(STEPS):
                for name in mats:
                    for key in ("M", "W"):
                        eager = res[rank][f"{kind}_0_s{step}_{name}_{key}"]
                        late = res[rank][f"{kind}_1_s{step}_{name}_{key}"]
                        err = (late - eager).abs().max().item() / eager.abs().max().item()
                        assert err <= 1e-6, (rank, kind, step, name, key, err)
