"""Container-only check of the drop-in boundary for the SHARDED kernel kinds, against the reference.

Run ONLY in the build container (the reference tree does not exist on the GPU box):

    PYTHONPATH=/root/reference DION_DISABLE_TORCH_COMPILE=1 python scripts/ref/ref_boundary_check_sharded.py

For three topologies on gloo ranks -- FS = 2 ("fsdp"), TP = 2 ("fsdp_tp") and FS = 2 x TP = 2 on four
ranks (the speedrun's topology, FS on the contraction side) -- it builds the SAME sharded inputs twice:

  A. the reference end to end: its MegatronDion (dion/algorithm.py:29) routed through its own
     build_dion_batches (distrib_dion/batches.py:971) with real FS / TP process groups and the
     resolvers its adapter installs (batches.py:571-584, 971-1067); every unseeded sketch the FS
     owner draws (dion/ortho.py:643-662) is recorded in call order;
  B. the reference's own batch builder again -- its DionBatch objects with their batch_collectives,
     ortho_group and q_norm_group -- but each batch executed by THIS repo's runtime
     (megatron_dion_amd.runtime.run_dion_batch_async under its AsyncRuntime) with the oracle codec:
     the FS owner replays A's sketches in call order, the TP row-sharded sketch is the reference's
     seeded one (ortho.py:575-640, restated in oracle/dion_oracle.py).

W, momentum and Q of every local shard on every rank are compared after every step (max-relative,
bar 1e-6).  Nothing is refused any more: the check fails if the runtime raises.  The result is written
to profiles/r04/ref_boundary_check.json together with the ddp result of ref_boundary_check.py.
"""
import json
import math
import os
import socket
import sys
import tempfile

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
STEPS = 2
HYPER = dict(lr=0.01, mu=0.95, weight_decay=0.01, epsilon=1e-8, rcqr_oversample=1.25,
             scale_mode="spectral", extra_scale_factor=0.2)
# (name, m, n, shard dim): for "fs" the FS shard dim, for "tp" / "fstp" the TP shard dim
TOPOLOGIES = {
    "fs": dict(world=2, FS=2, TP=1, rf=0.25, mats=[("a", 64, 48, 1), ("b", 64, 48, 1), ("c", 64, 48, 1),
                                                  ("x", 96, 40, 0), ("u", 80, 51, 1)]),
    "tp": dict(world=2, FS=1, TP=2, rf=0.2, mats=[("a", 64, 48, 0), ("b", 64, 48, 0), ("x", 40, 96, 1),
                                                 ("y", 40, 96, 1), ("w", 56, 40, 1)]),
    "fstp": dict(world=4, FS=2, TP=2, rf=0.25, mats=[("a", 64, 48, 0), ("b", 64, 48, 0), ("t", 48, 96, 1),
                                                    ("s", 80, 64, 0)]),
}


def split_range(size, world, rank):
    """remainder on the first ranks (dion/ortho.py:247-259 for TP; distrib_dion/sharding.py:44-61 for FS)."""
    base, rem = size // world, size % world
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def fs_range(size, world, rank):
    per = math.ceil(size / world)
    start = min(size, rank * per)
    return start, min(size, start + per)


def _worker(rank, world, topo, port, out_path):
    os.environ["DION_DISABLE_TORCH_COMPILE"] = "1"
    sys.path.insert(0, ROOT)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    torch.manual_seed(0)
    from megatron.core.optimizer.dion import ortho as d_ortho
    from megatron.core.optimizer.dion.algorithm import MegatronDion as RefDion
    from megatron.core.optimizer.dion.state import is_p_tp_sharded
    from megatron.core.optimizer.dion.types import DionDistMeta, DionParamConfig, DionStepParam
    from megatron.core.optimizer.distrib_dion.batches import build_dion_batches
    from megatron.core.optimizer.distrib_dion.sharding import compute_fs_shard_range

    import megatron_dion_amd as mda
    from megatron_dion_amd.runtime import AsyncRuntime, run_dion_batch_async
    from oracle import dion_oracle as O
    from oracle.cpu_codec import OracleCodec

    cfgT = TOPOLOGIES[topo]
    FS, TP, rf = cfgT["FS"], cfgT["TP"], cfgT["rf"]
    if topo == "fs":
        fs_group, tp_group, fs_rank, tp_rank = dist.group.WORLD, None, rank, 0
    elif topo == "tp":
        fs_group, tp_group, fs_rank, tp_rank = None, dist.group.WORLD, 0, rank
    else:
        tp_groups = [dist.new_group([0, 1]), dist.new_group([2, 3])]
        fs_groups = [dist.new_group([0, 2]), dist.new_group([1, 3])]
        tp_rank, fs_rank = rank % TP, rank // TP
        tp_group, fs_group = tp_groups[rank // TP], fs_groups[rank % TP]

    def shard(idx, name, m, n, dim):
        r = max(1, int(min(math.ceil(rf * min(m, n)), m, n)))
        low = rf < 1.0 and (m + n) * r < m * n
        rows, cols = (0, m), (0, n)
        extra = {}
        if topo == "fs":
            split = m if dim == 0 else n
            s0, s1 = compute_fs_shard_range(split, FS, fs_rank)
            assert (s0, s1) == fs_range(split, FS, fs_rank)
            rows, cols = ((s0, s1), cols) if dim == 0 else (rows, (s0, s1))
            transposed = dim == 0
            cfg = DionParamConfig(has_fs_shard=True, use_fs_shard=True, fs_shard_dim=dim, is_transposed=transposed,
                                  use_low_rank_sync=low)
            extra = dict(fs_start_idx=s0, fs_end_idx=s1, fs_shard_dim=dim, fs_group=fs_group, fs_world_size=FS,
                         fs_rank=fs_rank)
            q_rows = (s0, s1)
            q_cols = (0, r)
        else:
            tdim = dim
            transposed = tdim == 1
            t0, t1 = split_range(m if tdim == 0 else n, TP, tp_rank)
            if topo == "tp":
                rows, cols = ((t0, t1), cols) if tdim == 0 else (rows, (t0, t1))
                cfg = DionParamConfig(has_tp_shard=True, use_tp_shard=True, tp_shard_dim=tdim,
                                      is_transposed=transposed, use_low_rank_sync=low)
                extra = dict(tp_shard_dim=tdim, tp_group=tp_group, tp_world_size=TP, tp_rank=tp_rank)
                q_rows = (0, m if transposed else n)
            else:
                fdim = 1 - tdim
                f0, f1 = split_range(m if fdim == 0 else n, FS, fs_rank)
                rows, cols = ((t0, t1), (f0, f1)) if tdim == 0 else ((f0, f1), (t0, t1))
                cfg = DionParamConfig(has_tp_shard=True, use_tp_shard=True, tp_shard_dim=tdim, has_fs_shard=True,
                                      use_fs_shard=True, fs_shard_dim=fdim, is_transposed=transposed,
                                      use_low_rank_sync=low)
                extra = dict(fs_start_idx=f0, fs_end_idx=f1, tp_shard_dim=tdim, fs_shard_dim=fdim, fs_group=fs_group,
                             fs_world_size=FS, fs_rank=fs_rank, tp_group=tp_group, tp_world_size=TP, tp_rank=tp_rank)
                q_rows = rows if transposed else cols
            q_cols = split_range(r, TP, tp_rank)
        lm, ln = rows[1] - rows[0], cols[1] - cols[0]
        meta = DionDistMeta(shape=(lm, ln), global_shape=(m, n), rank_fraction=rf, is_transposed=transposed,
                            param_uid=(name,), is_dion_param=True, param_name=name, local_shape=(lm, ln),
                            param_config=cfg, **extra)
        w_full = torch.randn(m, n, generator=torch.Generator().manual_seed(1000 + idx)) * 0.02
        q_full = torch.randn(m if transposed else n, r, generator=torch.Generator().manual_seed(2000 + idx))
        grads = []
        for step in range(STEPS):
            g = torch.randn(m, n, generator=torch.Generator().manual_seed(99 + 17 * step + 131 * idx)) * 1e-3
            grads.append(g.to(torch.bfloat16).float()[rows[0]:rows[1], cols[0]:cols[1]].clone().contiguous())
        return dict(meta=meta, cfg=cfg, r=r, w=w_full[rows[0]:rows[1], cols[0]:cols[1]].clone().contiguous(),
                    q=q_full[q_rows[0]:q_rows[1], q_cols[0]:q_cols[1]].clone().contiguous(), grads=grads,
                    m=m, n=n, prow0=(rows[0] if not transposed else cols[0]), prows=(lm if not transposed else ln))

    S = {name: shard(idx, name, m, n, dim) for idx, (name, m, n, dim) in enumerate(cfgT["mats"])}
    names = sorted(S)

    def make(opt_ctor):
        params = {n: torch.nn.Parameter(S[n]["w"].clone()) for n in names}
        opt = opt_ctor([params[n] for n in names])
        for n in names:
            p = params[n]
            st = dict(momentum=torch.zeros_like(p), Q=S[n]["q"].clone(), r=S[n]["r"], local_shape=tuple(p.shape),
                      global_shape=(S[n]["m"], S[n]["n"]))
            opt.state[p] = st
        return opt, params

    def builder(opt, params, grads, cache):
        steps = [DionStepParam(param=params[n], grad=grads[n], optimizer_state=opt.state[params[n]],
                               optim_group=opt.param_groups[0], config=S[n]["cfg"], dist_meta=S[n]["meta"])
                 for n in names]
        return build_dion_batches(
            dion_params=steps, use_fs_collectives=True, state_replica_group=None,
            replica_validation_group=dist.group.WORLD, batch_key_cache=cache, global_rank=rank,
            group_size=dist.get_world_size, get_replicate_group=lambda: None,
            resolve_ortho_group=lambda c, m: m.tp_group if is_p_tp_sharded(c, tp_active=c.use_tp_shard) else None,
            resolve_tp_group=lambda m, expect_group: m.tp_group,
            resolve_fs_group_from_meta=lambda m, expect_group: m.fs_group)

    # ---- A: the reference end to end, FS-owner sketches recorded
    sketches = []
    orig = d_ortho.generate_random_sketch_matrix

    def rec(P, oversample=1.25, make_sketch=None):
        Sk = orig(P, oversample=oversample, make_sketch=make_sketch)
        sketches.append(Sk.detach().clone())
        return Sk

    d_ortho.generate_random_sketch_matrix = rec
    ref, rparams = make(lambda ps: RefDion(ps, rank_fraction=rf, use_fs_collectives=True, **HYPER))
    grads_now, cache_a = {}, {}
    ref.enable_distributed_mode(route_step_params=lambda: (builder(ref, rparams, grads_now, cache_a), []))
    ref_out = []
    for s in range(STEPS):
        for n in names:
            grads_now[n] = S[n]["grads"][s].clone()
        ref.step()
        ref_out.append({n: (rparams[n].detach().clone(), ref.state[rparams[n]]["momentum"].clone(),
                            ref.state[rparams[n]]["Q"].clone()) for n in names})
    d_ortho.generate_random_sketch_matrix = orig

    # ---- B: the reference's batches, this repo's runtime + the oracle codec
    replay = iter(sketches)
    codec = OracleCodec(sketch_lookup=lambda P: next(replay))
    ours, oparams = make(lambda ps: mda.MegatronDion(ps, rank_fraction=rf, codec=codec, defer_error_feedback=False,
                                                     coalesce_local=False, **HYPER))
    cache_b = {}
    worst = {"W": 0.0, "M": 0.0, "Q": 0.0}
    kinds = []
    error = None
    try:
        for s in range(STEPS):
            batches = builder(ours, oparams, {n: S[n]["grads"][s].clone() for n in names}, cache_b)
            kinds.append(sorted({str(b.batch_group.kernel_kind) for b in batches}))
            ours._step_count += 1
            for g in ours.param_groups:
                g["step"] = g.get("step", 0) + 1

            def tp_sketches(batch, step=s):
                if TP == 1 or str(batch.batch_group.kernel_kind) != "fsdp_tp":
                    return None
                out = {}
                for i, meta in enumerate(list(batch.dist_metas)[:int(batch.real_batch_size)]):
                    sh = S[meta.param_name]
                    ks = O.sketch_rows(int(sh["r"]), HYPER["rcqr_oversample"])
                    seed = O.distributed_sketch_seed(step + 1, meta.param_uid, meta.param_name)
                    glob = sh["n"] if meta.is_transposed else sh["m"]
                    out[i] = O.reference_sharded_sketch(seed, ks, glob, sh["prow0"], sh["prows"])
                return out

            with torch.no_grad():
                AsyncRuntime((run_dion_batch_async(ours, b, sketches=tp_sketches(b)) for b in batches), 3).run()
            for n in names:
                a = (oparams[n].detach(), ours.state[oparams[n]]["momentum"], ours.state[oparams[n]]["Q"])
                for k, x, y in zip("WMQ", a, ref_out[s][n]):
                    err = (x.double() - y.double()).abs().max().item() / max(y.double().abs().max().item(), 1e-30)
                    worst[k] = max(worst[k], err)
    except Exception as exc:  # the check records the failure rather than hiding it
        error = f"{type(exc).__name__}: {exc}"
    result = {"topology": topo, "world": world, "FS": FS, "TP": TP, "rank": rank, "steps": STEPS,
              "matrices": [list(x) for x in cfgT["mats"]], "rank_fraction": rf, "kernel_kinds": kinds,
              "fs_sketches_replayed": len(sketches), "max_rel": worst, "error": error,
              "pass": error is None and max(worst.values()) <= 1e-6}
    with open(out_path + f".{rank}", "w") as f:
        json.dump(result, f)
    dist.barrier()
    dist.destroy_process_group()


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main():
    results = []
    for topo, cfg in TOPOLOGIES.items():
        with tempfile.TemporaryDirectory() as tmp:
            out = os.path.join(tmp, "r.json")
            world = cfg["world"]
            mp.start_processes(_worker, args=(world, topo, _port(), out), nprocs=world, join=True,
                               start_method="spawn")
            for r in range(world):
                with open(out + f".{r}") as f:
                    results.append(json.load(f))
    ddp_path = os.path.join(ROOT, "profiles", "r04", "ref_boundary_check_ddp.json")
    ddp = json.load(open(ddp_path)) if os.path.exists(ddp_path) else []
    dest = os.path.join(ROOT, "profiles", "r04", "ref_boundary_check.json")
    os.makedirs(os.path.dirname(dest), exist_ok=True)
    with open(dest, "w") as f:
        json.dump({"ddp (ref_boundary_check.py)": ddp, "sharded": results}, f, indent=1)
    for r in results:
        print(r["topology"], "rank", r["rank"], r["kernel_kinds"], r["max_rel"], "error:", r["error"], "pass:", r["pass"])
    if not all(r["pass"] for r in results):
        raise SystemExit("sharded boundary check FAILED")


if __name__ == "__main__":
    main()
