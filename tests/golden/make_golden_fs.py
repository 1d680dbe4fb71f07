"""Golden fixtures of the FS ("fsdp") kernel kind, captured from the REFERENCE.

Run ONLY in the build container (the reference tree does not exist on the GPU box):

    PYTHONPATH=/root/reference DION_DISABLE_TORCH_COMPILE=1 python tests/golden/make_golden_fs.py

The default Megatron Dion topology is FS = DP, RP = 1 (megatron/training/initialize.py:79-81):
every matrix is sharded over the FS group along `fs_shard_dim`
(distrib_dion/parameter.py:424-466; the orientation follows the shard dim, dion/state.py:304-310),
and a batch holds FS-world same-key matrices whose partial P = X_local Q_local are
reduce-scattered (sum), orthonormalised by their owner rank and all-gathered
(dion/runtime.py:1729-1795), the column norm summing over the shards (q_norm_group,
runtime.py:965-1013).  This script drives the reference's own MegatronDion.step over its own
build_dion_batches (distrib_dion/batches.py:971) on 2 gloo ranks with FS group = WORLD and no
replicate group, and records, per rank and step, each matrix's local W / M / Q / G before and
after, the global shapes and shard ranges, every orthogonalize call with its sketch, and the
batch schedule (kernel kind, members, fs_collective indices).  Only data is committed.
"""
import json
import math
import os
import sys
import tempfile

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))

# name, mats = (name, m_global, n_global, fs_shard_dim), rank_fraction, steps
CASES = [
    # columns sharded (fs_shard_dim 1 -> not transposed), one full batch of 2
    dict(name="f1_fs2_cols", mats=[("a", 64, 48, 1), ("b", 64, 48, 1)], rf=1 / 6, steps=2),
    # rows sharded (fs_shard_dim 0 -> transposed), 3 matrices -> a full batch and a padded one
    dict(name="f2_fs2_rows_pad", mats=[("x", 96, 40, 0), ("y", 96, 40, 0), ("z", 96, 40, 0)], rf=0.2, steps=2),
    # uneven shards (51 columns over 2 ranks: 26 + 25), mixed with a row-sharded key
    dict(name="f3_fs2_uneven_mixed", mats=[("u", 80, 51, 1), ("v", 80, 51, 1), ("w", 72, 56, 0)], rf=0.25,
         steps=2),
    # the speedrun's bf16 momentum and Q (examples/dion/speedrun_nanogpt_mcore.py:36-62, 417-431:
    # FS = 4 with mixed_precision) on the FS kind: columns, and uneven + row-sharded mixed
    dict(name="f4_fs2_bf16_cols", mats=[("a", 64, 48, 1), ("b", 64, 48, 1)], rf=1 / 6, steps=2, bf16=True),
    dict(name="f5_fs2_bf16_mixed", mats=[("u", 80, 51, 1), ("v", 80, 51, 1), ("w", 72, 56, 0)], rf=0.25,
         steps=2, bf16=True),
    # round 6: the speedrun's FS = 4 itself with bf16 state, where the reduce-scatter of the bf16
    # partial P sums four terms (the reference's collective rounds per hop, in its own order):
    # a full batch of 4 column-sharded matrices + a padded batch, and uneven + row-sharded mixed
    dict(name="f6_fs4_bf16_cols", mats=[("a", 64, 48, 1), ("b", 64, 48, 1), ("c", 64, 48, 1), ("d", 64, 48, 1),
                                        ("e", 64, 48, 1)], rf=1 / 6, steps=2, bf16=True, world=4),
    dict(name="f7_fs4_bf16_mixed", mats=[("u", 80, 51, 1), ("v", 80, 51, 1), ("w", 72, 56, 0)], rf=0.25,
         steps=2, bf16=True, world=4),
]
HYPER = dict(lr=0.01, mu=0.95, weight_decay=0.01, epsilon=1e-8, rcqr_oversample=1.25,
             scale_mode="spectral", extra_scale_factor=0.2)


def fs_range(size, world, rank):
    """distrib_dion's even split with the remainder on the first ranks (compute_fs_shard_range)."""
    per = math.ceil(size / world)
    start = min(size, rank * per)
    return start, min(size, start + per)


def _worker(rank, world, case, port, out_path):
    os.environ["DION_DISABLE_TORCH_COMPILE"] = "1"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    torch.manual_seed(0)
    from megatron.core.optimizer.dion import ortho as d_ortho
    from megatron.core.optimizer.dion import runtime as d_rt
    from megatron.core.optimizer.dion.algorithm import MegatronDion
    from megatron.core.optimizer.dion.types import (DionDistMeta, DionMixedPrecisionConfig, DionParamConfig,
                                                    DionStepParam)
    from megatron.core.optimizer.distrib_dion.batches import build_dion_batches
    from megatron.core.optimizer.distrib_dion.sharding import compute_fs_shard_range

    fs_group = dist.group.WORLD
    rf = case["rf"]
    names = [n for n, _, _, _ in case["mats"]]
    params, cfgs, metas, info = {}, {}, {}, {}
    for idx, (name, m, n, dim) in enumerate(case["mats"]):
        split = m if dim == 0 else n
        start, end = compute_fs_shard_range(split, world, rank)
        assert (start, end) == fs_range(split, world, rank), (start, end)
        w_full = torch.randn(m, n, generator=torch.Generator().manual_seed(1000 + idx)) * 0.02
        w_loc = w_full[start:end] if dim == 0 else w_full[:, start:end]
        lm, ln = w_loc.shape
        transposed = dim == 0
        r = max(1, int(min(math.ceil(rf * min(m, n)), m, n)))  # dion/state.py:179-188 (rank_multiple_of 1)
        q_rows_global = m if transposed else n
        q_full = torch.randn(q_rows_global, r, generator=torch.Generator().manual_seed(2000 + idx))
        q_loc = q_full[start:end].clone()
        low = rf < 1.0 and (m + n) * r < m * n
        cfgs[name] = DionParamConfig(has_fs_shard=True, use_fs_shard=True, fs_shard_dim=dim,
                                     is_transposed=transposed, use_low_rank_sync=low)
        metas[name] = DionDistMeta(shape=(lm, ln), global_shape=(m, n), fs_start_idx=start, fs_end_idx=end,
                                   fs_shard_dim=dim, rank_fraction=rf, is_transposed=transposed,
                                   param_uid=(name,), is_dion_param=True, param_name=name, fs_group=fs_group,
                                   fs_world_size=world, fs_rank=rank, local_shape=(lm, ln),
                                   param_config=cfgs[name])
        params[name] = torch.nn.Parameter(w_loc.clone().contiguous())
        grads = []
        for step in range(case["steps"]):
            g_full = torch.randn(m, n, generator=torch.Generator().manual_seed(99 + 17 * step + 131 * idx)) * 1e-3
            g_full = g_full.to(torch.bfloat16).float()
            grads.append((g_full[start:end] if dim == 0 else g_full[:, start:end]).clone().contiguous())
        info[name] = dict(m=m, n=n, dim=dim, start=start, end=end, r=r, q=q_loc, grads=grads)
    sdt = torch.bfloat16 if case.get("bf16") else torch.float32
    mixed = DionMixedPrecisionConfig(momentum_dtype=sdt, q_dtype=sdt) if case.get("bf16") else None
    opt = MegatronDion([params[n] for n in names], rank_fraction=rf, use_fs_collectives=True,
                       mixed_precision_config=mixed, **HYPER)
    for name in names:
        d = info[name]
        p = params[name]
        opt.state[p] = dict(momentum=torch.zeros_like(p, dtype=sdt), Q=d["q"].clone().to(sdt), r=d["r"],
                            local_shape=tuple(p.shape), global_shape=(d["m"], d["n"]))
    id2name = {id(params[n]): n for n in names}
    grads_now, cache = {}, {}

    def route():
        steps = [DionStepParam(param=params[n], grad=grads_now[n], optimizer_state=opt.state[params[n]],
                               optim_group=opt.param_groups[0], config=cfgs[n], dist_meta=metas[n])
                 for n in sorted(names)]
        return build_dion_batches(
            dion_params=steps, use_fs_collectives=True, state_replica_group=None,
            replica_validation_group=dist.group.WORLD, batch_key_cache=cache, global_rank=rank,
            group_size=dist.get_world_size, get_replicate_group=lambda: None,
            resolve_ortho_group=lambda c, m: None, resolve_tp_group=lambda m, expect_group: None,
            resolve_fs_group_from_meta=lambda m, expect_group: m.fs_group), []

    opt.enable_distributed_mode(route_step_params=route)
    rec = {"batches": [], "ortho": []}
    sketches = []
    orig_sketch = d_ortho.generate_random_sketch_matrix

    def sketch_wrap(P, oversample=1.25, make_sketch=None):
        S = orig_sketch(P, oversample=oversample, make_sketch=make_sketch)
        sketches.append(S.detach().clone())
        return S

    d_ortho.generate_random_sketch_matrix = sketch_wrap
    orig_orth = d_rt.orthogonalize

    def orth_wrap(P, rcqr_oversample=1.25, make_sketch=None):
        n_before = len(sketches)
        out = orig_orth(P, rcqr_oversample=rcqr_oversample, make_sketch=make_sketch)
        S = sketches[-1] if len(sketches) > n_before else None
        rec["ortho"].append(dict(p_in=P.detach().clone(), p_out=out.detach().clone(), s=S))
        return out

    d_rt.orthogonalize = orth_wrap
    orig_bdu = d_rt.batch_dion_update_async

    def bdu_wrap(optimizer, params_l, *args, **kwargs):
        # positional order of runtime.py:341-357: momentums, Qs, configs, dist_metas, optim_groups,
        # grads, optimizer_states, param_shapes, real_batch_size, batch_cache_key, batch_group, collectives
        real, bg, bc = args[8], args[10], args[11]
        members = [id2name.get(id(p), "<pad>") for p in params_l]
        dm = args[3]
        members = [m if dm[i] is not None else "<pad>" for i, m in enumerate(members)]
        rec["batches"].append(dict(members=members, real=int(real), kind=str(bg.kernel_kind),
                                   fs_indices=list(bc.fs_collective.indices) if bc.fs_collective else None,
                                   q_norm=bg.q_norm_group is not None))
        return (yield from orig_bdu(optimizer, params_l, *args, **kwargs))

    d_rt.batch_dion_update_async = bdu_wrap
    arrays, meta = {}, {"steps": [], "shards": {n: {k: info[n][k] for k in ("m", "n", "dim", "start", "end", "r")}
                                                for n in names}}
    for step in range(case["steps"]):
        for name in names:
            p = params[name]
            arrays[f"s{step}_{name}_W0"] = p.detach().clone()
            arrays[f"s{step}_{name}_M0"] = opt.state[p]["momentum"].clone()
            arrays[f"s{step}_{name}_Q0"] = opt.state[p]["Q"].clone()
            grads_now[name] = info[name]["grads"][step].clone()
            arrays[f"s{step}_{name}_G"] = grads_now[name].clone()
        rec["batches"], rec["ortho"] = [], []
        opt.step()
        for name in names:
            p = params[name]
            arrays[f"s{step}_{name}_W1"] = p.detach().clone()
            arrays[f"s{step}_{name}_M1"] = opt.state[p]["momentum"].clone()
            arrays[f"s{step}_{name}_Q1"] = opt.state[p]["Q"].clone()
        smeta = {"batches": rec["batches"], "ortho": []}
        for i, o in enumerate(rec["ortho"]):
            arrays[f"s{step}_ortho{i}_pin"] = o["p_in"]
            arrays[f"s{step}_ortho{i}_pout"] = o["p_out"]
            if o["s"] is not None:
                arrays[f"s{step}_ortho{i}_S"] = o["s"]
            smeta["ortho"].append({"has_sketch": o["s"] is not None, "shape": list(o["p_in"].shape)})
        meta["steps"].append(smeta)
    np.savez_compressed(out_path, **{k: v.detach().float().numpy() for k, v in arrays.items()})
    with open(out_path + ".json", "w") as fh:
        json.dump(meta, fh)
    dist.barrier()
    dist.destroy_process_group()


def main():
    only = set(sys.argv[1:])
    path = os.path.join(HERE, "manifest_fs.json")
    manifest = {"hyper": HYPER, "cases": []}
    if only and os.path.exists(path):
        with open(path) as fh:
            manifest = json.load(fh)
        manifest["cases"] = [c for c in manifest["cases"] if c["name"] not in only]
    port = 29711
    for case in CASES:
        port += 1
        if only and case["name"] not in only:
            continue
        world = int(case.get("world", 2))
        with tempfile.TemporaryDirectory() as tmp:
            paths = [os.path.join(tmp, f"rank{r}") for r in range(world)]
            ctx = mp.get_context("spawn")
            procs = [ctx.Process(target=_worker, args=(r, world, case, port, paths[r])) for r in range(world)]
            for pr in procs:
                pr.start()
            for pr in procs:
                pr.join()
                if pr.exitcode != 0:
                    raise SystemExit(f"case {case['name']} failed: {pr.exitcode}")
            merged, metas = {}, []
            for r in range(world):
                with np.load(paths[r] + ".npz") as z:
                    for k in z.files:
                        merged[f"r{r}_{k}"] = z[k]
                with open(paths[r] + ".json") as fh:
                    metas.append(json.load(fh))
        out = os.path.join(HERE, f"{case['name']}.npz")
        np.savez_compressed(out, **merged)
        entry = dict(case, world=world, rank_meta=metas)
        entry["mats"] = [list(m) for m in case["mats"]]
        manifest["cases"].append(entry)
        print("wrote", out, os.path.getsize(out), "bytes", flush=True)
    order = [c["name"] for c in CASES]
    manifest["cases"].sort(key=lambda c: order.index(c["name"]) if c["name"] in order else len(order))
    with open(path, "w") as fh:
        json.dump(manifest, fh, indent=1, default=list)


if __name__ == "__main__":
    sys.exit(main())
