"""Golden fixtures of the speedrun's FS x TP topology, captured from the REFERENCE.

Run ONLY in the build container (the reference tree does not exist on the GPU box):

    PYTHONPATH=/root/reference DION_DISABLE_TORCH_COMPILE=1 python tests/golden/make_golden_fstp.py

examples/dion/speedrun_nanogpt_mcore.py:36-62, 395-431 runs Dion with FS = 4, TP = 2, bf16
momentum and Q and `--dion-split-qkv`.  Here 4 gloo ranks form FS = 2 x TP = 2 (TP groups
{0, 1}, {2, 3}; FS groups {0, 2}, {1, 3}).  Every matrix is TP-sharded on one dim and
FS-sharded on the other (get_fs_split_dim, distrib_dion/sharding.py:64-70), so its batches take
the "fsdp_tp" kind with an FS P all-reduce and an FS q_norm group (distrib_dion/batches.py:
496-603, 606-771; dion/runtime.py:680-962).  A fused QKV parent (TP on its rows, whole query
groups per TP rank) is optimised as q / k / v children built with the reference's own helpers:
qkv_child_local_shape / qkv_child_global_shape / extract_qkv_child / scatter_qkv_child_
(dion/qkv.py:306-532), resolve_row_child_layout (distrib_dion/row_child.py:30-117) and
build_split_child_dist_meta (distrib_dion/split_child.py:55-148), the way
dion_distrib_optimizer.py:2574-2790, 3417-3580 assembles them.  The script drives the
reference's MegatronDion.step over its own build_dion_batches and records, per rank and
step, each matrix's (and the QKV parent's) local W / M / G before and after, every Q, and the
children's layout as the reference computes it.  Only data is committed.
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

# (name, m_global, n_global, tp_shard_dim); FS shards the other dim.  "qkv" entries carry
# their split shapes (rows of q, k, v per query group).
CASES = [
    dict(name="x1_fs2tp2_speedrun", bf16=False, rf=0.25, steps=2,
         mats=[("a", 64, 48, 0), ("b", 64, 48, 0), ("w", 40, 96, 1)],
         qkv=[("attn.qkv", 4, (8, 4, 4), 48)]),
    dict(name="x2_fs2tp2_speedrun_bf16", bf16=True, rf=0.25, steps=2,
         mats=[("a", 64, 48, 0), ("b", 64, 48, 0), ("w", 40, 96, 1)],
         qkv=[("attn.qkv", 4, (8, 4, 4), 48)]),
]
HYPER = dict(lr=0.01, mu=0.95, weight_decay=0.01, epsilon=1e-8, rcqr_oversample=1.25,
             scale_mode="spectral", extra_scale_factor=0.2)
TP, FS = 2, 2


def split_range(size, world, rank):
    """distrib_dion/sharding.py:44-61 / dion/ortho.py:247-259: remainder on the first ranks."""
    base, rem = size // world, size % world
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def _worker(rank, world, case, port, out_path):
    os.environ["DION_DISABLE_TORCH_COMPILE"] = "1"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    torch.manual_seed(0)
    from megatron.core.optimizer.dion import ortho as d_ortho
    from megatron.core.optimizer.dion import qkv as d_qkv
    from megatron.core.optimizer.dion.algorithm import MegatronDion
    from megatron.core.optimizer.dion.state import is_p_tp_sharded
    from megatron.core.optimizer.dion.types import (DionDistMeta, DionMixedPrecisionConfig, DionParamConfig,
                                                    DionStepParam)
    from megatron.core.optimizer.distrib_dion.batches import build_dion_batches
    from megatron.core.optimizer.distrib_dion.row_child import resolve_row_child_layout
    from megatron.core.optimizer.distrib_dion.split_child import build_split_child_dist_meta

    tp_groups = [dist.new_group([0, 1]), dist.new_group([2, 3])]
    fs_groups = [dist.new_group([0, 2]), dist.new_group([1, 3])]
    tp_rank, fs_rank = rank % TP, rank // TP
    tp_group, fs_group = tp_groups[rank // TP], fs_groups[rank % TP]
    rf = case["rf"]
    sdt = torch.bfloat16 if case["bf16"] else torch.float32

    def shard_meta(name, m, n, tdim, uid):
        fdim = 1 - tdim
        t0, t1 = split_range(m if tdim == 0 else n, TP, tp_rank)
        f0, f1 = split_range(m if fdim == 0 else n, FS, fs_rank)
        rows, cols = ((t0, t1), (f0, f1)) if tdim == 0 else ((f0, f1), (t0, t1))
        transposed = tdim == 1                     # TP on the P-row side (dion/state.py:304-310)
        r = max(1, int(min(math.ceil(rf * min(m, n)), m, n)))
        low = rf < 1.0 and (m + n) * r < m * n
        cfg = DionParamConfig(has_tp_shard=True, use_tp_shard=True, tp_shard_dim=tdim, has_fs_shard=True,
                              use_fs_shard=True, fs_shard_dim=fdim, is_transposed=transposed, use_low_rank_sync=low)
        lm, ln = rows[1] - rows[0], cols[1] - cols[0]
        meta = DionDistMeta(shape=(lm, ln), global_shape=(m, n), fs_start_idx=f0, fs_end_idx=f1, tp_shard_dim=tdim,
                            fs_shard_dim=fdim, rank_fraction=rf, is_transposed=transposed, param_uid=uid,
                            is_dion_param=True, param_name=name, fs_group=fs_group, fs_world_size=FS, fs_rank=fs_rank,
                            tp_group=tp_group, tp_world_size=TP, tp_rank=tp_rank, local_shape=(lm, ln),
                            param_config=cfg)
        return meta, cfg, rows, cols, r

    params, metas, cfgs, info, states = {}, {}, {}, {}, {}
    names = []
    for idx, (name, m, n, tdim) in enumerate(case["mats"]):
        meta, cfg, rows, cols, r = shard_meta(name, m, n, tdim, (name,))
        w_full = torch.randn(m, n, generator=torch.Generator().manual_seed(1000 + idx)) * 0.02
        params[name] = torch.nn.Parameter(w_full[rows[0]:rows[1], cols[0]:cols[1]].clone().contiguous())
        c0, c1 = split_range(r, TP, tp_rank)
        q_rows_g = m if cfg.is_transposed else n
        q0, q1 = (rows if cfg.is_transposed else cols)
        q_full = torch.randn(q_rows_g, r, generator=torch.Generator().manual_seed(2000 + idx))
        states[name] = dict(momentum=torch.zeros_like(params[name], dtype=sdt),
                            Q=q_full[q0:q1, c0:c1].clone().contiguous().to(sdt), r=r,
                            local_shape=tuple(params[name].shape), global_shape=(m, n))
        grads = []
        for step in range(case["steps"]):
            g = torch.randn(m, n, generator=torch.Generator().manual_seed(99 + 17 * step + 131 * idx)) * 1e-3
            grads.append(g.to(torch.bfloat16).float()[rows[0]:rows[1], cols[0]:cols[1]].clone().contiguous())
        metas[name], cfgs[name] = meta, cfg
        info[name] = dict(m=m, n=n, tdim=tdim, rows=list(rows), cols=list(cols), r=r, c0=c0, c1=c1, grads=grads)
        names.append(name)

    # fused QKV parents: TP on the rows (whole query groups per TP rank), FS on the columns
    children = {}
    for pidx, (pname, groups, split, n) in enumerate(case["qkv"]):
        m = groups * sum(split)
        pmeta, _, rows, cols, _ = shard_meta(pname, m, n, 0, (pname,))
        pmeta.qkv_split_shapes = tuple(split)
        w_full = torch.randn(m, n, generator=torch.Generator().manual_seed(3000 + pidx)) * 0.02
        params[pname] = torch.nn.Parameter(w_full[rows[0]:rows[1], cols[0]:cols[1]].clone().contiguous())
        states[pname] = dict(momentum=torch.zeros_like(params[pname], dtype=sdt))
        grads = []
        for step in range(case["steps"]):
            g = torch.randn(m, n, generator=torch.Generator().manual_seed(77 + 13 * step + 101 * pidx)) * 1e-3
            grads.append(g.to(torch.bfloat16).float()[rows[0]:rows[1], cols[0]:cols[1]].clone().contiguous())
        info[pname] = dict(m=m, n=n, tdim=0, rows=list(rows), cols=list(cols), grads=grads, split=list(split),
                           children={})
        for kidx, kind in enumerate(d_qkv.iter_qkv_child_kinds()):
            assert d_qkv.qkv_child_has_local_overlap(tuple(split), pmeta, kind)
            cls = d_qkv.qkv_child_local_shape(tuple(params[pname].shape), tuple(split), kind, dist_meta=pmeta)
            cgs = d_qkv.qkv_child_global_shape((m, n), tuple(split), kind)
            ranges = tuple(d_qkv.qkv_child_row_range(parent_row_start=a, parent_row_end=b,
                                                     split_shapes=tuple(split), child_kind=kind)
                           for a, b in (split_range(m, TP, k) for k in range(TP)))
            tp_lay = resolve_row_child_layout(parent_group=tp_group, parent_world_size=TP, parent_rank=tp_rank,
                                              child_rows=cgs[0], child_ranges=ranges, label="TP",
                                              detail=f"{pname}:{kind}", error_prefix="QKV_CHILD",
                                              create_group=False, make_group=None).as_tuple()
            fs_lay = (fs_group, FS, fs_rank, pmeta.fs_start_idx, pmeta.fs_end_idx, None)
            cmeta = build_split_child_dist_meta(
                parent_dist_meta=pmeta, child_uid=d_qkv.qkv_child_param_uid((pname,), kind),
                child_name=d_qkv.qkv_child_name(pname, kind), child_local_shape=cls, child_global_shape=cgs,
                fs_layout=fs_lay, tp_layout=tp_lay,
                child_fields={"is_transposed": False, "is_qkv_child": True, "qkv_child_kind": kind,
                              "qkv_split_shapes": tuple(split)},
                error_prefix="QKV_CHILD", use_low_rank_sync=True, rank_fraction_default=rf,
                rank_multiple_of_default=1)
            ccfg = cmeta.param_config
            r = max(1, int(min(math.ceil(rf * min(cgs)), *cgs)))
            c0, c1 = split_range(r, TP, tp_rank)
            q_rows_g = cgs[0] if ccfg.is_transposed else cgs[1]
            q0, q1 = (tp_lay[3], tp_lay[4]) if ccfg.is_transposed else (cols[0], cols[1])
            q_full = torch.randn(q_rows_g, r, generator=torch.Generator().manual_seed(4000 + 10 * pidx + kidx))
            cname = cmeta.param_name
            children[cname] = dict(parent=pname, kind=kind, meta=cmeta, cfg=ccfg,
                                   state=dict(Q=q_full[q0:q1, c0:c1].clone().contiguous().to(sdt), r=r,
                                              local_shape=tuple(cls), global_shape=tuple(cgs)))
            info[pname]["children"][kind] = dict(
                name=cname, local_shape=list(cls), global_shape=list(cgs), r=r, c0=c0, c1=c1,
                member_ranges=[list(x) for x in ranges], tp_layout=[int(x) for x in tp_lay[1:5]],
                row_shard_sizes=list(cmeta.row_shard_sizes or ()),
                tensor_row_shard_sizes=list(cmeta.tensor_row_shard_sizes or ()),
                is_transposed=bool(ccfg.is_transposed), use_low_rank_sync=bool(ccfg.use_low_rank_sync))

    mixed = DionMixedPrecisionConfig(momentum_dtype=sdt, q_dtype=sdt) if case["bf16"] else None
    opt = MegatronDion([params[n] for n in params], rank_fraction=rf, use_fs_collectives=True,
                       mixed_precision_config=mixed, **HYPER)
    for name in names:
        opt.state[params[name]] = states[name]
    for pname, _, _, _ in case["qkv"]:
        opt.state[params[pname]] = states[pname]
    id2name = {id(params[n]): n for n in params}
    grads_now, cache = {}, {}

    def route():
        steps = [DionStepParam(param=params[n], grad=grads_now[n], optimizer_state=opt.state[params[n]],
                               optim_group=opt.param_groups[0], config=cfgs[n], dist_meta=metas[n])
                 for n in sorted(names)]
        for cname, ch in sorted(children.items()):
            p = params[ch["parent"]]
            pm = metas_parent[ch["parent"]]
            split = tuple(info[ch["parent"]]["split"])
            st = dict(ch["state"])
            st["momentum"] = d_qkv.extract_qkv_child(opt.state[p]["momentum"], split, ch["kind"], dist_meta=pm)

            def commit(up, um, p=p, pm=pm, split=split, kind=ch["kind"]):
                d_qkv.scatter_qkv_child_(p.data, up, split, kind, dist_meta=pm)
                d_qkv.scatter_qkv_child_(opt.state[p]["momentum"], um, split, kind, dist_meta=pm)

            steps.append(DionStepParam(
                param=d_qkv.extract_qkv_child(p.data, split, ch["kind"], dist_meta=pm),
                grad=d_qkv.extract_qkv_child(grads_now[ch["parent"]], split, ch["kind"], dist_meta=pm),
                optimizer_state=st, optim_group=opt.param_groups[0], config=ch["cfg"], dist_meta=ch["meta"],
                commit_update=commit))
            ch["live_state"] = st
        return build_dion_batches(
            dion_params=steps, use_fs_collectives=True, state_replica_group=None,
            replica_validation_group=dist.group.WORLD, batch_key_cache=cache, global_rank=rank,
            group_size=dist.get_world_size, get_replicate_group=lambda: None,
            resolve_ortho_group=lambda c, m: m.tp_group if is_p_tp_sharded(c, tp_active=c.use_tp_shard) else None,
            resolve_tp_group=lambda m, expect_group: m.tp_group,
            resolve_fs_group_from_meta=lambda m, expect_group: m.fs_group), []

    metas_parent = {}
    for pname, groups, split, n in case["qkv"]:
        m = groups * sum(split)
        metas_parent[pname], _, _, _, _ = shard_meta(pname, m, n, 0, (pname,))
        metas_parent[pname].qkv_split_shapes = tuple(split)

    opt.enable_distributed_mode(route_step_params=route)
    rec = {"batches": []}
    import megatron.core.optimizer.dion.runtime as d_rt
    orig_bdu = d_rt.batch_dion_update_async

    def bdu_wrap(optimizer, params_l, *args, **kwargs):
        real, bg = args[8], args[10]
        dm = args[3]
        members = [(dm[i].param_name if dm[i] is not None else "<pad>") for i in range(len(params_l))]
        rec["batches"].append(dict(members=members, real=int(real), kind=str(bg.kernel_kind)))
        return (yield from orig_bdu(optimizer, params_l, *args, **kwargs))

    d_rt.batch_dion_update_async = bdu_wrap
    arrays = {}
    meta = {"steps": [], "info": {n: {k: v for k, v in info[n].items() if k != "grads"} for n in info}}
    all_names = list(params)
    for step in range(case["steps"]):
        for name in all_names:
            p = params[name]
            arrays[f"s{step}_{name}_W0"] = p.detach().clone()
            arrays[f"s{step}_{name}_M0"] = opt.state[p]["momentum"].clone()
            grads_now[name] = info[name]["grads"][step].clone()
            arrays[f"s{step}_{name}_G"] = grads_now[name].clone()
            if "Q" in opt.state[p]:
                arrays[f"s{step}_{name}_Q0"] = opt.state[p]["Q"].clone()
        for cname, ch in children.items():
            arrays[f"s{step}_{cname}_Q0"] = ch["state"]["Q"].clone()
        rec["batches"] = []
        opt.step()
        for name in all_names:
            p = params[name]
            arrays[f"s{step}_{name}_W1"] = p.detach().clone()
            arrays[f"s{step}_{name}_M1"] = opt.state[p]["momentum"].clone()
            if "Q" in opt.state[p]:
                arrays[f"s{step}_{name}_Q1"] = opt.state[p]["Q"].clone()
        for cname, ch in children.items():
            arrays[f"s{step}_{cname}_Q1"] = ch["state"]["Q"].clone()
        meta["steps"].append({"batches": rec["batches"]})
    np.savez_compressed(out_path, **{k: v.detach().float().numpy() for k, v in arrays.items()})
    with open(out_path + ".json", "w") as fh:
        json.dump(meta, fh)
    dist.barrier()
    dist.destroy_process_group()


def main():
    only = set(sys.argv[1:])
    path = os.path.join(HERE, "manifest_fstp.json")
    manifest = {"hyper": HYPER, "tp": TP, "fs": FS, "cases": []}
    if only and os.path.exists(path):
        with open(path) as fh:
            manifest = json.load(fh)
        manifest["cases"] = [c for c in manifest["cases"] if c["name"] not in only]
    port = 29861
    world = TP * FS
    for case in CASES:
        port += 1
        if only and case["name"] not in only:
            continue
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
        entry["qkv"] = [[q[0], q[1], list(q[2]), q[3]] for q in case["qkv"]]
        manifest["cases"].append(entry)
        print("wrote", out, os.path.getsize(out), "bytes", flush=True)
    order = [c["name"] for c in CASES]
    manifest["cases"].sort(key=lambda c: order.index(c["name"]) if c["name"] in order else len(order))
    with open(path, "w") as fh:
        json.dump(manifest, fh, indent=1, default=list)


if __name__ == "__main__":
    sys.exit(main())
