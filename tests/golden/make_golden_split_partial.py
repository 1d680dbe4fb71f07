"""Golden fixtures of split-linear children whose rows miss members of the parent's FS row group,
captured from the REFERENCE.

Run ONLY in the build container (the reference tree does not exist on the GPU box):

    PYTHONPATH=/root/reference DION_DISABLE_TORCH_COMPILE=1 python tests/golden/make_golden_split_partial.py

A fused SwiGLU fc1 (gate rows then up rows, `--dion-split-linear`) whose rows are FS-sharded
(fs_shard_dim 0) over FS ranks that do not align with the gate/up boundary: each child is owned by
a SUBSET of the FS group.  The reference builds a child-specific process group for it, the same on
every rank before routing (distrib_dion/row_child.py:30-117, resolve_row_child_layout;
dion_distrib_optimizer.py:263-284 _ensure_child_group, :2940-3039), and the child's dist meta from
it (distrib_dion/split_child.py:55-148); a member-less rank holds no rows of the child and routes
no step param for it.  Cases:

  p1_fs3_partial: FS = 3, gate 24 + up 24 rows (FS ranges 16 | 16 | 16): gate on ranks {0, 1}, up on
                  ranks {1, 2} -- two 2-rank sub-groups, rank 1 in both;
  p2_fs2_single:  FS = 2, gate 24 + up 24 (24 | 24): each child has ONE owner (no group: an unsharded
                  child on its owner);
  p3_tp3_partial: the same fused fc1 TP-sharded on its rows (tp_shard_dim 0, partition stride 1:
                  dion_distrib_optimizer.py:3040-3110, linear.py:176-228) over TP = 3: each child is
                  a TP-sharded ("fsdp_tp") matrix over its 2-rank TP sub-group.

Each case also holds an ordinary sharded matrix (FS on its columns, or TP on its rows) in the same
optimizer.  The script
drives the reference's MegatronDion.step over its own build_dion_batches and records, per rank and
step, every local W / M / G and every Q (the parent's and each child's), the child layouts the
reference computes, and every orthogonalize call's sketch.  Only data is committed.
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
CASES = [
    dict(name="p1_fs3_partial", world=3, split=(24, 24), n=40, rf=0.25, steps=2, plain=("b", 64, 48)),
    dict(name="p2_fs2_single", world=2, split=(24, 24), n=40, rf=0.25, steps=2, plain=("b", 64, 48)),
    dict(name="p3_tp3_partial", world=3, split=(24, 24), n=40, rf=0.25, steps=2, plain=("b", 96, 40), axis="tp"),
]
HYPER = dict(lr=0.01, mu=0.95, weight_decay=0.01, epsilon=1e-8, rcqr_oversample=1.25,
             scale_mode="spectral", extra_scale_factor=0.2)
KINDS = ("gate", "up")


def _worker(rank, world, case, port, out_path):
    os.environ["DION_DISABLE_TORCH_COMPILE"] = "1"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    torch.manual_seed(0)
    from megatron.core.optimizer.dion import linear as d_lin
    from megatron.core.optimizer.dion import ortho as d_ortho
    from megatron.core.optimizer.dion import runtime as d_rt
    from megatron.core.optimizer.dion.algorithm import MegatronDion
    from megatron.core.optimizer.dion.state import is_p_tp_sharded
    from megatron.core.optimizer.dion.types import DionDistMeta, DionParamConfig, DionStepParam
    from megatron.core.optimizer.distrib_dion.batches import build_dion_batches
    from megatron.core.optimizer.distrib_dion.row_child import resolve_row_child_layout
    from megatron.core.optimizer.distrib_dion.sharding import compute_fs_shard_range
    from megatron.core.optimizer.distrib_dion.split_child import build_split_child_dist_meta

    fs_group = dist.group.WORLD
    rf = case["rf"]
    split = tuple(case["split"])
    m, n = sum(split), case["n"]
    groups = {}

    def make_group(ranks, create_group):
        # dion_distrib_optimizer.py:263-284 (_ensure_child_group): cached, None for one rank
        if len(ranks) <= 1:
            return None
        if ranks not in groups:
            groups[ranks] = dist.new_group(list(ranks))
        return groups[ranks]

    axis = case.get("axis", "fs")
    tp = axis == "tp"
    # the fused parent: FS (or TP) row shard
    f0, f1 = compute_fs_shard_range(m, world, rank)
    pname = "mlp.linear_fc1"
    if tp:
        pcfg = DionParamConfig(has_tp_shard=True, use_tp_shard=True, tp_shard_dim=0, is_transposed=False)
        pmeta = DionDistMeta(shape=(f1 - f0, n), global_shape=(m, n), tp_shard_dim=0, rank_fraction=rf,
                             is_transposed=False, param_uid=(pname,), is_dion_param=True, param_name=pname,
                             tp_group=fs_group, tp_world_size=world, tp_rank=rank, local_shape=(f1 - f0, n),
                             param_config=pcfg)
    else:
        pcfg = DionParamConfig(has_fs_shard=True, use_fs_shard=True, fs_shard_dim=0, is_transposed=False)
        pmeta = DionDistMeta(shape=(f1 - f0, n), global_shape=(m, n), fs_start_idx=f0, fs_end_idx=f1,
                             fs_shard_dim=0, rank_fraction=rf, is_transposed=False, param_uid=(pname,),
                             is_dion_param=True, param_name=pname, fs_group=fs_group, fs_world_size=world,
                             fs_rank=rank, local_shape=(f1 - f0, n), param_config=pcfg)
    pmeta.linear_split_rows = split
    pmeta.linear_partition_stride = 1
    w_full = torch.randn(m, n, generator=torch.Generator().manual_seed(3000)) * 0.02
    params = {pname: torch.nn.Parameter(w_full[f0:f1].clone().contiguous())}
    grads_full = [(torch.randn(m, n, generator=torch.Generator().manual_seed(77 + 13 * s)) * 1e-3)
                  .to(torch.bfloat16).float() for s in range(case["steps"])]
    info = {pname: dict(m=m, n=n, rows=[f0, f1], split=list(split), axis=axis, children={})}
    states = {pname: dict(momentum=torch.zeros_like(params[pname]))}

    # an ordinary sharded matrix in the same optimizer: FS on its columns, or TP on its rows
    bname, bm, bn = case["plain"]
    br = max(1, int(min(math.ceil(rf * min(bm, bn)), bm, bn)))
    low = rf < 1.0 and (bm + bn) * br < bm * bn
    bw = torch.randn(bm, bn, generator=torch.Generator().manual_seed(1000)) * 0.02
    bq = torch.randn(bn, br, generator=torch.Generator().manual_seed(2000))
    bg_full = [(torch.randn(bm, bn, generator=torch.Generator().manual_seed(99 + 17 * s)) * 1e-3)
               .to(torch.bfloat16).float() for s in range(case["steps"])]
    if tp:
        c0, c1 = compute_fs_shard_range(bm, world, rank)      # this rank's rows
        q0, q1 = compute_fs_shard_range(br, world, rank)      # and its columns of r
        bcfg = DionParamConfig(has_tp_shard=True, use_tp_shard=True, tp_shard_dim=0, is_transposed=False,
                               use_low_rank_sync=low)
        bmeta = DionDistMeta(shape=(c1 - c0, bn), global_shape=(bm, bn), tp_shard_dim=0, rank_fraction=rf,
                             is_transposed=False, param_uid=(bname,), is_dion_param=True, param_name=bname,
                             tp_group=fs_group, tp_world_size=world, tp_rank=rank, local_shape=(c1 - c0, bn),
                             param_config=bcfg)
        params[bname] = torch.nn.Parameter(bw[c0:c1].clone().contiguous())
        states[bname] = dict(momentum=torch.zeros_like(params[bname]), Q=bq[:, q0:q1].clone().contiguous(), r=br,
                             local_shape=(c1 - c0, bn), global_shape=(bm, bn))
        bgrads = [g[c0:c1].clone().contiguous() for g in bg_full]
        info[bname] = dict(m=bm, n=bn, rows=[c0, c1], qcols=[q0, q1], r=br)
    else:
        c0, c1 = compute_fs_shard_range(bn, world, rank)
        bcfg = DionParamConfig(has_fs_shard=True, use_fs_shard=True, fs_shard_dim=1, is_transposed=False,
                               use_low_rank_sync=low)
        bmeta = DionDistMeta(shape=(bm, c1 - c0), global_shape=(bm, bn), fs_start_idx=c0, fs_end_idx=c1,
                             fs_shard_dim=1, rank_fraction=rf, is_transposed=False, param_uid=(bname,),
                             is_dion_param=True, param_name=bname, fs_group=fs_group, fs_world_size=world,
                             fs_rank=rank, local_shape=(bm, c1 - c0), param_config=bcfg)
        params[bname] = torch.nn.Parameter(bw[:, c0:c1].clone().contiguous())
        states[bname] = dict(momentum=torch.zeros_like(params[bname]), Q=bq[c0:c1].clone().contiguous(), r=br,
                             local_shape=(bm, c1 - c0), global_shape=(bm, bn))
        bgrads = [g[:, c0:c1].clone().contiguous() for g in bg_full]
        info[bname] = dict(m=bm, n=bn, cols=[c0, c1], r=br)

    # children: dion_distrib_optimizer.py:2940-2998 (_resolve_linear_child_row_group_layout)
    children = {}
    for kidx, kind in enumerate(KINDS):
        cs = 0 if kind == "gate" else split[0]
        ce = cs + split[0 if kind == "gate" else 1]
        ranges = []
        for k in range(world):
            a, b = compute_fs_shard_range(m, world, k)
            lo, hi = max(a, cs), min(b, ce)
            ranges.append(None if hi <= lo else (lo - cs, hi - cs))
        lay = resolve_row_child_layout(parent_group=fs_group, parent_world_size=world, parent_rank=rank,
                                       child_rows=ce - cs, child_ranges=tuple(ranges), label="TP" if tp else "FS",
                                       detail=f"{pname}:{kind}", error_prefix="LINEAR_CHILD", create_group=True,
                                       make_group=make_group)
        cgs = d_lin.linear_child_global_shape((m, n), split, kind)
        members = [k for k in range(world) if ranges[k] is not None]
        entry = dict(member_ranges=[list(x) if x is not None else None for x in ranges], members=members,
                     child_world=int(lay.world_size), child_rank=int(lay.rank), start=int(lay.start_idx),
                     end=int(lay.end_idx), row_shard_sizes=list(lay.row_shard_sizes), global_shape=list(cgs))
        info[pname]["children"][kind] = entry
        if not d_lin.linear_child_has_local_overlap(split, pmeta, kind):
            continue
        cls = d_lin.linear_child_local_shape(tuple(params[pname].shape), split, pmeta, kind)
        if tp:
            fs_lay, tp_lay = (None, 1, -1, -1, -1, None), lay.as_tuple()
        else:
            fs_lay, tp_lay = lay.as_tuple(), (None, 1, 0, -1, -1, None)
        cmeta = build_split_child_dist_meta(
            parent_dist_meta=pmeta, child_uid=d_lin.linear_child_param_uid((pname,), kind),
            child_name=d_lin.linear_child_name(pname, kind), child_local_shape=cls, child_global_shape=cgs,
            fs_layout=fs_lay, tp_layout=tp_lay,
            child_fields={"linear_split_rows": split, "linear_partition_stride": 1, "is_linear_child": True,
                          "linear_child_kind": kind},
            error_prefix="LINEAR_CHILD", use_low_rank_sync=True, rank_fraction_default=rf,
            rank_multiple_of_default=1)
        ccfg = cmeta.param_config
        r = max(1, int(min(math.ceil(rf * min(cgs)), *cgs)))
        q_rows_g = cgs[0] if ccfg.is_transposed else cgs[1]
        q_full = torch.randn(q_rows_g, r, generator=torch.Generator().manual_seed(4000 + kidx))
        if tp and int(lay.world_size) > 1:
            # TP-sharded child: P rows on the TP side, Q = this rank's columns of r (state.py:159-217)
            assert not ccfg.is_transposed and ccfg.use_tp_shard
            qc0, qc1 = compute_fs_shard_range(r, int(lay.world_size), int(lay.rank))
            q_loc = q_full[:, qc0:qc1]
        else:
            q_loc = q_full[lay.start_idx:lay.end_idx] if ccfg.is_transposed and int(lay.world_size) > 1 else q_full
        children[cmeta.param_name] = dict(kind=kind, meta=cmeta, cfg=ccfg,
                                          state=dict(Q=q_loc.clone().contiguous(), r=r, local_shape=tuple(cls),
                                                     global_shape=tuple(cgs)))
        entry.update(name=cmeta.param_name, r=r, local_shape=list(cls), is_transposed=bool(ccfg.is_transposed),
                     fs_shard_dim=int(getattr(cmeta, "fs_shard_dim", -1)),
                     fs_world_size=int(getattr(cmeta, "fs_world_size", 1)),
                     tp_world_size=int(getattr(cmeta, "tp_world_size", 1)),
                     use_fs_shard=bool(ccfg.use_fs_shard), use_tp_shard=bool(ccfg.use_tp_shard),
                     use_low_rank_sync=bool(ccfg.use_low_rank_sync),
                     row_shard_sizes=list(getattr(cmeta, "row_shard_sizes", None) or ()),
                     tensor_row_shard_sizes=list(getattr(cmeta, "tensor_row_shard_sizes", None) or ()))

    opt = MegatronDion([params[k] for k in params], rank_fraction=rf, use_fs_collectives=True, **HYPER)
    for k in params:
        opt.state[params[k]] = states[k]
    grads_now, cache = {}, {}

    def route():
        p = params[pname]
        steps = [DionStepParam(param=params[bname], grad=grads_now[bname], optimizer_state=opt.state[params[bname]],
                               optim_group=opt.param_groups[0], config=bcfg, dist_meta=bmeta)]
        for cname, ch in sorted(children.items()):
            st = dict(ch["state"])
            st["momentum"] = d_lin.read_linear_child(opt.state[p]["momentum"], split, pmeta, ch["kind"])

            def commit(up, um, kind=ch["kind"]):
                d_lin.write_linear_child_(p.data, up, split, pmeta, kind)
                d_lin.write_linear_child_(opt.state[p]["momentum"], um, split, pmeta, kind)

            steps.append(DionStepParam(
                param=d_lin.read_linear_child(p.data, split, pmeta, ch["kind"]),
                grad=d_lin.read_linear_child(grads_now[pname], split, pmeta, ch["kind"]),
                optimizer_state=st, optim_group=opt.param_groups[0], config=ch["cfg"], dist_meta=ch["meta"],
                commit_update=commit))
            ch["live_state"] = st
        return build_dion_batches(
            dion_params=steps, use_fs_collectives=True, state_replica_group=None,
            replica_validation_group=dist.group.WORLD, batch_key_cache=cache, global_rank=rank,
            group_size=dist.get_world_size, get_replicate_group=lambda: None,
            resolve_ortho_group=lambda c, m_: m_.tp_group if is_p_tp_sharded(c, tp_active=c.use_tp_shard) else None,
            resolve_tp_group=lambda m_, expect_group: m_.tp_group,
            resolve_fs_group_from_meta=lambda m_, expect_group: m_.fs_group), []

    opt.enable_distributed_mode(route_step_params=route)
    rec = {"batches": []}
    sketches = []
    orig_sketch = d_ortho.generate_random_sketch_matrix

    def sketch_wrap(P, oversample=1.25, make_sketch=None):
        S = orig_sketch(P, oversample=oversample, make_sketch=make_sketch)
        sketches.append(S.detach().clone())
        return S

    d_ortho.generate_random_sketch_matrix = sketch_wrap
    orig_bdu = d_rt.batch_dion_update_async

    def bdu_wrap(optimizer, params_l, *args, **kwargs):
        real, bg = args[8], args[10]
        dm = args[3]
        members = [(dm[i].param_name if dm[i] is not None else "<pad>") for i in range(len(params_l))]
        rec["batches"].append(dict(members=members, real=int(real), kind=str(bg.kernel_kind)))
        return (yield from orig_bdu(optimizer, params_l, *args, **kwargs))

    d_rt.batch_dion_update_async = bdu_wrap
    arrays = {}
    meta = {"steps": [], "info": info}
    for step in range(case["steps"]):
        grads_now[pname] = grads_full[step][f0:f1].clone().contiguous()
        grads_now[bname] = bgrads[step].clone()
        for k, p in params.items():
            arrays[f"s{step}_{k}_W0"] = p.detach().clone()
            arrays[f"s{step}_{k}_M0"] = opt.state[p]["momentum"].clone()
            arrays[f"s{step}_{k}_G"] = grads_now[k].clone()
        arrays[f"s{step}_{bname}_Q0"] = opt.state[params[bname]]["Q"].clone()
        for cname, ch in children.items():
            arrays[f"s{step}_{cname}_Q0"] = ch["state"]["Q"].clone()
        rec["batches"] = []
        n_sk = len(sketches)
        opt.step()
        for k, p in params.items():
            arrays[f"s{step}_{k}_W1"] = p.detach().clone()
            arrays[f"s{step}_{k}_M1"] = opt.state[p]["momentum"].clone()
        arrays[f"s{step}_{bname}_Q1"] = opt.state[params[bname]]["Q"].clone()
        for cname, ch in children.items():
            ch["state"]["Q"] = ch["live_state"]["Q"]
            arrays[f"s{step}_{cname}_Q1"] = ch["state"]["Q"].clone()
        for i, S in enumerate(sketches[n_sk:]):
            arrays[f"s{step}_sketch{i}"] = S
        meta["steps"].append(dict(batches=rec["batches"], sketches=len(sketches) - n_sk))
    np.savez_compressed(out_path, **{k: v.detach().float().numpy() for k, v in arrays.items()})
    with open(out_path + ".json", "w") as fh:
        json.dump(meta, fh)
    dist.barrier()
    dist.destroy_process_group()


def main():
    path = os.path.join(HERE, "manifest_split_partial.json")
    manifest = {"hyper": HYPER, "cases": []}
    port = 29811
    for case in CASES:
        port += 1
        world = case["world"]
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
        entry = dict(case, rank_meta=metas)
        manifest["cases"].append(entry)
        print("wrote", out, os.path.getsize(out), "bytes", flush=True)
    with open(path, "w") as fh:
        json.dump(manifest, fh, indent=1, default=list)


if __name__ == "__main__":
    sys.exit(main())
