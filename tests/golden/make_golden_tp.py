"""Golden fixtures of the TP ("fsdp_tp") kernel kind, captured from the REFERENCE.

Run ONLY in the build container (the reference tree does not exist on the GPU box):

    PYTHONPATH=/root/reference DION_DISABLE_TORCH_COMPILE=1 python tests/golden/make_golden_tp.py

With tensor parallelism the reference shards a Dion matrix over the TP group on the P-row
side (dion/state.py:304-310 puts tp_shard_dim on m_P; is_p_tp_sharded, :407-416) and Q's
columns over the same group (resolve_q_state_layout, :159-217).  A batch then takes the
"fsdp_tp" kind (distrib_dion/batches.py:571-577): Q is all-gathered across TP
(runtime.py:680-873), P = X Q is orthonormalised by the row-sharded randomised Cholesky QR
(ortho.py:682-834, seeded sharded sketch :575-640), R = X^T P is all-reduced (sum) over TP
(runtime.py:923-962), and the updated Q is re-sharded by columns (ortho.py:837-871,
runtime.py:1101-1132).  This script drives the reference's own MegatronDion.step over its own
build_dion_batches on 2 gloo ranks (TP group = WORLD, no FS, no replicas) and records, per
rank and step, each matrix's local W / M / Q / G before and after, every distributed
orthogonalize call (local P in and out, the local sketch slice) and the batch schedule.
Only data is committed.
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

# name, mats = (name, m_global, n_global, tp_shard_dim), rank_fraction, steps
CASES = [
    # rows sharded (tp_shard_dim 0 -> not transposed, P rows = m), one batch of 2, r = 8 (4 + 4)
    dict(name="t1_tp2_rows", mats=[("a", 64, 48, 0), ("b", 64, 48, 0)], rf=1 / 6, steps=2),
    # columns sharded (tp_shard_dim 1 -> transposed, P rows = n), r = 8
    dict(name="t2_tp2_cols_T", mats=[("x", 40, 96, 1), ("y", 40, 96, 1)], rf=0.2, steps=2),
    # odd rank (r = 5: Q columns 3 + 2) and a single-matrix batch of another key
    dict(name="t3_tp2_odd_r_mixed", mats=[("u", 48, 36, 0), ("w", 56, 40, 1)], rf=0.125, steps=2),
    # global P rows <= r: the plain-QR branch of the distributed orthogonalize (ortho.py:752-775)
    dict(name="t4_tp2_plain_qr", mats=[("p", 16, 64, 0)], rf=1.0, steps=2),
    # the speedrun's bf16 momentum and Q (examples/dion/speedrun_nanogpt_mcore.py:36-62, 417-431:
    # TP = 2 with mixed_precision): rows, and odd r with a transposed key
    dict(name="t5_tp2_bf16_rows", mats=[("a", 64, 48, 0), ("b", 64, 48, 0)], rf=1 / 6, steps=2, bf16=True),
    dict(name="t6_tp2_bf16_odd_mixed", mats=[("u", 48, 36, 0), ("w", 56, 40, 1)], rf=0.125, steps=2, bf16=True),
]
HYPER = dict(lr=0.01, mu=0.95, weight_decay=0.01, epsilon=1e-8, rcqr_oversample=1.25,
             scale_mode="spectral", extra_scale_factor=0.2)


def split_range(size, world, rank):
    """dion/ortho.py:247-259 (_split_range): remainder on the first ranks."""
    base, rem = size // world, size % world
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def _worker(rank, world, case, port, out_path):
    os.environ["DION_DISABLE_TORCH_COMPILE"] = "1"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    torch.manual_seed(0)
    from megatron.core.optimizer.dion import ortho as d_ortho
    from megatron.core.optimizer.dion import runtime as d_rt
    from megatron.core.optimizer.dion.algorithm import MegatronDion
    from megatron.core.optimizer.dion.state import is_p_tp_sharded
    from megatron.core.optimizer.dion.types import (DionDistMeta, DionMixedPrecisionConfig, DionParamConfig,
                                                    DionStepParam)
    from megatron.core.optimizer.distrib_dion.batches import build_dion_batches

    tp_group = dist.group.WORLD
    rf = case["rf"]
    names = [n for n, _, _, _ in case["mats"]]
    params, cfgs, metas, info = {}, {}, {}, {}
    for idx, (name, m, n, dim) in enumerate(case["mats"]):
        split = m if dim == 0 else n
        start, end = split_range(split, world, rank)
        w_full = torch.randn(m, n, generator=torch.Generator().manual_seed(1000 + idx)) * 0.02
        w_loc = w_full[start:end] if dim == 0 else w_full[:, start:end]
        lm, ln = w_loc.shape
        transposed = dim == 1                       # dion/state.py:304-310
        r = max(1, int(min(math.ceil(rf * min(m, n)), m, n)))
        c0, c1 = split_range(r, world, rank)        # Q columns of this TP rank (state.py:190-194)
        q_rows = m if transposed else n             # the unsharded side
        q_full = torch.randn(q_rows, r, generator=torch.Generator().manual_seed(2000 + idx))
        q_loc = q_full[:, c0:c1].clone().contiguous()
        low = rf < 1.0 and (m + n) * r < m * n
        cfgs[name] = DionParamConfig(has_tp_shard=True, use_tp_shard=True, tp_shard_dim=dim,
                                     is_transposed=transposed, use_low_rank_sync=low)
        metas[name] = DionDistMeta(shape=(lm, ln), global_shape=(m, n), tp_shard_dim=dim, rank_fraction=rf,
                                   is_transposed=transposed, param_uid=(name,), is_dion_param=True, param_name=name,
                                   tp_group=tp_group, tp_world_size=world, tp_rank=rank, local_shape=(lm, ln),
                                   param_config=cfgs[name])
        params[name] = torch.nn.Parameter(w_loc.clone().contiguous())
        grads = []
        for step in range(case["steps"]):
            g_full = torch.randn(m, n, generator=torch.Generator().manual_seed(99 + 17 * step + 131 * idx)) * 1e-3
            g_full = g_full.to(torch.bfloat16).float()
            grads.append((g_full[start:end] if dim == 0 else g_full[:, start:end]).clone().contiguous())
        info[name] = dict(m=m, n=n, dim=dim, start=start, end=end, r=r, c0=c0, c1=c1, q=q_loc, grads=grads)
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
            resolve_ortho_group=lambda c, m: m.tp_group if is_p_tp_sharded(c, tp_active=c.use_tp_shard) else None,
            resolve_tp_group=lambda m, expect_group: m.tp_group,
            resolve_fs_group_from_meta=lambda m, expect_group: None), []

    opt.enable_distributed_mode(route_step_params=route)
    rec = {"batches": [], "ortho": []}
    sketches = []
    orig_sk = d_ortho._make_sharded_sketch

    def sk_wrap(**kw):
        S = orig_sk(**kw)
        sketches.append(S.detach().clone())
        return S

    d_ortho._make_sharded_sketch = sk_wrap
    orig_dortho = d_rt.distributed_orthogonalize

    def dortho_wrap(optimizer, P_batch, **kw):
        n_before = len(sketches)
        out = orig_dortho(optimizer, P_batch, **kw)
        S = sketches[-1] if len(sketches) > n_before else None
        rec["ortho"].append(dict(p_in=P_batch.detach().clone(), p_out=out.detach().clone(), s=S))
        return out

    d_rt.distributed_orthogonalize = dortho_wrap
    orig_bdu = d_rt.batch_dion_update_async

    def bdu_wrap(optimizer, params_l, *args, **kwargs):
        real, bg = args[8], args[10]
        members = [id2name.get(id(p), "<pad>") for p in params_l]
        dm = args[3]
        members = [mm if dm[i] is not None else "<pad>" for i, mm in enumerate(members)]
        rec["batches"].append(dict(members=members, real=int(real), kind=str(bg.kernel_kind)))
        return (yield from orig_bdu(optimizer, params_l, *args, **kwargs))

    d_rt.batch_dion_update_async = bdu_wrap
    arrays = {}
    meta = {"steps": [], "shards": {n: {k: info[n][k] for k in ("m", "n", "dim", "start", "end", "r", "c0", "c1")}
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
        sketches.clear()
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
    path = os.path.join(HERE, "manifest_tp.json")
    manifest = {"hyper": HYPER, "cases": []}
    if only and os.path.exists(path):
        with open(path) as fh:
            manifest = json.load(fh)
        manifest["cases"] = [c for c in manifest["cases"] if c["name"] not in only]
    port = 29761
    world = 2
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
        manifest["cases"].append(entry)
        print("wrote", out, os.path.getsize(out), "bytes", flush=True)
    order = [c["name"] for c in CASES]
    manifest["cases"].sort(key=lambda c: order.index(c["name"]) if c["name"] in order else len(order))
    with open(path, "w") as fh:
        json.dump(manifest, fh, indent=1, default=list)


if __name__ == "__main__":
    sys.exit(main())
