"""The speedrun's FS x TP topology on 4 gloo ranks (FS = 2 x TP = 2), CPU.

examples/dion/speedrun_nanogpt_mcore.py:36-62, 395-431 runs Dion with FS and TP together, bf16
momentum and Q, and split QKV children.  Here the product's own adapter
(`attach_dp_routing(..., fs_group=, fs_shards=, tp_group=, tp_shards=)` with `split_qkv=True`)
builds the batches: every matrix is TP-sharded on one dim and FS-sharded on the other, and the
fused QKV parent (TP on its rows, FS on its columns) is optimised as q / k / v children of its
shard (split.split_child_layouts).  The batch runtime (`_tp_batch_update`: Q all-gather over TP,
P all-reduce over FS, the row-sharded RCQR over TP, R sum over TP, the column norm over the FS
q_norm group) runs with the oracle codec, the sketch slices are the reference's seeded ones, and
every shard on every rank is checked against the reference's own captures
(tests/golden/make_golden_fstp.py), which also pin the children's layout as the reference's
helpers compute it (qkv.py, row_child.py, split_child.py).
"""
import json
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.slow

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
CASES = ["x1_fs2tp2_speedrun", "x2_fs2tp2_speedrun_bf16"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def load_case(name):
    with open(os.path.join(GOLDEN, "manifest_fstp.json")) as fh:
        man = json.load(fh)
    entry = next(c for c in man["cases"] if c["name"] == name)
    with np.load(os.path.join(GOLDEN, name + ".npz")) as z:
        arr = {k: z[k] for k in z.files}
    return man, entry, arr


def _worker(rank, world, port, name, out_dir, deferred, device):
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    import megatron_dion_amd as mda
    from megatron_dion_amd.optimizer import attach_dp_routing
    from oracle import dion_oracle as O
    from oracle.cpu_codec import OracleCodec

    dev = torch.device(device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    man, entry, arr = load_case(name)
    h, TP, FS = man["hyper"], int(man["tp"]), int(man["fs"])
    tp_groups = [dist.new_group([0, 1]), dist.new_group([2, 3])]   # the capture's layout
    fs_groups = [dist.new_group([0, 2]), dist.new_group([1, 3])]
    tp_group, fs_group = tp_groups[rank // TP], fs_groups[rank % TP]
    info = entry["rank_meta"][rank]["info"]

    def t(step, key):
        return torch.from_numpy(arr[f"r{rank}_s{step}_{key}"].copy()).to(dev)

    params, fs_shards, tp_shards = {}, {}, {}
    for n, m, k, tdim in entry["mats"]:
        params[n] = torch.nn.Parameter(t(0, f"{n}_W0").clone())
    for pname, groups, split, k in entry["qkv"]:
        params[pname] = torch.nn.Parameter(t(0, f"{pname}_W0").clone())
        params[pname].qkv_split_shapes = tuple(split)
    for n, d in info.items():
        gshape, tdim = (int(d["m"]), int(d["n"])), int(d["tdim"])
        rows, cols = d["rows"], d["cols"]
        trange, frange = (rows, cols) if tdim == 0 else (cols, rows)
        tp_shards[n] = (gshape, tdim, trange[0], trange[1])
        fs_shards[n] = (gshape, 1 - tdim, frange[0], frange[1])
    kw = {}
    if dev.type == "cpu":
        kw["codec"] = OracleCodec(deferred=deferred)
    if entry["bf16"]:
        kw["mixed_precision_config"] = mda.DionMixedPrecisionConfig(momentum_dtype=torch.bfloat16,
                                                                    q_dtype=torch.bfloat16)
    names = list(params)
    opt = mda.MegatronDion([params[n] for n in names], lr=h["lr"], mu=h["mu"], weight_decay=h["weight_decay"],
                           rank_fraction=float(entry["rf"]), epsilon=h["epsilon"],
                           rcqr_oversample=h["rcqr_oversample"], defer_error_feedback=deferred, split_qkv=True, **kw)
    attach_dp_routing(opt, [(n, params[n]) for n in names], fs_group=fs_group, fs_shards=fs_shards,
                      tp_group=tp_group, tp_shards=tp_shards)
    layout = {}
    for n, m, k, tdim in entry["mats"]:
        st = opt.state[params[n]]
        assert st["r"] == info[n]["r"], (n, st["r"], info[n]["r"])
        assert tuple(st["Q"].shape) == tuple(t(0, f"{n}_Q0").shape)
        st["Q"].copy_(t(0, f"{n}_Q0"))
    for pname, *_ in entry["qkv"]:
        st = opt.state[params[pname]]
        for kind, ch in info[pname]["children"].items():
            q = st[f"qkv_{kind}_Q"]
            assert tuple(q.shape) == tuple(t(0, f"{ch['name']}_Q0").shape), (kind, tuple(q.shape))
            q.copy_(t(0, f"{ch['name']}_Q0"))
            layout[kind] = dict(local_shape=list(st[f"qkv_{kind}_local_shape"]),
                                global_shape=list(st[f"qkv_{kind}_global_shape"]), r=int(st[f"qkv_{kind}_r"]))
    state = {"step": 0}

    def sketch_override(batch):
        out = {}
        for i, meta in enumerate(list(batch.dist_metas)[:int(batch.real_batch_size)]):
            r = int(batch.entries[i].optimizer_state["r"])
            gm, gn = (int(x) for x in meta.global_shape)
            transposed = bool(meta.param_config.is_transposed)
            ks = O.sketch_rows(r, h["rcqr_oversample"])
            seed = O.distributed_sketch_seed(state["step"] + 1, meta.param_uid, meta.param_name)
            start, end = int(meta.extra["tp_start_idx"]), int(meta.extra["tp_end_idx"])
            out[i] = O.reference_sharded_sketch(seed, ks, gn if transposed else gm, start, end - start).to(dev)
        return out

    opt._sketch_override = sketch_override
    results = {"layout": layout}
    for step in range(int(entry["steps"])):
        state["step"] = step
        for n in names:
            params[n].grad = t(step, f"{n}_G").clone()
        batches, _ = opt._route_step_params()
        results[f"s{step}_batches"] = [dict(members=[(d.param_name if d is not None else "<pad>")
                                                     for d in b.dist_metas] + ["<pad>"] * (len(b.entries) -
                                                                                           len(b.dist_metas)),
                                            real=int(b.real_batch_size), kind=b.batch_group.kernel_kind,
                                            row_sizes=[list(d.row_shard_sizes or ()) for d in b.dist_metas
                                                       if d is not None])
                                       for b in batches]
        opt.step()
        if deferred and step == int(entry["steps"]) - 1:
            opt.flush_error_feedback()
        for n in names:
            st = opt.state[params[n]]
            results[f"s{step}_{n}_W"] = params[n].detach().cpu().clone()
            results[f"s{step}_{n}_M"] = st["momentum"].float().cpu().clone()
            if n in dict((e[0], 1) for e in entry["mats"]):
                results[f"s{step}_{n}_Q"] = st["Q"].float().cpu().clone()
        for pname, *_ in entry["qkv"]:
            for kind, ch in info[pname]["children"].items():
                results[f"s{step}_{ch['name']}_Q"] = opt.state[params[pname]][f"qkv_{kind}_Q"].float().cpu().clone()
    torch.save(results, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def run_fstp(name, deferred=False, device="cpu"):
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_worker, args=(4, _free_port(), name, tmp, deferred, device), nprocs=4, join=True,
                           start_method="spawn")
        return [torch.load(os.path.join(tmp, f"rank{r}.pt"), weights_only=True) for r in range(4)]


def _maxrel(a, b):
    return (a.double() - b.double()).abs().max().item() / max(b.double().abs().max().item(), 1e-30)


def check_fstp_results(res, name, deferred, tol, bf16_tols=None):
    _, entry, arr = load_case(name)
    worst = 0.0
    for rank in range(4):
        meta = entry["rank_meta"][rank]
        for pname, *_ in entry["qkv"]:
            for kind, ch in meta["info"][pname]["children"].items():
                lay = res[rank]["layout"][kind]
                assert lay == dict(local_shape=ch["local_shape"], global_shape=ch["global_shape"], r=ch["r"]), \
                    (rank, kind, lay, ch)
        for step in range(int(entry["steps"])):
            ref_b = meta["steps"][step]["batches"]
            got_b = res[rank][f"s{step}_batches"]
            assert [(b["members"], b["real"], b["kind"]) for b in got_b] == \
                [(b["members"], b["real"], b["kind"]) for b in ref_b], (rank, step, got_b, ref_b)
            for b in got_b:
                for member, rs in zip(b["members"], b["row_sizes"]):
                    if "::" in member:
                        pname, kind = member.split("::")
                        assert rs == meta["info"][pname]["children"][kind]["row_shard_sizes"], (member, rs)
            keys = []
            for n, *_ in entry["mats"]:
                keys += [(n, "W", "W1"), (n, "Q", "Q1")]
                if not deferred or step == int(entry["steps"]) - 1:
                    keys.append((n, "M", "M1"))
            for pname, *_ in entry["qkv"]:
                keys += [(pname, "W", "W1"), (pname, "M", "M1")]
                keys += [(ch["name"], "Q", "Q1") for ch in meta["info"][pname]["children"].values()]
            for n, k, ref in keys:
                want = torch.from_numpy(arr[f"r{rank}_s{step}_{n}_{ref}"].copy())
                err = _maxrel(res[rank][f"s{step}_{n}_{k}"].float(), want)
                worst = max(worst, err)
                bar = bf16_tols[k] if (bf16_tols and entry["bf16"]) else tol
                assert err <= bar, (name, rank, step, n, k, err)
    return worst


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("deferred", [False, True], ids=["eager_ef", "deferred_ef"])
def test_gloo_fs2tp2_speedrun_matches_reference(name, deferred):
    res = run_fstp(name, deferred=deferred)
    check_fstp_results(res, name, deferred, 1e-5)
