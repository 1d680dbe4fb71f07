"""Split-linear children owned by part of the FS row group, against the reference's captures.

A fused SwiGLU fc1 (gate 24 + up 24 rows, `split_linear`) FS-sharded on its rows over 3 ranks
(16 rows each) has a gate child on ranks {0, 1} and an up child on ranks {1, 2}: each child is
sharded over its own 2-rank sub-group (row_child.py:94-106, dion_distrib_optimizer.py:260-284),
rank 1 belongs to both and ranks 2 / 0 hold nothing of gate / up.  Over 2 ranks (24 | 24) each
child has one owner and is a whole matrix there ("ddp" with world 1).  TP-sharded rows over 3
ranks (partition stride 1) give the same owners, each child a TP-sharded ("fsdp_tp") matrix over
its 2-rank TP sub-group, replayed with the reference's seeded TP sketch slices.  The product's
adapter (`attach_dp_routing(..., fs_group=, fs_shards=)` or `tp_group=, tp_shards=`, with
`split_linear=True`) builds the layouts and the sub-groups; the batches, every shard of W and M and every Q on every rank are checked against
the reference's own run (tests/golden/make_golden_split_partial.py), whose sketches are replayed.
The CPU leg runs the oracle codec; the GPU leg (`-m gpu`) the HIP codec over the same gloo ranks.
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

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
CASES = ["p1_fs3_partial", "p2_fs2_single", "p3_tp3_partial"]
PARENT = "mlp.linear_fc1"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def load_case(name):
    with open(os.path.join(GOLDEN, "manifest_split_partial.json")) as fh:
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
    h = man["hyper"]
    info = entry["rank_meta"][rank]["info"]
    rmeta = entry["rank_meta"][rank]

    def t(step, key):
        return torch.from_numpy(arr[f"r{rank}_s{step}_{key}"].copy()).to(dev)

    bname, bm, bn = entry["plain"]
    names = [PARENT, bname]
    params = {n: torch.nn.Parameter(t(0, f"{n}_W0").clone()) for n in names}
    fc1 = params[PARENT]
    fc1.is_linear_fc1, fc1.linear_split_rows = True, tuple(entry["split"])
    pi, bi = info[PARENT], info[bname]
    tp = entry.get("axis") == "tp"
    if tp:  # TP on the rows of both (the plain matrix's Q holds this rank's columns of r)
        shards = {PARENT: ((pi["m"], pi["n"]), 0, pi["rows"][0], pi["rows"][1]),
                  bname: ((bi["m"], bi["n"]), 0, bi["rows"][0], bi["rows"][1])}
    else:
        shards = {PARENT: ((pi["m"], pi["n"]), 0, pi["rows"][0], pi["rows"][1]),
                  bname: ((bi["m"], bi["n"]), 1, bi["cols"][0], bi["cols"][1])}
    kw = {"codec": OracleCodec(deferred=deferred)} if dev.type == "cpu" else {}
    opt = mda.MegatronDion([params[n] for n in names], lr=h["lr"], mu=h["mu"], weight_decay=h["weight_decay"],
                           rank_fraction=float(entry["rf"]), epsilon=h["epsilon"],
                           rcqr_oversample=h["rcqr_oversample"], defer_error_feedback=deferred, split_linear=True,
                           **kw)
    if tp:
        attach_dp_routing(opt, [(n, params[n]) for n in names], tp_group=dist.group.WORLD, tp_shards=shards)
    else:
        attach_dp_routing(opt, [(n, params[n]) for n in names], fs_group=dist.group.WORLD, fs_shards=shards)
    st_b = opt.state[params[bname]]
    assert st_b["r"] == bi["r"]
    st_b["Q"].copy_(t(0, f"{bname}_Q0"))
    pstate = opt.state[fc1]
    layout = {}
    for kind, ch in pi["children"].items():
        key = f"linear_{kind}_Q"
        if "name" not in ch:  # not an owner: the reference builds no state here
            layout[kind] = None if key not in pstate else "unexpected"
            continue
        q = pstate[key]
        assert tuple(q.shape) == tuple(t(0, f"{ch['name']}_Q0").shape), (kind, tuple(q.shape))
        q.copy_(t(0, f"{ch['name']}_Q0"))
        layout[kind] = dict(local_shape=list(pstate[f"linear_{kind}_local_shape"]),
                            global_shape=list(pstate[f"linear_{kind}_global_shape"]), r=int(pstate[f"linear_{kind}_r"]))
    cur = {"step": 0}

    def sketch_override(batch):
        # the sketch this rank drew in the reference for the entry it owns (one per batch whose
        # owned entry is real); the reference's async runtime ran the ortho calls in another
        # order than the batches, the P heights (the sketch widths) tell them apart here
        grp = batch.batch_group
        if grp.kernel_kind == "fsdp_tp":
            # the reference's seeded TP sketch: this rank's rows of every real entry's sketch
            # (ortho.py:577-640, 682-779; tests/test_dist_gloo_fstp.py)
            out = {}
            for i, meta in enumerate(list(batch.dist_metas)[:int(batch.real_batch_size)]):
                r = int(batch.entries[i].optimizer_state["r"])
                gm, gn = (int(x) for x in meta.global_shape)
                ks = O.sketch_rows(r, h["rcqr_oversample"])
                seed = O.distributed_sketch_seed(cur["step"] + 1, meta.param_uid, meta.param_name)
                start, end = int(meta.extra["tp_start_idx"]), int(meta.extra["tp_end_idx"])
                rows = gn if meta.param_config.is_transposed else gm
                out[i] = O.reference_sharded_sketch(seed, ks, rows, start, end - start).to(dev)
            return out
        own = int(dist.get_rank(grp.q_norm_group)) if grp.kernel_kind == "fsdp" else 0
        if own >= int(batch.real_batch_size):
            return None
        meta = batch.dist_metas[own]
        gm, gn = (int(x) for x in meta.global_shape)
        rows = gn if meta.param_config.is_transposed else gm
        left = cur["left"]
        i = next(i for i in left if arr[f"r{rank}_s{cur['step']}_sketch{i}"].shape[-1] == rows)
        left.remove(i)
        return {own: torch.from_numpy(arr[f"r{rank}_s{cur['step']}_sketch{i}"].copy()).to(dev)}

    opt._sketch_override = sketch_override
    results = {"layout": layout}
    for step in range(int(entry["steps"])):
        cur.update(step=step, left=list(range(int(rmeta["steps"][step]["sketches"]))))
        for n in names:
            params[n].grad = t(step, f"{n}_G").clone()
        batches, _ = opt._route_step_params()
        results[f"s{step}_batches"] = [dict(members=[(d.param_name if d is not None else "<pad>")
                                                     for d in b.dist_metas] + ["<pad>"] * (len(b.entries) -
                                                                                           len(b.dist_metas)),
                                            real=int(b.real_batch_size), kind=b.batch_group.kernel_kind)
                                       for b in batches]
        opt.step()
        if deferred and step == int(entry["steps"]) - 1:
            opt.flush_error_feedback()
        assert not cur["left"], "sketches left over"
        for n in names:
            results[f"s{step}_{n}_W"] = params[n].detach().cpu().clone()
            results[f"s{step}_{n}_M"] = opt.state[params[n]]["momentum"].float().cpu().clone()
        results[f"s{step}_{bname}_Q"] = st_b["Q"].float().cpu().clone()
        for kind, ch in pi["children"].items():
            if "name" in ch:
                results[f"s{step}_{ch['name']}_Q"] = pstate[f"linear_{kind}_Q"].float().cpu().clone()
    torch.save(results, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def run_split_partial(name, deferred=False, device="cpu"):
    _, entry, _ = load_case(name)
    world = int(entry["world"])
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_worker, args=(world, _free_port(), name, tmp, deferred, device), nprocs=world,
                           join=True, start_method="spawn")
        return [torch.load(os.path.join(tmp, f"rank{r}.pt"), weights_only=True) for r in range(world)]


def _maxrel(a, b):
    return (a.double() - b.double()).abs().max().item() / max(b.double().abs().max().item(), 1e-30)


def check_split_partial(res, name, deferred, tol):
    _, entry, arr = load_case(name)
    bname = entry["plain"][0]
    worst = 0.0
    for rank in range(int(entry["world"])):
        meta = entry["rank_meta"][rank]
        pi = meta["info"][PARENT]
        for kind, ch in pi["children"].items():
            want = None if "name" not in ch else dict(local_shape=ch["local_shape"], global_shape=ch["global_shape"],
                                                      r=ch["r"])
            assert res[rank]["layout"][kind] == want, (rank, kind, res[rank]["layout"][kind], want)
        for step in range(int(entry["steps"])):
            ref_b = [(b["members"], b["real"], b["kind"]) for b in meta["steps"][step]["batches"]]
            got_b = [(b["members"], b["real"], b["kind"]) for b in res[rank][f"s{step}_batches"]]
            assert got_b == ref_b, (rank, step, got_b, ref_b)
            keys = [(PARENT, "W", "W1"), (bname, "W", "W1"), (bname, "Q", "Q1")]
            if not deferred or step == int(entry["steps"]) - 1:
                keys += [(PARENT, "M", "M1"), (bname, "M", "M1")]
            keys += [(ch["name"], "Q", "Q1") for ch in pi["children"].values() if "name" in ch]
            for n, k, ref in keys:
                want = torch.from_numpy(arr[f"r{rank}_s{step}_{n}_{ref}"].copy())
                err = _maxrel(res[rank][f"s{step}_{n}_{k}"].float(), want)
                worst = max(worst, err)
                assert err <= tol, (name, rank, step, n, k, err)
    return worst


@pytest.mark.slow
@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("deferred", [False, True], ids=["eager_ef", "deferred_ef"])
def test_gloo_split_linear_partial_owners_match_reference(name, deferred):
    res = run_split_partial(name, deferred=deferred)
    check_split_partial(res, name, deferred, 1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("deferred", [False, True], ids=["eager_ef", "deferred_ef"])
def test_hip_split_linear_partial_owners_match_reference(name, deferred):
    res = run_split_partial(name, deferred=deferred, device="cuda:0")
    check_split_partial(res, name, deferred, 2e-5)


def _reinit_worker(rank, world, ports, out_dir):
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    from megatron_dion_amd.optimizer import _child_row_group, _prepare_child_row_groups

    seen = []
    for port in ports:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        # rank 0 asks for one owner set, rank 1 for another: the union is created everywhere
        _prepare_child_row_groups([(0, 1)] if rank == 0 else [(0, 1, 2)])
        g = _child_row_group(dist.group.WORLD, [0, 1])
        g3 = _child_row_group(dist.group.WORLD, [0, 1, 2])
        t = torch.ones(1)
        if rank < 2:
            dist.all_reduce(t, group=g)
        dist.all_reduce(t, group=g3)
        seen.append((id(g), float(t.item())))
        dist.barrier()
        dist.destroy_process_group()
    torch.save(seen, os.path.join(out_dir, f"rank{rank}.pt"))


def test_child_groups_follow_a_reinitialised_world():
    """owner groups cached across destroy_process_group() / init_process_group()
    belonged to the old world.  init -> prepare -> destroy -> init -> prepare on 3 ranks: the
    second world creates (and uses) new groups on every rank."""
    world = 3
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_reinit_worker, args=(world, [_free_port(), _free_port()], tmp), nprocs=world,
                           join=True, start_method="spawn")
        seen = [torch.load(os.path.join(tmp, f"rank{r}.pt"), weights_only=True) for r in range(world)]
    for rank in range(world):
        (id0, v0), (id1, v1) = seen[rank]
        assert v0 == v1 == 5.0  # (1 + 1) on {0, 1}, then 2 + 2 + 1 over {0, 1, 2}
