"""Container-only check of the drop-in boundary against the reference itself.

Run ONLY in the build container (the reference tree does not exist on the GPU box):

    PYTHONPATH=/root/reference DION_DISABLE_TORCH_COMPILE=1 python scripts/ref/ref_boundary_check.py

For world sizes 1 and 2 (gloo loopback) it builds the SAME inputs twice:

  A. the reference: its MegatronDion (dion/algorithm.py:29) routed through its own
     build_dion_batches (distrib_dion/batches.py:971), one step after another; every
     sketch the reference draws (dion/ortho.py:643-662) is recorded;
  B. the reference's own batch builder again (its DionBatch objects, its batch keys,
     order, chunking and padding), but each batch executed by THIS repo's runtime:
     megatron_dion_amd.runtime.run_dion_batch_async under its AsyncRuntime, with the
     oracle codec (oracle/cpu_codec.py) replaying A's sketches in call order.

It then compares W, momentum and Q after every step (max-relative, bar 1e-6).  The sharded
kinds ("fsdp", "fsdp_tp", FS x TP) are checked the same way by ref_boundary_check_sharded.py.
The matrix set avoids two same-shape batches in flight at once, where the reference
shares one P buffer between them (defect 1).  The result is written
to profiles/r04/ref_boundary_check_ddp.json.
"""
import json
import os
import socket
import sys
import tempfile

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# (name, m, n): one full W = 2 batch per shape, one padded batch, both orientations
MATS = [("a", 96, 64), ("b", 96, 64), ("t", 48, 112), ("u", 48, 112), ("v", 64, 160), ("odd", 80, 48)]
R_FRAC = 0.25
STEPS = 3
HYPER = dict(lr=0.01, mu=0.95, weight_decay=0.01, epsilon=1e-8, rcqr_oversample=1.25)


def _inputs(rank):
    out = {}
    for idx, (name, m, n) in enumerate(MATS):
        w0 = torch.randn(m, n, generator=torch.Generator().manual_seed(1000 + idx)) * 0.02
        r = max(1, int(R_FRAC * min(m, n)))
        q0 = torch.randn(min(m, n), r, generator=torch.Generator().manual_seed(2000 + idx))
        gs = [(torch.randn(m, n, generator=torch.Generator().manual_seed(99 + rank + 17 * s + 131 * idx))
               * 1e-3).to(torch.bfloat16).float() for s in range(STEPS)]
        out[name] = (w0, q0, gs, r)
    return out


def _ref_setup(opt_cls, inputs, types):
    DionDistMeta, DionParamConfig = types
    params, configs, metas = {}, {}, {}
    for name, m, n in MATS:
        w0, q0, _, r = inputs[name]
        params[name] = torch.nn.Parameter(w0.clone())
    opt = opt_cls([params[n] for n, _, _ in MATS], rank_fraction=R_FRAC, **HYPER)
    for name, m, n in MATS:
        w0, q0, _, r = inputs[name]
        low = (R_FRAC < 1.0) and ((m + n) * r < m * n)
        configs[name] = DionParamConfig(is_transposed=m < n, use_low_rank_sync=low)
        metas[name] = DionDistMeta(shape=(m, n), global_shape=(m, n), rank_fraction=R_FRAC, param_uid=(name,),
                                   is_dion_param=True, param_name=name, param_config=configs[name],
                                   is_transposed=m < n)
        opt.state[params[name]] = dict(momentum=torch.zeros(m, n), Q=q0.clone(), r=r, local_shape=(m, n),
                                       global_shape=(m, n))
    return opt, params, configs, metas


def _worker(rank, world, port, out_path):
    os.environ["DION_DISABLE_TORCH_COMPILE"] = "1"
    sys.path.insert(0, ROOT)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    torch.manual_seed(0)
    from megatron.core.optimizer.dion import ortho as d_ortho
    from megatron.core.optimizer.dion.algorithm import MegatronDion as RefDion
    from megatron.core.optimizer.dion.types import DionDistMeta, DionParamConfig, DionStepParam
    from megatron.core.optimizer.distrib_dion.batches import build_dion_batches

    import megatron_dion_amd as mda
    from megatron_dion_amd.runtime import AsyncRuntime, run_dion_batch_async
    from oracle.cpu_codec import OracleCodec

    inputs = _inputs(rank)
    group = dist.group.WORLD if world > 1 else None

    def builder(opt, params, configs, metas, grads, cache):
        steps = [DionStepParam(param=params[n], grad=grads[n], optimizer_state=opt.state[params[n]],
                               optim_group=opt.param_groups[0], config=configs[n], dist_meta=metas[n])
                 for n in sorted(params)]
        return build_dion_batches(
            dion_params=steps, use_fs_collectives=True, state_replica_group=None,
            replica_validation_group=dist.group.WORLD, batch_key_cache=cache, global_rank=rank,
            group_size=dist.get_world_size, get_replicate_group=lambda: group,
            resolve_ortho_group=lambda c, m: None, resolve_tp_group=lambda m, expect_group: None,
            resolve_fs_group_from_meta=lambda m, expect_group: None)

    # ---- A: the reference end to end, sketches recorded
    sketches = []
    orig = d_ortho.generate_random_sketch_matrix

    def rec(P, oversample=1.25, make_sketch=None):
        S = orig(P, oversample=oversample, make_sketch=make_sketch)
        sketches.append(S.detach().clone())
        return S

    d_ortho.generate_random_sketch_matrix = rec
    ref, rparams, configs, metas = _ref_setup(RefDion, inputs, (DionDistMeta, DionParamConfig))
    grads_now, cache_a = {}, {}
    ref.enable_distributed_mode(route_step_params=lambda: (
        builder(ref, rparams, configs, metas, grads_now, cache_a), []))
    ref_out = []
    for s in range(STEPS):
        for n in rparams:
            grads_now[n] = inputs[n][2][s].clone()
        ref.step()
        ref_out.append({n: (rparams[n].detach().clone(), ref.state[rparams[n]]["momentum"].clone(),
                            ref.state[rparams[n]]["Q"].clone()) for n in rparams})
    d_ortho.generate_random_sketch_matrix = orig

    # ---- B: the reference's batches, this repo's runtime + the oracle codec
    replay = iter(sketches)
    codec = OracleCodec(sketch_lookup=lambda P: next(replay))
    ours = mda.MegatronDion([torch.nn.Parameter(inputs[n][0].clone()) for n, _, _ in MATS], rank_fraction=R_FRAC,
                            codec=codec, defer_error_feedback=False, coalesce_local=False, **HYPER)
    oparams = {n: p for (n, _, _), p in zip(MATS, ours.param_groups[0]["params"])}
    for n, m, k in MATS:
        w0, q0, _, r = inputs[n]
        ours.state[oparams[n]].update(momentum=torch.zeros(m, k), Q=q0.clone(), r=r, local_shape=(m, k),
                                      global_shape=(m, k))
    cache_b = {}
    worst = {"W": 0.0, "M": 0.0, "Q": 0.0}
    schedules = []
    for s in range(STEPS):
        ograds = {n: inputs[n][2][s].clone() for n in oparams}
        batches = builder(ours, oparams, configs, metas, ograds, cache_b)
        schedules.append([(b.batch_group.kernel_kind, int(b.real_batch_size), len(b.entries)) for b in batches])
        ours._step_count += 1
        for g in ours.param_groups:
            g["step"] = g.get("step", 0) + 1
        with torch.no_grad():
            AsyncRuntime((run_dion_batch_async(ours, b) for b in batches), 3).run()
        for n in oparams:
            a = (oparams[n].detach(), ours.state[oparams[n]]["momentum"], ours.state[oparams[n]]["Q"])
            for k, x, y in zip("WMQ", a, ref_out[s][n]):
                err = (x.double() - y.double()).abs().max().item() / max(y.double().abs().max().item(), 1e-30)
                worst[k] = max(worst[k], err)
    result = {"world": world, "rank": rank, "steps": STEPS, "matrices": [list(x) for x in MATS],
              "rank_fraction": R_FRAC, "sketches_replayed": len(sketches), "max_rel": worst,
              "schedule_step0": schedules[0], "pass": max(worst.values()) <= 1e-6}
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(result, f)
    dist.barrier()
    dist.destroy_process_group()


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main():
    results = []
    for world in (1, 2):
        with tempfile.TemporaryDirectory() as tmp:
            out = os.path.join(tmp, "r.json")
            mp.start_processes(_worker, args=(world, _port(), out), nprocs=world, join=True, start_method="spawn")
            with open(out) as f:
                results.append(json.load(f))
    dest = os.path.join(ROOT, "profiles", "r04", "ref_boundary_check_ddp.json")
    os.makedirs(os.path.dirname(dest), exist_ok=True)
    with open(dest, "w") as f:
        json.dump(results, f, indent=1)
    print(json.dumps(results, indent=1))
    if not all(r["pass"] for r in results):
        raise SystemExit("boundary check FAILED")


if __name__ == "__main__":
    main()
