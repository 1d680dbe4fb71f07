"""Container-only: the CPU restatement's step time against the reference's own step.

Run ONLY in the build container (needs /root/reference):

    PYTHONPATH=/root/reference DION_DISABLE_TORCH_COMPILE=1 python scripts/ref/cpu_speed_check.py

SURVEY.md 8(d) asks that the CPU baseline bench.py reports on the GPU box (oracle/
cpu_baseline.py: the product host runtime + the oracle codec) runs within +-20 % of the
reference's own step.  This times both on the same host, same threads, same inputs:

  config 1: GPT-125M 2D set, r = 16, 2 gloo ranks x (cores / 2) threads
  config 3: one Llama-3-8B layer, r = 64, 1 process x cores threads

reference = its MegatronDion.step (dion/algorithm.py:149) over its build_dion_batches
(distrib_dion/batches.py:971), eager, DION_DISABLE_TORCH_COMPILE=1; 1 warm-up, median of 5.
Writes profiles/r02/cpu_port_vs_reference.json.
"""
import json
import os
import socket
import statistics
import sys
import tempfile
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import cpu_baseline as CB  # noqa: E402

STEPS, WARMUP = 5, 1


def _ref_times(shapes, rank_fraction, rank, group):
    from megatron.core.optimizer.dion.algorithm import MegatronDion
    from megatron.core.optimizer.dion.types import DionDistMeta, DionParamConfig, DionStepParam
    from megatron.core.optimizer.distrib_dion.batches import build_dion_batches

    gen_g = torch.Generator().manual_seed(99 + rank)
    params, grads, cfgs, metas = [], {}, {}, {}
    for idx, (name, m, n) in enumerate(shapes):
        p = torch.nn.Parameter(torch.randn(m, n, generator=torch.Generator().manual_seed(idx)) * 0.02)
        grads[name] = (torch.randn(m, n, generator=gen_g) * 1e-3).to(torch.bfloat16).float()
        params.append((name, p))
    opt = MegatronDion([p for _, p in params], lr=0.01, mu=0.95, weight_decay=0.01, rank_fraction=rank_fraction)
    for name, p in params:
        m, n = p.shape
        r = max(1, int(rank_fraction * min(m, n) + 0.5))
        cfgs[name] = DionParamConfig(is_transposed=m < n, use_low_rank_sync=(m + n) * r < m * n)
        metas[name] = DionDistMeta(shape=(m, n), global_shape=(m, n), rank_fraction=rank_fraction,
                                   param_uid=(name,), is_dion_param=True, param_name=name,
                                   param_config=cfgs[name], is_transposed=m < n)
        q = torch.randn(min(m, n), r, generator=torch.Generator().manual_seed(2000 + len(opt.state)))
        opt.state[p] = dict(momentum=torch.zeros(m, n), Q=q, r=r, local_shape=(m, n), global_shape=(m, n))
    cache = {}
    world_group = dist.group.WORLD

    def route():
        steps = [DionStepParam(param=p, grad=grads[name], optimizer_state=opt.state[p],
                               optim_group=opt.param_groups[0], config=cfgs[name], dist_meta=metas[name])
                 for name, p in sorted(params)]
        return build_dion_batches(
            dion_params=steps, use_fs_collectives=True, state_replica_group=None,
            replica_validation_group=world_group, batch_key_cache=cache, global_rank=rank,
            group_size=dist.get_world_size, get_replicate_group=lambda: group,
            resolve_ortho_group=lambda c, m: None, resolve_tp_group=lambda m, expect_group: None,
            resolve_fs_group_from_meta=lambda m, expect_group: None), []

    opt.enable_distributed_mode(route_step_params=route)
    times = []
    for _ in range(WARMUP + STEPS):
        dist.barrier()
        t0 = time.perf_counter()
        opt.step()
        dist.barrier()
        times.append(time.perf_counter() - t0)
    return times[WARMUP:]


def _worker(rank, world, port, threads, which, out_path):
    os.environ["DION_DISABLE_TORCH_COMPILE"] = "1"
    sys.path.insert(0, ROOT)
    torch.set_num_threads(threads)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    if which == "gpt":
        shapes, rf = CB._shapes(CB.GPT125M_LAYER, 12), 1 / 48
    else:
        shapes, rf = CB._shapes(CB.LLAMA3_8B_LAYER, 1), 1 / 64
    times = _ref_times(shapes, rf, rank, dist.group.WORLD if world > 1 else None)
    t = torch.tensor(times, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(t.tolist(), f)
    dist.destroy_process_group()


def _ref(world, threads, which):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    with tempfile.TemporaryDirectory() as tmp:
        out = os.path.join(tmp, "t.json")
        mp.start_processes(_worker, args=(world, port, threads, which, out), nprocs=world, join=True,
                           start_method="spawn")
        with open(out) as f:
            return json.load(f)


def main():
    cores = CB.host_cores()
    res = {"host_cores": cores, "torch": torch.__version__, "steps": STEPS, "warmup": WARMUP}
    ref1 = _ref(2, cores // 2, "gpt")
    port1 = CB.gpt125m_gloo(world=2, steps=STEPS, warmup=WARMUP, threads=cores // 2)
    ref3 = _ref(1, cores, "llama")
    port3 = CB.llama_layer(steps=STEPS, warmup=WARMUP, threads=cores)
    for key, ref, port in (("config1_gpt125m_2rank_gloo_r16", ref1, port1), ("llama_layer_r64", ref3, port3)):
        r_med, p_med = statistics.median(ref), port["step_s_median"]
        res[key] = {"reference_step_s": [round(x, 4) for x in ref], "reference_median_s": round(r_med, 4),
                    "port_step_s": port["step_s"], "port_median_s": p_med,
                    "port_over_reference": round(p_med / r_med, 3), "within_20pct": abs(p_med / r_med - 1) <= 0.2}
    dest = os.path.join(ROOT, "profiles", "r02", "cpu_port_vs_reference.json")
    os.makedirs(os.path.dirname(dest), exist_ok=True)
    with open(dest, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
