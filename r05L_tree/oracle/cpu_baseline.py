"""CPU baseline of the Dion step, timed on the host cores.  TEST INFRASTRUCTURE ONLY.

bench.py's `cpu_baseline` leg calls this module (rank 0, N = 1) to time the
reference's algorithm on the CPU next to the GPU number, as BASELINE.md:49-63 and
SURVEY.md 8(d) plan it:

  config 1  GPT-125M 2D set (12 x {qkv 2304x768, proj 768x768, fc1 3072x768,
            fc2 768x3072} = 48 matrices, 84,934,656 elements), Dion rank 16,
            2 gloo ranks over loopback (RP = 2), cores / 2 threads per rank;
  config 3  one Llama-3-8B layer (qkv, proj, fc1, fc2; 218,103,808 elements), r = 64,
            one process, all cores (the full 32-layer set is 32 x this work).

Each config runs 1 warm-up step and reports the median of >= 5 timed steps.  The
step is the product's host runtime (megatron_dion_amd: batching, padding, the
reduce-scatter / all-gather / all-reduce schedule over gloo) with the oracle codec
(oracle/cpu_codec.py: the reference's torch-CPU fp32 arithmetic, oracle/dion_oracle.py),
the eager error-feedback schedule of the reference.  Its speed against the reference's
own step is checked in the container by scripts/ref/cpu_speed_check.py
(profiles/r02/cpu_port_vs_reference.json).

Synthetic inputs follow SURVEY.md 8(d): W0 ~ N(0, 0.02^2), G ~ N(0, 1e-3^2) rounded to
bf16 (seed 99 + rank), M0 = 0, Q0 from the reference's seeded init (identical on ranks).
"""
from __future__ import annotations

import json
import os
import socket
import statistics
import tempfile
import time

import torch

GPT125M_LAYER = (("linear_qkv", 2304, 768), ("linear_proj", 768, 768), ("linear_fc1", 3072, 768),
                 ("linear_fc2", 768, 3072))
LLAMA3_8B_LAYER = (("linear_qkv", 6144, 4096), ("linear_proj", 4096, 4096), ("linear_fc1", 28672, 4096),
                   ("linear_fc2", 4096, 14336))


def _shapes(layer, count):
    return [(f"layers.{i}.{n}.weight", m, k) for i in range(count) for n, m, k in layer]


def host_cores() -> int:
    """The cores this process may use: its affinity set, capped by OMP_NUM_THREADS when set
    (the GPU box exposes the whole machine's CPUs; this job's share is OMP_NUM_THREADS)."""
    cores = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        cores = min(cores, int(omp))
    return max(1, cores)


def _time_steps(shapes, rank_fraction, steps, warmup, rank=0, group=None):
    import megatron_dion_amd as mda
    from megatron_dion_amd.optimizer import attach_dp_routing

    from .cpu_codec import OracleCodec

    named = []
    gen_g = torch.Generator().manual_seed(99 + rank)
    for idx, (name, m, n) in enumerate(shapes):
        w = torch.nn.Parameter(torch.randn(m, n, generator=torch.Generator().manual_seed(idx)) * 0.02)
        w.grad = (torch.randn(m, n, generator=gen_g) * 1e-3).to(torch.bfloat16).float()
        named.append((name, w))
    opt = mda.MegatronDion([p for _, p in named], lr=0.01, mu=0.95, weight_decay=0.01, rank_fraction=rank_fraction,
                           codec=OracleCodec(), defer_error_feedback=False)
    attach_dp_routing(opt, named, replicate_group=group)
    times = []
    for _ in range(warmup + steps):
        if group is not None:
            torch.distributed.barrier(group)
        t0 = time.perf_counter()
        opt.step()
        if group is not None:
            torch.distributed.barrier(group)
        times.append(time.perf_counter() - t0)
    return times[warmup:]


def _gloo_worker(rank, world, port, threads, steps, warmup, out_path):
    import torch.distributed as dist

    torch.set_num_threads(threads)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        times = _time_steps(_shapes(GPT125M_LAYER, 12), 1 / 48, steps, warmup, rank=rank, group=dist.group.WORLD)
        t = torch.tensor(times, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)  # a step ends when the slowest rank ends
        if rank == 0:
            with open(out_path, "w") as f:
                json.dump(t.tolist(), f)
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def gpt125m_gloo(world: int = 2, steps: int = 5, warmup: int = 1, threads: int = 0) -> dict:
    """Config 1: GPT-125M 2D set, r = 16, `world` gloo ranks on loopback."""
    import torch.multiprocessing as mp

    threads = threads or max(1, host_cores() // world)
    saved = {k: os.environ.get(k) for k in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")}
    with tempfile.TemporaryDirectory() as tmp:
        out = os.path.join(tmp, "times.json")
        try:  # the CPU ranks never touch the GPU
            os.environ["HIP_VISIBLE_DEVICES"] = os.environ["CUDA_VISIBLE_DEVICES"] = ""
            mp.start_processes(_gloo_worker, args=(world, _free_port(), threads, steps, warmup, out), nprocs=world,
                               join=True, start_method="spawn")
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        with open(out) as f:
            times = json.load(f)
    elems = sum(m * n for _, m, n in _shapes(GPT125M_LAYER, 12))
    med = statistics.median(times)
    return {"config": "examples/dion 2-rank CPU/gloo loopback, GPT-125M 2D grads, Dion rank=16",
            "ranks": world, "threads_per_rank": threads, "grad_elements_per_rank": elems,
            "step_s_median": round(med, 4), "step_s": [round(x, 4) for x in times],
            "GiB_s_per_rank": round(elems * 2 / med / 2 ** 30, 4)}


def llama_layer(steps: int = 5, warmup: int = 1, threads: int = 0) -> dict:
    """Config 3 sample: one Llama-3-8B layer at r = 64, one process."""
    threads = threads or host_cores()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        times = _time_steps(_shapes(LLAMA3_8B_LAYER, 1), 1 / 64, steps, warmup)
    finally:
        torch.set_num_threads(prev)
    elems = sum(m * n for _, m, n in LLAMA3_8B_LAYER)
    med = statistics.median(times)
    return {"config": "1 of 32 Llama-3-8B layers (qkv, proj, fc1, fc2), r=64, one process", "threads": threads,
            "grad_elements": elems, "step_s_median": round(med, 4), "step_s": [round(x, 4) for x in times],
            "GiB_s": round(elems * 2 / med / 2 ** 30, 4)}
