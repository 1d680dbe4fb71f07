"""Benchmark: device-resident Dion step over the Llama-3-8B 2D gradient set, rank 64.

Contract (see the task's bench section and BASELINE.json):
  python bench.py [--gpus N --steps K --warmup W]
  N > 1: one rank per GPU over RCCL.  The driver launches the N ranks with
  torch.distributed.run; run directly with --gpus N (WORLD_SIZE unset), bench.py starts
  that launcher itself as a child process (nothing GPU-side runs in the parent) and
  exits with its status.  Every rank compresses its own full gradient set (weak
  scaling) and exchanges P (reduce-scatter + all-gather) and R (all-reduce) over the
  replicate group, exactly the reference's RP = N low-rank path.  One JSON line on
  rank 0: `value` is the whole-job aggregate (all ranks' gradient bytes / the slowest
  rank's time); `value_per_gpu` is the metric's per-GPU figure (value / N).

A step = MegatronDion.step() over all matrices of the workload:
  llama3-8b (default, BASELINE config 3/4): 32 x {qkv 6144x4096, proj 4096x4096,
      fc1 28672x4096, fc2 4096x14336 (transposed)}, r = 64;
  mixtral-8x7b-experts (config 5): 8 layers x 8 experts x {fc1 28672x4096,
      fc2 4096x14336}, r = 128;
  single-4096 (config 2): one 4096x4096 matrix, r = 64.
M += G, P = M Q, RCQR, R = M^T P, fix-up, error feedback, column norm, weight update.
G is bf16 (synthetic N(0, 1e-3^2)), M / W / Q fp32, all resident in HBM.  The
optimizer is built with MegatronDion's defaults (deferred error feedback), i.e. exactly
what INTEGRATION.md's Megatron kwargs construct.
"""
import argparse
import json
import os
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "grad GiB/s/GPU (device-resident) Dion-compressed, Llama-3-8B 2D weights r=64"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)

LLAMA3_8B_LAYER = (("linear_qkv", 6144, 4096), ("linear_proj", 4096, 4096),
                   ("linear_fc1", 28672, 4096), ("linear_fc2", 4096, 14336))

# algorithmic HBM bytes per matrix element of each codec call (DESIGN.md "bytes per unit");
# "ef_apply_w" is the weight-only update of the deferred-EF schedule
BYTES_PER_ELEM = {"project_p": 10.0, "project_p_ef": 10.0, "project_r": 4.0, "ef_apply": 16.0, "ef_apply_w": 8.0}


def llama_shapes(layers):
    return [(f"layers.{i}.{n}.weight", m, k) for i in range(layers) for n, m, k in LLAMA3_8B_LAYER]


# Mixtral-8x7B experts (examples/mixtral/train_mixtral_8x7b_distributed.sh:32-55): hidden 4096,
# ffn 14336 (SwiGLU: fc1 fuses gate and up, 28672 rows), 8 experts; 8 of the 32 layers fit
# one GPU with W, M and G resident
MIXTRAL_EXPERT = (("linear_fc1", 28672, 4096), ("linear_fc2", 4096, 14336))


def mixtral_shapes(layers, experts=8):
    return [(f"layers.{i}.mlp.experts.local_experts.{e}.{n}.weight", m, k)
            for i in range(layers) for e in range(experts) for n, m, k in MIXTRAL_EXPERT]


WORKLOADS = {
    # name: (shapes(layers), rank, default layers, BASELINE config)
    "llama3-8b-2d-grad-set-r64": (llama_shapes, 64, 32, "Llama-3-8B full 2D-weight grad set, rank=64"),
    "mixtral-8x7b-experts-r128": (mixtral_shapes, 128, 8,
                                  "Mixtral-8x7B expert-weight grads batched (8 layers x 8 experts), rank=128"),
    "single-4096x4096-r64": (lambda layers: [("w", 4096, 4096)] * 1, 64, 1,
                             "single 4096x4096 bf16 grad matrix, rank=64"),
}


# kernel instance behind each (codec call, orientation) on the Llama set (r = 64 -> RB = RU = 4);
# ef_apply is two launches of the same instance (M, then W), each streaming 8 B per element
KERNEL_OF = {("project_p", False): ("rowproj_fast_kernel<4, 2>", 1),
             ("project_p", True): ("colproj_fast_kernel<4, 2>", 1),
             ("project_p_ef", False): ("rowproj_efh3_kernel<4, 2, 1, 2, 4>", 1),
             ("project_p_ef", True): ("colproj_efh3_kernel<4, 2>", 1),
             ("ef_apply_w", False): ("rank_stream_kernel<4, false, 8, 2, true>", 1),
             ("ef_apply_w", True): ("rank_stream_kernel<4, false, 8, 2, true>", 1),
             ("project_r", False): ("colproj_h3_kernel<4, 4, 4>", 1),
             ("project_r", True): ("rowproj_h3gl_kernel<4, 8, 3>", 1),
             ("ef_apply", False): ("rank_stream_kernel<4, false, 8, 2>", 2),
             ("ef_apply", True): ("rank_stream_kernel<4, false, 8, 2>", 2)}


# --state-dtype bf16 (the speedrun's bf16 momentum and Q, SURVEY 8c case viii), bytes per
# element: pass A G 2 + M 2 + M 2 (the deferred EF rides along), B: M 2, the weight update W 8
# (16 per step); eager EF: the update pass also moves M (EF + weight update: M 4 + W 8, 20 per step)
BYTES_PER_ELEM_BF16 = {"project_p": 6.0, "project_p_ef": 6.0, "project_r": 2.0, "ef_apply": 12.0,
                       "ef_apply_w": 8.0}
KERNEL_OF_BF16 = {("project_p", False): ("b16_row_kernel<4, 2>", 1),
                  ("project_p", True): ("b16_col_kernel<4, 2>", 1),
                  ("project_r", False): ("b16_col_kernel<4, 0>", 1),
                  ("project_r", True): ("b16_row_kernel<4, 0>", 1),
                  ("project_p_ef", False): ("b16_row_ef_kernel<4, 2>", 1),
                  ("project_p_ef", True): ("b16_col_ef_kernel<4, 2>", 1),
                  ("ef_apply", False): ("b16_stream_kernel<4, 8, false>", 1),
                  ("ef_apply", True): ("b16_stream_kernel<4, 8, true>", 1),
                  ("ef_apply_w", False): ("b16_stream_kernel<4, 8, false>", 1),
                  ("ef_apply_w", True): ("b16_stream_kernel<4, 8, true>", 1)}


class TimedCodec:
    """Wraps the HIP codec; records HIP events around each call on the stream it launches on."""

    def __init__(self, inner):
        self.inner = inner
        self.name = inner.name
        self.enabled = False
        self.events = {}

    def __getattr__(self, item):
        fn = getattr(self.inner, item)
        if item not in ("project_p", "project_p_ef", "orthonormalize", "project_r", "project_r_fixup", "fixup_colnorm",
                        "ef_apply"):
            return fn

        def wrapped(*args, **kwargs):
            if not self.enabled:
                return fn(*args, **kwargs)
            stream = torch.cuda.current_stream()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(stream)
            out = fn(*args, **kwargs)
            e.record(stream)
            elems = 0
            key = item
            if item == "ef_apply" and args[0] is None:
                key = "ef_apply_w"
            if item == "project_r_fixup":
                key = "project_r"  # pass B with the fix-up on its reduction (W = 1, fp32 state)
            transposed = None
            if key in BYTES_PER_ELEM:
                transposed = bool(args[5] if item == "project_p_ef" else args[-1])
                mats = args[1] if item in ("project_p", "project_p_ef") else (args[0] if args[0] is not None
                                                                              else args[1])
                elems = sum(int(t.numel()) for t in mats)
            self.events.setdefault((key, transposed), []).append((s, e, elems))
            return out

        return wrapped

    def summary(self):
        out = {}
        for k, lst in self.events.items():
            ms = [s.elapsed_time(e) for s, e, _ in lst]
            elems = sum(n for _, _, n in lst)
            out[k] = {"calls": len(lst), "total_ms": sum(ms), "elems": elems}
        return out


def load_pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed PMC pass (scripts/pmc_traffic.py), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            data = json.load(f)
        return data["kernels"][kernel]["hbm_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        return None


def cpu_baseline():
    """The CPU restatement (`port`) timed on this host's cores per BASELINE.md:49-63: config 1
    (GPT-125M 2D set, 2 gloo ranks, r = 16) and one Llama-3-8B layer (r = 64); 1 warm-up,
    median of 5 steps each (oracle/cpu_baseline.py).  `value` is the Llama layer's rate, the
    bench workload's unit; the full Llama set is 32 layers of the same work."""
    from oracle import cpu_baseline as CB

    c1 = CB.gpt125m_gloo(world=2, steps=5, warmup=1)
    c3 = CB.llama_layer(steps=5, warmup=1)
    return {"value": c3["GiB_s"], "unit": "GiB/s", "cores": c3["threads"], "kind": "port",
            "sample": f"one Llama-3-8B layer ({c3['grad_elements']} bf16 grad elements, 1/32 of the set), r=64, "
                      f"median of 5 steps after 1 warm-up = {c3['step_s_median']} s/step, torch CPU fp32, "
                      f"{c3['threads']} threads; product host runtime + oracle codec, eager error feedback",
            "config1_gpt125m_2rank_gloo": c1, "llama_layer": c3}


# MFMA work each kernel issues, in flops per gradient element per unit of rank r (2 r per
# real product, times the split products): fp16x3 (h3) = 3, bf16x6 = 6, fp32 MFMA = 1.
# Pass A carries two rank-r products (P = X Q, and the deferred EF P' R'^T); the
# rank_stream update one (W -= s P Q^T, or the eager EF).  (family, flops / (elem r), peak)
MFMA_BF16_PEAK_TFLOPS = 2500.0   # dense BF16/FP16, MI355X_MICROARCH.md
MFMA_F32_PEAK_TFLOPS = 157.3
MFMA_WORK = (("rowproj_efh3_kernel", 2 * 2 * 3, MFMA_BF16_PEAK_TFLOPS),
             ("colproj_efh3_kernel", 2 * 2 * 3, MFMA_BF16_PEAK_TFLOPS),
             ("rowproj_efgl_kernel", 2 * 2 * 3, MFMA_BF16_PEAK_TFLOPS),  # r = 128 LDS-DMA pass A (same products)
             ("colproj_efgl_kernel", 2 * 2 * 3, MFMA_BF16_PEAK_TFLOPS),
             ("b16_row_ef_kernel", 2 * 2, MFMA_BF16_PEAK_TFLOPS),        # bf16 state: EF + projection
             ("b16_col_ef_kernel", 2 * 2, MFMA_BF16_PEAK_TFLOPS),
             ("b16_row_kernel", 2, MFMA_BF16_PEAK_TFLOPS),
             ("b16_col_kernel", 2, MFMA_BF16_PEAK_TFLOPS),
             ("rowproj_h3_kernel", 2 * 3, MFMA_BF16_PEAK_TFLOPS),
             ("colproj_h3_kernel", 2 * 3, MFMA_BF16_PEAK_TFLOPS),
             ("rowproj_h3gl_kernel", 2 * 3, MFMA_BF16_PEAK_TFLOPS),  # the same products, LDS-DMA staging
             ("colproj_h3gl_kernel", 2 * 3, MFMA_BF16_PEAK_TFLOPS),
             ("colproj_x6_kernel", 2 * 6, MFMA_BF16_PEAK_TFLOPS),
             ("rank_stream_kernel@h3", 2 * 3, MFMA_BF16_PEAK_TFLOPS),  # <..., true>: the weight update
             ("rank_stream_kernel", 2 * 6, MFMA_BF16_PEAK_TFLOPS),
             ("rowproj_fast_kernel", 2, MFMA_F32_PEAK_TFLOPS),
             ("colproj_fast_kernel", 2, MFMA_F32_PEAK_TFLOPS))


def mfma_of(kernel, elems, r, ms):
    """Issued MFMA TFLOP/s of one kernel over its probe time and the fraction of the dtype's
    dense peak (the split products count as issued work: that is what the matrix cores do)."""
    for fam, per, peak in MFMA_WORK:
        base, _, tag = fam.partition("@")
        if kernel.startswith(base) and (not tag or kernel.endswith(", true>")):
            tf = per * elems * r / (ms * 1e-3) / 1e12
            return {"issued_TFLOPs": round(tf, 1), "peak_TFLOPs": peak, "util": round(tf / peak, 4)}
    return None


def kernel_roofline(per_kernel, elems, ms_per_step, probe_steps, deferred, step_bpe=None, r=64):
    """`roofline` of the dominant kernel (most probe time) + every kernel's rate + the step-level view."""
    dominant = max(per_kernel, key=lambda k: per_kernel[k]["ms"])
    d = per_kernel[dominant]
    avg_launch_ms = d["ms"] / d["launches"]
    bytes_per_launch = d["bytes"] / d["launches"]
    achieved = bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9
    traffic = load_pmc_traffic(dominant)
    # the schedule's own bytes: 30 B/elem eager, 22 B/elem with the deferred error feedback
    # (the EF's M read + write rides on pass A)
    step_bytes = (step_bpe if step_bpe is not None else (22.0 if deferred else 30.0)) * elems
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": None if traffic is None else round(traffic),
                "kernel": dominant, "bytes_per_launch": round(bytes_per_launch),
                "avg_launch_ms": round(avg_launch_ms, 4), "probe_steps": probe_steps,
                "mfma": mfma_of(dominant, d["elems"], r, d["ms"]),
                "kernels": {k: {"avg_launch_ms": round(v["ms"] / v["launches"], 4),
                                "GB/s": round(v["bytes"] / v["launches"] / (v["ms"] / v["launches"] * 1e-3) / 1e9, 1),
                                "mfma": mfma_of(k, v["elems"], r, v["ms"])}
                            for k, v in per_kernel.items()},
                "step": {"algorithmic_bytes": step_bytes,
                         "achieved": round(step_bytes / (ms_per_step * 1e-3) / 1e9, 1),
                         "frac": round(step_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "eager_equivalent_GBps": round(30.0 * elems / (ms_per_step * 1e-3) / 1e9, 1)}}
    return roofline


class LoopbackGroup:
    """--simulate-world W: a replicate group of W ranks whose collectives are local copies.

    Runs the W > 1 batch schedule (batches of W same-shape matrices, the owner rank's
    single-matrix orthonormalisation, the AsyncRuntime interleave) on one GPU with the
    exchange itself removed, to time the compute side of the N = W step."""

    def __init__(self, world):
        self.ranks = tuple(range(world))


class _DoneWork:
    def wait(self):
        return True


def install_loopback(world):
    group = LoopbackGroup(world)
    real = {k: getattr(dist, k) for k in ("get_world_size", "get_rank", "reduce_scatter_tensor",
                                          "all_gather_into_tensor", "all_reduce", "get_process_group_ranks",
                                          "all_gather_object")}

    def get_world_size(g=None):
        return world if isinstance(g, LoopbackGroup) else real["get_world_size"](g)

    def get_rank(g=None):
        return 0 if isinstance(g, LoopbackGroup) else real["get_rank"](g)

    def reduce_scatter_tensor(out, inp, op=None, group=None, async_op=False):
        if not isinstance(group, LoopbackGroup):
            return real["reduce_scatter_tensor"](out, inp, op=op, group=group, async_op=async_op)
        out.copy_(inp[: out.shape[0]])
        return _DoneWork() if async_op else None

    def all_gather_into_tensor(out, inp, group=None, async_op=False):
        if not isinstance(group, LoopbackGroup):
            return real["all_gather_into_tensor"](out, inp, group=group, async_op=async_op)
        out[: inp.shape[0]].copy_(inp)
        return _DoneWork() if async_op else None

    def all_reduce(t, op=None, group=None, async_op=False):
        if not isinstance(group, LoopbackGroup):
            return real["all_reduce"](t, op=op, group=group, async_op=async_op)
        return _DoneWork() if async_op else None

    def get_process_group_ranks(g):
        return list(g.ranks) if isinstance(g, LoopbackGroup) else real["get_process_group_ranks"](g)

    def all_gather_object(out, obj, group=None):
        # the batch-order check (batches.verify_sync_group_order): every simulated rank issues
        # rank 0's order
        if not isinstance(group, LoopbackGroup):
            return real["all_gather_object"](out, obj, group=group)
        for i in range(len(out)):
            out[i] = obj

    dist.get_world_size, dist.get_rank = get_world_size, get_rank
    dist.get_process_group_ranks, dist.all_gather_object = get_process_group_ranks, all_gather_object
    dist.reduce_scatter_tensor, dist.all_gather_into_tensor, dist.all_reduce = (
        reduce_scatter_tensor, all_gather_into_tensor, all_reduce)
    return group


def kernel_names(r):
    """KERNEL_OF / KERNEL_OF_BF16 with the rank-block template argument of rank r (dispatch_rb);
    the h3 pass-B column kernel keeps 2 columns per lane at r > 64 (colh3_ct)."""
    rb = {1: 1, 2: 2, 3: 4, 4: 4}.get((r + 15) // 16, 8)
    table = KERNEL_OF_BF16 if BYTES_PER_ELEM is BYTES_PER_ELEM_BF16 else KERNEL_OF
    out = {k: (name.replace("<4", f"<{rb}", 1), n) for k, (name, n) in table.items()}
    if r > 64 and ("project_r", False) in out and table is KERNEL_OF:
        # r = 128: pass B on LDS-DMA staging (colproj_h3gl_kernel, 8 waves, 2 columns per lane)
        out[("project_r", False)] = (f"colproj_h3gl_kernel<{rb}, 8, 2, 3>", 1)
    if r > 64 and ("project_p_ef", False) in out:
        # r = 128: the LDS-DMA row kernel (bf16 G, rows a multiple of 256: every bench set)
        out[("project_p_ef", False)] = ("rowproj_efgl_kernel<8, 2>", 1)
    if r > 64 and ("project_p_ef", True) in out:
        out[("project_p_ef", True)] = ("colproj_efgl_kernel<8, 2>", 1)
    if r > 64:
        # r = 128: the weight update keeps one X tile in flight (kRankD8)
        out = {k: (name.replace(f"rank_stream_kernel<{rb}, false, 8, 2", f"rank_stream_kernel<{rb}, false, 8, 1"), n)
               for k, (name, n) in out.items()}
    return out


def launch_ranks(args) -> int:
    """--gpus N without a launcher: start torch.distributed.run as a CHILD process (this
    process never touches the GPU) with the same arguments, and return its exit status."""
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="llama3-8b-2d-grad-set-r64", choices=sorted(WORKLOADS))
    ap.add_argument("--layers", type=int, default=0, help="layers of the workload (0 = its default); "
                                                          "fewer only for debugging")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--streams", type=int, default=3, help="HIP streams for independent batches (N=1 path)")
    ap.add_argument("--probe-steps", type=int, default=2, help="single-stream steps timed per kernel for `roofline`")
    ap.add_argument("--coalesce", type=int, default=16, help="matrices per launch group at N = 1")
    ap.add_argument("--lookahead", type=int, default=2,
                    help="N = 1 software pipeline depth (groups whose pass A runs before a pass B); 0 = two "
                         "alternating streams")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="collective backend for N > 1 (nccl = RCCL; gloo only to rehearse on one GPU)")
    ap.add_argument("--eager-ef", action="store_true",
                    help="apply each step's error feedback in its own pass (default: deferred into the next pass A)")
    ap.add_argument("--state-dtype", default="f32", choices=("f32", "bf16"),
                    help="momentum/Q dtype; bf16 = the speedrun's mixed precision (eager EF, not the bench line)")
    ap.add_argument("--simulate-world", type=int, default=0,
                    help="time the W-rank batch schedule on one GPU with loopback collectives (not a bench line)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.backend == "gloo":
        # rehearsal of the multi-rank path on fewer GPUs than ranks (gloo exchanges through the host)
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    group = None
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        group = dist.group.WORLD

    import megatron_dion_amd as mda
    from megatron_dion_amd.codec import HipDionCodec
    from megatron_dion_amd.optimizer import attach_dp_routing

    make_shapes, rank_r, default_layers, config_name = WORKLOADS[args.workload]
    shapes = make_shapes(args.layers or default_layers)
    torch.manual_seed(1234 + rank)
    named = []
    for name, m, n in shapes:
        w = torch.nn.Parameter(torch.empty(m, n, device=dev).normal_(0.0, 0.02))
        w.main_grad = torch.empty(m, n, device=dev).normal_(0.0, 1e-3).to(torch.bfloat16)
        named.append((name, w))
    codec = TimedCodec(HipDionCodec(dev))
    bf16_state = args.state_dtype == "bf16"
    if bf16_state:
        global BYTES_PER_ELEM
        BYTES_PER_ELEM = BYTES_PER_ELEM_BF16
    mpc = mda.DionMixedPrecisionConfig(momentum_dtype=torch.bfloat16, q_dtype=torch.bfloat16) if bf16_state else None
    kw = {} if not args.eager_ef else {"defer_error_feedback": False}
    min_side = min(min(m, n) for _, m, n in shapes)
    opt = mda.MegatronDion([p for _, p in named], lr=0.01, mu=0.95, weight_decay=0.01,
                           rank_fraction=rank_r / min_side, codec=codec, local_streams=args.streams,
                           coalesce_max_entries=args.coalesce, pipeline_lookahead=args.lookahead,
                           mixed_precision_config=mpc, **kw)
    if args.simulate_world > 1:
        group = install_loopback(args.simulate_world)
    attach_dp_routing(opt, named, replicate_group=group, q_stream="cpu")
    assert all(opt.state[p]["r"] == rank_r for _, p in named), "rank rule gave another r"
    sdt = torch.bfloat16 if bf16_state else torch.float32
    deferred = bool(opt._defer_ef) and all(
        codec.supports_deferred_ef(m, n, rank_r, m < n, state_dtype=sdt, grad_dtype=torch.bfloat16)
        for _, m, n in shapes)
    elems = sum(m * n for _, m, n in shapes)

    for _ in range(args.warmup):
        opt.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        opt.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    value = world * elems * 2 / (elapsed / args.steps) / 2 ** 30

    # Roofline probe: a few extra steps on ONE stream (not part of `value`), HIP events around
    # every codec call, so each kernel's duration is its own and not its share of a concurrent
    # pair; `scripts/gpu_prof.sh` profiles the same single-stream configuration with rocprofv3.
    opt._local_streams = 1
    # one unprobed single-stream step first: the caching allocator's blocks and the codec's
    # workspaces belong to the streams that allocated them, so the first step on this stream
    # allocates afresh, and a hipMalloc stall inside an event window is host time, not kernel
    # time (round 5's r = 128 pass-B probe read 3.82 ms against a 1.67 ms kernel)
    opt.step()
    torch.cuda.synchronize()
    codec.enabled = True
    for _ in range(args.probe_steps):
        opt.step()
    torch.cuda.synchronize()
    codec.enabled = False
    opt._local_streams = args.streams
    summ = codec.summary()
    per_kernel = {}
    knames = kernel_names(rank_r)
    for key, v in summ.items():
        if key not in knames:
            continue
        kname, launches_per_call = knames[key]
        agg = per_kernel.setdefault(kname, {"ms": 0.0, "bytes": 0.0, "launches": 0, "elems": 0.0})
        agg["ms"] += v["total_ms"]
        agg["bytes"] += BYTES_PER_ELEM[key[0]] * v["elems"]
        agg["elems"] += v["elems"] * launches_per_call
        agg["launches"] += v["calls"] * launches_per_call
    roofline = None
    if per_kernel:
        roofline = kernel_roofline(per_kernel, elems, ms_per_step, args.probe_steps, deferred,
                                   step_bpe=(16.0 if deferred else 20.0) if bf16_state else None, r=rank_r)

    wl = args.workload if (args.layers or default_layers) == default_layers else \
        f"{args.workload} ({args.layers} layers, debug)"
    # the BASELINE metric names the Llama set; other workloads say which set they measured
    metric = METRIC if args.workload == "llama3-8b-2d-grad-set-r64" else \
        f"grad GiB/s/GPU (device-resident) Dion-compressed, {config_name}"
    out = {"metric": metric, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None,
           "dtype": "f32 state, fp16x3-split MFMA, fp32 accumulate",
           "value_per_gpu": round(value / world, 2),
           "value_definition": "value = aggregate bf16-grad GiB/s of all ranks (bench contract); "
                               "value_per_gpu = value / n_gpus (the metric's per-GPU figure)",
           "data": "synthetic (random-init weights of the workload's 2D shapes, bf16 grads N(0,1e-3^2))",
           "config": {"workload": wl, "baseline_config": config_name, "matrices": len(shapes),
                      "grad_elements": elems, "rank": rank_r, "grad_dtype": "bf16", "state_dtype": args.state_dtype,
                      "error_feedback": "deferred (applied in the next step's pass A)" if deferred else "eager",
                      "parallelism": f"dp{world} (replicate, low-rank P/R exchange, {args.backend})" if world > 1
                      else "dp1"},
           "roofline": roofline}
    if bf16_state:
        out["dtype"] = "bf16 state, bf16 MFMA, fp32 accumulate"
    if args.simulate_world > 1:
        out["simulated_world"] = args.simulate_world
        out["metric"] = "SIMULATED (loopback collectives, not a bench line): " + metric
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
