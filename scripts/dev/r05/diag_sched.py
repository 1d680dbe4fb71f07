"""Dev diagnostic (not a bench line): stream schedules of the Llama step, one configuration per
process (--config):

  base            the product schedule (two streams, stagger plan)
  base_hi         the same with both streams high priority
  pipeN           pipelined (N groups of pass A ahead), streaming streams + latency stream
  pipeN_hi        the same, latency stream high priority (orthonormalisation first at every free slot)
  pipeN_mask      the same, latency stream on 16 CUs and streaming streams on the other 240
                  (hipExtStreamCreateWithCUMask; run with GPU_MAX_HW_QUEUES >= 4 free queues)

    python scripts/dev/r05/diag_sched.py --config pipe2_hi [--steps 10]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)


def masked_stream(dev, cus, ncu):
    torch.cuda.init()
    path = next(line.split()[-1] for line in open("/proc/self/maps") if "libamdhip64" in line)
    hip = ctypes.CDLL(path)
    words = (ncu + 31) // 32
    arr = (ctypes.c_uint32 * words)()
    for c in cus:
        arr[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), arr)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask rc={rc}")
    return torch.cuda.ExternalStream(s.value, device=dev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--config", default="base")
    ap.add_argument("--workload", default="llama3-8b-2d-grad-set-r64")
    args = ap.parse_args()
    import bench
    import megatron_dion_amd as mda
    from megatron_dion_amd.codec import HipDionCodec
    from megatron_dion_amd.optimizer import attach_dp_routing

    dev = torch.device("cuda", 0)
    make_shapes, rank_r, layers, _ = bench.WORKLOADS[args.workload]
    shapes = make_shapes(layers)
    torch.manual_seed(1234)
    named = []
    for name, m, n in shapes:
        w = torch.nn.Parameter(torch.empty(m, n, device=dev).normal_(0.0, 0.02))
        w.main_grad = torch.empty(m, n, device=dev).normal_(0.0, 1e-3).to(torch.bfloat16)
        named.append((name, w))
    codec = HipDionCodec(dev)
    min_side = min(min(m, n) for _, m, n in shapes)
    opt = mda.MegatronDion([p for _, p in named], lr=0.01, mu=0.95, weight_decay=0.01,
                           rank_fraction=rank_r / min_side, codec=codec, local_streams=2, coalesce_max_entries=16)
    attach_dp_routing(opt, named, q_stream="cpu")
    elems = sum(m * n for _, m, n in shapes)
    cfg = args.config
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
    if cfg == "base_hi":
        opt._streams = [torch.cuda.Stream(device=dev, priority=-1) for _ in range(2)]
    elif cfg.startswith("pipe"):
        look = int(cfg[4])
        opt._local_streams, opt._pipeline_lookahead = 3, look
        if cfg.endswith("_hi"):
            opt._pstreams = [torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev),
                             torch.cuda.Stream(device=dev, priority=-1)]
        elif cfg.endswith("_mask"):
            ncu = torch.cuda.get_device_properties(dev).multi_processor_count
            lat = [c for c in range(ncu) if c % 16 == 15]
            big = [c for c in range(ncu) if c % 16 != 15]
            opt._pstreams = [masked_stream(dev, big, ncu), masked_stream(dev, big, ncu), masked_stream(dev, lat, ncu)]
    for _ in range(2):
        opt.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        opt.step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / args.steps * 1e3
    print(json.dumps({"config": cfg, "ms_per_step": round(ms, 3), "GiB/s": round(elems * 2 / (ms * 1e-3) / 2 ** 30, 1),
                      "priority_range": [lo, hi]}), flush=True)


if __name__ == "__main__":
    main()
