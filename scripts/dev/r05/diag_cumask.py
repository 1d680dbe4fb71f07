"""Dev diagnostic (not a bench line): the Llama step with the latency-bound orthonormalisation on a
HIP stream restricted to a few CUs (hipExtStreamCreateWithCUMask) and the streaming passes on
streams restricted to the rest, so the small kernels never wait for CU slots that the streaming
kernels' resident blocks hold.  Uses the existing pipelined schedule (MegatronDion._run_local_pipelined:
streaming streams + one latency stream).

    python scripts/dev/r05/diag_cumask.py [--steps 10]
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


def hip_lib():
    torch.cuda.init()
    with open("/proc/self/maps") as fh:
        for line in fh:
            if "libamdhip64" in line:
                return ctypes.CDLL(line.split()[-1])
    raise RuntimeError("libamdhip64 not mapped")


def masked_stream(hip, dev, cus, ncu):
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
    ap.add_argument("--workload", default="llama3-8b-2d-grad-set-r64")
    args = ap.parse_args()
    import bench
    import megatron_dion_amd as mda
    from megatron_dion_amd.codec import HipDionCodec
    from megatron_dion_amd.optimizer import attach_dp_routing

    dev = torch.device("cuda", 0)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    hip = hip_lib()
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

    def timed(label):
        for _ in range(2):
            opt.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            opt.step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / args.steps * 1e3
        print(json.dumps({"mode": label, "ms_per_step": round(ms, 3),
                          "GiB/s": round(elems * 2 / (ms * 1e-3) / 2 ** 30, 1)}), flush=True)
        return ms

    allc = list(range(ncu))
    out = {"ncu": ncu}
    out["base_2streams"] = timed("base_2streams")
    for look in (1, 2):
        opt._local_streams, opt._pipeline_lookahead, opt._pstreams = 3, look, None
        out[f"pipe{look}_unmasked"] = timed(f"pipe{look}_unmasked")
        for nl, spread in ((16, True), (16, False), (8, True), (32, True)):
            lat = [c for c in allc if c % (ncu // nl) == ncu // nl - 1] if spread else allc[ncu - nl:]
            big = [c for c in allc if c not in lat]
            opt._pstreams = [masked_stream(hip, dev, big, ncu), masked_stream(hip, dev, big, ncu),
                             masked_stream(hip, dev, lat, ncu)]
            key = f"pipe{look}_L{nl}_{'spread' if spread else 'tail'}"
            out[key] = timed(key)
        # latency stream masked, streaming streams on every CU
        lat = [c for c in allc if c % 16 == 15]
        opt._pstreams = [masked_stream(hip, dev, allc, ncu), masked_stream(hip, dev, allc, ncu),
                         masked_stream(hip, dev, lat, ncu)]
        out[f"pipe{look}_Lonly16"] = timed(f"pipe{look}_Lonly16")
    opt._local_streams, opt._pipeline_lookahead, opt._pstreams = 2, 0, None
    out["base_again"] = timed("base_again")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
