"""Dev diagnostic (not a bench line): what each phase of the Llama step costs in the two-stream
schedule.  Runs the bench's Llama-3-8B set and optimizer, then times the step with one codec
entry point replaced by a no-op at a time (the numbers of such a step are garbage; only its time
is read): the difference to the full step is the phase's marginal cost on the critical path.

    python scripts/dev/r05/diag_phases.py [--modes base,no_ortho,...] [--steps 10]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)

MODES = {
    "base": (),
    "no_ortho": ("orthonormalize",),
    "no_passb": ("project_r", "project_r_fixup"),
    "no_update": ("ef_apply",),
    "no_fixup": ("fixup_colnorm",),  # the W = 1 fp32 path fixes inside project_r_fixup
    "no_passa": ("project_p_ef", "project_p"),
    "only_streaming": ("orthonormalize", "fixup_colnorm"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default=",".join(MODES))
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--workload", default="llama3-8b-2d-grad-set-r64")
    ap.add_argument("--streams", default="2,1")
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
    orig = {k: getattr(codec, k) for ks in MODES.values() for k in ks}
    out = {}
    for streams in (int(s) for s in args.streams.split(",")):
        opt._local_streams = streams
        for mode in args.modes.split(","):
            for k, f in orig.items():
                setattr(codec, k, f)
            for k in MODES[mode]:
                setattr(codec, k, lambda *a, **kw: None)
            for _ in range(2):
                opt.step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                opt.step()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / args.steps * 1e3
            out[f"s{streams}_{mode}"] = round(ms, 3)
            print(json.dumps({"streams": streams, "mode": mode, "ms_per_step": round(ms, 3),
                              "GiB/s": round(elems * 2 / (ms * 1e-3) / 2 ** 30, 1)}), flush=True)
    for k, f in orig.items():
        setattr(codec, k, f)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
