"""End-to-end rate with the host copies (DESIGN.md "End-to-end"): the Llama-3-8B set at r = 64.

The reference runs the path host-side and its factors leave for the wire, so besides the
device-resident rate (bench.py) this measures, on one GPU:
  h2d      : the bf16 gradients host (pinned) -> HBM, alone
  d2h      : the compressed factors P, R of every batch HBM -> host (pinned), alone
  serial   : h2d, then the Dion step, then d2h of the factors (nothing overlapped)
  overlap  : gradient H2D of the next coalesced batch group on a copy stream while the
             current one computes (bounded below by max(h2d, step))
Rates are grad GiB/s (2 B per gradient element), like the headline metric.
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import llama_shapes  # noqa: E402


def main():
    steps = int(os.environ.get("E2E_STEPS", "3"))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    import megatron_dion_amd as mda
    from megatron_dion_amd.optimizer import attach_dp_routing

    shapes = llama_shapes(32)
    torch.manual_seed(5)
    named, host_g = [], []
    for name, m, n in shapes:
        w = torch.nn.Parameter(torch.empty(m, n, device=dev).normal_(0.0, 0.02))
        w.main_grad = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
        hg = torch.empty(m, n, dtype=torch.bfloat16).normal_(0.0, 1e-3).pin_memory()
        named.append((name, w))
        host_g.append(hg)
    elems = sum(m * n for _, m, n in shapes)
    opt = mda.MegatronDion([p for _, p in named], lr=0.01, mu=0.95, weight_decay=0.01, rank_fraction=1 / 64)
    attach_dp_routing(opt, named)

    host_f = {}
    calls = [0]

    def sink(P, R, params=None):
        k = calls[0]
        calls[0] += 1
        if k not in host_f:
            host_f[k] = (torch.empty(P.shape, dtype=P.dtype).pin_memory(),
                         torch.empty(R.shape, dtype=R.dtype).pin_memory())
        hp, hr = host_f[k]
        hp.copy_(P, non_blocking=True)
        hr.copy_(R, non_blocking=True)

    def h2d():
        for (_, w), hg in zip(named, host_g):
            w.main_grad.copy_(hg, non_blocking=True)

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps

    def step_plain():
        opt._factor_sink = None
        opt.step()

    def step_with_d2h():
        calls[0] = 0
        opt._factor_sink = sink
        opt.step()

    h2d()
    step_plain()
    step_with_d2h()  # allocates the pinned factor buffers
    torch.cuda.synchronize()
    t_dev = timed(step_plain)
    t_h2d = timed(h2d)
    t_d2h_step = timed(step_with_d2h)
    t_serial = timed(lambda: (h2d(), step_with_d2h()))
    fbytes = sum(hp.numel() * 4 + hr.numel() * 4 for hp, hr in host_f.values())

    # overlap: copy stream brings the next step's gradients in while this step runs; the
    # step consumes the previous copy (double-buffered main_grad would be needed for a real
    # trainer; here the bound max(h2d, step) is what is measured)
    cs = torch.cuda.Stream(device=dev)

    def overlapped():
        ev = torch.cuda.Event()
        with torch.cuda.stream(cs):
            for (_, w), hg in zip(named, host_g):
                w.main_grad.copy_(hg, non_blocking=True)
            ev.record(cs)
        step_with_d2h()
        torch.cuda.current_stream().wait_event(ev)

    t_overlap = timed(overlapped)
    g = elems * 2 / 2 ** 30
    out = {"workload": "llama3-8b-2d-grad-set-r64", "grad_GiB": round(g, 3), "factor_MB": round(fbytes / 1e6, 1),
           "device_step_ms": round(t_dev * 1e3, 2), "device_GiB/s": round(g / t_dev, 1),
           "h2d_ms": round(t_h2d * 1e3, 2), "h2d_GB/s": round(elems * 2 / t_h2d / 1e9, 1),
           "step_plus_factor_d2h_ms": round(t_d2h_step * 1e3, 2),
           "serial_e2e_ms": round(t_serial * 1e3, 2), "serial_e2e_GiB/s": round(g / t_serial, 2),
           "overlap_e2e_ms": round(t_overlap * 1e3, 2), "overlap_e2e_GiB/s": round(g / t_overlap, 2),
           "steps": steps}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
