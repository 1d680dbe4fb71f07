"""Dev: do kernels on two torch streams run concurrently on this box?  Latency-bound spin
kernels (torch.cuda._sleep) on two streams: concurrent -> wall ~ one kernel, serialised -> the
sum.  Also a streaming kernel beside a spin kernel (the Dion overlap case)."""
import os
import time

import torch

print("GPU_MAX_HW_QUEUES", os.environ.get("GPU_MAX_HW_QUEUES"), "HIP_FORCE", os.environ.get("HIP_FORCE_QUEUE_PROFILING"),
      flush=True)
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
cycles = 20_000_000
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
print("streams", s1.cuda_stream, s2.cuda_stream, torch.cuda.current_stream().cuda_stream, flush=True)


def run(streams, reps=3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        for s in streams:
            with torch.cuda.stream(s):
                torch.cuda._sleep(cycles)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


run([s1])
one = run([s1])
two_same = run([s1, s1])
two = run([s1, s2])
print(f"sleep: one {one:.2f} ms, two on one stream {two_same:.2f} ms, two streams {two:.2f} ms "
      f"-> {'CONCURRENT' if two < 1.5 * one else 'SERIALISED'}", flush=True)

x = torch.empty(1 << 30, dtype=torch.float32, device=dev)
y = torch.empty_like(x)


def stream_and_sleep(reps=3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        with torch.cuda.stream(s1):
            for _ in range(4):
                y.copy_(x)
        with torch.cuda.stream(s2):
            torch.cuda._sleep(cycles)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def only_copy(reps=3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        with torch.cuda.stream(s1):
            for _ in range(4):
                y.copy_(x)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


stream_and_sleep()
c = only_copy()
cs = stream_and_sleep()
print(f"copy {c:.2f} ms, sleep {one:.2f} ms, copy beside sleep {cs:.2f} ms -> "
      f"{'CONCURRENT' if cs < 0.8 * (c + one) else 'SERIALISED'}", flush=True)
