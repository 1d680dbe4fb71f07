"""Time dion_grad_sum_sq over the Llama-3-8B bf16 gradient set (one layer's four shapes x 32)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import megatron_dion_amd as mda

dev = torch.device("cuda", 0)
shapes = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)] * 32
grads = [torch.empty(m, n, device=dev, dtype=torch.bfloat16).normal_(0, 1e-3) for m, n in shapes]
opt = mda.MegatronDion([torch.nn.Parameter(torch.zeros(2, 2, device=dev))])
for _ in range(2):
    mda.dion_grad_norm_sq(opt, grads)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(5):
    mda.dion_grad_norm_sq(opt, grads)
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / 5
nbytes = sum(m * n for m, n in shapes) * 2
print(f"dion_grad_sum_sq Llama set: {ms:.3f} ms, {nbytes / ms / 1e6:.1f} GB/s of bf16 gradient")
