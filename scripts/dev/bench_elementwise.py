"""Time dion_elementwise_adamw on the Llama-3-8B elementwise set (embedding + output 128256x4096, 65 norms)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import megatron_dion_amd as mda

dev = torch.device("cuda", 0)
shapes = [(128256, 4096), (128256, 4096)] + [(4096,)] * 65
P = [torch.randn(s, device=dev) * 0.02 for s in shapes]
G = [(torch.randn(s, device=dev) * 1e-2).to(torch.bfloat16) for s in shapes]
M1 = [torch.zeros(s, device=dev) for s in shapes]
M2 = [torch.zeros(s, device=dev) for s in shapes]
codec = mda.MegatronDion([torch.nn.Parameter(torch.zeros(2, 2, device=dev))]).codec
kw = dict(lr=3e-4, beta1=0.9, beta2=0.95, weight_decay=0.1, epsilon=1e-8)
for i in range(2):
    codec.elementwise_adamw(P, G, M1, M2, step=i + 1, **kw)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for i in range(5):
    codec.elementwise_adamw(P, G, M1, M2, step=i + 3, **kw)
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / 5
n = sum(p.numel() for p in P)
print(f"dion_elementwise_adamw Llama elementwise set: {n} elements, {ms:.3f} ms, "
      f"{n * 26 / ms / 1e6:.1f} GB/s (26 B/elem: W, m, v read+write, bf16 G read)")
