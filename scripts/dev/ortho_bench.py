"""Dev: time dion_orthonormalize on a Llama fc1 launch group (16 x 28672 x 64), for rocprofv3 --stats."""
import os, sys, time, torch
sys.path.insert(0, os.getcwd())
from megatron_dion_amd.codec import HipDionCodec
dev = torch.device("cuda", 0)
codec = HipDionCodec(dev)
B, mp, r = 16, int(os.environ.get("OB_MP", "28672")), int(os.environ.get("OB_R", "64"))
torch.manual_seed(0)
P0 = torch.randn(B, mp, r, device=dev)
P = P0.clone()
for _ in range(3):
    P.copy_(P0); codec.orthonormalize(P, mp, 4096, False, seed=1)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    P.copy_(P0); codec.orthonormalize(P, mp, 4096, False, seed=1)
torch.cuda.synchronize()
print(f"{os.environ.get('DION_LIB_PATH', 'default')}: {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms per orthonormalize (incl. copy)")
