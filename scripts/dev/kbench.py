"""Dev micro-driver: one codec op on a Llama-size batch, repeated (for rocprofv3 --pmc / --stats)."""
import os, sys, time, torch
sys.path.insert(0, os.getcwd())
from megatron_dion_amd.codec import HipDionCodec

op = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
m, n = (4096, 14336) if op.endswith("_T") else (28672, 4096)
T = m < n
B, r = 16 if not T else 16, int(os.environ.get("KB_R", "64"))  # KB_R=128: Mixtral's rank
mp, nq = (n, m) if T else (m, n)
dev = torch.device("cuda", 0)
codec = HipDionCodec(dev)
torch.manual_seed(0)
Ms = [torch.randn(m, n, device=dev) * 1e-3 for _ in range(B)]
Gs = [(torch.randn(m, n, device=dev) * 1e-3).to(torch.bfloat16) for _ in range(B)]
Ws = [torch.randn(m, n, device=dev) * 0.02 for _ in range(B)]
Qs = [torch.randn(nq, r, device=dev) for _ in range(B)]
P = torch.randn(B, mp, r, device=dev) * 0.01
R = torch.randn(B, nq, r, device=dev) * 0.01
nz = torch.ones(B, dtype=torch.int32, device=dev)
# pass A's flags for these M (max |M| bits): the fixed-scale pass B ("pbf")
nzf = torch.stack([M.abs().max() for M in Ms]).view(torch.int32).contiguous()
def run():
    if op.startswith("pa_ef0"):
        codec.project_p_ef(Gs, Ms, Qs, P, nz, T, [None] * B, [None] * B, -0.05)
    elif op.startswith("pa_ef"):
        codec.project_p_ef(Gs, Ms, Qs, P, nz, T, [P[i] for i in range(B)], [R[i] for i in range(B)], -0.05)
    elif op.startswith("pa"):
        codec.project_p(Gs, Ms, Qs, P, nz, T)
    elif op.startswith("pbf"):
        codec.project_r(Ms, P, R, T, nonzero=nzf)
    elif op.startswith("pb"):
        codec.project_r(Ms, P, R, T)
    elif op.startswith("w"):
        codec.ef_apply(None, Ws, P, R, Qs, nz, 0.95, 0.01, 0.01, 0.5, T)
    elif op.startswith("efm"):
        codec.ef_apply(Ms, None, P, R, Qs, nz, 0.95, 0.01, 0.01, 0.5, T)
run(); torch.cuda.synchronize()
variants = [op] if len(sys.argv) <= 3 else sys.argv[3].split(",")
for rnd in range(3):
    for v in variants:
        op = v
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            run()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        print(f"round {rnd} {op}: {dt*1e3:.3f} ms per call, {B*m*n/dt/1e9:.1f} Gelem/s")
