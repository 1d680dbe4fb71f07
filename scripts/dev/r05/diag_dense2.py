"""Dev: the W = 2 dense-branch case, recording every orthonormalize call (input P, sketch, output
P) of rank 0 on both backends; prints per call the input and output differences and flipped
columns."""
import math
import os
import sys
import tempfile
import zlib

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)


def worker(rank, world, port, out_dir):
    sys.path.insert(0, ROOT)
    torch.set_num_threads(4)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    import megatron_dion_amd as mda
    from megatron_dion_amd.codec import HipDionCodec
    from megatron_dion_amd.optimizer import attach_dp_routing
    from oracle import dion_oracle as O
    from oracle.cpu_codec import OracleCodec
    from tests.test_gpu_configs import DENSE
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    shapes, r, steps = DENSE, 32, 3
    min_side = min(min(m, c) for _, m, c in shapes)
    rec, q0 = {}, {}
    for backend in ("hip", "oracle"):
        on = dev if backend == "hip" else torch.device("cpu")
        named = [(n, torch.nn.Parameter((torch.randn(m, c, generator=torch.Generator().manual_seed(i)) * 0.02).to(on)))
                 for i, (n, m, c) in enumerate(shapes)]
        codec = OracleCodec(deferred=True) if backend == "oracle" else HipDionCodec(dev)
        calls = []
        orig = codec.orthonormalize

        def hooked(P, m, n, transposed, seed, oversample=1.25, sketch=None, _orig=orig, _calls=calls, **kw):
            pin = P.detach().cpu().clone()
            _orig(P, m, n, transposed, seed, oversample, sketch=sketch, **kw)
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            _calls.append((cur["s"], pin, None if sketch is None else sketch.detach().cpu().clone(),
                           P.detach().cpu().clone()))
        codec.orthonormalize = hooked
        opt = mda.MegatronDion([p for _, p in named], lr=0.01, mu=0.95, weight_decay=0.01,
                               rank_fraction=r / min_side, use_low_rank_sync=False, codec=codec)
        attach_dp_routing(opt, named, replicate_group=dist.group.WORLD)
        ks = {id(p): O.sketch_rows(int(opt.state[p]["r"])) for _, p in named}
        if backend == "hip":
            q0 = {n: opt.state[p]["Q"].detach().cpu().clone() for n, p in named}
        else:
            for n, p in named:
                opt.state[p]["Q"].copy_(q0[n])
        name_of = {id(p): n for n, p in named}
        cur = {"s": 0}

        def override(batch, _on=on):
            out = {}
            for i, bp in enumerate(batch.params):
                m, c = bp.shape
                kk = ks[id(bp)]
                g = torch.Generator().manual_seed(7919 * cur["s"] + zlib.crc32(name_of[id(bp)].encode()))
                out[i] = (torch.randn(kk, max(m, c), generator=g) * math.sqrt(1.0 / kk)).to(_on)
            return out
        opt._sketch_override = override
        for s in range(steps):
            cur["s"] = s
            for i, (n, p) in enumerate(named):
                g = torch.Generator().manual_seed(1000 * s + 10 * rank + i)
                p.main_grad = (torch.randn(p.shape, generator=g) * 1e-3).to(torch.bfloat16).to(on)
            opt.step()
        rec[backend] = calls
    if rank == 0:
        for k, (hc, oc) in enumerate(zip(rec["hip"], rec["oracle"])):
            s, hin, hsk, hout = hc
            _, oin, osk, oout = oc
            ein = ((hin - oin).abs().max() / oin.abs().max()).item()
            sgn = torch.where((hout.double() * oout.double()).sum(-2) < 0, -1.0, 1.0)
            flips = [int(i) for i in torch.nonzero(sgn.flatten() < 0).flatten()]
            eout = ((hout.double() * sgn - oout.double()).abs().max() / oout.abs().max()).item()
            skd = None if hsk is None else (hsk - osk).abs().max().item()
            print(f"call {k} step {s} shape {tuple(hin.shape)} in {ein:.2e} sketch {skd} flips {flips} "
                  f"out-aligned {eout:.2e}", flush=True)
            if flips:
                SP = (osk.double().reshape(-1, osk.shape[-1]) @ oin.double()[0])
                A = SP.clone()
                for j in range(A.shape[1]):
                    x = A[j:, j].clone()
                    if j in flips:
                        print(f"   col {j}: alpha/norm {abs(x[0].item()) / x.norm().item():.3e}", flush=True)
                    v = x.clone()
                    sv = -math.copysign(x.norm().item(), x[0].item())
                    v[0] -= sv
                    v = v / v.norm()
                    A[j:, :] -= 2 * torch.outer(v, v @ A[j:, :])
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    mp.start_processes(worker, args=(2, port, None), nprocs=2, join=True, start_method="spawn")
