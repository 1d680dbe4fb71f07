"""FS ("fsdp") kernel kind on the GPU (`pytest -m gpu`): two processes share cuda:0 and form
a 2-rank FS group over gloo; everything else is the product path (HIP kernels through the
C ABI: pass A on the shard, RCQR of the owned entry, pass B, dion_fixup_colsum /
dion_colnorm_apply around the column-sum all-reduce, the update).

  * the reference's own FS=2 captures (tests/golden/make_golden_fs.py), replayed with the
    sketch the reference drew for each owned entry: W, Q every step, M after the flush;
  * a fast-path case (r = 64, both shard dims, padding, deferred error feedback, 3 steps)
    against the same runtime driven by the CPU oracle codec over gloo.
Tolerance: max |a - b| / max |b| <= 1e-5.
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.test_dist_gloo_fs import BF16_GPU_TOLS, check_fs_results, run_fs

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("name", ["f1_fs2_cols", "f2_fs2_rows_pad", "f3_fs2_uneven_mixed", "f4_fs2_bf16_cols",
                                  "f5_fs2_bf16_mixed"])
@pytest.mark.parametrize("deferred", [False, True], ids=["eager_ef", "deferred_ef"])
def test_hip_fs2_matches_reference(name, deferred):
    _need_gpu()
    res = run_fs(name, deferred=deferred, device="cuda:0")
    check_fs_results(res, name, deferred, TOL, bf16_tols=BF16_GPU_TOLS)


FAST = [("a", (1024, 768), 1), ("b", (1024, 768), 1), ("t", (768, 2048), 0), ("u", (768, 2048), 0),
        ("v", (768, 2048), 0)]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _fast_worker(rank, world, port, out_dir):
    import math
    import sys
    import zlib
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    import megatron_dion_amd as mda
    from megatron_dion_amd.optimizer import attach_dp_routing
    from oracle import dion_oracle as O
    from oracle.cpu_codec import OracleCodec

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    r = 64
    k = O.sketch_rows(r)
    res = {}
    q0 = {}
    for backend in ("hip", "oracle"):
        on = dev if backend == "hip" else torch.device("cpu")
        named, shards = [], {}
        for i, (n, (m, c), dim) in enumerate(FAST):
            full = torch.randn(m, c, generator=torch.Generator().manual_seed(i)) * 0.02
            split = m if dim == 0 else c
            per = math.ceil(split / world)
            s0, s1 = rank * per, min(split, rank * per + per)
            loc = full[s0:s1] if dim == 0 else full[:, s0:s1]
            named.append((n, torch.nn.Parameter(loc.contiguous().to(on))))
            shards[n] = ((m, c), dim, s0, s1)
        kw = dict(codec=OracleCodec(deferred=True)) if backend == "oracle" else {}
        opt = mda.MegatronDion([p for _, p in named], lr=0.01, mu=0.95, weight_decay=0.01, rank_fraction=r / 768,
                               **kw)
        attach_dp_routing(opt, named, fs_group=dist.group.WORLD, fs_shards=shards)
        # one Q0 for both backends: the device stream (HIP) and the CPU stream (oracle) of
        # the seeded Q init differ (state.py init_q), the runs must start from the same Q
        if backend == "hip":
            q0 = {n: opt.state[p]["Q"].detach().cpu().clone() for n, p in named}
        else:
            for n, p in named:
                opt.state[p]["Q"].copy_(q0[n])
        name_of = {id(p): n for n, p in named}
        cur = {"s": 0}

        def override(batch, _on=on, _name_of=name_of, _cur=cur):
            out = {}
            for i, bp in enumerate(batch.params[:batch.real_batch_size]):
                n = _name_of[id(bp)]
                m, c = next(g for nn, g, _ in FAST if nn == n)
                # P rows = the unsharded dim (dim 1 -> not transposed, P has m rows; dim 0 -> n rows)
                mp_ = m if next(d for nn, _, d in FAST if nn == n) == 1 else c
                g = torch.Generator().manual_seed(7919 * _cur["s"] + zlib.crc32(n.encode()))
                out[i] = (torch.randn(k, mp_, generator=g) * math.sqrt(1.0 / k)).to(_on)
            return out

        opt._sketch_override = override
        for s in range(3):
            cur["s"] = s
            for i, (n, p) in enumerate(named):
                g = torch.Generator().manual_seed(100 * s + 10 * rank + i)
                p.main_grad = (torch.randn(p.shape, generator=g) * 1e-3).to(torch.bfloat16).to(on)
            opt.step()
            if s == 2:
                opt.flush_error_feedback()
            if backend == "hip":
                torch.cuda.synchronize()
            for n, p in named:
                res[f"{backend}_s{s}_{n}_W"] = p.detach().cpu().clone()
                res[f"{backend}_s{s}_{n}_Q"] = opt.state[p]["Q"].detach().cpu().clone()
                if s == 2:
                    res[f"{backend}_s{s}_{n}_M"] = opt.state[p]["momentum"].detach().cpu().clone()
        res[f"{backend}_deferred"] = torch.tensor([int("_dion_pending_ef" in opt.state[named[0][1]])])
    torch.save(res, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_hip_fs2_fast_path_matches_oracle_runtime():
    _need_gpu()
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_fast_worker, args=(2, _port(), tmp), nprocs=2, join=True, start_method="spawn")
        res = [torch.load(os.path.join(tmp, f"rank{r}.pt"), weights_only=True) for r in range(2)]
    for rank in range(2):
        for key, v in res[rank].items():
            if not key.startswith("hip_s"):
                continue
            ref = res[rank]["oracle" + key[3:]]
            e = (v.double() - ref.double()).abs().max().item() / max(ref.double().abs().max().item(), 1e-30)
            assert e <= TOL, (rank, key, e)
