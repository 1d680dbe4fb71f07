"""TP ("fsdp_tp") kernel kind on the GPU (`pytest -m gpu`): two processes share cuda:0 and form a
2-rank TP group over gloo; everything else is the product path (HIP kernels through the C ABI:
pass A on the shard with the all-gathered Q, the row-sharded RCQR pieces dion_dortho_sketch /
_qr_inv / _apply / _gram / _chol_inv between the collectives, pass B, the fix-up / column norm,
the update, the Q re-shard).

  * the reference's own TP=2 captures (tests/golden/make_golden_tp.py), replayed with the
    reference's seeded sketch slices: W, Q every step, M after the flush (eager and deferred EF);
  * a fast-path case (r = 64, both shard dims, a padded batch, deferred EF, 3 steps) with the
    in-kernel sketch generator against the same runtime driven by the CPU oracle codec with the
    reference's sketch: W and M are sketch-invariant (P Q^T and P R^T do not see column signs),
    Q is compared sign-aligned, and the gathered P of the last step is orthonormal.
Tolerance: max |a - b| / max |b| <= 1e-5.
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.test_dist_gloo_fs import BF16_GPU_TOLS
from tests.test_dist_gloo_tp import check_tp_results, run_tp

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("name", ["t1_tp2_rows", "t2_tp2_cols_T", "t3_tp2_odd_r_mixed", "t4_tp2_plain_qr",
                                  "t5_tp2_bf16_rows", "t6_tp2_bf16_odd_mixed"])
@pytest.mark.parametrize("deferred", [False, True], ids=["eager_ef", "deferred_ef"])
def test_hip_tp2_matches_reference(name, deferred):
    _need_gpu()
    res = run_tp(name, deferred=deferred, device="cuda:0")
    check_tp_results(res, name, deferred, TOL, bf16_tols=BF16_GPU_TOLS)


FAST = [("a", (2048, 1024), 0), ("b", (2048, 1024), 0), ("t", (1024, 3072), 1), ("u", (1024, 3072), 1),
        ("v", (1024, 3072), 1)]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _fast_worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    import megatron_dion_amd as mda
    from megatron_dion_amd.optimizer import attach_dp_routing
    from oracle import dion_oracle as O
    from oracle.cpu_codec import OracleCodec

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    r = 64
    res = {}
    q0 = {}
    for backend in ("hip", "oracle"):
        on = dev if backend == "hip" else torch.device("cpu")
        named, shards, rng = [], {}, {}
        for i, (n, (m, c), dim) in enumerate(FAST):
            full = torch.randn(m, c, generator=torch.Generator().manual_seed(i)) * 0.02
            split = m if dim == 0 else c
            s0, s1 = O.split_range(split, world, rank)
            loc = full[s0:s1] if dim == 0 else full[:, s0:s1]
            named.append((n, torch.nn.Parameter(loc.contiguous().to(on))))
            shards[n] = ((m, c), dim, s0, s1)
            rng[n] = (split, s0, s1)
        kw = dict(codec=OracleCodec(deferred=True)) if backend == "oracle" else {}
        opt = mda.MegatronDion([p for _, p in named], lr=0.01, mu=0.95, weight_decay=0.01, rank_fraction=r / 1024,
                               **kw)
        opt._keep_factors = True
        attach_dp_routing(opt, named, tp_group=dist.group.WORLD, tp_shards=shards)
        if backend == "hip":
            q0 = {n: opt.state[p]["Q"].detach().cpu().clone() for n, p in named}
        else:
            for n, p in named:
                opt.state[p]["Q"].copy_(q0[n])
            cur = {"s": 0}

            def override(batch, _cur=cur):
                out = {}
                for i, meta in enumerate(list(batch.dist_metas)[:int(batch.real_batch_size)]):
                    split, s0, s1 = rng[meta.param_name]
                    seed = O.distributed_sketch_seed(_cur["s"] + 1, (meta.param_name,), meta.param_name)
                    out[i] = O.reference_sharded_sketch(seed, O.sketch_rows(r), split, s0, s1 - s0)
                return out

            opt._sketch_override = override
        for s in range(3):
            if backend == "oracle":
                cur["s"] = s
            for i, (n, p) in enumerate(named):
                g = torch.Generator().manual_seed(100 * s + i)   # TP shards of one full gradient
                m, c = FAST[i][1]
                gfull = (torch.randn(m, c, generator=g) * 1e-3).to(torch.bfloat16)
                split, s0, s1 = rng[n]
                gl = gfull[s0:s1] if FAST[i][2] == 0 else gfull[:, s0:s1]
                p.main_grad = gl.contiguous().to(on)
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
        P_last = opt._last_batch_factors[0]
        res[f"{backend}_P_last"] = P_last.detach().cpu().clone()
    torch.save(res, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_hip_tp2_generated_sketch_matches_oracle_runtime():
    _need_gpu()
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_fast_worker, args=(2, _port(), tmp), nprocs=2, join=True, start_method="spawn")
        res = [torch.load(os.path.join(tmp, f"rank{r}.pt"), weights_only=True) for r in range(2)]
    for rank in range(2):
        for key, v in res[rank].items():
            if not key.startswith("hip_s"):
                continue
            ref = res[rank]["oracle" + key[3:]].double()
            got = v.double()
            if key.endswith("_Q"):  # sketch-dependent column signs
                sign = torch.sign((got * ref).sum(dim=0))
                sign[sign == 0] = 1
                got = got * sign
            e = (got - ref).abs().max().item() / max(ref.abs().max().item(), 1e-30)
            assert e <= TOL, (rank, key, e)
    # the last batch's P, rows of both ranks: orthonormal columns
    P = torch.cat([res[0]["hip_P_last"], res[1]["hip_P_last"]], dim=1).double()
    real = P.shape[0] if P.abs().sum() > 0 else 0
    for b in range(real):
        if P[b].abs().sum() == 0:
            continue
        G = P[b].t() @ P[b]
        assert (G - torch.eye(G.shape[0], dtype=G.dtype)).abs().max().item() <= 1e-5
