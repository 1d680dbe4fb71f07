"""BASELINE configs that ran only as CPU baselines or only at world size 1, now through the
HIP path on one GPU (`pytest -m gpu`): two processes share cuda:0 and form a gloo replicate
group (RCCL needs one GPU per rank; the 8-GPU RCCL run is the driver's).  Each case runs the
product runtime twice per rank -- HIP codec on the GPU, test-only oracle codec on the CPU --
from the same W0, Q0 and gradients with one explicit sketch per (step, matrix), and compares:

  * config 1: the examples/dion GPT-125M 2D set (12 x {qkv 2304x768, proj 768x768, fc1
    3072x768, fc2 768x3072}), Dion rank 16, W = 2 (the reference's own 2-rank loopback
    config, BASELINE.json configs[0]);
  * the W > 1 branch without low-rank sync (dion/runtime.py:439-491, 1656-1728): dense
    gradient all-reduce, every rank orthonormalises its entries, R local;
  * Llama-3-8B fc1 (28672 x 4096) and fc2 (4096 x 14336, transposed) at W = 2, r = 64, four
    of each, so the replicated schedule runs rank-major groups of k = 2;
  * config 4's schedule at W = 4 and W = 8 (4 and 8 processes on cuda:0): the Llama shapes
    scaled down 16x (qkv 384x256, proj 256x256, fc1 896x256, fc2 256x448 transposed; r = 16)
    with 16 matrices per shape (>= 2 W) and the bench's coalesce_max_entries = 16, so every
    shape runs one rank-major group of k = 16 / W full batches (position r k + c holds entry
    c W + r), and fc1 carries 3 more matrices, a padded batch after its group; deferred EF and
    the 3 AsyncRuntime slot streams as in bench.py.

Tolerance: max |a - b| / max |b| <= 1e-5 for W, M, Q (Q up to column signs,
tests/_metrics.q_err: a near-zero Householder pivot of the sketch QR fixes a column's sign by
rounding); the weight step alone (tests/_metrics.dw_err) <= 5e-6 of its own scale.  W and Q must also be bit-identical across
the two ranks (replicas).
"""
import math
import os
import socket
import tempfile
import zlib

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests._metrics import dw_err, q_err

pytestmark = pytest.mark.gpu

TOL = 1e-5
TOL_DW = 5e-6
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

GPT125M = [(f"layers.{i}.{n}.weight", m, k) for i in range(12)
           for n, m, k in (("linear_qkv", 2304, 768), ("linear_proj", 768, 768), ("linear_fc1", 3072, 768),
                           ("linear_fc2", 768, 3072))]
DENSE = [(f"a{i}", 512, 384) for i in range(4)] + [(f"t{i}", 384, 1024) for i in range(2)] + [("odd", 256, 192)]
LLAMA_FC = [(f"layers.{i}.linear_fc1.weight", 28672, 4096) for i in range(4)] + \
           [(f"layers.{i}.linear_fc2.weight", 4096, 14336) for i in range(4)]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir, shapes, r, steps, low_rank, check, opt_kw=None):
    import sys
    sys.path.insert(0, ROOT)
    torch.set_num_threads(max(1, 8 // world))
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    import megatron_dion_amd as mda
    from megatron_dion_amd.optimizer import attach_dp_routing
    from oracle import dion_oracle as O
    from oracle.cpu_codec import OracleCodec

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    min_side = min(min(m, c) for _, m, c in shapes)
    res, q0 = {}, {}
    for backend in ("hip", "oracle"):
        on = dev if backend == "hip" else torch.device("cpu")
        named = [(n, torch.nn.Parameter((torch.randn(m, c, generator=torch.Generator().manual_seed(i)) * 0.02)
                                        .to(on))) for i, (n, m, c) in enumerate(shapes)]
        kw = dict(codec=OracleCodec(deferred=True)) if backend == "oracle" else {}
        opt = mda.MegatronDion([p for _, p in named], lr=0.01, mu=0.95, weight_decay=0.01,
                               rank_fraction=r / min_side, use_low_rank_sync=low_rank, **kw, **(opt_kw or {}))
        attach_dp_routing(opt, named, replicate_group=dist.group.WORLD)
        ks = {id(p): O.sketch_rows(int(opt.state[p]["r"])) for _, p in named}  # r = rank_fraction min(m, n)
        if backend == "hip":
            q0 = {n: opt.state[p]["Q"].detach().cpu().clone() for n, p in named}
        else:
            for n, p in named:
                opt.state[p]["Q"].copy_(q0[n])
        name_of = {id(p): n for n, p in named}
        cur = {"s": 0}

        def override(batch, _on=on, _name_of=name_of, _cur=cur, _ks=ks):
            out = {}
            for i, bp in enumerate(batch.params):
                m, c = bp.shape
                kk = _ks[id(bp)]
                g = torch.Generator().manual_seed(7919 * _cur["s"] + zlib.crc32(_name_of[id(bp)].encode()))
                out[i] = (torch.randn(kk, max(m, c), generator=g) * math.sqrt(1.0 / kk)).to(_on)
            return out

        opt._sketch_override = override
        for n, p in named:
            if n in check:
                res[f"{backend}_sinit_{n}_W"] = p.detach().cpu().clone()
        for s in range(steps):
            cur["s"] = s
            for i, (n, p) in enumerate(named):
                g = torch.Generator().manual_seed(1000 * s + 10 * rank + i)
                p.main_grad = (torch.randn(p.shape, generator=g) * 1e-3).to(torch.bfloat16).to(on)
            if s == 0:
                res[f"{backend}_chunks"] = torch.tensor([int(getattr(b, "_chunks", 0) or 0)
                                                         for b in opt._batches()[0]])
            opt.step()
            if s == steps - 1:
                opt.flush_error_feedback()
            if backend == "hip":
                torch.cuda.synchronize()
            for n, p in named:
                if n not in check:
                    continue
                res[f"{backend}_s{s}_{n}_W"] = p.detach().cpu().clone()
                res[f"{backend}_s{s}_{n}_Q"] = opt.state[p]["Q"].detach().cpu().clone()
                if s == steps - 1:
                    res[f"{backend}_s{s}_{n}_M"] = opt.state[p]["momentum"].detach().cpu().clone()
        del opt, named
        if backend == "hip":
            torch.cuda.empty_cache()
    torch.save(res, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _run_and_check(shapes, r, steps, low_rank, check=None, world=2, opt_kw=None):
    """`check`: the matrices whose W / M / Q are compared (default all)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    check = set(check) if check is not None else {n for n, _, _ in shapes}
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_worker, args=(world, _port(), tmp, shapes, r, steps, low_rank, check, opt_kw),
                           nprocs=world, join=True, start_method="spawn")
        res = [torch.load(os.path.join(tmp, f"rank{q}.pt"), weights_only=True) for q in range(world)]
    worst = {"W": 0.0, "dW": 0.0, "M": 0.0, "Q": 0.0}
    for rank in range(world):
        R = res[rank]
        assert torch.equal(R["hip_chunks"], R["oracle_chunks"]), (R["hip_chunks"], R["oracle_chunks"])
        for key, v in R.items():
            if not key.startswith("hip_s") or key.startswith("hip_sinit"):
                continue
            ref = R["oracle" + key[3:]]
            e = q_err(v, ref) if key.endswith("_Q") else \
                (v.double() - ref.double()).abs().max().item() / max(ref.double().abs().max().item(), 1e-30)
            worst[key[-1]] = max(worst[key[-1]], e)
            assert e <= TOL, (rank, key, e)
        for s in range(steps):
            for n in sorted(check):
                before = "sinit" if s == 0 else f"s{s - 1}"
                e = dw_err(R[f"hip_{before}_{n}_W"], R[f"hip_s{s}_{n}_W"], R[f"oracle_{before}_{n}_W"],
                           R[f"oracle_s{s}_{n}_W"], 1.0 - 0.01 * 0.01)
                worst["dW"] = max(worst["dW"], e)
                assert e <= TOL_DW, (rank, s, n, e)
    for key in res[0]:
        if key.startswith("hip_s") and not key.startswith("hip_sinit") and (key.endswith("_W") or key.endswith("_Q")):
            for q in range(1, world):
                assert torch.equal(res[0][key], res[q][key]), (q, key)
    return worst, res[0]["hip_chunks"].tolist()


def test_config1_gpt125m_w2_hip_matches_oracle():
    _run_and_check(GPT125M, 16, 2, low_rank=True)


def test_w2_dense_branch_hip_matches_oracle():
    _run_and_check(DENSE, 32, 3, low_rank=False)


def _llama_scaled(world):
    """The Llama-3-8B 2D shapes / 16, 16 matrices per shape (one rank-major group of 16 / W
    full batches), fc1 with 3 more (a padded batch after its group)."""
    out = []
    for name, m, n, extra in (("linear_qkv", 384, 256, 0), ("linear_proj", 256, 256, 0),
                              ("linear_fc1", 896, 256, 3), ("linear_fc2", 256, 448, 0)):
        out += [(f"layers.{i}.{name}.weight", m, n) for i in range(16 + extra)]
    return out


@pytest.mark.parametrize("world", [4, 8])
def test_config4_schedule_w4_w8_hip_matches_oracle(world):
    """Config 4's replicated schedule at W = 4 / 8 (what one GPU can run of it; RCCL needs a GPU
    per rank): gloo ranks sharing cuda:0, HIP codec against the CPU oracle codec under the same
    runtime, W / M / Q / dW <= the bars, W and Q bit-identical on all ranks."""
    shapes = _llama_scaled(world)
    worst, chunks = _run_and_check(shapes, 16, 2, low_rank=True, world=world,
                                   opt_kw=dict(coalesce_max_entries=16))
    k = 16 // world
    # 3 full-size groups of k batches (qkv, proj, fc2), fc1's group + its padded batch
    assert sorted(chunks) == sorted([k, k, k, k, 0]), chunks


def test_w2_llama_fc1_fc2_rank_major_hip_matches_oracle():
    # the first and the last matrix of each shape: the two ends of a rank-major group
    _run_and_check(LLAMA_FC, 64, 2, low_rank=True, check=[LLAMA_FC[0][0], LLAMA_FC[3][0], LLAMA_FC[4][0],
                                                          LLAMA_FC[7][0]])
