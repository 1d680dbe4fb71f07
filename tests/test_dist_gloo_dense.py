"""World-size-2 gloo test of the replicate branch WITHOUT low-rank sync.

With `use_low_rank_sync=False` the reference all-reduces the dense gradients across the
replicas (runtime.py:439-491) and then runs the ddp schedule without averaging P or R
(runtime.py:1656-1728): every rank holds the same momentum, each orthonormalises the
entries it owns, the all-gather hands them round, and R is local.  The result must be
the world-size-1 step on the replica-averaged gradient, on every rank and bit-identical
across ranks.  The product's runtime runs unchanged with the test-only oracle codec.
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.slow

SHAPES = [("a0", 64, 48), ("a1", 64, 48), ("a2", 64, 48), ("t0", 40, 96), ("s0", 32, 32)]
STEPS = 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _sketch(P, step):
    mp_ = P.shape[-2]
    g = torch.Generator().manual_seed(1000 * step + mp_)
    return torch.randn(1, 128, mp_, generator=g) / 128 ** 0.5


def _grads(rank, step):
    g = torch.Generator().manual_seed(100 * step + 7 * rank)
    return {n: torch.randn(m, k, generator=g) * 1e-3 for n, m, k in SHAPES}


def _make(codec, group=None, low_rank=False):
    import megatron_dion_amd as mda
    from megatron_dion_amd.optimizer import attach_dp_routing

    params = {n: torch.nn.Parameter(torch.randn(m, k, generator=torch.Generator().manual_seed(i)) * 0.02)
              for i, (n, m, k) in enumerate(SHAPES)}
    opt = mda.MegatronDion(list(params.values()), lr=0.01, mu=0.95, weight_decay=0.01, rank_fraction=0.25,
                           codec=codec, use_low_rank_sync=low_rank, defer_error_feedback=False)
    attach_dp_routing(opt, list(params.items()), replicate_group=group)
    return opt, params


def _worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    from tests._cpu_codec import OracleCodec

    cur = {"s": 0}
    opt, params = _make(OracleCodec(sketch_lookup=lambda P: _sketch(P, cur["s"])), dist.group.WORLD)
    out = {}
    for s in range(STEPS):
        cur["s"] = s
        for n, g in _grads(rank, s).items():
            params[n].grad = g
        opt.step()
        for n, p in params.items():
            out[f"s{s}_{n}_W"] = p.detach().clone()
            out[f"s{s}_{n}_M"] = opt.state[p]["momentum"].clone()
            out[f"s{s}_{n}_Q"] = opt.state[p]["Q"].clone()
    torch.save(out, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_w2_dense_branch_equals_the_step_on_the_averaged_gradient():
    from tests._cpu_codec import OracleCodec

    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_worker, args=(2, _free_port(), tmp), nprocs=2, join=True, start_method="spawn")
        res = [torch.load(os.path.join(tmp, f"rank{r}.pt"), weights_only=True) for r in range(2)]
    cur = {"s": 0}
    ref_opt, ref_params = _make(OracleCodec(sketch_lookup=lambda P: _sketch(P, cur["s"])))
    for s in range(STEPS):
        cur["s"] = s
        g0, g1 = _grads(0, s), _grads(1, s)
        for n, p in ref_params.items():
            p.grad = (g0[n] + g1[n]) / 2
        ref_opt.step()
        for n, p in ref_params.items():
            for key, ref in (("W", p.detach()), ("M", ref_opt.state[p]["momentum"]), ("Q", ref_opt.state[p]["Q"])):
                got0, got1 = res[0][f"s{s}_{n}_{key}"], res[1][f"s{s}_{n}_{key}"]
                assert torch.equal(got0, got1), (s, n, key)  # identical across replicas
                err = (got0 - ref).abs().max().item() / max(ref.abs().max().item(), 1e-30)
                assert err <= 1e-6, (s, n, key, err)
