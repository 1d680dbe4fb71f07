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


def _clip_worker(rank, world, port, out_dir):
    """Grad norm (clipping) then step, both without low-rank sync: count the dense exchanges."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    import megatron_dion_amd.grad_norm as gn
    from tests._cpu_codec import OracleCodec

    calls = []
    real_all_reduce = dist.all_reduce

    def counting_all_reduce(tensor, *args, **kwargs):
        calls.append(int(tensor.numel()))
        return real_all_reduce(tensor, *args, **kwargs)

    dist.all_reduce = counting_all_reduce
    out = {}
    try:
        for clip in (False, True):
            cur = {"s": 0}
            opt, params = _make(OracleCodec(sketch_lookup=lambda P: _sketch(P, cur["s"])), dist.group.WORLD)
            grad_sizes = sorted(int(p.numel()) for p in params.values())
            for s in range(STEPS):
                cur["s"] = s
                for n, g in _grads(rank, s).items():
                    params[n].grad = g
                calls.clear()
                if clip:
                    plist = list(params.values())
                    grads = [p.grad for p in plist]
                    flags = gn.dense_reuse_flags(opt, plist)
                    assert all(flags), flags
                    out[f"clip_s{s}_norm"] = gn.dion_grad_norm_sq(opt, grads, replica_group=dist.group.WORLD,
                                                                  dense_reuse=flags)
                opt.step()
                dense = sorted(c for c in calls if c > 1)
                out[f"{int(clip)}_s{s}_exchanges"] = torch.tensor([int(dense == grad_sizes)])
                for n, p in params.items():
                    out[f"{int(clip)}_s{s}_{n}_W"] = p.detach().clone()
                    out[f"{int(clip)}_s{s}_{n}_M"] = opt.state[p]["momentum"].clone()
                if clip:
                    out[f"clip_s{s}_cache_left"] = torch.tensor([int(hasattr(opt, "_dion_dense_grad_reduction_cache"))])
    finally:
        dist.all_reduce = real_all_reduce
    torch.save(out, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_w2_clip_then_step_exchanges_each_dense_gradient_once():
    """distrib_dion/grad_norm.py:161-258 + dion/dense_grad_cache.py: with clipping, the norm
    all-reduces the dense (no low-rank sync) gradients in place and the step reuses them --
    one exchange per gradient per step, and the same W, M as without clipping."""
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_clip_worker, args=(2, _free_port(), tmp), nprocs=2, join=True, start_method="spawn")
        res = [torch.load(os.path.join(tmp, f"rank{r}.pt"), weights_only=True) for r in range(2)]
    for r in range(2):
        for s in range(STEPS):
            # one all-reduce per gradient: in the step without clipping, in the norm with it
            assert int(res[r][f"0_s{s}_exchanges"]) == 1 and int(res[r][f"1_s{s}_exchanges"]) == 1, (r, s)
            assert int(res[r][f"clip_s{s}_cache_left"]) == 0  # the step consumed every mark
            g0, g1 = _grads(0, s), _grads(1, s)
            ref = sum(((g0[n].double() + g1[n].double()) / 2).square().sum().item() for n in g0)
            assert res[r][f"clip_s{s}_norm"].item() == pytest.approx(ref, rel=1e-6)
            for n, _, _ in SHAPES:
                for key in ("W", "M"):
                    assert torch.equal(res[r][f"1_s{s}_{n}_{key}"], res[r][f"0_s{s}_{n}_{key}"]), (r, s, n, key)


def _skip_worker(rank, world, port, out_dir):
    """norm on persistent gradient buffers, the step skipped (an AMP-style inf), the
    next iteration's gradients written into the SAME buffers after zero_grad(), then norm + step.
    The second norm must exchange the new gradients (not trust the first norm's marks)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    import megatron_dion_amd.grad_norm as gn
    from tests._cpu_codec import OracleCodec

    opt, params = _make(OracleCodec(sketch_lookup=lambda P: _sketch(P, 0)), dist.group.WORLD)
    plist = list(params.values())
    for n, g in _grads(rank, 0).items():
        params[n].grad = g.clone()  # persistent buffers from here on
    flags = gn.dense_reuse_flags(opt, plist)
    out = {"norm0": gn.dion_grad_norm_sq(opt, [p.grad for p in plist], replica_group=dist.group.WORLD,
                                         dense_reuse=flags)}
    # the step is skipped; the next iteration zeroes and refills the same storage
    opt.zero_grad(set_to_none=False)
    for n, g in _grads(rank, 1).items():
        params[n].grad.add_(g)
    out["norm1"] = gn.dion_grad_norm_sq(opt, [p.grad for p in plist], replica_group=dist.group.WORLD,
                                        dense_reuse=flags)
    opt.step()
    for n, p in params.items():
        out[f"{n}_W"] = p.detach().clone()
        out[f"{n}_G"] = p.grad.detach().clone()
    torch.save(out, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_w2_skipped_step_then_refilled_buffers_are_exchanged_again():
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_skip_worker, args=(2, _free_port(), tmp), nprocs=2, join=True, start_method="spawn")
        res = [torch.load(os.path.join(tmp, f"rank{r}.pt"), weights_only=True) for r in range(2)]
    g0, g1 = _grads(0, 1), _grads(1, 1)
    ref = sum(((g0[n].double() + g1[n].double()) / 2).square().sum().item() for n in g0)
    for r in range(2):
        assert res[r]["norm1"].item() == pytest.approx(ref, rel=1e-6), r
        for n, _, _ in SHAPES:
            # the gradients the step consumed are the replica average, identical on both ranks
            avg = (g0[n] + g1[n]) / 2
            assert torch.allclose(res[r][f"{n}_G"], avg, rtol=0, atol=1e-9), (r, n)
            assert torch.equal(res[0][f"{n}_W"], res[1][f"{n}_W"]), n
