"""Host logic of the Dion grad-norm term on CPU.

Known answers restated from the reference's own tests:
  tests/unit_tests/optimizer/test_dion_grad_norm_efficiency.py:7-27 (chunked fp64 sum)
  tests/unit_tests/optimizer/test_dion_optimizer_contracts.py:576-624 (replica SUM reduce,
  local grads untouched, count_dion_grad=False still reduces and returns None)
and a world-size-2 gloo run against the oracle.  The sum of squares itself runs in the
test-only oracle codec here; tests/test_gpu_grad_norm.py checks the HIP kernel.
"""
import os
import socket
import tempfile
from types import SimpleNamespace

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import dion_oracle as O
from tests._cpu_codec import OracleCodec


def test_oracle_grad_sum_sq_known_answer():
    # test_dion_grad_norm_efficiency.py:7-27: arange(1, 6) in 16-byte chunks -> 55
    t = torch.arange(1, 6, dtype=torch.float32)
    assert O.grad_sum_sq_fp64([t], chunk_bytes=16).item() == 55.0
    assert O.grad_sum_sq_fp64([t]).item() == 55.0


def test_as_matrices_fits_the_abi():
    from megatron_dion_amd.grad_norm import as_matrices
    assert as_matrices(torch.empty(0)) == []
    assert [tuple(m.shape) for m in as_matrices(torch.empty(7))] == [(1, 7)]
    n = 3 * (1 << 20) + 5
    mats = as_matrices(torch.arange(n, dtype=torch.float32))
    assert [tuple(m.shape) for m in mats] == [(3, 1 << 20), (1, 5)]
    assert mats[1][0, -1].item() == n - 1


def test_local_sum_without_a_replica_group():
    import megatron_dion_amd.grad_norm as gn

    opt = SimpleNamespace(defaults={"rp_average_in_collective": False}, codec=OracleCodec())
    ga, gb = torch.tensor([1.0, 2.0]), torch.tensor([3.0])
    assert gn.dion_grad_norm_sq(opt, [ga, gb]).item() == 14.0
    assert gn.dion_grad_norm_sq(opt, [ga, gb], count_dion_grad=False) is None
    with pytest.raises(RuntimeError, match="DION_INVALID_GRAD_NORM_MODE"):
        gn.dion_grad_norm_sq(opt, [ga], mode="bogus")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    import megatron_dion_amd.grad_norm as gn
    from tests._cpu_codec import OracleCodec as Codec

    out = {}
    # test_dion_optimizer_contracts.py:576-624's known answer, on two real ranks: the same
    # local grads, replicate op SUM -> the norm of 2 g; local grads untouched; with
    # count_dion_grad=False the collectives still run and None comes back
    opt_sum = SimpleNamespace(defaults={"rp_average_in_collective": False}, codec=Codec())
    ga, gb = torch.tensor([1.0, 2.0]), torch.tensor([3.0])
    out["kat"] = gn.dion_grad_norm_sq(opt_sum, [ga, gb], replica_group=dist.group.WORLD)
    out["kat_untouched"] = torch.tensor(ga.tolist() == [1.0, 2.0] and gb.tolist() == [3.0])
    out["kat_none"] = torch.tensor(gn.dion_grad_norm_sq(opt_sum, [ga, gb], replica_group=dist.group.WORLD,
                                                        count_dion_grad=False) is None)
    # local_bound under SUM: W sum_i ||G_i||^2 bounds ||sum_i G_i||^2 (here 2 * 28 = 56, exact 56)
    out["kat_bound_sum"] = gn.dion_grad_norm_sq(opt_sum, [ga, gb], replica_group=dist.group.WORLD,
                                                mode="local_bound")
    gen = torch.Generator().manual_seed(10 + rank)
    grads = [(torch.randn(48, 80, generator=gen) * 1e-3).to(torch.bfloat16),
             torch.randn(33, 17, generator=gen), (torch.randn(8, 8, generator=gen)).to(torch.bfloat16),
             torch.randn(3, 5, 7, generator=gen)]
    opt = SimpleNamespace(defaults={"rp_average_in_collective": True}, codec=Codec())
    out["total"] = gn.dion_grad_norm_sq(opt, grads, replica_group=dist.group.WORLD)
    # tiny staging chunks: many reduce-scatters, ragged tails, padding
    out["chunked"] = gn.dion_grad_norm_sq(opt, grads, replica_group=dist.group.WORLD, chunk_bytes=100)
    out["bound"] = gn.dion_grad_norm_sq(opt, grads, replica_group=dist.group.WORLD, mode="local_bound")
    out["grads"] = grads
    torch.save(out, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_w2_grad_norm_of_the_averaged_gradient():
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_worker, args=(2, _free_port(), tmp), nprocs=2, join=True, start_method="spawn")
        res = [torch.load(os.path.join(tmp, f"rank{r}.pt"), weights_only=True) for r in range(2)]
    for r in range(2):
        assert res[r]["kat"].item() == 2.0 ** 2 + 4.0 ** 2 + 6.0 ** 2
        assert bool(res[r]["kat_untouched"]) and bool(res[r]["kat_none"])
        assert res[r]["kat_bound_sum"].item() == 56.0 >= res[r]["kat"].item()
    # the reference's semantics: all-reduce(AVG) in the gradient dtype, then the fp64 sum of squares
    avg = [((a.float() + b.float()) / 2).to(a.dtype) if a.dtype == torch.bfloat16 else (a + b) / 2
           for a, b in zip(res[0]["grads"], res[1]["grads"])]
    ref = O.grad_sum_sq_fp64(avg).item()
    for r in range(2):
        assert res[r]["total"].item() == pytest.approx(ref, rel=1e-6)
        assert res[r]["chunked"].item() == pytest.approx(ref, rel=1e-6)
    assert res[0]["total"].item() == res[1]["total"].item()
    # local_bound: the mean of the local squares, an upper bound of the exact value
    bound = sum(O.grad_sum_sq_fp64(res[r]["grads"]).item() for r in range(2)) / 2
    for r in range(2):
        assert res[r]["bound"].item() == pytest.approx(bound, rel=1e-12)
        assert res[r]["bound"].item() >= ref
