"""GPU parity of dion_grad_sum_sq, the Dion grad-norm term (`pytest -m gpu`).

Checked against the oracle's restatement of distrib_dion/grad_norm.py:54-68 (fp64):
only the fp64 summation order differs, so the bar is 1e-12 relative; repeated calls
are bitwise identical (fixed-order reduction).
"""
import pytest
import torch

import megatron_dion_amd as mda
from oracle import dion_oracle as O

pytestmark = pytest.mark.gpu

TOL = 1e-12


def _opt(dev):
    return mda.MegatronDion([torch.nn.Parameter(torch.zeros(2, 2, device=dev))])


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_grad_sum_sq_matches_oracle(dtype):
    dev = _dev()
    gen = torch.Generator().manual_seed(3)
    grads = [(torch.randn(m, n, generator=gen) * 1e-3).to(dtype) for m, n in
             [(330, 203), (64, 48), (48, 96), (1, 7)]]
    grads += [(torch.randn(40, 24, generator=gen) * 1e-3).to(dtype) for _ in range(70)]  # > 64 per launch
    base = (torch.randn(96, 200, generator=gen) * 1e-3).to(dtype)
    grads.append(base[:, 8:168])                                                          # row stride > n
    ref = O.grad_sum_sq_fp64(grads).item()
    opt = _opt(dev)
    gd = [g.to(dev) if g.is_contiguous() else base.to(dev)[:, 8:168] for g in grads]
    got = mda.dion_grad_norm_sq(opt, gd).item()
    assert abs(got - ref) <= TOL * ref, (got, ref)
    again = mda.dion_grad_norm_sq(opt, gd).item()
    assert again == got


def test_grad_sum_sq_llama_fc1_bf16():
    dev = _dev()
    g = (torch.randn(28672, 4096, device=dev) * 1e-3).to(torch.bfloat16)
    got = mda.dion_grad_norm_sq(_opt(dev), [g]).item()
    ref = O.grad_sum_sq_fp64([g.cpu()]).item()
    assert abs(got - ref) <= TOL * ref, (got, ref)
    assert mda.dion_grad_norm(_opt(dev), [g]) == pytest.approx(ref ** 0.5, rel=1e-12)
