"""The elementwise branch of MegatronDion.step (AdamW / Lion, algorithm.py:247-429).

1. The oracle (oracle/dion_oracle.py elementwise_adamw / elementwise_lion, the
   reference's foreach chain restated) against the golden vectors captured from the
   reference itself (tests/golden/make_golden_elementwise.py): exact.
2. The product's routing, grouping and state handling (MegatronDion with the
   test-only oracle codec) against the same vectors: exact.
3. `-m gpu`: the HIP multi-tensor kernel through the same optimizer, against the
   same vectors (fp32 elementwise arithmetic in the reference's order; bar 1e-6
   max-relative, see the test).
"""
import json
import os

import numpy as np
import pytest
import torch

import megatron_dion_amd as mda
from megatron_dion_amd.types import ElementwiseStepParam
from oracle import dion_oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _manifest():
    with open(os.path.join(GOLD, "manifest_elementwise.json")) as fh:
        return json.load(fh)


def _cases():
    return [c["name"] for c in _manifest()["cases"]]


def _load(name):
    man = _manifest()
    case = next(c for c in man["cases"] if c["name"] == name)
    with np.load(os.path.join(GOLD, name + ".npz")) as z:
        arr = {k: torch.from_numpy(z[k].copy()) for k in z.files}
    return man, case, arr


def _maxrel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


@pytest.mark.parametrize("name", _cases())
def test_oracle_matches_reference_elementwise(name):
    man, case, arr = _load(name)
    names = [n for n, _ in man["tensors"]]
    W = [arr[f"s0_{n}_W0"].clone() for n in names]
    sdt = getattr(torch, case.get("state_dtype", "float32"))
    vdt = getattr(torch, case.get("variance_dtype", case.get("state_dtype", "float32")))
    m1 = [torch.zeros_like(w, dtype=sdt) for w in W]
    m2 = [torch.zeros_like(w, dtype=vdt) for w in W]
    b1, b2 = case["betas"]
    for step in range(man["steps"]):
        G = [arr[f"s{step}_{n}_G"].to(getattr(torch, case["gdtype"])) for n in names]
        if case["opt"] == "lion":
            O.elementwise_lion(W, G, m1, lr=case["lr"], beta1=b1, beta2=b2, weight_decay=case["wd"])
        else:
            O.elementwise_adamw(W, G, m1, m2, lr=case["lr"], beta1=b1, beta2=b2, weight_decay=case["wd"],
                                step=step + 1, epsilon=case["eps"])
        for i, n in enumerate(names):
            assert torch.equal(W[i], arr[f"s{step}_{n}_W1"])
            assert torch.equal(m1[i].float(), arr[f"s{step}_{n}_m1"])
            if case["opt"] != "lion":
                assert torch.equal(m2[i].float(), arr[f"s{step}_{n}_m2"])


def run_through_optimizer(name, dev, codec=None):
    """Replay a golden case through MegatronDion.step; yield per step and tensor (ours, reference)."""
    man, case, arr = _load(name)
    names = [n for n, _ in man["tensors"]]
    params = {n: torch.nn.Parameter(arr[f"s0_{n}_W0"].clone().to(dev)) for n in names}
    sdt = getattr(torch, case.get("state_dtype", "float32"))
    vdt = getattr(torch, case.get("variance_dtype", case.get("state_dtype", "float32")))
    mpc = mda.DionMixedPrecisionConfig(momentum_dtype=sdt, q_dtype=sdt, variance_dtype=vdt) \
        if case.get("state_dtype") else None
    opt = mda.MegatronDion(list(params.values()), lr=case["lr"], weight_decay=case["wd"], betas=tuple(case["betas"]),
                           elementwise_eps=case["eps"], elementwise_optimizer=case["opt"], codec=codec,
                           mixed_precision_config=mpc)
    grads = {}
    opt.enable_distributed_mode(route_step_params=lambda: ([], [
        ElementwiseStepParam(param=params[n], grad=grads[n], optimizer_state=opt.state[params[n]],
                             optim_group=opt.param_groups[0]) for n in names]))
    for step in range(man["steps"]):
        for n in names:
            grads[n] = arr[f"s{step}_{n}_G"].to(getattr(torch, case["gdtype"])).to(dev)
        opt.step()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        assert opt._elementwise_update_count == len(names)
        for n in names:
            st = opt.state[params[n]]
            assert st["step"] == step + 1
            assert st["first_moment"].dtype == sdt
            yield step, n, "W", params[n], arr[f"s{step}_{n}_W1"]
            yield step, n, "m1", st["first_moment"].float(), arr[f"s{step}_{n}_m1"]
            if case["opt"] != "lion":
                yield step, n, "m2", st["second_moment"].float(), arr[f"s{step}_{n}_m2"]


@pytest.mark.parametrize("name", _cases())
def test_optimizer_elementwise_branch_matches_reference(name):
    from tests._cpu_codec import OracleCodec
    for step, n, k, ours, ref in run_through_optimizer(name, torch.device("cpu"), codec=OracleCodec()):
        assert torch.equal(ours.detach(), ref), (name, step, n, k)
