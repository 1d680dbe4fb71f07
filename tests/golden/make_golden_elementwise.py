"""Golden vectors for the elementwise branch of MegatronDion.step, from the REFERENCE.

Run ONLY in the build container (the reference tree does not exist on the GPU box):

    PYTHONPATH=/root/reference DION_DISABLE_TORCH_COMPILE=1 \\
        python tests/golden/make_golden_elementwise.py

Drives the reference's own `MegatronDion.step` (dion/algorithm.py:149-221) with a
routing callback that hands it only ElementwiseStepParam items, so the step runs
`_apply_elementwise_batches` (:247-429 -> elementwise_opts.py AdamW / Lion), and
records W, first_moment and second_moment after every step.  Data only is committed.
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))

CASES = [
    dict(name="e1_adamw", opt="adam", betas=(0.9, 0.95), wd=0.01, lr=0.01, eps=1e-8, gdtype="float32"),
    dict(name="e2_lion", opt="lion", betas=(0.9, 0.99), wd=0.1, lr=0.003, eps=1e-8, gdtype="float32"),
    dict(name="e3_adamw_bf16grad_nowd", opt="adamw", betas=(0.8, 0.999), wd=0.0, lr=0.02, eps=1e-6,
         gdtype="bfloat16"),
    # the speedrun's mixed precision (speedrun_nanogpt_mcore.py:422-431): bf16 moments
    dict(name="e4_adamw_bf16_moments", opt="adam", betas=(0.9, 0.95), wd=0.01, lr=0.01, eps=1e-8,
         gdtype="float32", state_dtype="bfloat16"),
    dict(name="e5_lion_bf16_moments", opt="lion", betas=(0.9, 0.99), wd=0.1, lr=0.003, eps=1e-8,
         gdtype="bfloat16", state_dtype="bfloat16"),
    # independent momentum_dtype / variance_dtype (algorithm.py:308-332)
    dict(name="e6_adamw_bf16m_f32v", opt="adam", betas=(0.9, 0.95), wd=0.01, lr=0.01, eps=1e-8,
         gdtype="bfloat16", state_dtype="bfloat16", variance_dtype="float32"),
    dict(name="e7_adamw_f32m_bf16v", opt="adam", betas=(0.8, 0.99), wd=0.05, lr=0.01, eps=1e-6,
         gdtype="float32", state_dtype="float32", variance_dtype="bfloat16"),
]
TENSORS = [("ln", (64,)), ("emb", (40, 24)), ("bias", (33,)), ("head", (17, 96))]
STEPS = 3


def run_case(case):
    from megatron.core.optimizer.dion.algorithm import MegatronDion
    from megatron.core.optimizer.dion.types import DionMixedPrecisionConfig, ElementwiseStepParam

    gen = torch.Generator().manual_seed(7)
    params = {n: torch.nn.Parameter(torch.randn(*s, generator=gen) * 0.02) for n, s in TENSORS}
    sdt = getattr(torch, case.get("state_dtype", "float32"))
    vdt = getattr(torch, case.get("variance_dtype", case.get("state_dtype", "float32")))
    mpc = DionMixedPrecisionConfig(momentum_dtype=sdt, q_dtype=sdt, variance_dtype=vdt) \
        if case.get("state_dtype") else None
    opt = MegatronDion(list(params.values()), lr=case["lr"], weight_decay=case["wd"], betas=case["betas"],
                       elementwise_eps=case["eps"], elementwise_optimizer=case["opt"], mixed_precision_config=mpc)
    grads = {}

    def route():
        items = [ElementwiseStepParam(param=params[n], grad=grads[n], optimizer_state=opt.state[params[n]],
                                      optim_group=opt.param_groups[0]) for n, _ in TENSORS]
        return [], items

    opt.enable_distributed_mode(route_step_params=route)
    arrays = {}
    gdt = getattr(torch, case["gdtype"])
    for step in range(STEPS):
        for n, s in TENSORS:
            arrays[f"s{step}_{n}_W0"] = params[n].detach().clone()
            g = (torch.randn(*s, generator=gen) * 1e-2).to(gdt)
            grads[n] = g
            arrays[f"s{step}_{n}_G"] = g.float()
        opt.step()
        for n, _ in TENSORS:
            st = opt.state[params[n]]
            arrays[f"s{step}_{n}_W1"] = params[n].detach().clone()
            arrays[f"s{step}_{n}_m1"] = st["first_moment"].clone()
            if "second_moment" in st:
                arrays[f"s{step}_{n}_m2"] = st["second_moment"].clone()
    out = os.path.join(HERE, case["name"] + ".npz")
    np.savez_compressed(out, **{k: v.detach().float().numpy() for k, v in arrays.items()})
    print("wrote", out, os.path.getsize(out), "bytes", flush=True)


def main():
    os.environ["DION_DISABLE_TORCH_COMPILE"] = "1"
    only = set(sys.argv[1:])
    for case in CASES:
        if not only or case["name"] in only:
            run_case(case)
    man = {"tensors": [[n, list(s)] for n, s in TENSORS], "steps": STEPS,
           "cases": [dict(c, betas=list(c["betas"])) for c in CASES]}
    with open(os.path.join(HERE, "manifest_elementwise.json"), "w") as fh:
        json.dump(man, fh, indent=1)


if __name__ == "__main__":
    sys.exit(main())
