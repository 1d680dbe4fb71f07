"""World-size-2 replicate path with the HIP codec on the GPU (`pytest -m gpu`).

Two processes share cuda:0 and exchange through gloo (RCCL needs one GPU per
rank; the 8-GPU RCCL run is the driver's).  Everything else is the product
path: HIP kernels through the C ABI, per-slot HIP streams for the AsyncRuntime,
reduce-scatter / all-gather of P and all-reduce of R, deferred or eager error
feedback.  Checked against the reference's own 2-rank golden capture c8
(W1, Q1 every step; M1 after the flush).
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests._metrics import dw_err

pytestmark = pytest.mark.gpu

TOL_WM = 1e-5
TOL_Q = 1e-5
TOL_DW = 5e-6  # the weight step alone against the reference's (tests/_metrics.dw_err), fp32 state


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, name, out_dir, deferred):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    import megatron_dion_amd as mda
    from megatron_dion_amd.optimizer import attach_dp_routing
    from tests._golden import Case

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    case = Case(name)
    h = case.hyper
    names = [n for n, _, _ in case.mats]
    params = {n: torch.nn.Parameter(case.t(rank, 0, f"{n}_W0").to(dev)) for n in names}
    mpc = mda.DionMixedPrecisionConfig(momentum_dtype=torch.bfloat16, q_dtype=torch.bfloat16) \
        if case.entry.get("bf16") else None  # case (viii): bf16 momentum and Q
    opt = mda.MegatronDion([params[n] for n in names], lr=h["lr"], mu=h["mu"], weight_decay=h["weight_decay"],
                           rank_fraction=case.rank_fraction, epsilon=h["epsilon"],
                           rcqr_oversample=h["rcqr_oversample"], defer_error_feedback=deferred,
                           mixed_precision_config=mpc)
    attach_dp_routing(opt, [(n, params[n]) for n in names], replicate_group=dist.group.WORLD)
    for n in names:
        opt.state[params[n]]["Q"].copy_(case.t(rank, 0, f"{n}_Q0").to(dev))
    results = {}
    for step in range(case.steps):
        for n in names:
            params[n].grad = case.t(rank, step, f"{n}_G").to(dev)
        # the sketch this rank drew for the entry it owns (ortho calls are per owned entry)
        calls = case.ortho_calls(rank, step)
        opt._sketch_override = _owned_sketch(rank, calls, dev)
        opt.step()
        if deferred and step == case.steps - 1:
            opt.flush_error_feedback()
        torch.cuda.synchronize()
        for n in names:
            results[f"s{step}_{n}_W"] = params[n].detach().cpu()
            results[f"s{step}_{n}_M"] = opt.state[params[n]]["momentum"].cpu()
            results[f"s{step}_{n}_Q"] = opt.state[params[n]]["Q"].cpu()
    torch.save(results, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _owned_sketch(rank, calls, dev):
    """Sketch override for a W = 2 batch: rank k orthonormalises entry chunk_start + k."""
    S = [c["S"] for c in calls]

    def fn(batch):
        out = {}
        for i in range(len(batch.params)):
            if i % 2 == rank and S and S[0] is not None:
                out[i] = S[0][0].to(dev)
        return out or None
    return fn


@pytest.mark.parametrize("name,deferred", [("c8_w2_two_steps_T", False), ("c8_w2_two_steps_T", True),
                                            ("c12_bf16_w2_two_steps_T", False)],
                         ids=["eager_ef", "deferred_ef", "bf16_state"])
def test_hip_codec_w2_matches_reference(name, deferred):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tests._golden import Case

    case = Case(name)
    h = case.hyper
    bf16 = bool(case.entry.get("bf16"))
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_worker, args=(2, _free_port(), case.name, tmp, deferred), nprocs=2, join=True,
                           start_method="spawn")
        res = [torch.load(os.path.join(tmp, f"rank{r}.pt"), weights_only=True) for r in range(2)]
    names = [n for n, _, _ in case.mats]

    def maxrel(a, b):
        return (a.double() - b.double()).abs().max().item() / max(b.double().abs().max().item(), 1e-30)

    for rank in range(2):
        for step in range(case.steps):
            for n in names:
                # bf16 state: one bf16 ulp of the largest element (tests/test_gpu_bf16.py explains)
                keys = [("W", "W1", 1e-3 if bf16 else TOL_WM), ("Q", "Q1", 2e-2 if bf16 else TOL_Q)]
                if not deferred or step == case.steps - 1:
                    keys.append(("M", "M1", 2 ** -6 if bf16 else TOL_WM))
                for k, ref, tol in keys:
                    err = maxrel(res[rank][f"s{step}_{n}_{k}"].float(), case.t(rank, step, f"{n}_{ref}"))
                    assert err <= tol, (rank, step, n, k, err)
                if not bf16:
                    w_prev = case.t(rank, 0, f"{n}_W0") if step == 0 else res[rank][f"s{step - 1}_{n}_W"]
                    err = dw_err(w_prev, res[rank][f"s{step}_{n}_W"], case.t(rank, step, f"{n}_W0"),
                                 case.t(rank, step, f"{n}_W1"), 1.0 - h["lr"] * h["weight_decay"])
                    assert err <= TOL_DW, (rank, step, n, "dW", err)
    for n in names:
        assert torch.equal(res[0][f"s1_{n}_W"], res[1][f"s1_{n}_W"])
        assert torch.equal(res[0][f"s1_{n}_Q"], res[1][f"s1_{n}_Q"])
