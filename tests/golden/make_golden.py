"""Generate the golden Dion-step fixtures from the REFERENCE implementation.

Run ONLY in the build container (the reference tree does not exist on the GPU box):

    PYTHONPATH=/root/reference DION_DISABLE_TORCH_COMPILE=1 \
        python tests/golden/make_golden.py

It drives the reference's own `MegatronDion.step` through its own batch builder
(`megatron/core/optimizer/distrib_dion/batches.py:971 build_dion_batches`) on
gloo (1 or 2 ranks), exactly as SURVEY.md Appendix B describes, and records:

* inputs per matrix and step: W0, M0, Q0, G (bf16-valued fp32)
* every call into `dion.runtime.orthogonalize` (P in, sketch S used, P out)
  -- the sketch is captured by wrapping `dion.ortho.generate_random_sketch_matrix`
* every call into `dion.runtime.fix_all_zero_or_nan` and `normalize_columns`
* the batch schedule (`batch_dion_update_async` calls: member names, real size)
* outputs per matrix and step: W1, M1, Q1

The result is one small `.npz` per case plus `manifest.json`.  Only data is
committed (inputs and expected outputs); no reference source is copied.
"""

import json
import math
import os
import sys
import tempfile

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))

# name, list of (matrix name, m, n), r, world, steps, extra options
CASES = [
    dict(name="c1_64x48_r8", mats=[("w0", 64, 48)], r=8, world=1, steps=1),
    dict(name="c2_48x96_T_r8", mats=[("w0", 48, 96)], r=8, world=1, steps=1),
    dict(name="c3_32x32_r32_plainqr", mats=[("w0", 32, 32)], r=32, world=1, steps=1),
    dict(name="c3b_96x64_r16_widesketch", mats=[("w0", 96, 64)], r=16, world=1, steps=1),
    dict(
        name="c4_w2_pad3",
        mats=[("a", 64, 40), ("b", 64, 40), ("c", 64, 40)],
        r=8,
        world=2,
        steps=1,
    ),
    dict(
        name="c5_zero_entry",
        mats=[("nz", 48, 32), ("zz", 48, 32)],
        r=8,
        world=1,
        steps=1,
        zero=("zz",),
    ),
    dict(
        name="c6_rank_deficient",
        mats=[("rd", 64, 32)],
        r=8,
        world=1,
        steps=1,
        rank1=("rd",),
    ),
    dict(
        name="c7_two_steps_mixed",
        mats=[("p", 80, 48), ("q", 48, 112), ("s", 80, 48)],
        r=16,
        world=1,
        steps=2,
    ),
    dict(
        name="c8_w2_two_steps_T",
        mats=[("x", 40, 72), ("y", 40, 72)],
        r=8,
        world=2,
        steps=2,
    ),
    dict(
        name="c9_256x192_r64",
        mats=[("big", 256, 192)],
        r=64,
        world=1,
        steps=2,
    ),
    dict(
        name="c10_160x384_T_r64",
        mats=[("bigT", 160, 384)],
        r=64,
        world=1,
        steps=1,
    ),
    # (viii) the speedrun's mixed precision: bf16 momentum and bf16 Q
    # (examples/dion/speedrun_nanogpt_mcore.py:422-431, --dion-momentum-dtype/--dion-q-dtype bfloat16)
    dict(
        name="c11_bf16_two_steps_mixed",
        mats=[("p", 96, 64), ("q", 64, 160), ("s", 96, 64)],
        r=16,
        world=1,
        steps=2,
        bf16=True,
    ),
    dict(
        name="c12_bf16_w2_two_steps_T",
        mats=[("x", 48, 80), ("y", 48, 80)],
        r=8,
        world=2,
        steps=2,
        bf16=True,
    ),
    # independent momentum / Q dtypes (DionMixedPrecisionConfig, dion/types.py:10-17,
    # state.py:502-547): fp32 momentum with bf16 Q, and bf16 momentum with fp32 Q
    dict(
        name="c13_m32_q16_two_steps",
        mats=[("p", 96, 64), ("q", 64, 160)],
        r=16,
        world=1,
        steps=2,
        m_dtype="float32",
        q_dtype="bfloat16",
    ),
    dict(
        name="c14_m16_q32_two_steps",
        mats=[("p", 96, 64), ("q", 64, 160)],
        r=16,
        world=1,
        steps=2,
        m_dtype="bfloat16",
        q_dtype="float32",
    ),
    # world size 4 (BASELINE config 4's replicated schedule at W > 2): one full batch of
    # four 64x40 matrices and one padded batch of three transposed 40x72 ones (entry c W + r
    # owned by rank r, a zero padded entry on rank 3).  Each shape forms a single batch, so
    # the reference's shape-keyed "replicated_p_ortho_full" buffer (algorithm.py:233-244)
    # is never shared between batches in flight and the capture is the Dion step itself.
    dict(
        name="c15_w4_pad_two_steps",
        mats=[("a0", 64, 40), ("a1", 64, 40), ("a2", 64, 40), ("a3", 64, 40),
              ("t0", 40, 72), ("t1", 40, 72), ("t2", 40, 72)],
        r=8,
        world=4,
        steps=2,
    ),
]

HYPER = dict(lr=0.01, mu=0.95, weight_decay=0.01, epsilon=1e-8, rcqr_oversample=1.25,
             scale_mode="spectral", extra_scale_factor=0.2)


def _bf16_values(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.bfloat16).to(torch.float32)


def make_inputs(case, rank):
    """Deterministic synthetic inputs (SURVEY.md 8(d) recipe, scaled down)."""
    out = {}
    r = case["r"]
    for idx, (name, m, n) in enumerate(case["mats"]):
        transposed = m < n
        q_rows = m if transposed else n
        g = torch.Generator().manual_seed(1000 + idx)
        w0 = torch.randn(m, n, generator=g) * 0.02
        gq = torch.Generator().manual_seed(2000 + idx)
        q0 = torch.randn(q_rows, r, generator=gq)
        grads = []
        for step in range(case["steps"]):
            gg = torch.Generator().manual_seed(99 + rank + 17 * step + 131 * idx)
            if name in case.get("zero", ()):
                gr = torch.zeros(m, n)
            elif name in case.get("rank1", ()):
                u = torch.randn(m, 1, generator=gg)
                v = torch.randn(1, n, generator=gg)
                gr = (u @ v) * 1e-3
            else:
                gr = torch.randn(m, n, generator=gg) * 1e-3
            grads.append(_bf16_values(gr))
        out[name] = dict(w0=w0, q0=q0, grads=grads, m=m, n=n, transposed=transposed)
    return out


def _worker(rank, world, case, port, out_path):
    os.environ["DION_DISABLE_TORCH_COMPILE"] = "1"
    dist.init_process_group(
        "gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world
    )
    torch.manual_seed(0)  # global RNG drives the unseeded replicated-path sketch
    from megatron.core.optimizer.dion import ortho as d_ortho
    from megatron.core.optimizer.dion import runtime as d_rt
    from megatron.core.optimizer.dion.algorithm import MegatronDion
    from megatron.core.optimizer.dion.types import (
        DionDistMeta,
        DionMixedPrecisionConfig,
        DionParamConfig,
        DionStepParam,
    )
    from megatron.core.optimizer.distrib_dion.batches import build_dion_batches

    inputs = make_inputs(case, rank)
    r = case["r"]
    names = [name for name, _, _ in case["mats"]]
    params = {}
    for name in names:
        params[name] = torch.nn.Parameter(inputs[name]["w0"].clone())
    m0, n0 = inputs[names[0]]["m"], inputs[names[0]]["n"]
    rank_fraction = r / min(m0, n0)
    state_dtype = torch.bfloat16 if case.get("bf16") else torch.float32
    m_dtype = getattr(torch, case["m_dtype"]) if "m_dtype" in case else state_dtype
    q_dtype = getattr(torch, case["q_dtype"]) if "q_dtype" in case else state_dtype
    mixed = DionMixedPrecisionConfig(momentum_dtype=m_dtype, q_dtype=q_dtype) \
        if (case.get("bf16") or "m_dtype" in case) else None
    opt = MegatronDion(
        [params[n] for n in names],
        lr=HYPER["lr"],
        mu=HYPER["mu"],
        weight_decay=HYPER["weight_decay"],
        rank_fraction=rank_fraction,
        epsilon=HYPER["epsilon"],
        rcqr_oversample=HYPER["rcqr_oversample"],
        scale_mode=HYPER["scale_mode"],
        extra_scale_factor=HYPER["extra_scale_factor"],
        mixed_precision_config=mixed,
    )
    configs, metas = {}, {}
    for name in names:
        d = inputs[name]
        m, n = d["m"], d["n"]
        low_rank = (rank_fraction < 1.0) and ((m + n) * r < m * n)
        configs[name] = DionParamConfig(is_transposed=d["transposed"], use_low_rank_sync=low_rank)
        metas[name] = DionDistMeta(
            shape=(m, n), global_shape=(m, n), rank_fraction=rank_fraction,
            param_uid=(name,), is_dion_param=True, param_name=name,
            param_config=configs[name], is_transposed=d["transposed"],
        )
        opt.state[params[name]] = dict(
            momentum=torch.zeros(m, n, dtype=m_dtype),
            Q=d["q0"].clone().to(q_dtype),
            r=r,
            local_shape=(m, n),
            global_shape=(m, n),
        )
    id2name = {id(params[n]): n for n in names}
    grads_now = {}
    cache = {}

    def route():
        steps = []
        for name in sorted(names):
            p = params[name]
            steps.append(DionStepParam(
                param=p, grad=grads_now[name], optimizer_state=opt.state[p],
                optim_group=opt.param_groups[0], config=configs[name],
                dist_meta=metas[name]))
        batches = build_dion_batches(
            dion_params=steps, use_fs_collectives=True, state_replica_group=None,
            replica_validation_group=dist.group.WORLD, batch_key_cache=cache,
            global_rank=rank, group_size=dist.get_world_size,
            get_replicate_group=lambda: dist.group.WORLD,
            resolve_ortho_group=lambda c, m: None,
            resolve_tp_group=lambda m, expect_group: None,
            resolve_fs_group_from_meta=lambda m, expect_group: None,
        )
        return batches, []

    opt.enable_distributed_mode(route_step_params=route)

    rec = {"batches": [], "ortho": [], "fixup": [], "norm": []}
    sketches = []
    orig_sketch = d_ortho.generate_random_sketch_matrix

    def sketch_wrap(P, oversample=1.25, make_sketch=None):
        S = orig_sketch(P, oversample=oversample, make_sketch=make_sketch)
        sketches.append(S.detach().clone())
        return S

    d_ortho.generate_random_sketch_matrix = sketch_wrap
    orig_orth = d_rt.orthogonalize

    def orth_wrap(P, rcqr_oversample=1.25, make_sketch=None):
        n_before = len(sketches)
        out = orig_orth(P, rcqr_oversample=rcqr_oversample, make_sketch=make_sketch)
        S = sketches[-1] if len(sketches) > n_before else None
        rec["ortho"].append(dict(p_in=P.detach().clone(), p_out=out.detach().clone(), s=S))
        return out

    d_rt.orthogonalize = orth_wrap
    orig_fix = d_rt.fix_all_zero_or_nan

    def fix_wrap(P, R, Q, M, *, real_batch_size):
        p_out, r_out = orig_fix(P, R, Q, M, real_batch_size=real_batch_size)
        rec["fixup"].append(dict(p_in=P.clone(), r_in=R.clone(), p_out=p_out.clone(),
                                 r_out=r_out.clone(), real=int(real_batch_size)))
        return p_out, r_out

    d_rt.fix_all_zero_or_nan = fix_wrap
    orig_norm = d_rt.normalize_columns

    def norm_wrap(R, col_sum_sq, *, epsilon):
        q = orig_norm(R, col_sum_sq, epsilon=epsilon)
        rec["norm"].append(dict(r_in=R.clone(), q_out=q.clone()))
        return q

    d_rt.normalize_columns = norm_wrap
    orig_bdu = d_rt.batch_dion_update_async

    def bdu_wrap(optimizer, params_l, *args, **kwargs):
        real = kwargs.get("real_batch_size", args[8] if len(args) > 8 else len(params_l))
        members = [id2name.get(id(p), "<pad>") for p in params_l]
        rec["batches"].append(dict(members=members, real=int(real)))
        return (yield from orig_bdu(optimizer, params_l, *args, **kwargs))

    d_rt.batch_dion_update_async = bdu_wrap

    arrays = {}
    meta = {"steps": []}
    for step in range(case["steps"]):
        for name in names:
            p = params[name]
            arrays[f"s{step}_{name}_W0"] = p.detach().clone()
            arrays[f"s{step}_{name}_M0"] = opt.state[p]["momentum"].clone()
            arrays[f"s{step}_{name}_Q0"] = opt.state[p]["Q"].clone()
            g = inputs[name]["grads"][step].clone()
            arrays[f"s{step}_{name}_G"] = g.clone()
            grads_now[name] = g
        for key in rec:
            rec[key] = []
        opt.step()
        for name in names:
            p = params[name]
            arrays[f"s{step}_{name}_W1"] = p.detach().clone()
            arrays[f"s{step}_{name}_M1"] = opt.state[p]["momentum"].clone()
            arrays[f"s{step}_{name}_Q1"] = opt.state[p]["Q"].clone()
        smeta = {"batches": rec["batches"], "ortho": [], "fixup": [], "norm": len(rec["norm"])}
        for i, o in enumerate(rec["ortho"]):
            arrays[f"s{step}_ortho{i}_pin"] = o["p_in"]
            arrays[f"s{step}_ortho{i}_pout"] = o["p_out"]
            if o["s"] is not None:
                arrays[f"s{step}_ortho{i}_S"] = o["s"]
            smeta["ortho"].append({"has_sketch": o["s"] is not None,
                                   "shape": list(o["p_in"].shape)})
        for i, f in enumerate(rec["fixup"]):
            for k in ("p_in", "r_in", "p_out", "r_out"):
                arrays[f"s{step}_fix{i}_{k}"] = f[k]
            smeta["fixup"].append({"real": f["real"]})
        for i, nrm in enumerate(rec["norm"]):
            arrays[f"s{step}_norm{i}_rin"] = nrm["r_in"]
            arrays[f"s{step}_norm{i}_qout"] = nrm["q_out"]
        meta["steps"].append(smeta)
    # bf16 tensors are stored as their exact fp32 values (numpy has no bf16)
    np.savez_compressed(out_path, **{k: (v.detach().float() if v.dtype == torch.bfloat16 else v.detach()).numpy()
                                     for k, v in arrays.items()})
    with open(out_path + ".json", "w") as fh:
        json.dump(meta, fh)
    dist.barrier()
    dist.destroy_process_group()


def main():
    """`make_golden.py [name ...]` regenerates only the named cases and keeps the rest of the manifest."""
    only = set(sys.argv[1:])
    manifest = {"hyper": HYPER, "cases": []}
    if only and os.path.exists(os.path.join(HERE, "manifest.json")):
        with open(os.path.join(HERE, "manifest.json")) as fh:
            manifest = json.load(fh)
        manifest["cases"] = [c for c in manifest["cases"] if c["name"] not in only]
    port = 29611
    for case in CASES:
        if only and case["name"] not in only:
            port += 1
            continue
        world = case["world"]
        with tempfile.TemporaryDirectory() as tmp:
            paths = [os.path.join(tmp, f"rank{r}.npz") for r in range(world)]
            ctx = mp.get_context("spawn")
            procs = []
            for r in range(world):
                pr = ctx.Process(target=_worker, args=(r, world, case, port, paths[r][:-4]))
                pr.start()
                procs.append(pr)
            for pr in procs:
                pr.join()
                if pr.exitcode != 0:
                    raise SystemExit(f"case {case['name']} rank failed: {pr.exitcode}")
            port += 1
            merged = {}
            metas = []
            for r in range(world):
                with np.load(paths[r]) as z:
                    for k in z.files:
                        merged[f"r{r}_{k}"] = z[k]
                with open(paths[r][:-4] + ".json") as fh:
                    metas.append(json.load(fh))
        out = os.path.join(HERE, f"{case['name']}.npz")
        np.savez_compressed(out, **merged)
        entry = {k: v for k, v in case.items()}
        entry["mats"] = [list(m) for m in case["mats"]]
        entry["rank_meta"] = metas
        manifest["cases"].append(entry)
        print("wrote", out, os.path.getsize(out), "bytes", flush=True)
    order = [c["name"] for c in CASES]
    manifest["cases"].sort(key=lambda c: order.index(c["name"]) if c["name"] in order else len(order))
    with open(os.path.join(HERE, "manifest.json"), "w") as fh:
        json.dump(manifest, fh, indent=1, default=list)


if __name__ == "__main__":
    sys.exit(main())
