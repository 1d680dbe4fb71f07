"""Checkpoint compatibility of the product optimizer against the REFERENCE's own save / restore.

Run ONLY in the build container (the reference tree does not exist on the GPU box):

    PYTHONPATH=/root/reference DION_DISABLE_TORCH_COMPILE=1 python scripts/ref/ref_checkpoint_check.py

Megatron saves and restores Dion state with
`distrib_dion/checkpoint_io.py:247-268 build_persistent_param_state` (iterates
`optimizer.state[p].items()`, drops '_' keys, adds "param") and
`:271-378 restore_persistent_param_state_` (keeps the live '_' keys, installs new tensors for
every persistent key, sets the Q-sync flags, including the split children's).  This script
imports those two functions from /root/reference and drives them on the product's
`MegatronDion` / `DionStateMap` (oracle codec, CPU, deferred error feedback on -- the drop-in
default -- so the save happens while every plain matrix holds a pending EF):

  uninterrupted  6 steps
  interrupted    3 steps -> build_persistent_param_state -> torch.save / torch.load
                 (weights_only=True) -> a FRESH optimizer over fresh parameters ->
                 restore_persistent_param_state_ -> 3 more steps

and compares W, the momentum, Q and every split child's Q key of the two runs bitwise.  The
set: a fused QKV parent (split_qkv: q / k / v children), a fused SwiGLU fc1 (split_linear:
gate / up), a plain matrix and a transposed plain matrix.  Output:
profiles/r05/ref_checkpoint_check.json.
"""
import io
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import megatron_dion_amd as mda  # noqa: E402
from megatron_dion_amd.optimizer import attach_dp_routing  # noqa: E402
from megatron_dion_amd.runtime import _PENDING_EF  # noqa: E402
from oracle.cpu_codec import OracleCodec  # noqa: E402

GROUPS, SPLIT, COLS, LIN = 4, (8, 4, 4), 48, (40, 40)
NAMES = ("layers.0.self_attention.linear_qkv.weight", "layers.0.mlp.linear_fc1.weight",
         "layers.0.self_attention.linear_proj.weight", "layers.0.mlp.linear_fc2.weight")


def _sketch(P):
    mp_ = P.shape[-2]
    return torch.randn(1, 128, mp_, generator=torch.Generator().manual_seed(mp_)) / 128 ** 0.5


def _params(seed):
    g = torch.Generator().manual_seed(seed)
    qkv = torch.nn.Parameter(torch.randn(GROUPS * sum(SPLIT), COLS, generator=g) * 0.02)
    qkv.is_qkv, qkv.qkv_split_shapes = True, SPLIT
    fc1 = torch.nn.Parameter(torch.randn(sum(LIN), COLS, generator=g) * 0.02)
    fc1.is_linear_fc1, fc1.linear_split_rows = True, LIN
    proj = torch.nn.Parameter(torch.randn(COLS, 32, generator=g) * 0.02)
    fc2 = torch.nn.Parameter(torch.randn(40, 96, generator=g) * 0.02)
    return list(zip(NAMES, (qkv, fc1, proj, fc2)))


def _optimizer(named):
    opt = mda.MegatronDion([p for _, p in named], lr=0.02, mu=0.95, weight_decay=0.01, rank_fraction=0.25,
                           split_qkv=True, split_linear=True,
                           codec=OracleCodec(sketch_lookup=_sketch, deferred=True))
    assert opt._defer_ef
    attach_dp_routing(opt, named)
    return opt


def _step(opt, named, i):
    g = torch.Generator().manual_seed(100 + i)
    for _, p in named:
        p.grad = (torch.randn(p.shape, generator=g) * 1e-3).to(torch.bfloat16).float()
    opt.step()


def _snapshot(opt, named):
    opt.flush_error_feedback()
    out = {}
    for n, p in named:
        out[f"{n}.param"] = p.detach().clone()
        for k, v in opt.state[p].items():
            if torch.is_tensor(v) and (k == "momentum" or k == "Q" or k.endswith("_Q")):
                out[f"{n}.{k}"] = v.clone()
    return out


def main():
    from megatron.core.optimizer.distrib_dion.checkpoint_io import (build_persistent_param_state,
                                                                    restore_persistent_param_state_)

    before, after = 3, 3
    ref_named = _params(5)
    ref = _optimizer(ref_named)
    for i in range(before + after):
        _step(ref, ref_named, i)
    want = _snapshot(ref, ref_named)

    named = _params(5)
    opt = _optimizer(named)
    for i in range(before):
        _step(opt, named, i)
    name_of = {id(p): n for n, p in named}
    pending_at_save = sorted(n for n, p in named if _PENDING_EF in dict.keys(opt.state[p]))
    payload = build_persistent_param_state(opt.param_groups, opt.state, lambda p: name_of.get(id(p)))
    buf = io.BytesIO()
    torch.save(payload, buf)
    buf.seek(0)
    payload = torch.load(buf, weights_only=True)
    saved_keys = {n: sorted(k for k in st if k != "param") for n, st in payload.items()}

    fresh = _params(99)  # other initial weights: the restore must install the checkpoint's
    opt2 = _optimizer(fresh)
    fname_of = {id(p): n for n, p in fresh}
    summary = restore_persistent_param_state_(param_groups=opt2.param_groups, optimizer_state=opt2.state,
                                              get_param_key=lambda p: fname_of.get(id(p)), key_to_state=payload,
                                              mixed_precision_config=None)
    for i in range(before, before + after):
        _step(opt2, fresh, i)
    got = _snapshot(opt2, fresh)

    rows, ok = {}, True
    for key, w in want.items():
        g = got.get(key)
        same = g is not None and g.dtype == w.dtype and torch.equal(g, w)
        diff = None if g is None else (g.double() - w.double()).abs().max().item()
        rows[key] = {"bitwise_equal": bool(same), "max_abs_diff": diff}
        ok &= bool(same)
    ok &= summary["restored"] == len(named) and set(got) == set(want)
    out = {
        "check": "product MegatronDion state through the reference's build_persistent_param_state / "
                 "restore_persistent_param_state_ (checkpoint_io.py:247-378), deferred EF pending at the save",
        "steps": {"before_save": before, "after_restore": after},
        "pending_ef_at_save": pending_at_save,
        "saved_state_keys": saved_keys,
        "restore_summary": summary,
        "compared": rows,
        "pass": bool(ok),
    }
    dst = os.path.join(ROOT, "profiles", "r05")
    os.makedirs(dst, exist_ok=True)
    with open(os.path.join(dst, "ref_checkpoint_check.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps({"pass": out["pass"], "restored": summary, "tensors": len(rows),
                      "pending_ef_at_save": pending_at_save}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
