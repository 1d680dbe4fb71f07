"""Split-QKV / split-linear children (megatron_dion_amd/split.py) on CPU.

The semantics the reference's adapter gives `--dion-split-qkv` / `--dion-split-linear`
(dion_distrib_optimizer.py:3450-3580): each child is an independent Dion matrix on its
rows of the fused parent -- its own seeded Q (child uid, qkv.py:118-127, linear.py:105-113),
its own rank from its own global shape -- and its updated rows land back in the parent's
weight and momentum.  The check: the split run equals a run over separate matrices holding
the children's rows, started from the same Q, with the same sketches (test-only oracle
codec in both)."""
import torch

import megatron_dion_amd as mda
from megatron_dion_amd.optimizer import attach_dp_routing
from megatron_dion_amd.split import (child_uid, gather_rows, linear_child_segments, qkv_child_segments,
                                     qkvg_child_segments, state_key)
from megatron_dion_amd.state import init_q, q_seed_from_param_key
from tests._cpu_codec import OracleCodec

GROUPS, SPLIT = 4, (8, 4, 4)          # 4 query groups of [q 8 | k 4 | v 4] rows
COLS = 48
LIN = (40, 40)                        # gate / up rows of a fused fc1


def _sketch(P):
    mp_ = P.shape[-2]
    return torch.randn(1, 128, mp_, generator=torch.Generator().manual_seed(mp_)) / 128 ** 0.5


def test_qkv_segments_follow_the_grouped_layout():
    segs = qkv_child_segments(GROUPS * 16, SPLIT, "k")
    assert segs == [(8, 12), (24, 28), (40, 44), (56, 60)]
    assert qkv_child_segments(16, SPLIT, "q") == [(0, 8)]
    assert linear_child_segments(80, LIN, "up") == [(40, 80)]
    assert qkvg_child_segments(2 * 20, (8, 4, 4, 4), "gate") == [(8, 12), (28, 32)]
    t = torch.arange(GROUPS * 16).float().view(-1, 1)
    assert gather_rows(t, segs).view(-1).tolist() == [8, 9, 10, 11, 24, 25, 26, 27, 40, 41, 42, 43, 56, 57, 58, 59]
    assert gather_rows(t, linear_child_segments(80, LIN, "gate")).data_ptr() == t.data_ptr()  # a view


def _parents():
    g = torch.Generator().manual_seed(5)
    qkv = torch.nn.Parameter(torch.randn(GROUPS * sum(SPLIT), COLS, generator=g) * 0.02)
    qkv.is_qkv, qkv.qkv_split_shapes = True, SPLIT
    fc1 = torch.nn.Parameter(torch.randn(sum(LIN), COLS, generator=g) * 0.02)
    fc1.is_linear_fc1, fc1.linear_split_rows = True, LIN
    proj = torch.nn.Parameter(torch.randn(COLS, 32, generator=g) * 0.02)
    return [("layers.0.self_attention.linear_qkv.weight", qkv), ("layers.0.mlp.linear_fc1.weight", fc1),
            ("layers.0.self_attention.linear_proj.weight", proj)]


def _grads(step, named):
    g = torch.Generator().manual_seed(100 + step)
    return {n: torch.randn(p.shape, generator=g) * 1e-3 for n, p in named}


def test_split_run_equals_separate_children():
    named = _parents()
    opt = mda.MegatronDion([p for _, p in named], lr=0.02, mu=0.95, weight_decay=0.01, rank_fraction=0.25,
                           split_qkv=True, split_linear=True, codec=OracleCodec(sketch_lookup=_sketch))
    attach_dp_routing(opt, named)
    rows = {n: p.shape[0] for n, p in named}
    segs = {}
    for kind in ("q", "k", "v"):
        segs[(named[0][0], kind)] = ("qkv", qkv_child_segments(rows[named[0][0]], SPLIT, kind))
    for kind in ("gate", "up"):
        segs[(named[1][0], kind)] = ("linear", linear_child_segments(rows[named[1][0]], LIN, kind))
    # parent state: the reference's keys, per-child Q from the child identity
    st = opt.state[named[0][1]]
    assert st["qkv_split_qkv"] and tuple(st["qkv_split_shapes"]) == SPLIT and "Q" not in st
    assert tuple(st[state_key("qkv", "global_shape", "q")]) == (GROUPS * 8, COLS)
    assert st[state_key("qkv", "r", "k")] == max(1, int(0.25 * min(GROUPS * 4, COLS)))
    assert tuple(opt.state[named[1][1]][state_key("linear", "global_shape", "up")]) == (40, COLS)

    # separate matrices holding the children's rows, same Q0
    child_named, q0 = [], {}
    for (pname, kind), (family, sg) in segs.items():
        parent = dict(named)[pname]
        cp = torch.nn.Parameter(gather_rows(parent.data, sg).clone())
        child_named.append((f"{pname}::{kind}", cp))
        q0[f"{pname}::{kind}"] = opt.state[parent][state_key(family, "Q", kind)].clone()
    child_named.append(named[2][0:1] + (torch.nn.Parameter(named[2][1].data.clone()),))
    ref = mda.MegatronDion([p for _, p in child_named], lr=0.02, mu=0.95, weight_decay=0.01, rank_fraction=0.25,
                           codec=OracleCodec(sketch_lookup=_sketch), defer_error_feedback=False)
    attach_dp_routing(ref, child_named)
    ref_p = dict(child_named)
    for n, q in q0.items():
        ref.state[ref_p[n]]["Q"].copy_(q)
    # the child Q is the seeded draw of the child identity (state.py rules, uid-derived):
    # v child = (16, 48), transposed, r = 4, Q over its 16 rows
    seed = q_seed_from_param_key(base_seed=0, param_uid=child_uid((named[0][0],), "qkv", "v"),
                                 param_name=f"{named[0][0]}::v", q_global_shape=(16, 4), is_transposed=True)
    assert torch.equal(q0[f"{named[0][0]}::v"], init_q((16, 4), seed, "cpu"))

    for step in range(3):
        grads = _grads(step, named)
        for n, p in named:
            p.grad = grads[n].clone()
        for (pname, kind), (family, sg) in segs.items():
            ref_p[f"{pname}::{kind}"].grad = gather_rows(grads[pname], sg).clone()
        ref_p[named[2][0]].grad = grads[named[2][0]].clone()
        opt.step()
        ref.step()
        for (pname, kind), (family, sg) in segs.items():
            parent = dict(named)[pname]
            cn = f"{pname}::{kind}"
            for got, want in ((gather_rows(parent.data, sg), ref_p[cn].data),
                              (gather_rows(opt.state[parent]["momentum"], sg), ref.state[ref_p[cn]]["momentum"]),
                              (opt.state[parent][state_key(family, "Q", kind)], ref.state[ref_p[cn]]["Q"])):
                assert torch.allclose(got, want, rtol=0, atol=1e-7 * max(1.0, want.abs().max().item())), \
                    (step, cn, (got - want).abs().max().item())
        assert torch.allclose(named[2][1].data, ref_p[named[2][0]].data, rtol=0, atol=1e-8)
