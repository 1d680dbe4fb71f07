"""split.split_child_layouts against the reference's own child-segment helpers.

tests/golden/split_layouts.json holds, per case and per member of the parent's row-shard group,
the segments the reference's qkv.py / qkvg.py `_child_segments` and linear.py
`_linear_child_segments` return (made by tests/golden/make_golden_split_layout.py from the
reference tree).  For every member this rebuilds its shard of the fused parent, asks
split_child_layouts for its layout and checks the source rows, the child's row range, every
member's child row count and the refusal of children whose rows miss a member
([DION_SPLIT_CHILD_PARTIAL_OWNERS]; the reference builds a sub-group there, row_child.py:94-106)."""
import json
import os

import pytest
import torch

from megatron_dion_amd.split import split_child_layouts, split_plan

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "split_layouts.json")) as fh:
    CASES = json.load(fh)["cases"]
COLS = 8


def _member_param(case, rows):
    p = torch.empty(rows, COLS)
    split = tuple(case["split"])
    if case["family"] == "qkv":
        p.is_qkv, p.qkv_split_shapes = True, split
        return p, {"split_qkv": True}
    if case["family"] == "qkvg":
        p.is_qkvg, p.qkvg_split_shapes = True, split
        return p, {"split_qkv": True}
    p.is_linear_fc1, p.linear_split_rows = True, split
    p.partition_stride = int(case["partition_stride"])
    return p, {"split_linear": True}


def _layout(case, member):
    gm = int(case["global_rows"])
    a, b = member["parent_range"]
    world, rank = int(case["world"]), int(member["rank"])
    if case["family"] == "linear" and case["partition_stride"] == len(case["split"]):
        # Megatron's strided SwiGLU shard: this rank holds its split of gate, then of up
        rows = sum(seg[1] - seg[0] for k in case["kinds"] for seg in member["segments"][k])
    else:
        rows = b - a
    p, defaults = _member_param(case, rows)
    plan = split_plan(p, defaults, global_rows=gm)
    spec = ((gm, COLS), 0, a, b)
    if case["axis"] == "tp":
        return split_child_layouts(p, plan, tp_spec=spec, tp_world=world, tp_rank=rank)
    return split_child_layouts(p, plan, fs_spec=spec, fs_world=world, fs_rank=rank)


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_split_child_layouts_match_reference_segments(case):
    partial = any(not m["segments"][k] for m in case["members"] for k in case["kinds"])
    for member in case["members"]:
        if partial:
            with pytest.raises(RuntimeError, match="DION_SPLIT_CHILD_PARTIAL_OWNERS"):
                _layout(case, member)
            continue
        out = _layout(case, member)
        assert list(out) == case["kinds"]
        for kind in case["kinds"]:
            ref = member["segments"][kind]
            got = out[kind]
            assert [list(s) for s in got["segments"]] == [s[:2] for s in ref], (kind, member["rank"])
            # the reference's child rows of this member are one contiguous run
            assert all(x[3] == y[2] for x, y in zip(ref, ref[1:]))
            c0, c1 = ref[0][2], ref[-1][3]
            spec = got["tp"] if case["axis"] == "tp" else got["fs"]
            assert tuple(spec[0]) == (case["child_rows"][kind], COLS)
            assert (spec[1], spec[2], spec[3]) == (0, c0, c1)
            assert got["local_rows"] == c1 - c0
            assert got["row_axis"] == case["axis"]
            sizes = tuple(sum(s[3] - s[2] for s in m["segments"][kind]) for m in case["members"])
            assert got["row_sizes"] == sizes
            assert sum(sizes) == case["child_rows"][kind]
