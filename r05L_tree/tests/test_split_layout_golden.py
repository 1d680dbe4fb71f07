"""split.split_child_layouts against the reference's own child-segment helpers.

tests/golden/split_layouts.json holds, per case and per member of the parent's row-shard group,
the segments the reference's qkv.py / qkvg.py `_child_segments` and linear.py
`_linear_child_segments` return (made by tests/golden/make_golden_split_layout.py from the
reference tree).  For every member this rebuilds its shard of the fused parent, asks
split_child_layouts for its layout and checks the source rows, the child's row range and every
owner's child row count.  Children whose rows miss members of the group are owned by the members
holding some of their rows (row_child.py:62-106): a rank outside them gets no rows, a single owner
holds the child whole (no row shard), several owners shard it among themselves."""
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
    for member in case["members"]:
        out = _layout(case, member)
        assert list(out) == case["kinds"]
        for kind in case["kinds"]:
            ref = member["segments"][kind]
            got = out[kind]
            owners = [m for m in case["members"] if m["segments"][kind]]
            assert got["members"] == tuple(int(m["rank"]) for m in owners)
            sizes = tuple(sum(s[3] - s[2] for s in m["segments"][kind]) for m in owners)
            assert sum(sizes) == case["child_rows"][kind]
            if not ref:  # no rows of this child here (row_child.py:105-106)
                assert got["local_rows"] == 0 and got["segments"] == [] and got["child_rank"] == -1
                continue
            assert [list(s) for s in got["segments"]] == [s[:2] for s in ref], (kind, member["rank"])
            # the reference's child rows of this member are one contiguous run
            assert all(x[3] == y[2] for x, y in zip(ref, ref[1:]))
            c0, c1 = ref[0][2], ref[-1][3]
            assert got["local_rows"] == c1 - c0
            assert got["child_rank"] == [int(m["rank"]) for m in owners].index(int(member["rank"]))
            spec = got["tp"] if case["axis"] == "tp" else got["fs"]
            if len(owners) == 1:  # one owner: the whole child, no row shard (world 1)
                assert spec is None and got["row_sizes"] is None and got["row_axis"] is None
                assert (c0, c1) == (0, case["child_rows"][kind])
                continue
            assert tuple(spec[0]) == (case["child_rows"][kind], COLS)
            assert (spec[1], spec[2], spec[3]) == (0, c0, c1)
            assert got["row_axis"] == case["axis"]
            assert got["row_sizes"] == sizes
