"""Golden layouts of split children of row-sharded parents, computed by the REFERENCE's helpers.

Run ONLY in the build container (the reference tree does not exist on the GPU box):

    PYTHONPATH=/root/reference DION_DISABLE_TORCH_COMPILE=1 python tests/golden/make_golden_split_layout.py

For every member of the parent's row-shard group (TP on dim 0, or FS on dim 0; canonical
ranges, distrib_dion/sharding.py:44-61) this records the reference's (source_start,
source_end, child_start, child_end) segments of each child kind: dion/qkv.py and dion/qkvg.py
`_child_segments` over the member's parent row range, dion/linear.py `_linear_child_segments`
(incl. Megatron's strided SwiGLU TP shard, `linear_partition_stride` 2), and the child's global
rows.  tests/test_split_children.py checks split.split_child_layouts against it.  Only data is
committed (tests/golden/split_layouts.json).
"""
import json
import os
import sys
from types import SimpleNamespace

HERE = os.path.dirname(os.path.abspath(__file__))

# (name, family, split, global_rows, axis, world, partition_stride)
CASES = [
    ("qkv_tp2_whole_groups", "qkv", (8, 4, 4), 64, "tp", 2, 1),
    ("qkv_fs4_cut_groups", "qkv", (8, 4, 4), 96, "fs", 4, 1),
    ("qkv_fs3_uneven", "qkv", (8, 4, 4), 80, "fs", 3, 1),
    ("qkv_fs8_missing_member", "qkv", (8, 4, 4), 32, "fs", 8, 1),
    ("qkvg_tp2", "qkvg", (8, 8, 4, 4), 96, "tp", 2, 1),
    ("qkvg_fs3_cut", "qkvg", (8, 8, 4, 4), 72, "fs", 3, 1),
    ("linear_tp2_strided", "linear", (24, 24), 48, "tp", 2, 2),
    ("linear_tp4_strided", "linear", (20, 20), 40, "tp", 4, 2),
    ("linear_fs3_cut", "linear", (30, 30), 60, "fs", 3, 1),
    ("linear_tp2_plain", "linear", (16, 32), 48, "tp", 2, 1),
]


def main():
    os.environ.setdefault("DION_DISABLE_TORCH_COMPILE", "1")
    from megatron.core.optimizer.dion import linear as d_lin
    from megatron.core.optimizer.dion import qkv as d_qkv
    from megatron.core.optimizer.dion import qkvg as d_qkvg
    from megatron.core.optimizer.distrib_dion.sharding import compute_fs_shard_range

    out = {"cases": []}
    for name, family, split, rows, axis, world, stride in CASES:
        case = dict(name=name, family=family, split=list(split), global_rows=rows, axis=axis, world=world,
                    partition_stride=stride, members=[])
        kinds = {"qkv": d_qkv.QKV_CHILD_KINDS, "qkvg": d_qkvg.QKVG_CHILD_KINDS, "linear": ("gate", "up")}[family]
        case["kinds"] = list(kinds)
        if family == "linear":
            case["child_rows"] = {k: int(d_lin.linear_child_global_shape((rows, 8), tuple(split), k)[0]) for k in kinds}
        elif family == "qkv":
            case["child_rows"] = {k: int(d_qkv.qkv_child_global_shape((rows, 8), tuple(split), k)[0]) for k in kinds}
        else:
            case["child_rows"] = {k: int(d_qkvg.qkvg_child_global_shape((rows, 8), tuple(split), k)[0]) for k in kinds}
        for rank in range(world):
            a, b = compute_fs_shard_range(rows, world, rank)
            seg = {}
            for k in kinds:
                if family == "linear":
                    if axis == "tp":
                        meta = SimpleNamespace(tp_shard_dim=0, tp_world_size=world, tp_rank=rank,
                                               linear_partition_stride=stride, global_shape=(rows, 8),
                                               fs_shard_dim=1, fs_world_size=1)
                    else:
                        meta = SimpleNamespace(fs_shard_dim=0, fs_world_size=world, fs_rank=rank, fs_start_idx=a,
                                               fs_end_idx=b, tp_shard_dim=-1, tp_world_size=1,
                                               linear_partition_stride=1, global_shape=(rows, 8))
                    s = d_lin._linear_child_segments(local_rows=b - a, split_rows=tuple(split), dist_meta=meta,
                                                     child_kind=k, context="golden")
                else:
                    mod = d_qkv if family == "qkv" else d_qkvg
                    s = mod._child_segments(parent_row_start=a, parent_row_end=b, split_shapes=tuple(split),
                                            child_kind=k)
                seg[k] = [list(map(int, x)) for x in s]
            case["members"].append(dict(rank=rank, parent_range=[a, b], segments=seg))
        out["cases"].append(case)
    path = os.path.join(HERE, "split_layouts.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    sys.exit(main())
