"""Split-QKV and split-linear children for the stand-alone adapter.

The reference optimises a fused attention QKV weight as three Dion matrices (q, k, v)
and a fused SwiGLU linear_fc1 as two (gate, up) when `split_qkv` / `split_linear` are on
(`--dion-split-qkv`, used by examples/dion/speedrun_nanogpt_mcore.py:417):
  * dion/qkv.py: the fused rows are grouped per query group as [q | k | v] with
    `qkv_split_shapes` = (q, k, v) rows per group; child `kind` is the concatenation of
    its block of every group (_child_segments, :237-280), its global shape
    (split[kind] * groups, cols) (:314-327);
  * dion/qkvg.py: the gated-attention variant, groups of [q | gate | k | v] (four children);
  * dion/linear.py: rows [0, gate) are the gate child, [gate, gate + up) the up child
    (_direct_linear_rows, :140-155);
  * child identities: name `parent::kind`, uid (*parent_uid, ("qkv_child" | "qkvg_child" |
    "linear_child", kind)) (qkv.py:104-127, qkvg.py:118-141, linear.py:91-113), so each
    child has its own seeded Q, rank r and low-rank rule from its own global shape;
  * child state lives in the parent's state under `qkv_<kind>_<field>` /
    `linear_<kind>_<field>` (Q, r, local_shape, global_shape; qkv.py:98-101) beside
    `qkv_split_qkv` / `qkv_split_shapes` (`linear_split_linear` / `linear_split_rows`),
    the keys the reference's checkpoint code restores (checkpoint_io.py:351-369);
  * every step each child runs as its own DionStepParam on its rows of the parent's
    param, grad and momentum, and writes them back through `commit_update`
    (dion_distrib_optimizer.py:3450-3580; scatter_qkv_child_ is a no-op when the child is
    a view of the parent, qkv.py:472-500).
Children of one kind share a shape across layers, so they batch together as any other
matrices.  A single-segment child (split-linear, or qkv with one query group) is a view
of the parent and needs no copy; an interleaved qkv child is gathered into a contiguous
matrix and scattered back.  The commit hook turns the deferred error feedback off for
the children (their momentum may be a copy), which then take the eager schedule.
Whole-matrix parents only: FS- or TP-sharded parents are refused
([DION_SPLIT_SHARDED_PARENT]).
"""
from __future__ import annotations

from typing import Callable, List, Sequence, Tuple

import torch

QKV_CHILD_KINDS = ("q", "k", "v")
QKVG_CHILD_KINDS = ("q", "gate", "k", "v")
LINEAR_CHILD_KINDS = ("gate", "up")


def grouped_child_segments(rows: int, split_shapes: Sequence[int], kind: str,
                           kinds: Sequence[str] = QKV_CHILD_KINDS, tag: str = "QKV") -> List[Tuple[int, int]]:
    """Parent row ranges, in child-row order, of child `kind` of a grouped fused weight
    (qkv.py:237-280 / qkvg.py:267-300 for the parent range [0, rows))."""
    split = tuple(int(d) for d in split_shapes)
    if len(split) != len(kinds) or any(d <= 0 for d in split):
        raise RuntimeError(f"[DION_INVALID_{tag}_SPLIT_SHAPES] split_shapes={split}")
    total = sum(split)
    if rows <= 0 or rows % total:
        raise RuntimeError(f"[DION_{tag}_LOCAL_LAYOUT_MISMATCH] rows={rows} split_shapes={split}")
    idx = tuple(kinds).index(kind)
    off = sum(split[:idx])
    return [(g * total + off, g * total + off + split[idx]) for g in range(rows // total)]


def qkv_child_segments(rows: int, split_shapes: Sequence[int], kind: str) -> List[Tuple[int, int]]:
    return grouped_child_segments(rows, split_shapes, kind, QKV_CHILD_KINDS, "QKV")


def qkvg_child_segments(rows: int, split_shapes: Sequence[int], kind: str) -> List[Tuple[int, int]]:
    return grouped_child_segments(rows, split_shapes, kind, QKVG_CHILD_KINDS, "QKVG")


def linear_child_segments(rows: int, split_rows: Sequence[int], kind: str) -> List[Tuple[int, int]]:
    """linear.py:140-155: gate = rows [0, gate), up = rows [gate, gate + up)."""
    split = tuple(int(d) for d in split_rows)
    if len(split) != 2 or any(d <= 0 for d in split):
        raise RuntimeError(f"[DION_INVALID_LINEAR_SPLIT_ROWS] split_rows={split}")
    if rows != sum(split):
        raise RuntimeError(f"[DION_LINEAR_LOCAL_ROWS_MISMATCH] rows={rows} split_rows={split}")
    return [(0, split[0])] if kind == "gate" else [(split[0], rows)]


def merge_segments(segments: Sequence[Tuple[int, int]]) -> List[Tuple[int, int]]:
    out: List[Tuple[int, int]] = []
    for a, b in segments:
        if out and out[-1][1] == a:
            out[-1] = (out[-1][0], b)
        else:
            out.append((a, b))
    return out


def gather_rows(t: torch.Tensor, segments: Sequence[Tuple[int, int]]) -> torch.Tensor:
    """The child's rows of `t`: a view for one segment, else a contiguous copy."""
    segments = merge_segments(segments)
    if len(segments) == 1:
        a, b = segments[0]
        return t.narrow(0, a, b - a)
    return torch.cat([t.narrow(0, a, b - a) for a, b in segments], dim=0)


def scatter_rows_(dest: torch.Tensor, child: torch.Tensor, segments: Sequence[Tuple[int, int]]) -> None:
    """Write a gathered child back; a view of `dest` is already in place."""
    segments = merge_segments(segments)
    if len(segments) == 1 and child.data_ptr() == dest.narrow(0, segments[0][0], 1).data_ptr():
        return
    cur = 0
    for a, b in segments:
        dest.narrow(0, a, b - a).copy_(child.narrow(0, cur, b - a))
        cur += b - a


def child_uid(parent_uid, family: str, kind: str):
    tag = (f"{family}_child", kind)
    return (*parent_uid, tag) if isinstance(parent_uid, tuple) else (parent_uid, tag)


def state_key(family: str, field: str, kind: str) -> str:
    return f"{family}_{kind}_{field}"


def split_plan(param: torch.Tensor, defaults: dict):
    """(family, kinds, segments_of(kind), parent state flags) when `param` is split, else None."""
    rows = int(param.shape[0])
    # dion_distrib_optimizer.py:2020-2060: split_qkv covers QKVG (gated attention) first
    if defaults.get("split_qkv") and (getattr(param, "is_qkvg", False) or hasattr(param, "qkvg_split_shapes")):
        split = tuple(int(d) for d in getattr(param, "qkvg_split_shapes"))
        seg = {k: qkvg_child_segments(rows, split, k) for k in QKVG_CHILD_KINDS}
        return "qkvg", QKVG_CHILD_KINDS, seg, {"qkvg_split_qkvg": True, "qkvg_split_shapes": split}
    if defaults.get("split_qkv") and (getattr(param, "is_qkv", False) or hasattr(param, "qkv_split_shapes")):
        split = tuple(int(d) for d in getattr(param, "qkv_split_shapes"))
        seg = {k: qkv_child_segments(rows, split, k) for k in QKV_CHILD_KINDS}
        return "qkv", QKV_CHILD_KINDS, seg, {"qkv_split_qkv": True, "qkv_split_shapes": split}
    if defaults.get("split_linear") and getattr(param, "is_linear_fc1", False):
        split = tuple(int(d) for d in getattr(param, "linear_split_rows"))
        seg = {k: linear_child_segments(rows, split, k) for k in LINEAR_CHILD_KINDS}
        return "linear", LINEAR_CHILD_KINDS, seg, {"linear_split_linear": True, "linear_split_rows": split}
    return None


def make_commit(param: torch.Tensor, momentum: torch.Tensor,
                segments: Sequence[Tuple[int, int]]) -> Callable[[torch.Tensor, torch.Tensor], None]:
    def commit(updated_param, updated_momentum):
        scatter_rows_(param.data, updated_param, segments)
        scatter_rows_(momentum, updated_momentum, segments)
    return commit
