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
Sharded parents (the speedrun's FS x TP topology: TP on the rows, FS on the columns; or FS on
the rows) give each rank the children's rows inside its parent shard (split_child_layouts).
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

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


def grouped_child_segments_in_range(start: int, end: int, split_shapes: Sequence[int], kind: str,
                                    kinds: Sequence[str] = QKV_CHILD_KINDS,
                                    tag: str = "QKV") -> List[Tuple[int, int, int, int]]:
    """qkv.py:247-285 / qkvg.py (_child_segments): the parent's global row interval
    [start, end) (a row shard) mapped to (source_start, source_end, child_start, child_end)
    intervals, sources relative to `start`, child rows in the child's global coordinates."""
    split = tuple(int(d) for d in split_shapes)
    if len(split) != len(kinds) or any(d <= 0 for d in split):
        raise RuntimeError(f"[DION_INVALID_{tag}_SPLIT_SHAPES] split_shapes={split}")
    if start < 0 or end <= start:
        return []
    total = sum(split)
    idx = tuple(kinds).index(kind)
    per, off = split[idx], sum(split[:idx])
    out: List[Tuple[int, int, int, int]] = []
    for grp in range(start // total, (end - 1) // total + 1):
        c0 = grp * total + off
        a, b = max(start, c0), min(end, c0 + per)
        if b <= a:
            continue
        child_start = grp * per + (a - c0)
        if out and out[-1][3] != child_start:
            raise RuntimeError(f"[DION_{tag}_CHILD_NONCONTIGUOUS_LOCAL_RANGE] child_kind={kind} "
                               f"parent_row_range=({start}, {end})")
        out.append((a - start, b - start, child_start, child_start + (b - a)))
    return out


def linear_child_segments_in_range(start: int, end: int, split_rows: Sequence[int], kind: str, *,
                                   tp: Optional[Tuple[int, int]] = None,
                                   partition_stride: int = 1) -> List[Tuple[int, int, int, int]]:
    """linear.py:235-319 (_linear_child_segments).  `tp = (tp_world, tp_rank)` with
    `partition_stride` 2 is Megatron's strided SwiGLU TP shard: the local rows are
    [gate share | up share], each child's share its split_range of the child's rows; otherwise
    the parent's global row interval [start, end) is intersected with the child's rows."""
    split = tuple(int(d) for d in split_rows)
    idx = LINEAR_CHILD_KINDS.index(kind)
    if tp is not None and int(tp[0]) > 1:
        world, rank = int(tp[0]), int(tp[1])
        if partition_stride == len(split):
            out, cur = [], 0
            for si, rows in enumerate(split):
                a, b = _split_range(rows, world, rank)
                if si == idx and b > a:
                    out.append((cur, cur + b - a, a, b))
                cur += b - a
            if cur != end - start:
                raise RuntimeError(f"[DION_LINEAR_STRIDED_TP_LOCAL_ROWS_MISMATCH] local_rows={end - start} "
                                   f"expected_rows={cur} tp_world_size={world} tp_rank={rank} split_rows={split}")
            return out
        if partition_stride != 1:
            raise RuntimeError(f"[DION_LINEAR_UNSUPPORTED_TP_PARTITION_STRIDE] partition_stride={partition_stride} "
                               f"split_rows={split}")
    if start < 0:
        return []
    c0 = 0 if idx == 0 else split[0]
    a, b = max(start, c0), min(end, c0 + split[idx])
    if b <= a:
        return []
    return [(a - start, b - start, a - c0, b - c0)]


def _split_range(size: int, world: int, rank: int) -> Tuple[int, int]:
    base, rem = size // world, size % world
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


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


def split_plan(param: torch.Tensor, defaults: dict, global_rows: Optional[int] = None):
    """(family, kinds, segments_of(kind) over the global rows, parent state flags) when
    `param` is split, else None.  `global_rows`: the parent's global row count when `param`
    is a shard (default: its own rows)."""
    rows = int(param.shape[0]) if global_rows is None else int(global_rows)
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


def split_child_layouts(param: torch.Tensor, plan, *, fs_spec=None, tp_spec=None, fs_world: int = 1,
                        fs_rank: int = 0, tp_world: int = 1, tp_rank: int = 0) -> dict:
    """Per child kind: this rank's rows of the child and its FS / TP shard specs.

    `param` is the whole fused matrix or this rank's shard of it: `fs_spec` / `tp_spec` =
    (global_shape, shard_dim, start, end) as attach_dp_routing takes them.  The rows are
    sharded by TP when tp_shard_dim is 0, else by FS when fs_shard_dim is 0 (qkv.py:194-244,
    linear.py:176-228); each member's parent row range maps to child rows through
    `_child_segments` (qkv.py:247-285; linear.py:235-319 with Megatron's strided SwiGLU TP
    shard, `partition_stride` 2), and the child is sharded over the same group with those
    child rows (resolve_row_child_layout, distrib_dion/row_child.py:30-117; uneven members
    give explicit row sizes, split_child.py:10-52).  The columns keep the parent's shard.  A
    child whose rows miss members of the group is owned by the members that hold some of its
    rows (row_child.py:62-106): it is sharded over their sub-group (the caller builds it from
    `members`, row_child.py:94-101), a single owner holds it whole (no row shard, world 1), and
    a rank outside `members` has no rows of it (local_rows 0, no step param, :105-106).

    Returns {kind: dict(local_rows, segments (local source rows), fs, tp (child specs or
    None), row_sizes (every owner's child rows, or None), row_axis ("tp" | "fs" | None),
    members (indices in the parent's row group of the child's owners), child_rank (this rank's
    index among them, -1 outside), child_world)}."""
    family, kinds, _, flags = plan
    split = tuple(flags[f"{family}_split_shapes"] if family != "linear" else flags["linear_split_rows"])
    local_rows = int(param.shape[0])
    gshape = tuple(int(d) for d in (tp_spec or fs_spec)[0]) if (tp_spec or fs_spec) is not None else \
        (local_rows, int(param.shape[1]))
    gm = gshape[0]
    row_axis = None
    if tp_spec is not None and int(tp_spec[1]) == 0 and tp_world > 1:
        row_axis = "tp"
        ranges = [_split_range(gm, tp_world, k) for k in range(tp_world)]
        me = tp_rank
        if (int(tp_spec[2]), int(tp_spec[3])) != ranges[me]:
            raise RuntimeError(f"[DION_{family.upper()}_LOCAL_ROW_RANGE_MISMATCH] local_rows={local_rows} "
                               f"parent_row_range={ranges[me]} tp_spec=({tp_spec[2]}, {tp_spec[3]})")
    elif fs_spec is not None and int(fs_spec[1]) == 0 and fs_world > 1:
        row_axis = "fs"  # the members' canonical FS ranges (compute_fs_shard_range, sharding.py:44-61)
        ranges = [_split_range(gm, fs_world, k) for k in range(fs_world)]
        me = fs_rank
        if (int(fs_spec[2]), int(fs_spec[3])) != ranges[me]:
            raise RuntimeError(f"[DION_{family.upper()}_MISSING_FS_RANGE] fs_spec=({fs_spec[2]}, {fs_spec[3]}) is "
                               f"not the canonical FS range {ranges[me]}")
    else:
        ranges, me = [(0, gm)], 0
    if ranges[me][1] - ranges[me][0] != local_rows:
        raise RuntimeError(f"[DION_{family.upper()}_LOCAL_ROW_RANGE_MISMATCH] local_rows={local_rows} "
                           f"parent_row_range={ranges[me]}")
    stride = int(getattr(param, "partition_stride", 1))
    kinds_all = {"qkv": QKV_CHILD_KINDS, "qkvg": QKVG_CHILD_KINDS}.get(family)
    out = {}
    for kind in kinds:
        per = []
        for k, (a, b) in enumerate(ranges):
            if family == "linear":
                per.append(linear_child_segments_in_range(a, b, split, kind, partition_stride=stride,
                                                          tp=(tp_world, k) if row_axis == "tp" else None))
            else:
                per.append(grouped_child_segments_in_range(a, b, split, kind, kinds_all, family.upper()))
        members = tuple(k for k, s in enumerate(per) if s)
        if not members:
            raise RuntimeError(f"[DION_{family.upper()}_NO_{(row_axis or 'ROW').upper()}_OWNERS] child {kind}")
        child_ranges = [(per[k][0][2], per[k][-1][3]) for k in members]
        child_rows = (split[LINEAR_CHILD_KINDS.index(kind)] if family == "linear"
                      else split[kinds_all.index(kind)] * (gm // sum(split)))
        if child_ranges[0][0] != 0 or child_ranges[-1][1] != child_rows or any(
                x[1] != y[0] for x, y in zip(child_ranges, child_ranges[1:])):
            raise RuntimeError(f"[DION_{family.upper()}_{(row_axis or 'ROW').upper()}_COVERAGE_MISMATCH] child {kind} "
                               f"child_global_rows={child_rows} member_ranges={child_ranges}")
        sizes = None if row_axis is None else tuple(b - a for a, b in child_ranges)
        if me not in members:
            out[kind] = dict(local_rows=0, segments=[], fs=None, tp=None, row_sizes=sizes, row_axis=row_axis,
                             members=members, child_rank=-1, child_world=len(members))
            continue
        crank = members.index(me)
        c0, c1 = child_ranges[crank]
        cg = (child_rows, gshape[1])
        # a single owner holds the child whole: no shard on the row axis (row_child.py:102, world 1)
        sharded = len(members) > 1
        fs = tp = None
        if fs_spec is not None:
            if int(fs_spec[1]) != 0:
                fs = (cg, 1, int(fs_spec[2]), int(fs_spec[3]))
            elif sharded or row_axis != "fs":
                fs = (cg, 0, c0, c1)
        if tp_spec is not None:
            if int(tp_spec[1]) != 0:
                tp = (cg, 1, int(tp_spec[2]), int(tp_spec[3]))
            elif sharded or row_axis != "tp":
                tp = (cg, 0, c0, c1)
        out[kind] = dict(local_rows=c1 - c0, segments=[(a, b) for a, b, _, _ in per[me]], fs=fs, tp=tp,
                         row_sizes=sizes if sharded else None, row_axis=row_axis if sharded else None,
                         members=members, child_rank=crank, child_world=len(members))
    return out


def make_commit(param: torch.Tensor, momentum: torch.Tensor,
                segments: Sequence[Tuple[int, int]]) -> Callable[[torch.Tensor, torch.Tensor], None]:
    def commit(updated_param, updated_momentum):
        scatter_rows_(param.data, updated_param, segments)
        scatter_rows_(momentum, updated_momentum, segments)
    return commit
