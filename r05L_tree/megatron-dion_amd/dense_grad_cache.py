"""Reuse of replica-reduced dense gradients between the grad norm and the step.

A Dion parameter without low-rank sync is exchanged densely across the replicas: the
step all-reduces its gradient (dion/runtime.py:439-491).  With clipping on, the grad-norm
term has to reduce the same gradient first (distrib_dion/grad_norm.py:144-258), so the
reference records the reduction (/root/reference/megatron/core/optimizer/dion/
dense_grad_cache.py:44-147): the norm all-reduces the gradient IN PLACE and marks its
storage region as reduced "before step t" (t = the optimizer's step count at that
moment); the step (which has already counted itself, so it looks for t = step - 1) skips
its all-reduce when every gradient of the batch is inside a marked region, and consumes
the marks.  One exchange per step instead of two.

The record lives on the optimizer (attribute `_dion_dense_grad_reduction_cache`):
  {"entries": [{"ptr", "start", "end", "dtype", "device", "group", "op", "before_step"}]}
Lookups answer "match" (a mark for this region, step, group and op), "mismatch" (a mark
that covers the region but for another group / op: an error, the gradient was reduced
differently) or "missing".  Stale marks (another step) are dropped on lookup.

A mark says nothing about the bytes: if the step is skipped after the norm (an AMP loss
scaler finding an inf) and the next iteration's gradients land in the same storage, a mark
keyed on (storage, region, step) would still "match" and the new gradients would never be
exchanged.  `invalidate` drops every mark; `MegatronDion.zero_grad()` calls it, and a
caller that skips a step without zeroing through the optimizer calls it itself.  (Megatron's
own loop cannot hit this: it checks for infs before the norm and returns without one.)
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch

CACHE_ATTR = "_dion_dense_grad_reduction_cache"


def storage_span(t: torch.Tensor) -> Optional[Tuple[int, int, int]]:
    """(storage pointer, first element, one past the last element) a tensor touches."""
    if int(t.numel()) <= 0:
        return None
    lo = hi = int(t.storage_offset())
    for size, stride in zip(t.shape, t.stride()):
        reach = (int(size) - 1) * int(stride)
        if reach < 0:
            lo += reach
        else:
            hi += reach
    return int(t.untyped_storage().data_ptr()), lo, hi + 1


def _entries(owner, before_step: int, create: bool) -> Optional[List[dict]]:
    cache = getattr(owner, CACHE_ATTR, None)
    if cache is None:
        if not create:
            return None
        cache = {"entries": []}
        setattr(owner, CACHE_ATTR, cache)
    cache["entries"] = [e for e in cache["entries"] if e["before_step"] == int(before_step)]
    return cache["entries"]


def _covers(e: dict, t: torch.Tensor, span) -> bool:
    return (e["ptr"] == span[0] and e["dtype"] == t.dtype and e["device"] == t.device
            and e["start"] <= span[1] and span[2] <= e["end"])


def lookup(owner, t: torch.Tensor, *, group, op, before_step: int) -> Tuple[str, Optional[int]]:
    """("match" | "mismatch" | "missing", index of the matching mark)."""
    entries = _entries(owner, before_step, create=False)
    span = storage_span(t)
    if not entries or span is None:
        return "missing", None
    state = "missing"
    for i, e in enumerate(entries):
        if not _covers(e, t, span):
            continue
        if e["group"] is group and e["op"] == op:
            return "match", i
        state = "mismatch"
    return state, None


def mark_reduced(owner, t: torch.Tensor, *, group, op, before_step: int) -> None:
    """Record that `t` now holds its replica reduction (op over group) for step before_step + 1."""
    span = storage_span(t)
    if span is None:
        return
    _entries(owner, before_step, create=True).append(
        dict(ptr=span[0], start=span[1], end=span[2], dtype=t.dtype, device=t.device, group=group, op=op,
             before_step=int(before_step)))


def consume_if_reduced(owner, grads: Sequence[torch.Tensor], *, group, op) -> bool:
    """The step's check (dion/runtime.py:387-435): True (and the marks consumed) when every
    gradient was reduced by the grad norm of this step; False when none was; an error when
    only some were or one was reduced with another group / op."""
    if not grads:
        return False
    before = int(getattr(owner, "_step_count", 0)) - 1
    if not _entries(owner, before, create=False):
        if getattr(owner, CACHE_ATTR, None) is not None:
            delattr(owner, CACHE_ATTR)  # nothing (left) for this step
        return False
    hits, missing = [], False
    for g in grads:
        state, idx = lookup(owner, g, group=group, op=op, before_step=before)
        if state == "mismatch":
            raise RuntimeError(f"[DION_DENSE_RP_GRAD_CACHE_MISMATCH] step={getattr(owner, '_step_count', 0)} "
                               f"grad {tuple(g.shape)} was reduced with another replicate group or op")
        if state == "match":
            hits.append(idx)
        else:
            missing = True
    if missing:
        if hits:
            raise RuntimeError(f"[DION_DENSE_RP_GRAD_CACHE_PARTIAL] step={getattr(owner, '_step_count', 0)}: "
                               f"{len(hits)} of {len(grads)} gradients of the batch were reduced by the grad norm")
        return False
    cache = getattr(owner, CACHE_ATTR)
    keep = set(range(len(cache["entries"]))) - set(hits)
    cache["entries"] = [e for i, e in enumerate(cache["entries"]) if i in keep]
    if not cache["entries"]:
        delattr(owner, CACHE_ATTR)
    return True


def invalidate(owner) -> None:
    """Forget every reduction mark (gradients repopulated or a step skipped after the norm)."""
    if getattr(owner, CACHE_ATTR, None) is not None:
        delattr(owner, CACHE_ATTR)


def can_reuse_dense_grad(dist_meta) -> bool:
    """distrib_dion/grad_norm.py:37-52: a whole (not split) Dion parameter without low-rank sync."""
    if dist_meta is None:
        return False
    for attr in ("qkv_split_shapes", "qkvg_split_shapes", "linear_split_rows"):
        if getattr(dist_meta, attr, None) is not None:
            return False
    if "::" in str(getattr(dist_meta, "param_name", "") or ""):  # a split child (split.py)
        return False
    cfg = getattr(dist_meta, "param_config", None)
    return cfg is not None and not bool(getattr(cfg, "use_low_rank_sync", False))
