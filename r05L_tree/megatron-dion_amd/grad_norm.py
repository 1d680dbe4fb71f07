"""Dion term of the gradient norm, on device.

Megatron calls this before the step when gradient clipping is on.  The reference,
/root/reference/megatron/core/optimizer/distrib_dion/grad_norm.py:144-258
(`_dion_grad_norm_sq`), returns the fp64 sum of squares of the Dion gradients:
  * no replica group (or size 1): of the local gradients (:166-172);
  * replica group of size W > 1: of the gradients reduced across the replicas with the
    replicate op (AVG when `rp_average_in_collective`, else SUM; runtime.py:361-364).  It
    copies every Dion gradient into one flat buffer per dtype and ALL-REDUCES it
    (:214-233) -- a dense exchange of the whole gradient, which is exactly the traffic
    Dion's low-rank sync exists to avoid.  Local gradients are not modified.  With
    `count_dion_grad=False` the collective still runs and None is returned.

This module keeps the returned value and replaces the exchange:
  * mode="exact" (default): the same number with half the traffic and bounded memory.
    The gradients are packed, in `chunk_bytes` pieces (not one flat copy of the whole set:
    the reference's copy is 14 GB on Llama-3-8B), into a staging buffer that is
    REDUCE-SCATTERED with the replicate op: each rank receives 1/W of the reduced chunk,
    squares and sums it on device, and one all-reduce of the fp64 scalar (SUM) gives
    every rank the total.  Per rank that moves (W-1)/W of the gradient bytes instead of
    the all-reduce's 2 (W-1)/W, and nothing is all-gathered back.  The reduced values
    are those of the reference's all-reduce (same op, same dtype); the fp64 sum runs in
    a different order (per shard, then across shards), so the total agrees to fp64
    rounding, not bitwise.
  * mode="local_bound": no gradient traffic at all.  Returns mean_i ||G_i||^2 over the
    replicas (one scalar all-reduce), which bounds ||mean_i G_i||^2 from above (convexity
    of the square); under the SUM replicate op W sum_i ||G_i||^2, which bounds
    ||sum_i G_i||^2.  Clipping with it never clips less than the exact norm would.
    An opt-in deviation from the reference's number, for runs where the dense exchange
    costs more than the conservative clip.
The sum of squares runs in the HIP kernel `dion_grad_sum_sq` (fp64, exact squares,
fixed order), reading each gradient once in its own dtype: the reference's chunked
`.to(float64)` copies (:54-68) disappear.  Gradients of parameters without low-rank sync
(`dense_reuse`) are all-reduced in place instead and reused by the step (the reference's
dense-RP reduced-gradient cache, :161-211 and dion/dense_grad_cache.py).
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from .dense_grad_cache import can_reuse_dense_grad, lookup, mark_reduced

__all__ = ["dion_grad_norm_sq", "dion_grad_norm", "dense_reuse_flags", "as_matrices"]

_FLAT_COLS = 1 << 20
_CHUNK_BYTES = 256 << 20


def as_matrices(flat: torch.Tensor) -> List[torch.Tensor]:
    """A 1-D buffer as row-major matrices whose m, n fit the C ABI's int32 fields."""
    n = int(flat.numel())
    if n == 0:
        return []
    if n <= _FLAT_COLS:
        return [flat.view(1, n)]
    rows = n // _FLAT_COLS
    out = [flat[: rows * _FLAT_COLS].view(rows, _FLAT_COLS)]
    if n > rows * _FLAT_COLS:
        out.append(flat[rows * _FLAT_COLS:].view(1, n - rows * _FLAT_COLS))
    return out


def _abi_views(g: torch.Tensor) -> List[torch.Tensor]:
    """A gradient as matrices the kernel accepts: 2-D row-major ones as they are (n fits
    int32), anything else through its flat view (non-2D or very wide grads
    would overflow the descriptor's int32 n)."""
    if g.dim() == 2 and g.stride(1) == 1 and g.shape[1] <= _FLAT_COLS:
        return [g]
    return as_matrices(g.detach().reshape(-1))


def _replicate_op(optimizer):
    avg = bool(getattr(optimizer, "defaults", {}).get("rp_average_in_collective", True))
    return dist.ReduceOp.AVG if avg else dist.ReduceOp.SUM


def _local_sum_sq(codec, grads, device) -> torch.Tensor:
    total = torch.zeros(1, dtype=torch.float64, device=device)
    mats = [m for g in grads for m in _abi_views(g)]
    if mats:
        codec.grad_sum_sq(mats, total)
    return total


def _reduced_sum_sq(codec, members, op, group, world, device, dtype, chunk_bytes) -> torch.Tensor:
    """fp64 sum of squares of the replica-reduced `members` (one dtype), by chunked
    reduce-scatter; this rank's partial (the caller sums the partials over the group)."""
    total = torch.zeros(1, dtype=torch.float64, device=device)
    esize = torch.empty((), dtype=dtype).element_size()
    cap = max(world, (max(chunk_bytes // esize, world) // world) * world)
    numel = sum(int(g.numel()) for g in members)
    staging = torch.empty(min(cap, -(-numel // world) * world), dtype=dtype, device=device)
    fill = 0

    def flush(n):
        if n == 0:
            return
        padded = -(-n // world) * world
        if padded > n:
            staging[n:padded].zero_()  # zeros reduce to zeros and add nothing
        shard = torch.empty(padded // world, dtype=dtype, device=device)
        dist.reduce_scatter_tensor(shard, staging[:padded], op=op, group=group)
        codec.grad_sum_sq(as_matrices(shard), total)

    for g in members:
        flat = g.detach().reshape(-1)
        pos = 0
        while pos < flat.numel():
            take = min(int(flat.numel()) - pos, staging.numel() - fill)
            staging[fill:fill + take].copy_(flat[pos:pos + take])
            fill += take
            pos += take
            if fill == staging.numel():
                flush(fill)
                fill = 0
    flush(fill)
    return total


def _reduce_dense_in_place(optimizer, codec, grads, op, group, device) -> torch.Tensor:
    """grad_norm.py:174-258 for the dense-reuse gradients: all-reduce each in place (once per
    step: one already reduced by this step's norm is taken as it is), mark it for the step
    (dense_grad_cache), and return the fp64 sum of squares of the reduced values (the same
    on every rank)."""
    before = int(getattr(optimizer, "_step_count", 0))
    todo = []
    for g in grads:
        state, _ = lookup(optimizer, g, group=group, op=op, before_step=before)
        if state == "mismatch":
            raise RuntimeError(f"[DION_DENSE_RP_GRAD_CACHE_MISMATCH] grad {tuple(g.shape)} was reduced with another "
                               "replicate group or op")
        if state == "missing":
            todo.append(g)
    works = []
    for g in todo:
        works.append((g, None, dist.all_reduce(g, op=op, group=group, async_op=True)) if g.is_contiguous() else
                     (g, (c := g.contiguous()), dist.all_reduce(c, op=op, group=group, async_op=True)))
    for g, c, w in works:
        w.wait()
        if c is not None:
            g.copy_(c)
        mark_reduced(optimizer, g, group=group, op=op, before_step=before)
    return _local_sum_sq(codec, grads, device)


def dion_grad_norm_sq(optimizer, grads: Sequence[torch.Tensor], *, count_dion_grad: bool = True,
                      replica_group=None, mode: str = "exact", chunk_bytes: int = _CHUNK_BYTES,
                      dense_reuse: Optional[Sequence[bool]] = None) -> Optional[torch.Tensor]:
    """Sum of squares (fp64, shape (1,), on the gradients' device) of the Dion gradients
    (of their replica reduction when `replica_group` has more than one rank).

    `dense_reuse[i]` (distrib_dion/grad_norm.py:37-52, `can_reuse_dense_grad`): gradient i
    belongs to a parameter without low-rank sync, whose step all-reduces it anyway.  It is
    all-reduced here in place, once, and the step reuses it (dense_grad_cache): one exchange
    per step for those gradients (the reference's flow)."""
    if mode not in ("exact", "local_bound"):
        raise RuntimeError(f"[DION_INVALID_GRAD_NORM_MODE] mode={mode!r}")
    flags = list(dense_reuse) if dense_reuse is not None else [False] * len(grads)
    if len(flags) != len(grads):
        raise RuntimeError(f"[DION_GRAD_NORM_REUSE_FLAGS] {len(flags)} flags for {len(grads)} gradients")
    keep = [i for i, g in enumerate(grads) if g is not None]
    grads, flags = [grads[i] for i in keep], [bool(flags[i]) for i in keep]
    if not grads:
        return None
    codec = optimizer.codec
    world = dist.get_world_size(replica_group) if (replica_group is not None and dist.is_initialized()) else 1
    dev = grads[0].device
    if world <= 1:
        return _local_sum_sq(codec, grads, dev) if count_dion_grad else None
    op = _replicate_op(optimizer)
    dense = [g for g, f in zip(grads, flags) if f]
    grads = [g for g, f in zip(grads, flags) if not f]
    dense_sq = _reduce_dense_in_place(optimizer, codec, dense, op, replica_group, dev) if dense else None
    total = torch.zeros(1, dtype=torch.float64, device=dev)
    if mode == "local_bound":
        if grads:
            total = _local_sum_sq(codec, grads, dev)
        dist.all_reduce(total, op=dist.ReduceOp.SUM, group=replica_group)
        # ||mean_i G_i||^2 <= mean_i ||G_i||^2 (AVG);  ||sum_i G_i||^2 <= W sum_i ||G_i||^2 (SUM)
        if op == dist.ReduceOp.SUM:
            total *= world
        else:
            total /= world
    else:
        groups = {}
        for g in grads:
            groups.setdefault((g.dtype, g.device), []).append(g)
        for (dtype, device), members in groups.items():
            if sum(int(g.numel()) for g in members) <= 0:
                continue
            total += _reduced_sum_sq(codec, members, op, replica_group, world, device, dtype,
                                     int(chunk_bytes)).to(dev)
        dist.all_reduce(total, op=dist.ReduceOp.SUM, group=replica_group)
    if dense_sq is not None:
        total += dense_sq  # every rank holds the same reduced dense gradients
    return total if count_dion_grad else None


def dense_reuse_flags(optimizer, params: Sequence[torch.Tensor]) -> List[bool]:
    """`dense_reuse` for dion_grad_norm_sq from the adapter's per-parameter metadata
    (`optimizer.dist_metas`, as distrib_dion/grad_norm.py:27-34 looks it up)."""
    metas = getattr(optimizer, "dist_metas", None) or {}
    return [can_reuse_dense_grad(metas.get(p)) for p in params]


def dion_grad_norm(optimizer, grads: Sequence[torch.Tensor], **kwargs) -> float:
    """sqrt of dion_grad_norm_sq (host sync), 0.0 without gradients."""
    sq = dion_grad_norm_sq(optimizer, grads, **kwargs)
    return 0.0 if sq is None else math.sqrt(float(sq.item()))
