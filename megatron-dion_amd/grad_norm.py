"""Dion term of the gradient norm, on device.

Mirrors /root/reference/megatron/core/optimizer/distrib_dion/grad_norm.py:144-258
(`_dion_grad_norm_sq`), which Megatron calls before the step when gradient
clipping is on:
  * no replica group (or size 1): the fp64 sum of squares of the local Dion
    gradients (:166-172);
  * replica group of size W > 1: the gradients are copied into one flat buffer per
    dtype, all-reduced across the replicas with the replicate op (AVG when
    `rp_average_in_collective`, else SUM; runtime.py:361-364) and the sum of squares
    of the reduced buffer is taken (:214-233).  The local gradients are not modified.
    With `count_dion_grad=False` the all-reduce still runs and None is returned.
The sum of squares runs in the HIP kernel `dion_grad_sum_sq` (fp64, exact squares,
fixed order), reading each gradient once in its own dtype: the reference's chunked
`.to(float64)` copies (:54-68) disappear.  The reference's dense-RP reduced-gradient
cache (:161-211, only for parameters without low-rank sync) is outside this path.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

__all__ = ["dion_grad_norm_sq", "dion_grad_norm", "as_matrices"]

_FLAT_COLS = 1 << 20


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


def _replicate_op(optimizer):
    avg = bool(getattr(optimizer, "defaults", {}).get("rp_average_in_collective", True))
    return dist.ReduceOp.AVG if avg else dist.ReduceOp.SUM


def dion_grad_norm_sq(optimizer, grads: Sequence[torch.Tensor], *, count_dion_grad: bool = True,
                      replica_group=None) -> Optional[torch.Tensor]:
    """Sum of squares (fp64, shape (1,), on the gradients' device) of the Dion gradients."""
    grads = [g for g in grads if g is not None]
    if not grads:
        return None
    codec = optimizer.codec
    world = dist.get_world_size(replica_group) if (replica_group is not None and dist.is_initialized()) else 1
    dev = grads[0].device
    if world <= 1:
        if not count_dion_grad:
            return None
        total = torch.zeros(1, dtype=torch.float64, device=dev)
        codec.grad_sum_sq([g if g.dim() == 2 else g.reshape(1, -1) for g in grads], total)
        return total
    groups = {}
    for g in grads:
        groups.setdefault((g.dtype, g.device), []).append(g)
    total = None
    for (dtype, device), members in groups.items():
        numel = sum(int(g.numel()) for g in members)
        if numel <= 0:
            continue
        flat = torch.empty(numel, dtype=dtype, device=device)
        cursor = 0
        for g in members:
            flat[cursor:cursor + g.numel()].copy_(g.detach().reshape(-1))
            cursor += g.numel()
        dist.all_reduce(flat, op=_replicate_op(optimizer), group=replica_group)
        if count_dion_grad:
            if total is None:
                total = torch.zeros(1, dtype=torch.float64, device=device)
            codec.grad_sum_sq(as_matrices(flat), total)
    return total if count_dion_grad else None


def dion_grad_norm(optimizer, grads: Sequence[torch.Tensor], **kwargs) -> float:
    """sqrt of dion_grad_norm_sq (host sync), 0.0 without gradients."""
    sq = dion_grad_norm_sq(optimizer, grads, **kwargs)
    return 0.0 if sq is None else math.sqrt(float(sq.item()))
