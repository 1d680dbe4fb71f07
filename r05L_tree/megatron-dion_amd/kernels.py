"""Scalar helpers of the Dion step that stay on the host.

`scaled_lr_for_shape` restates dion/kernels.py:25-51 (the spectral mode has no
rank_fraction term; SURVEY.md 0.10 explains why the implementation, not the
contradicting unit test, is followed).
"""
from __future__ import annotations

import math


def scaled_lr_for_shape(*, lr: float, m_global: int, n_global: int, scale_mode: str,
                        rank_fraction: float, extra_scale_factor: float = 0.2) -> float:
    if m_global <= 0 or n_global <= 0:
        raise RuntimeError(f"[DION_INVALID_SCALE_SHAPE] m_global={m_global} n_global={n_global}")
    if rank_fraction <= 0.0:
        raise RuntimeError(f"[DION_INVALID_RANK_FRACTION] rank_fraction={rank_fraction}")
    if scale_mode == "spectral":
        return lr * extra_scale_factor * math.sqrt(float(max(m_global, n_global)))
    per_rank = extra_scale_factor / math.sqrt(float(rank_fraction))
    if scale_mode == "unit_rms_norm":
        return lr * per_rank * math.sqrt(float(m_global) / float(n_global))
    if scale_mode == "shape_scaling":
        return lr * per_rank * math.sqrt(max(1.0, float(m_global) / float(n_global)))
    raise RuntimeError(f"[DION_INVALID_SCALE_MODE] scale_mode={scale_mode!r}")
