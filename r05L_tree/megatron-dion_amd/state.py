"""Per-matrix Dion state rules: rank, orientation, low-rank sync, Q initialisation.

Integer rules are bit-exact restatements of the reference:
  rank rule            dion/state.py:179-188 (resolve_q_state_layout)
  low-rank sync rule   dion/state.py:220-230 (should_use_low_rank_sync)
  orientation rule     dion/state.py:304-310 (is_transposed = m < n, no TP/FS)
  Q-init seed          dion/state.py:233-260 (blake2b of the param key)
  Q-init values        dion/state.py:50-109 (CPU: one torch.randn of the global shape;
                       device: per-row Philox offsets, init_q)
State layout follows dion/state.py:527-654: momentum = zeros like the param
(m x n), Q = (n_Q x r), r, local_shape, global_shape.
"""
from __future__ import annotations

import hashlib
import math
from typing import Optional, Tuple

import torch

from .types import DionParamConfig


def rank_for_shape(m: int, n: int, rank_fraction: float, rank_multiple_of: int = 1) -> int:
    """r = max(1, int(min(mult * ceil(rf * min(m, n) / mult), m, n)))."""
    r = rank_fraction * min(m, n)
    r = rank_multiple_of * math.ceil(r / rank_multiple_of)
    r = min(r, m, n)
    return max(1, int(r))


def should_use_low_rank_sync(*, global_shape: Tuple[int, int], r_global: int, rank_fraction: float) -> bool:
    """Compressed exchange only when (m + n) r < m n and rank_fraction < 1."""
    m, n = int(global_shape[0]), int(global_shape[1])
    if rank_fraction >= 1.0:
        return False
    return (m + n) * int(r_global) < m * n


def is_transposed_shape(m: int, n: int) -> bool:
    """Orientation: P is taken over the longer side (m < n => work on M^T)."""
    return int(m) < int(n)


def q_seed_from_param_key(*, base_seed: int, param_uid, param_name: str,
                          q_global_shape: Tuple[int, int], is_transposed: bool) -> int:
    """63-bit seed of blake2b(repr(key)), topology-invariant like the reference."""
    if param_uid is None and not param_name:
        raise RuntimeError("[DION_Q_INIT_SEED_ID_MISSING] Dion Q init requires param_uid or param_name")
    key = repr(("dion_q_init", int(base_seed), param_uid if param_uid is not None else param_name,
                tuple(int(d) for d in q_global_shape), bool(is_transposed))).encode("utf-8")
    return int.from_bytes(hashlib.blake2b(key, digest_size=8).digest(), "little") & ((1 << 63) - 1)


def init_q(q_global_shape: Tuple[int, int], seed: int, device, dtype=torch.float32,
           rows: Optional[Tuple[int, int]] = None, cols: Optional[Tuple[int, int]] = None) -> torch.Tensor:
    """Rows [rows[0], rows[1]) and columns [cols[0], cols[1]) (default: all; columns are a TP
    rank's share of r) of the seeded Q0 ~ N(0, 1) of the global shape,
    drawn the way the reference draws on that device (dion/state.py:50-109,
    _normal_q_submatrix):
      * CPU: one torch.randn of the full global shape on a CPU generator, then the rows
        (state.py:94-96);
      * CUDA/HIP: every row from the device generator's Philox stream at the offset of the
        row's first element rounded down to a multiple of 4, dropping the rounding prefix
        (state.py:97-108), so any shard's rows are the full draw's rows.
    Draws are made in `dtype` itself, as the reference does.  Pinned by the reference's
    CPU captures (tests/test_host.py); the device stream is the same torch calls on the
    same torch build, checked for shard consistency on the GPU (tests/test_gpu_parity.py)."""
    q_rows, ncols = (int(d) for d in q_global_shape)
    r0, r1 = (0, q_rows) if rows is None else (int(rows[0]), int(rows[1]))
    c0, c1 = (0, ncols) if cols is None else (int(cols[0]), int(cols[1]))
    device = torch.device(device)
    if device.type == "cpu":
        gen = torch.Generator(device="cpu")
        gen.manual_seed(int(seed))
        q = torch.randn((q_rows, ncols), generator=gen, dtype=dtype)
        return q[r0:r1, c0:c1].contiguous()
    gen = torch.Generator(device=device)
    gen.manual_seed(int(seed))
    q = torch.empty((r1 - r0, c1 - c0), device=device, dtype=dtype)
    for i, row in enumerate(range(r0, r1)):
        first = row * ncols + c0
        base = first - first % 4
        gen.set_offset(base)
        draw = torch.empty(first - base + (c1 - c0), device=device, dtype=dtype)
        draw.normal_(0.0, 1.0, generator=gen)
        q[i].copy_(draw[first - base:])
    return q


def init_dion_state(param: torch.Tensor, *, rank_fraction: float, rank_multiple_of: int = 1,
                    base_seed: int = 0, param_uid=None, param_name: str = "",
                    momentum_dtype: Optional[torch.dtype] = None, q_dtype: Optional[torch.dtype] = None,
                    use_low_rank_sync: bool = True, fs_shard=None, tp_shard=None,
                    with_momentum: bool = True, q_stream: str = "device") -> Tuple[dict, DionParamConfig]:
    """Fresh optimizer state + config for one 2D parameter (no TP sharding).

    `param` is the whole matrix, or with `fs_shard = (global_shape, fs_shard_dim, start, end,
    fs_world)` this rank's FS shard of it (rows [start, end) for dim 0, columns for dim 1;
    distrib_dion/parameter.py:424-466).  The rank r and the low-rank rule use the global shape
    (state.py:159-230); the orientation follows the shard dim (dim 0 -> transposed, dim 1 ->
    not, state.py:304-310) so the sharded dim is always the contraction side of P = X Q; Q is
    the seeded global Q's rows [start, end), drawn on the parameter's device (init_q).
    `momentum_dtype` / `q_dtype` follow DionMixedPrecisionConfig (dion/state.py:502-514,
    544-547): None keeps the parameter's dtype; the speedrun sets both to bf16.

    `tp_shard = (global_shape, tp_shard_dim, start, end, tp_world, tp_rank)`: this rank's TP
    shard (rows for dim 0, columns for dim 1).  TP takes the P-row side (dim 0 -> not
    transposed, dim 1 -> transposed, state.py:304-310), Q keeps its rows and this rank's
    columns of r (resolve_q_state_layout, state.py:159-217: split_range(r, tp, rank)).

    Both (the speedrun's FS x TP topology): FS shards the other dim (get_fs_split_dim,
    distrib_dion/sharding.py:64-70), i.e. the contraction side of P; `param` is then the
    (TP rows x FS columns) block for TP dim 0 and Q holds the FS rows [start, end) of this
    rank's TP columns ("shard(0)", "shard(1)", state.py:203-206)."""
    if param.dim() != 2:
        raise RuntimeError(f"[DION_NOT_2D] shape={tuple(param.shape)}")
    ml, nl = (int(d) for d in param.shape)
    if tp_shard is not None:
        (m, n), dim, start, end, tp_world, tp_rank = tp_shard
        m, n, dim, tp_world, tp_rank = int(m), int(n), int(dim), int(tp_world), int(tp_rank)
        if dim not in (0, 1):
            raise RuntimeError(f"[DION_BAD_TP_SHARD_DIM] tp_shard_dim={dim}")
        q_rows, fs_dim, fs_world = None, -1, 1
        exp = [end - start, n] if dim == 0 else [m, end - start]
        if fs_shard is not None:
            (fm, fn), fs_dim, fs0, fs1, fs_world = fs_shard
            fs_dim, fs_world = int(fs_dim), int(fs_world)
            if (int(fm), int(fn)) != (m, n):
                raise RuntimeError(f"[DION_BAD_FS_TP_SHARD] FS global {(fm, fn)} != TP global {(m, n)}")
            if fs_dim != 1 - dim:
                raise RuntimeError(f"[DION_BAD_FS_SHARD_DIM] fs_shard_dim={fs_dim} with tp_shard_dim={dim}: FS "
                                   "shards the dim orthogonal to TP (distrib_dion/sharding.py:64-70)")
            exp[fs_dim] = int(fs1) - int(fs0)
            q_rows = (int(fs0), int(fs1))
        if (ml, nl) != tuple(exp):
            raise RuntimeError(f"[DION_BAD_TP_SHARD] local {(ml, nl)} vs global {(m, n)} dim {dim} [{start}, {end})"
                               + ("" if fs_shard is None else f" FS {q_rows}"))
        transposed = dim == 1
        r = rank_for_shape(m, n, rank_fraction, rank_multiple_of)
        base = r // tp_world
        rem = r % tp_world
        c0 = tp_rank * base + min(tp_rank, rem)
        c1 = c0 + base + (1 if tp_rank < rem else 0)
        if c1 <= c0:
            raise RuntimeError(f"[DION_EMPTY_Q_SHARD] r_global={r} tp_world_size={tp_world} tp_rank={tp_rank}")
        q_shape = (m if transposed else n, r)
        seed = q_seed_from_param_key(base_seed=base_seed, param_uid=param_uid, param_name=param_name,
                                     q_global_shape=q_shape, is_transposed=transposed)
        if q_stream not in ("device", "cpu"):
            raise RuntimeError(f"[DION_INVALID_Q_STREAM] q_stream={q_stream!r}")
        q = init_q(q_shape, seed, param.device if q_stream == "device" else "cpu", dtype=q_dtype or param.dtype,
                   rows=q_rows, cols=(c0, c1)).to(param.device)
        state = {"Q": q, "r": r, "local_shape": (ml, nl), "global_shape": (m, n)}
        if with_momentum:
            state = {"momentum": torch.zeros_like(param, dtype=momentum_dtype or param.dtype), **state}
        cfg = DionParamConfig(is_transposed=transposed, use_low_rank_sync=bool(use_low_rank_sync) and
                              should_use_low_rank_sync(global_shape=(m, n), r_global=r, rank_fraction=rank_fraction))
        cfg.has_tp_shard, cfg.use_tp_shard, cfg.tp_shard_dim = True, tp_world > 1, dim
        if fs_shard is not None:
            cfg.has_fs_shard, cfg.use_fs_shard, cfg.fs_shard_dim = True, fs_world > 1, fs_dim
        return state, cfg
    if fs_shard is None:
        m, n = ml, nl
        transposed = is_transposed_shape(m, n)
        dim, start, end, fs_world = -1, 0, (n if not transposed else m), 1
    else:
        (m, n), dim, start, end, fs_world = fs_shard
        m, n, dim = int(m), int(n), int(dim)
        if dim not in (0, 1):
            raise RuntimeError(f"[DION_BAD_FS_SHARD_DIM] fs_shard_dim={dim}")
        if (ml, nl) != ((end - start, n) if dim == 0 else (m, end - start)):
            raise RuntimeError(f"[DION_BAD_FS_SHARD] local {(ml, nl)} vs global {(m, n)} dim {dim} [{start}, {end})")
        transposed = dim == 0
    r = rank_for_shape(m, n, rank_fraction, rank_multiple_of)
    q_shape = (m if transposed else n, r)
    seed = q_seed_from_param_key(base_seed=base_seed, param_uid=param_uid, param_name=param_name,
                                 q_global_shape=q_shape, is_transposed=transposed)
    if q_stream not in ("device", "cpu"):
        raise RuntimeError(f"[DION_INVALID_Q_STREAM] q_stream={q_stream!r}")
    q = init_q(q_shape, seed, param.device if q_stream == "device" else "cpu", dtype=q_dtype or param.dtype,
               rows=None if fs_shard is None else (start, end)).to(param.device)
    state = {
        "Q": q,
        "r": r,
        "local_shape": (ml, nl),
        "global_shape": (m, n),
    }
    if with_momentum:  # split children (split.py) read their rows of the parent's momentum
        state = {"momentum": torch.zeros_like(param, dtype=momentum_dtype or param.dtype), **state}
    cfg = DionParamConfig(
        is_transposed=transposed,
        use_low_rank_sync=bool(use_low_rank_sync) and should_use_low_rank_sync(
            global_shape=(m, n), r_global=r, rank_fraction=rank_fraction),
    )
    if fs_shard is not None:
        cfg.has_fs_shard, cfg.use_fs_shard, cfg.fs_shard_dim = True, int(fs_world) > 1, dim
    return state, cfg
