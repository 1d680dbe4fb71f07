"""CPU restatement of the reference Dion data-parallel step.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package imports this module;
only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg use
it, and only as the checker / the timed CPU baseline.  The product path
(`megatron-dion_amd/`) runs the HIP kernels and fails loudly without them.

The reference's arithmetic for this path is plain torch (pinned torch 2.10.0,
`uv.lock:6836-6837`); this restatement uses the same fp32 torch CPU primitives
(`matmul`, `linalg.qr`, `linalg.cholesky_ex`, `linalg.solve_triangular`) in the
same order, so on identical inputs (and an identical sketch S) it reproduces the
reference bit-for-bit on this image.  It is pinned against the golden fixtures
captured from the reference itself (`tests/golden/make_golden.py`,
`tests/test_oracle_golden.py`).

Reference files (all under `/root/reference/megatron/core/optimizer/`):
  dion/runtime.py:1499-1911  batch_dion_update_async (the hot path)
  dion/runtime.py:1379-1496  ddp low-rank replica sync (RS/ortho/AG, R all-reduce)
  dion/ortho.py:71-123       orthogonalize (randomised Cholesky QR)
  dion/ortho.py:643-662      generate_random_sketch_matrix
  dion/kernels.py:25-51      scaled_lr_for_shape
  dion/kernels.py:54-154     apply_error_feedback
  dion/kernels.py:157-204    fix_all_zero_or_nan
  dion/kernels.py:207-210,279-290  column sum-of-squares + normalize_columns
  dion/kernels.py:229-276 + runtime.py:1105-1132  weight update and Q commit
  dion/state.py:179-188      rank rule;  state.py:220-230 low-rank-sync rule
  dion/runtime.py:1729-1795, :965-1013  the FS ("fsdp") kind: RS(sum)/ortho/AG of the
                             partial P, shard-local R / fix-up / EF, column norm over shards
  dion/runtime.py:1328-1377, :680-873, :923-962; ortho.py:575-640, 682-871  the TP ("fsdp_tp")
                             kind: Q unshard, row-sharded RCQR, R sum over TP, Q reshard
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence

import torch

__all__ = [
    "rank_for_shape",
    "use_low_rank_sync",
    "sketch_rows",
    "scaled_lr_for_shape",
    "orthogonalize",
    "fix_all_zero_or_nan",
    "column_normalize",
    "DionMatrix",
    "DionHyper",
    "dion_batch_step_local",
    "dion_batch_step_replicated",
    "dion_batch_step_tp",
    "split_range",
    "distributed_sketch_seed",
    "reference_sharded_sketch",
    "grad_sum_sq_fp64",
    "elementwise_adamw",
    "elementwise_lion",
]


# --------------------------------------------------------------------------- rules
def rank_for_shape(m: int, n: int, rank_fraction: float, rank_multiple_of: int = 1) -> int:
    """dion/state.py:183-188: r = max(1, int(min(mult*ceil(rf*min(m,n)/mult), m, n)))."""
    r = rank_fraction * min(m, n)
    r = rank_multiple_of * math.ceil(r / rank_multiple_of)
    r = min(r, m, n)
    return max(1, int(r))


def use_low_rank_sync(m: int, n: int, r: int, rank_fraction: float) -> bool:
    """dion/state.py:220-230."""
    if rank_fraction >= 1.0:
        return False
    return (m + n) * int(r) < m * n


def sketch_rows(r: int, oversample: float = 1.25) -> int:
    """dion/ortho.py:654 (k = ceil(oversample * r / 128) * 128)."""
    return int(math.ceil(oversample * r / 128.0) * 128)


def scaled_lr_for_shape(*, lr, m_global, n_global, scale_mode, rank_fraction,
                        extra_scale_factor=0.2) -> float:
    """dion/kernels.py:25-51 (spectral has no rank_fraction term)."""
    if m_global <= 0 or n_global <= 0:
        raise RuntimeError(f"[DION_INVALID_SCALE_SHAPE] m_global={m_global} n_global={n_global}")
    if rank_fraction <= 0.0:
        raise RuntimeError(f"[DION_INVALID_RANK_FRACTION] rank_fraction={rank_fraction}")
    if scale_mode == "spectral":
        return lr * extra_scale_factor * math.sqrt(float(max(m_global, n_global)))
    rank_scale = extra_scale_factor / math.sqrt(float(rank_fraction))
    if scale_mode == "unit_rms_norm":
        return lr * rank_scale * math.sqrt(float(m_global) / float(n_global))
    if scale_mode == "shape_scaling":
        return lr * rank_scale * math.sqrt(max(1.0, float(m_global) / float(n_global)))
    raise RuntimeError(f"[DION_INVALID_SCALE_MODE] scale_mode={scale_mode!r}")


# --------------------------------------------------------------------------- ortho
def orthogonalize(P: torch.Tensor, oversample: float = 1.25,
                  sketch: Optional[torch.Tensor] = None,
                  generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """Randomised Cholesky QR of a batch (B, m, r); dion/ortho.py:71-123.

    `sketch` (B, k, m) replaces the reference's unseeded N(0, 1/k) draw
    (ortho.py:659-661) so the result is reproducible; absent, one is drawn from
    `generator` the same way.
    """
    assert P.ndim >= 3
    dtype = P.dtype
    X = P.to(torch.float32)
    if X.size(-2) <= X.size(-1):                       # ortho.py:93-94
        X = torch.linalg.qr(X, mode="reduced")[0].to(torch.float32)
        return X.to(dtype).contiguous()
    k = sketch_rows(X.size(-1), oversample)
    if sketch is None:
        sketch = torch.empty((*X.shape[:-2], k, X.size(-2)), dtype=torch.float32)
        sketch.normal_(std=math.sqrt(1.0 / k), generator=generator)
    S = sketch.to(torch.float32)
    R1 = torch.linalg.qr(S @ X, mode="r")[1].to(torch.float32)          # ortho.py:101-104
    X = torch.linalg.solve_triangular(R1, X, upper=True, left=False).to(torch.float32)
    R2 = torch.linalg.cholesky_ex((X.mT @ X).to(torch.float32), upper=True)[0]
    X = torch.linalg.solve_triangular(R2.to(torch.float32), X, upper=True,
                                      left=False).to(torch.float32)     # ortho.py:112-121
    return X.to(dtype).contiguous()


# --------------------------------------------------------------------------- fix-up
def fix_all_zero_or_nan(P, R, Q, M, real_batch_size: int):
    """dion/kernels.py:157-204: sanitise the first `real_batch_size` entries."""
    B = P.size(0)
    real = int(real_batch_size)
    if real < 0 or real > B:
        raise RuntimeError(f"[DION_INVALID_FIXUP_REAL_BATCH_SIZE] real_batch_size={real} batch_size={B}")
    if real == 0:
        return P, R
    zero = (M[:real] == 0).all(dim=(-2, -1), keepdim=True)
    keep = ~zero
    p_fix = P[:real].nan_to_num() * keep
    r_fix = R[:real].nan_to_num() * keep + Q[:real].nan_to_num() * zero
    if real == B:
        return p_fix, r_fix
    p_out, r_out = torch.empty_like(P), torch.empty_like(R)
    p_out[:real] = p_fix
    r_out[:real] = r_fix
    p_out[real:] = P[real:]
    r_out[real:] = R[real:]
    return p_out, r_out


def column_normalize(R: torch.Tensor, epsilon: float) -> torch.Tensor:
    """dion/kernels.py:207-210 (fp32 column sum of squares) + :279-290."""
    col = R.to(torch.float32).square().sum(dim=-2, keepdim=True)
    denom = col.sqrt().add_(epsilon)
    return (R.to(torch.float32) / denom).to(R.dtype)


# --------------------------------------------------------------------------- step
@dataclass
class DionHyper:
    """Hyper-parameters read by the step (runtime.py:1068-1095; algorithm.py:82-105)."""
    lr: float = 0.01
    mu: float = 0.95
    weight_decay: float = 0.01
    epsilon: float = 1e-8
    rcqr_oversample: float = 1.25
    scale_mode: str = "spectral"
    extra_scale_factor: float = 0.2
    rank_fraction: float = 0.25


@dataclass
class DionMatrix:
    """One Dion parameter's state: W (m x n fp32), M (m x n), Q (n_Q x r); G read-only."""
    W: torch.Tensor
    M: torch.Tensor
    Q: torch.Tensor
    G: Optional[torch.Tensor]
    transposed: bool
    rank_fraction: float = 0.25
    trace: dict = field(default_factory=dict)


SketchFn = Callable[[int, torch.Tensor], Optional[torch.Tensor]]


def _project(mats: Sequence[DionMatrix]):
    """runtime.py:1560-1616: M += G, stack X = M or M^T, P = X @ Q (TF32 off)."""
    for mt in mats:
        if mt.G is not None:
            if mt.M.dtype == mt.G.dtype:
                mt.M.add_(mt.G)
            else:
                mt.M.add_(mt.G.to(mt.M.dtype))
    X = torch.stack([mt.M.mT if mt.transposed else mt.M for mt in mats], dim=0)
    Qb = torch.stack([mt.Q.to(X.dtype) for mt in mats], dim=0)
    return X, Qb, X @ Qb


def _finish(mats: Sequence[DionMatrix], X, Qb, P, R, real: int, hyper: DionHyper,
            m_global: int, n_global: int, colsum_reduce=None, q_cols=None):
    """runtime.py:1838-1901: fix-up, error feedback, column norm, weight update, Q commit.

    `colsum_reduce(col_sum_sq)` (FS kind) returns the column sums of squares summed over
    the q_norm group (runtime.py:994-1001); the local sums are used otherwise.  `q_cols`
    (TP kind) = (c0, c1): the rank keeps only those columns of the new Q
    (reshard_q_along_tp, ortho.py:837-871)."""
    P, R = fix_all_zero_or_nan(P, R, Qb, X, real)
    transposed = mats[0].transposed
    alpha = -(1.0 - hyper.mu)
    # kernels.py:54-83: update = A @ B.mT; X *= beta(=1); X += alpha*update
    upd = (R[:real] @ P[:real].mT) if transposed else (P[:real] @ R[:real].mT)
    upd = upd * alpha
    for i in range(real):
        mats[i].M.mul_(1.0)
        mats[i].M.add_(upd[i])
    if colsum_reduce is None:
        Qn = column_normalize(R[:real], hyper.epsilon)
    else:
        # kernels.py:207-210 local_column_sum_sq, summed over the shards, then :279-290
        col = colsum_reduce(R[:real].to(torch.float32).square().sum(dim=-2, keepdim=True))
        Qn = (R[:real].to(torch.float32) / col.sqrt().add_(hyper.epsilon)).to(R.dtype)
    s = scaled_lr_for_shape(lr=hyper.lr, m_global=m_global, n_global=n_global,
                            scale_mode=hyper.scale_mode,
                            rank_fraction=hyper.rank_fraction,
                            extra_scale_factor=hyper.extra_scale_factor)
    pd = P[:real]
    qd = Qn.to(pd.dtype)
    delta = torch.bmm(qd, pd.transpose(1, 2)) if transposed else torch.bmm(pd, qd.transpose(1, 2))
    for i in range(real):
        if hyper.weight_decay > 0:
            mats[i].W.mul_(1 - hyper.lr * hyper.weight_decay)
        mats[i].W.add_(delta[i].to(mats[i].W.dtype), alpha=-s)
        mats[i].Q.copy_(Qn[i] if q_cols is None else Qn[i][:, q_cols[0]:q_cols[1]])
        mats[i].trace.update(P=P[i].clone(), R=R[i].clone(), Qn=Qn[i].clone())


def dion_batch_step_local(mats: List[DionMatrix], hyper: DionHyper,
                          sketch_fn: Optional[SketchFn] = None) -> None:
    """One batch on one rank with no replicas (W = 1): runtime.py:1647-1731 + :1838-1901.

    `sketch_fn(i, P_i)` returns the sketch for entry i (or None to draw one).
    All matrices share one global shape (the batch contract, runtime.py:196-291).
    """
    real = len(mats)
    X, Qb, P = _project(mats)
    P_in = P.clone()
    outs = []
    for i in range(real):                     # orthogonalize over the real batch
        S = sketch_fn(i, P[i:i + 1]) if sketch_fn is not None else None
        outs.append(orthogonalize(P[i:i + 1], hyper.rcqr_oversample, sketch=S))
    P = torch.cat(outs, dim=0).to(X.dtype).contiguous()
    R = X.mT @ P
    m, n = mats[0].M.shape
    for i in range(real):
        mats[i].trace["P_raw"] = P_in[i]
    _finish(mats, X, Qb, P, R, real, hyper, m, n)


def _replicated_batch_gen(per_rank: List[List[DionMatrix]], real: int, hyper: DionHyper,
                          sketch_fn, buffers: Optional[List[dict]]):
    """Generator over all W ranks of one batch, yielding where runtime.py yields.

    runtime.py:1379-1496 (ddp, low-rank sync): P_w = X_w @ Q; ReduceScatter(avg)
    [yield, :1434] hands entry c*W+k to rank k, which orthogonalises it (zeros
    for padding, :1436-1441); AllGather [yield, :1454] into the per-optimizer
    cached buffer "replicated_p_ortho_full" (:1419-1424); R_w = X_w^T @ P;
    AllReduce(avg) of R [yield, :515-525]; then the fix-up/EF/update tail.

    `buffers[w]` emulates rank w's `optimizer._cached_buffer` dict.  The
    reference keys that buffer by name and shape only, so two same-shape
    batches in flight in its AsyncRuntime share it and the earlier batch's
    fix-up/EF/update reads the later batch's P (a reference defect,
    DESIGN.md "Reference defects").  Pass `buffers=None` for the intended
    per-batch semantics.
    """
    W = len(per_rank)
    B = len(per_rank[0])
    proj = [_project(mats) for mats in per_rank]
    P_avg = torch.stack([p[2] for p in proj], dim=0).sum(dim=0) / W
    yield                                                   # reduce-scatter in flight
    P_ortho = torch.zeros_like(P_avg)
    for start in range(0, B, W):
        for k in range(W):
            idx = start + k
            if idx >= B or idx >= real:
                continue
            S = sketch_fn(k, idx, P_avg[idx:idx + 1]) if sketch_fn is not None else None
            P_ortho[idx] = orthogonalize(P_avg[idx:idx + 1], hyper.rcqr_oversample, sketch=S)[0]
    yield                                                   # all-gather in flight
    P_views, Rs = [], []
    for w in range(W):
        if buffers is None:
            Pw = P_ortho.clone()
        else:
            key = ("replicated_p_ortho_full", tuple(P_ortho.shape))
            buf = buffers[w].get(key)
            if buf is None:
                buf = torch.empty_like(P_ortho)
                buffers[w][key] = buf
            buf.copy_(P_ortho)
            Pw = buf[:B]
        P_views.append(Pw)
        Rs.append(proj[w][0].mT @ Pw)
    yield                                                   # R all-reduce in flight
    R = torch.stack(Rs, dim=0).sum(dim=0) / W
    m, n = per_rank[0][0].M.shape
    for w in range(W):
        X, Qb, _ = proj[w]
        for i in range(real):
            per_rank[w][i].trace["P_raw"] = P_avg[i].clone()
        _finish(per_rank[w], X, Qb, P_views[w], R.clone(), real, hyper, m, n)


def _fs_batch_gen(per_rank: List[List[DionMatrix]], real: int, hyper: DionHyper, sketch_fn,
                  m_global: int, n_global: int, indices=None):
    """Generator over all FS ranks of one "fsdp" batch (FS world W, no replicas), yielding where
    dion/runtime.py yields on its FS-only path (:1729-1795; RP = 1, so no low-rank sync):

      every rank: M += G; X = M or M^T (its shard); P_k = X_k @ Q_k, a partial sum over the
        sharded dim (the orientation follows fs_shard_dim, dion/state.py:304-310)
      reduce_scatter(sum) [yield] -> rank k holds sum_k' P_k'[indices[k]]; orthogonalize it
        (zero for a padded entry, :1766-1777); all_gather [yield] (permuted back by indices)
      every rank: R_k = X_k^T @ P (its rows of R); fix-up with ITS shard's zero test
        (kernels.py:157-204 on the local M_batch); error feedback on its shard
      column norm: local fp32 sums of squares all-reduced (sum) over the FS group
        (q_norm_group, :994-1001) [yield]; Q_k = R_k / (sqrt(sum) + eps)
      weight update of its shard with the GLOBAL shape's scaled LR (:1056-1090)

    per_rank[k] holds rank k's B = W entries (padded entries carry zero G/M/Q); the reduce-
    scatter sums in rank order.  `sketch_fn(rank, entry, P)`."""
    W = len(per_rank)
    B = len(per_rank[0])
    idx_of = list(indices) if indices is not None else list(range(W))
    proj = [_project(mats) for mats in per_rank]
    P_sum = proj[0][2].clone()
    for k in range(1, W):
        P_sum = P_sum + proj[k][2]
    yield                                                   # reduce-scatter in flight
    P_ortho = torch.zeros_like(P_sum)
    for k in range(W):
        idx = idx_of[k]
        if idx >= real:
            continue
        S = sketch_fn(k, idx, P_sum[idx:idx + 1]) if sketch_fn is not None else None
        P_ortho[idx] = orthogonalize(P_sum[idx:idx + 1], hyper.rcqr_oversample, sketch=S)[0]
    yield                                                   # all-gather in flight
    Rs = [proj[k][0].mT @ P_ortho for k in range(W)]
    fixed = []
    for k in range(W):
        X, Qb, _ = proj[k]
        fixed.append(fix_all_zero_or_nan(P_ortho.clone(), Rs[k], Qb, X, real))
    sums = [f[1][:real].to(torch.float32).square().sum(dim=-2, keepdim=True) for f in fixed]
    total = sums[0].clone()
    for k in range(1, W):
        total = total + sums[k]
    yield                                                   # column-norm all-reduce in flight
    for k in range(W):
        X, Qb, _ = proj[k]
        for i in range(real):
            per_rank[k][i].trace["P_raw"] = P_sum[i].clone()
        _finish(per_rank[k], X, Qb, P_ortho.clone(), Rs[k], real, hyper, m_global, n_global,
                colsum_reduce=lambda _local, _t=total: _t)


def dion_step_fs(batches, hyper: DionHyper, sketch_fn=None, max_concurrent: int = 3) -> None:
    """One optimizer step over FS ("fsdp") batches, every FS rank simulated.

    `batches` is a list of (per_rank, real, (m_global, n_global)) as _fs_batch_gen takes them."""
    gens = (_fs_batch_gen(per_rank, real, hyper, sketch_fn, mg, ng) for per_rank, real, (mg, ng) in batches)
    run_async_runtime(gens, max_concurrent=max_concurrent)


def split_range(size: int, world: int, rank: int):
    """dion/ortho.py:247-259 (_split_range): contiguous shards, remainder on the first ranks."""
    base, rem = size // world, size % world
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def distributed_sketch_seed(step_count: int, param_uid, param_name: str) -> int:
    """dion/ortho.py:126-131 + 154-177: the seed of one matrix's distributed sketch,
    blake2b(repr(("distributed", step, param_uid, param_name)))."""
    import hashlib
    key = ("distributed", int(step_count), param_uid, param_name)
    return int.from_bytes(hashlib.blake2b(repr(key).encode("utf-8"), digest_size=8).digest(),
                          "little") & ((1 << 63) - 1)


def reference_sharded_sketch(seed: int, k: int, global_rows: int, row_start: int, rows: int) -> torch.Tensor:
    """dion/ortho.py:575-640 on CPU: one seeded N(0, 1/k) draw of the (k, global_rows) sketch,
    of which the rank keeps its columns [row_start, row_start + rows)."""
    gen = torch.Generator(device="cpu")
    gen.manual_seed(int(seed))
    full = torch.empty((k, global_rows), dtype=torch.float32)
    full.normal_(mean=0.0, std=math.sqrt(1.0 / k), generator=gen)
    return full[:, row_start:row_start + rows].clone()


def dion_batch_step_tp(per_rank: List[List[DionMatrix]], hyper: DionHyper, m_global: int, n_global: int,
                       sketch_fn=None) -> None:
    """One "fsdp_tp" batch, every TP rank simulated (TP world T; no FS, no replicas).

    per_rank[k][i]: rank k's shard of matrix i -- W/M/G its rows of the P side (tp_shard_dim on
    m_P, dion/state.py:304-310 and :407-416) and Q its columns of the rank (resolve_q_state_layout,
    state.py:159-217).  Reference order:
      M += G (local); Q all-gathered over TP, columns in rank order       runtime.py:1560-1566, :680-873
      P_k = X_k Q (this rank's rows of P)                                  runtime.py:1602-1616
      distributed RCQR over the row shards (ortho.py:682-834):
        global rows <= r: QR of the whole P (rows exchanged, :752-775)
        else SP = sum_k S[:, rows_k] P_k (reduce-scatter over batch shards), R1 = qr(SP).R,
             P_k = P_k R1^-1; G = sum_k P_k^T P_k, R2 = chol_upper(G), P_k = P_k R2^-1
      R = sum_k X_k^T P_k (all-reduce sum over TP, runtime.py:923-962)
      per rank: fix-up with ITS shard's zero test and the gathered Q, error feedback on its shard,
        column norm of the full R (no q_norm group), weight update with the GLOBAL shape's LR,
        Q <- its columns of the new Q (ortho.py:837-871)
    `sketch_fn(k, i, rows)` returns rank k's (k_s, rows) slice of entry i's sketch."""
    T = len(per_rank)
    real = len(per_rank[0])
    Qfull = [torch.cat([per_rank[k][i].Q for k in range(T)], dim=1) for i in range(real)]
    r = int(Qfull[0].shape[1])
    cols, start = [], 0
    for k in range(T):
        w = int(per_rank[k][0].Q.shape[1])
        cols.append((start, start + w))
        start += w
    Xs, Ps = [], []
    for k in range(T):
        for mt in per_rank[k]:
            if mt.G is not None:
                mt.M.add_(mt.G if mt.M.dtype == mt.G.dtype else mt.G.to(mt.M.dtype))
        X = torch.stack([mt.M.mT if mt.transposed else mt.M for mt in per_rank[k]], dim=0)
        Xs.append(X)
        Ps.append(X @ torch.stack([q.to(X.dtype) for q in Qfull], dim=0))
    rows = [int(P.shape[1]) for P in Ps]
    P_raw = [P.clone() for P in Ps]
    pdt = Ps[0].dtype  # ortho.py:699-750: fp32 inside, back to P's dtype at the end (:770, :829)
    Ps = [P.to(torch.float32) for P in Ps]
    if sum(rows) <= r:
        full = torch.linalg.qr(torch.cat(Ps, dim=1), mode="reduced")[0].to(torch.float32)
        offs = [sum(rows[:k]) for k in range(T)]
        Ps = [full[:, offs[k]:offs[k] + rows[k]].contiguous() for k in range(T)]
    else:
        SP = None
        for k in range(T):
            S = torch.stack([sketch_fn(k, i, rows[k]) for i in range(real)], dim=0).to(torch.float32)
            part = S @ Ps[k]
            SP = part if SP is None else SP + part
        R1 = torch.linalg.qr(SP.to(torch.float32), mode="r")[1].to(torch.float32)
        Ps = [torch.linalg.solve_triangular(R1, P, upper=True, left=False).to(torch.float32) for P in Ps]
        Gm = None
        for P in Ps:
            part = P.mT @ P
            Gm = part if Gm is None else Gm + part
        R2 = torch.linalg.cholesky_ex(Gm.to(torch.float32), upper=True)[0].to(torch.float32)
        Ps = [torch.linalg.solve_triangular(R2, P, upper=True, left=False).to(torch.float32) for P in Ps]
    Ps = [P.to(pdt) for P in Ps]
    R = None
    for k in range(T):
        part = Xs[k].mT @ Ps[k]
        R = part if R is None else R + part
    Qb = torch.stack(Qfull, dim=0)
    for k in range(T):
        for i in range(real):
            per_rank[k][i].trace["P_raw"] = P_raw[k][i].clone()
        _finish(per_rank[k], Xs[k], Qb, Ps[k].contiguous(), R.clone(), real, hyper, m_global, n_global,
                q_cols=cols[k])


def run_async_runtime(generators, max_concurrent: int = 3) -> None:
    """Round-robin of batch generators exactly as dion/runtime.py:140-171 (AsyncRuntime).

    A task is advanced to its first yield when created (AsyncTask.__init__,
    runtime.py:120-125); each loop admits at most one new task while fewer than
    `max_concurrent` are running, then advances every previous task once.
    """
    def start(gen):
        try:
            next(gen)
            return True
        except StopIteration:
            return False

    it = iter(generators)
    have_new = True
    previous = []
    while have_new or previous:
        running = []
        if have_new and len(previous) < max_concurrent:
            try:
                gen = next(it)
            except StopIteration:
                have_new = False
            else:
                if start(gen):
                    running.append(gen)
        for gen in previous:
            if start(gen):
                running.append(gen)
        previous = running


def dion_step_replicated(batches, hyper: DionHyper, sketch_fn=None,
                         reference_shared_p_buffer: bool = False,
                         max_concurrent: int = 3) -> None:
    """One optimizer step over a list of replicated batches (all W ranks simulated).

    `batches` is a list of (per_rank, real) where per_rank[w] holds rank w's B
    entries (padded entries carry zero G/M/Q).  `sketch_fn(rank, entry, P)`.
    """
    W = len(batches[0][0]) if batches else 1
    buffers = [dict() for _ in range(W)] if reference_shared_p_buffer else None
    gens = (_replicated_batch_gen(per_rank, real, hyper, sketch_fn, buffers)
            for per_rank, real in batches)
    run_async_runtime(gens, max_concurrent=max_concurrent)


def elementwise_adamw(params, grads, first_moments, second_moments, *, lr, beta1, beta2, weight_decay,
                      step, epsilon) -> None:
    """dion/elementwise_opts.py:45-80 (_adamw_update_foreach_chunk), same foreach chain."""
    n = len(params)
    g1 = [g.to(dtype=first_moments[0].dtype) for g in grads]
    torch._foreach_lerp_(first_moments, g1, [1.0 - beta1] * n)
    gsq = [g.to(dtype=second_moments[0].dtype) for g in torch._foreach_mul(g1, g1)]
    torch._foreach_lerp_(second_moments, gsq, [1.0 - beta2] * n)
    bc1 = 1.0 - beta1 ** step
    bc2_sqrt = (1.0 - beta2 ** step) ** 0.5
    denom = torch._foreach_sqrt(second_moments)
    torch._foreach_div_(denom, bc2_sqrt)
    torch._foreach_add_(denom, [epsilon] * n)
    upd = torch._foreach_div(first_moments, denom)
    torch._foreach_mul_(upd, lr / bc1)
    if weight_decay != 0.0:
        torch._foreach_mul_(params, 1.0 - lr * weight_decay)
    torch._foreach_sub_(params, upd)


def elementwise_lion(params, grads, first_moments, *, lr, beta1, beta2, weight_decay) -> None:
    """dion/elementwise_opts.py:83-105 (_lion_update_foreach_chunk), same foreach chain."""
    n = len(params)
    g1 = [g.to(dtype=first_moments[0].dtype) for g in grads]
    upd = torch._foreach_lerp(first_moments, g1, [1.0 - beta1] * n)
    torch._foreach_sign_(upd)
    torch._foreach_lerp_(first_moments, g1, [1.0 - beta2] * n)
    torch._foreach_mul_(upd, lr)
    if weight_decay != 0.0:
        torch._foreach_mul_(params, 1.0 - lr * weight_decay)
    torch._foreach_sub_(params, upd)


def grad_sum_sq_fp64(tensors, chunk_bytes: int = 128 * 1024 * 1024) -> torch.Tensor:
    """distrib_dion/grad_norm.py:54-68 (_grad_sum_sq_fp64), summed over `tensors`
    like _dion_grad_norm_sq (:166-172): chunked cast to fp64, square, sum."""
    total = torch.zeros(1, dtype=torch.float64)
    for t in tensors:
        flat = t.detach().reshape(-1)
        step = max(1, int(chunk_bytes) // 8)
        for start in range(0, flat.numel(), step):
            chunk = flat[start:start + step].to(torch.float64)
            chunk.mul_(chunk)
            total += chunk.sum()
    return total


def dion_batch_step_replicated(per_rank, real, hyper, sketch_fn=None) -> None:
    """A single replicated batch (no other batch in flight)."""
    dion_step_replicated([(per_rank, real)], hyper, sketch_fn)
