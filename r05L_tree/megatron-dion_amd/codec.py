"""Device codec: thin torch-facing wrapper over the C ABI (include/dion_codec.h).

`HipDionCodec` is the only compute backend of the product path.  It takes the
reference's per-parameter tensors (one device tensor per matrix, exactly like
`DionBatch.params / momentums / q_tensors / grads`,
/root/reference/megatron/core/optimizer/dion/types.py:161-226) plus the batch
factors P (B, m_P, r) and R (B, n_Q, r), and enqueues the HIP kernels on the
current HIP stream.  Torch is used only for memory and streams.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import torch

from . import _lib

__all__ = ["HipDionCodec", "factor_rows"]


def factor_rows(m: int, n: int, transposed: bool):
    """(m_P, n_Q): P rows and Q rows for one m x n matrix (state.py:304-310 orientation)."""
    return (n, m) if transposed else (m, n)


def _ptrs(tensors: Sequence[Optional[torch.Tensor]]):
    arr = (ctypes.c_void_p * max(1, len(tensors)))()
    for i, t in enumerate(tensors):
        arr[i] = None if t is None else t.data_ptr()
    return arr


def _dtype_code(t: Optional[torch.Tensor]) -> int:
    if t is None:
        return _lib.DTYPE_NONE
    if t.dtype == torch.float32:
        return _lib.DTYPE_F32
    if t.dtype == torch.bfloat16:
        return _lib.DTYPE_BF16
    raise RuntimeError(f"[DION_UNSUPPORTED_DTYPE] {t.dtype}")


def _dtype_code_state(dtype) -> int:
    if dtype == torch.float32:
        return _lib.DTYPE_F32
    if dtype == torch.bfloat16:
        return _lib.DTYPE_BF16
    raise RuntimeError(f"[DION_UNSUPPORTED_STATE_DTYPE] momentum/Q dtype {dtype}")


def _state_dtype(momentums, qs) -> torch.dtype:
    """Momentum and Q share one dtype (fp32, or bf16 for both: speedrun_nanogpt_mcore.py:422-431)."""
    dts = {t.dtype for t in list(momentums or []) + list(qs or [])}
    if len(dts) != 1:
        raise RuntimeError(f"[DION_UNSUPPORTED_MIXED_STATE_DTYPES] momentum/Q dtypes {sorted(map(str, dts))}")
    return dts.pop()


def _row_stride(t: torch.Tensor) -> int:
    if t.dim() != 2 or t.stride(1) != 1:
        raise RuntimeError(f"[DION_NON_ROW_MAJOR] shape={tuple(t.shape)} stride={t.stride()}")
    return int(t.stride(0))


class HipDionCodec:
    """Enqueue the Dion codec kernels for batches of same-shape matrices."""

    name = "hip"
    fuses_p_fixup = True  # orthonormalize(fix_nonzero=...) + fixup_colnorm(P=None)
    fuses_r_fixup = True  # project_r_fixup: project_r + fixup_colnorm(P=None) in one call

    def __init__(self, device: Optional[torch.device] = None):
        self.lib = _lib.load()
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self._ws = {}  # per-stream scratch: batches may run concurrently on several streams
        self._ef_ok = {}

    # ------------------------------------------------------------------ helpers
    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _desc(self, batch, m, n, r, transposed, g=None, M=None, W=None, state_dtype=None) -> _lib.DionBatchDesc:
        d = _lib.DionBatchDesc()
        d.batch = int(batch)
        d.m, d.n, d.r = int(m), int(n), int(r)
        d.transposed = 1 if transposed else 0
        d.g_dtype = _dtype_code(g)
        # momentum / Q dtype: fp32, or the speedrun's bf16 state (DionMixedPrecisionConfig)
        sdt = state_dtype if state_dtype is not None else (M.dtype if M is not None else torch.float32)
        d.m_dtype = _dtype_code_state(sdt)
        d.w_dtype = _lib.DTYPE_F32
        d.ld_g = _row_stride(g) if g is not None else 0
        d.ld_m = _row_stride(M) if M is not None else 0
        d.ld_w = _row_stride(W) if W is not None else 0
        return d

    def workspace(self, desc, op) -> torch.Tensor:
        nbytes = ctypes.c_size_t(0)
        _lib.check(self.lib.dion_workspace_bytes(ctypes.byref(desc), op, ctypes.byref(nbytes)),
                   "dion_workspace_bytes")
        key = torch.cuda.current_stream(self.device).cuda_stream
        ws = self._ws.get(key)
        if ws is None or nbytes.value > ws.numel():
            ws = torch.empty(max(int(nbytes.value), 1), dtype=torch.uint8, device=self.device)
            self._ws[key] = ws
        return ws

    def _check_batch(self, mats: Sequence[torch.Tensor], dtype=torch.float32):
        m, n = mats[0].shape
        for t in mats:
            if tuple(t.shape) != (m, n) or t.dtype != dtype or t.device != self.device:
                raise RuntimeError(f"[DION_INCONSISTENT_BATCH] {tuple(t.shape)} {t.dtype} {t.device}")
        return int(m), int(n)

    # ------------------------------------------------------------------ passes
    def project_p(self, grads: Optional[List[torch.Tensor]], momentums: List[torch.Tensor],
                  qs: List[torch.Tensor], P: torch.Tensor, nonzero: torch.Tensor, transposed: bool) -> None:
        """M += G; P = M Q (or M^T Q); nonzero flags.  runtime.py:1560-1616."""
        B = len(momentums)
        if B == 0:
            return
        m, n = self._check_batch(momentums, _state_dtype(momentums, qs))
        r = int(qs[0].shape[1])
        g0 = grads[0] if grads else None
        if grads:
            for g in grads:
                if g.dtype != g0.dtype or tuple(g.shape) != (m, n) or g.stride() != g0.stride():
                    raise RuntimeError("[DION_INCONSISTENT_GRADS]")
        d = self._desc(B, m, n, r, transposed, g=g0, M=momentums[0])
        ws = self.workspace(d, _lib.OP_PROJECT_P)
        rc = self.lib.dion_project_p(ctypes.byref(d), _ptrs(grads) if grads else None, _ptrs(momentums),
                                     _ptrs(qs), P.data_ptr(), nonzero.data_ptr(), ws.data_ptr(),
                                     ws.numel(), self._stream())
        _lib.check(rc, "dion_project_p")

    def supports_deferred_ef(self, m: int, n: int, r: int, transposed: bool, state_dtype=torch.float32,
                             grad_dtype=None) -> bool:
        """True when the fused deferred-EF pass A exists for this shape, state dtype and gradient
        dtype (dion_project_p_ef)."""
        key = (int(m), int(n), int(r), bool(transposed), state_dtype, grad_dtype)
        ok = self._ef_ok.get(key)
        if ok is None:
            d = self._desc(1, m, n, r, transposed, state_dtype=state_dtype)
            if grad_dtype is not None:
                d.g_dtype = _dtype_code(torch.empty(0, dtype=grad_dtype))
            nbytes = ctypes.c_size_t(0)
            ok = self.lib.dion_workspace_bytes(ctypes.byref(d), _lib.OP_PROJECT_P_EF, ctypes.byref(nbytes)) == 0
            self._ef_ok[key] = ok
        return ok

    def project_p_ef(self, grads: Optional[List[torch.Tensor]], momentums: List[torch.Tensor],
                     qs: List[torch.Tensor], P: torch.Tensor, nonzero: torch.Tensor, transposed: bool,
                     ef_P: Sequence[Optional[torch.Tensor]], ef_R: Sequence[Optional[torch.Tensor]],
                     alpha: float) -> None:
        """M += alpha P' R'^T (pending error feedback of the previous step), M += G, P = X Q."""
        B = len(momentums)
        if B == 0:
            return
        m, n = self._check_batch(momentums, momentums[0].dtype)
        r = int(qs[0].shape[1])
        g0 = grads[0] if grads else None
        if grads:
            for g in grads:
                if g.dtype != g0.dtype or tuple(g.shape) != (m, n) or g.stride() != g0.stride():
                    raise RuntimeError("[DION_INCONSISTENT_GRADS]")
        for t in list(ef_P) + list(ef_R):
            if t is not None and (not t.is_contiguous() or t.dtype != torch.float32 or t.device != self.device):
                raise RuntimeError(f"[DION_BAD_FACTOR] pending factor {tuple(t.shape)} {t.dtype} {t.stride()}")
        d = self._desc(B, m, n, r, transposed, g=g0, M=momentums[0])
        ws = self.workspace(d, _lib.OP_PROJECT_P_EF)
        pp, rr = _ptrs(ef_P), _ptrs(ef_R)
        ef = _lib.DionPendingEF(ctypes.cast(pp, ctypes.POINTER(ctypes.c_void_p)),
                                ctypes.cast(rr, ctypes.POINTER(ctypes.c_void_p)), float(alpha))
        rc = self.lib.dion_project_p_ef(ctypes.byref(d), _ptrs(grads) if grads else None, _ptrs(momentums),
                                        _ptrs(qs), P.data_ptr(), nonzero.data_ptr(), ctypes.byref(ef),
                                        ws.data_ptr(), ws.numel(), self._stream())
        _lib.check(rc, "dion_project_p_ef")

    def orthonormalize(self, P: torch.Tensor, m: int, n: int, transposed: bool, seed: int,
                       oversample: float = 1.25, sketch: Optional[torch.Tensor] = None,
                       state_dtype=torch.float32, fix_nonzero: Optional[torch.Tensor] = None,
                       p_split: Optional[torch.Tensor] = None) -> None:
        """Randomised Cholesky QR of every P_b in place.  ortho.py:71-123.

        With a bf16 state the fp32 result is rounded back to bf16 values (ortho.py:123).
        `fix_nonzero` (B,): also the fix-up of P (kernels.py:185-188; fixup_colnorm then gets
        P=None); `p_split` (psplit_buffer): also pass B's split of P (project_r(p_split=...))."""
        B, _, r = P.shape
        if B == 0:
            return
        d = self._desc(B, m, n, r, transposed, state_dtype=state_dtype)
        ws = self.workspace(d, _lib.OP_ORTHONORMALIZE)
        if fix_nonzero is None and p_split is None:
            rc = self.lib.dion_orthonormalize(ctypes.byref(d), P.data_ptr(),
                                              None if sketch is None else sketch.data_ptr(),
                                              int(seed) & ((1 << 64) - 1), float(oversample),
                                              ws.data_ptr(), ws.numel(), self._stream())
        else:
            rc = self.lib.dion_orthonormalize_fused(ctypes.byref(d), P.data_ptr(),
                                                    None if sketch is None else sketch.data_ptr(),
                                                    int(seed) & ((1 << 64) - 1), float(oversample),
                                                    None if fix_nonzero is None else fix_nonzero.data_ptr(),
                                                    None if p_split is None else p_split.data_ptr(),
                                                    ws.data_ptr(), ws.numel(), self._stream())
        _lib.check(rc, "dion_orthonormalize")

    def psplit_buffer(self, B: int, m: int, n: int, r: int, transposed: bool,
                      state_dtype=torch.float32) -> Optional[torch.Tensor]:
        """The (B, per-entry bytes) buffer for pass B's split of P written by the last solve of the
        orthonormalisation (DION_OP_PSPLIT), or None when this shape has no fused split."""
        key = ("psplit", int(m), int(n), int(r), bool(transposed), state_dtype)
        ok = self._ef_ok.get(key)
        if ok is None:
            d = self._desc(1, m, n, r, transposed, state_dtype=state_dtype)
            nbytes = ctypes.c_size_t(0)
            ok = self.lib.dion_workspace_bytes(ctypes.byref(d), _lib.OP_PSPLIT, ctypes.byref(nbytes)) == 0
            self._ef_ok[key] = (int(nbytes.value) if ok else 0)
            ok = self._ef_ok[key]
        if not ok:
            return None
        return torch.empty((int(B), int(ok)), dtype=torch.uint8, device=self.device)

    # ------------------------------------------------------------ distributed RCQR
    # the per-rank pieces of dion/ortho.py:682-834 (P row-sharded over the TP group); the
    # caller runs the collectives between them (runtime.distributed_orthonormalize)
    def dortho_sketch(self, P: torch.Tensor, m: int, n: int, transposed: bool, seed: int, row_offset: int,
                      oversample: float, SP: torch.Tensor, sketch: Optional[torch.Tensor] = None) -> None:
        """SP_b = S_b[:, rows] P_b (k x r): this rank's share of the sketch product.  `m, n`: the
        local shard's shape; `row_offset`: global index of the first local P row."""
        B, _, r = P.shape
        if B == 0:
            return
        d = self._desc(B, m, n, r, transposed)
        ws = self.workspace(d, _lib.OP_DORTHO)
        rc = self.lib.dion_dortho_sketch(ctypes.byref(d), P.data_ptr(), None if sketch is None else sketch.data_ptr(),
                                         int(seed) & ((1 << 64) - 1), int(row_offset), float(oversample),
                                         SP.data_ptr(), ws.data_ptr(), ws.numel(), self._stream())
        _lib.check(rc, "dion_dortho_sketch")

    def dortho_qr_inv(self, SP: torch.Tensor, R1inv: torch.Tensor) -> None:
        """R1inv_b = qr(SP_b).R^-1 (ortho.py:791-806)."""
        B, k, r = SP.shape
        if B == 0:
            return
        _lib.check(self.lib.dion_dortho_qr_inv(int(k), int(r), int(B), SP.data_ptr(), R1inv.data_ptr(),
                                               self._stream()), "dion_dortho_qr_inv")

    def dortho_apply(self, P_in: torch.Tensor, Uinv: torch.Tensor, P_out: torch.Tensor, m: int, n: int,
                     transposed: bool) -> None:
        """P_out_b = P_in_b Uinv_b (ortho.py:799-806, 821-828)."""
        B, _, r = P_in.shape
        if B == 0:
            return
        d = self._desc(B, m, n, r, transposed)
        _lib.check(self.lib.dion_dortho_apply(ctypes.byref(d), P_in.data_ptr(), Uinv.data_ptr(), P_out.data_ptr(),
                                              self._stream()), "dion_dortho_apply")

    def dortho_gram(self, P: torch.Tensor, gram: torch.Tensor, m: int, n: int, transposed: bool) -> None:
        """gram_b = P_b^T P_b, this rank's rows' share (ortho.py:808-812)."""
        B, _, r = P.shape
        if B == 0:
            return
        d = self._desc(B, m, n, r, transposed)
        ws = self.workspace(d, _lib.OP_DORTHO)
        _lib.check(self.lib.dion_dortho_gram(ctypes.byref(d), P.data_ptr(), gram.data_ptr(), ws.data_ptr(),
                                             ws.numel(), self._stream()), "dion_dortho_gram")

    def dortho_chol_inv(self, gram: torch.Tensor, R2inv: torch.Tensor) -> None:
        """R2inv_b = chol_upper(gram_b)^-1 (ortho.py:813-828)."""
        B, r, _ = gram.shape
        if B == 0:
            return
        _lib.check(self.lib.dion_dortho_chol_inv(int(r), int(B), gram.data_ptr(), R2inv.data_ptr(), self._stream()),
                   "dion_dortho_chol_inv")

    def project_r(self, momentums: List[torch.Tensor], P: torch.Tensor, R: torch.Tensor,
                  transposed: bool, nonzero: Optional[torch.Tensor] = None,
                  p_split: Optional[torch.Tensor] = None) -> None:
        """R = M^T P (or M P).  runtime.py:1476-1477.  `nonzero`: the flags project_p /
        project_p_ef left for these momentums (their max |M|: fixed-scale pass B).  `p_split`:
        P's limbs from orthonormalize(p_split=...) (no absmax / presplit of P here)."""
        B = len(momentums)
        if B == 0:
            return
        m, n = self._check_batch(momentums, momentums[0].dtype)
        r = int(P.shape[2])
        d = self._desc(B, m, n, r, transposed, M=momentums[0])
        ws = self.workspace(d, _lib.OP_PROJECT_R)
        rc = self.lib.dion_project_r_split(ctypes.byref(d), _ptrs(momentums), P.data_ptr(),
                                           None if p_split is None else p_split.data_ptr(), R.data_ptr(),
                                           None if nonzero is None else nonzero.data_ptr(),
                                           ws.data_ptr(), ws.numel(), self._stream())
        _lib.check(rc, "dion_project_r")

    def project_r_fixup(self, momentums: List[torch.Tensor], P: torch.Tensor, R: torch.Tensor,
                        qs: List[torch.Tensor], nonzero: torch.Tensor, eps: float, transposed: bool,
                        p_split: Optional[torch.Tensor] = None) -> None:
        """project_r then fixup_colnorm(P=None, ...) in one call (fp32 state; the W = 1 path
        after orthonormalize(fix_nonzero=...)): the fix-up's first phase rides on pass B's
        split-K reduction.  runtime.py:1476-1477, kernels.py:157-210, 279-290."""
        B = len(momentums)
        if B == 0:
            return
        m, n = self._check_batch(momentums, momentums[0].dtype)
        r = int(P.shape[2])
        d = self._desc(B, m, n, r, transposed, M=momentums[0])
        ws = self.workspace(d, _lib.OP_PROJECT_R)
        rc = self.lib.dion_project_r_fixup(ctypes.byref(d), _ptrs(momentums), P.data_ptr(),
                                           None if p_split is None else p_split.data_ptr(), R.data_ptr(),
                                           nonzero.data_ptr(), _ptrs(qs), nonzero.data_ptr(), float(eps),
                                           ws.data_ptr(), ws.numel(), self._stream())
        _lib.check(rc, "dion_project_r_fixup")

    def fixup_colnorm(self, P: Optional[torch.Tensor], R: torch.Tensor, qs: List[torch.Tensor],
                      nonzero: torch.Tensor, eps: float, m: int, n: int, transposed: bool) -> None:
        """fix_all_zero_or_nan + column normalisation; Q states receive Q_new.  P=None: P was
        already fixed (orthonormalize(fix_nonzero=...))."""
        B = len(qs)
        if B == 0:
            return
        r = int(R.shape[2])
        d = self._desc(B, m, n, r, transposed, state_dtype=_state_dtype(None, qs))
        ws = self.workspace(d, _lib.OP_FIXUP_COLNORM)
        rc = self.lib.dion_fixup_colnorm(ctypes.byref(d), None if P is None else P.data_ptr(), R.data_ptr(), _ptrs(qs),
                                         nonzero.data_ptr(), float(eps), ws.data_ptr(), ws.numel(),
                                         self._stream())
        _lib.check(rc, "dion_fixup_colnorm")

    def fixup_colsum(self, P: torch.Tensor, R: torch.Tensor, qs: List[torch.Tensor], nonzero: torch.Tensor,
                     colsum: torch.Tensor, m: int, n: int, transposed: bool) -> None:
        """FS kind, first half of the column norm: fix-up of P and R (kernels.py:157-204, local zero
        test) and the local fp32 column sums of squares of R into colsum (B, r)
        (kernels.py:207-210).  The caller all-reduces colsum over the FS group."""
        B = len(qs)
        if B == 0:
            return
        r = int(P.shape[2])
        if colsum.dtype != torch.float32 or not colsum.is_contiguous() or colsum.numel() < B * r:
            raise RuntimeError("[DION_BAD_COLSUM] colsum must be a contiguous fp32 (batch, r) buffer")
        d = self._desc(B, m, n, r, transposed, state_dtype=_state_dtype(None, qs))
        ws = self.workspace(d, _lib.OP_FIXUP_COLNORM)
        rc = self.lib.dion_fixup_colsum(ctypes.byref(d), P.data_ptr(), R.data_ptr(), _ptrs(qs), nonzero.data_ptr(),
                                        colsum.data_ptr(), ws.data_ptr(), ws.numel(), self._stream())
        _lib.check(rc, "dion_fixup_colsum")

    def colnorm_apply(self, R: torch.Tensor, qs: List[torch.Tensor], colsum: torch.Tensor, eps: float,
                      m: int, n: int, transposed: bool) -> None:
        """FS kind, second half: Q_b <- R_b / (sqrt(colsum_b) + eps) (kernels.py:279-290)."""
        B = len(qs)
        if B == 0:
            return
        r = int(R.shape[2])
        d = self._desc(B, m, n, r, transposed, state_dtype=_state_dtype(None, qs))
        rc = self.lib.dion_colnorm_apply(ctypes.byref(d), R.data_ptr(), _ptrs(qs), colsum.data_ptr(), float(eps),
                                         self._stream())
        _lib.check(rc, "dion_colnorm_apply")

    def ef_apply(self, momentums: Optional[List[torch.Tensor]], params: Optional[List[torch.Tensor]],
                 P: torch.Tensor, R: torch.Tensor, qs: List[torch.Tensor], nonzero: torch.Tensor,
                 mu: float, lr: float, wd: float, scaled_lr: float, transposed: bool) -> None:
        """Error feedback and weight update.  kernels.py:54-154, runtime.py:1105-1113.

        `momentums=None` updates the weights only (deferred-EF schedule); `params=None`
        applies the error feedback only."""
        B = len(qs)
        if B == 0:
            return
        if momentums is None and params is None:
            raise RuntimeError("[DION_INTERNAL] ef_apply needs momentums or params")
        sdt = _state_dtype(momentums, qs)
        if momentums is not None:
            m, n = self._check_batch(momentums, sdt)
        if params is not None:
            m, n = self._check_batch(params)
        r = int(P.shape[2])
        if not (P.is_contiguous() and R.is_contiguous()):
            raise RuntimeError("[DION_BAD_FACTOR] P and R must be contiguous (batch, rows, r)")
        d = self._desc(B, m, n, r, transposed, M=momentums[0] if momentums else None,
                       W=params[0] if params else None, state_dtype=sdt)
        ws = None  # the update splits its factors in-kernel (no workspace)
        rc = self.lib.dion_ef_apply(ctypes.byref(d), _ptrs(momentums) if momentums else None,
                                    _ptrs(params) if params else None,
                                    P.data_ptr(), R.data_ptr(), _ptrs(qs), nonzero.data_ptr(), float(mu),
                                    float(lr), float(wd), float(scaled_lr), None if ws is None else ws.data_ptr(),
                                    0 if ws is None else ws.numel(), self._stream())
        _lib.check(rc, "dion_ef_apply")

    def round_bf16(self, X: torch.Tensor) -> None:
        """X <- bf16(X) in place (fp32 storage): the bf16 state's rounding after an averaging
        collective on P or R (the reference reduces bf16 tensors, runtime.py:1428-1434, 1485-1491)."""
        if X.dtype != torch.float32 or not X.is_contiguous():
            raise RuntimeError(f"[DION_BAD_FACTOR] round_bf16 needs a contiguous fp32 buffer, got {X.dtype}")
        _lib.check(self.lib.dion_round_bf16(X.data_ptr(), X.numel(), self._stream()), "dion_round_bf16")

    def grad_sum_sq(self, grads: Sequence[torch.Tensor], out: torch.Tensor) -> None:
        """out (fp64, (1,)) += sum of squares of every gradient (grad_norm.py:54-68, :144-258)."""
        if out.dtype != torch.float64 or out.numel() != 1 or out.device != self.device:
            raise RuntimeError("[DION_BAD_NORM_OUT] out must be one float64 on the codec's device")
        groups = {}
        for g in grads:
            if g.dim() != 2 or g.stride(1) != 1:
                raise RuntimeError(f"[DION_NON_ROW_MAJOR] grad shape={tuple(g.shape)} stride={g.stride()}")
            groups.setdefault((tuple(g.shape), g.dtype, g.stride(0)), []).append(g)
        for (shape, _, _), members in groups.items():
            d = _lib.DionBatchDesc()
            d.batch = len(members)
            d.m, d.n, d.r = int(shape[0]), int(shape[1]), 1
            d.g_dtype = _dtype_code(members[0])
            d.m_dtype = d.w_dtype = _lib.DTYPE_F32
            d.ld_g = _row_stride(members[0])
            ws = self.workspace(d, _lib.OP_GRAD_SUM_SQ)
            rc = self.lib.dion_grad_sum_sq(ctypes.byref(d), _ptrs(members), out.data_ptr(), ws.data_ptr(),
                                           ws.numel(), self._stream())
            _lib.check(rc, "dion_grad_sum_sq")

    # ------------------------------------------------------------------ elementwise branch
    def _ew_lists(self, params, grads, moments):
        for t in params:
            if t.dtype != torch.float32 or not t.is_contiguous() or t.device != self.device:
                raise RuntimeError(f"[DION_ELEMENTWISE_STATE_DTYPE_UNSUPPORTED] param {t.dtype} {tuple(t.shape)} "
                                   f"{t.device}; the elementwise kernel takes contiguous fp32 params")
        for ms in moments:  # each moment list has its own dtype (momentum_dtype / variance_dtype)
            mdt = ms[0].dtype if ms else torch.float32
            for t in ms:
                if t.dtype != mdt or mdt not in (torch.float32, torch.bfloat16) or not t.is_contiguous() \
                        or t.device != self.device:
                    raise RuntimeError(f"[DION_ELEMENTWISE_STATE_DTYPE_UNSUPPORTED] moment {t.dtype} "
                                       f"{tuple(t.shape)}; each moment list is contiguous fp32 or bf16 of one dtype")
        by_gdt = {}
        for i, g in enumerate(grads):
            if not g.is_contiguous() or g.numel() != params[i].numel():
                raise RuntimeError(f"[DION_ELEMENTWISE_BAD_GRAD] {tuple(g.shape)} for param {tuple(params[i].shape)}")
            by_gdt.setdefault(_dtype_code(g), []).append(i)
        return by_gdt

    def elementwise_adamw(self, params, grads, first_moments, second_moments, *, lr, beta1, beta2, weight_decay,
                          step, epsilon) -> None:
        """elementwise_opts.py:45-80 in one multi-tensor pass (dion_elementwise_adamw)."""
        for gdt, idx in self._ew_lists(params, grads, (first_moments, second_moments)).items():
            numels = (ctypes.c_int64 * len(idx))(*[int(params[i].numel()) for i in idx])
            rc = self.lib.dion_elementwise_adamw(
                len(idx), numels, _ptrs([params[i] for i in idx]), _ptrs([grads[i] for i in idx]), gdt,
                _dtype_code_state(first_moments[0].dtype), _dtype_code_state(second_moments[0].dtype),
                _ptrs([first_moments[i] for i in idx]), _ptrs([second_moments[i] for i in idx]), float(lr),
                float(beta1), float(beta2), float(weight_decay), float(epsilon), int(step), self._stream())
            _lib.check(rc, "dion_elementwise_adamw")

    def elementwise_lion(self, params, grads, first_moments, *, lr, beta1, beta2, weight_decay) -> None:
        """elementwise_opts.py:83-105 in one multi-tensor pass (dion_elementwise_lion)."""
        for gdt, idx in self._ew_lists(params, grads, (first_moments,)).items():
            numels = (ctypes.c_int64 * len(idx))(*[int(params[i].numel()) for i in idx])
            rc = self.lib.dion_elementwise_lion(
                len(idx), numels, _ptrs([params[i] for i in idx]), _ptrs([grads[i] for i in idx]), gdt,
                _dtype_code_state(first_moments[0].dtype),
                _ptrs([first_moments[i] for i in idx]), float(lr), float(beta1), float(beta2), float(weight_decay),
                self._stream())
            _lib.check(rc, "dion_elementwise_lion")

