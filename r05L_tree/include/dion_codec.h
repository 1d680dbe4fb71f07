/*
 * dion_codec.h -- C ABI of the MI355X (gfx950) Dion gradient codec.
 *
 * Replaces the device work of the reference's Dion hot path
 *   /root/reference/megatron/core/optimizer/dion/runtime.py:1499-1911
 *   (batch_dion_update_async) and the helpers it calls.
 * Each entry point below names the reference code it stands in for.
 *
 * Conventions:
 *  - every function returns DION_OK (0) or a negative DION_E_* code; the text
 *    of the last failure on the calling thread is dion_last_error();
 *  - no allocation and no host synchronisation inside; everything is enqueued
 *    on `stream` (a hipStream_t; torch.cuda.current_stream().cuda_stream);
 *  - stateless and re-entrant; the caller owns every buffer;
 *  - one matrix per pointer (pointer arrays, host memory, `desc->batch`
 *    entries) exactly like the reference's per-parameter tensors; the small
 *    factors P, R are one contiguous (batch, rows, r) fp32 buffer each, like
 *    the reference's P_batch / R_batch;
 *  - M, W are fp32 row-major m x n (row stride ld_m / ld_w elements); G is
 *    bf16 or fp32 row-major (ld_g); Q is fp32 n_Q x r contiguous per matrix;
 *  - bf16 state mode (m_dtype == DION_DTYPE_BF16: the speedrun's
 *    --dion-momentum-dtype/--dion-q-dtype bfloat16, speedrun_nanogpt_mcore.py:422-431):
 *    every M and Q pointer then addresses bf16 (uint16) data, W stays fp32, and the
 *    fp32 P / R buffers hold bf16-representable values, rounded (nearest even)
 *    wherever the reference's bf16 tensors round (runtime.py:1560-1616, ortho.py:123,
 *    kernels.py:54-83, 229-290).  dion_project_p_ef exists in this mode for r a multiple
 *    of 32 and a bf16 (or no) gradient on whole streaming blocks (its workspace query
 *    says which); elsewhere it is DION_E_UNSUPPORTED;
 *  - orientation follows the reference's DionParamConfig.is_transposed
 *    (dion/state.py:304-310): transposed == 0 => P has m rows (P = M Q),
 *    transposed == 1 => P has n rows (P = M^T Q).  m_P = transposed ? n : m,
 *    n_Q = transposed ? m : n.
 */
#ifndef DION_CODEC_H_
#define DION_CODEC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* dion_stream_t; /* == hipStream_t */

#define DION_ABI_VERSION 15

#define DION_OK 0
#define DION_E_INVALID (-1)     /* bad descriptor / null pointer / misuse       */
#define DION_E_UNSUPPORTED (-2) /* shape or dtype outside the built kernels     */
#define DION_E_LAUNCH (-3)      /* HIP launch failure                           */
#define DION_E_WORKSPACE (-4)   /* workspace smaller than dion_workspace_bytes  */

#define DION_DTYPE_NONE 0
#define DION_DTYPE_F32 1
#define DION_DTYPE_BF16 2

/* operations that need scratch (argument `op` of dion_workspace_bytes) */
#define DION_OP_PROJECT_P 1
#define DION_OP_ORTHONORMALIZE 2
#define DION_OP_PROJECT_R 3
#define DION_OP_FIXUP_COLNORM 4
#define DION_OP_PROJECT_P_EF 5 /* DION_E_UNSUPPORTED: no fused kernel for this shape */
#define DION_OP_EF_APPLY 6     /* optional: pre-split P for the rank-update kernels   */
#define DION_OP_GRAD_SUM_SQ 7  /* dion_grad_sum_sq (only batch, m, n, g_dtype, ld_g used) */
#define DION_OP_DORTHO 8       /* dion_dortho_sketch / dion_dortho_gram (row-sharded P)   */
#define DION_OP_PSPLIT 9       /* not scratch: bytes of the p_split buffer of
                                  dion_orthonormalize_fused / dion_project_r_split;
                                  DION_E_UNSUPPORTED: no fused split for this shape        */

typedef struct DionBatchDesc {
  int32_t batch;      /* matrices in this call (all the same shape)            */
  int32_t m, n;       /* storage shape of every M / G / W                      */
  int32_t r;          /* rank = columns of P, Q, R  (1..128)                   */
  int32_t transposed; /* reference DionParamConfig.is_transposed               */
  int32_t g_dtype;    /* DION_DTYPE_NONE (no accumulate), _F32 or _BF16        */
  int32_t m_dtype;    /* DION_DTYPE_F32, or _BF16 (bf16 momentum and Q)         */
  int32_t w_dtype;    /* DION_DTYPE_F32                                        */
  int64_t ld_g;       /* row strides in elements; 0 means n                    */
  int64_t ld_m;
  int64_t ld_w;
} DionBatchDesc;

/* ABI version of the loaded library (== DION_ABI_VERSION). */
int dion_abi_version(void);

/* Build id: the first 16 hex digits of the SHA-256 of the sources the library was compiled
 * from (csrc/dion_codec.hip, csrc/*.hpp, include/dion_codec.h; name + bytes, sorted by name),
 * passed by the build as -DDION_BUILD_ID.  The loader recomputes it from the in-tree sources
 * and refuses a library built from other sources.  No reference counterpart (build hygiene). */
const char* dion_build_id(void);

/* Text of the last error raised on this thread ("" if none). */
const char* dion_last_error(void);

/* Scratch bytes `op` needs for `desc` (0 is a valid answer). */
int dion_workspace_bytes(const DionBatchDesc* desc, int op, size_t* bytes);

/*
 * Pass A.  For every matrix b:  M_b += G_b (when g_dtype != NONE),
 *   P_b = X_b Q_b  with X_b = M_b (or M_b^T when transposed), fp32 (TF32 off),
 *   nonzero[b] != 0 iff some element of the accumulated M_b is != 0.
 * `nonzero` must be zeroed by the caller before the call.  A nonzero flag carries the
 * bit pattern of max |M_b| (fp32) when the kernel measured it, or a value >= 0x7F800000
 * (inf's bits) when it did not; hand the array to dion_project_r as `m_absmax`.
 * Replaces runtime.py:1560-1566 (momentum accumulate), :1602-1616 (stack +
 * P = M Q) and the all-zero test of kernels.py:185 (is_all_zero).
 */
int dion_project_p(const DionBatchDesc* desc, const void* const* G, float* const* M,
                   const float* const* Q, float* P, uint32_t* nonzero, void* ws,
                   size_t ws_bytes, dion_stream_t stream);

/* The previous step's error feedback, not yet applied to M (see dion_project_p_ef). */
typedef struct DionPendingEF {
  const float* const* P; /* per matrix: its m_P x r factor P_b of the previous step (after the
                            fix-up: orthonormal or zero columns, every |x| < 2; the fp32 kernels
                            split it on the fixed scale 2^14), or NULL */
  const float* const* R; /* per matrix: its n_Q x r factor R_b of the previous step, or NULL */
  float alpha;           /* -(1 - mu) of that step */
} DionPendingEF;

/*
 * Pass A with the previous step's error feedback folded in ("deferred EF"):
 *   M_b <- (M_b + alpha (P_b R_b^T or R_b P_b^T)) + G_b ;  P = X_b Q_b ;  nonzero
 * for every entry whose pending factors are non-NULL (the rest as dion_project_p).
 * Same sums, same order as the eager schedule (error feedback of step t,
 * kernels.py:54-154, then M += G of step t+1, runtime.py:1560-1566), but the
 * momentum is read and written once instead of twice.  bf16 state: the eager
 * update's M = rne(M + rne(alpha rne(P R^T))) on the same value (each element, before
 * its gradient), the increment from fp32 sums of the exact bf16 products.  Returns
 * DION_E_UNSUPPORTED (and enqueues nothing) for shapes without the fused kernel
 * (query: dion_workspace_bytes(desc, DION_OP_PROJECT_P_EF, ...)); the caller then
 * applies the pending EF with dion_ef_apply(W = NULL) and calls dion_project_p.
 */
int dion_project_p_ef(const DionBatchDesc* desc, const void* const* G, float* const* M,
                      const float* const* Q, float* P, uint32_t* nonzero, const DionPendingEF* ef,
                      void* ws, size_t ws_bytes, dion_stream_t stream);

/*
 * Randomised Cholesky QR of every P_b (m_P x r), in place
 *   (ortho.py:71-123 orthogonalize):  m_P <= r: Q factor of a Householder QR;
 *   else R1 = qr(S P).R, P <- P R1^-1, R2 = chol_upper(P^T P), P <- P R2^-1,
 *   with S ~ N(0, 1/k), k = ceil(oversample r / 128) * 128.
 * `sketch` (batch x k x m_P fp32, row-major) is used when non-null (parity
 * tests); otherwise S is generated on the fly from (seed, b, row, col) by a
 * counter-based hash as a Rademacher matrix, entries +-1/sqrt(k) (exact in bf16),
 * in place of the reference's unseeded N(0, 1/k) draw (ortho.py:643-662): the
 * orthonormalised P is the Q factor of P whatever the sketch, up to column signs
 * (tests/test_gpu_fullsize.py compares the generated path with the oracle's
 * Gaussian-sketch step at bench shapes).
 */
int dion_orthonormalize(const DionBatchDesc* desc, float* P, const float* sketch,
                        uint64_t seed, float oversample, void* ws, size_t ws_bytes,
                        dion_stream_t stream);

/*
 * Distributed randomised Cholesky QR of a row-sharded P (the "fsdp_tp" kernel kind: P's
 * rows are split over the TP group, dion/ortho.py:682-834 distributed_orthogonalize).
 * The collectives stay with the caller; these are the per-rank pieces between them:
 *
 *   dion_dortho_sketch:   SP_b = S_b[:, rows] P_b  (k x r per entry, fp32), the local
 *                         rows' share of the sketch product (ortho.py:777-787), to be
 *                         reduced (sum) over the group.  `desc` describes the LOCAL shard
 *                         (m_P local rows, which may be fewer than r); `row_offset` is the
 *                         global index of this rank's first P row, so a generated sketch is
 *                         the same global S on every rank (ortho.py:575-640 slices one
 *                         seeded draw the same way); `sketch` (batch x k x m_P local) may
 *                         be given instead.  Scratch: DION_OP_DORTHO.
 *   dion_dortho_qr_inv:   R1inv_b = qr(SP_b).R ^ -1  (r x r; ortho.py:791-792, the solve of
 *                         :799-806 becomes a product with the inverse).
 *   dion_dortho_apply:    P_out_b = P_in_b Uinv_b  (ortho.py:799-806, 821-828).
 *   dion_dortho_gram:     gram_b = P_b^T P_b  (r x r), the local rows' share (ortho.py:808-812).
 *   dion_dortho_chol_inv: R2inv_b = chol_upper(gram_b) ^ -1 (ortho.py:813-814; a failed
 *                         pivot poisons the columns from it on with NaN, as cholesky_ex).
 */
int dion_dortho_sketch(const DionBatchDesc* desc, const float* P, const float* sketch, uint64_t seed,
                       int64_t row_offset, float oversample, float* SP, void* ws, size_t ws_bytes,
                       dion_stream_t stream);
int dion_dortho_qr_inv(int32_t k, int32_t r, int32_t batch, const float* SP, float* R1inv,
                       dion_stream_t stream);
int dion_dortho_apply(const DionBatchDesc* desc, const float* P_in, const float* Uinv, float* P_out,
                      dion_stream_t stream);
int dion_dortho_gram(const DionBatchDesc* desc, const float* P, float* gram, void* ws, size_t ws_bytes,
                     dion_stream_t stream);
int dion_dortho_chol_inv(int32_t r, int32_t batch, const float* gram, float* R2inv, dion_stream_t stream);

/*
 * Pass B.  R_b = X_b^T P_b  (n_Q x r), fp32.  runtime.py:1476-1477.
 * `m_absmax` (optional, may be NULL): the `nonzero` flags pass A left for exactly these
 * M_b.  A finite max |M_b| lets the fp16x3 kernel use one power-of-two scale per matrix
 * instead of one per column and step (same accuracy, fewer instructions); other values
 * or NULL select the per-step scales.
 */
int dion_project_r(const DionBatchDesc* desc, const float* const* M, const float* P,
                   float* R, const uint32_t* m_absmax, void* ws, size_t ws_bytes,
                   dion_stream_t stream);

/*
 * The W = 1 path with fewer passes over P (same results as dion_orthonormalize,
 * dion_project_r and dion_fixup_colnorm in that order, for every input those reach:
 * an orthonormalised P is NaN only in whole columns, and a whole NaN column gives
 * R = 0 in that column either way).
 * dion_orthonormalize_fused: dion_orthonormalize, then
 *   `nonzero` (optional): the fix-up of P, P_b <- z ? 0 : nan_to_num(P_b) (in the last
 *     solve's epilogue where it can; dion_fixup_colnorm is then called with P = NULL);
 *   `p_split` (optional, DION_OP_PSPLIT bytes, 16-byte aligned): the fp16x3 limbs of the
 *     final P in pass B's operand layout on the fixed scale 2^14 (|P| <= 1: orthonormal
 *     columns), written by the last solve; DION_E_UNSUPPORTED (nothing enqueued) when
 *     DION_OP_PSPLIT is unsupported for this desc.
 * dion_project_r_split: dion_project_r reading P's limbs from `p_split` (NULL: as
 *   dion_project_r); a pass B whose h3 kernel does not run for these pointers ignores it.
 * No reference counterpart beyond the functions they fuse (ortho.py:71-123,
 * runtime.py:1476-1477, kernels.py:185-188).
 */
int dion_orthonormalize_fused(const DionBatchDesc* desc, float* P, const float* sketch, uint64_t seed,
                              float oversample, const uint32_t* nonzero, void* p_split, void* ws,
                              size_t ws_bytes, dion_stream_t stream);
int dion_project_r_split(const DionBatchDesc* desc, const float* const* M, const float* P,
                         const void* p_split, float* R, const uint32_t* m_absmax, void* ws,
                         size_t ws_bytes, dion_stream_t stream);
/*
 * dion_project_r_fixup: dion_project_r_split, then dion_fixup_colnorm with P = NULL (the P
 * half done by dion_orthonormalize_fused), bitwise; the fix-up's first phase rides on pass
 * B's split-K reduction.  fp32 state only (DION_E_UNSUPPORTED otherwise, nothing enqueued);
 * scratch = dion_workspace_bytes(DION_OP_PROJECT_R), which includes the fix-up's partials.
 */
int dion_project_r_fixup(const DionBatchDesc* desc, const float* const* M, const float* P,
                         const void* p_split, float* R, const uint32_t* m_absmax, float* const* Q,
                         const uint32_t* nonzero, float eps, void* ws, size_t ws_bytes,
                         dion_stream_t stream);

/*
 * fix_all_zero_or_nan (kernels.py:157-204) + column normalisation
 * (kernels.py:207-210, 279-290) + Q commit (runtime.py:1132), for the
 * `desc->batch` real entries:
 *   z = !nonzero[b];  P_b <- z ? 0 : nan_to_num(P_b)   (skipped when P is NULL: fixed by
 *                                                     dion_orthonormalize_fused);
 *   R_b <- z ? nan_to_num(Q_b) : nan_to_num(R_b);
 *   Q_b <- R_b / (sqrt(sum_rows R_b^2) + eps)          (Q_b is overwritten)
 */
int dion_fixup_colnorm(const DionBatchDesc* desc, float* P, float* R, float* const* Q,
                       const uint32_t* nonzero, float eps, void* ws, size_t ws_bytes,
                       dion_stream_t stream);

/*
 * The column norm split in two for the FS ("fsdp") kernel kind, where every rank holds a
 * shard of R's rows and the sums of squares are all-reduced over the FS group between
 * the halves (q_norm_group, runtime.py:965-1013):
 *
 * dion_fixup_colsum: the fix-up of dion_fixup_colnorm on P and R (in place; the zero
 * test is the caller's local shard, as the reference's local M_batch) and
 *   colsum[b][c] = sum_rows R_b[.][c]^2            (fp32, fixed order; kernels.py:207-210)
 * `colsum` is (batch, r) fp32; scratch = dion_workspace_bytes(DION_OP_FIXUP_COLNORM).
 *
 * dion_colnorm_apply:  Q_b <- R_b / (sqrt(colsum_b) + eps)   (kernels.py:279-290;
 * bf16 state: the quotient rounded to bf16).  `colsum` is the reduced (batch, r) sum.
 */
int dion_fixup_colsum(const DionBatchDesc* desc, float* P, float* R, const void* const* Q,
                      const uint32_t* nonzero, float* colsum, void* ws, size_t ws_bytes,
                      dion_stream_t stream);
int dion_colnorm_apply(const DionBatchDesc* desc, const float* R, void* const* Q, const float* colsum,
                       float eps, dion_stream_t stream);

/*
 * Error feedback + weight update (kernels.py:54-154, 229-276; runtime.py:1105-1113):
 *   M_b += -(1-mu) * (P_b R_b^T  or  R_b P_b^T when transposed)
 *   W_b  = (wd > 0 ? (1 - lr*wd) : 1) * W_b - scaled_lr * (P_b Qn_b^T or Qn_b P_b^T)
 * Qn_b is the committed Q (output of dion_fixup_colnorm).  W may be NULL
 * (error feedback only); M may be NULL (weight update only, the deferred-EF
 * schedule; DION_E_UNSUPPORTED for shapes without the rank-update kernel).
 * Entries with nonzero[b] == 0 keep M and only decay W.
 * `ws` is optional: with dion_workspace_bytes(desc, DION_OP_EF_APPLY) bytes the
 * streamed factor P is split into bf16 limbs once per call instead of per tile.
 * The hyper-parameters are the reference's Python doubles (ABI 12): -(1 - mu), 1 - lr*wd
 * and -scaled_lr are formed in double and rounded to fp32 once, as torch casts a Python
 * scalar operand (kernels.py:54-83 _foreach_mul(update, alpha); runtime.py:1110-1113
 * W.mul_(1 - lr*wd), W.add_(delta, alpha=-scaled_lr)).
 */
int dion_ef_apply(const DionBatchDesc* desc, float* const* M, float* const* W,
                  const float* P, const float* R, const float* const* Qn,
                  const uint32_t* nonzero, double mu, double lr, double wd, double scaled_lr,
                  void* ws, size_t ws_bytes, dion_stream_t stream);

/*
 * x[i] <- bf16(x[i]) (round to nearest even, kept in fp32 storage), i < n.
 * The bf16 state mode's rounding after a collective that averages an fp32
 * buffer of bf16 values (the reference reduces bf16 P / R tensors:
 * runtime.py:1428-1434 reduce-scatter, :1485-1491 all-reduce).
 */
int dion_round_bf16(float* x, int64_t n, dion_stream_t stream);

/*
 * *out += sum_b sum_ij G_b[i][j]^2, in fp64 (every square exact, fixed summation
 * order: bitwise reproducible).  The Dion term of the gradient norm that gradient
 * clipping needs before the step: replaces distrib_dion/grad_norm.py:54-68
 * (_grad_sum_sq_fp64) as used by _dion_grad_norm_sq (:144-258).  `out` is one
 * device double the caller zeroes; only batch, m, n, g_dtype (_F32 / _BF16) and
 * ld_g of `desc` are read.  Scratch: dion_workspace_bytes(desc, DION_OP_GRAD_SUM_SQ).
 */
int dion_grad_sum_sq(const DionBatchDesc* desc, const void* const* G, double* out, void* ws,
                     size_t ws_bytes, dion_stream_t stream);

/*
 * The elementwise branch of MegatronDion.step (algorithm.py:247-429) for one bucket of
 * n_tensors same-hyper-parameter tensors: W fp32; exp_avg (first_moment) in m1_dtype and
 * exp_avg_sq (second_moment) in m2_dtype (Lion: exp_avg in m_dtype), each DION_DTYPE_F32 or
 * _BF16 (the reference's independent momentum_dtype / variance_dtype, algorithm.py:308-332:
 * every foreach result rounded to its tensor's dtype as torch does, g*g in the first
 * moment's dtype then cast to the second's, m / denom in the promoted dtype); G fp32 or
 * bf16 (g_dtype); numels[i] elements each, contiguous.  ABI 11 split m_dtype in two.
 * One read and one write of every tensor replaces the reference's chain of
 * torch._foreach_* passes:
 *   AdamW  elementwise_opts.py:45-80:  m = lerp(m, g, 1-b1); v = lerp(v, g*g, 1-b2);
 *          W = W (1 - lr wd) - (m / (sqrt(v) / sqrt(1-b2^t) + eps)) (lr / (1-b1^t))
 *   Lion   elementwise_opts.py:83-105: u = sign(lerp(m, g, 1-b1)); m = lerp(m, g, 1-b2);
 *          W = W (1 - lr wd) - lr u
 * (the decay multiply only when weight_decay != 0).  Scalars are the reference's
 * Python doubles; step > 0 for AdamW ([DION_INVALID_ELEMENTWISE_ADAMW_STEP]).
 */
int dion_elementwise_adamw(int32_t n_tensors, const int64_t* numels, float* const* W, const void* const* G,
                           int32_t g_dtype, int32_t m1_dtype, int32_t m2_dtype, void* const* exp_avg,
                           void* const* exp_avg_sq, double lr, double beta1, double beta2, double weight_decay,
                           double eps, int32_t step, dion_stream_t stream);
int dion_elementwise_lion(int32_t n_tensors, const int64_t* numels, float* const* W, const void* const* G,
                          int32_t g_dtype, int32_t m_dtype, void* const* exp_avg, double lr, double beta1,
                          double beta2, double weight_decay, dion_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* DION_CODEC_H_ */
