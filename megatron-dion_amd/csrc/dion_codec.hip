// dion_codec.hip -- MI355X (gfx950, CDNA4) kernels of the Dion gradient codec.
//
// What each kernel replaces in the reference (all paths under
// /root/reference/megatron/core/optimizer/):
//   rowproj_kernel / colproj_kernel  dion/runtime.py:1560-1616 (M += G, P = M Q),
//                                     dion/runtime.py:1476-1477 (R = M^T P)
//   sketch_rad_kernel, sketch_qr_inv_kernel, gram_h3_kernel, chol_reg_kernel,
//   tsolve_mfma_kernel (explicit-inverse solves; trsm_* substitution kernels for other r)
//                                     dion/ortho.py:71-123 (randomised Cholesky QR)
//   fixup_partial / colnorm_apply / reduce_fix_partial, pfix_kernel
//                                     dion/kernels.py:157-210, 279-290
//   ef_update_kernel                  dion/kernels.py:54-154, 229-276;
//                                     dion/runtime.py:1105-1113
//
// Design (DESIGN.md has the long form):
//  * All arithmetic is fp32 (the reference disables TF32, ortho.py:25-45); the
//    contractions run on the exact-f32 MFMA (v_mfma_f32_16x16x4_f32 for the
//    projections, v_mfma_f32_32x32x2_f32 for the rank-r updates), which is a
//    k-ordered fmaf chain.
//  * The big operand (momentum M, m x n fp32 row-major) is streamed once per
//    pass straight into MFMA operand registers with 16-byte loads: for P = M Q
//    each lane reads 8 consecutive columns of one row (16 rows x 128 B per
//    load pair), for R = M^T P each lane reads 4 consecutive columns
//    (4 rows x 256 B per load).  The K order inside an MFMA is free, so no LDS
//    transpose is needed.  The thin operand (Q or P, <= 1 MB) is L2-resident.
//  * Split-K partials go to fp32 slabs in the caller's workspace and are summed
//    by a deterministic reduction (no float atomics: bitwise-reproducible).
//  * Per-matrix pointers travel in the kernel-argument block (up to 64
//    matrices per launch), so there is no pointer-array upload.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <stdarg.h>

#include <type_traits>

#include "../../include/dion_codec.h"

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define MAXB 64  // matrices per launch (pointer arrays live in kernel arguments)

// Cache policy of the big once-touched streams (G, M, W): non-temporal ("nt") loads
// and stores.  Measured on MI355X (scripts/ubench/stream_modes.hip): an in-place
// read-modify-write stream rises from 5.2 to 5.8 TB/s and a read-only stream from
// 6.3 to 7.0 TB/s with nt on both sides.  Small factors (P, Q, R) keep the default
// policy: every block re-reads them from L2.
constexpr int kNt = 1;
// waves per block of the pass-B column kernel and its min-blocks-per-CU hint (measured defaults)
constexpr int kColx6Minb = 1;
constexpr int kStreamAux = kNt ? 2 : 0;  // buffer-op cache-policy bits (nt)
// streaming projection kernels: issue the next step's split-operand staging loads before the big
// operand's prefetch, so the wait before the LDS store retires only the split and the
// prefetch stays in flight across the barrier (measured default)
// (pass A kernels; _B: the pass-B kernels, measured neutral there)
constexpr int kSplitFirst = 1;
constexpr int kSplitFirstB = 0;

template <typename T>
__device__ __forceinline__ T ld_stream(const T* p) {
  if constexpr (kNt) return __builtin_nontemporal_load(p);
  else return *p;
}

// Row-kernel accesses cover a 128-B line in two instructions (64-B segments per
// row); nt on those re-fetches the line (measured 18 % slower on pass A), so they
// keep the default policy.
template <typename T>
__device__ __forceinline__ T ld_part(const T* p) { return *p; }
template <typename T>
__device__ __forceinline__ void st_part(T* p, const T& v) { *p = v; }

typedef unsigned u32x2_ __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 ld_stream(const uint4* p) {
  const u32x4 v = ld_stream(reinterpret_cast<const u32x4*>(p));
  return uint4{v[0], v[1], v[2], v[3]};
}
__device__ __forceinline__ uint2 ld_stream(const uint2* p) {
  const u32x2_ v = ld_stream(reinterpret_cast<const u32x2_*>(p));
  return uint2{v[0], v[1]};
}

template <typename T>
__device__ __forceinline__ void st_stream(T* p, const T& v) {
  if constexpr (kNt) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// ---- LDS-DMA staging (global_load_lds_dwordx4).  Lane l's 16 source bytes land at LDS
// byte lds_base + 16 l (lds_base wave-uniform, in M0).  Written as inline asm so that hipcc
// neither counts these loads in its own s_waitcnt bookkeeping nor drains them at a barrier
// or before an LDS read (with the builtin it waits vmcnt(0) before every ds_read of an LDS
// array it cannot tell apart from the DMA's target); completion is counted by hand
// (gl_wait_barrier).  Vector-memory operations retire in issue order on gfx9 (loads and
// stores share vmcnt), which the counts below rely on.
__device__ __forceinline__ uint32_t lds_off(const void* p) {
  return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) void*)p));
}
template <bool NT>
__device__ __forceinline__ void glds16(const void* sbase, uint32_t voff, uint32_t lds_base) {
  // saddr form: wave-uniform 64-bit base in SGPRs, the lane's 32-bit byte offset in a VGPR
  unsigned keep;
  if constexpr (NT)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds_base) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds_base) : "memory");
}
// wait until at most N of this wave's vector-memory operations are outstanding and its LDS
// operations are done, then the block barrier (the "memory" clobber keeps hipcc's LDS
// accesses on their side of it)
template <int N>
__device__ __forceinline__ void gl_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"i"(N) : "memory");
}

// ----------------------------------------------------------------------------- errors
static thread_local char g_err[512];

static int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
static int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

static int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(DION_E_LAUNCH, "%s: %s", what, hipGetErrorString(e));
  return DION_OK;
}

// ----------------------------------------------------------------------------- helpers
__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  return __uint_as_float(static_cast<uint32_t>(h) << 16);
}

__device__ __forceinline__ float nan_to_num(float x) {
  // torch.nan_to_num defaults: NaN -> 0, +inf -> FLT_MAX, -inf -> -FLT_MAX
  if (x != x) return 0.f;
  if (x == INFINITY) return 3.402823466e38f;
  if (x == -INFINITY) return -3.402823466e38f;
  return x;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Wave sum on the DPP network (no LDS permutes): quad swaps, half-row and row mirrors give
// every lane its 16-lane row sum, two row broadcasts carry rows 0-2 into row 3, and lane 63's
// total comes back as a wave-uniform value (scalar register).  6 VALU adds + 1 readlane,
// against wave_sum's 6 cross-lane permutes; another summation order than wave_sum's.
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROWS, 0xF, false));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dpp_f<0xB1>(v);        // quad_perm [1, 0, 3, 2]
  v += dpp_f<0x4E>(v);        // quad_perm [2, 3, 0, 1]
  v += dpp_f<0x141>(v);       // row_half_mirror
  v += dpp_f<0x140>(v);       // row_mirror
  v += dpp_f<0x142, 0xA>(v);  // row_bcast15 into rows 1, 3
  v += dpp_f<0x143, 0xC>(v);  // row_bcast31 into rows 2, 3
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}
template <int N>
__device__ __forceinline__ void wave_sum_dpp_n(float (&v)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += dpp_f<0xB1>(v[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += dpp_f<0x4E>(v[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += dpp_f<0x141>(v[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += dpp_f<0x140>(v[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += dpp_f<0x142, 0xA>(v[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += dpp_f<0x143, 0xC>(v[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v[i]), 63));
}

// N independent wave sums in the butterfly order of wave_sum (bit-identical to N calls):
// the N cross-lane permutes of a level are issued back to back, so their latencies overlap
template <int N>
__device__ __forceinline__ void wave_sum_n(float (&v)[N]) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += __shfl_xor(v[i], off, 64);
}

// Counter-based N(0,1) draw for the on-device sketch: two 32-bit outputs of a
// splitmix64-style mix of (seed, row, col) feed Box-Muller.  Stateless, so any
// tile of S can be regenerated anywhere without storing S in HBM.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ float gauss(uint64_t seed, uint32_t row, uint32_t col) {
  const uint64_t h = mix64(seed ^ mix64((static_cast<uint64_t>(row) << 32) | col));
  const float u1 = (static_cast<float>(static_cast<uint32_t>(h >> 40)) + 0.5f) * (1.0f / 16777216.0f);
  const float u2 = static_cast<float>(static_cast<uint32_t>(h & 0xFFFFFFu)) * (1.0f / 16777216.0f);
  return sqrtf(-2.0f * __logf(u1)) * __cosf(6.283185307179586f * u2);
}

// ----------------------------------------------------------------------------- args
struct ProjArgs {
  const void* g[MAXB];     // gradient per matrix (pass A) or null
  float* m[MAXB];          // momentum per matrix (read; written when G present)
  const float* thin[MAXB]; // thin operand per matrix: Q (pass A) or P_b (pass B) or P_b (panels)
  float* out;              // (batch, nchunk, out_rows, r) slab or final (nchunk == 1)
  uint32_t* nonzero;       // per-matrix nonzero flags (pass A) or null
  const float* sketch;     // explicit sketch (batch, k, m_P) or null
  uint64_t seed;
  long sketch_row0;        // generated sketch: global index of P's first row (row-sharded P)
  float sketch_std;
  int rows, cols, r;       // X is rows x cols; thin is (rows or cols) x r
  long ld_m, ld_g;
  int kchunk, nchunk, out_rows;
  int vec;                 // 16-byte loads allowed
  const void* tsplit;      // thin operand pre-split (presplit_kernel layout 0, KMAP 0) for the x6 kernels
  long ts_stride;          // 16-byte units per matrix of tsplit
  const float* tinv;       // h3 kernels: 1 / scale of each matrix's thin-operand split
  const uint32_t* mabs;    // pass B: pass A's flag per matrix (max |M_b| bits when measured) or null
};

// The nonzero flag pass A leaves per matrix (DionBatchDesc docs, dion_project_p): 0 iff
// every element of the accumulated M_b is +-0; otherwise the bit pattern of max |M_b|
// (non-negative floats order like their bits) when the kernel measured it, or kAbsUnknown
// (inf's bits; NaN's sort above) when it did not.  Combined across blocks with atomicMax.
constexpr uint32_t kAbsUnknown = 0x7F800000u;

// ============================================================================
// Row projection:  out[b][i][c] = sum_j X_b[i][j] * T_b[j][c]    (X = M (+ G))
//   P = M Q for is_transposed == 0 (pass A) and R = M P for is_transposed == 1
//   (pass B).  256 threads = 4 waves, wave tile 32 rows x r, block 128 rows,
//   split-K over columns (blockIdx.y).  MFMA 16x16x4 f32:
//   A operand lane l = X[row0 + (l&15)][j0 + 8*(l>>4) + s], s = 0..7 (one
//   16-byte load pair per lane = 128 contiguous bytes per row per wave);
//   B operand lane l = T[j0 + 8*(l>>4) + s][16*cb + (l&15)].
// ============================================================================
template <int GDT>
__device__ __forceinline__ void load_row8(const ProjArgs& a, float* __restrict__ M,
                                          const void* __restrict__ G, int row, int jj, int j_end,
                                          float (&x)[8], bool& nz) {
  if (row >= a.rows) {
#pragma unroll
    for (int s = 0; s < 8; ++s) x[s] = 0.f;
    return;
  }
  float* p = M + static_cast<long>(row) * a.ld_m + jj;
  if (a.vec && jj + 8 <= j_end) {
    f32x4 v0 = *reinterpret_cast<const f32x4*>(p);
    f32x4 v1 = *reinterpret_cast<const f32x4*>(p + 4);
    if constexpr (GDT == DION_DTYPE_F32) {
      const float* gp = static_cast<const float*>(G) + static_cast<long>(row) * a.ld_g + jj;
      v0 += *reinterpret_cast<const f32x4*>(gp);
      v1 += *reinterpret_cast<const f32x4*>(gp + 4);
    } else if constexpr (GDT == DION_DTYPE_BF16) {
      const uint16_t* gp = static_cast<const uint16_t*>(G) + static_cast<long>(row) * a.ld_g + jj;
      const uint4 gv = *reinterpret_cast<const uint4*>(gp);
      v0[0] += __uint_as_float(gv.x << 16);
      v0[1] += __uint_as_float(gv.x & 0xFFFF0000u);
      v0[2] += __uint_as_float(gv.y << 16);
      v0[3] += __uint_as_float(gv.y & 0xFFFF0000u);
      v1[0] += __uint_as_float(gv.z << 16);
      v1[1] += __uint_as_float(gv.z & 0xFFFF0000u);
      v1[2] += __uint_as_float(gv.w << 16);
      v1[3] += __uint_as_float(gv.w & 0xFFFF0000u);
    }
    if constexpr (GDT != DION_DTYPE_NONE) {
      *reinterpret_cast<f32x4*>(p) = v0;
      *reinterpret_cast<f32x4*>(p + 4) = v1;
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      x[s] = v0[s];
      x[s + 4] = v1[s];
    }
  } else {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      float v = 0.f;
      if (jj + s < j_end) {
        v = p[s];
        if constexpr (GDT == DION_DTYPE_F32) {
          v += static_cast<const float*>(G)[static_cast<long>(row) * a.ld_g + jj + s];
        } else if constexpr (GDT == DION_DTYPE_BF16) {
          v += bf16_to_f32(static_cast<const uint16_t*>(G)[static_cast<long>(row) * a.ld_g + jj + s]);
        }
        if constexpr (GDT != DION_DTYPE_NONE) p[s] = v;
      }
      x[s] = v;
    }
  }
  if constexpr (GDT != DION_DTYPE_NONE) {
#pragma unroll
    for (int s = 0; s < 8; ++s) nz |= (x[s] != 0.f);
  }
}

template <int RB, int GDT>
__global__ void __launch_bounds__(256) rowproj_kernel(const ProjArgs a) {
  const int b = blockIdx.z;
  const int kc = blockIdx.y;
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int t = lane & 15;
  const int g = lane >> 4;
  const int row_base = blockIdx.x * 128 + wave * 32;
  const int j_begin = kc * a.kchunk;
  const int j_end = min(a.cols, j_begin + a.kchunk);
  float* __restrict__ M = a.m[b];
  const void* __restrict__ G = a.g[b];
  const float* __restrict__ T = a.thin[b];
  const int r = a.r;

  f32x4 acc[2][RB];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) acc[rb][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  bool nz = false;

  for (int j0 = j_begin; j0 < j_end; j0 += 32) {
    const int jj = j0 + 8 * g;
    float xv[2][8];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) load_row8<GDT>(a, M, G, row_base + 16 * rb + t, jj, j_end, xv[rb], nz);
    float tv[8][RB];
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int cb = 0; cb < RB; ++cb) {
        const int j = jj + s;
        const int c = 16 * cb + t;
        tv[s][cb] = (j < j_end && c < r) ? T[static_cast<long>(j) * r + c] : 0.f;
      }
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int cb = 0; cb < RB; ++cb)
          acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[rb][s], tv[s][cb], acc[rb][cb], 0, 0, 0);
  }

  float* out = a.out + (static_cast<long>(b) * a.nchunk + kc) * a.out_rows * r;
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = row_base + 16 * rb + 4 * g + q;
        const int c = 16 * cb + t;
        if (row < a.rows && c < r) out[static_cast<long>(row) * r + c] = acc[rb][cb][q];
      }
  if constexpr (GDT != DION_DTYPE_NONE) {
    if (a.nonzero != nullptr && __any(nz) && lane == 0) atomicMax(&a.nonzero[b], kAbsUnknown);
  }
}

// ============================================================================
// Column projection:  out[b][j][c] = sum_i X_b[i][j] * T_b[i][c]
//   P = M^T Q for is_transposed == 1 (pass A), R = M^T P for is_transposed == 0
//   (pass B); in PANEL mode also the RCQR reductions S P (X = S^T, generated or
//   explicit) and P^T P (X = P).
//   MFMA 16x16x4 f32: A operand lane l = X[i0 + (l>>4)][col0 + 4*(l&15) + e]
//   (one 16-byte load per lane covers 4 rows x 256 contiguous bytes), block e
//   of the output holds columns col0 + 4*t + e; B operand = T[i0 + (l>>4)][16cb + (l&15)].
//   PANEL == 0: 4 waves split 256 columns; PANEL == 1: 4 waves split the rows
//   of a 64-column tile and reduce through LDS (for narrow X such as P).
//   XMODE: 0 = row-major X (momentum, optional fused G), 1 = explicit sketch
//   S^T, 2 = generated sketch.
// ============================================================================
template <int GDT, int XMODE>
__device__ __forceinline__ void load_col4(const ProjArgs& a, int b, float* __restrict__ M,
                                          const void* __restrict__ G, int i, int i_end, int col,
                                          float (&x)[4], bool& nz) {
  if (i >= i_end) {
#pragma unroll
    for (int e = 0; e < 4; ++e) x[e] = 0.f;
    return;
  }
  if constexpr (XMODE == 1) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int aa = col + e;
      x[e] = (aa < a.cols) ? a.sketch[(static_cast<long>(b) * a.cols + aa) * a.rows + i] : 0.f;
    }
    return;
  } else if constexpr (XMODE == 2) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int aa = col + e;
      x[e] = (aa < a.cols) ? a.sketch_std * gauss(a.seed + 0x632BE59BD9B4E019ull * (b + 1), aa,
                                                          static_cast<uint32_t>(i + a.sketch_row0)) : 0.f;
    }
    return;
  } else {
    float* p = M + static_cast<long>(i) * a.ld_m + col;
    if (a.vec && col + 4 <= a.cols) {
      f32x4 v = *reinterpret_cast<const f32x4*>(p);
      if constexpr (GDT == DION_DTYPE_F32) {
        v += *reinterpret_cast<const f32x4*>(static_cast<const float*>(G) + static_cast<long>(i) * a.ld_g + col);
      } else if constexpr (GDT == DION_DTYPE_BF16) {
        const uint2 gv = *reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(G) +
                                                         static_cast<long>(i) * a.ld_g + col);
        v[0] += __uint_as_float(gv.x << 16);
        v[1] += __uint_as_float(gv.x & 0xFFFF0000u);
        v[2] += __uint_as_float(gv.y << 16);
        v[3] += __uint_as_float(gv.y & 0xFFFF0000u);
      }
      if constexpr (GDT != DION_DTYPE_NONE) *reinterpret_cast<f32x4*>(p) = v;
#pragma unroll
      for (int e = 0; e < 4; ++e) x[e] = v[e];
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = 0.f;
        if (col + e < a.cols) {
          v = p[e];
          if constexpr (GDT == DION_DTYPE_F32) {
            v += static_cast<const float*>(G)[static_cast<long>(i) * a.ld_g + col + e];
          } else if constexpr (GDT == DION_DTYPE_BF16) {
            v += bf16_to_f32(static_cast<const uint16_t*>(G)[static_cast<long>(i) * a.ld_g + col + e]);
          }
          if constexpr (GDT != DION_DTYPE_NONE) p[e] = v;
        }
        x[e] = v;
      }
    }
    if constexpr (GDT != DION_DTYPE_NONE) {
#pragma unroll
      for (int e = 0; e < 4; ++e) nz |= (x[e] != 0.f);
    }
  }
}

template <int RB, int GDT, int XMODE, int PANEL>
__global__ void __launch_bounds__(256) colproj_kernel(const ProjArgs a) {
  const int b = blockIdx.z;
  const int kc = blockIdx.y;
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int t = lane & 15;
  const int g = lane >> 4;
  const int col_base = PANEL ? blockIdx.x * 64 : blockIdx.x * 256 + wave * 64;
  const int i_begin = kc * a.kchunk;
  const int i_end = min(a.rows, i_begin + a.kchunk);
  float* __restrict__ M = (XMODE == 0) ? a.m[b] : nullptr;
  const void* __restrict__ G = (XMODE == 0) ? a.g[b] : nullptr;
  const float* __restrict__ T = a.thin[b];
  const int r = a.r;
  const int col = col_base + 4 * t;

  f32x4 acc[4][RB];
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) acc[e][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  bool nz = false;

  const int i_first = i_begin + (PANEL ? 4 * wave : 0);
  const int i_step = PANEL ? 16 : 4;
  for (int i0 = i_first; i0 < i_end; i0 += i_step) {
    const int i = i0 + g;
    float xv[4];
    load_col4<GDT, XMODE>(a, b, M, G, i, i_end, col, xv, nz);
    float tv[RB];
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) {
      const int c = 16 * cb + t;
      tv[cb] = (i < i_end && c < r) ? T[static_cast<long>(i) * r + c] : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int cb = 0; cb < RB; ++cb)
        acc[e][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[e], tv[cb], acc[e][cb], 0, 0, 0);
  }

  if constexpr (PANEL) {
    // fixed-order cross-wave reduction through one LDS buffer (deterministic)
    __shared__ float red[64][4 * RB * 4 + 1];
    for (int w = 1; w < 4; ++w) {
      __syncthreads();
      if (wave == w) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int cb = 0; cb < RB; ++cb)
#pragma unroll
            for (int q = 0; q < 4; ++q) red[lane][(e * RB + cb) * 4 + q] = acc[e][cb][q];
      }
      __syncthreads();
      if (wave == 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int cb = 0; cb < RB; ++cb)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[e][cb][q] += red[lane][(e * RB + cb) * 4 + q];
      }
    }
    if (wave != 0) return;
  }

  float* out = a.out + (static_cast<long>(b) * a.nchunk + kc) * a.out_rows * r;
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = col_base + 4 * (4 * g + q) + e;
        const int c = 16 * cb + t;
        if (j < a.cols && c < r) out[static_cast<long>(j) * r + c] = acc[e][cb][q];
      }
  if constexpr (GDT != DION_DTYPE_NONE) {
    if (a.nonzero != nullptr && __any(nz) && lane == 0) atomicMax(&a.nonzero[b], kAbsUnknown);
  }
}

// ============================================================================
// Fast projections (the Llama-class shapes): no bounds checks, the thin
// operand staged once per block in LDS, the big operand streamed one K-step
// ahead in named register sets (no copies, so the prefetch stays in flight).
// Preconditions (checked on the host): rows % (64 kRB) == 0 (row kernel) or
// cols % 256 == 0 (column kernel), K-chunks aligned to the step, r == 16 RB,
// row strides multiple of 8 elements, 16-byte aligned pointers.
// ============================================================================
constexpr int kRB = 2;     // 16-row MFMA blocks per wave in the fast row projection

template <int GDT>
struct RowStep {           // kRB row blocks x 8 consecutive columns per lane
  f32x4 x[kRB][2];
  uint4 gb[kRB];           // bf16 G (8 values)
  f32x4 gf[kRB][2];        // f32 G
};

template <int GDT>
__device__ __forceinline__ void rp_load(RowStep<GDT>& S, const float* __restrict__ M, const void* __restrict__ G,
                                        long ld_m, long ld_g, int j) {
#pragma unroll
  for (int rb = 0; rb < kRB; ++rb) {
    const float* p = M + rb * 16 * ld_m + j;
    S.x[rb][0] = ld_part(reinterpret_cast<const f32x4*>(p));
    S.x[rb][1] = ld_part(reinterpret_cast<const f32x4*>(p + 4));
    if constexpr (GDT == DION_DTYPE_BF16) {
      S.gb[rb] = ld_part(reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(G) + rb * 16 * ld_g + j));
    } else if constexpr (GDT == DION_DTYPE_F32) {
      const float* gp = static_cast<const float*>(G) + rb * 16 * ld_g + j;
      S.gf[rb][0] = ld_part(reinterpret_cast<const f32x4*>(gp));
      S.gf[rb][1] = ld_part(reinterpret_cast<const f32x4*>(gp + 4));
    }
  }
}

template <int RB>
struct TStage {            // this thread's share of the 32 x r thin slice
  float2 v[RB];
};

template <int RB>
__device__ __forceinline__ void rp_tload(TStage<RB>& T, const float* __restrict__ Tp, int j0, int tid) {
  constexpr int R = 16 * RB;
  const float* src = Tp + static_cast<long>(j0 + tid / 8) * R + (tid % 8) * 2 * RB;
#pragma unroll
  for (int u = 0; u < RB; ++u) T.v[u] = *reinterpret_cast<const float2*>(src + 2 * u);
}

template <int RB>
__device__ __forceinline__ void rp_tstore(const TStage<RB>& T, float* tl, int tid) {
  constexpr int LDT = 16 * RB + 2;
  float* dst = tl + (tid / 8) * LDT + (tid % 8) * 2 * RB;
#pragma unroll
  for (int u = 0; u < RB; ++u) *reinterpret_cast<float2*>(dst + 2 * u) = T.v[u];
}

template <int RB, int GDT>
__device__ __forceinline__ void rp_compute(RowStep<GDT>& S, f32x4 (&acc)[kRB][RB], const float* tl,
                                           float* __restrict__ M, long ld_m, int j, int g, int t, bool& nz) {
  constexpr int LDT = 16 * RB + 2;
  if constexpr (GDT != DION_DTYPE_NONE) {
#pragma unroll
    for (int rb = 0; rb < kRB; ++rb) {
      if constexpr (GDT == DION_DTYPE_BF16) {
        const uint4 gv = S.gb[rb];
        S.x[rb][0][0] += __uint_as_float(gv.x << 16);
        S.x[rb][0][1] += __uint_as_float(gv.x & 0xFFFF0000u);
        S.x[rb][0][2] += __uint_as_float(gv.y << 16);
        S.x[rb][0][3] += __uint_as_float(gv.y & 0xFFFF0000u);
        S.x[rb][1][0] += __uint_as_float(gv.z << 16);
        S.x[rb][1][1] += __uint_as_float(gv.z & 0xFFFF0000u);
        S.x[rb][1][2] += __uint_as_float(gv.w << 16);
        S.x[rb][1][3] += __uint_as_float(gv.w & 0xFFFF0000u);
      } else {
        S.x[rb][0] += S.gf[rb][0];
        S.x[rb][1] += S.gf[rb][1];
      }
      float* p = M + rb * 16 * ld_m + j;
      st_part(reinterpret_cast<f32x4*>(p), S.x[rb][0]);
      st_part(reinterpret_cast<f32x4*>(p + 4), S.x[rb][1]);
#pragma unroll
      for (int e = 0; e < 4; ++e) nz |= (S.x[rb][0][e] != 0.f) | (S.x[rb][1][e] != 0.f);
    }
  }
#pragma unroll
  for (int s = 0; s < 8; ++s) {
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) {
      const float bv = tl[(8 * g + s) * LDT + 16 * cb + t];
#pragma unroll
      for (int rb = 0; rb < kRB; ++rb)
        acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(S.x[rb][s >> 2][s & 3], bv, acc[rb][cb], 0, 0, 0);
    }
  }
}

// XCD-aware block order of the row kernels (rowproj_fast / rowproj_ef / rowproj_x6).
// Workgroups land on the 8 XCDs round-robin by linear id, and each XCD has its own
// 4 MiB L2.  In launch order, the ~64 blocks resident on one XCD would belong to 3-4
// matrices, whose pre-split thin operands (n x r x 6 B: 1.5 MiB each for Q at
// n = 4096) then fight the M/G stream for L2 and are refetched from memory (PMC:
// 1.7x the algorithmic bytes).  Remapped, XCD x walks the contiguous range
// [x T/8, (x+1) T/8) of the logical blocks, so its resident blocks are neighbouring
// row blocks of one matrix that read the same thin rows at the same time.
// waves per block of the fused pass-A row kernel (rowproj_efh3_kernel; 8 measured slower)
#ifndef DION_PA_NW
#define DION_PA_NW 4
#endif
constexpr int kPaNW = DION_PA_NW;
// r <= 64 pass-A row kernel: no register prefetch ring (PD 1) and 3 blocks per CU (166
// VGPRs, 3 waves per SIMD, 144 KB LDS) -- the PD-2 ring needs 228 VGPRs (2 waves per SIMD;
// at 3 it spills 113).  Measured on the Llama set: kernel 5307 vs 5165 GB/s (3-round A/B)
constexpr int kPaPD = 1;
#ifndef DION_PA_MINB
#define DION_PA_MINB 3
#endif
constexpr int kPaMinb = DION_PA_MINB;
// 16-row blocks per wave of the r <= 64 pass-A row kernel (a dev build option; 2 = kRBE)
#ifndef DION_PA_KR
#define DION_PA_KR 2
#endif
constexpr int kPaKR = DION_PA_KR;

constexpr int kXcdRemap = 1;
struct BlockXYZ {
  int x, y, z, xcd;
};

__device__ __forceinline__ BlockXYZ xcd_block() {
  const int gx = gridDim.x, gy = gridDim.y, gz = gridDim.z;
  const int id = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  if (!kXcdRemap) return {static_cast<int>(blockIdx.x), static_cast<int>(blockIdx.y),
                               static_cast<int>(blockIdx.z), id & 7};
  const int T = gx * gy * gz;
  const int xcd = id & 7, slot = id >> 3;
  const int L = xcd * (T >> 3) + min(xcd, T & 7) + slot;
  return {L % gx, (L / gx) % gy, L / (gx * gy), xcd};
}

// the same remap for the column kernels (colproj_x6 / colproj_ef), whose thin rows are
// shared by the blocks of one (K chunk, matrix); kXcdRemapCol=0 turns it off
constexpr int kXcdRemapCol = 1;
__device__ __forceinline__ BlockXYZ xcd_block_col() {
  if (kXcdRemapCol) return xcd_block();
  return {static_cast<int>(blockIdx.x), static_cast<int>(blockIdx.y), static_cast<int>(blockIdx.z), 0};
}


template <int RB, int GDT>
__global__ void __launch_bounds__(256, RB >= 8 ? 1 : 2) rowproj_fast_kernel(const ProjArgs a) {
  constexpr int R = 16 * RB;
  constexpr int LDT = R + 2;
  __shared__ __attribute__((aligned(16))) float tl[2][32 * LDT];
  const BlockXYZ blk = xcd_block();
  const int b = blk.z;
  const int kc = blk.y;
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int t = lane & 15;
  const int g = lane >> 4;
  const int row_base = blk.x * (64 * kRB) + wave * (16 * kRB);
  const int j_begin = kc * a.kchunk;
  const int j_end = min(a.cols, j_begin + a.kchunk);

  auto cj = [](int j) { return j; };
  float* __restrict__ M = a.m[b] + static_cast<long>(row_base + t) * a.ld_m + 8 * g;
  const void* G = nullptr;
  if constexpr (GDT == DION_DTYPE_BF16)
    G = static_cast<const uint16_t*>(a.g[b]) + static_cast<long>(row_base + t) * a.ld_g + 8 * g;
  else if constexpr (GDT == DION_DTYPE_F32)
    G = static_cast<const float*>(a.g[b]) + static_cast<long>(row_base + t) * a.ld_g + 8 * g;
  const float* __restrict__ Tp = a.thin[b];

  f32x4 acc[kRB][RB];
#pragma unroll
  for (int rb = 0; rb < kRB; ++rb)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) acc[rb][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  bool nz = false;

  RowStep<GDT> SA, SB;
  TStage<RB> TA;
  rp_load<GDT>(SA, M, G, a.ld_m, a.ld_g, cj(j_begin));
  rp_tload<RB>(TA, Tp, cj(j_begin), tid);
  rp_tstore<RB>(TA, tl[0], tid);
  __syncthreads();
  int cur = 0;
  for (int j0 = j_begin; j0 < j_end; j0 += 64) {
    const bool more = j0 + 32 < j_end;
    if (more) {
      rp_load<GDT>(SB, M, G, a.ld_m, a.ld_g, cj(j0 + 32));
      rp_tload<RB>(TA, Tp, cj(j0 + 32), tid);
    }
    rp_compute<RB, GDT>(SA, acc, tl[cur], M, a.ld_m, cj(j0), g, t, nz);
    if (!more) break;
    rp_tstore<RB>(TA, tl[cur ^ 1], tid);
    __syncthreads();
    cur ^= 1;
    const bool more2 = j0 + 64 < j_end;
    if (more2) {
      rp_load<GDT>(SA, M, G, a.ld_m, a.ld_g, cj(j0 + 64));
      rp_tload<RB>(TA, Tp, cj(j0 + 64), tid);
    }
    rp_compute<RB, GDT>(SB, acc, tl[cur], M, a.ld_m, cj(j0 + 32), g, t, nz);
    if (!more2) break;
    rp_tstore<RB>(TA, tl[cur ^ 1], tid);
    __syncthreads();
    cur ^= 1;
  }

  float* out = a.out + (static_cast<long>(b) * a.nchunk + kc) * a.out_rows * R;
#pragma unroll
  for (int rb = 0; rb < kRB; ++rb)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        out[static_cast<long>(row_base + 16 * rb + 4 * g + q) * R + 16 * cb + t] = acc[rb][cb][q];
  if constexpr (GDT != DION_DTYPE_NONE) {
    if (a.nonzero != nullptr && __any(nz) && lane == 0) atomicMax(&a.nonzero[b], kAbsUnknown);
  }
}

// ---------------------------------------------------------------------------
// Fast column projection: block = 4 waves x 64 columns; per 16-row step the
// block stages T[i0:i0+16][0:r] in LDS; each wave streams 16 rows x 64 columns
// of X (+G, written back) as four 4-row MFMA K-steps, one step ahead.
// ---------------------------------------------------------------------------
template <int GDT>
struct ColStep {
  f32x4 x[4];
  uint2 gb[4];
  f32x4 gf[4];
};

template <int GDT>
__device__ __forceinline__ void cp_load(ColStep<GDT>& S, const float* __restrict__ M, const void* __restrict__ G,
                                        long ld_m, long ld_g, int i0) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    S.x[k] = ld_stream(reinterpret_cast<const f32x4*>(M + static_cast<long>(i0 + 4 * k) * ld_m));
    if constexpr (GDT == DION_DTYPE_BF16)
      S.gb[k] = ld_stream(reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(G) + static_cast<long>(i0 + 4 * k) * ld_g));
    else if constexpr (GDT == DION_DTYPE_F32)
      S.gf[k] = ld_stream(reinterpret_cast<const f32x4*>(static_cast<const float*>(G) + static_cast<long>(i0 + 4 * k) * ld_g));
  }
}

template <int RB>
struct CTStage {
  float v[RB];
};

template <int RB>
__device__ __forceinline__ void cp_tload(CTStage<RB>& T, const float* __restrict__ Tp, int i0, int tid) {
  constexpr int R = 16 * RB;
  const float* src = Tp + static_cast<long>(i0 + tid / 16) * R + (tid % 16) * RB;
#pragma unroll
  for (int u = 0; u < RB; ++u) T.v[u] = src[u];
}

template <int RB>
__device__ __forceinline__ void cp_tstore(const CTStage<RB>& T, float* tl, int tid) {
  constexpr int R = 16 * RB;
  constexpr int LDT = (R % 32 == 0) ? R + 16 : R + 32;
  float* dst = tl + (tid / 16) * LDT + (tid % 16) * RB;
#pragma unroll
  for (int u = 0; u < RB; ++u) dst[u] = T.v[u];
}

template <int RB, int GDT>
__device__ __forceinline__ void cp_compute(ColStep<GDT>& S, f32x4 (&acc)[4][RB], const float* tl, float* __restrict__ M,
                                           long ld_m, int i0, int g, int t, bool& nz) {
  constexpr int R = 16 * RB;
  constexpr int LDT = (R % 32 == 0) ? R + 16 : R + 32;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if constexpr (GDT != DION_DTYPE_NONE) {
      if constexpr (GDT == DION_DTYPE_BF16) {
        S.x[k][0] += __uint_as_float(S.gb[k].x << 16);
        S.x[k][1] += __uint_as_float(S.gb[k].x & 0xFFFF0000u);
        S.x[k][2] += __uint_as_float(S.gb[k].y << 16);
        S.x[k][3] += __uint_as_float(S.gb[k].y & 0xFFFF0000u);
      } else {
        S.x[k] += S.gf[k];
      }
      st_stream(reinterpret_cast<f32x4*>(M + static_cast<long>(i0 + 4 * k) * ld_m), S.x[k]);
#pragma unroll
      for (int e = 0; e < 4; ++e) nz |= (S.x[k][e] != 0.f);
    }
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) {
      const float bv = tl[(4 * k + g) * LDT + 16 * cb + t];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        acc[e][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(S.x[k][e], bv, acc[e][cb], 0, 0, 0);
    }
  }
}

template <int RB, int GDT>
__global__ void __launch_bounds__(256, RB >= 8 ? 1 : 2) colproj_fast_kernel(const ProjArgs a) {
  constexpr int R = 16 * RB;
  constexpr int LDT = (R % 32 == 0) ? R + 16 : R + 32;
  __shared__ __attribute__((aligned(16))) float tl[2][16 * LDT];
  const int b = blockIdx.z;
  const int kc = blockIdx.y;
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int t = lane & 15;
  const int g = lane >> 4;
  const int col_base = blockIdx.x * 256 + wave * 64;
  const int i_begin = kc * a.kchunk;
  const int i_end = min(a.rows, i_begin + a.kchunk);
  float* __restrict__ M = a.m[b] + static_cast<long>(g) * a.ld_m + col_base + 4 * t;
  const void* G = nullptr;
  if constexpr (GDT == DION_DTYPE_BF16)
    G = static_cast<const uint16_t*>(a.g[b]) + static_cast<long>(g) * a.ld_g + col_base + 4 * t;
  else if constexpr (GDT == DION_DTYPE_F32)
    G = static_cast<const float*>(a.g[b]) + static_cast<long>(g) * a.ld_g + col_base + 4 * t;
  const float* __restrict__ Tp = a.thin[b];

  f32x4 acc[4][RB];
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) acc[e][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  bool nz = false;

  ColStep<GDT> SA, SB;
  CTStage<RB> TA;
  cp_load<GDT>(SA, M, G, a.ld_m, a.ld_g, i_begin);
  cp_tload<RB>(TA, Tp, i_begin, tid);
  cp_tstore<RB>(TA, tl[0], tid);
  __syncthreads();
  int cur = 0;
  for (int i0 = i_begin; i0 < i_end; i0 += 32) {
    const bool more = i0 + 16 < i_end;
    if (more) {
      cp_load<GDT>(SB, M, G, a.ld_m, a.ld_g, i0 + 16);
      cp_tload<RB>(TA, Tp, i0 + 16, tid);
    }
    cp_compute<RB, GDT>(SA, acc, tl[cur], M, a.ld_m, i0, g, t, nz);
    if (!more) break;
    cp_tstore<RB>(TA, tl[cur ^ 1], tid);
    __syncthreads();
    cur ^= 1;
    const bool more2 = i0 + 32 < i_end;
    if (more2) {
      cp_load<GDT>(SA, M, G, a.ld_m, a.ld_g, i0 + 32);
      cp_tload<RB>(TA, Tp, i0 + 32, tid);
    }
    cp_compute<RB, GDT>(SB, acc, tl[cur], M, a.ld_m, i0 + 16, g, t, nz);
    if (!more2) break;
    cp_tstore<RB>(TA, tl[cur ^ 1], tid);
    __syncthreads();
    cur ^= 1;
  }

  float* out = a.out + (static_cast<long>(b) * a.nchunk + kc) * a.out_rows * R;
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        out[static_cast<long>(col_base + 4 * (4 * g + q) + e) * R + 16 * cb + t] = acc[e][cb][q];
  if constexpr (GDT != DION_DTYPE_NONE) {
    if (a.nonzero != nullptr && __any(nz) && lane == 0) atomicMax(&a.nonzero[b], kAbsUnknown);
  }
}

// sum_k p[k stride] for k = 0 .. n - 1, added in k order (the fixed order the slab reductions
// promise), with eight loads in flight instead of one dependent load per add: these partial-
// sum chains (pass B's split-K slabs, the column-norm partials: 64 of them per Llama column)
// were latency-bound, one L2 round trip per term
__device__ __forceinline__ float ordered_sum_strided(const float* __restrict__ p, long stride, int n) {
  float v = 0.f;
  int k = 0;
  for (; k + 8 <= n; k += 8) {
    float t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = p[(k + u) * stride];
#pragma unroll
    for (int u = 0; u < 8; ++u) v += t[u];
  }
  for (; k < n; ++k) v += p[k * stride];
  return v;
}

// out[b][e] = sum_k slab[b][k][e] in fixed k order.
__global__ void __launch_bounds__(256) reduce_slabs_kernel(float* __restrict__ out,
                                                           const float* __restrict__ slab, int nchunk,
                                                           long per_entry, int batch) {
  const long total = per_entry * batch;
  for (long idx = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; idx < total;
       idx += static_cast<long>(gridDim.x) * blockDim.x) {
    const long b = idx / per_entry;
    const long e = idx - b * per_entry;
    const float* s = slab + b * nchunk * per_entry + e;
    out[idx] = ordered_sum_strided(s, per_entry, nchunk);
  }
}

// ============================================================================
// Householder QR of one K x r matrix per block (LAPACK dgeqr2 / dlarfg sign
// convention, which torch.linalg.qr on CPU and the reference inherit):
//   mode 0: write R (r x r upper) to R_out[b];
//   mode 1: form the K x r Q factor in place (dorg2r) and write it to Q_out[b]
//           (the m_P <= r branch of ortho.py:93-94).
// The matrix lives column-major in LDS.
// ============================================================================
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float s = 0.f;
  const int nw = blockDim.x >> 6;
  for (int w = 0; w < nw; ++w) s += red[w];
  return s;
}

__global__ void __launch_bounds__(256) householder_qr_kernel(const float* __restrict__ A_in,
                                                             float* __restrict__ R_out,
                                                             float* __restrict__ Q_out, int K, int r,
                                                             int mode) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int b = blockIdx.x;
  const int ld = K + 1;
  float* As = sm;               // r columns x ld
  float* tau = As + r * ld;     // r
  float* red = tau + r + 3;     // reduction scratch (8)
  float* bc = red + 8;          // broadcast scalars (4)
  const int tid = threadIdx.x;
  const int nt = blockDim.x;
  const float* A = A_in + static_cast<long>(b) * K * r;
  for (int idx = tid; idx < K * r; idx += nt) {
    const int i = idx / r, c = idx - i * r;
    As[c * ld + i] = A[idx];
  }
  __syncthreads();
  const int kmax = min(K, r);
  int tpc = 64;  // lanes per trailing column: a power of two with tpc * r <= 2 * nt
  while (tpc > 1 && tpc * r > 2 * nt) tpc >>= 1;
  for (int j = 0; j < kmax; ++j) {
    float* aj = As + j * ld;
    float ss = 0.f;
    for (int i = j + 1 + tid; i < K; i += nt) ss += aj[i] * aj[i];
    ss = block_sum(ss, red);
    if (tid == 0) {
      const float alpha = aj[j];
      const float xnorm = sqrtf(ss);
      float tj, beta, scale;
      if (xnorm == 0.f) {
        tj = 0.f;
        beta = alpha;
        scale = 1.f;
      } else {
        beta = -copysignf(hypotf(alpha, xnorm), alpha);
        tj = (beta - alpha) / beta;
        scale = 1.f / (alpha - beta);
      }
      tau[j] = tj;
      bc[0] = scale;
      bc[1] = beta;
    }
    __syncthreads();
    const float scale = bc[0];
    for (int i = j + 1 + tid; i < K; i += nt) aj[i] *= scale;
    __syncthreads();
    if (tid == 0) aj[j] = bc[1];
    const float tj = tau[j];
    // apply H_j = I - tau v v^T (v_j = 1) to the trailing columns: `tpc` lanes per
    // column split the rows, reduce with butterfly shuffles inside their group
    for (int c0 = j + 1; c0 < r; c0 += nt / tpc) {
      const int c = c0 + tid / tpc;
      const int p = tid % tpc;
      float w = 0.f;
      if (c < r) {
        const float* ac = As + c * ld;
        for (int i = j + 1 + p; i < K; i += tpc) w += aj[i] * ac[i];
      }
      for (int off = tpc >> 1; off > 0; off >>= 1) w += __shfl_xor(w, off, 64);
      if (c < r) {
        float* ac = As + c * ld;
        w = (w + ac[j]) * tj;
        if (p == 0) ac[j] -= w;
        for (int i = j + 1 + p; i < K; i += tpc) ac[i] -= w * aj[i];
      }
    }
    __syncthreads();
  }
  if (mode == 0) {
    float* R = R_out + static_cast<long>(b) * r * r;
    for (int idx = tid; idx < r * r; idx += nt) {
      const int i = idx / r, c = idx - i * r;
      R[idx] = (i <= c && i < K) ? As[c * ld + i] : 0.f;
    }
    return;
  }
  // dorg2r: form Q (K x r) in place from the stored reflectors
  for (int j = kmax - 1; j >= 0; --j) {
    float* aj = As + j * ld;
    const float tj = tau[j];
    for (int c0 = j + 1; c0 < r; c0 += nt / tpc) {
      const int c = c0 + tid / tpc;
      const int p = tid % tpc;
      float w = 0.f;
      if (c < r) {
        const float* ac = As + c * ld;
        for (int i = j + 1 + p; i < K; i += tpc) w += aj[i] * ac[i];
      }
      for (int off = tpc >> 1; off > 0; off >>= 1) w += __shfl_xor(w, off, 64);
      if (c < r) {
        float* ac = As + c * ld;
        w = (w + ac[j]) * tj;  // v_j = 1
        if (p == 0) ac[j] -= w;
        for (int i = j + 1 + p; i < K; i += tpc) ac[i] -= w * aj[i];
      }
    }
    __syncthreads();
    for (int i = j + 1 + tid; i < K; i += nt) aj[i] *= -tj;
    if (tid == 0) aj[j] = 1.f - tj;
    for (int i = tid; i < j; i += nt) aj[i] = 0.f;
    __syncthreads();
  }
  float* Q = Q_out + static_cast<long>(b) * K * r;
  for (int idx = tid; idx < K * r; idx += nt) {
    const int i = idx / r, c = idx - i * r;
    Q[idx] = As[c * ld + i];
  }
}

// the back substitution itself, for a block of nt threads (TIP lanes per column, TIP adjacent
// lanes of one wave): F upper-triangular n x n at F[i ldf + k] (LDS), dinv[i] = 1 / F[i][i]
// (LDS), Xs the n x ldx column scratch (LDS, ldx = n + TIP), out the n x n row-major inverse
template <int TIP>
__device__ __forceinline__ void tri_inv_cols(const float* F, int ldf, const float* dinv, float* Xs, int ldx, int n,
                                             float* __restrict__ out, int tid, int nt) {
  const int c = tid / TIP, p = tid % TIP;
  const bool act = c < n;
  for (int i = n - 1; i >= 0; --i) {
    float acc = 0.f;
    if (act)
      for (int k = i + 1 + p; k <= c; k += TIP) acc = fmaf(-F[i * ldf + k], Xs[c * ldx + k], acc);
#pragma unroll
    for (int o = 1; o < TIP; o <<= 1) acc += __shfl_xor(acc, o, 64);
    const float x = (act && i <= c) ? (((i == c) ? 1.f : 0.f) + acc) * dinv[i] : 0.f;
    if (act && p == 0) Xs[c * ldx + i] = x;
    __builtin_amdgcn_wave_barrier();  // the column's lanes share a wave: LDS in order
  }
  __syncthreads();
  for (int idx = tid; idx < n * n; idx += nt) out[idx] = Xs[(idx % n) * ldx + idx / n];
}

// ============================================================================
// Small-factor kernels of the randomised Cholesky QR, one block per matrix.
//
// sketch_qr_inv_kernel: Householder QR (LAPACK dgeqr2/dlarfg sign convention)
//   of the K x r sketch product S P held in REGISTERS -- lane l owns rows
//   l + 64 s (s < RPL), wave w owns columns w + 4 cc (cc < CPW, cyclic, so the
//   triangular work stays balanced).  Per pivot j the owning wave forms the
//   reflector, publishes v and tau through LDS (double-buffered) and every wave
//   updates its own columns with wave-level reductions: one barrier per pivot.
//   A wave's consumed pivot column is shifted out so every register index is
//   static.  Then R^-1 is formed in LDS (tri_inverse_lds) and written out.
// chol_inv_kernel: upper Cholesky (dpotf2 order) of the r x r Gram matrix with
//   one lane per column, then its inverse the same way.  A non-positive pivot
//   poisons the inverse's columns from that pivot on with NaN (cholesky_ex
//   does not raise; the fix-up's nan_to_num then zeroes those P columns).
// ============================================================================
template <typename XT>
__device__ void tri_inverse_lds(const float* Rs, int rld, XT* Xs, int r, int tid, int nthreads) {
  // X = R^-1 (upper) by back substitution, column c by a group of tpc lanes of one wave:
  //   X[i][c] = ((i == c) - sum_{k=i+1..c} R[i][k] X[k][c]) / R[i][i],  i = c .. 0
  // the group splits the k-sum (stride tpc) and combines it with xor shuffles; X[k][c] comes
  // back from LDS, written by the group's lane 0 in an earlier i (same wave: LDS in order)
  int tpc = 1;
  while (tpc < 16 && 2 * tpc * r <= nthreads) tpc *= 2;
  const int c = tid / tpc, p = tid % tpc;
  const bool act = c < r;
  for (int i = r - 1; i >= 0; --i) {
    double acc = 0.0;
    if (act && i < c)
      for (int k = i + 1 + p; k <= c; k += tpc)
        acc += static_cast<double>(Rs[i * rld + k]) * static_cast<double>(Xs[k * r + c]);
    for (int off = tpc >> 1; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (act && p == 0)
      Xs[i * r + c] = static_cast<XT>(i > c ? 0.0 : ((i == c ? 1.0 : 0.0) - acc) / static_cast<double>(Rs[i * rld + i]));
    __builtin_amdgcn_wave_barrier();
  }
}

// Output of the factor kernels without the inverse (INV = false): per matrix the factor
// padded to rt x rt (unit diagonal, zero off-diagonal past r) and then its rt reciprocal
// diagonal entries, the operand layout of trsm_right_kernel<rt>.
__device__ __forceinline__ void write_padded_factor(const float* Rs, int rld, int r, int rt, float* O, int tid,
                                                    int nt) {
  for (int idx = tid; idx < rt * rt; idx += nt) {
    const int i = idx / rt, c = idx - i * rt;
    O[idx] = (i < r && c < r) ? (c >= i ? Rs[i * rld + c] : 0.f) : (i == c ? 1.f : 0.f);
  }
  for (int j = tid; j < rt; j += nt) O[rt * rt + j] = j < r ? 1.f / Rs[j * rld + j] : 1.f;
}

template <int RPL, int CPW, typename XT, bool INV = true, int NWQ = 4, bool TINV = false>
__global__ void __launch_bounds__(64 * NWQ) sketch_qr_inv_kernel(const float* __restrict__ SP, float* __restrict__ Rinv,
                                                                 int K, int r, int rt = 0) {
  extern __shared__ __attribute__((aligned(16))) char qsm[];
  const int rld = r + 1;
  float* vbuf = reinterpret_cast<float*>(qsm);         // 2 x 256
  float* tsc = vbuf + 512;                             // 2 (+pad)
  float* Rs = tsc + 8;                                 // r x rld
  XT* Xs = reinterpret_cast<XT*>(qsm + ((sizeof(float) * (520 + r * rld) + 15) / 16) * 16);
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const float* A0 = SP + static_cast<long>(b) * K * r;
  for (int idx = tid; idx < r * rld; idx += blockDim.x) Rs[idx] = 0.f;
  float A[RPL][CPW];
#pragma unroll
  for (int s = 0; s < RPL; ++s)
#pragma unroll
    for (int cc = 0; cc < CPW; ++cc) {
      const int row = lane + 64 * s, col = w + NWQ * cc;
      A[s][cc] = (row < K && col < r) ? A0[static_cast<long>(row) * r + col] : 0.f;
    }
  const int n_w = (r > w) ? (r - w + NWQ - 1) / NWQ : 0;
  int consumed = 0;
  __syncthreads();
  for (int j = 0; j < r; ++j) {
    const int buf = j & 1;
    if (j % NWQ == w) {
      float xs[RPL];
      float ss = 0.f;
      float alpha_l = 0.f;
#pragma unroll
      for (int s = 0; s < RPL; ++s) {
        const int row = lane + 64 * s;
        xs[s] = A[s][0];
        if (row > j) ss += xs[s] * xs[s];
        if (s == (j >> 6)) alpha_l = xs[s];
      }
      ss = wave_sum_dpp(ss);
      const float alpha = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, alpha_l), j & 63));
      const float xnorm = sqrtf(ss);
      float tau, beta, scale;
      if (xnorm == 0.f) {
        tau = 0.f;
        beta = alpha;
        scale = 1.f;
      } else {
        beta = -copysignf(hypotf(alpha, xnorm), alpha);
        tau = (beta - alpha) / beta;
        scale = 1.f / (alpha - beta);
      }
#pragma unroll
      for (int s = 0; s < RPL; ++s) {
        const int row = lane + 64 * s;
        vbuf[buf * 256 + row] = (row > j) ? xs[s] * scale : (row == j ? 1.f : 0.f);
        if (row < j) Rs[row * rld + j] = xs[s];
        else if (row == j) Rs[row * rld + j] = beta;
      }
      if (lane == 0) tsc[buf] = tau;
#pragma unroll
      for (int s = 0; s < RPL; ++s) {
#pragma unroll
        for (int cc = 0; cc + 1 < CPW; ++cc) A[s][cc] = A[s][cc + 1];
        A[s][CPW - 1] = 0.f;
      }
      ++consumed;
    }
    __syncthreads();
    const float tau = tsc[buf];
    float v[RPL];
#pragma unroll
    for (int s = 0; s < RPL; ++s) v[s] = vbuf[buf * 256 + lane + 64 * s];
    // H_j on this wave's live columns; consumed columns were shifted out and are zero, so a
    // column past `rem` takes d = 0 and stays zero.  The column sums of a pivot are reduced
    // together (wave_sum_n), over the first 4, 8 or all CPW columns as `rem` allows
    const int rem = n_w - consumed;
    auto trail = [&](auto NCc) {
      constexpr int NC = decltype(NCc)::value;
      float d[NC];
#pragma unroll
      for (int cc = 0; cc < NC; ++cc) {
        d[cc] = 0.f;
#pragma unroll
        for (int s = 0; s < RPL; ++s) d[cc] += v[s] * A[s][cc];
      }
      wave_sum_dpp_n<NC>(d);
#pragma unroll
      for (int cc = 0; cc < NC; ++cc) {
        const float dt = d[cc] * tau;
#pragma unroll
        for (int s = 0; s < RPL; ++s) A[s][cc] -= dt * v[s];
      }
    };
    if (rem > CPW / 2)
      trail(std::integral_constant<int, CPW>{});
    else if (rem > CPW / 4 || CPW < 8)
      trail(std::integral_constant<int, (CPW / 2 > 0 ? CPW / 2 : 1)>{});
    else if (rem > 0)
      trail(std::integral_constant<int, (CPW / 4 > 0 ? CPW / 4 : 1)>{});
  }
  __syncthreads();
  if constexpr (TINV) {
    // R^-1 in fp32 by tri_inv_cols (8 lanes per column: r = 8 NWQ), straight after the QR; the
    // reflector buffer holds the reciprocal diagonal, Xs the column scratch (r x (r + 8) floats)
    for (int j = tid; j < r; j += blockDim.x) vbuf[j] = 1.f / Rs[j * rld + j];
    __syncthreads();
    tri_inv_cols<8>(Rs, rld, vbuf, reinterpret_cast<float*>(Xs), r + 8, r, Rinv + static_cast<long>(b) * r * r, tid,
                    blockDim.x);
    return;
  }
  if constexpr (!INV) {
    write_padded_factor(Rs, rld, r, rt, Rinv + static_cast<long>(b) * (rt * rt + rt), tid, blockDim.x);
    return;
  }
  tri_inverse_lds<XT>(Rs, rld, Xs, r, tid, blockDim.x);
  __syncthreads();
  float* O = Rinv + static_cast<long>(b) * r * r;
  for (int idx = tid; idx < r * r; idx += blockDim.x) O[idx] = static_cast<float>(Xs[idx]);
}

template <typename XT, bool INV = true>
__global__ void __launch_bounds__(256) chol_inv_kernel(const float* __restrict__ G_in, float* __restrict__ Uinv,
                                                       int r, int rt = 0) {
  // Right-looking upper Cholesky: at pivot j the whole block updates the trailing upper
  // triangle, G[i][c] -= u_ji u_jc (u_j* = row j / sqrt(d_j)), one barrier per pivot.  Every
  // element receives the same fused products in the same order (k = 0, 1, ..) as the
  // left-looking dpotf2 dot products, so the factor is the same.  Factor row j is parked
  // transposed in the strictly lower triangle (G[c][j] = u_jc, never read by the upper
  // updates) and its diagonal in ud[], then moved to the upper triangle for the inverse.
  extern __shared__ __attribute__((aligned(16))) char csm[];
  const int ld = r + 1;
  float* Gs = reinterpret_cast<float*>(csm);       // r x ld
  float* ud = Gs + r * ld;                          // r: the factor's diagonal
  XT* Xs = reinterpret_cast<XT*>(csm + ((sizeof(float) * (r * ld + r + 4) + 15) / 16) * 16);
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int nt = blockDim.x;
  const float* Gm = G_in + static_cast<long>(b) * r * r;
  for (int idx = tid; idx < r * r; idx += nt) {
    const int i = idx / r, c = idx - i * r;
    Gs[i * ld + c] = (c >= i) ? Gm[idx] : 0.f;
  }
  int jf = r;
  for (int j = 0; j < r; ++j) {
    __syncthreads();
    const float d = Gs[j * ld + j];
    if (!(d > 0.f)) {  // uniform
      jf = j;
      break;
    }
    const float ujj = sqrtf(d);
    const float inv = 1.f / ujj;
    if (tid == 0) ud[j] = ujj;
    for (int c = j + 1 + tid; c < r; c += nt) Gs[c * ld + j] = Gs[j * ld + c] * inv;
    // trailing update: lane tid % 64 takes columns c, the block's 4 waves split the rows
    for (int c = j + 1 + (tid & 63); c < r; c += 64) {
      const float ujc = Gs[j * ld + c] * inv;
      for (int i = j + 1 + (tid >> 6); i <= c; i += nt >> 6)
        Gs[i * ld + c] -= (Gs[j * ld + i] * inv) * ujc;
    }
  }
  __syncthreads();
  // factor rows to the upper triangle; rows from a failed pivot on: placeholders whose
  // columns are poisoned with NaN (cholesky_ex does not raise; the fix-up's nan_to_num then
  // zeroes those P columns): in the inverse below, or through a NaN diagonal for the solve
  for (int idx = tid; idx < r * r; idx += nt) {
    const int i = idx / r, c = idx - i * r;
    if (c < i) continue;
    Gs[i * ld + c] = (i >= jf) ? (i == c ? (INV ? 1.f : __builtin_nanf("")) : 0.f)
                               : (i == c ? ud[i] : Gs[c * ld + i]);
  }
  __syncthreads();
  if constexpr (!INV) {
    write_padded_factor(Gs, ld, r, rt, Uinv + static_cast<long>(b) * (rt * rt + rt), tid, nt);
    return;
  }
  tri_inverse_lds<XT>(Gs, ld, Xs, r, tid, nt);
  __syncthreads();
  float* O = Uinv + static_cast<long>(b) * r * r;
  for (int idx = tid; idx < r * r; idx += nt) {
    const int c = idx % r;
    O[idx] = (c >= jf) ? __builtin_nanf("") : static_cast<float>(Xs[idx]);
  }
}

// ============================================================================
// Fix-up + column normalisation + Q commit, one block per matrix.
//   R <- z ? nan_to_num(Q) : nan_to_num(R);  Q <- R / (sqrt(sum_rows R^2) + eps)
// Threads are grouped per column (tpc threads per column, fixed-order tree
// reduction), so the column sums are deterministic.
// ============================================================================
struct FixArgs {
  float* q[MAXB];     // fp32, or bf16 (uint16_t) when q_bf16
  int q_bf16;
  float* R;           // (batch, nq, r)
  float* part;        // (batch, nchunk, r) partial column sums of squares
  const uint32_t* nonzero;
  int nq, r, tpc, nchunk, rows_per_chunk;
  float eps;
};

// rows of R per fix-up block: 64 (was 256) gives 4x the blocks, so the fix-up and the column
// norm, latency-bound row loops of 256 / r rows per thread, run wide (they sit on the
// critical path between pass B and the weight update of every launch group)
constexpr int kFixRows = 64;

// phase 1: fix R rows of one chunk and write its column partial sums
__global__ void __launch_bounds__(256) fixup_partial_kernel(const FixArgs a) {
  __shared__ float red[256];
  const int b = blockIdx.y, ch = blockIdx.x;
  const int tid = threadIdx.x;
  const int r = a.r, nq = a.nq, tpc = a.tpc;
  const bool zero = (a.nonzero[b] == 0u);
  float* R = a.R + static_cast<long>(b) * nq * r;
  const float* Q = a.q[b];
  const int c = tid % r, p = tid / r;
  const int row0 = ch * a.rows_per_chunk;
  const int row1 = min(nq, row0 + a.rows_per_chunk);
  float ss = 0.f;
  if (p < tpc) {
    for (int row = row0 + p; row < row1; row += tpc) {
      const long idx = static_cast<long>(row) * r + c;
      const float qv = a.q_bf16 ? bf16_to_f32(reinterpret_cast<const uint16_t*>(Q)[idx]) : Q[idx];
      const float v = zero ? nan_to_num(qv) : nan_to_num(R[idx]);
      R[idx] = v;
      ss += v * v;
    }
  }
  red[tid] = ss;
  __syncthreads();
  if (tid < r) {
    float s = 0.f;
    for (int k = 0; k < tpc; ++k) s += red[k * r + tid];
    a.part[(static_cast<long>(b) * a.nchunk + ch) * r + tid] = s;
  }
}

// phase 2: column norms from the partials (fixed order), Q <- R / (norm + eps)
__global__ void __launch_bounds__(256) colnorm_apply_kernel(const FixArgs a) {
  __shared__ float denom[256];
  const int b = blockIdx.y, ch = blockIdx.x;
  const int tid = threadIdx.x;
  const int r = a.r, nq = a.nq, tpc = a.tpc;
  if (tid < r) {
    const float* pp = a.part + static_cast<long>(b) * a.nchunk * r + tid;
    const float s = ordered_sum_strided(pp, r, a.nchunk);
    denom[tid] = sqrtf(s) + a.eps;
  }
  __syncthreads();
  const float* R = a.R + static_cast<long>(b) * nq * r;
  float* Q = a.q[b];
  const int c = tid % r, p = tid / r;
  const int row0 = ch * a.rows_per_chunk;
  const int row1 = min(nq, row0 + a.rows_per_chunk);
  if (p < tpc) {
    const float d = denom[c];
    for (int row = row0 + p; row < row1; row += tpc) {
      const long idx = static_cast<long>(row) * r + c;
      if (a.q_bf16) {
        // kernels.py:287-290: the fp32 quotient cast back to R's dtype (bf16, round to nearest even)
        const uint32_t u = __float_as_uint(R[idx] / d);
        reinterpret_cast<uint16_t*>(Q)[idx] = ((u & 0x7FFFFFFFu) > 0x7F800000u)
                                                  ? static_cast<uint16_t>((u >> 16) | 0x40u)
                                                  : static_cast<uint16_t>((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
      } else {
        Q[idx] = R[idx] / d;
      }
    }
  }
}

// phase 1 fused with pass B's split-K reduction (dion_project_r_fixup): R = the sum of the
// slabs in reduce_slabs_kernel's order, then fixup_partial_kernel's fix and chunk partials, in
// its thread mapping and order (bitwise the two kernels; one launch and one pass over R fewer)
__global__ void __launch_bounds__(256) reduce_fix_partial_kernel(const FixArgs a, const float* __restrict__ slab,
                                                                 int nslab) {
  __shared__ float red[256];
  const int b = blockIdx.y, ch = blockIdx.x;
  const int tid = threadIdx.x;
  const int r = a.r, nq = a.nq, tpc = a.tpc;
  const long per_entry = static_cast<long>(nq) * r;
  const bool zero = (a.nonzero[b] == 0u);
  float* R = a.R + b * per_entry;
  const float* S = slab + b * nslab * per_entry;
  const float* Q = a.q[b];
  const int c = tid % r, p = tid / r;
  const int row0 = ch * a.rows_per_chunk;
  const int row1 = min(nq, row0 + a.rows_per_chunk);
  float ss = 0.f;
  if (p < tpc) {
    for (int row = row0 + p; row < row1; row += tpc) {
      const long idx = static_cast<long>(row) * r + c;
      float v = ordered_sum_strided(S + idx, per_entry, nslab);
      const float qv = a.q_bf16 ? bf16_to_f32(reinterpret_cast<const uint16_t*>(Q)[idx]) : Q[idx];
      v = zero ? nan_to_num(qv) : nan_to_num(v);
      R[idx] = v;
      ss += v * v;
    }
  }
  red[tid] = ss;
  __syncthreads();
  if (tid < r) {
    float s2 = 0.f;
    for (int k = 0; k < tpc; ++k) s2 += red[k * r + tid];
    a.part[(static_cast<long>(b) * a.nchunk + ch) * r + tid] = s2;
  }
}

// FS column norm, first half: the chunk partials of fixup_partial_kernel summed in fixed order
__global__ void __launch_bounds__(256) colsum_reduce_kernel(const FixArgs a, float* __restrict__ colsum) {
  const int b = blockIdx.x;
  for (int c = threadIdx.x; c < a.r; c += 256) {
    float s = 0.f;
    const float* pp = a.part + static_cast<long>(b) * a.nchunk * a.r + c;
    for (int k = 0; k < a.nchunk; ++k) s += pp[static_cast<long>(k) * a.r];
    colsum[static_cast<long>(b) * a.r + c] = s;
  }
}

// FS column norm, second half: Q <- R / (sqrt(colsum) + eps) with the all-reduced sums
__global__ void __launch_bounds__(256) colnorm_given_kernel(const FixArgs a, const float* __restrict__ colsum) {
  __shared__ float denom[256];
  const int b = blockIdx.y, ch = blockIdx.x;
  const int tid = threadIdx.x;
  const int r = a.r, nq = a.nq, tpc = a.tpc;
  if (tid < r) denom[tid] = sqrtf(colsum[static_cast<long>(b) * r + tid]) + a.eps;
  __syncthreads();
  const float* R = a.R + static_cast<long>(b) * nq * r;
  float* Q = a.q[b];
  const int c = tid % r, p = tid / r;
  const int row0 = ch * a.rows_per_chunk;
  const int row1 = min(nq, row0 + a.rows_per_chunk);
  if (p < tpc) {
    const float d = denom[c];
    for (int row = row0 + p; row < row1; row += tpc) {
      const long idx = static_cast<long>(row) * r + c;
      if (a.q_bf16) {
        const uint32_t u = __float_as_uint(R[idx] / d);
        reinterpret_cast<uint16_t*>(Q)[idx] = ((u & 0x7FFFFFFFu) > 0x7F800000u)
                                                  ? static_cast<uint16_t>((u >> 16) | 0x40u)
                                                  : static_cast<uint16_t>((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
      } else {
        Q[idx] = R[idx] / d;
      }
    }
  }
}

// P <- z ? 0 : nan_to_num(P) for the real entries (kernels.py:185-188)
__global__ void __launch_bounds__(256) pfix_kernel(float* __restrict__ P, const uint32_t* __restrict__ nonzero,
                                                   long per_entry, int batch) {
  const long total = per_entry * batch;
  for (long idx = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; idx < total;
       idx += static_cast<long>(gridDim.x) * blockDim.x) {
    const long b = idx / per_entry;
    P[idx] = (nonzero[b] == 0u) ? 0.f : nan_to_num(P[idx]);
  }
}

// ============================================================================
// Error feedback + weight update on the m x n storage of every matrix:
//   M[i][j] += sum_c (ra_m[i][c]) (ca_m[j][c])      (scales folded into the R / Qn side)
//   W[i][j]  = d W[i][j] + sum_c (ra_w[i][c]) (ca_w[j][c])
// MFMA 32x32x2 f32 with K = r split over the two lane halves (c = h*RH + s):
// A operand lane l = rowF[i0 + (l&31)][h*RH + s], B operand = colF[j0 + (l&31)][h*RH + s];
// the accumulator tile is loaded from / stored to M and W directly (each
// register = two 128-byte row segments per wave).  Block = 4 waves = 64 x 128.
// ============================================================================
struct EfArgs {
  float* m[MAXB];
  float* w[MAXB];
  const float* qn[MAXB];
  const float* P;     // (batch, m_P, r)
  const float* R;     // (batch, n_Q, r)
  const uint32_t* nonzero;
  int rows, cols, r, transposed;
  long ld_m, ld_w;
  float alpha;        // -(1 - mu)
  float beta;         // -scaled_lr
  float decay;        // 1 - lr*wd (or 1)
  int has_w;
};

template <int RH>
__device__ __forceinline__ void load_factor(const float* __restrict__ F, int idx, int nrows, int r, int h,
                                            float scale, float (&v)[RH]) {
  const int c0 = h * RH;
  if (idx < nrows) {
    const float* p = F + static_cast<long>(idx) * r + c0;
    if ((r % 4) == 0 && c0 + RH <= r) {
#pragma unroll
      for (int s = 0; s < RH; s += 4) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(p + s);
        v[s] = x[0] * scale;
        v[s + 1] = x[1] * scale;
        v[s + 2] = x[2] * scale;
        v[s + 3] = x[3] * scale;
      }
    } else {
#pragma unroll
      for (int s = 0; s < RH; ++s) v[s] = (c0 + s < r) ? p[s] * scale : 0.f;
    }
  } else {
#pragma unroll
    for (int s = 0; s < RH; ++s) v[s] = 0.f;
  }
}

// v2 geometry: a wave owns a 32-wide strip of the side whose factors differ
// between the two updates (R for M, Qn for W) and keeps both in registers;
// it then streams 32 x 32 tiles along the other side, where the shared factor
// P lives, with the next tile's loads (P slice, M tile, W tile) in flight while
// the current tile's MFMA chains run.  ROWFIX = transposed (R, Qn indexed by
// rows); otherwise R, Qn are indexed by columns and P by rows.
constexpr int kEfStream = 512;  // streamed extent per block (16 tiles)

template <int RH, bool ROWFIX>
struct EfTile {
  float sp[RH];
  f32x16 accm, accw;
};

// Tile addressing: element (i, j) of the 32 x 32 tile at (row0, col0) held in
// accumulator register q of lane (t, h) is (row0 + (q&3) + 8(q>>2) + 4h, col0 + t).
// Its byte offset splits into a per-lane part 4(4h ld + t), loop-invariant, and
// a wave-uniform part 4((row0 + (q&3) + 8(q>>2)) ld + col0), so full tiles use
// buffer loads/stores with one VGPR offset and an SGPR offset per register.
struct EfBuf {
  __amdgpu_buffer_rsrc_t m, w;
  int voff_m, voff_w;
};

template <int RH, bool ROWFIX, bool FAST>
__device__ __forceinline__ void ef_load_tile(const EfArgs& a, const EfBuf& bf, int b, int fbase, int s0, int t,
                                             int h, bool zero, const float* __restrict__ Pb,
                                             EfTile<RH, ROWFIX>& T) {
  const int rows = a.rows, cols = a.cols, r = a.r;
  load_factor<RH>(Pb, s0 + t, ROWFIX ? cols : rows, r, h, 1.f, T.sp);
  const int row0 = ROWFIX ? fbase : s0;
  const int col0 = ROWFIX ? s0 : fbase;
  if constexpr (FAST) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int rq = row0 + (q & 3) + 8 * (q >> 2);
      if (!zero) {
        const int so = __builtin_amdgcn_readfirstlane((rq * static_cast<int>(a.ld_m) + col0) * 4);
        T.accm[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(bf.m, bf.voff_m, so, 0));
      } else {
        T.accm[q] = 0.f;
      }
      if (a.has_w) {
        const int so = __builtin_amdgcn_readfirstlane((rq * static_cast<int>(a.ld_w) + col0) * 4);
        T.accw[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(bf.w, bf.voff_w, so, 0)) * a.decay;
      } else {
        T.accw[q] = 0.f;
      }
    }
    return;
  } else {
  const float* M = a.m[b];
  const float* W = a.w[b];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int i = row0 + (q & 3) + 8 * (q >> 2) + 4 * h;
    const int j = col0 + t;
    const bool ok = (i < rows) && (j < cols);
    T.accm[q] = (ok && !zero) ? M[static_cast<long>(i) * a.ld_m + j] : 0.f;
    T.accw[q] = (ok && a.has_w) ? W[static_cast<long>(i) * a.ld_w + j] * a.decay : 0.f;
  }
  }
}

template <int RH, bool ROWFIX, bool FAST>
__device__ __forceinline__ void ef_compute_store(const EfArgs& a, const EfBuf& bf, int b, int fbase, int s0, int t,
                                                 int h, bool zero, const float (&fm)[RH], const float (&fw)[RH],
                                                 EfTile<RH, ROWFIX>& T) {
  if (!zero) {
#pragma unroll
    for (int s = 0; s < RH; ++s)
      T.accm = ROWFIX ? __builtin_amdgcn_mfma_f32_32x32x2f32(fm[s], T.sp[s], T.accm, 0, 0, 0)
                      : __builtin_amdgcn_mfma_f32_32x32x2f32(T.sp[s], fm[s], T.accm, 0, 0, 0);
  }
  if (a.has_w && !zero) {
#pragma unroll
    for (int s = 0; s < RH; ++s)
      T.accw = ROWFIX ? __builtin_amdgcn_mfma_f32_32x32x2f32(fw[s], T.sp[s], T.accw, 0, 0, 0)
                      : __builtin_amdgcn_mfma_f32_32x32x2f32(T.sp[s], fw[s], T.accw, 0, 0, 0);
  }
  const int rows = a.rows, cols = a.cols;
  const int row0 = ROWFIX ? fbase : s0;
  const int col0 = ROWFIX ? s0 : fbase;
  if constexpr (FAST) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int rq = row0 + (q & 3) + 8 * (q >> 2);
      if (!zero) {
        const int so = __builtin_amdgcn_readfirstlane((rq * static_cast<int>(a.ld_m) + col0) * 4);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(T.accm[q]), bf.m, bf.voff_m, so, 0);
      }
      if (a.has_w) {
        const int so = __builtin_amdgcn_readfirstlane((rq * static_cast<int>(a.ld_w) + col0) * 4);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(T.accw[q]), bf.w, bf.voff_w, so, 0);
      }
    }
    return;
  } else {
  float* M = a.m[b];
  float* W = a.w[b];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int i = row0 + (q & 3) + 8 * (q >> 2) + 4 * h;
    const int j = col0 + t;
    if (i < rows && j < cols) {
      if (!zero) M[static_cast<long>(i) * a.ld_m + j] = T.accm[q];
      if (a.has_w) W[static_cast<long>(i) * a.ld_w + j] = T.accw[q];
    }
  }
  }
}

template <int RH, bool ROWFIX, bool FAST>
__device__ __forceinline__ void ef_stream(const EfArgs& a, const EfBuf& bf, int b, int fbase, int s_begin, int s_end,
                                          int t, int h, bool zero, const float* __restrict__ Pb,
                                          const float (&fm)[RH], const float (&fw)[RH]) {
  EfTile<RH, ROWFIX> A, B;
  ef_load_tile<RH, ROWFIX, FAST>(a, bf, b, fbase, s_begin, t, h, zero, Pb, A);
  for (int s0 = s_begin; s0 < s_end; s0 += 64) {
    const bool more = s0 + 32 < s_end;
    if (more) ef_load_tile<RH, ROWFIX, FAST>(a, bf, b, fbase, s0 + 32, t, h, zero, Pb, B);
    ef_compute_store<RH, ROWFIX, FAST>(a, bf, b, fbase, s0, t, h, zero, fm, fw, A);
    if (!more) break;
    if (s0 + 64 < s_end) ef_load_tile<RH, ROWFIX, FAST>(a, bf, b, fbase, s0 + 64, t, h, zero, Pb, A);
    ef_compute_store<RH, ROWFIX, FAST>(a, bf, b, fbase, s0 + 32, t, h, zero, fm, fw, B);
  }
}

template <int RH, bool ROWFIX, bool FAST>
__global__ void __launch_bounds__(256, (RH >= 64 ? 1 : 2)) ef_update_kernel(const EfArgs a) {
  const int b = blockIdx.z;
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int t = lane & 31;
  const int h = lane >> 5;
  const int rows = a.rows, cols = a.cols, r = a.r;
  const bool zero = (a.nonzero[b] == 0u);
  const int m_p = ROWFIX ? cols : rows;
  const int n_q = ROWFIX ? rows : cols;
  const float* Pb = a.P + static_cast<long>(b) * m_p * r;
  const float* Rb = a.R + static_cast<long>(b) * n_q * r;
  const float* Qb = a.qn[b];
  const int fbase = blockIdx.x * 128 + __builtin_amdgcn_readfirstlane(wave) * 32;  // fixed strip
  const int flen = ROWFIX ? rows : cols;
  const int s_begin = blockIdx.y * kEfStream;
  const int s_end = min(ROWFIX ? cols : rows, s_begin + kEfStream);
  if (fbase >= flen) return;
  float fm[RH], fw[RH];
  load_factor<RH>(Rb, fbase + t, n_q, r, h, a.alpha, fm);
  load_factor<RH>(Qb, fbase + t, n_q, r, h, a.beta, fw);

  EfBuf bf;
  bf.m = __builtin_amdgcn_make_buffer_rsrc(a.m[b], static_cast<short>(0),
                                           static_cast<int>(min(static_cast<long>(rows) * a.ld_m * 4, 0x7FFFFFF0L)),
                                           0x00020000);
  bf.w = __builtin_amdgcn_make_buffer_rsrc(a.has_w ? a.w[b] : a.m[b], static_cast<short>(0),
                                           static_cast<int>(min(static_cast<long>(rows) * a.ld_w * 4, 0x7FFFFFF0L)),
                                           0x00020000);
  bf.voff_m = (4 * h * static_cast<int>(a.ld_m) + t) * 4;
  bf.voff_w = (4 * h * static_cast<int>(a.ld_w) + t) * 4;

  // FAST: every tile is full (m, n multiples of 32), chosen per launch by the host
  ef_stream<RH, ROWFIX, FAST>(a, bf, b, fbase, s_begin, s_end, t, h, zero, Pb, fm, fw);
}

// ----------------------------------------------------------------------------
// Fast path of the same update for the common case (m, n multiples of 32,
// r == 2 RH with r % 4 == 0, ld_w == ld_m, 16-byte aligned factors): all
// addressing is precomputed -- 16 per-register VGPR offsets shared by M and W,
// one SGPR tile offset -- so the loop body is loads, MFMAs and stores only.
// ----------------------------------------------------------------------------
template <int RH>
__device__ __forceinline__ void load_factor_vec(const float* __restrict__ F, int idx, int h, float scale,
                                                float (&v)[RH]) {
  const float* p = F + static_cast<long>(idx) * (2 * RH) + h * RH;
#pragma unroll
  for (int s = 0; s < RH; s += 4) {
    const f32x4 x = *reinterpret_cast<const f32x4*>(p + s);
    v[s] = x[0] * scale;
    v[s + 1] = x[1] * scale;
    v[s + 2] = x[2] * scale;
    v[s + 3] = x[3] * scale;
  }
}

template <int RH, bool ROWFIX, bool DO_M>
__global__ void __launch_bounds__(256, (RH >= 64 ? 1 : 2)) ef_fast_kernel(const EfArgs a) {
  const int b = blockIdx.z;
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  const int t = lane & 31;
  const int h = lane >> 5;
  const int rows = a.rows, cols = a.cols;
  const int m_p = ROWFIX ? cols : rows;
  const int n_q = ROWFIX ? rows : cols;
  constexpr int r = 2 * RH;
  // entries whose accumulated momentum is all zero take the DO_M == false
  // instantiation (host splits nothing: the flag is read here, uniformly)
  const bool zero = __builtin_amdgcn_readfirstlane(a.nonzero[b]) == 0u;
  if (DO_M == zero) return;
  const float* Pb = a.P + static_cast<long>(b) * m_p * r;
  const float* Rb = a.R + static_cast<long>(b) * n_q * r;
  const float* Qb = a.qn[b];
  const int fbase = blockIdx.x * 128 + wave * 32;
  if (fbase >= (ROWFIX ? rows : cols)) return;  // partial last block: whole waves idle
  const int s_begin = blockIdx.y * kEfStream;
  const int s_end = min(ROWFIX ? cols : rows, s_begin + kEfStream);
  const int ld = static_cast<int>(a.ld_m);
  const __amdgpu_buffer_rsrc_t rm = __builtin_amdgcn_make_buffer_rsrc(
      a.m[b], static_cast<short>(0), static_cast<int>(min(static_cast<long>(rows) * ld * 4, 0x7FFFFFF0L)), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      a.has_w ? a.w[b] : a.m[b], static_cast<short>(0),
      static_cast<int>(min(static_cast<long>(rows) * ld * 4, 0x7FFFFFF0L)), 0x00020000);
  int voff[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) voff[q] = (((q & 3) + 8 * (q >> 2) + 4 * h) * ld + t) * 4;

  float fm[RH], fw[RH];
  if (DO_M) load_factor_vec<RH>(Rb, fbase + t, h, a.alpha, fm);
  load_factor_vec<RH>(Qb, fbase + t, h, a.beta, fw);

  auto tile_soff = [&](int s0) {
    const int row0 = ROWFIX ? fbase : s0;
    const int col0 = ROWFIX ? s0 : fbase;
    return (row0 * ld + col0) * 4;
  };
  float spA[RH], spB[RH];
  f32x16 mA, wA, mB, wB;
  auto load = [&](int s0, float (&sp)[RH], f32x16& am, f32x16& aw) {
    if (DO_M) load_factor_vec<RH>(Pb, s0 + t, h, 1.f, sp);
    __builtin_amdgcn_sched_barrier(0);
    const int so = tile_soff(s0);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      if (DO_M) am[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rm, voff[q], so, kStreamAux));
      aw[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rw, voff[q], so, kStreamAux));
    }
  };
  auto compute_store = [&](int s0, const float (&sp)[RH], f32x16& am, f32x16& aw) {
    const int so = tile_soff(s0);
    if (DO_M) {
#pragma unroll
      for (int s = 0; s < RH; ++s)
        am = ROWFIX ? __builtin_amdgcn_mfma_f32_32x32x2f32(fm[s], sp[s], am, 0, 0, 0)
                    : __builtin_amdgcn_mfma_f32_32x32x2f32(sp[s], fm[s], am, 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 16; ++q)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(am[q]), rm, voff[q], so, kStreamAux);
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) aw[q] *= a.decay;
    if (DO_M) {
#pragma unroll
      for (int s = 0; s < RH; ++s)
        aw = ROWFIX ? __builtin_amdgcn_mfma_f32_32x32x2f32(fw[s], sp[s], aw, 0, 0, 0)
                    : __builtin_amdgcn_mfma_f32_32x32x2f32(sp[s], fw[s], aw, 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 16; ++q)
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(aw[q]), rw, voff[q], so, kStreamAux);
  };

  // Order per tile: wait for this tile's loads (an empty asm "use" makes the
  // compiler place the vmcnt wait here), THEN issue the next tile's loads, then
  // the MFMA chains and stores.  Issuing the next loads first would put them
  // between this tile's loads and its use, and with the previous tile's 32
  // stores that exceeds the 6-bit vmcnt window, forcing a full drain.
  auto touch = [&](const float (&sp)[RH], f32x16& am, f32x16& aw) {
    if (DO_M) {
#pragma unroll
      for (int s = 0; s < RH; ++s) asm volatile("" ::"v"(sp[s]));
      asm volatile("" ::"v"(am));
    }
    asm volatile("" ::"v"(aw));
  };
  // The wait for a tile's loads sits at the END of the previous tile's work
  // (after its stores), never at the loop header, where the waitcnt pass would
  // merge the prologue state and drain everything.
  load(s_begin, spA, mA, wA);
  touch(spA, mA, wA);
  __builtin_amdgcn_sched_barrier(0);
  for (int s0 = s_begin; s0 < s_end; s0 += 64) {
    const bool more = s0 + 32 < s_end;
    if (more) load(s0 + 32, spB, mB, wB);
    __builtin_amdgcn_sched_barrier(0);
    compute_store(s0, spA, mA, wA);
    __builtin_amdgcn_sched_barrier(0);
    if (!more) break;
    touch(spB, mB, wB);
    __builtin_amdgcn_sched_barrier(0);
    const bool more2 = s0 + 64 < s_end;
    if (more2) load(s0 + 64, spA, mA, wA);
    __builtin_amdgcn_sched_barrier(0);
    compute_store(s0 + 32, spB, mB, wB);
    __builtin_amdgcn_sched_barrier(0);
    if (more2) touch(spA, mA, wA);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// ============================================================================
// Rank-r update with split-bf16 MFMA ("bf16x6"), the production EF / weight path:
//   X = decay * X + U,   U = sum_c A[i][c] B[j][c]   (one update per launch:
//   M with (P, -(1-mu) R), then W with (P, -s Qn) -- separate launches keep one
//   fixed factor per kernel, so the registers allow two waves per SIMD).
// Each fp32 factor value is split exactly into hi + mid + lo bf16 pieces
// (x - bf16(x) is exact in fp32) and U accumulates the six products
// hi.hi, hi.mid, mid.hi, hi.lo, lo.hi, mid.mid on v_mfma_f32_32x32x16_bf16
// (dropped terms are below 2^-25 relative: fp32-level accuracy at 16/6 times
// the f32-MFMA rate).  U is accumulated from zero and added to decay * X at the
// end, the reference's order (kernels.py:54-83: X*beta + alpha*(A B^T);
// runtime.py:1110-1113: W*(1-lr wd) then add).
// Geometry as ef_fast_kernel: a wave keeps the fixed factor of a 32-wide strip
// (pre-split in registers) and streams 32 x 32 tiles along the other side.
// ============================================================================
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

struct RankArgs {
  float* x[MAXB];            // M or W per matrix
  const float* fixed[MAXB];  // factor indexed by the fixed strip (R_b or Qn_b)
  const float* S;            // streamed factor base: P (batch, len, r)
  const float* sptr[MAXB];   // rank_stream_kernel: per-matrix streamed factor (overrides S when set)
  const u32x4* Ssplit;       // P pre-split (presplit_kernel layout 2), or null
  long ss_stride;            // 16-byte units per matrix of Ssplit
  int s_len;                 // streamed extent per block (multiple of 64)
  const uint32_t* nonzero;
  long s_stride;             // elements between consecutive P_b
  int rows, cols;
  long ld;
  float scale;               // applied to the fixed factor
  float decay;               // X multiplier (1 for M)
  int skip_zero;             // 1: entries with an all-zero momentum are left untouched
  // rank_stream_kernel<..., H3 = true> (the weight update: both factors bounded by 1 in
  // magnitude, P orthonormal, Qn column-normalised): power-of-two h3 scales fixed by that
  // bound instead of measured
  float h3_fixed_mul;        // s_fixed (a power of two)
  float h3_stream_scale;     // s_streamed (a power of two)
  float h3_inv;              // scale / (s_fixed s_streamed)
};

// fp16x3 ("h3") split types and helpers: see the h3 section below
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

struct Split2h {
  f16x8 hi, lo;
};

// power-of-two scale s (and 1/s) with amax * s in [2^14, 2^15); clamped to normal floats
__device__ __forceinline__ float h3_scale(float amax, float& inv) {
  const int be = static_cast<int>((__float_as_uint(amax) >> 23) & 0xFFu);  // biased exponent
  int es = 127 + 14 - (be - 127);                                           // 2^(14 - e)
  es = es < 1 ? 1 : (es > 253 ? 253 : es);  // s and inv both normal: inv == 1 / s exactly
  inv = __uint_as_float(static_cast<uint32_t>(254 - es) << 23);
  return __uint_as_float(static_cast<uint32_t>(es) << 23);
}

// s MUST be a power of two (every caller's is): x s is then exact, so the hi limb is the
// same whether the compiler forms it from the product in one step (v_fma_mixlo_f16) or
// from the fp32 product, and hi + lo represents x s.  With any other s the two roundings
// differ now and then and the pair misses x s by an ulp of hi.
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split2h(const f32x4& a, const f32x4& b, float s, Split2h& o) {
  // x s is rounded to fp32 ONCE and both limbs come from that value: with contraction the
  // compiler fuses x s - hi into one mixed-precision FMA on the exact product, and where
  // the rounded product is an fp16 tie, hi and lo then disagree by an ulp of hi.  Two values
  // per instruction (v_pk_mul_f32, v_cvt_pk_f16_f32, v_pk_add_f32): 3 VALU per value, not 5
#pragma clang fp contract(off)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f32x2 x = f32x2{j < 2 ? a[2 * j] : b[2 * j - 4], j < 2 ? a[2 * j + 1] : b[2 * j - 3]} * s;
    const f16x2v h = __builtin_convertvector(x, f16x2v);
    const f16x2v l = __builtin_convertvector(x - __builtin_convertvector(h, f32x2), f16x2v);
    o.hi[2 * j] = h[0];
    o.hi[2 * j + 1] = h[1];
    o.lo[2 * j] = l[0];
    o.lo[2 * j + 1] = l[1];
  }
}

struct Split3 {
  bf16x8 hi, mid, lo;
};

__device__ __forceinline__ void split3(const f32x4& a, const f32x4& b, float scale, Split3& o) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float x = (j < 4 ? a[j] : b[j - 4]) * scale;
    const __bf16 h = static_cast<__bf16>(x);
    const float r1 = x - static_cast<float>(h);
    const __bf16 m = static_cast<__bf16>(r1);
    const float r2 = r1 - static_cast<float>(m);
    o.hi[j] = h;
    o.mid[j] = m;
    o.lo[j] = static_cast<__bf16>(r2);
  }
}

__device__ __forceinline__ f32x16 mfma6(const Split3& A, const Split3& B, f32x16 acc) {
  // smallest terms first
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A.mid, B.mid, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A.lo, B.hi, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A.hi, B.lo, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A.mid, B.hi, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A.hi, B.mid, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A.hi, B.hi, acc, 0, 0, 0);
  return acc;
}

// D += A B on 32x32x16 fp16 with both operands h3-split (fp32 accumulate): the two small
// cross terms first
__device__ __forceinline__ f32x16 mfma3h32(const Split2h& A, const Split2h& B, f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(A.lo, B.hi, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(A.hi, B.lo, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(A.hi, B.hi, acc, 0, 0, 0);
  return acc;
}

template <int RU, bool PRE>
struct RTile {
  f32x4 s[RU][2];  // streamed factor row: 8 consecutive values per k-step (fp32, split per tile)
  f32x16 x;        // X tile (accumulator layout)
};

template <int RU>
struct RTile<RU, true> {
  u32x4 s[RU][3];  // streamed factor row, pre-split hi / mid / lo (presplit_kernel layout 2)
  f32x16 x;
};

// ============================================================================
// Rank-r update, block-shared streamed factor ("rank_stream"): the production
// weight / error-feedback path.  Same arithmetic and order as rank_update_kernel
// (bf16x6 on v_mfma_f32_32x32x16_bf16, accumulator from zero, X*decay + acc), but
//  - the NW waves of a block own NW adjacent 32-wide strips of the fixed side and
//    walk the same 32-long steps of the streamed side, so a step's streamed
//    factor rows (32 x r fp32) are loaded and split ONCE per block into LDS
//    (double-buffered, one barrier per step) instead of once per wave: the L2
//    factor traffic drops NW-fold and so does the split's VALU work;
//  - each wave keeps D X tiles in flight (register ring), with nt loads/stores.
// LDS layout of a step: [u][part][lane] bf16x8 (the 32x32x16 operand run of lane
// (t, h): factor row t, columns 16 u + 8 h .. +7), conflict-free ds_read_b128.
// ============================================================================
// rank_stream_kernel's tile offsets: 1 = the q-dependent part in the scalar offset (one VGPR
// of lane offset instead of 16: r = 128 135 -> 120 VGPRs, two 8-wave blocks per CU).  Measured
// (profiles/r06/p_ab_update_soff.txt): the r = 128 kernel alone 2.055 -> 1.977 ms, the steps
// slower (Mixtral 398.9 -> 396.2, Llama 484.3 -> 481.7 GiB/s): the second block takes issue
// slots from the other stream's kernel.  Kept at 0 (a dev build option)
#ifndef DION_RS_SOFF
#define DION_RS_SOFF 0
#endif
constexpr int kRsSoff = DION_RS_SOFF;
template <int RU, bool ROWFIX, int NW, int D, bool H3 = false>
__global__ void __launch_bounds__(64 * NW, (RU >= 7 || NW >= 8) ? 1 : 2) rank_stream_kernel(const RankArgs a) {
  constexpr int R = 16 * RU;
  constexpr int NT = 64 * NW;
  constexpr int kGroups = RU * 64;                   // 8-value groups of one 32-row step
  constexpr int kPer = (kGroups + NT - 1) / NT;      // groups per thread
  constexpr int NP = H3 ? 2 : 3;                     // limbs per staged value
  __shared__ bf16x8 sp[2][RU * NP * 64];
  const int b = blockIdx.z;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(tid >> 6));
  const int lane = tid & 63;
  const int t = lane & 31;
  const int h = lane >> 5;
  const int rows = a.rows, cols = a.cols;
  if (a.skip_zero && __builtin_amdgcn_readfirstlane(a.nonzero[b]) == 0u) return;
  const int flen = ROWFIX ? rows : cols;
  const int fbase = blockIdx.x * (32 * NW) + wave * 32;
  const bool active = fbase < flen;  // a wave past the edge still joins the block's staging and barriers
  const int s_begin = blockIdx.y * a.s_len;
  const int s_end = min(ROWFIX ? cols : rows, s_begin + a.s_len);
  const int ld = static_cast<int>(a.ld);
  const float* Sb = a.sptr[b] != nullptr ? a.sptr[b] : a.S + static_cast<long>(b) * a.s_stride;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      a.x[b], static_cast<short>(0), static_cast<int>(min(static_cast<long>(rows) * ld * 4, 0x7FFFFFF0L)), 0x00020000);
  // lane offset of tile value q: ((q & 3) + 8 (q >> 2) + 4 h) ld + t.  kRsSoff: the lane part
  // (4 h ld + t) in one VGPR, the q part (wave-uniform) in the scalar offset, instead of 16
  // VGPRs of offsets
  int voff[kRsSoff ? 1 : 16];
  if constexpr (kRsSoff) {
    voff[0] = (4 * h * ld + t) * 4;
  } else {
#pragma unroll
    for (int q = 0; q < 16; ++q) voff[q] = (((q & 3) + 8 * (q >> 2) + 4 * h) * ld + t) * 4;
  }
  auto qoff = [&](int q) { return ((q & 3) + 8 * (q >> 2)) * ld * 4; };

  Split3 F[H3 ? 1 : RU];
  Split2h FH[H3 ? RU : 1];
  if (active) {
    const float* fp = a.fixed[b] + static_cast<long>(fbase + t) * R + 8 * h;
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const f32x4 lo4 = *reinterpret_cast<const f32x4*>(fp + 16 * u);
      const f32x4 hi4 = *reinterpret_cast<const f32x4*>(fp + 16 * u + 4);
      if constexpr (H3)
        split2h(lo4, hi4, a.h3_fixed_mul, FH[u]);
      else
        split3(lo4, hi4, a.scale, F[u]);
    }
  }

  // staging of one step's streamed rows: thread item g = tid + NT * it -> (u, lane') =
  // (g / 64, g % 64): row s0 + lane' % 32, columns 16 u + 8 (lane' / 32) .. +7
  f32x4 pv[kPer][2];
  auto p_load = [&](int s0) {
#pragma unroll
    for (int it = 0; it < kPer; ++it) {
      const int g = tid + NT * it;
      if (g < kGroups) {
        const int u = g >> 6, l = g & 63;
        const float* src = Sb + static_cast<long>(s0 + (l & 31)) * R + 16 * u + 8 * (l >> 5);
        pv[it][0] = *reinterpret_cast<const f32x4*>(src);
        pv[it][1] = *reinterpret_cast<const f32x4*>(src + 4);
      }
    }
  };
  auto p_store = [&](bf16x8* dst) {
#pragma unroll
    for (int it = 0; it < kPer; ++it) {
      const int g = tid + NT * it;
      if (g < kGroups) {
        const int u = g >> 6, l = g & 63;
        if constexpr (H3) {
          Split2h o;
          split2h(pv[it][0], pv[it][1], a.h3_stream_scale, o);
          dst[(u * 2 + 0) * 64 + l] = __builtin_bit_cast(bf16x8, o.hi);
          dst[(u * 2 + 1) * 64 + l] = __builtin_bit_cast(bf16x8, o.lo);
        } else {
          Split3 o;
          split3(pv[it][0], pv[it][1], 1.f, o);
          dst[(u * 3 + 0) * 64 + l] = o.hi;
          dst[(u * 3 + 1) * 64 + l] = o.mid;
          dst[(u * 3 + 2) * 64 + l] = o.lo;
        }
      }
    }
  };

  f32x16 X[D];
  auto x_load = [&](int s0, f32x16& T) {
    const int row0 = ROWFIX ? fbase : s0;
    const int col0 = ROWFIX ? s0 : fbase;
    const int so = (row0 * ld + col0) * 4;
#pragma unroll
    for (int q = 0; q < 16; ++q)
      T[q] = __uint_as_float(kRsSoff ? __builtin_amdgcn_raw_buffer_load_b32(rx, voff[0], so + qoff(q), kStreamAux)
                                     : __builtin_amdgcn_raw_buffer_load_b32(rx, voff[kRsSoff ? 0 : q], so, kStreamAux));
  };
  auto compute_store = [&](int s0, const f32x16& T, const bf16x8* src) {
    f32x16 acc;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.f;
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      if constexpr (H3) {
        Split2h Sp;
        Sp.hi = __builtin_bit_cast(f16x8, src[(u * 2 + 0) * 64 + lane]);
        Sp.lo = __builtin_bit_cast(f16x8, src[(u * 2 + 1) * 64 + lane]);
        acc = ROWFIX ? mfma3h32(FH[u], Sp, acc) : mfma3h32(Sp, FH[u], acc);
      } else {
        Split3 Sp;
        Sp.hi = src[(u * 3 + 0) * 64 + lane];
        Sp.mid = src[(u * 3 + 1) * 64 + lane];
        Sp.lo = src[(u * 3 + 2) * 64 + lane];
        acc = ROWFIX ? mfma6(F[u], Sp, acc) : mfma6(Sp, F[u], acc);
      }
    }
    const int row0 = ROWFIX ? fbase : s0;
    const int col0 = ROWFIX ? s0 : fbase;
    const int so = (row0 * ld + col0) * 4;
    const float ainv = H3 ? a.h3_inv : 1.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      // X d rounded first (the reference's W.mul_(1 - lr wd)), then the update added
      const float v = H3 ? fmaf(acc[q], ainv, __fmul_rn(T[q], a.decay)) : __fmul_rn(T[q], a.decay) + acc[q];
      if constexpr (kRsSoff)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rx, voff[0], so + qoff(q), kStreamAux);
      else
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rx, voff[kRsSoff ? 0 : q], so, kStreamAux);
    }
  };

  // prologue: step 0's factor rows into LDS, X tiles of steps 0 .. D-2 in flight
  p_load(s_begin);
  if (active) {
#pragma unroll
    for (int k = 0; k < D - 1; ++k)
      if (s_begin + 32 * k < s_end) x_load(s_begin + 32 * k, X[k]);
  }
  p_store(sp[0]);
  __syncthreads();
  int cur = 0;
  for (int s0 = s_begin; s0 < s_end; s0 += 32 * D) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const int s = s0 + 32 * k;
      if (s >= s_end) break;
      const bool more = s + 32 < s_end;
      if (more) p_load(s + 32);
      if (active && s + 32 * (D - 1) < s_end) x_load(s + 32 * (D - 1), X[(k + D - 1) % D]);
      if (active) compute_store(s, X[k], sp[cur]);
      if (!more) break;
      p_store(sp[cur ^ 1]);
      __syncthreads();
      cur ^= 1;
    }
  }
}

// ============================================================================
// Upper Cholesky of the r x r Gram matrix (ortho.py:112-115, cholesky_ex upper) with the
// matrix in registers: thread (g, c) of NG = 256 / RP row groups holds column c of rows
// g, g + NG, ..  Pivot j: its owner group publishes row j through LDS (ping-pong, one
// barrier), every thread forms u_j* = row / sqrt(d_j) for its column and rows and updates
// them, G[i][c] -= u_ji u_jc: the fused products of chol_inv_kernel (and of dpotf2's dot
// products) in the same k order, so the same factor.  Output: the padded factor + reciprocal
// diagonal of trsm_right_kernel<RP>; G is padded to RP with the identity.  A non-positive
// pivot stops the factorisation: its row and the later ones get a NaN diagonal, so the solve
// turns their P columns into NaN (cholesky_ex does not raise; the fix-up's nan_to_num zeroes
// them, ortho.py:113 / kernels.py:157-204).
// ============================================================================
template <int RP, int NT = 256, bool TINV = false>
__global__ void __launch_bounds__(NT) chol_reg_kernel(const float* __restrict__ G_in, float* __restrict__ Fout,
                                                      int r) {
  constexpr int NG = NT / RP, RPT = RP / NG;
  __shared__ float row[2][RP];
  // TINV: the factor kept in LDS and inverted in fp32 right after (tri_inv_cols, NG lanes per
  // column); Fout then receives R^-1 (RP x RP) instead of the padded factor
  __shared__ float Fs[TINV ? RP * RP + RP : 1];
  __shared__ float Xs[TINV ? RP * (RP + NG) : 1];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int c = tid % RP, g = tid / RP;
  const float* Gm = G_in + static_cast<long>(b) * r * r;
  float* O = Fout + static_cast<long>(b) * (RP * RP + RP);
  float a[RPT];
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int i = g + NG * q;
    a[q] = (i < r && c < r) ? Gm[i * r + c] : (i == c ? 1.f : 0.f);
  }
  int jf = RP;
#pragma unroll 1
  for (int j = 0; j < RP; ++j) {
    const int buf = j & 1;
    if (g == j % NG) {
#pragma unroll
      for (int q = 0; q < RPT; ++q)
        if (q == j / NG) row[buf][c] = a[q];
    }
    __syncthreads();
    const float d = row[buf][j];
    if (!(d > 0.f)) {  // uniform
      jf = j;
      break;
    }
    const float ujj = sqrtf(d);
    const float inv = 1.f / ujj;
    const float uc = row[buf][c] * inv;
    if constexpr (TINV) {
      if (g == j % NG) Fs[j * RP + c] = c < j ? 0.f : (c == j ? ujj : uc);
      if (tid == 0) Fs[RP * RP + j] = inv;
    } else {
      if (g == j % NG) O[j * RP + c] = c < j ? 0.f : (c == j ? ujj : uc);
      if (tid == 0) O[RP * RP + j] = inv;
    }
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const int i = g + NG * q;
      if (i > j) a[q] -= (row[buf][i] * inv) * uc;
    }
  }
  float* F = TINV ? Fs : O;
  for (int idx = tid; idx < (RP - jf) * RP; idx += NT) {
    const int i = jf + idx / RP, cc = idx % RP;
    F[i * RP + cc] = (i == cc) ? __builtin_nanf("") : 0.f;
  }
  for (int j = jf + tid; j < RP; j += NT) F[RP * RP + j] = __builtin_nanf("");
  if constexpr (TINV) {
    __syncthreads();
    tri_inv_cols<NG>(Fs, RP, Fs + RP * RP, Xs, RP + NG, RP, Fout + static_cast<long>(b) * RP * RP, tid, NT);
  }
}

// ============================================================================
// X_b = P_b R_b^-1 for an upper-triangular R_b: the triangular solves of the RCQR
// (ortho.py:105-121, torch.linalg.solve_triangular(R, P, upper=True, left=False)), one row
// per thread as the reference BLAS strsm (right, upper, no transpose) orders it:
//   x_j = (p_j - sum_{k<j} R_kj x_k) * (1 / R_jj)
// with the subtractions in k order (right-looking: once x_k is final, every later x_j takes
// its fused term).  R (the factor kernels' padded RT x RT layout plus reciprocal diagonal)
// is read with wave-uniform addresses from a per-block LDS copy (broadcast reads).  Scalar
// (s_load) reads of the factor measured faster ALONE at RT <= 64 (fc1 group 76.5 vs 130 us,
// scripts/ubench/trsm_ab.hip) but slower inside the two-stream Llama step (456.5 / 457.8 GiB/s
// with LDS factors against 450.6 / 451.5, same box, profiles/r05/k_ab_and_solves.txt), where the
// solves share the scalar caches and L2 with the streaming kernels; at RT = 128 scalar reads
// thrash the scalar cache outright (2272 vs 176 us per fc1-size launch, even with the factor
// read in three 16 KB blocks).  The vector traffic is the row in and out.  Columns past r are
// zero and stay zero.  In place (src == dst) is allowed.
// ============================================================================
#ifndef DION_TRSM_LDS_MIN_RT
#define DION_TRSM_LDS_MIN_RT 32  // the smallest padded order whose solve stages the factor in LDS
#endif
template <int RT>
__global__ void __launch_bounds__(256) trsm_right_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                         const float* __restrict__ Rf, int mp, int r,
                                                         const uint32_t* __restrict__ nonzero) {
  // DION_TRSM_LDS_MIN_RT (a dev build option for A/B runs): below it, scalar factor loads
  constexpr bool kLds = RT >= DION_TRSM_LDS_MIN_RT;
  __shared__ f32x4 Rs4[kLds ? (RT * RT + RT) / 4 : 1];
  const int b = blockIdx.y;
  const float* R = Rf + static_cast<long>(b) * (RT * RT + RT);
  if constexpr (kLds) {
    const f32x4* Rg = reinterpret_cast<const f32x4*>(R);
    for (int i = threadIdx.x; i < (RT * RT + RT) / 4; i += 256) Rs4[i] = Rg[i];
    __syncthreads();
    R = reinterpret_cast<const float*>(Rs4);
  }
  const long row = static_cast<long>(blockIdx.x) * 256 + threadIdx.x;
  if (row >= mp) return;
  const float* p = src + (static_cast<long>(b) * mp + row) * r;
  float x[RT];
  if ((r & 3) == 0) {
#pragma unroll
    for (int j = 0; j < RT; j += 4) {
      if (j < r) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(p + j);
        x[j] = v[0], x[j + 1] = v[1], x[j + 2] = v[2], x[j + 3] = v[3];
      } else {
        x[j] = x[j + 1] = x[j + 2] = x[j + 3] = 0.f;
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < RT; ++j) x[j] = j < r ? p[j] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < RT; ++k) {
    x[k] *= R[RT * RT + k];
#pragma unroll
    for (int j = k + 1; j < RT; ++j) x[j] = fmaf(-x[k], R[k * RT + j], x[j]);
  }
  if (nonzero != nullptr) {
    // the last solve of the RCQR with pfix_kernel folded in (kernels.py:185-188)
    const bool zero = nonzero[b] == 0u;
#pragma unroll
    for (int j = 0; j < RT; ++j) x[j] = zero ? 0.f : nan_to_num(x[j]);
  }
  float* q = dst + (static_cast<long>(b) * mp + row) * r;
  if ((r & 3) == 0) {
#pragma unroll
    for (int j = 0; j < RT; j += 4)
      if (j < r) *reinterpret_cast<f32x4*>(q + j) = f32x4{x[j], x[j + 1], x[j + 2], x[j + 3]};
  } else {
#pragma unroll
    for (int j = 0; j < RT; ++j)
      if (j < r) q[j] = x[j];
  }
}

// The same solve for r = RT = 32 or 64 with the rows staged through LDS.  trsm_right_kernel
// reads a row per lane straight from HBM (each load instruction touches 64 rows); here each
// wave owns 64 consecutive rows (one contiguous 64 x RT fp32 block), stages them by LDS-DMA
// (global_load_lds_dwordx4: every instruction reads 1 KB of consecutive lines), solves its
// row from LDS, writes the row back into the same LDS image and stores the block as
// consecutive lines.  No block barrier: a wave reads only what it loaded.  The LDS image is
// XOR-swizzled by 16-B chunk (chunk c of row i at slot i CH + (c ^ swz(i))) so the per-row
// ds_read_b128 / ds_write_b128 are conflict-free; the DMA's LDS side is lane-linear, so the
// swizzle is applied on the source offsets.  Same arithmetic, in the same order, as
// trsm_right_kernel (bitwise identical).
//
// FINAL (the last solve of the RCQR, P = P1 R2^-1) can fold in what follows it on the W = 1
// path, from the LDS image of the finished rows:
//   * `nonzero`: the fix-up of P (kernels.py:185-188, pfix_kernel): z ? 0 : nan_to_num(x);
//   * `psplit`: the fp16x3 limbs of P in pass B's operand layout (presplit16_kernel layout 0,
//     `kmap`), on the fixed scale 2^14: the columns of P are orthonormal, so |x| <= 1 and
//     x 2^14 stays far inside fp16 (the measured-maximum scale of presplit16 would be 2^14 or
//     larger); a NaN column stays NaN in both limbs.  Pass B then needs no absmax / presplit.
template <int RT>
__device__ __forceinline__ int trsm_swz(int row) {
  return RT == 64 ? (row & 15) : ((row >> 1) & 7);
}
constexpr float kPSplitScale = 16384.f;  // 2^14: the fixed h3 scale of an orthonormal P
constexpr float kPSplitInv = 1.f / 16384.f;

struct TrsmArgs {
  const float* src;
  float* dst;
  const float* fac;           // (batch, RT RT + RT): factor + reciprocal diagonal
  const uint32_t* nonzero;    // FINAL: fix P with these flags (null: no fix)
  f16x8* psplit;              // FINAL: pass-B split of P (null: none)
  long pstride;               // f16x8 units per matrix of psplit
  int mp, kmap;
  float* gram;                // tsolve_mfma_kernel GRAM: (batch, gridDim.x, RT, RT) partial Grams of X
};

constexpr int kTrsmWaves = 2;  // 128-row blocks: 2 x 16 KB row images

template <int RT, bool FINAL>
__global__ void __launch_bounds__(64 * kTrsmWaves, 3) trsm_lds_kernel(const TrsmArgs a) {
  static_assert(RT == 32 || RT == 64, "trsm_lds_kernel: r = 32 or 64");
  constexpr int CH = RT / 4;  // 16-B chunks per row
  constexpr int RB = RT / 16;
  __shared__ f32x4 img[kTrsmWaves][64 * CH];
  // the factor as in trsm_right_kernel: scalar loads, or a per-block LDS copy
  constexpr bool kLds = RT >= DION_TRSM_LDS_MIN_RT;
  __shared__ f32x4 Rs4[kLds ? (RT * RT + RT) / 4 : 1];
  const int b = blockIdx.y;
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6)), lane = threadIdx.x & 63;
  const long row0 = static_cast<long>(blockIdx.x) * (64 * kTrsmWaves) + wave * 64;
  const int mp = a.mp;
  const int nrows = static_cast<int>(min(static_cast<long>(64), static_cast<long>(mp) - row0));
  const float* R = a.fac + static_cast<long>(b) * (RT * RT + RT);  // wave-uniform (scalar) loads
  if constexpr (kLds) {
    const f32x4* Rg = reinterpret_cast<const f32x4*>(R);
    for (int i = threadIdx.x; i < (RT * RT + RT) / 4; i += 64 * kTrsmWaves) Rs4[i] = Rg[i];
    __syncthreads();
    R = reinterpret_cast<const float*>(Rs4);
  }
  if (nrows <= 0) return;
  f32x4* w = img[wave];
  const char* s = reinterpret_cast<const char*>(a.src + (static_cast<long>(b) * mp + row0) * RT);
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int slot = 64 * i + lane, row = slot / CH, cp = slot % CH;
    if (row < nrows) glds16<false>(s, static_cast<uint32_t>((row * CH + (cp ^ trsm_swz<RT>(row))) * 16), lds_off(&w[64 * i]));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float x[RT];
  if (lane < nrows) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const f32x4 v = w[lane * CH + (c ^ trsm_swz<RT>(lane))];
      x[4 * c] = v[0], x[4 * c + 1] = v[1], x[4 * c + 2] = v[2], x[4 * c + 3] = v[3];
    }
#pragma unroll
    for (int k = 0; k < RT; ++k) {
      x[k] *= R[RT * RT + k];
#pragma unroll
      for (int j = k + 1; j < RT; ++j) x[j] = fmaf(-x[k], R[k * RT + j], x[j]);
    }
    if constexpr (FINAL) {
      if (a.nonzero != nullptr) {
        const bool zero = a.nonzero[b] == 0u;
#pragma unroll
        for (int j = 0; j < RT; ++j) x[j] = zero ? 0.f : nan_to_num(x[j]);
      }
    }
#pragma unroll
    for (int c = 0; c < CH; ++c)
      w[lane * CH + (c ^ trsm_swz<RT>(lane))] = f32x4{x[4 * c], x[4 * c + 1], x[4 * c + 2], x[4 * c + 3]};
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  f32x4* d = reinterpret_cast<f32x4*>(a.dst + (static_cast<long>(b) * mp + row0) * RT);
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int slot = 64 * i + lane, row = slot / CH, cp = slot % CH;
    if (row < nrows) d[row * CH + (cp ^ trsm_swz<RT>(row))] = w[slot];
  }
  if constexpr (FINAL) {
    if (a.psplit != nullptr) {
      // unit (32-row block q, column block cb), lane (t, g): rows 32 q + kmap(g, e), column 16 cb + t
      const float* wf = reinterpret_cast<const float*>(w);
      const int t = lane & 15, g = lane >> 4;
      f16x8* out = a.psplit + b * a.pstride;
#pragma unroll
      for (int u = 0; u < 2 * RB; ++u) {
        const int q = u / RB, cb = u % RB;
        if (32 * q >= nrows) break;
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int row = 32 * q + (a.kmap == 0 ? 8 * g + e : 16 * (e >> 2) + 4 * g + (e & 3));
          const int col = 16 * cb + t;
          v[e] = wf[(row * CH + ((col >> 2) ^ trsm_swz<RT>(row))) * 4 + (col & 3)];
        }
        Split2h sp;
        split2h(f32x4{v[0], v[1], v[2], v[3]}, f32x4{v[4], v[5], v[6], v[7]}, kPSplitScale, sp);
        const long grp = (row0 / 32 + q) * RB + cb;
        out[grp * 128 + lane] = sp.hi;
        out[grp * 128 + 64 + lane] = sp.lo;
      }
    }
  }
}

// ============================================================================
// S P for a generated sketch (ortho.py:90-104: SP = sketch @ P, k = ceil(1.25 r / 128) 128
// rows).  The reference draws S ~ N(0, 1/k) from the unseeded global RNG (ortho.py:659-661),
// so any draw is as valid as its own, and the randomised Cholesky QR returns the same
// orthonormal P up to column signs for every full-rank sketch.  Here S is
// a Rademacher sketch, S[k][i] = +-1/sqrt(k) with the sign the bit (i mod 32) of a 32-bit
// hash of (seed, matrix, k, i / 32): exact in bf16, so one operand of the product needs no
// split, P is split into three bf16 limbs (24 bits), and S P is three bf16 MFMAs per tile
// instead of the fp32 MFMA (16x slower) with a Box-Muller draw per element.
//   v_mfma_f32_32x32x16_bf16: A = S tile (32 sketch rows x 16 P rows, from the sign
//   bits), B = P tile (16 rows x 32 columns, 8 rows of one column per lane).  A block takes
//   kchunk rows of one matrix in 32-row panels, each loaded once (16-byte loads, one panel
//   ahead) into LDS for all four waves; wave w owns sketch-row tiles w, w + 4 (KT4 of them)
//   and all NT column tiles, so no cross-wave reduction; partial sums go to fixed-order
//   slabs (reduce_slabs_kernel).
// ============================================================================
__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

// 8 sign bits -> 8 bf16 values +-1 (bit j set: element j is -1)
__device__ __forceinline__ bf16x8 signs_bf16x8(uint32_t bits) {
  u32x4 w;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t v = bits >> (2 * q);
    w[q] = 0x3F803F80u | ((v & 1u) << 15) | ((v & 2u) << 30);
  }
  return __builtin_bit_cast(bf16x8, w);
}

struct SketchArgs {
  const float* P;   // (batch, mp, r)
  float* out;       // (batch, nchunk, K, r) partial sums (the final (batch, K, r) when nchunk == 1)
  uint64_t seed;
  float scale;      // 1 / sqrt(K)
  int mp, r, K, kchunk, nchunk;
  int vec;          // P 16-byte aligned and r % 4 == 0
};

template <int KT4, int NT>
__global__ void __launch_bounds__(256, 2) sketch_rad_kernel(const SketchArgs a) {
  constexpr int R = 32 * NT;  // the column tiles (r <= R; the tile's columns past r are zero)
  __shared__ __attribute__((aligned(16))) float tile[2][32 * R];
  const int b = blockIdx.y, chunk = blockIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int tid = threadIdx.x, lane = tid & 63, t = lane & 31, h = lane >> 5;
  const int i_begin = chunk * a.kchunk;
  const int i_end = min(a.mp, i_begin + a.kchunk);
  const int r = a.r;
  const float* __restrict__ Pb = a.P + static_cast<long>(b) * a.mp * r;
  const uint32_t sb = hash32(static_cast<uint32_t>(a.seed) ^ hash32(static_cast<uint32_t>(a.seed >> 32) +
                                                                      0x9E3779B9u * static_cast<uint32_t>(b + 1)));
  uint32_t hk[KT4];
#pragma unroll
  for (int q = 0; q < KT4; ++q) hk[q] = hash32(sb + 0x85EBCA6Bu * static_cast<uint32_t>(32 * (wave + 4 * q) + t));
  f32x16 acc[KT4][NT];
#pragma unroll
  for (int q = 0; q < KT4; ++q)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[q][nt][e] = 0.f;
  // the 32-row panel P[i0 .. i0 + 31][0 .. r) staged through LDS once per block (one 16-byte
  // slot per thread and column tile), loaded one panel ahead; rows past i_end are zero
  f32x4 pre[NT];
  auto load = [&](int i0) {
#pragma unroll
    for (int v = 0; v < NT; ++v) {
      const int idx = tid + 256 * v, row = i0 + idx / (R / 4), c = 4 * (idx % (R / 4));
      if (row < i_end && a.vec && c < r) {
        pre[v] = *reinterpret_cast<const f32x4*>(Pb + static_cast<long>(row) * r + c);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) pre[v][e] = (row < i_end && c + e < r) ? Pb[static_cast<long>(row) * r + c + e] : 0.f;
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int v = 0; v < NT; ++v) reinterpret_cast<f32x4*>(tile[buf])[tid + 256 * v] = pre[v];
  };
  if (i_begin >= i_end) return;
  load(i_begin);
  store(0);
  __syncthreads();
  int cur = 0;
  for (int i0 = i_begin; i0 < i_end; i0 += 32) {
    const bool more = i0 + 32 < i_end;
    if (more) load(i0 + 32);
    uint32_t bits[KT4];
#pragma unroll
    for (int q = 0; q < KT4; ++q) bits[q] = hash32(hk[q] ^ (0xC2B2AE35u * static_cast<uint32_t>(i0 >> 5)));
#pragma unroll 1
    for (int half = 0; half < 2; ++half) {
      bf16x8 S[KT4];
#pragma unroll
      for (int q = 0; q < KT4; ++q) S[q] = signs_bf16x8(bits[q] >> (16 * half + 8 * h));
      // one column tile at a time (all NT split tiles live would cost a wave per SIMD at
      // r = 128); the KT4 accumulators of a limb are independent MFMAs
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = tile[cur][(16 * half + 8 * h + j) * R + 32 * nt + t];
        Split3 B;
        split3(f32x4{v[0], v[1], v[2], v[3]}, f32x4{v[4], v[5], v[6], v[7]}, 1.f, B);
#pragma unroll
        for (int q = 0; q < KT4; ++q) acc[q][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(S[q], B.lo, acc[q][nt], 0, 0, 0);
#pragma unroll
        for (int q = 0; q < KT4; ++q) acc[q][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(S[q], B.mid, acc[q][nt], 0, 0, 0);
#pragma unroll
        for (int q = 0; q < KT4; ++q) acc[q][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(S[q], B.hi, acc[q][nt], 0, 0, 0);
      }
    }
    if (!more) break;
    store(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
  float* out = a.out + (static_cast<long>(b) * a.nchunk + chunk) * a.K * r;
#pragma unroll
  for (int q = 0; q < KT4; ++q)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int col = 32 * nt + t;
      if (col >= r) continue;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int krow = 32 * (wave + 4 * q) + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (krow < a.K) out[static_cast<long>(krow) * r + col] = acc[q][nt][e] * a.scale;
      }
    }
}

// ============================================================================
// Pass A with the previous step's error feedback folded in ("deferred EF").
//   X = (M + alpha P'_b R'_b^T) + G      (transposed: alpha R'_b P'_b^T)
//   M <- X ;  P = X Q  (or X^T Q) ;  nonzero flag
// P'_b, R'_b are the previous step's factors of matrix b (after the fix-up);
// alpha = -(1 - mu).  The sum order is the reference's: the step-t error
// feedback lands on M before the step-(t+1) gradient (kernels.py:54-83 then
// runtime.py:1560-1566), so M matches the eager schedule.  Saves the M read +
// write of the separate error-feedback launch (8 of the 30 B per element).
// The EF product is split-bf16 (bf16x6) on v_mfma_f32_16x16x32_bf16, laid out
// so its accumulator is exactly the lane's slice of the M tile; the
// projection stays fp32 MFMA.  The streamed factor rows (R' for the row
// kernel, R' rows for the column kernel) are split once per block per step
// into LDS; the wave's fixed factor is split once into registers.
// ============================================================================
struct EfProjArgs {
  ProjArgs p;
  const float* efp[MAXB];  // pending P'_b (m_P x r) or null (no pending EF for b)
  const float* efr[MAXB];  // pending R'_b (n_Q x r)
  const u32x4* qsplit;     // Q_b pre-split, B-operand layout (KMAP 1), split_stride 16-byte units per matrix
  const u32x4* rsplit;     // R'_b pre-split, A-operand layout
  long split_stride;
  float alpha;
  const uint32_t* amax;    // h3 kernels: (2, batch) max |x| bits of Q, R' (P' is split on the fixed scale 2^14)
  const float* inv;        // h3 kernels: (2, batch) 1 / scale of the Q and R' splits
};

// Pre-split of a small factor (rows x r fp32) into hi/mid/lo bf16, laid out so a
// K-step's operands are one contiguous run: dst[(grp * 3 + part) * 64 + lane].
//   layout 0 (B operand):  grp = (row / 32) * RB + cb, lane (t, g) <- rows 32 blk + kmap(g, e), column 16 cb + t
//   layout 1 (A operand):  grp = (row / 16) * KK + kk, lane (t, g) <- row 16 blk + t, columns 32 kk + 8 g + e
struct PresplitArgs {
  const float* src[MAXB];
  u32x4* dst;
  long stride;  // 16-byte units per matrix
  int rows, r, layout, kmap;
};

__global__ void __launch_bounds__(256) presplit_kernel(const PresplitArgs a) {
  const int b = blockIdx.y;
  const float* __restrict__ src = a.src[b];
  if (src == nullptr) return;
  const long items = static_cast<long>(a.rows) * a.r / 8;
  const long item = static_cast<long>(blockIdx.x) * 256 + threadIdx.x;
  if (item >= items) return;
  const int ln = static_cast<int>(item & 63);
  const long grp = item >> 6;
  const int t = ln & 15, g = ln >> 4;
  float v[8];
  if (a.layout == 0) {
    const int RB = a.r / 16;
    const long blk = grp / RB;
    const int cb = static_cast<int>(grp - blk * RB);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = a.kmap == 0 ? 8 * g + e : 16 * (e >> 2) + 4 * g + (e & 3);
      v[e] = src[(blk * 32 + k) * a.r + 16 * cb + t];
    }
  } else if (a.layout == 1) {
    const int KK = a.r / 32;
    const long blk = grp / KK;
    const int kk = static_cast<int>(grp - blk * KK);
    const float* p = src + (blk * 16 + t) * a.r + 32 * kk + 8 * g;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = p[e];
  } else {
    // layout 2 (32x32x16 operand of rank_update_kernel): grp = (row / 32) * RU + u,
    // lane (t5 = lane & 31, h = lane >> 5) <- row 32 blk + t5, columns 16 u + 8 h + e
    const int RU = a.r / 16;
    const long blk = grp / RU;
    const int u = static_cast<int>(grp - blk * RU);
    const float* p = src + (blk * 32 + (ln & 31)) * a.r + 16 * u + 8 * (ln >> 5);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = p[e];
  }
  Split3 sp;
  split3(f32x4{v[0], v[1], v[2], v[3]}, f32x4{v[4], v[5], v[6], v[7]}, 1.f, sp);
  u32x4* d = a.dst + b * a.stride + (grp * 3) * 64 + ln;
  d[0] = __builtin_bit_cast(u32x4, sp.hi);
  d[64] = __builtin_bit_cast(u32x4, sp.mid);
  d[128] = __builtin_bit_cast(u32x4, sp.lo);
}

// Copy of one K-step's pre-split operands (NU 16-byte units, contiguous) into LDS.
template <int NU>
struct SplitCopy {
  static constexpr int kPer = (NU + 255) / 256;
  u32x4 v[kPer];
};

template <int NU>
__device__ __forceinline__ void split_copy_load(SplitCopy<NU>& C, const u32x4* __restrict__ src, int tid) {
#pragma unroll
  for (int it = 0; it < SplitCopy<NU>::kPer; ++it)
    if (NU % 256 == 0 || tid + 256 * it < NU) C.v[it] = src[tid + 256 * it];
}

template <int NU>
__device__ __forceinline__ void split_copy_store(const SplitCopy<NU>& C, bf16x8* dst, int tid) {
  u32x4* d = reinterpret_cast<u32x4*>(dst);
#pragma unroll
  for (int it = 0; it < SplitCopy<NU>::kPer; ++it)
    if (NU % 256 == 0 || tid + 256 * it < NU) d[tid + 256 * it] = C.v[it];
}

// the same staging copy for blocks of NT threads
template <int NU, int NT>
struct SplitCopyN {
  static constexpr int kPer = (NU + NT - 1) / NT;
  u32x4 v[kPer];
};

template <int NU, int NT>
__device__ __forceinline__ void split_copy_load_n(SplitCopyN<NU, NT>& C, const u32x4* __restrict__ src, int tid) {
#pragma unroll
  for (int it = 0; it < SplitCopyN<NU, NT>::kPer; ++it)
    if (NU % NT == 0 || tid + NT * it < NU) C.v[it] = src[tid + NT * it];
}

template <int NU, int NT>
__device__ __forceinline__ void split_copy_store_n(const SplitCopyN<NU, NT>& C, bf16x8* dst, int tid) {
  u32x4* d = reinterpret_cast<u32x4*>(dst);
#pragma unroll
  for (int it = 0; it < SplitCopyN<NU, NT>::kPer; ++it)
    if (NU % NT == 0 || tid + NT * it < NU) d[tid + NT * it] = C.v[it];
}

__device__ __forceinline__ f32x4 mfma6_16(const Split3& A, const Split3& B, f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A.mid, B.mid, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A.lo, B.hi, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A.hi, B.lo, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A.mid, B.hi, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A.hi, B.mid, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A.hi, B.hi, acc, 0, 0, 0);
  return acc;
}

__device__ __forceinline__ void ef_sread(const bf16x8* rs, int ck, int lane, Split3& A) {
  A.hi = rs[(ck * 3 + 0) * 64 + lane];
  A.mid = rs[(ck * 3 + 1) * 64 + lane];
  A.lo = rs[(ck * 3 + 2) * 64 + lane];
}

template <int KMAP>
__device__ __forceinline__ int kmap(int g, int e) {
  return KMAP == 0 ? 8 * g + e : 16 * (e >> 2) + 4 * g + (e & 3);
}

// swizzle of the 32 x 8 (16-byte unit) LDS transpose tile: chunk k of row r is stored at
// k ^ ((r >> 1) & 7), conflict-free for 16 consecutive lanes on 64 banks (the alternative
// 5 (r >> 1) & 7 measured twice the bank conflicts, round 2)
// slot swizzle of the [rows][8 x 16 B] transpose tiles: row r's slot k sits at k ^ (r & 7).
// Conflict-free for every access the row kernels make (cdna_hip_programming.md section 2 bank
// rules): row-wise ds_write_b128 (8 lanes = one row) and ds_read_b128, and lane (t, g) =
// (row t, slot 4c + g) ds_read_b128 AND ds_write_b128 -- the earlier (r >> 1) & 7 put rows
// 2i, 2i + 1 of an 8-lane write group on one 16-B slot (2-way, rowproj_efh3_kernel's
// write-back: 32 extra LDS cycles per wave-step)
__device__ __forceinline__ int xt_swz(int r) { return r & 7; }

constexpr int kRBE = 2;   // 16-row blocks per wave in the fused row kernel (measured default)

// ---- row kernel (not transposed): wave = kRBE x 16 rows, step = 32 columns;
// lane (t, g) holds columns 16c + 4g .. +3 (c = 0, 1) of rows 16 rb + t.
template <int GDT, int KR = kRBE>
struct RowStepE {
  f32x4 x[KR][2];
  uint2 gb[KR][2];
  f32x4 gf[KR][2];
};

template <int GDT, int KR = kRBE>
__device__ __forceinline__ void rpe_load(RowStepE<GDT, KR>& S, const float* __restrict__ M, const void* __restrict__ G,
                                         long ld_m, long ld_g, int j) {
#pragma unroll
  for (int rb = 0; rb < KR; ++rb)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      if (M != nullptr) S.x[rb][c] = ld_part(reinterpret_cast<const f32x4*>(M + rb * 16 * ld_m + j + 16 * c));
      if constexpr (GDT == DION_DTYPE_BF16)
        S.gb[rb][c] = ld_part(reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(G) + rb * 16 * ld_g + j + 16 * c));
      else if constexpr (GDT == DION_DTYPE_F32)
        S.gf[rb][c] = ld_part(reinterpret_cast<const f32x4*>(static_cast<const float*>(G) + rb * 16 * ld_g + j + 16 * c));
    }
}


// ---- column kernel (transposed): block = 4 waves x 32 columns, step = 32 rows;
// lane (t, g) holds columns 2t, 2t + 1 of rows 16 h + 4 g + q (h = 0, 1; q = 0..3):
// per half h that is the EF accumulator's slice, and per column the 8 rows are
// the projection's k-run (KMAP 1).
// cache policy of the transposed pass A's bf16 G loads (64-B row pieces): nt (measured faster)
constexpr int kCpeGnt = 1;

template <int GDT>
struct ColStepE {
  f32x2 x[2][4];
  uint32_t gb[2][4];
  f32x2 gf[2][4];
};

template <int GDT>
__device__ __forceinline__ void cpe_load(ColStepE<GDT>& S, const float* __restrict__ M, const void* __restrict__ G,
                                         long ld_m, long ld_g, int i0) {
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const long row = i0 + 16 * h + q;
      S.x[h][q] = ld_stream(reinterpret_cast<const f32x2*>(M + row * ld_m));
      if constexpr (GDT == DION_DTYPE_BF16)
        S.gb[h][q] = kCpeGnt
                         ? ld_stream(reinterpret_cast<const uint32_t*>(static_cast<const uint16_t*>(G) + row * ld_g))
                         : *reinterpret_cast<const uint32_t*>(static_cast<const uint16_t*>(G) + row * ld_g);
      else if constexpr (GDT == DION_DTYPE_F32)
        S.gf[h][q] = ld_stream(reinterpret_cast<const f32x2*>(static_cast<const float*>(G) + row * ld_g));
    }
}


// ---- column projection, no gradient (pass B, not transposed: R = M^T P):
// block = 4 waves x 16 CT columns, K-step = 32 rows; lane (t, g) loads the run
// of columns CT t .. CT t + CT - 1 of rows 8g + e (e = 0..7): per tile c
// (columns CT t + c) its 8 values are the A operand's k-run, KMAP 0.
template <int CT>
struct ColStepX6 {
  typedef float vec __attribute__((ext_vector_type(CT)));
  vec x[8];
};

template <int CT>
__device__ __forceinline__ void cpx_load(ColStepX6<CT>& S, const float* __restrict__ M, long ld_m, int i0) {
  typedef typename ColStepX6<CT>::vec vec;
#pragma unroll
  for (int e = 0; e < 8; ++e) S.x[e] = ld_stream(reinterpret_cast<const vec*>(M + static_cast<long>(i0 + e) * ld_m));
}

template <int RB, int CT>
__device__ __forceinline__ void cpx_compute(const ColStepX6<CT>& S, f32x4 (&acc)[CT][RB], const bf16x8* tq,
                                            int lane) {
  // split the whole step first (the fp32 tile dies here), then one B read per cb
  Split3 A[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c)
    split3(f32x4{S.x[0][c], S.x[1][c], S.x[2][c], S.x[3][c]}, f32x4{S.x[4][c], S.x[5][c], S.x[6][c], S.x[7][c]},
           1.f, A[c]);
#pragma unroll
  for (int cb = 0; cb < RB; ++cb) {
    Split3 B;
    ef_sread(tq, cb, lane, B);
#pragma unroll
    for (int c = 0; c < CT; ++c) acc[c][cb] = mfma6_16(A[c], B, acc[c][cb]);
  }
}

template <int RB>
constexpr int colx6_ct() { return RB >= 4 ? 2 : 4; }

constexpr int kColX6PD = 2;  // register-ring depth of the pass-B column kernel (measured default)

template <int RB, int NW>
__global__ void __launch_bounds__(64 * NW, RB >= 8 ? 1 : (NW >= 8 ? kColx6Minb : 2)) colproj_x6_kernel(const ProjArgs a) {
  constexpr int R = 16 * RB;
  constexpr int CT = colx6_ct<RB>();
  __shared__ bf16x8 tq[2][RB * 3 * 64];
  const BlockXYZ blk = xcd_block_col();
  const int b = blk.z;
  const int kc = blk.y;
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int t = lane & 15;
  const int g = lane >> 4;
  const int col_base = blk.x * (16 * CT * NW) + wave * (16 * CT);
  const int i_begin = kc * a.kchunk;
  const int i_end = min(a.rows, i_begin + a.kchunk);
  const float* __restrict__ M = a.m[b] + static_cast<long>(8 * g) * a.ld_m + col_base + CT * t;

  f32x4 acc[CT][RB];
#pragma unroll
  for (int c = 0; c < CT; ++c)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) acc[c][cb] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int NQ = RB * 3 * 64;
  const u32x4* qs = static_cast<const u32x4*>(a.tsplit) + b * a.ts_stride;
  SplitCopyN<NQ, 64 * NW> TA;
  // M arrives PD - 1 K-steps ahead in a register ring (bytes in flight per wave =
  // (PD - 1) x 32 rows x 16 CT columns x 4 B); the split thin operand one step ahead
  constexpr int PD = kColX6PD;
  ColStepX6<CT> S[PD];
#pragma unroll
  for (int k = 0; k < PD - 1; ++k)
    if (i_begin + 32 * k < i_end) cpx_load<CT>(S[k], M, a.ld_m, i_begin + 32 * k);
  split_copy_load_n(TA, qs + static_cast<long>(i_begin / 32) * NQ, tid);
  split_copy_store_n(TA, tq[0], tid);
  __syncthreads();
  int cur = 0;
  for (int i0 = i_begin; i0 < i_end; i0 += 32 * PD) {
#pragma unroll
    for (int k = 0; k < PD; ++k) {
      const int i = i0 + 32 * k;
      if (i >= i_end) break;
      const bool more = i + 32 < i_end;
      if (i + 32 * (PD - 1) < i_end) cpx_load<CT>(S[(k + PD - 1) % PD], M, a.ld_m, i + 32 * (PD - 1));
      if (more) split_copy_load_n(TA, qs + static_cast<long>(i / 32 + 1) * NQ, tid);
      cpx_compute<RB, CT>(S[k], acc, tq[cur], lane);
      if (!more) break;
      split_copy_store_n(TA, tq[cur ^ 1], tid);
      __syncthreads();
      cur ^= 1;
    }
  }

  float* out = a.out + (static_cast<long>(b) * a.nchunk + kc) * a.out_rows * R;
#pragma unroll
  for (int c = 0; c < CT; ++c)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        out[static_cast<long>(col_base + CT * (4 * g + q) + c) * R + 16 * cb + t] = acc[c][cb][q];
}

// ============================================================================
// fp16x3 ("h3") products.  Each fp32 operand is scaled by a power of two s and split
// exactly into two fp16 limbs, x s = hi + lo + e with |e| <= 2^-22 |x s|; the three
// products hi.hi + hi.lo + lo.hi (v_mfma_f32_16x16x32_f16, exact products, fp32
// accumulation) give the fp32 product to ~2^-22 relative, with HALF the MFMA work of
// the bf16x6 split (fp16 has 11 mantissa bits to bf16's 8).  fp16's narrow exponent is
// handled by the scale: s maps the block's |x| maximum into [2^14, 2^15) (no overflow);
// any element down to 2^-17 of that maximum keeps both limbs normal, and smaller ones
// err by at most 2^-40 of the maximum in absolute terms.  Zero / NaN / inf maxima keep
// s = 1 or shrink it, so NaN and inf propagate as in fp32.
// ============================================================================
// (f16x8, Split2h, h3_scale and split2h are defined with the bf16x6 types above)

// D += A B with both operands h3-split: the two small cross terms first
__device__ __forceinline__ f32x4 mfma3h(const Split2h& A, const Split2h& B, f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(A.lo, B.hi, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(A.hi, B.lo, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(A.hi, B.hi, acc, 0, 0, 0);
  return acc;
}

__device__ __forceinline__ float max8abs(const f32x4& a, const f32x4& b) {
  return fmaxf(fmaxf(fmaxf(fabsf(a[0]), fabsf(a[1])), fmaxf(fabsf(a[2]), fabsf(a[3]))),
               fmaxf(fmaxf(fabsf(b[0]), fabsf(b[1])), fmaxf(fabsf(b[2]), fabsf(b[3]))));
}

// ============================================================================
// Gram G_b = P1_b^T P1_b of the randomised Cholesky QR (ortho.py:110, P.mT @ P in fp32) on
// fp16x3 MFMAs, for r = 16 RB = 64 or 128.  A block owns a chunk of rows (its slab of partial
// sums goes through reduce_slabs_kernel) and steps it 32 rows at a time: the 32 x r panel is
// staged through LDS (row pad 2: the two 16-lane groups of a ds_read_b32 half land on
// opposite bank halves), then every wave reads lane (t, g) = rows 8g .. 8g + 7 of column
// 16 cb + t for every column block cb -- the A operand of block cb is the B operand of
// block cb, so one split serves both -- and takes the panel's max |x| (the same in every
// wave) for a power-of-two scale s.  Wave w accumulates the output rows of column blocks
// RB/4 w .. + RB/4 - 1 against every cb: three fp16 MFMAs per 16 x 16 tile into a zero
// accumulator, added with the step's 1/s twice (1/s^2 may underflow where the products do
// not).  Per product the dropped lo*lo term and the fp16 rounding of lo are 2^-22 of |x s||y s|,
// against fp32's 2^-24 per product.
// ============================================================================
struct GramArgs {
  const float* p;  // batch x mp x r, contiguous (the orthonormalisation's P1 workspace)
  float* out;      // batch x nchunk x r x r partial sums (nchunk 1: the Gram itself)
  int mp, kchunk, nchunk;
};

template <int RB>
__global__ void __launch_bounds__(256, 2) gram_h3_kernel(const GramArgs a) {
  constexpr int R = 16 * RB;
  constexpr int LD = R + 2;
  constexpr int TA = RB / 4;             // output column blocks per wave
  constexpr int NV = 32 * R / 4 / 256;   // 16-byte loads per thread per 32-row step
  __shared__ __attribute__((aligned(16))) float tile[2][32 * LD];
  const int b = blockIdx.y, kc = blockIdx.x;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, t = lane & 15, g = lane >> 4;
  const float* __restrict__ P = a.p + static_cast<long>(b) * a.mp * R;
  const int i_begin = kc * a.kchunk;
  const int i_end = min(a.mp, i_begin + a.kchunk);
  f32x4 acc[TA][RB];
#pragma unroll
  for (int ta = 0; ta < TA; ++ta)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) acc[ta][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 pre[NV];
  auto load = [&](int i0) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int idx = tid + 256 * v, row = idx / (R / 4), c4 = idx % (R / 4);
      pre[v] = *reinterpret_cast<const f32x4*>(P + static_cast<long>(i0 + row) * R + 4 * c4);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int idx = tid + 256 * v, row = idx / (R / 4), c4 = idx % (R / 4);
      f32x2* d = reinterpret_cast<f32x2*>(&tile[buf][row * LD + 4 * c4]);  // 8-byte aligned (LD even)
      d[0] = f32x2{pre[v][0], pre[v][1]};
      d[1] = f32x2{pre[v][2], pre[v][3]};
    }
  };
  if (i_begin >= i_end) return;
  load(i_begin);
  store(0);
  __syncthreads();
  int cur = 0;
  for (int i0 = i_begin; i0 < i_end; i0 += 32) {
    const bool more = i0 + 32 < i_end;
    if (more) load(i0 + 32);
    f32x4 v[RB][2];
    float m = 0.f;
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[cb][e >> 2][e & 3] = tile[cur][(8 * g + e) * LD + 16 * cb + t];
      m = fmaxf(m, max8abs(v[cb][0], v[cb][1]));
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    float inv;
    const float s = h3_scale(m, inv);
    Split2h S[RB];
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) split2h(v[cb][0], v[cb][1], s, S[cb]);
    // this wave's A operands (a register array indexed by the wave number would go to scratch)
    Split2h A[TA];
#pragma unroll
    for (int ta = 0; ta < TA; ++ta)
#pragma unroll
      for (int cb = ta; cb < RB; cb += TA)
        if (cb == wave * TA + ta) A[ta] = S[cb];
#pragma unroll
    for (int ta = 0; ta < TA; ++ta) {
#pragma unroll
      for (int cb = 0; cb < RB; ++cb) {
        const f32x4 d = mfma3h(A[ta], S[cb], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[ta][cb][q] = fmaf(d[q] * inv, inv, acc[ta][cb][q]);
      }
    }
    if (!more) break;
    store(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
  // lane (t, g), element q: G[16 (TA w + ta) + 4 g + q][16 cb + t]
  float* out = a.out + (static_cast<long>(b) * a.nchunk + kc) * R * R;
#pragma unroll
  for (int ta = 0; ta < TA; ++ta)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb)
#pragma unroll
      for (int q = 0; q < 4; ++q) out[(16 * (TA * wave + ta) + 4 * g + q) * R + 16 * cb + t] = acc[ta][cb][q];
}

// ============================================================================
// The two triangular solves as GEMMs with the explicit inverse, X_b = P_b T_b, T_b = R_b^-1 (the
// r x r upper-triangular inverses that sketch_qr_inv_kernel / chol_inv_kernel write with INV),
// on fp16x3 MFMAs.  The solve kernels above run one row per lane and read every factor value
// once per row (2 080 reads per row at r = 64, from LDS or the scalar cache): LDS- or
// scalar-cache-bound at 2-8x the time of the row traffic, and they hold the CUs the streaming
// kernels of the other stream need.  Here a wave takes 16 rows per MFMA tile: Xt = Tt Pt on
// v_mfma_f32_16x16x32_f16 (A = T^T: lane (t, g) holds T[32 j + 8 g + e][16 i + t]; B = P^T: lane
// (t, g) holds P[row t][32 j + 8 g + e]; D lane (t, g): X[row t][16 i + 4 g + q]), three products
// (hi hi, hi lo, lo hi), T split with one power-of-two scale per column and P with one per row,
// zero blocks of T skipped.  The rounding differs from substitution's (the product, not the
// k-ordered fma chain); numpy over 0-8 decades of conditioning puts the final P's error at
// 0.6-1.6x the fp32 substitution's.
//   RT <= 64 (IMG): each wave's 64 rows are staged by LDS-DMA as in trsm_lds_kernel, X goes back
//   into the image, and the epilogue (coalesced store, FINAL fix-up, pass-B split) is that
//   kernel's.  RT = 128: operands straight from HBM (32 B per lane and k-step), X stored as
//   16-byte row pieces, FINAL fix-up only (no pass-B split at r = 128).
// ============================================================================
// T_b = F_b^-1 for the padded upper-triangular factor F_b of the factor kernels (RT x RT, then
// its RT reciprocal diagonal entries: the INV = false output of sketch_qr_inv_kernel and
// chol_reg_kernel), the operand of tsolve_mfma_kernel.  One block per matrix; column c is
// back-substituted by TIP adjacent lanes, x_i = (d_ic - sum_{i < k <= c} F_ik x_k) (1/F_ii) for
// i = c .. 0 (x_i = 0 for i > c), fp32: lane p of the column sums the k = i + 1 + p (mod TIP)
// terms and the partial sums meet by xor shuffles (every lane gets the same x_i); the factor
// row is a broadcast LDS read, the column lives in LDS (column-major, padded).  A NaN diagonal (a failed
// factorisation) makes its column and every later one NaN, as the substitution would.  Numpy
// over 0-6 decades: the final P within 0.8-1.0x the error of an fp64 inverse (DESIGN.md
// section 4).  Per 16-matrix launch at r = 64 / 128: one lane per column 55 / 185 us (one-stream
// profile, profiles/r05/n_gemm_default.txt), eight interleaved sums per lane 116 / 470, 8-16 lanes
// per column 23.2 / 71.5 (scripts/ubench/qr_ab.hip, profiles/r05/p_tri_inv_lanes.txt).  In the
// orthonormalisation it runs fused into the QR and Cholesky kernels (TINV); the kernel stays for
// the microbenchmark.
template <int RT>
constexpr int tri_inv_tip() { return RT >= 128 ? 8 : 16; }
template <int RT>
__global__ void __launch_bounds__(RT * tri_inv_tip<RT>()) tri_inv_kernel(const float* __restrict__ F,
                                                                           float* __restrict__ T) {
  constexpr int TIP = tri_inv_tip<RT>();
  constexpr int NT = RT * TIP;
  constexpr int LDX = RT + TIP;   // Xs[c LDX + k] = x_k of column c: the TIP lanes of a column
  __shared__ __attribute__((aligned(16))) float Fs[RT * RT + RT];
  __shared__ float Xs[RT * LDX];  // read consecutive k, and columns sit TIP banks apart
  const int b = blockIdx.x, tid = threadIdx.x;
  {
    const f32x4* src = reinterpret_cast<const f32x4*>(F + static_cast<long>(b) * (RT * RT + RT));
    for (int i = tid; i < (RT * RT + RT) / 4; i += NT) reinterpret_cast<f32x4*>(Fs)[i] = src[i];
    __syncthreads();
  }
  tri_inv_cols<TIP>(Fs, RT, Fs + RT * RT, Xs, LDX, RT, T + static_cast<long>(b) * RT * RT, tid, NT);
}

constexpr int kTgWavesImg = 2, kTgWavesDirect = 4;

// DION_TSOLVE_DIRECT_FIRST (a dev build option, off): the first solve at r <= 64 without the
// LDS row image, straight from HBM with 17 KB of LDS per block instead of 50 KB.  Alone and
// beside a streaming copy it is faster (fc1 group 26.5 vs 38.9 us; marginal 1.9 vs 8.4 us,
// scripts/ubench/trsm_conc.hip), in the step it is within noise (Llama 470.8 / 470.7 against
// 471.4 / 472.6 GiB/s, Mixtral 372.9 against 371.7, same box, profiles/r05/t_direct_first.txt)
#ifndef DION_TSOLVE_DIRECT_FIRST
#define DION_TSOLVE_DIRECT_FIRST 0
#endif
template <int RT, bool FINAL, bool GRAM>
constexpr bool tsolve_img() { return RT <= 64 && (FINAL || GRAM || !DION_TSOLVE_DIRECT_FIRST); }

template <int RT, bool FINAL, bool GRAM = false>
__global__ void __launch_bounds__(64 * (tsolve_img<RT, FINAL, GRAM>() ? kTgWavesImg : kTgWavesDirect),
                                  (tsolve_img<RT, FINAL, GRAM>() ? 3 : 2))
tsolve_mfma_kernel(const TrsmArgs a) {
  static_assert(RT == 32 || RT == 64 || RT == 128, "tsolve_mfma_kernel: r = 32, 64 or 128");
  static_assert(!GRAM || (RT <= 64 && !FINAL), "tsolve_mfma_kernel: the fused Gram is for the first solve at r <= 64");
  constexpr bool IMG = tsolve_img<RT, FINAL, GRAM>();
  constexpr int NW = IMG ? kTgWavesImg : kTgWavesDirect;
  constexpr int CH = RT / 4;   // 16-B chunks per row
  constexpr int KS = RT / 32;  // 32-wide k-steps
  constexpr int NT = RT / 16;  // 16-wide output column tiles
  constexpr int LDT = RT + 4;  // T^T row pitch: lanes t of a ds_read_b128 group land 4 banks apart
  __shared__ f32x4 img[IMG ? NW : 1][IMG ? 64 * CH : 1];
  __shared__ __attribute__((aligned(16))) float Tt[RT * LDT];
  __shared__ float scol[RT], icol[RT];
  const int b = blockIdx.y;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(tid >> 6)), lane = tid & 63;
  const int t = lane & 15, g = lane >> 4;
  const int mp = a.mp;
  // T^T into LDS (T row-major: coalesced reads, transposed writes), then per column of T its
  // max |x| and power-of-two scale (a NaN column -- a failed factorisation -- stays NaN)
  {
    const float* Tg = a.fac + static_cast<long>(b) * RT * RT;
    for (int idx = tid; idx < RT * RT; idx += 64 * NW) {
      const int k = idx / RT, n = idx % RT;
      Tt[n * LDT + k] = Tg[idx];
    }
    __syncthreads();
    for (int n = tid; n < RT; n += 64 * NW) {
      float m = 0.f;
      for (int k = 0; k <= n; ++k) m = fmaxf(m, fabsf(Tt[n * LDT + k]));
      float inv;
      scol[n] = h3_scale(m, inv);
      icol[n] = inv;
    }
    __syncthreads();
  }
  constexpr int RB = RT / 16;
  f32x4 gacc[GRAM ? RB : 1][GRAM ? RB : 1];
  if constexpr (GRAM) {
#pragma unroll
    for (int ta = 0; ta < RB; ++ta)
#pragma unroll
      for (int cb = 0; cb < RB; ++cb) gacc[ta][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // one 64-row chunk of this wave: stage, solve, store (and, GRAM, add X^T X of the chunk)
  auto chunk = [&](const long row0) {
  const int nrows = static_cast<int>(min(static_cast<long>(64), static_cast<long>(mp) - row0));
  if (nrows <= 0) return;
  const float* src = a.src + (static_cast<long>(b) * mp + row0) * RT;
  float* dst = a.dst + (static_cast<long>(b) * mp + row0) * RT;
  f32x4* w = img[IMG ? wave : 0];
  if constexpr (IMG) {
    const char* s = reinterpret_cast<const char*>(src);
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int slot = 64 * i + lane, row = slot / CH, cp = slot % CH;
      if (row < nrows) glds16<false>(s, static_cast<uint32_t>((row * CH + (cp ^ trsm_swz<RT>(row))) * 16), lds_off(&w[64 * i]));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  const bool zero = FINAL && a.nonzero != nullptr && a.nonzero[b] == 0u;
  float xmax = 0.f;  // GRAM: max |X| over the chunk's rows, the Gram's split scale
  auto tile_body = [&](const int tile) {
    const int row = 16 * tile + t;
    const bool valid = row < nrows;
    // this lane's B operand: P[row][32 j + 8 g .. + 7] for every k-step j
    f32x4 v[KS][2];
#pragma unroll
    for (int j = 0; j < KS; ++j) {
      const int c0 = 8 * j + 2 * g;
      if constexpr (IMG) {
        v[j][0] = valid ? w[row * CH + (c0 ^ trsm_swz<RT>(row))] : f32x4{0.f, 0.f, 0.f, 0.f};
        v[j][1] = valid ? w[row * CH + ((c0 + 1) ^ trsm_swz<RT>(row))] : f32x4{0.f, 0.f, 0.f, 0.f};
      } else {
        const f32x4* p = reinterpret_cast<const f32x4*>(src + static_cast<long>(row) * RT);
        v[j][0] = valid ? p[c0] : f32x4{0.f, 0.f, 0.f, 0.f};
        v[j][1] = valid ? p[c0 + 1] : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    // the row's max |x| (lanes t, t + 16, t + 32, t + 48 hold row t) and its scale
    float m = 0.f;
#pragma unroll
    for (int j = 0; j < KS; ++j) m = fmaxf(m, max8abs(v[j][0], v[j][1]));
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float irow;
    const float srow = h3_scale(m, irow);
    Split2h B[KS];
#pragma unroll
    for (int j = 0; j < KS; ++j) split2h(v[j][0], v[j][1], srow, B[j]);
    f32x4 x[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      f32x4 acc{0.f, 0.f, 0.f, 0.f};
      const int n = 16 * i + t;
      const float sc = scol[n];
#pragma unroll
      for (int j = 0; j < KS; ++j) {
        if (32 * j > 16 * i + 15) break;  // T[k][n] = 0 for k > n
        const f32x4* tp = reinterpret_cast<const f32x4*>(&Tt[n * LDT + 32 * j + 8 * g]);
        Split2h A;
        split2h(tp[0], tp[1], sc, A);
        acc = mfma3h(A, B[j], acc);
      }
      const f32x4 ic = *reinterpret_cast<const f32x4*>(&icol[16 * i + 4 * g]);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float y = (acc[q] * irow) * ic[q];
        if constexpr (FINAL) y = zero ? 0.f : (a.nonzero != nullptr ? nan_to_num(y) : y);
        x[i][q] = y;
        if constexpr (GRAM) xmax = valid ? fmaxf(xmax, fabsf(y)) : xmax;
      }
    }
    if (valid) {
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        if constexpr (IMG)
          w[row * CH + ((4 * i + g) ^ trsm_swz<RT>(row))] = x[i];
        else
          reinterpret_cast<f32x4*>(dst + static_cast<long>(row) * RT)[4 * i + g] = x[i];
      }
    }
  };
  if constexpr (GRAM) {
    // one tile at a time: the unrolled tile loop beside the Gram accumulators needs > 256 VGPRs
#pragma unroll 1
    for (int tile = 0; tile < 4; ++tile) {
      if (16 * tile >= nrows) break;
      tile_body(tile);
    }
  } else {
    for (int tile = 0; tile < 4; ++tile) {
      if (16 * tile >= nrows) break;
      tile_body(tile);
    }
  }
  if constexpr (IMG) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    f32x4* d = reinterpret_cast<f32x4*>(dst);
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int slot = 64 * i + lane, row = slot / CH, cp = slot % CH;
      if (row < nrows) d[row * CH + (cp ^ trsm_swz<RT>(row))] = w[slot];
    }
    if constexpr (FINAL) {
      if (a.psplit != nullptr) {
        constexpr int RB = RT / 16;
        const float* wf = reinterpret_cast<const float*>(w);
        f16x8* out = a.psplit + b * a.pstride;
#pragma unroll
        for (int u = 0; u < 2 * RB; ++u) {
          const int q = u / RB, cb = u % RB;
          if (32 * q >= nrows) break;
          float vv[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int rr = 32 * q + (a.kmap == 0 ? 8 * g + e : 16 * (e >> 2) + 4 * g + (e & 3));
            const int col = 16 * cb + t;
            vv[e] = wf[(rr * CH + ((col >> 2) ^ trsm_swz<RT>(rr))) * 4 + (col & 3)];
          }
          Split2h sp;
          split2h(f32x4{vv[0], vv[1], vv[2], vv[3]}, f32x4{vv[4], vv[5], vv[6], vv[7]}, kPSplitScale, sp);
          const long grp = (row0 / 32 + q) * RB + cb;
          out[grp * 128 + lane] = sp.hi;
          out[grp * 128 + 64 + lane] = sp.lo;
        }
      }
    }
    if constexpr (GRAM) {
      // X^T X of the chunk from the image, as gram_h3_kernel but with one scale for the chunk
      // (its max |X|, from the solve): lane (t, g) splits rows 8 g .. + 7 of column 16 cb + t
      // of each 32-row k-step (the A operand of block cb is the B operand of block cb); rows
      // past nrows count as zero
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) xmax = fmaxf(xmax, __shfl_xor(xmax, o, 64));
      float inv;
      const float sc = h3_scale(xmax, inv);
      const float* wf = reinterpret_cast<const float*>(w);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if (32 * ks >= nrows) break;
        Split2h S[RB];
#pragma unroll
        for (int cb = 0; cb < RB; ++cb) {
          f32x4 v[2];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int rr = 32 * ks + 8 * g + e, col = 16 * cb + t;
            v[e >> 2][e & 3] = rr < nrows ? wf[(rr * CH + ((col >> 2) ^ trsm_swz<RT>(rr))) * 4 + (col & 3)] : 0.f;
          }
          split2h(v[0], v[1], sc, S[cb]);
        }
        // the block upper triangle only (cb >= ta): chol_reg_kernel reads G on and above the
        // diagonal; the lower tiles are written as zeros
#pragma unroll
        for (int ta = 0; ta < RB; ++ta)
#pragma unroll
          for (int cb = ta; cb < RB; ++cb) {
            const f32x4 d = mfma3h(S[ta], S[cb], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
            for (int q = 0; q < 4; ++q) gacc[ta][cb][q] = fmaf(d[q] * inv, inv, gacc[ta][cb][q]);
          }
      }
    }
  }
  };
  if constexpr (!GRAM) {
    chunk(static_cast<long>(blockIdx.x) * (64 * NW) + wave * 64);
  } else {
    // persistent over the rows: block x of gridDim.x takes the 64 NW-row steps x, x + gridDim.x, ..
    for (long base = static_cast<long>(blockIdx.x) * (64 * NW); base < mp; base += static_cast<long>(gridDim.x) * (64 * NW))
      chunk(base + wave * 64);
    // the waves' partial Grams summed through LDS (the image of wave 1), then one slab per block:
    // lane (t, g), element q of tile (ta, cb) = G[16 ta + 4 g + q][16 cb + t]
    __syncthreads();
    float* red = reinterpret_cast<float*>(img[IMG ? NW - 1 : 0]);
    for (int wv = NW - 1; wv >= 1; --wv) {
      if (wave == wv) {
#pragma unroll
        for (int ta = 0; ta < RB; ++ta)
#pragma unroll
          for (int cb = ta; cb < RB; ++cb)
#pragma unroll
            for (int q = 0; q < 4; ++q) red[((ta * RB + cb) * 4 + q) * 64 + lane] = gacc[ta][cb][q];
      }
      __syncthreads();
      if (wave == 0) {
#pragma unroll
        for (int ta = 0; ta < RB; ++ta)
#pragma unroll
          for (int cb = ta; cb < RB; ++cb)
#pragma unroll
            for (int q = 0; q < 4; ++q) gacc[ta][cb][q] += red[((ta * RB + cb) * 4 + q) * 64 + lane];
      }
      __syncthreads();
    }
    if (wave == 0) {
      float* go = a.gram + (static_cast<long>(b) * gridDim.x + blockIdx.x) * RT * RT;
#pragma unroll
      for (int ta = 0; ta < RB; ++ta)
#pragma unroll
        for (int cb = 0; cb < RB; ++cb)
#pragma unroll
          for (int q = 0; q < 4; ++q) go[(16 * ta + 4 * g + q) * RT + 16 * cb + t] = cb >= ta ? gacc[ta][cb][q] : 0.f;
    }
  }
}

// per-matrix max |x| of a small factor (rows x r fp32) over its FINITE values, as the float's
// bit pattern (non-negative floats order like their bits).  A non-finite value counts as 0: it
// turns its own products non-finite whatever the scale, and left in the max (a NaN's bits sort
// above inf's) it would push the scale to 2^-114 and flush every finite product of the matrix
// to zero -- a P with one NaN column (a failed Cholesky pivot) then lost all of its R instead of
// that column (round 6, tests/test_gpu_fused_tail.py).
__device__ __forceinline__ uint32_t finite_abs_bits(float x) {
  const uint32_t b = __float_as_uint(x) & 0x7FFFFFFFu;
  return b < 0x7F800000u ? b : 0u;
}

struct AbsMaxArgs {
  const float* src[3 * MAXB];  // group-major: matrix b of group k at k * nb + b (null: skipped)
  uint32_t* out;               // (groups * nb,) zero-initialised, same order
  long count[3];               // values per matrix of each group
  int nb;                      // matrices per group
  int vec;                     // every src 16-byte aligned and every count % 4 == 0
};

// all groups in one launch: blockIdx.y = k * nb + b, blocks stride over the matrix in
// 16-byte loads (4 in flight per thread)
__global__ void __launch_bounds__(256) absmax_kernel(const AbsMaxArgs a) {
  const int y = blockIdx.y;
  const long count = a.count[y / a.nb];
  const float* __restrict__ src = a.src[y];
  uint32_t m = 0;
  if (src != nullptr) {
    const long stride = static_cast<long>(gridDim.x) * 256;
    long i = static_cast<long>(blockIdx.x) * 256 + threadIdx.x;
    if (a.vec) {
      const f32x4* s4 = reinterpret_cast<const f32x4*>(src);
      const long n4 = count / 4;
      for (; i + 3 * stride < n4; i += 4 * stride) {
        f32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = s4[i + u * stride];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int q = 0; q < 4; ++q) m = max(m, finite_abs_bits(v[u][q]));
      }
      for (; i < n4; i += stride) {
        const f32x4 v = s4[i];
#pragma unroll
        for (int q = 0; q < 4; ++q) m = max(m, finite_abs_bits(v[q]));
      }
    } else {
      for (; i < count; i += stride) m = max(m, finite_abs_bits(src[i]));
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = max(m, static_cast<uint32_t>(__shfl_xor(static_cast<int>(m), off, 64)));
  // one atomic per block: many blocks hammering one address serialise at the L2
  __shared__ uint32_t wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(&a.out[y], max(max(wm[0], wm[1]), max(wm[2], wm[3])));
}

// h3 pre-split of a small factor in the MFMA operand layouts of presplit_kernel, two fp16
// limbs per 8 values: dst[(grp * 2 + part) * 64 + lane], scale from amax[b]
//   layout 0 (B-operand-style):  grp = (row / 32) RB + cb; lane (t, g) <- rows 32 blk + kmap(g, e), column 16 cb + t
//   layout 1 (A-operand-style):  grp = (row / 16) KK + kk; lane (t, g) <- row 16 blk + t, columns 32 kk + 8 g + e
struct Presplit16Args {
  const float* src[MAXB];
  f16x8* dst;
  const uint32_t* amax;  // (batch,) max |x| bits; null: the fixed scale 2^14 of an orthonormal P
  float* inv_scale;      // (batch,) 1 / s, written by the blocks of x = 0 (with amax only)
  long stride;           // f16x8 units per matrix
  int rows, r, kmap, layout;
  const uint32_t* fix;   // layout 0 only (dion_pfix_split): P_b <- fix[b] == 0 ? 0 : nan_to_num(P_b)
                         // in place before the split (null: src is only read)
};

__global__ void __launch_bounds__(256) presplit16_kernel(const Presplit16Args a) {
  const int b = blockIdx.y;
  const float* __restrict__ src = a.src[b];
  if (src == nullptr) return;
  float s = kPSplitScale;
  if (a.amax != nullptr) {
    float inv;
    s = h3_scale(__uint_as_float(a.amax[b]), inv);
    if (blockIdx.x == 0 && threadIdx.x == 0) a.inv_scale[b] = inv;
  }
  const long items = static_cast<long>(a.rows) * a.r / 8;
  const long item = static_cast<long>(blockIdx.x) * 256 + threadIdx.x;
  if (item >= items) return;
  const int ln = static_cast<int>(item & 63);
  const long grp = item >> 6;
  const int t = ln & 15, g = ln >> 4;
  float v[8];
  if (a.layout == 0) {
    const int RB = a.r / 16;
    const long blk = grp / RB;
    const int cb = static_cast<int>(grp - blk * RB);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = a.kmap == 0 ? 8 * g + e : 16 * (e >> 2) + 4 * g + (e & 3);
      v[e] = src[(blk * 32 + k) * a.r + 16 * cb + t];
    }
    if (a.fix != nullptr) {
      // the fix-up's P half (kernels.py:185-188) with this rank's zero test: every element of
      // P is one (unit, lane, e) of the layout, so each is rewritten exactly once
      // (only a value the fix-up changes is written back: an orthonormalised P is normally all
      // finite and its momentum nonzero, so P is read once and nothing but the split is written)
      const bool zero = a.fix[b] == 0u;
      float* __restrict__ dst = const_cast<float*>(src);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = a.kmap == 0 ? 8 * g + e : 16 * (e >> 2) + 4 * g + (e & 3);
        const float f = zero ? 0.f : nan_to_num(v[e]);
        if (__float_as_uint(f) != __float_as_uint(v[e])) dst[(blk * 32 + k) * a.r + 16 * cb + t] = f;
        v[e] = f;
      }
    }
  } else {
    const int KK = a.r / 32;
    const long blk = grp / KK;
    const int kk = static_cast<int>(grp - blk * KK);
    const float* p = src + (blk * 16 + t) * a.r + 32 * kk + 8 * g;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = p[e];
  }
  Split2h sp;
  split2h(f32x4{v[0], v[1], v[2], v[3]}, f32x4{v[4], v[5], v[6], v[7]}, s, sp);
  f16x8* d = a.dst + b * a.stride + (grp * 2) * 64 + ln;
  d[0] = sp.hi;
  d[64] = sp.lo;
}

// ---- pass B, not transposed (R = M^T P), h3 products.  Geometry and loads of
// colproj_x6_kernel; the roles are swapped so the streamed M is the B operand: lane
// (t, g) holds column CT t + c of rows 8 g + e, i.e. B[k = 8 g + e][col t], and the
// per-step scale of that column is the max over the four lanes (t, g = 0..3).  The
// pre-split P is the A operand (A[row j = 16 cb + t'][k]), one scale per matrix.  Each
// step's product lands in a fresh accumulator D[j][col] (lane (t, g): R rows CT t + c,
// r columns 16 cb + 4 g + q) and is added as acc += D / s_col.
// the r = 128 fused pass A row kernel without LDS-DMA (fp32 G, odd 128-row block counts; bf16
// G takes rowproj_efgl_kernel): 32-row waves in 4-wave blocks, one-step pipeline (242-256
// VGPRs, two waves per SIMD, no tile in flight).  Measured slower: 16-row waves in 4-wave
// blocks with a prefetch stage (5.33 vs 4.60 ms, round 2: twice the staging traffic), and
// 16-row waves in 8-wave blocks (184 VGPRs, two waves per SIMD, the same 128 rows per staged
// step: 5.84 vs 4.79 ms, round 3) -- each wave reads the whole staged Q and R' splits (32 KB
// per 32-column step at r = 128) for its rows, so halving the rows per wave doubles the LDS
// operand reads per HBM byte (6.4x), and LDS bandwidth, not occupancy, bounds the kernel.
constexpr int kKR8 = 2;
constexpr int kNW8 = 4;
constexpr int kPD8 = 1;
// r = 128 fused pass A row kernel: 1 = rowproj_efgl_kernel (M/G and the splits by LDS-DMA;
// bf16 or no G, an even number of 128-row blocks), 0 = rowproj_efh3_kernel everywhere
constexpr int kPaGl8 = 1;
// cache policy of its bf16 G loads (64-B row pieces, the other half of the line one step later)
#ifndef DION_PAGL_GNT
#define DION_PAGL_GNT 0
#endif
constexpr int kPaGlGnt = DION_PAGL_GNT;
// the 8-wave LDS-DMA kernels (pass A at r = 128, pass B): priority 1 for waves 4-7 (the guide's
// static form for two waves per SIMD); a dev build option
#ifndef DION_GL_PRIO
#define DION_GL_PRIO 0
#endif
constexpr int kGlPrio = DION_GL_PRIO;
// its bf16 G in step pairs: one step's G row is 64 B, half a 128-B line, and issued a step
// apart the two halves were fetched twice for ~1 in 6 lines (PMC: pass A 1.12x its algorithmic
// bytes, G nt 1.21x); 1 = both halves of every line in one issue at every odd step, one step
// ahead instead of two (split-K chunks on 64-column bounds).  Measured (profiles/r06/l_*): the
// launch 21.07 -> 20.04 GB (1.066x; reads 1.179x -> 1.049x), 4.78 -> 4.66 ms, Mixtral +0.6 %
#ifndef DION_PAGL_GPAIR
#define DION_PAGL_GPAIR 1
#endif
constexpr int kPaGlGpair = DION_PAGL_GPAIR;
// the smallest rank block (r = 16 RB) that takes it, row / transposed kernel (r = 64 measured
// slower in round 4; dev build options)
#ifndef DION_PA_GL_MINRB
#define DION_PA_GL_MINRB 8
#endif
#ifndef DION_PA_GLT_MINRB
#define DION_PA_GLT_MINRB 8
#endif
constexpr int kPaGlMinRB = DION_PA_GL_MINRB, kPaGlMinRBT = DION_PA_GLT_MINRB;
// blocks per CU the r = 128 transposed fused pass A is compiled for
// transposed pass-A kernel (colproj_efh3_kernel) at r <= 64: 1 = the two-step SA/SB register
// ring (234 VGPRs, 2 waves per SIMD; it spills at 3), 0 = no ring, the step's M/G loads
// issued right before use and the CU's other blocks covering their latency (162 VGPRs, 3
// blocks per CU).  Measured (Llama set, 3-round A/B): ring 5459 vs 5313 GB/s.  r = 128 always
// runs ring-free: 252 VGPRs at 2 waves per SIMD against the ring's 256 + 103 AGPRs at 1,
// 3098 -> 3888 GB/s (Mixtral set)
constexpr int kCpeRing = 1;
// transposed pass-B row kernel (rowproj_h3_kernel): ring-free (r <= 64: 114 VGPRs, 4 waves per
// SIMD; r = 128: 153, 3) -- the ring needs 188 (2 per SIMD) and 256 with 10 spilled.
// Measured: Llama 4593 -> 4831 GB/s, Mixtral 3730 -> 3954 GB/s
constexpr int kPbrRing = 0;
// blocks per CU the r <= 64 pass-B row kernel is compiled for
constexpr int kPbrMinb = 2;
// r > 64 pass-B h3 kernels: the split P two cb at a time, two waves per SIMD
constexpr int kH3Pairs = 1;
template <int RB, int NW, int CT>
__global__ void __launch_bounds__(64 * NW, (RB >= 8 && !kH3Pairs) ? 1 : 2) colproj_h3_kernel(const ProjArgs a) {
  constexpr int R = 16 * RB;
  constexpr int NQ = RB * 2 * 64;  // f16x8 units of one K-step's P split
  __shared__ f16x8 tq[2][NQ];
  const BlockXYZ blk = xcd_block_col();
  const int b = blk.z;
  const int kc = blk.y;
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int t = lane & 15;
  const int g = lane >> 4;
  const int col_base = blk.x * (16 * CT * NW) + wave * (16 * CT);
  const int i_begin = kc * a.kchunk;
  const int i_end = min(a.rows, i_begin + a.kchunk);
  const float* __restrict__ M = a.m[b] + static_cast<long>(8 * g) * a.ld_m + col_base + CT * t;

  f32x4 acc[CT][RB];
#pragma unroll
  for (int c = 0; c < CT; ++c)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) acc[c][cb] = f32x4{0.f, 0.f, 0.f, 0.f};

  const u32x4* qs = static_cast<const u32x4*>(a.tsplit) + b * a.ts_stride;
  // pass A's max |M_b| (when measured and finite): one power-of-two scale for the whole
  // matrix, the products accumulate in place; else a scale per column and 32-row step
  const uint32_t mab = a.mabs != nullptr ? a.mabs[b] : kAbsUnknown;
  float finv = 1.f;
  const float fs = h3_scale(__uint_as_float(mab), finv);
  auto run = [&](auto FIXc) {
    constexpr bool FIX = decltype(FIXc)::value;
    SplitCopyN<NQ, 64 * NW> TA;
    constexpr int PD = kColX6PD;
    ColStepX6<CT> S[PD];
#pragma unroll
    for (int k = 0; k < PD - 1; ++k)
      if (i_begin + 32 * k < i_end) cpx_load<CT>(S[k], M, a.ld_m, i_begin + 32 * k);
    split_copy_load_n(TA, qs + static_cast<long>(i_begin / 32) * NQ, tid);
    split_copy_store_n(TA, reinterpret_cast<bf16x8*>(tq[0]), tid);
    __syncthreads();
    int cur = 0;
    for (int i0 = i_begin; i0 < i_end; i0 += 32 * PD) {
#pragma unroll
      for (int k = 0; k < PD; ++k) {
        const int i = i0 + 32 * k;
        if (i >= i_end) break;
        const bool more = i + 32 < i_end;
        if (kSplitFirstB && more) split_copy_load_n(TA, qs + static_cast<long>(i / 32 + 1) * NQ, tid);
        if (i + 32 * (PD - 1) < i_end) cpx_load<CT>(S[(k + PD - 1) % PD], M, a.ld_m, i + 32 * (PD - 1));
        if (!kSplitFirstB && more) split_copy_load_n(TA, qs + static_cast<long>(i / 32 + 1) * NQ, tid);
        {
          const ColStepX6<CT>& X = S[k];
          Split2h B[CT];
          float inv[CT];
#pragma unroll
          for (int c = 0; c < CT; ++c) {
            const f32x4 lo4{X.x[0][c], X.x[1][c], X.x[2][c], X.x[3][c]};
            const f32x4 hi4{X.x[4][c], X.x[5][c], X.x[6][c], X.x[7][c]};
            if constexpr (FIX) {
              split2h(lo4, hi4, fs, B[c]);
            } else {
              float m8 = max8abs(lo4, hi4);
              m8 = fmaxf(m8, __shfl_xor(m8, 16, 64));
              m8 = fmaxf(m8, __shfl_xor(m8, 32, 64));
              const float sc = h3_scale(m8, inv[c]);
              split2h(lo4, hi4, sc, B[c]);
            }
          }
          if constexpr (FIX && RB >= 8 && kH3Pairs) {
            // r > 64: the split P of two cb at a time (all RB of them would need 64 VGPRs
            // and push the kernel to one wave per SIMD); term by term over (c, cb pair)
#pragma unroll
            for (int cp = 0; cp < RB; cp += 2) {
              Split2h A0, A1;
              A0.hi = tq[cur][(cp * 2 + 0) * 64 + lane];
              A0.lo = tq[cur][(cp * 2 + 1) * 64 + lane];
              A1.hi = tq[cur][(cp * 2 + 2) * 64 + lane];
              A1.lo = tq[cur][(cp * 2 + 3) * 64 + lane];
#pragma unroll
              for (int c = 0; c < CT; ++c) {
                acc[c][cp] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0.lo, B[c].hi, acc[c][cp], 0, 0, 0);
                acc[c][cp + 1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1.lo, B[c].hi, acc[c][cp + 1], 0, 0, 0);
              }
#pragma unroll
              for (int c = 0; c < CT; ++c) {
                acc[c][cp] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0.hi, B[c].lo, acc[c][cp], 0, 0, 0);
                acc[c][cp + 1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1.hi, B[c].lo, acc[c][cp + 1], 0, 0, 0);
              }
#pragma unroll
              for (int c = 0; c < CT; ++c) {
                acc[c][cp] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0.hi, B[c].hi, acc[c][cp], 0, 0, 0);
                acc[c][cp + 1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1.hi, B[c].hi, acc[c][cp + 1], 0, 0, 0);
              }
            }
          } else if constexpr (FIX) {
            // the three products term by term over all (c, cb): consecutive MFMAs are
            // independent (a back-to-back dependent MFMA waits for its predecessor)
            Split2h A[RB];
#pragma unroll
            for (int cb = 0; cb < RB; ++cb) {
              A[cb].hi = tq[cur][(cb * 2 + 0) * 64 + lane];
              A[cb].lo = tq[cur][(cb * 2 + 1) * 64 + lane];
            }
#pragma unroll
            for (int c = 0; c < CT; ++c)
#pragma unroll
              for (int cb = 0; cb < RB; ++cb)
                acc[c][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[cb].lo, B[c].hi, acc[c][cb], 0, 0, 0);
#pragma unroll
            for (int c = 0; c < CT; ++c)
#pragma unroll
              for (int cb = 0; cb < RB; ++cb)
                acc[c][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[cb].hi, B[c].lo, acc[c][cb], 0, 0, 0);
#pragma unroll
            for (int c = 0; c < CT; ++c)
#pragma unroll
              for (int cb = 0; cb < RB; ++cb)
                acc[c][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[cb].hi, B[c].hi, acc[c][cb], 0, 0, 0);
          } else {
#pragma unroll
            for (int cb = 0; cb < RB; ++cb) {
              Split2h A;
              A.hi = tq[cur][(cb * 2 + 0) * 64 + lane];
              A.lo = tq[cur][(cb * 2 + 1) * 64 + lane];
#pragma unroll
              for (int c = 0; c < CT; ++c) {
                const f32x4 d = mfma3h(A, B[c], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[c][cb][q] = fmaf(d[q], inv[c], acc[c][cb][q]);
              }
            }
          }
        }
        if (!more) break;
        split_copy_store_n(TA, reinterpret_cast<bf16x8*>(tq[cur ^ 1]), tid);
        __syncthreads();
        cur ^= 1;
      }
    }
  };
  const bool fixed = mab < kAbsUnknown;
  if (fixed)
    run(std::true_type{});
  else
    run(std::false_type{});

  // P's per-matrix scale (a.tinv: presplit16's; null: the fixed scale of an orthonormal P split
  // by the final solve, trsm_lds_kernel<..., true>) and M's (fixed mode), then lane (t, g): R row
  // CT t + c, columns 16 cb + 4 g .. + 3
  const float ps = (a.tinv != nullptr ? a.tinv[b] : kPSplitInv) * (fixed ? finv : 1.f);
  float* out = a.out + (static_cast<long>(b) * a.nchunk + kc) * a.out_rows * R;
#pragma unroll
  for (int c = 0; c < CT; ++c)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb)
      *reinterpret_cast<f32x4*>(out + static_cast<long>(col_base + CT * t + c) * R + 16 * cb + 4 * g) =
          acc[c][cb] * ps;
}

// ---- pass B, not transposed (R = M^T P), h3, with LDS-DMA staging (round 6):
// colproj_h3_kernel's arithmetic at CT columns per lane (bitwise the same products in the same
// order), with rowproj_h3gl_kernel's staging: each step (32 rows) is one unit of D slots -- the
// wave's M tile (32 rows x 16 CT columns, global_load_lds_dwordx4, row-major; row r sits in
// row slot r ^ ((r >> 3) & 1), so the four 8-row groups g that one ds_read serves alternate
// bank halves) and the block's P split of the step -- issued D - 1 steps ahead, D - 2 units in
// flight across each step's closing barrier.  LDS: D (NW 64 CT B x 32 + r 128 B).
template <int CT>
__device__ __forceinline__ int colgl_rs(int r) {
  return CT == 2 ? (r ^ ((r >> 3) & 1)) : r;  // CT = 4: a 256-B row spans all banks
}

template <int RB, int NW, int CT, int D>
__global__ void __launch_bounds__(64 * NW, 1) colproj_h3gl_kernel(const ProjArgs a) {
  constexpr int R = 16 * RB;
  constexpr int NQ = RB * 2 * 64;      // f16x8 units of one step's P split
  constexpr int NS = NQ / (64 * NW);   // split DMA loads per wave and step
  constexpr int WC = 16 * CT;          // columns per wave
  constexpr int RC = WC / 4;           // 16-B chunks per tile row
  constexpr int RPI = 64 / RC;         // tile rows per DMA instruction
  constexpr int NMI = 32 / RPI;        // DMA instructions of M per wave and step
  constexpr int NU = NS + NMI;         // DMA loads per wave and unit
  static_assert(NQ % (64 * NW) == 0 && D >= 2 && D <= 4 && (CT == 2 || CT == 4), "colproj_h3gl_kernel geometry");
  typedef float vec __attribute__((ext_vector_type(CT)));
  __shared__ f16x8 tq[D][NQ];
  __shared__ f32x4 ms[D][NW][32 * RC];
  const BlockXYZ blk = xcd_block_col();
  const int b = blk.z;
  const int kc = blk.y;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (kGlPrio && wave >= 4) __builtin_amdgcn_s_setprio(1);  // the younger half of the 8 waves
  const int lane = tid & 63;
  const int t = lane & 15;
  const int g = lane >> 4;
  const int col_base = blk.x * (WC * NW) + wave * WC;
  const int i_begin = kc * a.kchunk;
  const int i_end = min(a.rows, i_begin + a.kchunk);
  const int nsteps = (i_end - i_begin + 31) / 32;
  // DMA lane: row slot q RPI + lane / RC, chunk lane % RC, loading source row colgl_rs(slot):
  // CT = 2 (RPI 8: instruction q is the 8-row group q) swaps row pairs in odd groups
  const char* Mb = reinterpret_cast<const char*>(a.m[b] + col_base);
  const uint32_t m_off0 = static_cast<uint32_t>((static_cast<long>(lane / RC) * a.ld_m + 4 * (lane % RC)) * 4);
  const uint32_t m_off1 =
      static_cast<uint32_t>((static_cast<long>((lane / RC) ^ (CT == 2 ? 1 : 0)) * a.ld_m + 4 * (lane % RC)) * 4);
  const u32x4* qs = static_cast<const u32x4*>(a.tsplit) + b * a.ts_stride;
  const uint32_t u_off = static_cast<uint32_t>(tid) * 16;
  auto issue = [&](int s, int slot) {
    const long u0 = static_cast<long>((i_begin + 32 * s) / 32);
#pragma unroll
    for (int it = 0; it < NS; ++it)
      glds16<false>(qs + u0 * NQ + it * 64 * NW, u_off, lds_off(&tq[slot][it * 64 * NW + wave * 64]));
    const long i = i_begin + 32 * s;
#pragma unroll
    for (int q = 0; q < NMI; ++q)
      glds16<kNt != 0>(Mb + (i + q * RPI) * a.ld_m * 4, (CT == 2 && (q & 1)) ? m_off1 : m_off0,
                       lds_off(&ms[slot][wave][q * 64]));
  };
  auto wait_units = [](int ahead) {
    if (D >= 4 && ahead >= 2)
      gl_wait_barrier<(D >= 4 ? 2 : 0) * NU>();
    else if (D >= 3 && ahead >= 1)
      gl_wait_barrier<NU>();
    else
      gl_wait_barrier<0>();
  };

  f32x4 acc[CT][RB];
#pragma unroll
  for (int c = 0; c < CT; ++c)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) acc[c][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  const uint32_t mab = a.mabs != nullptr ? a.mabs[b] : kAbsUnknown;
  float finv = 1.f;
  const float fs = h3_scale(__uint_as_float(mab), finv);
  const bool fixed = mab < kAbsUnknown;

#pragma unroll
  for (int s = 0; s < D - 1; ++s)
    if (s < nsteps) issue(s, s);
  wait_units(min(D - 2, nsteps - 1));

  // the scale mode is a template argument of the loop, as in colproj_h3_kernel (with a run-time
  // branch inside the step the per-column scales of the CT = 2 path came out wrong: round 6)
  auto run = [&](auto FIXc) {
  constexpr bool FIX = decltype(FIXc)::value;
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s % D;
    const int nxt = s + D - 1;
    if (nxt < nsteps) issue(nxt, nxt % D);
    const float* xw = reinterpret_cast<const float*>(ms[cur][wave]);
    vec x[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = *reinterpret_cast<const vec*>(xw + colgl_rs<CT>(8 * g + e) * WC + CT * t);
    const f16x8* tqc = tq[cur];
    Split2h B[CT];
    float inv[CT];
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      const f32x4 lo4{x[0][c], x[1][c], x[2][c], x[3][c]};
      const f32x4 hi4{x[4][c], x[5][c], x[6][c], x[7][c]};
      if constexpr (FIX) {
        split2h(lo4, hi4, fs, B[c]);
      } else {
        float m8 = max8abs(lo4, hi4);
        m8 = fmaxf(m8, __shfl_xor(m8, 16, 64));
        m8 = fmaxf(m8, __shfl_xor(m8, 32, 64));
        const float sc = h3_scale(m8, inv[c]);
        split2h(lo4, hi4, sc, B[c]);
      }
    }
    if constexpr (FIX) {
      if constexpr (RB >= 8 && kH3Pairs) {
#pragma unroll
        for (int cp = 0; cp < RB; cp += 2) {
          Split2h A0, A1;
          A0.hi = tqc[(cp * 2 + 0) * 64 + lane];
          A0.lo = tqc[(cp * 2 + 1) * 64 + lane];
          A1.hi = tqc[(cp * 2 + 2) * 64 + lane];
          A1.lo = tqc[(cp * 2 + 3) * 64 + lane];
#pragma unroll
          for (int c = 0; c < CT; ++c) {
            acc[c][cp] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0.lo, B[c].hi, acc[c][cp], 0, 0, 0);
            acc[c][cp + 1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1.lo, B[c].hi, acc[c][cp + 1], 0, 0, 0);
          }
#pragma unroll
          for (int c = 0; c < CT; ++c) {
            acc[c][cp] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0.hi, B[c].lo, acc[c][cp], 0, 0, 0);
            acc[c][cp + 1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1.hi, B[c].lo, acc[c][cp + 1], 0, 0, 0);
          }
#pragma unroll
          for (int c = 0; c < CT; ++c) {
            acc[c][cp] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0.hi, B[c].hi, acc[c][cp], 0, 0, 0);
            acc[c][cp + 1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1.hi, B[c].hi, acc[c][cp + 1], 0, 0, 0);
          }
        }
      } else {
        Split2h A[RB];
#pragma unroll
        for (int cb = 0; cb < RB; ++cb) {
          A[cb].hi = tqc[(cb * 2 + 0) * 64 + lane];
          A[cb].lo = tqc[(cb * 2 + 1) * 64 + lane];
        }
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
          for (int cb = 0; cb < RB; ++cb)
            acc[c][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[cb].lo, B[c].hi, acc[c][cb], 0, 0, 0);
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
          for (int cb = 0; cb < RB; ++cb)
            acc[c][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[cb].hi, B[c].lo, acc[c][cb], 0, 0, 0);
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
          for (int cb = 0; cb < RB; ++cb)
            acc[c][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[cb].hi, B[c].hi, acc[c][cb], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int cb = 0; cb < RB; ++cb) {
        Split2h A;
        A.hi = tqc[(cb * 2 + 0) * 64 + lane];
        A.lo = tqc[(cb * 2 + 1) * 64 + lane];
#pragma unroll
        for (int c = 0; c < CT; ++c) {
          const f32x4 d = mfma3h(A, B[c], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[c][cb][q] = fmaf(d[q], inv[c], acc[c][cb][q]);
        }
      }
    }
    if (s + 1 < nsteps) wait_units(min(nxt, nsteps - 1) - (s + 1));
  }
  };
  if (fixed)
    run(std::true_type{});
  else
    run(std::false_type{});

  const float ps = (a.tinv != nullptr ? a.tinv[b] : kPSplitInv) * (fixed ? finv : 1.f);
  float* out = a.out + (static_cast<long>(b) * a.nchunk + kc) * a.out_rows * R;
#pragma unroll
  for (int c = 0; c < CT; ++c)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb)
      *reinterpret_cast<f32x4*>(out + static_cast<long>(col_base + CT * t + c) * R + 16 * cb + 4 * g) =
          acc[c][cb] * ps;
}

// ---- pass A, not transposed, h3 products (fp16x3): rowproj_ef_kernel's geometry, TJ
// line loads and line stores; the error feedback's fixed operands (P', R') carry
// per-matrix scales, and in the projection the streamed X is the B operand (lane (t, g)
// holds row 16 rb + t, k-run KMAP 1) with a per-step scale per row (max over the lanes
// (t, g = 0..3)), Q the A operand: each step lands in a fresh accumulator
// D[16 cb + 4 g + q][row t] and is added as acc += D / s_row.
template <int RB, int GDT, int PD, int KR = kRBE, int NW = kPaNW>
__global__ void __launch_bounds__(64 * NW, NW >= 8 ? 1 : (RB >= 8 ? 8 / NW : kPaMinb)) rowproj_efh3_kernel(const EfProjArgs e) {
  constexpr int R = 16 * RB;
  constexpr int KK = RB / 2;
  constexpr int NQ = RB * 2 * 64, NR = 2 * KK * 2 * 64;  // f16x8 units of one K-step's splits
  __shared__ f16x8 tq[2][NQ];
  __shared__ f16x8 rs[2][NR];
  __shared__ f32x4 xt[NW][16 * KR * 8];
  const ProjArgs& a = e.p;
  const BlockXYZ blk = xcd_block();
  const int b = blk.z;
  const int nb = gridDim.z;
  const int kc = blk.y;
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int t = lane & 15;
  const int g = lane >> 4;
  const int row_base = blk.x * (16 * KR * NW) + wave * (16 * KR);
  const int j_begin = kc * a.kchunk;
  const int j_end = min(a.cols, j_begin + a.kchunk);
  const void* G = nullptr;
  if constexpr (GDT == DION_DTYPE_BF16)
    G = static_cast<const uint16_t*>(a.g[b]) + static_cast<long>(row_base + t) * a.ld_g + 4 * g;
  else if constexpr (GDT == DION_DTYPE_F32)
    G = static_cast<const float*>(a.g[b]) + static_cast<long>(row_base + t) * a.ld_g + 4 * g;
  float* __restrict__ Mw = a.m[b] + static_cast<long>(row_base + (lane >> 3)) * a.ld_m + 4 * (lane & 7);
  const bool has_ef = e.efr[b] != nullptr;
  const float invQ = e.inv[b];
  const float invR = e.inv[nb + b];
  float invF;
  const float sF = h3_scale(1.f, invF);  // P' (fixed-up P: orthonormal columns, |x| <= 1) on 2^14: exact
  const float efinv = e.alpha * invF * invR;

  Split2h F[KR][KK];
  if (has_ef) {
#pragma unroll
    for (int rb = 0; rb < KR; ++rb)
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const float* src = e.efp[b] + static_cast<long>(row_base + 16 * rb + t) * R + 32 * kk + 8 * g;
        split2h(*reinterpret_cast<const f32x4*>(src), *reinterpret_cast<const f32x4*>(src + 4), sF, F[rb][kk]);
      }
  } else {
#pragma unroll
    for (int rb = 0; rb < KR; ++rb)
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) F[rb][kk] = Split2h{};
  }

  f32x4 acc[KR][RB];
#pragma unroll
  for (int rb = 0; rb < KR; ++rb)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) acc[rb][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint32_t nzb = 0;
  float mx = 0.f;  // max |M| over this wave's rows (m8 of every step)

  const u32x4* qs = e.qsplit + b * e.split_stride;
  const u32x4* rsp = e.rsplit + b * e.split_stride;
  RowStepE<GDT, KR> S[PD];
  auto xload = [&](RowStepE<GDT, KR>& T, int j) {
#pragma unroll
    for (int q = 0; q < 2 * KR; ++q)
      T.x[q >> 1][q & 1] = ld_stream(reinterpret_cast<const f32x4*>(Mw + static_cast<long>(8 * q) * a.ld_m + j));
    rpe_load<GDT, KR>(T, nullptr, G, 0, a.ld_g, j);
  };
  auto xpose = [&](RowStepE<GDT, KR>& T) {
    f32x4* xw = xt[wave];
#pragma unroll
    for (int q = 0; q < 2 * KR; ++q) {
      const int r = 8 * q + (lane >> 3), k = lane & 7;
      xw[r * 8 + (k ^ xt_swz(r))] = T.x[q >> 1][q & 1];
    }
#pragma unroll
    for (int rb = 0; rb < KR; ++rb)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int r = 16 * rb + t, k = 4 * c + g;
        T.x[rb][c] = xw[r * 8 + (k ^ xt_swz(r))];
      }
  };
  auto xstore = [&](const RowStepE<GDT, KR>& T, int j) {
    f32x4* xw = xt[wave];
#pragma unroll
    for (int rb = 0; rb < KR; ++rb)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int r = 16 * rb + t, k = 4 * c + g;
        xw[r * 8 + (k ^ xt_swz(r))] = T.x[rb][c];
      }
#pragma unroll
    for (int q = 0; q < 2 * KR; ++q) {
      const int r = 8 * q + (lane >> 3), k = lane & 7;
      st_stream(reinterpret_cast<f32x4*>(Mw + static_cast<long>(8 * q) * a.ld_m + j), xw[r * 8 + (k ^ xt_swz(r))]);
    }
  };
  auto compute = [&](RowStepE<GDT, KR>& X, const f16x8* tqc, const f16x8* rsc) {
    if (has_ef) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        f32x4 ev[KR];
#pragma unroll
        for (int rb = 0; rb < KR; ++rb) ev[rb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
          Split2h A;
          A.hi = rsc[((c * KK + kk) * 2 + 0) * 64 + lane];
          A.lo = rsc[((c * KK + kk) * 2 + 1) * 64 + lane];
#pragma unroll
          for (int rb = 0; rb < KR; ++rb) ev[rb] = mfma3h(A, F[rb][kk], ev[rb]);
        }
#pragma unroll
        for (int rb = 0; rb < KR; ++rb)
#pragma unroll
          for (int q = 0; q < 4; ++q) X.x[rb][c][q] = fmaf(ev[rb][q], efinv, X.x[rb][c][q]);
      }
    }
#pragma unroll
    for (int rb = 0; rb < KR; ++rb)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        if constexpr (GDT == DION_DTYPE_BF16) {
          const uint2 gv = X.gb[rb][c];
          X.x[rb][c][0] += __uint_as_float(gv.x << 16);
          X.x[rb][c][1] += __uint_as_float(gv.x & 0xFFFF0000u);
          X.x[rb][c][2] += __uint_as_float(gv.y << 16);
          X.x[rb][c][3] += __uint_as_float(gv.y & 0xFFFF0000u);
        } else if constexpr (GDT == DION_DTYPE_F32) {
          X.x[rb][c] += X.gf[rb][c];
        }
        nzb |= __float_as_uint(X.x[rb][c][0]) | __float_as_uint(X.x[rb][c][1]) | __float_as_uint(X.x[rb][c][2]) |
               __float_as_uint(X.x[rb][c][3]);
      }
    Split2h Bx[KR];
    float invx[KR];
#pragma unroll
    for (int rb = 0; rb < KR; ++rb) {
      float m8 = max8abs(X.x[rb][0], X.x[rb][1]);
      m8 = fmaxf(m8, __shfl_xor(m8, 16, 64));
      m8 = fmaxf(m8, __shfl_xor(m8, 32, 64));
      mx = fmaxf(mx, m8);
      const float sx = h3_scale(m8, invx[rb]);
      split2h(X.x[rb][0], X.x[rb][1], sx, Bx[rb]);
    }
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) {
      Split2h A;
      A.hi = tqc[(cb * 2 + 0) * 64 + lane];
      A.lo = tqc[(cb * 2 + 1) * 64 + lane];
#pragma unroll
      for (int rb = 0; rb < KR; ++rb) {
        const f32x4 d = mfma3h(A, Bx[rb], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[rb][cb][q] = fmaf(d[q], invx[rb], acc[rb][cb][q]);
      }
    }
  };

  SplitCopyN<NQ, 64 * NW> TA;
  SplitCopyN<NR, 64 * NW> EA;
#pragma unroll
  for (int k = 0; k < PD - 1; ++k)
    if (j_begin + 32 * k < j_end) xload(S[k], j_begin + 32 * k);
  split_copy_load_n(TA, qs + static_cast<long>(j_begin / 32) * NQ, tid);
  split_copy_store_n(TA, reinterpret_cast<bf16x8*>(tq[0]), tid);
  if (has_ef) {
    split_copy_load_n(EA, rsp + static_cast<long>(j_begin / 32) * NR, tid);
    split_copy_store_n(EA, reinterpret_cast<bf16x8*>(rs[0]), tid);
  }
  __syncthreads();
  int cur = 0;
  for (int j0 = j_begin; j0 < j_end; j0 += 32 * PD) {
#pragma unroll
    for (int k = 0; k < PD; ++k) {
      const int j = j0 + 32 * k;
      if (j >= j_end) break;
      const bool more = j + 32 < j_end;
      if (!kSplitFirst && j + 32 * (PD - 1) < j_end) xload(S[(k + PD - 1) % PD], j + 32 * (PD - 1));
      if (more) {
        split_copy_load_n(TA, qs + static_cast<long>((j + 32) / 32) * NQ, tid);
        if (has_ef) split_copy_load_n(EA, rsp + static_cast<long>((j + 32) / 32) * NR, tid);
      }
      if (kSplitFirst && j + 32 * (PD - 1) < j_end) xload(S[(k + PD - 1) % PD], j + 32 * (PD - 1));
      xpose(S[k]);
      compute(S[k], tq[cur], rs[cur]);
      xstore(S[k], j);
      if (!more) break;
      split_copy_store_n(TA, reinterpret_cast<bf16x8*>(tq[cur ^ 1]), tid);
      if (has_ef) split_copy_store_n(EA, reinterpret_cast<bf16x8*>(rs[cur ^ 1]), tid);
      __syncthreads();
      cur ^= 1;
    }
  }

  float* out = a.out + (static_cast<long>(b) * a.nchunk + kc) * a.out_rows * R;
#pragma unroll
  for (int rb = 0; rb < KR; ++rb)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb)
      *reinterpret_cast<f32x4*>(out + static_cast<long>(row_base + 16 * rb + t) * R + 16 * cb + 4 * g) =
          acc[rb][cb] * invQ;
  if (a.nonzero != nullptr) {
    // the matrix's max |M| for pass B's fixed scale (colproj_h3_kernel); m8 ignores NaN,
    // so an M of zeros and NaNs reports 1 (nonzero, tiny)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    const bool nz = __any((nzb & 0x7FFFFFFFu) != 0u);
    const uint32_t mb = __float_as_uint(mx);
    if (nz && lane == 0) atomicMax(&a.nonzero[b], mb > 1u ? mb : 1u);
  }
}

// ---- pass A, not transposed, r = 128, with LDS-DMA staging: rowproj_efh3_kernel's
// arithmetic on 32-row waves and 32-column steps, in 8-wave blocks (256 rows, two waves per
// SIMD, one block per CU).  Nothing in flight sits in registers: each wave's M and G tiles
// arrive by LDS-DMA two steps ahead into its two slots, the block's Q / R' splits one step
// ahead into a double buffer.  A slot is refilled as soon as the step has read it (the new
// M goes back to HBM straight from the MFMA layout, two 64-B pieces per 128-B line).
//   M slot (per wave, per step): 32 rows x 8 16-B chunks, chunk k of row r at r * 8 + (k ^ (r & 7))
//   G slot (bf16): 32 rows x 4 chunks, chunk k of row r at r * 4 + (k ^ ((r >> 2) & 3))
// The DMA's LDS side is lane-linear, so the swizzles are on the source addresses.  LDS:
// 2 x (16 + 16) KB of splits + 8 waves x 2 slots x 6 KB = 160 KB.  Per wave and step: 4
// LDS-DMA loads of the splits, 4 of M, 2 of G (bf16), 4 stores; the wait before each
// step's barrier leaves the newest M/G step and the stores in flight.
template <int RB, int GDT>
__global__ void __launch_bounds__(512, 1) rowproj_efgl_kernel(const EfProjArgs e) {
  constexpr int R = 16 * RB, KK = RB / 2, KR = 2, NW = 8;
  constexpr int NQ = RB * 2 * 64, NR = 2 * KK * 2 * 64;  // f16x8 units of one step's splits
  constexpr int GCH = GDT == DION_DTYPE_BF16 ? 4 : 0;    // 16-B chunks per G row
  constexpr int NGI = 32 * GCH / 64;
  constexpr int NMG = 4 + NGI;  // M/G LDS-DMA loads per wave and step
  constexpr bool GP = kPaGlGpair != 0 && GCH > 0;  // G in step pairs: gs[h] = half h of the pair
  static_assert(GDT != DION_DTYPE_F32, "f32 G slots do not fit next to the splits (rowproj_efh3_kernel runs)");
  __shared__ f16x8 tq[2][NQ];
  __shared__ f16x8 rs[2][NR];
  __shared__ f32x4 ms[2][NW][32 * 8];
  __shared__ u32x4 gs[2][NW][GCH > 0 ? 32 * GCH : 1];
  const ProjArgs& a = e.p;
  const BlockXYZ blk = xcd_block();
  const int b = blk.z;
  const int nb = gridDim.z;
  const int kc = blk.y;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform (scalar addressing)
  if (kGlPrio && wave >= 4) __builtin_amdgcn_s_setprio(1);  // the younger half of the 8 waves
  const int lane = tid & 63;
  const int t = lane & 15;
  const int g = lane >> 4;
  const int row_base = blk.x * (16 * KR * NW) + wave * (16 * KR);  // the grid's x is rows / 256
  const int j_begin = kc * a.kchunk;
  const int j_end = min(a.cols, j_begin + a.kchunk);
  const int nsteps = (j_end - j_begin + 31) / 32;
  // M: the DMA lane (row 8 q + lane / 8, slot chunk lane % 8) reads source chunk (lane % 8) ^ (lane / 8)
  const char* Mb = reinterpret_cast<const char*>(a.m[b] + static_cast<long>(row_base) * a.ld_m);
  const uint32_t m_off = static_cast<uint32_t>(((lane >> 3) * a.ld_m + 4 * ((lane & 7) ^ (lane >> 3))) * 4);
  // the write-back lane (t, g): rows 16 rb + t, columns 16 c + 4 g .. + 3
  float* __restrict__ Mw = a.m[b] + static_cast<long>(row_base + t) * a.ld_m + 4 * g;
  const char* Gb = nullptr;
  uint32_t g_off = 0;
  if constexpr (GDT == DION_DTYPE_BF16) {  // DMA lane: row 16 i + lane / 4, slot chunk lane % 4
    Gb = reinterpret_cast<const char*>(static_cast<const uint16_t*>(a.g[b]) + static_cast<long>(row_base) * a.ld_g);
    g_off = static_cast<uint32_t>(((lane >> 2) * a.ld_g + 8 * ((lane & 3) ^ ((lane >> 4) & 3))) * 2);
  }
  const bool has_ef = e.efr[b] != nullptr;
  const float invQ = e.inv[b];
  const float invR = e.inv[nb + b];
  float invF;
  const float sF = h3_scale(1.f, invF);  // P' (fixed-up P: orthonormal columns, |x| <= 1) on 2^14: exact
  const float efinv = e.alpha * invF * invR;

  // the EF's fixed operand (P' rows of this wave), loaded before any LDS-DMA is issued
  Split2h F[KR][KK];
  if (has_ef) {
#pragma unroll
    for (int rb = 0; rb < KR; ++rb)
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const float* src = e.efp[b] + static_cast<long>(row_base + 16 * rb + t) * R + 32 * kk + 8 * g;
        split2h(*reinterpret_cast<const f32x4*>(src), *reinterpret_cast<const f32x4*>(src + 4), sF, F[rb][kk]);
      }
  } else {
#pragma unroll
    for (int rb = 0; rb < KR; ++rb)
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) F[rb][kk] = Split2h{};
  }

  f32x4 acc[KR][RB];
#pragma unroll
  for (int rb = 0; rb < KR; ++rb)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) acc[rb][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint32_t nzb = 0;
  float mx = 0.f;

  const u32x4* qs = e.qsplit + b * e.split_stride;
  const u32x4* rsp = e.rsplit + b * e.split_stride;
  // the step's Q and R' splits: unit it * 512 + tid of each (R' is staged whether or not
  // the matrix has a pending EF, so the counts stay fixed; the workspace is always there)
  const uint32_t u_off = static_cast<uint32_t>(tid) * 16;
  auto issue_splits = [&](int s, int buf) {
    const long u0 = static_cast<long>((j_begin + 32 * s) / 32);
#pragma unroll
    for (int it = 0; it < NQ / (64 * NW); ++it)
      glds16<false>(qs + u0 * NQ + it * 64 * NW, u_off, lds_off(&tq[buf][it * 64 * NW + wave * 64]));
#pragma unroll
    for (int it = 0; it < NR / (64 * NW); ++it)
      glds16<false>(rsp + u0 * NR + it * 64 * NW, u_off, lds_off(&rs[buf][it * 64 * NW + wave * 64]));
  };
  auto issue_mg = [&](int s, int slot) {
    const int j = j_begin + 32 * s;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      glds16<kNt != 0>(Mb + (static_cast<long>(8 * q) * a.ld_m + j) * 4, m_off, lds_off(&ms[slot][wave][q * 64]));
    if constexpr (GDT == DION_DTYPE_BF16 && !GP) {
#pragma unroll
      for (int i = 0; i < NGI; ++i)
        glds16<kPaGlGnt != 0>(Gb + (static_cast<long>(16 * i) * a.ld_g + j) * 2, g_off, lds_off(&gs[slot][wave][i * 64]));
    }
  };
  // GP: G of the even step s and of s + 1 (both halves of each 128-B line back to back) into
  // gs[0] / gs[1]; past the chunk's end the second half loads the first again
  auto issue_gpair = [&](int s) {
    if constexpr (GP) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int jh = j_begin + 32 * (s + h < nsteps ? s + h : s);
#pragma unroll
        for (int i = 0; i < NGI; ++i)
          glds16<kPaGlGnt != 0>(Gb + (static_cast<long>(16 * i) * a.ld_g + jh) * 2, g_off, lds_off(&gs[h][wave][i * 64]));
      }
    }
  };

  issue_splits(0, 0);
  issue_mg(0, 0);
  issue_gpair(0);
  if (nsteps > 1) {
    issue_mg(1, 1);
    gl_wait_barrier<GP ? 4 : NMG>();
  } else {
    gl_wait_barrier<0>();
  }
  // GP: the next pair is issued at the odd step, once gs[1] is read: a step ahead of its first
  // use and before that step's M tiles (which stay two steps ahead), so it retires with the
  // splits at the step's barrier

  // the loop runs in step pairs, so the slot and the G pair's parity are compile-time
  auto step = [&](const int s, auto PARc) {
    constexpr int cur = decltype(PARc)::value;  // = s & 1
    const int j = j_begin + 32 * s;
    const bool more = s + 1 < nsteps;
    const bool ahead = s + 2 < nsteps;
    if (more) issue_splits(s + 1, cur ^ 1);

    // the step's M (+ G) in the MFMA layout: lane (t, g) rows 16 rb + t, columns 16 c + 4 g .. + 3
    const f32x4* xw = ms[cur][wave];
    f32x4 X[KR][2];
    uint2 gv[KR][2];
#pragma unroll
    for (int rb = 0; rb < KR; ++rb)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int r = 16 * rb + t, k = 4 * c + g;
        X[rb][c] = xw[r * 8 + (k ^ xt_swz(r))];
        if constexpr (GDT == DION_DTYPE_BF16) {
          const int p = (2 * c + (g >> 1)) ^ ((t >> 2) & 3);
          gv[rb][c] = reinterpret_cast<const uint2*>(gs[cur][wave])[(r * GCH + p) * 2 + (g & 1)];
        }
      }
    if constexpr (GP && cur == 1) {
      if (more) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        issue_gpair(s + 1);
      }
    }
    if (ahead) {
      // the slot is read: refill it (the reads retire first; the DMA writes the same bytes)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      issue_mg(s + 2, cur);
    }
    const f16x8* tqc = tq[cur];
    const f16x8* rsc = rs[cur];
    if (has_ef) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        f32x4 ev[KR];
#pragma unroll
        for (int rb = 0; rb < KR; ++rb) ev[rb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
          Split2h A;
          A.hi = rsc[((c * KK + kk) * 2 + 0) * 64 + lane];
          A.lo = rsc[((c * KK + kk) * 2 + 1) * 64 + lane];
#pragma unroll
          for (int rb = 0; rb < KR; ++rb) ev[rb] = mfma3h(A, F[rb][kk], ev[rb]);
        }
#pragma unroll
        for (int rb = 0; rb < KR; ++rb)
#pragma unroll
          for (int q = 0; q < 4; ++q) X[rb][c][q] = fmaf(ev[rb][q], efinv, X[rb][c][q]);
      }
    }
#pragma unroll
    for (int rb = 0; rb < KR; ++rb)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        if constexpr (GDT == DION_DTYPE_BF16) {
          X[rb][c][0] += __uint_as_float(gv[rb][c].x << 16);
          X[rb][c][1] += __uint_as_float(gv[rb][c].x & 0xFFFF0000u);
          X[rb][c][2] += __uint_as_float(gv[rb][c].y << 16);
          X[rb][c][3] += __uint_as_float(gv[rb][c].y & 0xFFFF0000u);
        }
        nzb |= __float_as_uint(X[rb][c][0]) | __float_as_uint(X[rb][c][1]) | __float_as_uint(X[rb][c][2]) |
               __float_as_uint(X[rb][c][3]);
        st_part(reinterpret_cast<f32x4*>(Mw + static_cast<long>(16 * rb) * a.ld_m + j + 16 * c), X[rb][c]);
      }
    Split2h Bx[KR];
    float invx[KR];
#pragma unroll
    for (int rb = 0; rb < KR; ++rb) {
      float m8 = max8abs(X[rb][0], X[rb][1]);
      m8 = fmaxf(m8, __shfl_xor(m8, 16, 64));
      m8 = fmaxf(m8, __shfl_xor(m8, 32, 64));
      mx = fmaxf(mx, m8);
      const float sx = h3_scale(m8, invx[rb]);
      split2h(X[rb][0], X[rb][1], sx, Bx[rb]);
    }
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) {
      Split2h A;
      A.hi = tqc[(cb * 2 + 0) * 64 + lane];
      A.lo = tqc[(cb * 2 + 1) * 64 + lane];
#pragma unroll
      for (int rb = 0; rb < KR; ++rb) {
        const f32x4 d = mfma3h(A, Bx[rb], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[rb][cb][q] = fmaf(d[q], invx[rb], acc[rb][cb][q]);
      }
    }
    if (more) {
      // retire the next step's splits (and, in order, every older load: the next step's M slot
      // and G); the newest M step and this step's 4 stores may stay in flight
      if (ahead)
        gl_wait_barrier<(GP ? 4 : NMG) + 2 * KR>();
      else
        gl_wait_barrier<2 * KR>();
    }
  };
  for (int s = 0; s < nsteps; s += 2) {
    step(s, std::integral_constant<int, 0>{});
    if (s + 1 < nsteps) step(s + 1, std::integral_constant<int, 1>{});
  }

  float* out = a.out + (static_cast<long>(b) * a.nchunk + kc) * a.out_rows * R;
#pragma unroll
  for (int rb = 0; rb < KR; ++rb)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb)
      *reinterpret_cast<f32x4*>(out + static_cast<long>(row_base + 16 * rb + t) * R + 16 * cb + 4 * g) =
          acc[rb][cb] * invQ;
  if (a.nonzero != nullptr) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    const bool nz = __any((nzb & 0x7FFFFFFFu) != 0u);
    const uint32_t mb = __float_as_uint(mx);
    if (nz && lane == 0) atomicMax(&a.nonzero[b], mb > 1u ? mb : 1u);
  }
}

// ---- pass A, transposed, h3 products: colproj_ef_kernel's geometry (block = 4 waves x
// 32 columns, step = 32 rows; lane (t, g) holds columns 2t, 2t + 1 of rows 16 h + 4 g + q)
// with rowproj_efh3_kernel's arithmetic.  The error feedback's fixed operand is P' of
// the lane's two columns (per-matrix scale), the streamed one R' of the step's rows (the
// A operand, as in the row kernel).  In the projection each column of the step is the B
// operand (its 8 rows are the k-run, KMAP 1) with its own per-step scale (max over the
// four lanes (t, g = 0..3)), Q the A operand: D[16 cb + 4 g + q][col 2t + c] is added as
// acc += D / s_col.  The matrix's max |M| goes into the flag for a fixed-scale pass B.
template <int RB, int GDT>
__global__ void __launch_bounds__(256, (RB >= 8 || kCpeRing) ? 2 : 3) colproj_efh3_kernel(const EfProjArgs e) {
  constexpr int R = 16 * RB;
  constexpr int KK = RB / 2;
  constexpr int NQ = RB * 2 * 64, NR = 2 * KK * 2 * 64;  // f16x8 units of one K-step's splits
  __shared__ f16x8 tq[2][NQ];
  __shared__ f16x8 rs[2][NR];
  const ProjArgs& a = e.p;
  const BlockXYZ blk = xcd_block_col();
  const int b = blk.z;
  const int nb = gridDim.z;
  const int kc = blk.y;
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int t = lane & 15;
  const int g = lane >> 4;
  const int col_base = blk.x * 128 + wave * 32;
  const int i_begin = kc * a.kchunk;
  const int i_end = min(a.rows, i_begin + a.kchunk);
  float* __restrict__ M = a.m[b] + static_cast<long>(4 * g) * a.ld_m + col_base + 2 * t;
  const void* G = nullptr;
  if constexpr (GDT == DION_DTYPE_BF16)
    G = static_cast<const uint16_t*>(a.g[b]) + static_cast<long>(4 * g) * a.ld_g + col_base + 2 * t;
  else if constexpr (GDT == DION_DTYPE_F32)
    G = static_cast<const float*>(a.g[b]) + static_cast<long>(4 * g) * a.ld_g + col_base + 2 * t;
  const bool has_ef = e.efr[b] != nullptr;
  const float invQ = e.inv[b];
  const float invR = e.inv[nb + b];
  float invF;
  const float sF = h3_scale(1.f, invF);  // P' (fixed-up P: orthonormal columns, |x| <= 1) on 2^14: exact
  const float efinv = e.alpha * invF * invR;

  // fixed EF factor: P'[col_base + 2t + c][32 kk + 8 g ...] (B operand of tile c)
  Split2h F[2][KK];
  if (has_ef) {
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const float* src = e.efp[b] + static_cast<long>(col_base + 2 * t + c) * R + 32 * kk + 8 * g;
        split2h(*reinterpret_cast<const f32x4*>(src), *reinterpret_cast<const f32x4*>(src + 4), sF, F[c][kk]);
      }
  } else {
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) F[c][kk] = Split2h{};
  }

  f32x4 acc[2][RB];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) acc[c][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint32_t nzb = 0;
  float mx = 0.f;

  auto compute = [&](ColStepE<GDT>& S, const f16x8* tqc, const f16x8* rsc, int i0) {
    if (has_ef) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f32x4 ev[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
          Split2h A;
          A.hi = rsc[((h * KK + kk) * 2 + 0) * 64 + lane];
          A.lo = rsc[((h * KK + kk) * 2 + 1) * 64 + lane];
#pragma unroll
          for (int c = 0; c < 2; ++c) ev[c] = mfma3h(A, F[c][kk], ev[c]);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          S.x[h][q][0] = fmaf(ev[0][q], efinv, S.x[h][q][0]);
          S.x[h][q][1] = fmaf(ev[1][q], efinv, S.x[h][q][1]);
        }
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if constexpr (GDT == DION_DTYPE_BF16) {
          S.x[h][q][0] += __uint_as_float(S.gb[h][q] << 16);
          S.x[h][q][1] += __uint_as_float(S.gb[h][q] & 0xFFFF0000u);
        } else if constexpr (GDT == DION_DTYPE_F32) {
          S.x[h][q] += S.gf[h][q];
        }
        if (GDT != DION_DTYPE_NONE || has_ef)
          st_stream(reinterpret_cast<f32x2*>(M + static_cast<long>(i0 + 16 * h + q) * a.ld_m), S.x[h][q]);
        nzb |= __float_as_uint(S.x[h][q][0]) | __float_as_uint(S.x[h][q][1]);
      }
    Split2h Bx[2];
    float invx[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const f32x4 lo4{S.x[0][0][c], S.x[0][1][c], S.x[0][2][c], S.x[0][3][c]};
      const f32x4 hi4{S.x[1][0][c], S.x[1][1][c], S.x[1][2][c], S.x[1][3][c]};
      float m8 = max8abs(lo4, hi4);
      m8 = fmaxf(m8, __shfl_xor(m8, 16, 64));
      m8 = fmaxf(m8, __shfl_xor(m8, 32, 64));
      mx = fmaxf(mx, m8);
      const float sx = h3_scale(m8, invx[c]);
      split2h(lo4, hi4, sx, Bx[c]);
    }
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) {
      Split2h A;
      A.hi = tqc[(cb * 2 + 0) * 64 + lane];
      A.lo = tqc[(cb * 2 + 1) * 64 + lane];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const f32x4 d = mfma3h(A, Bx[c], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[c][cb][q] = fmaf(d[q], invx[c], acc[c][cb][q]);
      }
    }
  };

  const u32x4* qs = e.qsplit + b * e.split_stride;
  const u32x4* rsp = e.rsplit + b * e.split_stride;
  if constexpr (RB >= 8 || !kCpeRing) {
    // no register ring: the step's M/G load is issued right before its use, the other
    // blocks of the CU (3 per CU at this register count) cover its latency
    ColStepE<GDT> S;
    SplitCopy<NQ> TA;
    SplitCopy<NR> EA;
    split_copy_load<NQ>(TA, qs + static_cast<long>(i_begin / 32) * NQ, tid);
    split_copy_store<NQ>(TA, reinterpret_cast<bf16x8*>(tq[0]), tid);
    if (has_ef) {
      split_copy_load<NR>(EA, rsp + static_cast<long>(i_begin / 32) * NR, tid);
      split_copy_store<NR>(EA, reinterpret_cast<bf16x8*>(rs[0]), tid);
    }
    __syncthreads();
    int cur = 0;
    for (int i0 = i_begin; i0 < i_end; i0 += 32) {
      const bool more = i0 + 32 < i_end;
      cpe_load<GDT>(S, M, G, a.ld_m, a.ld_g, i0);
      if (more) {
        split_copy_load<NQ>(TA, qs + static_cast<long>(i0 / 32 + 1) * NQ, tid);
        if (has_ef) split_copy_load<NR>(EA, rsp + static_cast<long>(i0 / 32 + 1) * NR, tid);
      }
      compute(S, tq[cur], rs[cur], i0);
      if (!more) break;
      split_copy_store<NQ>(TA, reinterpret_cast<bf16x8*>(tq[cur ^ 1]), tid);
      if (has_ef) split_copy_store<NR>(EA, reinterpret_cast<bf16x8*>(rs[cur ^ 1]), tid);
      __syncthreads();
      cur ^= 1;
    }
  } else {
  ColStepE<GDT> SA, SB;
  SplitCopy<NQ> TA;
  SplitCopy<NR> EA;
  cpe_load<GDT>(SA, M, G, a.ld_m, a.ld_g, i_begin);
  split_copy_load<NQ>(TA, qs + static_cast<long>(i_begin / 32) * NQ, tid);
  split_copy_store<NQ>(TA, reinterpret_cast<bf16x8*>(tq[0]), tid);
  if (has_ef) {
    split_copy_load<NR>(EA, rsp + static_cast<long>(i_begin / 32) * NR, tid);
    split_copy_store<NR>(EA, reinterpret_cast<bf16x8*>(rs[0]), tid);
  }
  __syncthreads();
  int cur = 0;
  for (int i0 = i_begin; i0 < i_end; i0 += 64) {
    const bool more = i0 + 32 < i_end;
    if (more) {
      if (!kSplitFirst) cpe_load<GDT>(SB, M, G, a.ld_m, a.ld_g, i0 + 32);
      split_copy_load<NQ>(TA, qs + static_cast<long>(i0 / 32 + 1) * NQ, tid);
      if (has_ef) split_copy_load<NR>(EA, rsp + static_cast<long>(i0 / 32 + 1) * NR, tid);
      if (kSplitFirst) cpe_load<GDT>(SB, M, G, a.ld_m, a.ld_g, i0 + 32);
    }
    compute(SA, tq[cur], rs[cur], i0);
    if (!more) break;
    split_copy_store<NQ>(TA, reinterpret_cast<bf16x8*>(tq[cur ^ 1]), tid);
    if (has_ef) split_copy_store<NR>(EA, reinterpret_cast<bf16x8*>(rs[cur ^ 1]), tid);
    __syncthreads();
    cur ^= 1;
    const bool more2 = i0 + 64 < i_end;
    if (more2) {
      if (!kSplitFirst) cpe_load<GDT>(SA, M, G, a.ld_m, a.ld_g, i0 + 64);
      split_copy_load<NQ>(TA, qs + static_cast<long>(i0 / 32 + 2) * NQ, tid);
      if (has_ef) split_copy_load<NR>(EA, rsp + static_cast<long>(i0 / 32 + 2) * NR, tid);
      if (kSplitFirst) cpe_load<GDT>(SA, M, G, a.ld_m, a.ld_g, i0 + 64);
    }
    compute(SB, tq[cur], rs[cur], i0 + 32);
    if (!more2) break;
    split_copy_store<NQ>(TA, reinterpret_cast<bf16x8*>(tq[cur ^ 1]), tid);
    if (has_ef) split_copy_store<NR>(EA, reinterpret_cast<bf16x8*>(rs[cur ^ 1]), tid);
    __syncthreads();
    cur ^= 1;
  }
  }

  float* out = a.out + (static_cast<long>(b) * a.nchunk + kc) * a.out_rows * R;
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb)
      *reinterpret_cast<f32x4*>(out + static_cast<long>(col_base + 2 * t + c) * R + 16 * cb + 4 * g) =
          acc[c][cb] * invQ;
  if (a.nonzero != nullptr) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    const bool nz = __any((nzb & 0x7FFFFFFFu) != 0u);
    const uint32_t mb = __float_as_uint(mx);
    if (nz && lane == 0) atomicMax(&a.nonzero[b], mb > 1u ? mb : 1u);
  }
}

// ---- pass A, transposed, r = 128, with LDS-DMA staging: colproj_efh3_kernel's arithmetic
// (lane (t, g): columns 2t, 2t + 1 of rows 16 h + 4 g + q) in 8-wave blocks of 256 columns,
// the slots and splits staged as in rowproj_efgl_kernel (M/G two steps ahead, splits one).
//   M slot: 32 rows x 128 B (row-major, as in HBM), G slot (bf16): 32 rows x 64 B.
// Per wave and step: 4 LDS-DMA loads of the splits, 4 of M, 2 of G (bf16), 8 stores.
template <int RB, int GDT>
__global__ void __launch_bounds__(512, 1) colproj_efgl_kernel(const EfProjArgs e) {
  constexpr int R = 16 * RB, KK = RB / 2, NW = 8;
  constexpr int NQ = RB * 2 * 64, NR = 2 * KK * 2 * 64;
  constexpr int NGI = GDT == DION_DTYPE_BF16 ? 2 : 0;
  constexpr int NMG = 4 + NGI;
  static_assert(GDT != DION_DTYPE_F32, "f32 G slots do not fit next to the splits (colproj_efh3_kernel runs)");
  __shared__ f16x8 tq[2][NQ];
  __shared__ f16x8 rs[2][NR];
  __shared__ f32x4 ms[2][NW][32 * 8];
  __shared__ u32x4 gs[2][NW][NGI > 0 ? 32 * 4 : 1];
  const ProjArgs& a = e.p;
  const BlockXYZ blk = xcd_block_col();
  const int b = blk.z;
  const int nb = gridDim.z;
  const int kc = blk.y;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (kGlPrio && wave >= 4) __builtin_amdgcn_s_setprio(1);  // the younger half of the 8 waves
  const int lane = tid & 63;
  const int t = lane & 15;
  const int g = lane >> 4;
  const int col_base = blk.x * (32 * NW) + wave * 32;  // the grid's x is columns / 256
  const int i_begin = kc * a.kchunk;
  const int i_end = min(a.rows, i_begin + a.kchunk);
  const int nsteps = (i_end - i_begin + 31) / 32;
  const char* Mb = reinterpret_cast<const char*>(a.m[b] + col_base);
  const uint32_t m_off = static_cast<uint32_t>(((lane >> 3) * a.ld_m + 4 * (lane & 7)) * 4);  // row lane / 8, chunk lane % 8
  float* __restrict__ Mw = a.m[b] + static_cast<long>(4 * g) * a.ld_m + col_base + 2 * t;
  const char* Gb = nullptr;
  uint32_t g_off = 0;
  if constexpr (GDT == DION_DTYPE_BF16) {  // row lane / 4, chunk lane % 4
    Gb = reinterpret_cast<const char*>(static_cast<const uint16_t*>(a.g[b]) + col_base);
    g_off = static_cast<uint32_t>(((lane >> 2) * a.ld_g + 8 * (lane & 3)) * 2);
  }
  const bool has_ef = e.efr[b] != nullptr;
  const float invQ = e.inv[b];
  const float invR = e.inv[nb + b];
  float invF;
  const float sF = h3_scale(1.f, invF);  // P' (fixed-up P: orthonormal columns, |x| <= 1) on 2^14: exact
  const float efinv = e.alpha * invF * invR;

  Split2h F[2][KK];
  if (has_ef) {
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const float* src = e.efp[b] + static_cast<long>(col_base + 2 * t + c) * R + 32 * kk + 8 * g;
        split2h(*reinterpret_cast<const f32x4*>(src), *reinterpret_cast<const f32x4*>(src + 4), sF, F[c][kk]);
      }
  } else {
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) F[c][kk] = Split2h{};
  }

  f32x4 acc[2][RB];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) acc[c][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint32_t nzb = 0;
  float mx = 0.f;

  const u32x4* qs = e.qsplit + b * e.split_stride;
  const u32x4* rsp = e.rsplit + b * e.split_stride;
  const uint32_t u_off = static_cast<uint32_t>(tid) * 16;
  auto issue_splits = [&](int s, int buf) {
    const long u0 = static_cast<long>((i_begin + 32 * s) / 32);
#pragma unroll
    for (int it = 0; it < NQ / (64 * NW); ++it)
      glds16<false>(qs + u0 * NQ + it * 64 * NW, u_off, lds_off(&tq[buf][it * 64 * NW + wave * 64]));
#pragma unroll
    for (int it = 0; it < NR / (64 * NW); ++it)
      glds16<false>(rsp + u0 * NR + it * 64 * NW, u_off, lds_off(&rs[buf][it * 64 * NW + wave * 64]));
  };
  auto issue_mg = [&](int s, int slot) {
    const long i0 = i_begin + 32 * s;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      glds16<kNt != 0>(Mb + (i0 + 8 * q) * a.ld_m * 4, m_off, lds_off(&ms[slot][wave][q * 64]));
    if constexpr (GDT == DION_DTYPE_BF16) {
#pragma unroll
      for (int i = 0; i < NGI; ++i)
        glds16<kCpeGnt != 0>(Gb + (i0 + 16 * i) * a.ld_g * 2, g_off, lds_off(&gs[slot][wave][i * 64]));
    }
  };

  issue_splits(0, 0);
  issue_mg(0, 0);
  if (nsteps > 1) {
    issue_mg(1, 1);
    gl_wait_barrier<NMG>();
  } else {
    gl_wait_barrier<0>();
  }

  for (int s = 0; s < nsteps; ++s) {
    const int i0 = i_begin + 32 * s;
    const int cur = s & 1;
    const bool more = s + 1 < nsteps;
    const bool ahead = s + 2 < nsteps;
    if (more) issue_splits(s + 1, cur ^ 1);

    f32x2 X[2][4];
    uint32_t gv[2][4];
    const f32x2* xw = reinterpret_cast<const f32x2*>(ms[cur][wave]);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = 16 * h + 4 * g + q;
        X[h][q] = xw[r * 16 + t];
        if constexpr (GDT == DION_DTYPE_BF16) gv[h][q] = reinterpret_cast<const uint32_t*>(gs[cur][wave])[r * 16 + t];
      }
    if (ahead) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      issue_mg(s + 2, cur);
    }
    const f16x8* tqc = tq[cur];
    const f16x8* rsc = rs[cur];
    if (has_ef) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f32x4 ev[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
          Split2h A;
          A.hi = rsc[((h * KK + kk) * 2 + 0) * 64 + lane];
          A.lo = rsc[((h * KK + kk) * 2 + 1) * 64 + lane];
#pragma unroll
          for (int c = 0; c < 2; ++c) ev[c] = mfma3h(A, F[c][kk], ev[c]);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          X[h][q][0] = fmaf(ev[0][q], efinv, X[h][q][0]);
          X[h][q][1] = fmaf(ev[1][q], efinv, X[h][q][1]);
        }
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if constexpr (GDT == DION_DTYPE_BF16) {
          X[h][q][0] += __uint_as_float(gv[h][q] << 16);
          X[h][q][1] += __uint_as_float(gv[h][q] & 0xFFFF0000u);
        }
        if (GDT != DION_DTYPE_NONE || has_ef)
          st_stream(reinterpret_cast<f32x2*>(Mw + static_cast<long>(i0 + 16 * h + q) * a.ld_m), X[h][q]);
        nzb |= __float_as_uint(X[h][q][0]) | __float_as_uint(X[h][q][1]);
      }
    Split2h Bx[2];
    float invx[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const f32x4 lo4{X[0][0][c], X[0][1][c], X[0][2][c], X[0][3][c]};
      const f32x4 hi4{X[1][0][c], X[1][1][c], X[1][2][c], X[1][3][c]};
      float m8 = max8abs(lo4, hi4);
      m8 = fmaxf(m8, __shfl_xor(m8, 16, 64));
      m8 = fmaxf(m8, __shfl_xor(m8, 32, 64));
      mx = fmaxf(mx, m8);
      const float sx = h3_scale(m8, invx[c]);
      split2h(lo4, hi4, sx, Bx[c]);
    }
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) {
      Split2h A;
      A.hi = tqc[(cb * 2 + 0) * 64 + lane];
      A.lo = tqc[(cb * 2 + 1) * 64 + lane];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const f32x4 d = mfma3h(A, Bx[c], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[c][cb][q] = fmaf(d[q], invx[c], acc[c][cb][q]);
      }
    }
    if (more) {
      // the stores of this step: 8 when M is written, else none
      if (GDT != DION_DTYPE_NONE || has_ef) {
        if (ahead)
          gl_wait_barrier<NMG + 8>();
        else
          gl_wait_barrier<8>();
      } else {
        if (ahead)
          gl_wait_barrier<NMG>();
        else
          gl_wait_barrier<0>();
      }
    }
  }

  float* out = a.out + (static_cast<long>(b) * a.nchunk + kc) * a.out_rows * R;
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb)
      *reinterpret_cast<f32x4*>(out + static_cast<long>(col_base + 2 * t + c) * R + 16 * cb + 4 * g) =
          acc[c][cb] * invQ;
  if (a.nonzero != nullptr) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    const bool nz = __any((nzb & 0x7FFFFFFFu) != 0u);
    const uint32_t mb = __float_as_uint(mx);
    if (nz && lane == 0) atomicMax(&a.nonzero[b], mb > 1u ? mb : 1u);
  }
}

// ---- pass B, transposed (R = M P), h3 products: rowproj_x6_kernel's geometry and whole-
// line loads (lane (t, g) after the LDS transpose: row 16 rb + t, k-run KMAP 1 = columns
// 16 c + 4 g .. + 3).  The streamed M is the B operand, the pre-split P the A operand
// (one scale per matrix); with pass A's max |M| the step's products accumulate in place
// under one scale for the matrix, else each row gets a per-step scale (as in pass A).
template <int RB, int NW>
__global__ void __launch_bounds__(64 * NW, ((RB >= 8 && !kH3Pairs) || NW >= 8) ? 1 : (kPbrRing ? (RB <= 4 ? kPbrMinb : 2) : 3))
    rowproj_h3_kernel(const ProjArgs a) {
  constexpr int R = 16 * RB;
  constexpr int NQ = RB * 2 * 64;
  __shared__ f16x8 tq[2][NQ];
  __shared__ f32x4 xt[NW][32 * 8];
  const BlockXYZ blk = xcd_block();
  const int b = blk.z;
  const int kc = blk.y;
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int t = lane & 15;
  const int g = lane >> 4;
  const int row_base = blk.x * (16 * kRBE * NW) + wave * (16 * kRBE);
  const int j_begin = kc * a.kchunk;
  const int j_end = min(a.cols, j_begin + a.kchunk);

  auto cj = [](int j) { return j; };
  const float* __restrict__ Mw = a.m[b] + static_cast<long>(row_base + (lane >> 3)) * a.ld_m + 4 * (lane & 7);
  auto xload = [&](RowStepE<DION_DTYPE_NONE>& T, int j) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      T.x[q >> 1][q & 1] = ld_stream(reinterpret_cast<const f32x4*>(Mw + static_cast<long>(8 * q) * a.ld_m + j));
  };
  auto xpose = [&](RowStepE<DION_DTYPE_NONE>& T) {
    f32x4* xw = xt[wave];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = 8 * q + (lane >> 3), k = lane & 7;
      xw[r * 8 + (k ^ xt_swz(r))] = T.x[q >> 1][q & 1];
    }
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int r = 16 * rb + t, k = 4 * c + g;
        T.x[rb][c] = xw[r * 8 + (k ^ xt_swz(r))];
      }
  };

  f32x4 acc[kRBE][RB];
#pragma unroll
  for (int rb = 0; rb < kRBE; ++rb)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) acc[rb][cb] = f32x4{0.f, 0.f, 0.f, 0.f};

  const u32x4* qs = static_cast<const u32x4*>(a.tsplit) + b * a.ts_stride;
  const uint32_t mab = a.mabs != nullptr ? a.mabs[b] : kAbsUnknown;
  float finv = 1.f;
  const float fs = h3_scale(__uint_as_float(mab), finv);
  auto run = [&](auto FIXc) {
    constexpr bool FIX = decltype(FIXc)::value;
    RowStepE<DION_DTYPE_NONE> SA, SB;
    SplitCopyN<NQ, 64 * NW> TA;
    auto compute = [&](RowStepE<DION_DTYPE_NONE>& X, const f16x8* tqc) {
      Split2h Bx[kRBE];
      float invx[kRBE];
#pragma unroll
      for (int rb = 0; rb < kRBE; ++rb) {
        if constexpr (FIX) {
          split2h(X.x[rb][0], X.x[rb][1], fs, Bx[rb]);
        } else {
          float m8 = max8abs(X.x[rb][0], X.x[rb][1]);
          m8 = fmaxf(m8, __shfl_xor(m8, 16, 64));
          m8 = fmaxf(m8, __shfl_xor(m8, 32, 64));
          const float sx = h3_scale(m8, invx[rb]);
          split2h(X.x[rb][0], X.x[rb][1], sx, Bx[rb]);
        }
      }
      if constexpr (FIX && RB >= 8 && kH3Pairs) {
        // r > 64: two cb of the split P at a time (see colproj_h3_kernel)
#pragma unroll
        for (int cp = 0; cp < RB; cp += 2) {
          Split2h A0, A1;
          A0.hi = tqc[(cp * 2 + 0) * 64 + lane];
          A0.lo = tqc[(cp * 2 + 1) * 64 + lane];
          A1.hi = tqc[(cp * 2 + 2) * 64 + lane];
          A1.lo = tqc[(cp * 2 + 3) * 64 + lane];
#pragma unroll
          for (int rb = 0; rb < kRBE; ++rb) {
            acc[rb][cp] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0.lo, Bx[rb].hi, acc[rb][cp], 0, 0, 0);
            acc[rb][cp + 1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1.lo, Bx[rb].hi, acc[rb][cp + 1], 0, 0, 0);
          }
#pragma unroll
          for (int rb = 0; rb < kRBE; ++rb) {
            acc[rb][cp] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0.hi, Bx[rb].lo, acc[rb][cp], 0, 0, 0);
            acc[rb][cp + 1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1.hi, Bx[rb].lo, acc[rb][cp + 1], 0, 0, 0);
          }
#pragma unroll
          for (int rb = 0; rb < kRBE; ++rb) {
            acc[rb][cp] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0.hi, Bx[rb].hi, acc[rb][cp], 0, 0, 0);
            acc[rb][cp + 1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1.hi, Bx[rb].hi, acc[rb][cp + 1], 0, 0, 0);
          }
        }
      } else if constexpr (FIX) {
        // the three products term by term: consecutive MFMAs are independent
        Split2h A[RB];
#pragma unroll
        for (int cb = 0; cb < RB; ++cb) {
          A[cb].hi = tqc[(cb * 2 + 0) * 64 + lane];
          A[cb].lo = tqc[(cb * 2 + 1) * 64 + lane];
        }
#pragma unroll
        for (int rb = 0; rb < kRBE; ++rb)
#pragma unroll
          for (int cb = 0; cb < RB; ++cb)
            acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[cb].lo, Bx[rb].hi, acc[rb][cb], 0, 0, 0);
#pragma unroll
        for (int rb = 0; rb < kRBE; ++rb)
#pragma unroll
          for (int cb = 0; cb < RB; ++cb)
            acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[cb].hi, Bx[rb].lo, acc[rb][cb], 0, 0, 0);
#pragma unroll
        for (int rb = 0; rb < kRBE; ++rb)
#pragma unroll
          for (int cb = 0; cb < RB; ++cb)
            acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[cb].hi, Bx[rb].hi, acc[rb][cb], 0, 0, 0);
      } else {
#pragma unroll
        for (int cb = 0; cb < RB; ++cb) {
          Split2h A;
          A.hi = tqc[(cb * 2 + 0) * 64 + lane];
          A.lo = tqc[(cb * 2 + 1) * 64 + lane];
#pragma unroll
          for (int rb = 0; rb < kRBE; ++rb) {
            const f32x4 d = mfma3h(A, Bx[rb], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[rb][cb][q] = fmaf(d[q], invx[rb], acc[rb][cb][q]);
          }
        }
      }
    };
    if constexpr (!kPbrRing) {
      split_copy_load_n(TA, qs + static_cast<long>(cj(j_begin) / 32) * NQ, tid);
      split_copy_store_n(TA, reinterpret_cast<bf16x8*>(tq[0]), tid);
      __syncthreads();
      int cur = 0;
      for (int j0 = j_begin; j0 < j_end; j0 += 32) {
        const bool more = j0 + 32 < j_end;
        xload(SA, cj(j0));
        if (more) split_copy_load_n(TA, qs + static_cast<long>(cj(j0 + 32) / 32) * NQ, tid);
        xpose(SA);
        compute(SA, tq[cur]);
        if (!more) break;
        split_copy_store_n(TA, reinterpret_cast<bf16x8*>(tq[cur ^ 1]), tid);
        __syncthreads();
        cur ^= 1;
      }
      return;
    }
    xload(SA, cj(j_begin));
    split_copy_load_n(TA, qs + static_cast<long>(cj(j_begin) / 32) * NQ, tid);
    split_copy_store_n(TA, reinterpret_cast<bf16x8*>(tq[0]), tid);
    __syncthreads();
    int cur = 0;
    for (int j0 = j_begin; j0 < j_end; j0 += 64) {
      const bool more = j0 + 32 < j_end;
      if (more) {
        if (!kSplitFirstB) xload(SB, cj(j0 + 32));
        split_copy_load_n(TA, qs + static_cast<long>(cj(j0 + 32) / 32) * NQ, tid);
        if (kSplitFirstB) xload(SB, cj(j0 + 32));
      }
      xpose(SA);
      compute(SA, tq[cur]);
      if (!more) break;
      split_copy_store_n(TA, reinterpret_cast<bf16x8*>(tq[cur ^ 1]), tid);
      __syncthreads();
      cur ^= 1;
      const bool more2 = j0 + 64 < j_end;
      if (more2) {
        if (!kSplitFirstB) xload(SA, cj(j0 + 64));
        split_copy_load_n(TA, qs + static_cast<long>(cj(j0 + 64) / 32) * NQ, tid);
        if (kSplitFirstB) xload(SA, cj(j0 + 64));
      }
      xpose(SB);
      compute(SB, tq[cur]);
      if (!more2) break;
      split_copy_store_n(TA, reinterpret_cast<bf16x8*>(tq[cur ^ 1]), tid);
      __syncthreads();
      cur ^= 1;
    }
  };
  const bool fixed = mab < kAbsUnknown;
  if (fixed)
    run(std::true_type{});
  else
    run(std::false_type{});

  // lane (t, g): R row 16 rb + t, columns 16 cb + 4 g .. + 3 (a.tinv null: fixed P split scale)
  const float ps = (a.tinv != nullptr ? a.tinv[b] : kPSplitInv) * (fixed ? finv : 1.f);
  float* out = a.out + (static_cast<long>(b) * a.nchunk + kc) * a.out_rows * R;
#pragma unroll
  for (int rb = 0; rb < kRBE; ++rb)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb)
      *reinterpret_cast<f32x4*>(out + static_cast<long>(row_base + 16 * rb + t) * R + 16 * cb + 4 * g) =
          acc[rb][cb] * ps;
}

// ---- pass B, transposed (R = M P), h3, with LDS-DMA staging (round 6): rowproj_h3_kernel's
// arithmetic (bitwise: the same products in the same order), but nothing in flight sits in
// registers.  rowproj_h3_kernel loads a step's M into registers and needs it at once, so the
// only latency cover is the other resident waves, each with one 4 KB step in flight during
// its load phase; its SQ counters show the waves waiting (wait_any 0.58) at 0.65 of 8 TB/s
// on a read-only stream.  Here every step is one unit of D slots: the wave's M tile (32 rows
// x 32 columns, 4 KB, global_load_lds_dwordx4 straight into the transpose tile's swizzled
// layout: chunk k of row r at r * 8 + (k ^ (r & 7)), the swizzle on the source address) and
// the block's P split of the step (NQ x 16 B).  Units are issued in step order D - 1 steps
// ahead; the wait that closes a step retires only the next step's unit (vector-memory
// operations retire in issue order), so D - 2 units stay in flight across every barrier.  A
// unit's slot is refilled at the top of the step after the one that read it, behind that
// step's closing barrier (all waves are done with its split).  LDS: D (NW 4 KB + NQ 16 B).
template <int RB, int NW, int D>
__global__ void __launch_bounds__(64 * NW, 1) rowproj_h3gl_kernel(const ProjArgs a) {
  constexpr int R = 16 * RB;
  constexpr int NQ = RB * 2 * 64;          // f16x8 units of one step's P split
  constexpr int NS = NQ / (64 * NW);       // split DMA loads per wave and step
  constexpr int NU = NS + 4;               // DMA loads per wave and unit
  static_assert(NQ % (64 * NW) == 0 && D >= 2 && D <= 4, "rowproj_h3gl_kernel geometry");
  __shared__ f16x8 tq[D][NQ];
  __shared__ f32x4 ms[D][NW][32 * 8];
  const BlockXYZ blk = xcd_block();
  const int b = blk.z;
  const int kc = blk.y;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (kGlPrio && wave >= 4) __builtin_amdgcn_s_setprio(1);  // the younger half of the 8 waves
  const int lane = tid & 63;
  const int t = lane & 15;
  const int g = lane >> 4;
  const int row_base = blk.x * (32 * NW) + wave * 32;
  const int j_begin = kc * a.kchunk;
  const int j_end = min(a.cols, j_begin + a.kchunk);
  const int nsteps = (j_end - j_begin + 31) / 32;
  // DMA lane (row 8 q + lane / 8, slot chunk lane % 8) reads source chunk (lane % 8) ^ (lane / 8)
  const char* Mb = reinterpret_cast<const char*>(a.m[b] + static_cast<long>(row_base) * a.ld_m);
  const uint32_t m_off = static_cast<uint32_t>(((lane >> 3) * a.ld_m + 4 * ((lane & 7) ^ (lane >> 3))) * 4);
  const u32x4* qs = static_cast<const u32x4*>(a.tsplit) + b * a.ts_stride;
  const uint32_t u_off = static_cast<uint32_t>(tid) * 16;
  auto issue = [&](int s, int slot) {
    const long u0 = static_cast<long>((j_begin + 32 * s) / 32);
#pragma unroll
    for (int it = 0; it < NS; ++it)
      glds16<false>(qs + u0 * NQ + it * 64 * NW, u_off, lds_off(&tq[slot][it * 64 * NW + wave * 64]));
    const int j = j_begin + 32 * s;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      glds16<kNt != 0>(Mb + (static_cast<long>(8 * q) * a.ld_m + j) * 4, m_off, lds_off(&ms[slot][wave][q * 64]));
  };
  // retire every unit but the newest `ahead` (0 .. D - 2) and meet the block
  auto wait_units = [](int ahead) {
    if (D >= 4 && ahead >= 2)
      gl_wait_barrier<(D >= 4 ? 2 : 0) * NU>();
    else if (D >= 3 && ahead >= 1)
      gl_wait_barrier<NU>();
    else
      gl_wait_barrier<0>();
  };

  f32x4 acc[kRBE][RB];
#pragma unroll
  for (int rb = 0; rb < kRBE; ++rb)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) acc[rb][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  const uint32_t mab = a.mabs != nullptr ? a.mabs[b] : kAbsUnknown;
  float finv = 1.f;
  const float fs = h3_scale(__uint_as_float(mab), finv);
  const bool fixed = mab < kAbsUnknown;

#pragma unroll
  for (int s = 0; s < D - 1; ++s)
    if (s < nsteps) issue(s, s);
  wait_units(min(D - 2, nsteps - 1));

  // the scale mode is a template argument of the loop (colproj_h3gl_kernel: a run-time branch
  // inside the step gave wrong per-column scales there)
  auto run = [&](auto FIXc) {
  constexpr bool FIX = decltype(FIXc)::value;
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s % D;
    const int nxt = s + D - 1;  // its slot (s - 1) % D was read by every wave before the last barrier
    if (nxt < nsteps) issue(nxt, nxt % D);
    const f32x4* xw = ms[cur][wave];
    f32x4 X[kRBE][2];
#pragma unroll
    for (int rb = 0; rb < kRBE; ++rb)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int r = 16 * rb + t, k = 4 * c + g;
        X[rb][c] = xw[r * 8 + (k ^ xt_swz(r))];
      }
    const f16x8* tqc = tq[cur];
    Split2h Bx[kRBE];
    float invx[kRBE];
    if constexpr (FIX) {
#pragma unroll
      for (int rb = 0; rb < kRBE; ++rb) split2h(X[rb][0], X[rb][1], fs, Bx[rb]);
      if constexpr (RB >= 8 && kH3Pairs) {
        // r > 64: two cb of the split P at a time (rowproj_h3_kernel's order)
#pragma unroll
        for (int cp = 0; cp < RB; cp += 2) {
          Split2h A0, A1;
          A0.hi = tqc[(cp * 2 + 0) * 64 + lane];
          A0.lo = tqc[(cp * 2 + 1) * 64 + lane];
          A1.hi = tqc[(cp * 2 + 2) * 64 + lane];
          A1.lo = tqc[(cp * 2 + 3) * 64 + lane];
#pragma unroll
          for (int rb = 0; rb < kRBE; ++rb) {
            acc[rb][cp] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0.lo, Bx[rb].hi, acc[rb][cp], 0, 0, 0);
            acc[rb][cp + 1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1.lo, Bx[rb].hi, acc[rb][cp + 1], 0, 0, 0);
          }
#pragma unroll
          for (int rb = 0; rb < kRBE; ++rb) {
            acc[rb][cp] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0.hi, Bx[rb].lo, acc[rb][cp], 0, 0, 0);
            acc[rb][cp + 1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1.hi, Bx[rb].lo, acc[rb][cp + 1], 0, 0, 0);
          }
#pragma unroll
          for (int rb = 0; rb < kRBE; ++rb) {
            acc[rb][cp] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0.hi, Bx[rb].hi, acc[rb][cp], 0, 0, 0);
            acc[rb][cp + 1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1.hi, Bx[rb].hi, acc[rb][cp + 1], 0, 0, 0);
          }
        }
      } else {
        Split2h A[RB];
#pragma unroll
        for (int cb = 0; cb < RB; ++cb) {
          A[cb].hi = tqc[(cb * 2 + 0) * 64 + lane];
          A[cb].lo = tqc[(cb * 2 + 1) * 64 + lane];
        }
#pragma unroll
        for (int rb = 0; rb < kRBE; ++rb)
#pragma unroll
          for (int cb = 0; cb < RB; ++cb)
            acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[cb].lo, Bx[rb].hi, acc[rb][cb], 0, 0, 0);
#pragma unroll
        for (int rb = 0; rb < kRBE; ++rb)
#pragma unroll
          for (int cb = 0; cb < RB; ++cb)
            acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[cb].hi, Bx[rb].lo, acc[rb][cb], 0, 0, 0);
#pragma unroll
        for (int rb = 0; rb < kRBE; ++rb)
#pragma unroll
          for (int cb = 0; cb < RB; ++cb)
            acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[cb].hi, Bx[rb].hi, acc[rb][cb], 0, 0, 0);
      }
    } else {
      // no max |M| from pass A: a per-step scale per row, as in rowproj_h3_kernel
#pragma unroll
      for (int rb = 0; rb < kRBE; ++rb) {
        float m8 = max8abs(X[rb][0], X[rb][1]);
        m8 = fmaxf(m8, __shfl_xor(m8, 16, 64));
        m8 = fmaxf(m8, __shfl_xor(m8, 32, 64));
        const float sx = h3_scale(m8, invx[rb]);
        split2h(X[rb][0], X[rb][1], sx, Bx[rb]);
      }
#pragma unroll
      for (int cb = 0; cb < RB; ++cb) {
        Split2h A;
        A.hi = tqc[(cb * 2 + 0) * 64 + lane];
        A.lo = tqc[(cb * 2 + 1) * 64 + lane];
#pragma unroll
        for (int rb = 0; rb < kRBE; ++rb) {
          const f32x4 d = mfma3h(A, Bx[rb], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[rb][cb][q] = fmaf(d[q], invx[rb], acc[rb][cb][q]);
        }
      }
    }
    if (s + 1 < nsteps) wait_units(min(nxt, nsteps - 1) - (s + 1));
  }
  };
  if (fixed)
    run(std::true_type{});
  else
    run(std::false_type{});

  const float ps = (a.tinv != nullptr ? a.tinv[b] : kPSplitInv) * (fixed ? finv : 1.f);
  float* out = a.out + (static_cast<long>(b) * a.nchunk + kc) * a.out_rows * R;
#pragma unroll
  for (int rb = 0; rb < kRBE; ++rb)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb)
      *reinterpret_cast<f32x4*>(out + static_cast<long>(row_base + 16 * rb + t) * R + 16 * cb + 4 * g) =
          acc[rb][cb] * ps;
}

// ============================================================================
// host side
// ============================================================================
namespace {

int rblocks16(int r) { return (r + 15) / 16; }

int round_up(long v, long m) { return static_cast<int>((v + m - 1) / m * m); }

long ceil_div(long a, long b) { return (a + b - 1) / b; }

int validate(const DionBatchDesc* d) {
  if (d == nullptr) return fail(DION_E_INVALID, "desc is null");
  if (d->batch < 0) return fail(DION_E_INVALID, "batch=%d", d->batch);
  if (d->m <= 0 || d->n <= 0) return fail(DION_E_INVALID, "bad shape m=%d n=%d", d->m, d->n);
  if (d->r <= 0 || d->r > 128)
    return fail(DION_E_UNSUPPORTED, "rank r=%d outside 1..128", d->r);
  if (d->m_dtype != DION_DTYPE_F32 && d->m_dtype != DION_DTYPE_BF16)
    return fail(DION_E_UNSUPPORTED, "momentum dtype %d", d->m_dtype);
  if (d->w_dtype != DION_DTYPE_F32) return fail(DION_E_UNSUPPORTED, "weight dtype %d", d->w_dtype);
  if (d->g_dtype != DION_DTYPE_NONE && d->g_dtype != DION_DTYPE_F32 && d->g_dtype != DION_DTYPE_BF16)
    return fail(DION_E_UNSUPPORTED, "grad dtype %d", d->g_dtype);
  if (d->transposed != 0 && d->transposed != 1) return fail(DION_E_INVALID, "transposed=%d", d->transposed);
  return DION_OK;
}

// the distributed-RCQR pieces: P is a row shard (m_P local rows may be fewer than r)
int validate_dortho(const DionBatchDesc* d) {
  if (d == nullptr) return fail(DION_E_INVALID, "desc is null");
  if (d->batch < 0) return fail(DION_E_INVALID, "batch=%d", d->batch);
  if (d->m <= 0 || d->n <= 0) return fail(DION_E_INVALID, "bad shape m=%d n=%d", d->m, d->n);
  if (d->r <= 0 || d->r > 128) return fail(DION_E_UNSUPPORTED, "rank r=%d outside 1..128", d->r);
  if (d->transposed != 0 && d->transposed != 1) return fail(DION_E_INVALID, "transposed=%d", d->transposed);
  return DION_OK;
}

long ldv(long ld, int n) { return ld == 0 ? n : ld; }

// split-K geometry of one projection; identical in workspace sizing and launch
struct Geo {
  int gx, nchunk, kchunk, out_rows;
};

constexpr int kTargetBlocks = 2048;
// pass A's row-kernel target: 1024 against 2048 / 512 in call Q (profiles/r06/q_ab_pass_a_targets.txt:
// Llama 478.7 -> 481.2 GiB/s; qkv / proj in 2 K chunks instead of 3 / 4: fewer slab and P' bytes)
#ifndef DION_TB_PA
#define DION_TB_PA 1024
#endif
#ifndef DION_TB_PBC
#define DION_TB_PBC 512
#endif
#ifndef DION_TB_PBR
#define DION_TB_PBR 1024
#endif
#ifndef DION_TB_PAT
#define DION_TB_PAT 1024
#endif
#ifndef DION_RSL
#define DION_RSL 256
#endif
constexpr int kTbPa = DION_TB_PA, kTbPbc = DION_TB_PBC, kTbPbr = DION_TB_PBR, kTbPat = DION_TB_PAT;

// row projection: X rows x cols, reduce over cols (block_rows 128 generic, 256 fast)
Geo rowproj_geo(int rows, int cols, int batch, int block_rows = 128, int target = kTargetBlocks, int kalign = 32) {
  Geo g;
  g.gx = static_cast<int>(ceil_div(rows, block_rows));
  long want = ceil_div(target, static_cast<long>(g.gx) * (batch > 0 ? batch : 1));
  long maxc = ceil_div(cols, 256);
  long nc = want < maxc ? want : maxc;
  if (nc < 1) nc = 1;
  g.kchunk = round_up(ceil_div(cols, nc), kalign);
  g.nchunk = static_cast<int>(ceil_div(cols, g.kchunk));
  g.out_rows = rows;
  return g;
}

// transposed pass B on LDS-DMA staging (rowproj_h3gl_kernel, round 6): 1 = wherever its
// geometry fits (r = 64 / 128, rows in 32 NW-row blocks, whole 32-column steps), else
// rowproj_h3_kernel; NW waves per block (one block per CU), D staging units (LDS
// D (NW 4 KB + r 128 B); r = 128 keeps at most 3).  Measured (profiles/r06/d_*, one box,
// kernel-only): Llama fc2 group 687.7 us (register) -> D 2 647.0, D 3 617.1, D 4 670.5;
// Mixtral 1055 -> 870 us at D 3
#ifndef DION_PBR_GL
#define DION_PBR_GL 1
#endif
#ifndef DION_PBR_GL_NW
#define DION_PBR_GL_NW 8
#endif
#ifndef DION_PBR_GL_D
#define DION_PBR_GL_D 3
#endif
// target blocks of its split-K geometry: 512 (one 8-wave block per CU, two rounds) measured
// against 1024 / 2048 in call I (profiles/r06/i_ab_split_k_targets.txt): r = 128 transposed pass
// B 0.849 -> 0.808 ms per call, r = 64 equal; half the split-K slab bytes of 1024
#ifndef DION_TB_PBRGL
#define DION_TB_PBRGL 512
#endif
constexpr int kPbrGlNW = DION_PBR_GL_NW;
template <int RB>
constexpr int pbr_gl_d() { return RB >= 8 && DION_PBR_GL_D > 3 ? 3 : DION_PBR_GL_D; }
bool pbr_gl_ok(int rows, int cols, int r) {
  return DION_PBR_GL && (r == 64 || r == 128) && rows % (32 * kPbrGlNW) == 0 && cols % 32 == 0;
}
// the transposed pass B's h3 geometry (launch and workspace sizing)
Geo pbr_geo(int rows, int cols, int batch, int r);

// pass B, not transposed, on LDS-DMA staging (colproj_h3gl_kernel, round 6): 1 = at r = 128
// wherever its geometry fits (rows in 32-row steps, columns in 16 CT NW-column blocks), else
// colproj_h3_kernel; CT columns per lane, D staging units (capped by the 160 KB of LDS).
// Measured (profiles/r06/e_*): r = 128 Mixtral fc1 group 1636 -> 1518 us (kernel), 391.7 ->
// 393.8 GiB/s; r = 64 slower than the register kernel (587 vs 556-580 us), so r = 64 keeps it
#ifndef DION_PBC_GL
#define DION_PBC_GL 1
#endif
#ifndef DION_PBC_GL_CT
#define DION_PBC_GL_CT 2
#endif
#ifndef DION_PBC_GL_D
#define DION_PBC_GL_D 3
#endif
#ifndef DION_TB_PBCGL
#define DION_TB_PBCGL 512  // call I: r = 128 pass B 1.542 -> 1.506 ms per call against 1024
#endif
constexpr int kPbcGlNW = 8, kPbcGlCT = DION_PBC_GL_CT;
template <int RB>
constexpr int pbc_gl_d() {
  constexpr int unit = kPbcGlNW * 32 * 16 * kPbcGlCT * 4 + RB * 2 * 64 * 16;  // bytes per staging unit
  constexpr int most = 160 * 1024 / unit;
  return DION_PBC_GL_D < most ? DION_PBC_GL_D : most;
}
bool pbc_gl_ok(int rows, int cols, int r) {
  return DION_PBC_GL && r == 128 && rows % 32 == 0 && cols % (16 * kPbcGlCT * kPbcGlNW) == 0;
}
Geo pbc_geo(int rows, int cols, int batch, int r);

// column projection: X rows x cols, reduce over rows
Geo colproj_geo(int rows, int cols, int batch, bool panel, int kalign = 16) {
  Geo g;
  g.gx = static_cast<int>(ceil_div(cols, panel ? 64 : 256));
  long want = ceil_div(kTargetBlocks, static_cast<long>(g.gx) * (batch > 0 ? batch : 1));
  long maxc = ceil_div(rows, panel ? 512 : 256);
  long nc = want < maxc ? want : maxc;
  if (nc < 1) nc = 1;
  g.kchunk = round_up(ceil_div(rows, nc), kalign);
  g.nchunk = static_cast<int>(ceil_div(rows, g.kchunk));
  g.out_rows = cols;
  return g;
}

// colproj_x6_kernel: NW waves of 16 CT columns per block (CT = 2 for r >= 64, else 4), 32-row K-steps
constexpr int kColX6NW = 4;
Geo colx6_geo(int rows, int cols, int batch, int r) {
  Geo g;
  g.gx = static_cast<int>(ceil_div(cols, (r >= 64 ? 32 : 64) * kColX6NW));
  long want = ceil_div(kTargetBlocks, static_cast<long>(g.gx) * (batch > 0 ? batch : 1));
  long maxc = ceil_div(rows, 256);
  long nc = want < maxc ? want : maxc;
  if (nc < 1) nc = 1;
  g.kchunk = round_up(ceil_div(rows, nc), 32);
  g.nchunk = static_cast<int>(ceil_div(rows, g.kchunk));
  g.out_rows = cols;
  return g;
}

bool rowproj_fast_ok(int rows, int cols, int r) { return rows % (64 * kRB) == 0 && cols % 32 == 0 && r % 16 == 0 && r <= 128 && r != 48 && r != 80 && r != 96 && r != 112; }
bool colproj_fast_ok(int rows, int cols, int r) { return cols % 256 == 0 && rows % 16 == 0 && r % 16 == 0 && r <= 128 && r != 48 && r != 80 && r != 96 && r != 112; }

// rank_stream_kernel: rows (or columns) one block streams, waves per block, X tiles in flight
// (measured fastest of (NW, D) in {4, 8} x {2, 3} on the Llama set, round 2)
constexpr int kRankStreamLen = DION_RSL;
// r > 64: rows per update block (DION_RSL128, a dev build option): Mixtral 376.0-376.5 -> 381.0-382.0
// GiB/s against 256 (profiles/r05/ac_rsl128.txt)
#ifndef DION_RSL128
#define DION_RSL128 512
#endif
constexpr int kRankNW = 8;
constexpr int kRankD = 2;
// r = 128 (RU 8): one X tile in flight -- 135 VGPRs, 3 waves per SIMD, against D 2's 202 at 2.
// Measured on the Mixtral set 5050 -> 5332 GB/s; at r = 64 D 1 (102 VGPRs, 4 per SIMD) is
// slower, 5970 -> 5716
constexpr int kRankD8 = 1;

// pre-split thin operand of the x6 projections (rows = the contraction index)
size_t thin_presplit_bytes(int rows, int r, int batch) { return static_cast<size_t>(rows) * r * 6 * batch + 1024; }

// pass B through the fp16x3 column kernel (colproj_h3_kernel) instead of bf16x6 (measured default)
constexpr int kPbH3 = 1;
// pass B, transposed, through the fp16x3 row kernel (rowproj_h3_kernel) instead of bf16x6 (measured default)
constexpr int kPbH3r = 1;
// waves per block of rowproj_h3_kernel: one LDS copy of the step's P split serves 32 NW rows
// of M (measured default)
constexpr int kPbRNW = 4;
// columns per lane of colproj_h3_kernel (2: 8-byte loads, 4: 16-byte loads)
constexpr int kColH3CT = 4;
// r > 64 (RB = 8) keeps 2 columns per lane: 4 would need 256+ VGPRs (one wave per SIMD)
constexpr int colh3_ct(int r) { return r > 64 ? 2 : kColH3CT; }
Geo pbr_geo(int rows, int cols, int batch, int r) {
  return pbr_gl_ok(rows, cols, r) ? rowproj_geo(rows, cols, batch, 32 * kPbrGlNW, DION_TB_PBRGL)
                                  : rowproj_geo(rows, cols, batch, 16 * kRBE * kPbRNW, kTbPbr);
}
bool colh3_ok(int rows, int cols, int r) {
  return kPbH3 && rows % 32 == 0 && cols % (16 * colh3_ct(r) * kColX6NW) == 0;
}
Geo colh3_geo(int rows, int cols, int batch, int r) {
  if (pbc_gl_ok(rows, cols, r)) return pbc_geo(rows, cols, batch, r);
  Geo g;
  g.gx = static_cast<int>(ceil_div(cols, 16 * colh3_ct(r) * kColX6NW));
  long want = ceil_div(kTbPbc, static_cast<long>(g.gx) * (batch > 0 ? batch : 1));
  long maxc = ceil_div(rows, 256);
  long nc = want < maxc ? want : maxc;
  if (nc < 1) nc = 1;
  g.kchunk = round_up(ceil_div(rows, nc), 32);
  g.nchunk = static_cast<int>(ceil_div(rows, g.kchunk));
  g.out_rows = cols;
  return g;
}

Geo pbc_geo(int rows, int cols, int batch, int r) {
  (void)r;
  Geo g;
  g.gx = static_cast<int>(ceil_div(cols, 16 * kPbcGlCT * kPbcGlNW));
  long want = ceil_div(DION_TB_PBCGL, static_cast<long>(g.gx) * (batch > 0 ? batch : 1));
  long maxc = ceil_div(rows, 256);
  long nc = want < maxc ? want : maxc;
  if (nc < 1) nc = 1;
  g.kchunk = round_up(ceil_div(rows, nc), 32);
  g.nchunk = static_cast<int>(ceil_div(rows, g.kchunk));
  g.out_rows = cols;
  return g;
}

// pre-split streamed factor P (m_P x r per matrix) of the rank-update kernels
// host twin of h3_scale: the power of two s with amax s in [2^14, 2^15) (1 for amax 0 or
// not finite)
float h3_scale_host(float amax) {
  if (!(amax > 0.f) || !isfinite(amax)) return 1.f;
  int e = 0;
  frexpf(amax, &e);  // amax = m 2^e, m in [0.5, 1)
  int k = 15 - e;
  k = k < -126 ? -126 : (k > 126 ? 126 : k);
  return ldexpf(1.f, k);
}

// the weight update's rank_stream_kernel on h3 products (3 fp16 MFMAs per product instead
// of bf16x6's 6)
constexpr bool kRankH3 = (1) != 0;


// two pre-split operand buffers (Q and R', n_Q x r each) of dion_project_p_ef, after the slabs
size_t presplit_stride(int nq, int r) { return static_cast<size_t>(nq) * r * 3 / 8; }  // uint4 per matrix
size_t presplit_bytes(int nq, int r, int batch) { return 2 * 16 * presplit_stride(nq, r) * batch + 256; }

// deferred-EF pass A (rowproj_ef_kernel / colproj_ef_kernel)
// rows per block of the fused pass A row kernel (r = 128 may run 16-row waves)
int pa_row_block(int r) { return r > 64 ? 16 * kKR8 * kNW8 : 16 * kPaKR * kPaNW; }

bool proj_ef_ok(int m, int n, int r, bool transposed) {
  // r = 128 (the Mixtral config) only through the h3 kernels
  if (r != 32 && r != 64 && r != 128) return false;
  return transposed ? (n % 128 == 0 && m % 32 == 0) : (m % pa_row_block(r) == 0 && n % 32 == 0);
}

Geo proj_ef_geo(int m, int n, int batch, bool transposed, int r) {
  // r = 128: K chunks on 64-column bounds (rowproj_efgl_kernel's G step pairs are whole lines)
  if (!transposed) return rowproj_geo(m, n, batch, pa_row_block(r), kTbPa, r > 64 && kPaGlGpair ? 64 : 32);
  Geo g;
  g.gx = static_cast<int>(ceil_div(n, 128));
  long want = ceil_div(kTbPat, static_cast<long>(g.gx) * (batch > 0 ? batch : 1));
  long maxc = ceil_div(m, 256);
  long nc = want < maxc ? want : maxc;
  if (nc < 1) nc = 1;
  g.kchunk = round_up(ceil_div(m, nc), 32);
  g.nchunk = static_cast<int>(ceil_div(m, g.kchunk));
  g.out_rows = n;
  return g;
}

size_t slab_bytes(const Geo& g, int batch, int r) {
  return g.nchunk > 1 ? sizeof(float) * static_cast<size_t>(batch) * g.nchunk * g.out_rows * r : 0;
}

int sketch_k(int r, float oversample) {
  return static_cast<int>(ceil(static_cast<double>(oversample) * r / 128.0)) * 128;
}

// sketch_rad_kernel: ~512 blocks over the batch (2 per CU), 32-row aligned row chunks
Geo sketch_rad_geo(int mp, int K, int batch) {
  Geo g;
  const long want = ceil_div(512L, batch > 0 ? batch : 1);
  const long maxc = ceil_div(mp, 256);
  long nc = want < maxc ? want : maxc;
  if (nc < 1) nc = 1;
  g.kchunk = round_up(ceil_div(mp, nc), 32);
  g.nchunk = static_cast<int>(ceil_div(mp, g.kchunk));
  g.gx = g.nchunk;
  g.out_rows = K;
  return g;
}

// the orthonormalisation's Gram on gram_h3_kernel (r = 64 or 128, m_P % 32 == 0) instead of
// the fp32 panel kernel
constexpr int kGramH3 = 1;
bool gram_h3_ok(int mp, int r) { return kGramH3 && (r == 64 || r == 128) && mp % 32 == 0; }
// ~512 blocks over the batch (2 per CU), 32-row aligned chunks of >= 128 rows
Geo gram_geo(int mp, int r, int batch) {
  Geo g;
  const long want = ceil_div(512L, batch > 0 ? batch : 1);
  const long maxc = ceil_div(mp, 128);
  long nc = want < maxc ? want : maxc;
  if (nc < 1) nc = 1;
  g.kchunk = round_up(ceil_div(mp, nc), 32);
  g.nchunk = static_cast<int>(ceil_div(mp, g.kchunk));
  g.gx = g.nchunk;
  g.out_rows = r;
  return g;
}

// the padded order of trsm_right_kernel and its factor layout (rt x rt + rt floats per matrix)
int trsm_rt(int r) { return r <= 32 ? 32 : (r <= 64 ? 64 : 128); }
size_t factor_floats(int r) { return static_cast<size_t>(trsm_rt(r)) * (trsm_rt(r) + 1); }

struct OrthoPlan {
  bool plain_qr;
  int k;
  Geo sk, gr;
  size_t off_sk_slab, off_sp, off_r1, off_gslab, off_g, off_r2, off_inv, off_p1, total;
};

// the orthonormalisation's two solves as GEMMs with the explicit inverses (tri_inv_kernel +
// tsolve_mfma_kernel) for r = 32, 64, 128; 0 (a dev build option) keeps the substitution
// kernels.  Same-box Llama 460.6 / 449.8 -> 465.8 / 455.2 GiB/s, Mixtral 350.0 -> 352.3 with the
// inverses from the factor kernels (profiles/r05/m_solves_gemm_ab.txt); the solves alone beside a streaming copy:
// r = 64 8.4 vs 33.7 us marginal per fc1 group, r = 128 41.2 vs 105.9 (scripts/ubench/trsm_conc.hip)
#ifndef DION_TSOLVE_GEMM
#define DION_TSOLVE_GEMM 1
#endif
bool tsolve_gemm_ok(int mp, int r) { return DION_TSOLVE_GEMM && (r == 32 || r == 64 || r == 128) && mp > r; }

// the first GEMM solve summing the Gram of its output (tsolve_mfma_kernel GRAM, r <= 64): off.
// Alone it beats solve + gram_h3_kernel (58.3 vs 39.6 + 27.1 us per Llama group, one stream), in
// the two-stream step it loses (Llama 469.5 / 469.2 -> 464.9 / 466.8 GiB/s, same box,
// profiles/r05/r_tsolve_gram.txt): its persistent blocks hold 50 KB of LDS each for the whole
// solve, beside the other stream's streaming kernel.
constexpr bool kTsolveGram = false;
// persistent blocks of the first solve + Gram per matrix
int tgram_chunks(int mp, int batch) {
  const long steps = ceil_div(mp, 64 * kTgWavesImg);
  const long want = ceil_div(1024L, batch > 0 ? batch : 1);
  return static_cast<int>(steps < want ? steps : want);
}

OrthoPlan ortho_plan(int mp, int r, int batch, float oversample) {
  OrthoPlan p{};
  p.plain_qr = (mp <= r);
  p.k = sketch_k(r, oversample);
  if (p.plain_qr) return p;
  p.sk = colproj_geo(mp, p.k, batch, true);
  p.gr = gram_h3_ok(mp, r) ? gram_geo(mp, r, batch) : colproj_geo(mp, r, batch, true);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += (bytes + 255) / 256 * 256;
    return o;
  };
  const Geo rad = sketch_rad_geo(mp, p.k, batch);
  const size_t rad_slab = rad.nchunk > 1 ? sizeof(float) * static_cast<size_t>(batch) * rad.nchunk * p.k * r : 0;
  p.off_sk_slab = take(std::max(slab_bytes(p.sk, batch, r), rad_slab));
  p.off_sp = take(sizeof(float) * static_cast<size_t>(batch) * p.k * r);
  p.off_r1 = take(sizeof(float) * static_cast<size_t>(batch) * r * r);
  p.off_gslab = take(std::max(slab_bytes(p.gr, batch, r),
                              kTsolveGram && tsolve_gemm_ok(mp, r) && r <= 64
                                  ? sizeof(float) * static_cast<size_t>(batch) * tgram_chunks(mp, batch) * r * r
                                  : size_t(0)));
  p.off_g = take(sizeof(float) * static_cast<size_t>(batch) * r * r);
  p.off_r2 = take(sizeof(float) * static_cast<size_t>(batch) * r * r);
  p.off_inv = take(sizeof(float) * static_cast<size_t>(batch) * std::max(static_cast<size_t>(r) * r, factor_floats(r)));
  p.off_p1 = take(sizeof(float) * static_cast<size_t>(batch) * mp * r);
  p.total = off;
  return p;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// P <- z ? 0 : nan_to_num(P) over batch entries of per_entry values (kernels.py:185-188)
int launch_pfix(float* P, const uint32_t* nonzero, long per_entry, int batch, hipStream_t st) {
  long blocks = ceil_div(per_entry * batch, 256);
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) return DION_OK;
  hipLaunchKernelGGL(pfix_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, st, P, nonzero, per_entry, batch);
  return check_launch("pfix");
}

// The final solve of the orthonormalisation writes pass B's fp16x3 split of P (fixed scale,
// trsm_lds_kernel<..., true>) when pass B runs its h3 kernels on this shape: fp32 state, r = 32
// or 64, m_P > r (the Cholesky QR path), m_P a multiple of 32, and run_projection's h3 shape
// conditions for the orientation (the layout / ld / alignment conditions are checked per call:
// a pass B that cannot use the split ignores it).
// r = 128 (round 6): the final solve has no LDS row image there, so the split is one
// fixed-scale presplit16_kernel launch after it (launch_psplit_fixed), which still spares pass
// B its absmax and measured-scale split.
bool psplit_ok(const DionBatchDesc* d) {
  if (d->m_dtype != DION_DTYPE_F32 || !(d->r == 32 || d->r == 64 || d->r == 128)) return false;
  const bool tr = d->transposed != 0;
  const int mp = tr ? d->n : d->m;
  if (mp <= d->r || mp % 32 != 0) return false;
  if (tr) return kPbH3r && rowproj_fast_ok(d->m, d->n, d->r) && d->m % (16 * kRBE * kPbRNW) == 0;
  return colproj_fast_ok(d->m, d->n, d->r) && colh3_ok(d->m, d->n, d->r);
}

// pass B's fp16x3 split of nb orthonormal P_b (m_P x r, contiguous from P) on the fixed scale
// 2^14 into `out` (layout 0, pass B's kmap), with the fix-up of P in place first when `fix` is
// given (presplit16_kernel with amax = null)
int launch_psplit_fixed(float* P, int mp, int r, int nb, const uint32_t* fix, f16x8* out, int kmap,
                        hipStream_t st) {
  Presplit16Args pa;
  memset(&pa, 0, sizeof(pa));
  for (int b = 0; b < nb; ++b) pa.src[b] = P + static_cast<long>(b) * mp * r;
  pa.dst = out;
  pa.stride = static_cast<long>(mp) * r / 4;
  pa.rows = mp;
  pa.r = r;
  pa.kmap = kmap;
  pa.layout = 0;
  pa.fix = fix;
  const dim3 pgrid(static_cast<unsigned>(ceil_div(static_cast<long>(mp) * r / 8, 256)), nb);
  hipLaunchKernelGGL(presplit16_kernel, pgrid, dim3(256), 0, st, pa);
  return check_launch("presplit16(fixed)");
}

// the fix-up partials of dion_project_r_fixup at the end of the pass-B workspace
size_t fix_part_bytes(int nq, int r, int batch) {
  return (sizeof(float) * static_cast<size_t>(batch) * ceil_div(nq, kFixRows) * r + 255) / 256 * 256;
}

// one absmax_kernel launch over `groups` groups of nb matrices (AbsMaxArgs order)
void launch_absmax(AbsMaxArgs& ma, int groups, hipStream_t st) {
  long most = 0;
  bool vec = true;
  for (int k = 0; k < groups; ++k) {
    most = ma.count[k] > most ? ma.count[k] : most;
    vec = vec && ma.count[k] % 4 == 0;
    for (int b = 0; b < ma.nb; ++b) vec = vec && (ma.src[k * ma.nb + b] == nullptr || aligned16(ma.src[k * ma.nb + b]));
  }
  ma.vec = vec ? 1 : 0;
  long bx = ceil_div(most, 256L * 16);  // >= 4 16-byte loads per thread, <= 32 blocks per matrix
  bx = bx < 1 ? 1 : (bx > 32 ? 32 : bx);
  hipLaunchKernelGGL(absmax_kernel, dim3(static_cast<unsigned>(bx), groups * ma.nb), dim3(256), 0, st, ma);
}


template <class F>
int dispatch_rb(int r, F&& f) {
  switch (rblocks16(r)) {
    case 1: return f(std::integral_constant<int, 1>{});
    case 2: return f(std::integral_constant<int, 2>{});
    case 3:
    case 4: return f(std::integral_constant<int, 4>{});
    case 5: case 6: case 7: case 8: return f(std::integral_constant<int, 8>{});
  }
  return fail(DION_E_UNSUPPORTED, "rank %d", r);
}

template <class F>
int dispatch_gdt(int gdt, F&& f) {
  switch (gdt) {
    case DION_DTYPE_NONE: return f(std::integral_constant<int, DION_DTYPE_NONE>{});
    case DION_DTYPE_F32: return f(std::integral_constant<int, DION_DTYPE_F32>{});
    case DION_DTYPE_BF16: return f(std::integral_constant<int, DION_DTYPE_BF16>{});
  }
  return fail(DION_E_UNSUPPORTED, "grad dtype %d", gdt);
}

int launch_reduce(float* out, const float* slab, int nchunk, long per_entry, int batch, hipStream_t st) {
  long total = per_entry * batch;
  long blocks = ceil_div(total, 256);
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(reduce_slabs_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, st, out, slab,
                     nchunk, per_entry, batch);
  return check_launch("reduce_slabs");
}

// One projection over up to MAXB matrices.  `row_mode`: reduce over columns.
int run_projection(bool row_mode, int rows, int cols, int r, int batch, const void* const* G, float* const* M,
                   const float* const* thin, long ld_m, long ld_g, int gdt, float* out, uint32_t* nonzero,
                   void* ws, size_t ws_bytes, hipStream_t st, const uint32_t* mabs = nullptr,
                   const f16x8* thin_split = nullptr, const FixArgs* fix = nullptr) {
  bool fast = row_mode ? rowproj_fast_ok(rows, cols, r) : colproj_fast_ok(rows, cols, r);
  fast = fast && (ld_m % 8) == 0 && (gdt == DION_DTYPE_NONE || (ld_g % 8) == 0);
  for (int b = 0; b < batch && fast; ++b)
    fast = aligned16(M[b]) && aligned16(thin[b]) && (gdt == DION_DTYPE_NONE || aligned16(G[b]));
  // no gradient (pass B): split-bf16 MFMA kernels (the column one steps 32 rows)
  const bool x6 = fast && gdt == DION_DTYPE_NONE &&
                  (row_mode ? rows % (64 * kRBE) == 0
                            : (rows % 32 == 0 && cols % ((r >= 64 ? 32 : 64) * kColX6NW) == 0));
  const bool h3 = fast && gdt == DION_DTYPE_NONE &&
                  (row_mode ? (kPbH3r && rows % (16 * kRBE * kPbRNW) == 0) : colh3_ok(rows, cols, r));
  const Geo geo = row_mode ? (h3 ? pbr_geo(rows, cols, batch, r)
                                : rowproj_geo(rows, cols, batch, x6 ? 64 * kRBE : (fast ? 64 * kRB : 128), kTargetBlocks))
                 : h3      ? colh3_geo(rows, cols, batch, r)
                 : x6      ? colx6_geo(rows, cols, batch, r)
                           : colproj_geo(rows, cols, batch, false);
  const size_t slab = (slab_bytes(geo, batch, r) + 255) / 256 * 256;
  const int thin_rows = row_mode ? cols : rows;  // the contraction index
  const size_t need = slab + ((x6 || h3) ? thin_presplit_bytes(thin_rows, r, batch) : 0);
  if (need > ws_bytes || (need > 0 && ws == nullptr))
    return fail(DION_E_WORKSPACE, "projection needs %zu workspace bytes, got %zu", need, ws_bytes);
  ProjArgs a;
  memset(&a, 0, sizeof(a));
  if (h3 && thin_split != nullptr) {
    // the final solve of the orthonormalisation already wrote P's limbs (fixed scale)
    a.tsplit = thin_split;
    a.ts_stride = static_cast<long>(thin_rows) * r / 8 * 2;
    a.tinv = nullptr;
  } else if (h3) {
    // fp16x3: the thin operand's per-matrix |max|, then its two fp16 limbs
    char* base = static_cast<char*>(ws) + slab;
    const long per = static_cast<long>(thin_rows) * r;
    const size_t sbytes = (static_cast<size_t>(per) * 4 * batch + 255) / 256 * 256;
    uint32_t* amax = reinterpret_cast<uint32_t*>(base + sbytes);
    float* inv = reinterpret_cast<float*>(base + sbytes + 256);
    hipError_t me = hipMemsetAsync(amax, 0, sizeof(uint32_t) * batch, st);
    if (me != hipSuccess) return fail(DION_E_LAUNCH, "memset: %s", hipGetErrorString(me));
    AbsMaxArgs ma;
    memset(&ma, 0, sizeof(ma));
    for (int b = 0; b < batch; ++b) ma.src[b] = thin[b];
    ma.out = amax;
    ma.count[0] = per;
    ma.nb = batch;
    launch_absmax(ma, 1, st);
    Presplit16Args pa;
    memset(&pa, 0, sizeof(pa));
    for (int b = 0; b < batch; ++b) pa.src[b] = thin[b];
    pa.dst = reinterpret_cast<f16x8*>(base);
    pa.amax = amax;
    pa.inv_scale = inv;
    pa.stride = per / 8 * 2;
    pa.rows = thin_rows;
    pa.r = r;
    pa.kmap = row_mode ? 1 : 0;  // rowproj_h3 steps columns 16c + 4g (KMAP 1), colproj_h3 rows 8g + e
    pa.layout = 0;
    const dim3 pgrid(static_cast<unsigned>(ceil_div(per / 8, 256)), batch);
    hipLaunchKernelGGL(presplit16_kernel, pgrid, dim3(256), 0, st, pa);
    int rc = check_launch("presplit16(thin)");
    if (rc != DION_OK) return rc;
    a.tsplit = pa.dst;
    a.ts_stride = pa.stride;
    a.tinv = inv;
  } else if (x6) {
    // the thin operand split into bf16 limbs once per call, in the MFMA B-operand layout
    PresplitArgs pa;
    memset(&pa, 0, sizeof(pa));
    for (int b = 0; b < batch; ++b) pa.src[b] = thin[b];
    pa.dst = reinterpret_cast<u32x4*>(static_cast<char*>(ws) + slab);
    pa.stride = static_cast<long>(thin_rows) * r * 3 / 8;
    pa.rows = thin_rows;
    pa.r = r;
    pa.layout = 0;
    pa.kmap = row_mode ? 1 : 0;  // rowproj_x6 loads columns 16c + 4g (KMAP 1), colproj_x6 rows 8g + e
    const dim3 pgrid(static_cast<unsigned>(ceil_div(static_cast<long>(thin_rows) * r / 8, 256)), batch);
    hipLaunchKernelGGL(presplit_kernel, pgrid, dim3(256), 0, st, pa);
    int rc = check_launch("presplit(thin)");
    if (rc != DION_OK) return rc;
    a.tsplit = pa.dst;
    a.ts_stride = pa.stride;
  }
  bool vec = (ld_m % 4) == 0 && (gdt == DION_DTYPE_NONE || (ld_g % (gdt == DION_DTYPE_BF16 ? 8 : 4)) == 0);
  for (int b = 0; b < batch; ++b) {
    a.g[b] = G ? G[b] : nullptr;
    a.m[b] = M[b];
    a.thin[b] = thin[b];
    if (M[b] == nullptr || thin[b] == nullptr || (gdt != DION_DTYPE_NONE && G[b] == nullptr))
      return fail(DION_E_INVALID, "null matrix pointer at entry %d", b);
    vec = vec && aligned16(M[b]) && (gdt == DION_DTYPE_NONE || aligned16(G[b]));
  }
  a.out = geo.nchunk > 1 ? static_cast<float*>(ws) : out;
  a.nonzero = nonzero;
  a.mabs = mabs;
  a.rows = rows;
  a.cols = cols;
  a.r = r;
  a.ld_m = ld_m;
  a.ld_g = ld_g;
  a.kchunk = geo.kchunk;
  a.nchunk = geo.nchunk;
  a.out_rows = geo.out_rows;
  a.vec = vec ? 1 : 0;
  const dim3 grid(geo.gx, geo.nchunk, batch);
  int rc = dispatch_rb(r, [&](auto RBc) {
    constexpr int RB = decltype(RBc)::value;
    return dispatch_gdt(gdt, [&](auto Gc) {
      constexpr int GD = decltype(Gc)::value;
      if (h3 && row_mode) {
        if constexpr (RB == 4 || RB == 8) {
          if (pbr_gl_ok(rows, cols, r)) {
            hipLaunchKernelGGL((rowproj_h3gl_kernel<RB, kPbrGlNW, pbr_gl_d<RB>()>), grid, dim3(64 * kPbrGlNW), 0, st, a);
            return check_launch("rowproj_h3gl");
          }
        }
        hipLaunchKernelGGL((rowproj_h3_kernel<RB, kPbRNW>), grid, dim3(64 * kPbRNW), 0, st, a);
      }
      else if (h3) {
        if constexpr (RB == 4 || RB == 8) {
          if (pbc_gl_ok(rows, cols, r)) {
            hipLaunchKernelGGL((colproj_h3gl_kernel<RB, kPbcGlNW, kPbcGlCT, pbc_gl_d<RB>()>), grid, dim3(64 * kPbcGlNW), 0,
                               st, a);
            return check_launch("colproj_h3gl");
          }
        }
        hipLaunchKernelGGL((colproj_h3_kernel<RB, kColX6NW, colh3_ct(16 * RB)>), grid, dim3(64 * kColX6NW), 0, st, a);
      }
      else if (x6)
        hipLaunchKernelGGL((colproj_x6_kernel<RB, kColX6NW>), grid, dim3(64 * kColX6NW), 0, st, a);
      else if (fast && row_mode)
        hipLaunchKernelGGL((rowproj_fast_kernel<RB, GD>), grid, dim3(256), 0, st, a);
      else if (fast)
        hipLaunchKernelGGL((colproj_fast_kernel<RB, GD>), grid, dim3(256), 0, st, a);
      else if (row_mode)
        hipLaunchKernelGGL((rowproj_kernel<RB, GD>), grid, dim3(256), 0, st, a);
      else
        hipLaunchKernelGGL((colproj_kernel<RB, GD, 0, 0>), grid, dim3(256), 0, st, a);
      return check_launch(row_mode ? "rowproj" : "colproj");
    });
  });
  if (rc != DION_OK) return rc;
  if (fix != nullptr) {
    // dion_project_r_fixup: the fix-up's first phase rides on the split-K reduction
    if (geo.nchunk > 1)
      hipLaunchKernelGGL(reduce_fix_partial_kernel, dim3(fix->nchunk, batch), dim3(256), 0, st, *fix,
                         static_cast<const float*>(ws), geo.nchunk);
    else
      hipLaunchKernelGGL(fixup_partial_kernel, dim3(fix->nchunk, batch), dim3(256), 0, st, *fix);
    rc = check_launch("fixup_partial(pass B)");
    if (rc != DION_OK) return rc;
    hipLaunchKernelGGL(colnorm_apply_kernel, dim3(fix->nchunk, batch), dim3(256), 0, st, *fix);
    return check_launch("fixup_colnorm(pass B)");
  }
  if (geo.nchunk > 1)
    return launch_reduce(out, static_cast<const float*>(ws), geo.nchunk, static_cast<long>(geo.out_rows) * r, batch, st);
  return DION_OK;
}

// panel reduction over the rows of P: out[b] (cols x r) = X_b^T P_b
int run_panel(int xmode, int mp, int cols, int r, int batch, const float* P, const float* sketch, uint64_t seed,
              float std_, float* out, void* slab, const Geo& geo, hipStream_t st, long sketch_row0 = 0) {
  ProjArgs a;
  memset(&a, 0, sizeof(a));
  a.sketch_row0 = sketch_row0;
  for (int b = 0; b < batch; ++b) {
    a.thin[b] = P + static_cast<long>(b) * mp * r;
    a.m[b] = const_cast<float*>(P + static_cast<long>(b) * mp * r);
  }
  a.out = geo.nchunk > 1 ? static_cast<float*>(slab) : out;
  a.sketch = sketch;
  a.seed = seed;
  a.sketch_std = std_;
  a.rows = mp;
  a.cols = cols;
  a.r = r;
  a.ld_m = r;
  a.ld_g = 0;
  a.kchunk = geo.kchunk;
  a.nchunk = geo.nchunk;
  a.out_rows = geo.out_rows;
  a.vec = ((r % 4) == 0 && aligned16(P)) ? 1 : 0;
  const dim3 grid(geo.gx, geo.nchunk, batch);
  int rc = dispatch_rb(r, [&](auto RBc) {
    constexpr int RB = decltype(RBc)::value;
    if (xmode == 0)
      hipLaunchKernelGGL((colproj_kernel<RB, DION_DTYPE_NONE, 0, 1>), grid, dim3(256), 0, st, a);
    else if (xmode == 1)
      hipLaunchKernelGGL((colproj_kernel<RB, DION_DTYPE_NONE, 1, 1>), grid, dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((colproj_kernel<RB, DION_DTYPE_NONE, 2, 1>), grid, dim3(256), 0, st, a);
    return check_launch("panel colproj");
  });
  if (rc != DION_OK) return rc;
  if (geo.nchunk > 1)
    return launch_reduce(out, static_cast<const float*>(slab), geo.nchunk, static_cast<long>(cols) * r, batch, st);
  return DION_OK;
}

// kernels that take more than the default 64 KiB of dynamic LDS must opt in
template <class K>
int allow_lds(K kernel, size_t bytes) {
  if (bytes <= 64 * 1024) return DION_OK;
  if (bytes > 160 * 1024) return fail(DION_E_UNSUPPORTED, "kernel needs %zu bytes of LDS (> 160 KiB)", bytes);
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(bytes));
  if (e != hipSuccess) return fail(DION_E_LAUNCH, "hipFuncSetAttribute(%zu): %s", bytes, hipGetErrorString(e));
  return DION_OK;
}

// inv: R^-1 (r x r, the distributed RCQR's exchange format); else the padded factor for
// trsm_right_kernel (factor_floats(r) per matrix)
int launch_sketch_qr_inv(const float* SP, float* Rinv, int K, int r, int batch, hipStream_t st, bool inv = true,
                         bool tinv = false) {
  if (K > 256 || r > 128 || r > K) return fail(DION_E_UNSUPPORTED, "sketch QR %dx%d", K, r);
  const bool dbl = r <= 64;
  const size_t base_lds = ((sizeof(float) * (520 + static_cast<size_t>(r) * (r + 1)) + 15) / 16) * 16;
  const size_t lds = base_lds + std::max((dbl ? sizeof(double) : sizeof(float)) * static_cast<size_t>(r) * r,
                                         tinv ? sizeof(float) * static_cast<size_t>(r) * (r + 8) : size_t(0));
  auto go = [&](auto RPLc, auto CPWc, auto XTc) {
    constexpr int RPLv = decltype(RPLc)::value;
    constexpr int CPWv = decltype(CPWc)::value;
    using XTv = typename decltype(XTc)::type;
    if (tinv) {
      // the fp32 inverse fused after the QR (the GEMM solves): 8 lanes per column, r = 8 NWQ
      constexpr int NWQ = CPWv >= 32 ? 16 : (CPWv >= 16 ? 8 : 4);
      constexpr int CPWq = CPWv * 4 / NWQ;
      if (r * 8 != 64 * NWQ) return fail(DION_E_UNSUPPORTED, "fused sketch-QR inverse at r=%d", r);
      int rc = allow_lds(sketch_qr_inv_kernel<RPLv, CPWq, XTv, false, NWQ, true>, lds);
      if (rc != DION_OK) return rc;
      hipLaunchKernelGGL((sketch_qr_inv_kernel<RPLv, CPWq, XTv, false, NWQ, true>), dim3(batch), dim3(64 * NWQ), lds,
                         st, SP, Rinv, K, r, 0);
      return check_launch("sketch_qr(inverse)");
    }
    if (!inv) {
      // more waves per matrix where each wave keeps >= 8 columns (the column arithmetic and
      // its reductions are the same whichever wave owns the column: bitwise the same factor;
      // K 128 / r 64: 62.0 -> 51.1 us, K 256 / r 128: 233.2 -> 166.9 us per 16 matrices,
      // scripts/ubench/qr_ab.hip, profiles/r05/o_qr_tri_inv.txt)
      constexpr int NWQ = CPWv >= 32 ? 16 : (CPWv >= 16 ? 8 : 4);
      constexpr int CPWq = CPWv * 4 / NWQ;
      int rc = allow_lds(sketch_qr_inv_kernel<RPLv, CPWq, XTv, false, NWQ>, lds);
      if (rc != DION_OK) return rc;
      hipLaunchKernelGGL((sketch_qr_inv_kernel<RPLv, CPWq, XTv, false, NWQ>), dim3(batch), dim3(64 * NWQ), lds, st, SP,
                         Rinv, K, r, trsm_rt(r));
      return check_launch("sketch_qr");
    }
    int rc = allow_lds(sketch_qr_inv_kernel<RPLv, CPWv, XTv>, lds);
    if (rc != DION_OK) return rc;
    hipLaunchKernelGGL((sketch_qr_inv_kernel<RPLv, CPWv, XTv>), dim3(batch), dim3(256), lds, st, SP, Rinv, K, r, 0);
    return check_launch("sketch_qr_inv");
  };
  struct D { using type = double; };
  struct F { using type = float; };
  if (K <= 128) {
    if (r <= 16) return go(std::integral_constant<int, 2>{}, std::integral_constant<int, 4>{}, D{});
    if (r <= 32) return go(std::integral_constant<int, 2>{}, std::integral_constant<int, 8>{}, D{});
    if (r <= 64) return go(std::integral_constant<int, 2>{}, std::integral_constant<int, 16>{}, D{});
    return go(std::integral_constant<int, 2>{}, std::integral_constant<int, 32>{}, F{});
  }
  if (r <= 64) return go(std::integral_constant<int, 4>{}, std::integral_constant<int, 16>{}, D{});
  return go(std::integral_constant<int, 4>{}, std::integral_constant<int, 32>{}, F{});
}

int launch_chol_inv(const float* G, float* Uinv, int r, int batch, hipStream_t st, bool inv = true,
                    bool tinv = false) {
  if (tinv) {
    // the GEMM solves: Cholesky + fp32 inverse in one launch (r = RP only)
    switch (r) {
      case 32: hipLaunchKernelGGL((chol_reg_kernel<32, 256, true>), dim3(batch), dim3(256), 0, st, G, Uinv, r); break;
      case 64: hipLaunchKernelGGL((chol_reg_kernel<64, 512, true>), dim3(batch), dim3(512), 0, st, G, Uinv, r); break;
      case 128: hipLaunchKernelGGL((chol_reg_kernel<128, 1024, true>), dim3(batch), dim3(1024), 0, st, G, Uinv, r); break;
      default: return fail(DION_E_UNSUPPORTED, "fused Cholesky inverse at r=%d", r);
    }
    return check_launch("chol(inverse)");
  }
  const bool dbl = r <= 96;
  const size_t lds = ((sizeof(float) * (static_cast<size_t>(r) * (r + 1) + r + 4) + 15) / 16) * 16 +
                     (dbl ? sizeof(double) : sizeof(float)) * static_cast<size_t>(r) * r;
  const int threads = 256;
  if (!inv) {
    switch (trsm_rt(r)) {
      case 32: hipLaunchKernelGGL((chol_reg_kernel<32>), dim3(batch), dim3(256), 0, st, G, Uinv, r); break;
      // 512 threads: 39.8 vs 53.0 us per 16-matrix launch, bitwise the same (scripts/ubench/chol_ab.hip)
      case 64: hipLaunchKernelGGL((chol_reg_kernel<64, 512>), dim3(batch), dim3(512), 0, st, G, Uinv, r); break;
      default: hipLaunchKernelGGL((chol_reg_kernel<128, 1024>), dim3(batch), dim3(1024), 0, st, G, Uinv, r); break;
    }
    return check_launch("chol");
  }
  if (dbl) {
    int rc = allow_lds(chol_inv_kernel<double>, lds);
    if (rc != DION_OK) return rc;
    hipLaunchKernelGGL((chol_inv_kernel<double>), dim3(batch), dim3(threads), lds, st, G, Uinv, r, 0);
  } else {
    int rc = allow_lds(chol_inv_kernel<float>, lds);
    if (rc != DION_OK) return rc;
    hipLaunchKernelGGL((chol_inv_kernel<float>), dim3(batch), dim3(threads), lds, st, G, Uinv, r, 0);
  }
  return check_launch("chol_inv");
}


int launch_tri_inv(const float* F, float* T, int r, int batch, hipStream_t st) {
  switch (r) {
    case 32: hipLaunchKernelGGL((tri_inv_kernel<32>), dim3(batch), dim3(32 * tri_inv_tip<32>()), 0, st, F, T); break;
    case 64: hipLaunchKernelGGL((tri_inv_kernel<64>), dim3(batch), dim3(64 * tri_inv_tip<64>()), 0, st, F, T); break;
    case 128: hipLaunchKernelGGL((tri_inv_kernel<128>), dim3(batch), dim3(128 * tri_inv_tip<128>()), 0, st, F, T); break;
    default: return fail(DION_E_UNSUPPORTED, "tri_inv r=%d", r);
  }
  return check_launch("tri_inv");
}

// the first solve with the Gram of its output folded in (r = 32 / 64: tsolve_mfma_kernel GRAM):
// persistent blocks, one partial Gram per block into `gram` (batch x tgram_chunks x r x r)
int launch_tsolve_gram(const float* src, float* dst, const float* T, int mp, int r, int batch, float* gram,
                       hipStream_t st) {
  TrsmArgs ta{src, dst, T, nullptr, nullptr, 0, mp, 0, gram};
  const dim3 grid(static_cast<unsigned>(tgram_chunks(mp, batch)), batch);
  if (r == 64)
    hipLaunchKernelGGL((tsolve_mfma_kernel<64, false, true>), grid, dim3(64 * kTgWavesImg), 0, st, ta);
  else if (r == 32)
    hipLaunchKernelGGL((tsolve_mfma_kernel<32, false, true>), grid, dim3(64 * kTgWavesImg), 0, st, ta);
  else
    return fail(DION_E_UNSUPPORTED, "tsolve+Gram r=%d", r);
  return check_launch("tsolve_mfma(gram)");
}

int launch_tsolve(const float* src, float* dst, const float* T, int mp, int r, int batch, hipStream_t st, bool final_,
                  const uint32_t* nonzero, f16x8* psplit, long pstride, int kmap) {
  TrsmArgs ta{src, dst, T, nonzero, psplit, pstride, mp, kmap};
  auto go = [&](auto RTc, auto Fc) {
    constexpr int RT = decltype(RTc)::value;
    constexpr bool F = decltype(Fc)::value;
    constexpr int NW = tsolve_img<RT, F, false>() ? kTgWavesImg : kTgWavesDirect;
    hipLaunchKernelGGL((tsolve_mfma_kernel<RT, F>), dim3(static_cast<unsigned>(ceil_div(mp, 64 * NW)), batch),
                       dim3(64 * NW), 0, st, ta);
    return check_launch("tsolve_mfma");
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  switch (r) {
    case 32: return final_ ? go(std::integral_constant<int, 32>{}, T_{}) : go(std::integral_constant<int, 32>{}, F_{});
    case 64: return final_ ? go(std::integral_constant<int, 64>{}, T_{}) : go(std::integral_constant<int, 64>{}, F_{});
    case 128: return final_ ? go(std::integral_constant<int, 128>{}, T_{}) : go(std::integral_constant<int, 128>{}, F_{});
  }
  return fail(DION_E_UNSUPPORTED, "tsolve r=%d", r);
}

// dst_b = src_b R_b^-1 by forward substitution (trsm_right_kernel; factor from the INV = false
// factor kernels)
int launch_trsm(const float* src, float* dst, const float* fac, int mp, int r, int batch, hipStream_t st,
                const uint32_t* nonzero = nullptr) {
  const dim3 grid(static_cast<unsigned>(ceil_div(mp, 256)), batch);
  switch (trsm_rt(r)) {
    case 32: hipLaunchKernelGGL((trsm_right_kernel<32>), grid, dim3(256), 0, st, src, dst, fac, mp, r, nonzero); break;
    case 64: hipLaunchKernelGGL((trsm_right_kernel<64>), grid, dim3(256), 0, st, src, dst, fac, mp, r, nonzero); break;
    default: hipLaunchKernelGGL((trsm_right_kernel<128>), grid, dim3(256), 0, st, src, dst, fac, mp, r, nonzero); break;
  }
  return check_launch("trsm_right");
}

// S P with the generated Rademacher sketch (sketch_rad_kernel), reduced into out (batch, K, r)
int run_sketch_rad(const float* P, int mp, int K, int r, int batch, uint64_t seed, float* out, void* slab,
                   hipStream_t st) {
  const Geo g = sketch_rad_geo(mp, K, batch);
  SketchArgs a;
  memset(&a, 0, sizeof(a));
  a.P = P;
  a.out = g.nchunk > 1 ? static_cast<float*>(slab) : out;
  a.seed = seed;
  a.scale = 1.0f / sqrtf(static_cast<float>(K));
  a.mp = mp;
  a.r = r;
  a.K = K;
  a.kchunk = g.kchunk;
  a.nchunk = g.nchunk;
  a.vec = (r % 4 == 0 && aligned16(P)) ? 1 : 0;
  const dim3 grid(static_cast<unsigned>(g.nchunk), batch);
  auto go = [&](auto KTc, auto NTc) {
    constexpr int KT = decltype(KTc)::value, NT = decltype(NTc)::value;
    hipLaunchKernelGGL((sketch_rad_kernel<KT, NT>), grid, dim3(256), 0, st, a);
    return check_launch("sketch_rad");
  };
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  using I4 = std::integral_constant<int, 4>;
  int rc;
  const int nt = (r + 31) / 32;
  if (K == 128) {
    rc = nt == 1 ? go(I1{}, I1{}) : nt == 2 ? go(I1{}, I2{}) : nt == 3 ? go(I1{}, I3{}) : go(I1{}, I4{});
  } else if (K == 256) {
    rc = nt == 1 ? go(I2{}, I1{}) : nt == 2 ? go(I2{}, I2{}) : nt == 3 ? go(I2{}, I3{}) : go(I2{}, I4{});
  } else {
    return fail(DION_E_UNSUPPORTED, "generated sketch with k=%d rows", K);
  }
  if (rc != DION_OK) return rc;
  if (g.nchunk > 1) return launch_reduce(out, static_cast<const float*>(slab), g.nchunk, static_cast<long>(K) * r, batch, st);
  return DION_OK;
}

// dst_b = src_b Uinv_b for every matrix (m_P x r times r x r), an MFMA row projection
int apply_right(const float* src, float* dst, const float* Uinv, int mp, int r, int batch, hipStream_t st) {
  const Geo geo = rowproj_geo(mp, r, batch);
  if (geo.nchunk != 1) return fail(DION_E_INVALID, "internal: right-apply split");
  ProjArgs a;
  memset(&a, 0, sizeof(a));
  bool vec = (r % 4) == 0;
  for (int b = 0; b < batch; ++b) {
    a.m[b] = const_cast<float*>(src + static_cast<long>(b) * mp * r);
    a.thin[b] = Uinv + static_cast<long>(b) * r * r;
    vec = vec && aligned16(a.m[b]);
  }
  a.out = dst;
  a.rows = mp;
  a.cols = r;
  a.r = r;
  a.ld_m = r;
  a.kchunk = geo.kchunk;
  a.nchunk = 1;
  a.out_rows = mp;
  a.vec = vec ? 1 : 0;
  const dim3 grid(geo.gx, 1, batch);
  return dispatch_rb(r, [&](auto RBc) {
    constexpr int RB = decltype(RBc)::value;
    hipLaunchKernelGGL((rowproj_kernel<RB, DION_DTYPE_NONE>), grid, dim3(256), 0, st, a);
    return check_launch("apply_right");
  });
}

size_t qr_lds_bytes(int K, int r) { return sizeof(float) * (static_cast<size_t>(r) * (K + 1) + r + 3 + 8 + 4); }

}  // namespace

// ============================================================================
// C ABI
// ============================================================================
#include "dion_bf16.hpp"
#include "dion_gradnorm.hpp"
#include "dion_elementwise.hpp"

namespace {
int validate_grads(const DionBatchDesc* d) {
  if (d == nullptr) return fail(DION_E_INVALID, "desc is null");
  if (d->batch < 0) return fail(DION_E_INVALID, "batch=%d", d->batch);
  if (d->m <= 0 || d->n <= 0) return fail(DION_E_INVALID, "bad shape m=%d n=%d", d->m, d->n);
  if (d->g_dtype != DION_DTYPE_F32 && d->g_dtype != DION_DTYPE_BF16)
    return fail(DION_E_UNSUPPORTED, "grad dtype %d", d->g_dtype);
  if (d->ld_g != 0 && d->ld_g < d->n) return fail(DION_E_INVALID, "ld_g=%lld < n=%d", static_cast<long long>(d->ld_g), d->n);
  return DION_OK;
}
}  // namespace

extern "C" {

int dion_abi_version(void) { return DION_ABI_VERSION; }

#ifndef DION_BUILD_ID
#define DION_BUILD_ID "unknown"
#endif
const char* dion_build_id(void) { return DION_BUILD_ID; }

const char* dion_last_error(void) { return g_err; }

int dion_workspace_bytes(const DionBatchDesc* d, int op, size_t* bytes) {
  if (op == DION_OP_DORTHO) {
    const int rcd = validate_dortho(d);
    if (rcd != DION_OK) return rcd;
    if (bytes == nullptr) return fail(DION_E_INVALID, "bytes is null");
    const int mp = d->transposed ? d->n : d->m;
    const int nb = d->batch < MAXB ? d->batch : MAXB;
    const size_t a = slab_bytes(colproj_geo(mp, sketch_k(d->r, 2.0f), nb, true), nb, d->r);
    const size_t g = slab_bytes(colproj_geo(mp, d->r, nb, true), nb, d->r);
    size_t need = a > g ? a : g;
    // the sketch slab grows with k; any oversample up to 2 fits (k <= 256 for r <= 128)
    for (int k = 128; k <= 256; k += 128) {
      const size_t x = slab_bytes(colproj_geo(mp, k, nb, true), nb, d->r);
      need = x > need ? x : need;
    }
    *bytes = need;
    return DION_OK;
  }
  if (op == DION_OP_GRAD_SUM_SQ) {
    const int rcg = validate_grads(d);
    if (rcg != DION_OK) return rcg;
    if (bytes == nullptr) return fail(DION_E_INVALID, "bytes is null");
    *bytes = gnorm::ws_bytes(d->m, d->batch);
    return DION_OK;
  }
  int rc = validate(d);
  if (rc != DION_OK) return rc;
  if (bytes == nullptr) return fail(DION_E_INVALID, "bytes is null");
  const int mp = d->transposed ? d->n : d->m;
  const int nq = d->transposed ? d->m : d->n;
  if (op == DION_OP_PSPLIT) {
    // not scratch: the caller's buffer for dion_orthonormalize_fused -> dion_project_r_split
    if (!psplit_ok(d)) return fail(DION_E_UNSUPPORTED, "no fused pass-B split for %dx%d r=%d", d->m, d->n, d->r);
    *bytes = sizeof(uint16_t) * 2 * static_cast<size_t>(d->batch) * mp * d->r;
    return DION_OK;
  }
  size_t need = 0;
  const int chunks[2] = {d->batch < MAXB ? d->batch : MAXB, d->batch % MAXB};
  if (d->m_dtype == DION_DTYPE_BF16) {
    if (op == DION_OP_PROJECT_P_EF) {
      const bool row_mode = !d->transposed;
      if (!b16::ef_ok(row_mode, d->m, d->n, d->r, d->g_dtype))
        return fail(DION_E_UNSUPPORTED, "no deferred-EF bf16 pass A for %dx%d r=%d", d->m, d->n, d->r);
      for (int ci = 0; ci < 2; ++ci)
        if (chunks[ci] > 0) {
          const size_t n = b16::proj_ws(d->m, d->n, d->r, chunks[ci], row_mode, true);
          if (n > need) need = n;
        }
      *bytes = need;
      return DION_OK;
    }
    if (op == DION_OP_PROJECT_P || op == DION_OP_PROJECT_R) {
      const bool row_mode = (op == DION_OP_PROJECT_P) ? !d->transposed : d->transposed;
      for (int ci = 0; ci < 2; ++ci)
        if (chunks[ci] > 0) {
          const size_t n = b16::proj_ws(d->m, d->n, d->r, chunks[ci], row_mode);
          if (n > need) need = n;
        }
      *bytes = need;
      return DION_OK;
    }
    if (op == DION_OP_EF_APPLY) {
      *bytes = 0;
      return DION_OK;
    }
  }
  for (int ci = 0; ci < 2; ++ci) {
    const int chunk = chunks[ci];
    if (chunk <= 0) continue;
    size_t n = 0;
    switch (op) {
      case DION_OP_PROJECT_P:
      case DION_OP_PROJECT_R: {
        const bool row_mode = (op == DION_OP_PROJECT_P) ? !d->transposed : d->transposed;
        Geo g = row_mode ? rowproj_geo(d->m, d->n, chunk) : colproj_geo(d->m, d->n, chunk, false);
        n = slab_bytes(g, chunk, d->r);
        if (row_mode) {
          const size_t nf = slab_bytes(rowproj_geo(d->m, d->n, chunk, 64 * kRB), chunk, d->r);
          if (nf > n) n = nf;
          const size_t ne = slab_bytes(rowproj_geo(d->m, d->n, chunk, 64 * kRBE), chunk, d->r);
          if (ne > n) n = ne;
          const size_t nh = slab_bytes(rowproj_geo(d->m, d->n, chunk, 16 * kRBE * kPbRNW, kTbPbr), chunk, d->r);
          if (nh > n) n = nh;
          const size_t ng = slab_bytes(pbr_geo(d->m, d->n, chunk, d->r), chunk, d->r);
          if (ng > n) n = ng;
        } else {
          const size_t nx = slab_bytes(colx6_geo(d->m, d->n, chunk, d->r), chunk, d->r);
          if (nx > n) n = nx;
          const size_t nh = slab_bytes(colh3_geo(d->m, d->n, chunk, d->r), chunk, d->r);
          if (nh > n) n = nh;
        }
        if (op == DION_OP_PROJECT_R)  // + the fix-up partials of dion_project_r_fixup
          n = (n + 255) / 256 * 256 + thin_presplit_bytes(row_mode ? d->n : d->m, d->r, chunk) + 256 +
              fix_part_bytes(nq, d->r, chunk);
        break;
      }
      case DION_OP_PROJECT_P_EF: {
        if (!proj_ef_ok(d->m, d->n, d->r, d->transposed != 0))
          return fail(DION_E_UNSUPPORTED, "no deferred-EF pass A for %dx%d r=%d", d->m, d->n, d->r);
        n = slab_bytes(proj_ef_geo(d->m, d->n, chunk, d->transposed != 0, d->r), chunk, d->r) +
            presplit_bytes(nq, d->r, chunk);
        break;
      }
      case DION_OP_EF_APPLY:
        n = 0;  // the update splits its factors in-kernel
        break;
      case DION_OP_ORTHONORMALIZE: {
        if (d->r > d->m || d->r > d->n)
          return fail(DION_E_INVALID, "rank r=%d exceeds min(m=%d, n=%d) of a whole matrix", d->r, d->m, d->n);
        // k = ceil(oversample r / 128) * 128 is bounded by the value at oversample 2
        n = ortho_plan(mp, d->r, chunk, 2.0f).total;
        break;
      }
      case DION_OP_FIXUP_COLNORM: {
        const int nq = d->transposed ? d->m : d->n;
        n = sizeof(float) * static_cast<size_t>(chunk) * ceil_div(nq, kFixRows) * d->r;
        break;
      }
      default:
        return fail(DION_E_INVALID, "unknown op %d", op);
    }
    if (n > need) need = n;
  }
  (void)nq;
  *bytes = need;
  return DION_OK;
}

int dion_project_p(const DionBatchDesc* d, const void* const* G, float* const* M, const float* const* Q, float* P,
                   uint32_t* nonzero, void* ws, size_t ws_bytes, dion_stream_t stream) {
  int rc = validate(d);
  if (rc != DION_OK) return rc;
  if (M == nullptr || Q == nullptr || P == nullptr) return fail(DION_E_INVALID, "null argument");
  if (d->g_dtype != DION_DTYPE_NONE && G == nullptr) return fail(DION_E_INVALID, "G is null");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int mp = d->transposed ? d->n : d->m;
  const long ld_m = ldv(d->ld_m, d->n), ld_g = ldv(d->ld_g, d->n);
  if (d->m_dtype == DION_DTYPE_BF16) {
    // bf16 momentum / Q: M = rne(M + rne(G)), P = rne(X Q)
    for (int b0 = 0; b0 < d->batch; b0 += MAXB) {
      const int nb = d->batch - b0 < MAXB ? d->batch - b0 : MAXB;
      rc = b16::project(!d->transposed, d->m, d->n, d->r, nb, G ? G + b0 : nullptr, d->g_dtype,
                        reinterpret_cast<uint16_t* const*>(M + b0), ld_m, ld_g,
                        reinterpret_cast<const void* const*>(Q + b0), true, P + static_cast<long>(b0) * mp * d->r,
                        nonzero ? nonzero + b0 : nullptr, ws, ws_bytes, st);
      if (rc != DION_OK) return rc;
    }
    return DION_OK;
  }
  for (int b0 = 0; b0 < d->batch; b0 += MAXB) {
    const int nb = d->batch - b0 < MAXB ? d->batch - b0 : MAXB;
    rc = run_projection(!d->transposed, d->m, d->n, d->r, nb, G ? G + b0 : nullptr, M + b0, Q + b0, ld_m, ld_g,
                        d->g_dtype, P + static_cast<long>(b0) * mp * d->r, nonzero ? nonzero + b0 : nullptr, ws,
                        ws_bytes, st);
    if (rc != DION_OK) return rc;
  }
  return DION_OK;
}

int dion_project_p_ef(const DionBatchDesc* d, const void* const* G, float* const* M, const float* const* Q,
                      float* P, uint32_t* nonzero, const DionPendingEF* ef, void* ws, size_t ws_bytes,
                      dion_stream_t stream) {
  if (ef == nullptr) return dion_project_p(d, G, M, Q, P, nonzero, ws, ws_bytes, stream);
  int rc = validate(d);
  if (rc != DION_OK) return rc;
  if (M == nullptr || Q == nullptr || P == nullptr || ef->P == nullptr || ef->R == nullptr)
    return fail(DION_E_INVALID, "null argument");
  if (d->g_dtype != DION_DTYPE_NONE && G == nullptr) return fail(DION_E_INVALID, "G is null");
  const bool tr = d->transposed != 0;
  const int mp = tr ? d->n : d->m;
  const long ld_m = ldv(d->ld_m, d->n), ld_g = ldv(d->ld_g, d->n);
  if (d->m_dtype == DION_DTYPE_BF16) {
    // bf16 momentum / Q: M = rne(M + rne(alpha rne(P' R'^T))), M = rne(M + rne(G)), P = rne(X Q).
    // Every entry is checked before the first launch (as the fp32 branch below does): the
    // fused kernels need the whole-line layout (16-byte aligned M / G / factors, ld % 8), so
    // an UNSUPPORTED return has enqueued nothing and the caller can still run the eager path.
    if (!b16::ef_ok(!tr, d->m, d->n, d->r, d->g_dtype) || ld_m % 8 != 0 ||
        (d->g_dtype != DION_DTYPE_NONE && ld_g % 8 != 0))
      return fail(DION_E_UNSUPPORTED, "no deferred-EF bf16 pass A for %dx%d r=%d ld_m=%ld ld_g=%ld", d->m, d->n,
                  d->r, ld_m, ld_g);
    for (int b = 0; b < d->batch; ++b) {
      if (M[b] == nullptr || Q[b] == nullptr || (d->g_dtype != DION_DTYPE_NONE && G[b] == nullptr))
        return fail(DION_E_INVALID, "null matrix pointer at entry %d", b);
      if ((ef->P[b] == nullptr) != (ef->R[b] == nullptr))
        return fail(DION_E_INVALID, "pending EF of entry %d has only one factor", b);
      if (!aligned16(M[b]) || (d->g_dtype != DION_DTYPE_NONE && !aligned16(G[b])) ||
          (ef->P[b] && (!aligned16(ef->P[b]) || !aligned16(ef->R[b]))))
        return fail(DION_E_UNSUPPORTED, "deferred-EF bf16 pass A needs 16-byte aligned operands (entry %d)", b);
    }
    {
      const int nb0 = d->batch < MAXB ? d->batch : MAXB;  // the largest chunk sizes the workspace
      const size_t need = b16::proj_ws(d->m, d->n, d->r, nb0, !tr, true);
      if (ws == nullptr || ws_bytes < need)
        return fail(DION_E_WORKSPACE, "bf16 projection needs %zu workspace bytes, got %zu", need, ws_bytes);
    }
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    for (int b0 = 0; b0 < d->batch; b0 += MAXB) {
      const int nb = d->batch - b0 < MAXB ? d->batch - b0 : MAXB;
      rc = b16::project(!tr, d->m, d->n, d->r, nb, G ? G + b0 : nullptr, d->g_dtype,
                        reinterpret_cast<uint16_t* const*>(M + b0), ld_m, ld_g,
                        reinterpret_cast<const void* const*>(Q + b0), true, P + static_cast<long>(b0) * mp * d->r,
                        nonzero ? nonzero + b0 : nullptr, ws, ws_bytes, st,
                        reinterpret_cast<const float* const*>(ef->P) + b0,
                        reinterpret_cast<const float* const*>(ef->R) + b0, ef->alpha);
      if (rc != DION_OK) return rc;
    }
    return DION_OK;
  }
  if (!proj_ef_ok(d->m, d->n, d->r, tr) || ld_m % 8 != 0 || (d->g_dtype != DION_DTYPE_NONE && ld_g % 8 != 0))
    return fail(DION_E_UNSUPPORTED, "no deferred-EF pass A for %dx%d r=%d", d->m, d->n, d->r);
  for (int b = 0; b < d->batch; ++b) {
    if (M[b] == nullptr || Q[b] == nullptr || (d->g_dtype != DION_DTYPE_NONE && G[b] == nullptr))
      return fail(DION_E_INVALID, "null matrix pointer at entry %d", b);
    if ((ef->P[b] == nullptr) != (ef->R[b] == nullptr))
      return fail(DION_E_INVALID, "pending EF of entry %d has only one factor", b);
    if (!aligned16(M[b]) || !aligned16(Q[b]) || (d->g_dtype != DION_DTYPE_NONE && !aligned16(G[b])) ||
        (ef->P[b] && (!aligned16(ef->P[b]) || !aligned16(ef->R[b]))))
      return fail(DION_E_UNSUPPORTED, "deferred-EF pass A needs 16-byte aligned operands (entry %d)", b);
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int b0 = 0; b0 < d->batch; b0 += MAXB) {
    const int nb = d->batch - b0 < MAXB ? d->batch - b0 : MAXB;
    const Geo geo = proj_ef_geo(d->m, d->n, nb, tr, d->r);
    const int nq = tr ? d->m : d->n;
    const size_t slab = (slab_bytes(geo, nb, d->r) + 255) / 256 * 256;
    const size_t need = slab + presplit_bytes(nq, d->r, nb);
    if (need > ws_bytes || ws == nullptr)
      return fail(DION_E_WORKSPACE, "projection needs %zu workspace bytes, got %zu", need, ws_bytes);
    const long sstride = static_cast<long>(nq) * d->r / 4;
    u32x4* qsplit = reinterpret_cast<u32x4*>(static_cast<char*>(ws) + slab);
    u32x4* rsplit = qsplit + sstride * nb;
    uint32_t* amax = nullptr;
    float* inv = nullptr;
    {
      // fp16x3: per-matrix |max| of Q and R', then the two fp16 limbs of Q and R'.  P' is the
      // previous step's fixed-up P, orthonormal columns with |x| <= 1: the kernels split it on
      // the fixed scale 2^14 (no pass over P' for its maximum)
      char* tail = reinterpret_cast<char*>(rsplit + sstride * nb);
      amax = reinterpret_cast<uint32_t*>(tail);
      inv = reinterpret_cast<float*>(tail + 1024);
      hipError_t me = hipMemsetAsync(amax, 0, sizeof(uint32_t) * 2 * nb, st);
      if (me != hipSuccess) return fail(DION_E_LAUNCH, "memset: %s", hipGetErrorString(me));
      AbsMaxArgs ma;
      memset(&ma, 0, sizeof(ma));
      for (int b = 0; b < nb; ++b) {
        ma.src[b] = Q[b0 + b];
        ma.src[nb + b] = ef->R[b0 + b];
      }
      ma.out = amax;
      ma.count[0] = ma.count[1] = static_cast<long>(nq) * d->r;
      ma.nb = nb;
      launch_absmax(ma, 2, st);
      Presplit16Args pa;
      memset(&pa, 0, sizeof(pa));
      pa.rows = nq;
      pa.r = d->r;
      pa.stride = sstride;
      const dim3 pgrid(static_cast<unsigned>(ceil_div(static_cast<long>(nq) * d->r / 8, 256)), nb);
      for (int b = 0; b < nb; ++b) pa.src[b] = Q[b0 + b];
      pa.dst = reinterpret_cast<f16x8*>(qsplit);
      pa.amax = amax;
      pa.inv_scale = inv;
      pa.layout = 0;
      pa.kmap = 1;
      hipLaunchKernelGGL(presplit16_kernel, pgrid, dim3(256), 0, st, pa);
      for (int b = 0; b < nb; ++b) pa.src[b] = ef->R[b0 + b];
      pa.dst = reinterpret_cast<f16x8*>(rsplit);
      pa.amax = amax + nb;
      pa.inv_scale = inv + nb;
      pa.layout = 1;
      pa.kmap = 0;
      hipLaunchKernelGGL(presplit16_kernel, pgrid, dim3(256), 0, st, pa);
      rc = check_launch("presplit16");
      if (rc != DION_OK) return rc;
    }
    float* out = P + static_cast<long>(b0) * mp * d->r;
    EfProjArgs e;
    memset(&e, 0, sizeof(e));
    ProjArgs& a = e.p;
    for (int b = 0; b < nb; ++b) {
      a.g[b] = G ? G[b0 + b] : nullptr;
      a.m[b] = M[b0 + b];
      a.thin[b] = Q[b0 + b];
      e.efp[b] = ef->P[b0 + b];
      e.efr[b] = ef->R[b0 + b];
    }
    e.alpha = ef->alpha;
    e.qsplit = qsplit;
    e.rsplit = rsplit;
    e.split_stride = sstride;
    e.amax = amax;
    e.inv = inv;
    a.out = geo.nchunk > 1 ? static_cast<float*>(ws) : out;
    a.nonzero = nonzero ? nonzero + b0 : nullptr;
    a.rows = d->m;
    a.cols = d->n;
    a.r = d->r;
    a.ld_m = ld_m;
    a.ld_g = ld_g;
    a.kchunk = geo.kchunk;
    a.nchunk = geo.nchunk;
    a.out_rows = geo.out_rows;
    a.vec = 1;
    const dim3 grid(geo.gx, geo.nchunk, nb);
    auto go = [&](auto RBc) {
      constexpr int RB = decltype(RBc)::value;
      return dispatch_gdt(d->g_dtype, [&](auto Gc) {
        constexpr int GD = decltype(Gc)::value;
        if (tr) {
          if (RB >= kPaGlMinRBT && GD != DION_DTYPE_F32 && kPaGl8 && geo.gx % 2 == 0)  // LDS-DMA staging
            hipLaunchKernelGGL((colproj_efgl_kernel<(RB >= kPaGlMinRBT ? RB : kPaGlMinRBT), GD == DION_DTYPE_F32 ? DION_DTYPE_NONE : GD>),
                               dim3(geo.gx / 2, geo.nchunk, nb), dim3(512), 0, st, e);
          else
            hipLaunchKernelGGL((colproj_efh3_kernel<RB, GD>), grid, dim3(256), 0, st, e);
        } else if (RB >= kPaGlMinRB && GD != DION_DTYPE_F32 && kPaGl8 && geo.gx % 2 == 0)  // LDS-DMA staging
          hipLaunchKernelGGL((rowproj_efgl_kernel<(RB >= kPaGlMinRB ? RB : kPaGlMinRB), GD == DION_DTYPE_F32 ? DION_DTYPE_NONE : GD>),
                             dim3(geo.gx / 2, geo.nchunk, nb), dim3(512), 0, st, e);
        else  // r = 128 without it: one-step pipeline (register budget)
          hipLaunchKernelGGL((rowproj_efh3_kernel<RB, GD, RB >= 8 ? kPD8 : kPaPD, RB >= 8 ? kKR8 : kPaKR, RB >= 8 ? kNW8 : kPaNW>),
                             grid, dim3(64 * (RB >= 8 ? kNW8 : kPaNW)), 0, st, e);
        return check_launch(tr ? "colproj_ef" : "rowproj_ef");
      });
    };
    rc = d->r == 32    ? go(std::integral_constant<int, 2>{})
         : d->r == 64  ? go(std::integral_constant<int, 4>{})
                       : go(std::integral_constant<int, 8>{});
    if (rc != DION_OK) return rc;
    if (geo.nchunk > 1) {
      rc = launch_reduce(out, static_cast<const float*>(ws), geo.nchunk, static_cast<long>(geo.out_rows) * d->r, nb, st);
      if (rc != DION_OK) return rc;
    }
  }
  return DION_OK;
}

int dion_project_r(const DionBatchDesc* d, const float* const* M, const float* P, float* R,
                   const uint32_t* m_absmax, void* ws, size_t ws_bytes, dion_stream_t stream) {
  return dion_project_r_split(d, M, P, nullptr, R, m_absmax, ws, ws_bytes, stream);
}

int dion_project_r_split(const DionBatchDesc* d, const float* const* M, const float* P, const void* p_split,
                         float* R, const uint32_t* m_absmax, void* ws, size_t ws_bytes, dion_stream_t stream) {
  int rc = validate(d);
  if (rc != DION_OK) return rc;
  if (M == nullptr || P == nullptr || R == nullptr) return fail(DION_E_INVALID, "null argument");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int mp = d->transposed ? d->n : d->m;
  const int nq = d->transposed ? d->m : d->n;
  const long ld_m = ldv(d->ld_m, d->n);
  if (d->m_dtype == DION_DTYPE_BF16) {
    // R = rne(X^T P), P already bf16-valued
    for (int b0 = 0; b0 < d->batch; b0 += MAXB) {
      const int nb = d->batch - b0 < MAXB ? d->batch - b0 : MAXB;
      const void* thin[MAXB];
      for (int b = 0; b < nb; ++b) thin[b] = P + static_cast<long>(b0 + b) * mp * d->r;
      rc = b16::project(d->transposed != 0, d->m, d->n, d->r, nb, nullptr, DION_DTYPE_NONE,
                        reinterpret_cast<uint16_t* const*>(const_cast<float* const*>(M + b0)), ld_m, 0, thin, false,
                        R + static_cast<long>(b0) * nq * d->r, nullptr, ws, ws_bytes, st);
      if (rc != DION_OK) return rc;
    }
    return DION_OK;
  }
  for (int b0 = 0; b0 < d->batch; b0 += MAXB) {
    const int nb = d->batch - b0 < MAXB ? d->batch - b0 : MAXB;
    const float* thin[MAXB];
    for (int b = 0; b < nb; ++b) thin[b] = P + static_cast<long>(b0 + b) * mp * d->r;
    rc = run_projection(d->transposed != 0, d->m, d->n, d->r, nb, nullptr, const_cast<float* const*>(M + b0), thin,
                        ld_m, 0, DION_DTYPE_NONE, R + static_cast<long>(b0) * nq * d->r, nullptr, ws, ws_bytes, st,
                        m_absmax != nullptr ? m_absmax + b0 : nullptr,
                        p_split != nullptr ? static_cast<const f16x8*>(p_split) + static_cast<long>(b0) * mp * d->r / 4
                                           : nullptr);
    if (rc != DION_OK) return rc;
  }
  return DION_OK;
}

int dion_project_r_fixup(const DionBatchDesc* d, const float* const* M, const float* P, const void* p_split,
                         float* R, const uint32_t* m_absmax, float* const* Q, const uint32_t* nonzero, float eps,
                         void* ws, size_t ws_bytes, dion_stream_t stream) {
  int rc = validate(d);
  if (rc != DION_OK) return rc;
  if (M == nullptr || P == nullptr || R == nullptr || Q == nullptr || nonzero == nullptr)
    return fail(DION_E_INVALID, "null argument");
  if (d->m_dtype != DION_DTYPE_F32) return fail(DION_E_UNSUPPORTED, "dion_project_r_fixup: fp32 state only");
  if (d->batch == 0) return DION_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int mp = d->transposed ? d->n : d->m;
  const int nq = d->transposed ? d->m : d->n;
  const int r = d->r;
  const long ld_m = ldv(d->ld_m, d->n);
  const int nb0 = d->batch < MAXB ? d->batch : MAXB;
  const size_t pbytes = fix_part_bytes(nq, r, nb0);
  if (ws == nullptr || ws_bytes < pbytes)
    return fail(DION_E_WORKSPACE, "project_r_fixup needs %zu more workspace bytes", pbytes);
  const size_t proj_bytes = (ws_bytes - pbytes) / 256 * 256;
  float* part = reinterpret_cast<float*>(static_cast<char*>(ws) + proj_bytes);
  for (int b0 = 0; b0 < d->batch; b0 += MAXB) {
    const int nb = d->batch - b0 < MAXB ? d->batch - b0 : MAXB;
    const float* thin[MAXB];
    FixArgs fa;
    memset(&fa, 0, sizeof(fa));
    for (int b = 0; b < nb; ++b) {
      thin[b] = P + static_cast<long>(b0 + b) * mp * r;
      if (Q[b0 + b] == nullptr) return fail(DION_E_INVALID, "null Q at %d", b0 + b);
      fa.q[b] = Q[b0 + b];
    }
    fa.R = R + static_cast<long>(b0) * nq * r;
    fa.part = part;
    fa.nonzero = nonzero + b0;
    fa.nq = nq;
    fa.r = r;
    fa.tpc = 256 / r;
    fa.rows_per_chunk = kFixRows;
    fa.nchunk = static_cast<int>(ceil_div(nq, kFixRows));
    fa.eps = eps;
    rc = run_projection(d->transposed != 0, d->m, d->n, r, nb, nullptr, const_cast<float* const*>(M + b0), thin, ld_m,
                        0, DION_DTYPE_NONE, fa.R, nullptr, ws, proj_bytes, st,
                        m_absmax != nullptr ? m_absmax + b0 : nullptr,
                        p_split != nullptr ? static_cast<const f16x8*>(p_split) + static_cast<long>(b0) * mp * r / 4
                                           : nullptr,
                        &fa);
    if (rc != DION_OK) return rc;
  }
  return DION_OK;
}

int dion_pfix_split(const DionBatchDesc* d, float* P, const uint32_t* nonzero, void* p_split, dion_stream_t stream) {
  int rc = validate(d);
  if (rc != DION_OK) return rc;
  if (P == nullptr || (nonzero == nullptr && p_split == nullptr)) return fail(DION_E_INVALID, "null argument");
  if (d->m_dtype != DION_DTYPE_F32) return fail(DION_E_UNSUPPORTED, "dion_pfix_split: fp32 state only");
  if (p_split != nullptr && (!psplit_ok(d) || !aligned16(P) || !aligned16(p_split)))
    return fail(DION_E_UNSUPPORTED, "no fused pass-B split for %dx%d r=%d", d->m, d->n, d->r);
  if (d->batch == 0) return DION_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int mp = d->transposed ? d->n : d->m;
  const int r = d->r;
  if (p_split == nullptr) return launch_pfix(P, nonzero, static_cast<long>(mp) * r, d->batch, st);
  for (int b0 = 0; b0 < d->batch; b0 += MAXB) {
    const int nb = d->batch - b0 < MAXB ? d->batch - b0 : MAXB;
    rc = launch_psplit_fixed(P + static_cast<long>(b0) * mp * r, mp, r, nb, nonzero != nullptr ? nonzero + b0 : nullptr,
                             static_cast<f16x8*>(p_split) + static_cast<long>(b0) * mp * r / 4, d->transposed ? 1 : 0,
                             st);
    if (rc != DION_OK) return rc;
  }
  return DION_OK;
}

int dion_orthonormalize(const DionBatchDesc* d, float* P, const float* sketch, uint64_t seed, float oversample,
                        void* ws, size_t ws_bytes, dion_stream_t stream) {
  return dion_orthonormalize_fused(d, P, sketch, seed, oversample, nullptr, nullptr, ws, ws_bytes, stream);
}

int dion_orthonormalize_fused(const DionBatchDesc* d, float* P, const float* sketch, uint64_t seed, float oversample,
                              const uint32_t* nonzero, void* p_split, void* ws, size_t ws_bytes,
                              dion_stream_t stream) {
  int rc = validate(d);
  if (rc != DION_OK) return rc;
  if (d->r > d->m || d->r > d->n)
    return fail(DION_E_INVALID, "rank r=%d exceeds min(m=%d, n=%d) of a whole matrix", d->r, d->m, d->n);
  if (P == nullptr) return fail(DION_E_INVALID, "P is null");
  if (!(oversample > 0.f)) return fail(DION_E_INVALID, "oversample=%f", oversample);
  if (p_split != nullptr && (!psplit_ok(d) || !aligned16(P) || !aligned16(p_split)))
    return fail(DION_E_UNSUPPORTED, "no fused pass-B split for %dx%d r=%d", d->m, d->n, d->r);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int mp = d->transposed ? d->n : d->m;
  const int r = d->r;
  // the fix-up of P rides on the last solve of an fp32 P (the LDS solve at r = 32 / 64 with
  // an aligned P, else trsm_right_kernel); elsewhere (plain QR, bf16 rounding first)
  // pfix_kernel runs after the orthonormalisation
  const bool fuse_fix = nonzero != nullptr && d->m_dtype == DION_DTYPE_F32 && mp > r;
  const bool lds_fix = fuse_fix && (r == 32 || r == 64) && aligned16(P);
  for (int b0 = 0; b0 < d->batch; b0 += MAXB) {
    const int nb = d->batch - b0 < MAXB ? d->batch - b0 : MAXB;
    float* Pb = P + static_cast<long>(b0) * mp * r;
    const OrthoPlan plan = ortho_plan(mp, r, nb, oversample);
    if (plan.plain_qr) {
      const size_t lds = qr_lds_bytes(mp, r);
      if (lds > 160 * 1024) return fail(DION_E_UNSUPPORTED, "plain QR of %dx%d does not fit LDS", mp, r);
      rc = allow_lds(householder_qr_kernel, lds);
      if (rc != DION_OK) return rc;
      hipLaunchKernelGGL(householder_qr_kernel, dim3(nb), dim3(256), lds, st, Pb, nullptr, Pb, mp, r, 1);
      rc = check_launch("householder_qr(Q)");
      if (rc != DION_OK) return rc;
      if (d->m_dtype == DION_DTYPE_BF16) {
        rc = b16::round_buffer(Pb, static_cast<long>(nb) * mp * r, st);
        if (rc != DION_OK) return rc;
      }
      continue;
    }
    if (plan.total > ws_bytes || ws == nullptr)
      return fail(DION_E_WORKSPACE, "orthonormalize needs %zu workspace bytes, got %zu", plan.total, ws_bytes);
    char* base = static_cast<char*>(ws);
    float* sk_slab = reinterpret_cast<float*>(base + plan.off_sk_slab);
    float* sp = reinterpret_cast<float*>(base + plan.off_sp);
    float* r1 = reinterpret_cast<float*>(base + plan.off_r1);
    float* gslab = reinterpret_cast<float*>(base + plan.off_gslab);
    float* gm = reinterpret_cast<float*>(base + plan.off_g);
    float* r2 = reinterpret_cast<float*>(base + plan.off_r2);
    const int K = plan.k;
    const size_t lds = qr_lds_bytes(K, r);
    if (lds > 160 * 1024) return fail(DION_E_UNSUPPORTED, "sketch QR of %dx%d does not fit LDS", K, r);
    rc = allow_lds(householder_qr_kernel, lds);
    if (rc != DION_OK) return rc;
    // (1) S P  (K x r): the caller's sketch (parity replays), else a generated Rademacher one
    const uint64_t bseed = seed + 0x9E3779B97F4A7C15ull * static_cast<uint64_t>(b0);
    if (sketch)
      rc = run_panel(1, mp, K, r, nb, Pb, sketch + static_cast<long>(b0) * K * mp, bseed,
                     sqrtf(1.0f / static_cast<float>(K)), sp, sk_slab, plan.sk, st);
    else
      rc = run_sketch_rad(Pb, mp, K, r, nb, bseed, sp, sk_slab, st);
    if (rc != DION_OK) return rc;
    float* fac = reinterpret_cast<float*>(base + plan.off_inv);
    float* p1 = reinterpret_cast<float*>(base + plan.off_p1);
    // (2) R1 = qr(S P).R, (3) P1 = P R1^-1 (into workspace): by forward substitution, or as
    // the GEMM P T1 with the explicit inverse T1 (tsolve_mfma_kernel)
    const bool gemm = tsolve_gemm_ok(mp, r);
    // gemm: T1 = R1^-1 written by the QR kernel itself (r1)
    rc = gemm ? launch_sketch_qr_inv(sp, r1, K, r, nb, st, false, true) : launch_sketch_qr_inv(sp, fac, K, r, nb, st, false);
    if (rc != DION_OK) return rc;
    // gemm at r <= 64: the solve also sums P1^T P1 (upper block triangle) per block
    const bool tgram = kTsolveGram && gemm && r <= 64;
    if (tgram) {
      const int nck = tgram_chunks(mp, nb);
      rc = launch_tsolve_gram(Pb, p1, r1, mp, r, nb, nck > 1 ? gslab : gm, st);
      if (rc == DION_OK && nck > 1) rc = launch_reduce(gm, gslab, nck, static_cast<long>(r) * r, nb, st);
    } else {
      rc = gemm ? launch_tsolve(Pb, p1, r1, mp, r, nb, st, false, nullptr, nullptr, 0, 0)
                : launch_trsm(Pb, p1, fac, mp, r, nb, st);
    }
    if (rc != DION_OK) return rc;
    // (4) Gram = P1^T P1
    if (tgram) {
      // done by the solve
    } else if (gram_h3_ok(mp, r)) {
      const GramArgs ga{p1, plan.gr.nchunk > 1 ? gslab : gm, mp, plan.gr.kchunk, plan.gr.nchunk};
      if (r == 64)
        hipLaunchKernelGGL((gram_h3_kernel<4>), dim3(plan.gr.nchunk, nb), dim3(256), 0, st, ga);
      else
        hipLaunchKernelGGL((gram_h3_kernel<8>), dim3(plan.gr.nchunk, nb), dim3(256), 0, st, ga);
      rc = check_launch("gram_h3");
      if (rc == DION_OK && plan.gr.nchunk > 1)
        rc = launch_reduce(gm, gslab, plan.gr.nchunk, static_cast<long>(r) * r, nb, st);
    } else {
      rc = run_panel(0, mp, r, r, nb, p1, nullptr, 0, 0.f, gm, gslab, plan.gr, st);
    }
    if (rc != DION_OK) return rc;
    // (5) R2 = chol_upper(Gram)
    // gemm: T2 = R2^-1 written by the Cholesky kernel itself (r1)
    rc = gemm ? launch_chol_inv(gm, r1, r, nb, st, false, true) : launch_chol_inv(gm, fac, r, nb, st, false);
    if (rc != DION_OK) return rc;
    (void)r2;
    // (6) P = P1 R2^-1 (back into the caller's buffer), with the fix-up and pass B's split
    if (gemm) {
      rc = launch_tsolve(p1, Pb, r1, mp, r, nb, st, true, fuse_fix ? nonzero + b0 : nullptr,
                         p_split != nullptr ? static_cast<f16x8*>(p_split) + static_cast<long>(b0) * mp * r / 4 : nullptr,
                         static_cast<long>(mp) * r / 4, d->transposed ? 1 : 0);
    } else if (lds_fix || (p_split != nullptr && r <= 64)) {
      TrsmArgs ta{p1, Pb, fac, fuse_fix ? nonzero + b0 : nullptr,
                  p_split != nullptr ? static_cast<f16x8*>(p_split) + static_cast<long>(b0) * mp * r / 4 : nullptr,
                  static_cast<long>(mp) * r / 4, mp, d->transposed ? 1 : 0};
      const dim3 grid(static_cast<unsigned>(ceil_div(mp, 64 * kTrsmWaves)), nb);
      if (r == 64)
        hipLaunchKernelGGL((trsm_lds_kernel<64, true>), grid, dim3(64 * kTrsmWaves), 0, st, ta);
      else
        hipLaunchKernelGGL((trsm_lds_kernel<32, true>), grid, dim3(64 * kTrsmWaves), 0, st, ta);
      rc = check_launch("trsm_lds(final)");
    } else {
      rc = launch_trsm(p1, Pb, fac, mp, r, nb, st, fuse_fix ? nonzero + b0 : nullptr);
    }
    if (rc != DION_OK) return rc;
    if (p_split != nullptr && r == 128)  // no row image in the r = 128 solve: split after it
      rc = launch_psplit_fixed(Pb, mp, r, nb, nullptr, static_cast<f16x8*>(p_split) + static_cast<long>(b0) * mp * r / 4,
                               d->transposed ? 1 : 0, st);
    if (rc != DION_OK) return rc;
  }
  // ortho.py:123: the fp32 result is cast back to P's dtype
  if (d->m_dtype == DION_DTYPE_BF16) {
    rc = b16::round_buffer(P, static_cast<long>(d->batch) * mp * r, st);
    if (rc != DION_OK) return rc;
  }
  if (nonzero != nullptr && !fuse_fix) return launch_pfix(P, nonzero, static_cast<long>(mp) * r, d->batch, st);
  return DION_OK;
}

// ---- distributed (row-sharded) randomised Cholesky QR: the per-rank pieces of
// dion/ortho.py:682-834 distributed_orthogonalize, between the caller's collectives
int dion_dortho_sketch(const DionBatchDesc* d, const float* P, const float* sketch, uint64_t seed,
                       int64_t row_offset, float oversample, float* SP, void* ws, size_t ws_bytes,
                       dion_stream_t stream) {
  int rc = validate_dortho(d);
  if (rc != DION_OK) return rc;
  if (P == nullptr || SP == nullptr) return fail(DION_E_INVALID, "null argument");
  if (!(oversample > 0.f)) return fail(DION_E_INVALID, "oversample=%f", oversample);
  if (row_offset < 0) return fail(DION_E_INVALID, "row_offset=%lld", static_cast<long long>(row_offset));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int mp = d->transposed ? d->n : d->m;
  const int r = d->r;
  const int K = sketch_k(r, oversample);
  const float std_ = sqrtf(1.0f / static_cast<float>(K));
  for (int b0 = 0; b0 < d->batch; b0 += MAXB) {
    const int nb = d->batch - b0 < MAXB ? d->batch - b0 : MAXB;
    const Geo geo = colproj_geo(mp, K, nb, true);
    if (slab_bytes(geo, nb, r) > ws_bytes || (slab_bytes(geo, nb, r) > 0 && ws == nullptr))
      return fail(DION_E_WORKSPACE, "sketch product needs %zu workspace bytes", slab_bytes(geo, nb, r));
    rc = run_panel(sketch ? 1 : 2, mp, K, r, nb, P + static_cast<long>(b0) * mp * r,
                   sketch ? sketch + static_cast<long>(b0) * K * mp : nullptr,
                   seed + 0x9E3779B97F4A7C15ull * static_cast<uint64_t>(b0), std_,
                   SP + static_cast<long>(b0) * K * r, ws, geo, st, static_cast<long>(row_offset));
    if (rc != DION_OK) return rc;
  }
  return DION_OK;
}

int dion_dortho_qr_inv(int32_t k, int32_t r, int32_t batch, const float* SP, float* R1inv, dion_stream_t stream) {
  if (SP == nullptr || R1inv == nullptr) return fail(DION_E_INVALID, "null argument");
  if (batch < 0 || r <= 0 || r > 128 || k < r || k > 256) return fail(DION_E_UNSUPPORTED, "sketch QR %dx%d", k, r);
  if (batch == 0) return DION_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int b0 = 0; b0 < batch; b0 += 65535) {
    const int nb = batch - b0 < 65535 ? batch - b0 : 65535;
    int rc = launch_sketch_qr_inv(SP + static_cast<long>(b0) * k * r, R1inv + static_cast<long>(b0) * r * r, k, r,
                                  nb, st);
    if (rc != DION_OK) return rc;
  }
  return DION_OK;
}

int dion_dortho_gram(const DionBatchDesc* d, const float* P, float* gram, void* ws, size_t ws_bytes,
                     dion_stream_t stream) {
  int rc = validate_dortho(d);
  if (rc != DION_OK) return rc;
  if (P == nullptr || gram == nullptr) return fail(DION_E_INVALID, "null argument");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int mp = d->transposed ? d->n : d->m;
  const int r = d->r;
  for (int b0 = 0; b0 < d->batch; b0 += MAXB) {
    const int nb = d->batch - b0 < MAXB ? d->batch - b0 : MAXB;
    const Geo geo = colproj_geo(mp, r, nb, true);
    if (slab_bytes(geo, nb, r) > ws_bytes || (slab_bytes(geo, nb, r) > 0 && ws == nullptr))
      return fail(DION_E_WORKSPACE, "Gram product needs %zu workspace bytes", slab_bytes(geo, nb, r));
    rc = run_panel(0, mp, r, r, nb, P + static_cast<long>(b0) * mp * r, nullptr, 0, 0.f,
                   gram + static_cast<long>(b0) * r * r, ws, geo, st);
    if (rc != DION_OK) return rc;
  }
  return DION_OK;
}

int dion_dortho_chol_inv(int32_t r, int32_t batch, const float* gram, float* R2inv, dion_stream_t stream) {
  if (gram == nullptr || R2inv == nullptr) return fail(DION_E_INVALID, "null argument");
  if (batch < 0 || r <= 0 || r > 128) return fail(DION_E_UNSUPPORTED, "Cholesky of %dx%d", r, r);
  if (batch == 0) return DION_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int b0 = 0; b0 < batch; b0 += 65535) {
    const int nb = batch - b0 < 65535 ? batch - b0 : 65535;
    int rc = launch_chol_inv(gram + static_cast<long>(b0) * r * r, R2inv + static_cast<long>(b0) * r * r, r, nb, st);
    if (rc != DION_OK) return rc;
  }
  return DION_OK;
}

int dion_dortho_apply(const DionBatchDesc* d, const float* P_in, const float* Uinv, float* P_out,
                      dion_stream_t stream) {
  int rc = validate_dortho(d);
  if (rc != DION_OK) return rc;
  if (P_in == nullptr || Uinv == nullptr || P_out == nullptr) return fail(DION_E_INVALID, "null argument");
  if (P_in == P_out) return fail(DION_E_INVALID, "P_in and P_out must not alias");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int mp = d->transposed ? d->n : d->m;
  const int r = d->r;
  for (int b0 = 0; b0 < d->batch; b0 += MAXB) {
    const int nb = d->batch - b0 < MAXB ? d->batch - b0 : MAXB;
    rc = apply_right(P_in + static_cast<long>(b0) * mp * r, P_out + static_cast<long>(b0) * mp * r,
                     Uinv + static_cast<long>(b0) * r * r, mp, r, nb, st);
    if (rc != DION_OK) return rc;
  }
  return DION_OK;
}

int dion_fixup_colnorm(const DionBatchDesc* d, float* P, float* R, float* const* Q, const uint32_t* nonzero,
                       float eps, void* ws, size_t ws_bytes, dion_stream_t stream) {
  int rc = validate(d);
  if (rc != DION_OK) return rc;
  if (R == nullptr || Q == nullptr || nonzero == nullptr) return fail(DION_E_INVALID, "null argument");
  if (d->batch == 0) return DION_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int mp = d->transposed ? d->n : d->m;
  const int nq = d->transposed ? d->m : d->n;
  const int r = d->r;
  if (P != nullptr) {  // null: P was fixed by dion_orthonormalize_fused
    rc = launch_pfix(P, nonzero, static_cast<long>(mp) * r, d->batch, st);
    if (rc != DION_OK) return rc;
  }
  for (int b0 = 0; b0 < d->batch; b0 += MAXB) {
    const int nb = d->batch - b0 < MAXB ? d->batch - b0 : MAXB;
    FixArgs a;
    memset(&a, 0, sizeof(a));
    for (int b = 0; b < nb; ++b) {
      if (Q[b0 + b] == nullptr) return fail(DION_E_INVALID, "null Q at %d", b0 + b);
      a.q[b] = Q[b0 + b];
    }
    a.q_bf16 = d->m_dtype == DION_DTYPE_BF16 ? 1 : 0;
    a.R = R + static_cast<long>(b0) * nq * r;
    a.nonzero = nonzero + b0;
    a.nq = nq;
    a.r = r;
    a.tpc = 256 / r;
    a.rows_per_chunk = kFixRows;
    a.nchunk = static_cast<int>(ceil_div(nq, a.rows_per_chunk));
    if (ws_bytes < sizeof(float) * static_cast<size_t>(nb) * a.nchunk * r || ws == nullptr)
      return fail(DION_E_WORKSPACE, "fixup needs %zu workspace bytes", sizeof(float) * static_cast<size_t>(nb) * a.nchunk * r);
    a.part = static_cast<float*>(ws);
    a.eps = eps;
    hipLaunchKernelGGL(fixup_partial_kernel, dim3(a.nchunk, nb), dim3(256), 0, st, a);
    rc = check_launch("fixup_partial");
    if (rc != DION_OK) return rc;
    hipLaunchKernelGGL(colnorm_apply_kernel, dim3(a.nchunk, nb), dim3(256), 0, st, a);
    rc = check_launch("fixup_colnorm");
    if (rc != DION_OK) return rc;
  }
  return DION_OK;
}

int dion_fixup_colsum(const DionBatchDesc* d, float* P, float* R, const void* const* Q, const uint32_t* nonzero,
                      float* colsum, void* ws, size_t ws_bytes, dion_stream_t stream) {
  int rc = validate(d);
  if (rc != DION_OK) return rc;
  if (P == nullptr || R == nullptr || Q == nullptr || nonzero == nullptr || colsum == nullptr)
    return fail(DION_E_INVALID, "null argument");
  if (d->batch == 0) return DION_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int mp = d->transposed ? d->n : d->m;
  const int nq = d->transposed ? d->m : d->n;
  const int r = d->r;
  {
    const long per = static_cast<long>(mp) * r;
    long blocks = ceil_div(per * d->batch, 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(pfix_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, st, P, nonzero, per, d->batch);
    rc = check_launch("pfix");
    if (rc != DION_OK) return rc;
  }
  for (int b0 = 0; b0 < d->batch; b0 += MAXB) {
    const int nb = d->batch - b0 < MAXB ? d->batch - b0 : MAXB;
    FixArgs a;
    memset(&a, 0, sizeof(a));
    for (int b = 0; b < nb; ++b) {
      if (Q[b0 + b] == nullptr) return fail(DION_E_INVALID, "null Q at %d", b0 + b);
      a.q[b] = static_cast<float*>(const_cast<void*>(Q[b0 + b]));
    }
    a.q_bf16 = d->m_dtype == DION_DTYPE_BF16 ? 1 : 0;
    a.R = R + static_cast<long>(b0) * nq * r;
    a.nonzero = nonzero + b0;
    a.nq = nq;
    a.r = r;
    a.tpc = 256 / r;
    a.rows_per_chunk = kFixRows;
    a.nchunk = static_cast<int>(ceil_div(nq, a.rows_per_chunk));
    if (ws_bytes < sizeof(float) * static_cast<size_t>(nb) * a.nchunk * r || ws == nullptr)
      return fail(DION_E_WORKSPACE, "fixup needs %zu workspace bytes", sizeof(float) * static_cast<size_t>(nb) * a.nchunk * r);
    a.part = static_cast<float*>(ws);
    hipLaunchKernelGGL(fixup_partial_kernel, dim3(a.nchunk, nb), dim3(256), 0, st, a);
    rc = check_launch("fixup_partial");
    if (rc != DION_OK) return rc;
    hipLaunchKernelGGL(colsum_reduce_kernel, dim3(nb), dim3(256), 0, st, a, colsum + static_cast<long>(b0) * r);
    rc = check_launch("colsum_reduce");
    if (rc != DION_OK) return rc;
  }
  return DION_OK;
}

int dion_colnorm_apply(const DionBatchDesc* d, const float* R, void* const* Q, const float* colsum, float eps,
                       dion_stream_t stream) {
  int rc = validate(d);
  if (rc != DION_OK) return rc;
  if (R == nullptr || Q == nullptr || colsum == nullptr) return fail(DION_E_INVALID, "null argument");
  if (d->batch == 0) return DION_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int nq = d->transposed ? d->m : d->n;
  const int r = d->r;
  for (int b0 = 0; b0 < d->batch; b0 += MAXB) {
    const int nb = d->batch - b0 < MAXB ? d->batch - b0 : MAXB;
    FixArgs a;
    memset(&a, 0, sizeof(a));
    for (int b = 0; b < nb; ++b) {
      if (Q[b0 + b] == nullptr) return fail(DION_E_INVALID, "null Q at %d", b0 + b);
      a.q[b] = static_cast<float*>(Q[b0 + b]);
    }
    a.q_bf16 = d->m_dtype == DION_DTYPE_BF16 ? 1 : 0;
    a.R = const_cast<float*>(R) + static_cast<long>(b0) * nq * r;
    a.nq = nq;
    a.r = r;
    a.tpc = 256 / r;
    a.rows_per_chunk = kFixRows;
    a.nchunk = static_cast<int>(ceil_div(nq, a.rows_per_chunk));
    a.eps = eps;
    hipLaunchKernelGGL(colnorm_given_kernel, dim3(a.nchunk, nb), dim3(256), 0, st, a,
                       colsum + static_cast<long>(b0) * r);
    rc = check_launch("colnorm_given");
    if (rc != DION_OK) return rc;
  }
  return DION_OK;
}

int dion_ef_apply(const DionBatchDesc* d, float* const* M, float* const* W, const float* P, const float* R,
                  const float* const* Qn, const uint32_t* nonzero, double mu, double lr, double wd,
                  double scaled_lr, void* ws, size_t ws_bytes, dion_stream_t stream) {
  int rc = validate(d);
  if (rc != DION_OK) return rc;
  if (P == nullptr || R == nullptr || Qn == nullptr || nonzero == nullptr || (M == nullptr && W == nullptr))
    return fail(DION_E_INVALID, "null argument");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (d->m_dtype == DION_DTYPE_BF16) {
    // kernels.py:54-83 (bf16): M = rne(M + rne(alpha rne(P R^T)));  runtime.py:1111-1113: W = W d - s rne(P Qn^T)
    const float alpha = static_cast<float>(-(1.0 - mu));
    return b16::update(d, reinterpret_cast<uint16_t* const*>(M), W, P, R,
                       reinterpret_cast<const uint16_t* const*>(Qn), alpha, static_cast<float>(-scaled_lr),
                       (wd > 0.0) ? static_cast<float>(1.0 - lr * wd) : 1.0f, st);
  }
  const int mp = d->transposed ? d->n : d->m;
  const int nq = d->transposed ? d->m : d->n;
  const int r = d->r;
  const int rpad = (r + 1) / 2 * 2;
  for (int b0 = 0; b0 < d->batch; b0 += MAXB) {
    const int nb = d->batch - b0 < MAXB ? d->batch - b0 : MAXB;
    EfArgs a;
    memset(&a, 0, sizeof(a));
    for (int b = 0; b < nb; ++b) {
      a.m[b] = M ? M[b0 + b] : nullptr;
      a.w[b] = W ? W[b0 + b] : nullptr;
      a.qn[b] = Qn[b0 + b];
      if ((M && a.m[b] == nullptr) || a.qn[b] == nullptr || (W && a.w[b] == nullptr))
        return fail(DION_E_INVALID, "null pointer at entry %d", b0 + b);
    }
    a.P = P + static_cast<long>(b0) * mp * r;
    a.R = R + static_cast<long>(b0) * nq * r;
    a.nonzero = nonzero + b0;
    a.rows = d->m;
    a.cols = d->n;
    a.r = r;
    a.transposed = d->transposed;
    a.ld_m = ldv(d->ld_m, d->n);
    a.ld_w = ldv(d->ld_w, d->n);
    a.alpha = static_cast<float>(-(1.0 - mu));
    a.beta = static_cast<float>(-scaled_lr);
    a.decay = (wd > 0.0) ? static_cast<float>(1.0 - lr * wd) : 1.0f;
    a.has_w = W ? 1 : 0;
    const int flen = d->transposed ? d->m : d->n;
    const int slen = d->transposed ? d->n : d->m;
    const dim3 grid(static_cast<unsigned>(ceil_div(flen, 128)), static_cast<unsigned>(ceil_div(slen, kEfStream)), nb);
    bool split_ok = (d->m % 32 == 0) && (d->n % 32 == 0) && (r % 16 == 0) && r <= 128 &&
                    aligned16(a.P) && aligned16(a.R) && (ldv(d->ld_m, d->n) % 4 == 0) &&
                    (W == nullptr || ldv(d->ld_w, d->n) % 4 == 0);
    for (int b = 0; b < nb && split_ok; ++b) split_ok = aligned16(a.qn[b]);
    if (M == nullptr && !split_ok)
      return fail(DION_E_UNSUPPORTED, "weight-only update needs the rank-update kernel (%dx%d r=%d)", d->m, d->n, r);
    if (split_ok) {
      const int s_len = r > 64 ? DION_RSL128 : kRankStreamLen;
      for (int pass = 0; pass < 2; ++pass) {
        if (pass == 1 && W == nullptr) break;
        if (pass == 0 && M == nullptr) continue;
        RankArgs ra;
        memset(&ra, 0, sizeof(ra));
        for (int b = 0; b < nb; ++b) {
          ra.x[b] = pass == 0 ? a.m[b] : a.w[b];
          ra.fixed[b] = pass == 0 ? a.R + static_cast<long>(b) * nq * r : a.qn[b];
        }
        ra.S = a.P;
        ra.s_stride = static_cast<long>(mp) * r;
        ra.s_len = s_len;
        ra.nonzero = a.nonzero;
        ra.rows = d->m;
        ra.cols = d->n;
        ra.ld = pass == 0 ? a.ld_m : a.ld_w;
        ra.scale = pass == 0 ? a.alpha : a.beta;
        ra.decay = pass == 0 ? 1.0f : a.decay;
        ra.skip_zero = pass == 0 ? 1 : 0;
        if (pass == 1) {
          // h3 scales from the factors' bound |P|, |Qn| <= 1 (2 leaves headroom for rounding).
          // Both are powers of two, so x s is exact and each limb pair splits one value; the
          // step's -scaled_lr rides on the final fma instead: W = fma(acc, -s / (s_f s_s), W d),
          // the reference's W.mul_(d) then W.add_(P Qn^T, alpha=-s) (runtime.py:1110-1113).
          // (Folding -s into the fixed factor's split made x s inexact: the compiler then forms
          // the hi limb from the exact product (v_fma_mix) and the lo limb from the rounded
          // one, and where the two roundings differ the pair misses x by an ulp of hi: ~3e-5
          // of max |dW|, tests/test_gpu_update_precision.py.)
          const float sf = h3_scale_host(2.f);
          const float ss = h3_scale_host(2.f);
          ra.h3_fixed_mul = sf;
          ra.h3_stream_scale = ss;
          ra.h3_inv = ra.scale / (sf * ss);
        }
        auto launch = [&](auto RUc) {
          constexpr int RUv = decltype(RUc)::value;
          {
            // rank_stream_kernel: NW-wave blocks share the split streamed factor through LDS
            ra.s_len = s_len;
            // Both orientations run with the 32-wide strips across X's columns and the
            // steps down its rows (a block's accesses are 32 x NW-wide rows of 1 KB runs).
            // Transposed (X += s Fq P^T, Fq = R or Qn indexed by X's rows): the fixed
            // strip factor is P (indexed by X's columns), the staged one Fq; the scale
            // moves with the fixed factor.
            if (d->transposed) {
              for (int b = 0; b < nb; ++b) {
                ra.sptr[b] = ra.fixed[b];
                ra.fixed[b] = a.P + static_cast<long>(b) * mp * r;
              }
            }
            auto go = [&](auto NWc, auto Dc) {
              constexpr int NWv = decltype(NWc)::value, Dv = decltype(Dc)::value;
              const dim3 g2(static_cast<unsigned>(ceil_div(d->n, 32 * NWv)),
                            static_cast<unsigned>(ceil_div(d->m, s_len)), grid.z);
              if (pass == 1 && kRankH3)
                hipLaunchKernelGGL((rank_stream_kernel<RUv, false, NWv, Dv, true>), g2, dim3(64 * NWv), 0, st, ra);
              else
                hipLaunchKernelGGL((rank_stream_kernel<RUv, false, NWv, Dv>), g2, dim3(64 * NWv), 0, st, ra);
            };
            go(std::integral_constant<int, kRankNW>{}, std::integral_constant<int, (RUv >= 8 ? kRankD8 : kRankD)>{});
          }
        };
        switch (r / 16) {
          case 1: launch(std::integral_constant<int, 1>{}); break;
          case 2: launch(std::integral_constant<int, 2>{}); break;
          case 3: launch(std::integral_constant<int, 3>{}); break;
          case 4: launch(std::integral_constant<int, 4>{}); break;
          case 5: launch(std::integral_constant<int, 5>{}); break;
          case 6: launch(std::integral_constant<int, 6>{}); break;
          case 7: launch(std::integral_constant<int, 7>{}); break;
          default: launch(std::integral_constant<int, 8>{}); break;
        }
        rc = check_launch("rank_update");
        if (rc != DION_OK) return rc;
      }
      continue;
    }
    bool fast = (d->m % 32 == 0) && (d->n % 32 == 0) && (r % 4 == 0) && (r % 2 == 0) &&
                (W == nullptr || ldv(d->ld_w, d->n) == ldv(d->ld_m, d->n)) && aligned16(a.P) && aligned16(a.R) &&
                ((static_cast<long>(mp) * r) % 4 == 0) && ((static_cast<long>(nq) * r) % 4 == 0);
    for (int b = 0; b < nb && fast; ++b) fast = aligned16(a.qn[b]);
    const int rhv = rpad / 2;
    const bool exact_rh = (rhv == 4 || rhv == 8 || rhv == 16 || rhv == 32 || rhv == 64);
    auto go = [&](auto RHc) {
      constexpr int RHv = decltype(RHc)::value;
      if (fast && exact_rh && 2 * RHv == r) {
        // two launches over the same grid: entries with a nonzero momentum do EF + W,
        // all-zero entries only decay W (each block exits early in the other launch)
        if (d->transposed) {
          hipLaunchKernelGGL((ef_fast_kernel<RHv, true, true>), grid, dim3(256), 0, st, a);
          hipLaunchKernelGGL((ef_fast_kernel<RHv, true, false>), grid, dim3(256), 0, st, a);
        } else {
          hipLaunchKernelGGL((ef_fast_kernel<RHv, false, true>), grid, dim3(256), 0, st, a);
          hipLaunchKernelGGL((ef_fast_kernel<RHv, false, false>), grid, dim3(256), 0, st, a);
        }
      } else if (d->transposed) {
        hipLaunchKernelGGL((ef_update_kernel<RHv, true, false>), grid, dim3(256), 0, st, a);
      } else {
        hipLaunchKernelGGL((ef_update_kernel<RHv, false, false>), grid, dim3(256), 0, st, a);
      }
    };
    if (rhv <= 4) go(std::integral_constant<int, 4>{});
    else if (rhv <= 8) go(std::integral_constant<int, 8>{});
    else if (rhv <= 16) go(std::integral_constant<int, 16>{});
    else if (rhv <= 32) go(std::integral_constant<int, 32>{});
    else go(std::integral_constant<int, 64>{});
    rc = check_launch("ef_update");
    if (rc != DION_OK) return rc;
  }
  return DION_OK;
}

int dion_round_bf16(float* x, int64_t n, dion_stream_t stream) {
  if (n < 0 || (n > 0 && x == nullptr)) return fail(DION_E_INVALID, "bad buffer (n=%lld)", static_cast<long long>(n));
  return b16::round_buffer(x, static_cast<long>(n), reinterpret_cast<hipStream_t>(stream));
}

int dion_grad_sum_sq(const DionBatchDesc* d, const void* const* G, double* out, void* ws, size_t ws_bytes,
                     dion_stream_t stream) {
  int rc = validate_grads(d);
  if (rc != DION_OK) return rc;
  if (out == nullptr || (d->batch > 0 && G == nullptr)) return fail(DION_E_INVALID, "null argument");
  return gnorm::run(d, G, out, ws, ws_bytes, reinterpret_cast<hipStream_t>(stream));
}

// the host-side scalars follow the reference's Python doubles (elementwise_opts.py:64-78,
// 98-104): bias corrections and 1 - lr wd in double, cast to fp32 once
int dion_elementwise_adamw(int32_t n_tensors, const int64_t* numels, float* const* W, const void* const* G,
                           int32_t g_dtype, int32_t m1_dtype, int32_t m2_dtype, void* const* exp_avg,
                           void* const* exp_avg_sq, double lr, double beta1, double beta2, double weight_decay,
                           double eps, int32_t step, dion_stream_t stream) {
  if (step <= 0) return fail(DION_E_INVALID, "[DION_INVALID_ELEMENTWISE_ADAMW_STEP] step=%d", step);
  const double bc1 = 1.0 - pow(beta1, step);
  const double bc2 = 1.0 - pow(beta2, step);
  return ew::run(n_tensors, numels, W, G, g_dtype, m1_dtype, m2_dtype, exp_avg, exp_avg_sq, false,
                 static_cast<float>(1.0 - beta1),
                 static_cast<float>(1.0 - beta2), static_cast<float>(sqrt(bc2)), static_cast<float>(eps),
                 static_cast<float>(lr / bc1), static_cast<float>(1.0 - lr * weight_decay), weight_decay != 0.0,
                 reinterpret_cast<hipStream_t>(stream));
}

int dion_elementwise_lion(int32_t n_tensors, const int64_t* numels, float* const* W, const void* const* G,
                          int32_t g_dtype, int32_t m_dtype, void* const* exp_avg, double lr, double beta1, double beta2,
                          double weight_decay, dion_stream_t stream) {
  return ew::run(n_tensors, numels, W, G, g_dtype, m_dtype, m_dtype, exp_avg, nullptr, true, static_cast<float>(1.0 - beta1),
                 static_cast<float>(1.0 - beta2), 1.0f, 0.0f, static_cast<float>(lr),
                 static_cast<float>(1.0 - lr * weight_decay), weight_decay != 0.0, reinterpret_cast<hipStream_t>(stream));
}

}  // extern "C"
