// dion_bf16.hpp -- the Dion step with bf16 momentum and bf16 Q (the speedrun's
// mixed precision: examples/dion/speedrun_nanogpt_mcore.py:422-431,
// --dion-momentum-dtype / --dion-q-dtype bfloat16).  Included by dion_codec.hip
// just before the C ABI; the entry points dispatch here when desc->m_dtype is
// DION_DTYPE_BF16.
//
// Reference semantics (all under /root/reference/megatron/core/optimizer/):
//   dion/runtime.py:1560-1566   M += G.to(bf16)                -> rne(M + rne(G))
//   dion/runtime.py:1602-1616   P = M_batch @ Q_batch (bf16)    -> rne(sum_k fp32)
//   dion/ortho.py:90-123        orthogonalize in fp32, cast back -> rne(P)
//   dion/runtime.py:1476-1477   R = M^T @ P (bf16)              -> rne(sum_k fp32)
//   dion/kernels.py:54-83       update = rne(P R^T); update = rne(alpha update); M = rne(M + update)
//   dion/kernels.py:279-290     Qn = rne(R.float() / (sqrt(colsum) + eps))
//   dion/kernels.py:229-276     delta = rne(P Qn^T)  (bf16 bmm)
//   dion/runtime.py:1111-1113   W = W (1 - lr wd);  W += -s delta.float()
// Every bf16 product runs on v_mfma_f32_16x16x32_bf16: exact bf16 x bf16 products
// accumulated in fp32, rounded once to bf16 (round-to-nearest-even) where torch
// rounds its bf16 matmul output.  P and R keep the ABI's fp32 buffers; in this
// mode every value they hold is bf16-representable.
//
// Data layout: M (m x n bf16 row-major, ld_m), Q (n_Q x r bf16 per matrix),
// G bf16 or fp32 (ld_g), W fp32 (ld_w).  The thin operand of a projection (Q or P)
// is first transposed into a (batch, rpad, K) bf16 panel in the workspace so every
// MFMA operand is one 16-byte load.

typedef short bf16x8s __attribute__((ext_vector_type(8)));

// fp32 -> bf16, round to nearest even: v_cvt_pk_bf16_f32 (gfx950; fp32 denormals are kept,
// .amdhsa_float_denorm_mode_32 3, and a NaN stays a quiet NaN -- MI355X_MICROARCH.md), one
// instruction where the integer form takes five
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint16_t f32_to_bf16_rne(float x) { return __builtin_bit_cast(uint16_t, static_cast<__bf16>(x)); }
// two values at once: (lo, hi) -> lo | hi << 16
__device__ __forceinline__ uint32_t f32x2_to_bf16x2_rne(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v{lo, hi}), bf16x2v));
}

__device__ __forceinline__ float bf16_round(float x) { return bf16_to_f32(f32_to_bf16_rne(x)); }

// ----------------------------------------------------------------------------- args
struct B16ProjArgs {
  uint16_t* x[MAXB];     // M (bf16), accumulated in place when g != null
  const void* g[MAXB];   // gradient (bf16 or fp32) or null
  const uint16_t* tt;    // thin operand, transposed: (batch, rpad, K) bf16
  float* slab;           // (batch, nchunk, out_rows, r) fp32 partial sums
  uint32_t* nonzero;     // pass A: nonzero flags (may be null)
  int rows, cols, r, rpad, kchunk, nchunk, out_rows;
  int K, Kp;             // contraction length; row stride of the tt panel (multiple of 32)
  int vec;               // 16-byte X / G accesses allowed (aligned bases, strides multiple of 8)
  long ld_x, ld_g;
};

// one 8-wide bf16 run of X at (row, col..col+7), optionally accumulated with G
// (rne(x + rne(g)), written back); 16-byte accesses when `a.vec` (aligned bases,
// row strides multiple of 8), per-element bounds checks at the ragged edges
template <int GDT>
__device__ __forceinline__ bf16x8s b16_xload(const B16ProjArgs& a, int b, int row, int col, uint32_t& nz) {
  bf16x8s v = {0, 0, 0, 0, 0, 0, 0, 0};
  if (row >= a.rows || col >= a.cols) return v;
  uint16_t* px = a.x[b] + static_cast<long>(row) * a.ld_x + col;
  const bool full = a.vec && (col + 8 <= a.cols);
  uint16_t e[8];
  if (full) {
    const uint4 w = *reinterpret_cast<const uint4*>(px);
    e[0] = w.x & 0xFFFF; e[1] = w.x >> 16; e[2] = w.y & 0xFFFF; e[3] = w.y >> 16;
    e[4] = w.z & 0xFFFF; e[5] = w.z >> 16; e[6] = w.w & 0xFFFF; e[7] = w.w >> 16;
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) e[i] = (col + i < a.cols) ? px[i] : 0;
  }
  if constexpr (GDT != DION_DTYPE_NONE) {
    float gv[8];
    const long go = static_cast<long>(row) * a.ld_g + col;
    if (full) {
      if constexpr (GDT == DION_DTYPE_BF16) {
        const uint4 q = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(a.g[b]) + go);
        const uint32_t qq[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          gv[2 * i] = __uint_as_float(qq[i] << 16);
          gv[2 * i + 1] = __uint_as_float(qq[i] & 0xFFFF0000u);
        }
      } else {
        const f32x4 g0 = *reinterpret_cast<const f32x4*>(static_cast<const float*>(a.g[b]) + go);
        const f32x4 g1 = *reinterpret_cast<const f32x4*>(static_cast<const float*>(a.g[b]) + go + 4);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          gv[i] = bf16_round(g0[i]);
          gv[4 + i] = bf16_round(g1[i]);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        gv[i] = 0.f;
        if (col + i < a.cols) {
          if constexpr (GDT == DION_DTYPE_BF16) gv[i] = bf16_to_f32(static_cast<const uint16_t*>(a.g[b])[go + i]);
          else gv[i] = bf16_round(static_cast<const float*>(a.g[b])[go + i]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) e[i] = f32_to_bf16_rne(bf16_to_f32(e[i]) + gv[i]);
    if (full) {
      uint4 w;
      w.x = e[0] | (static_cast<uint32_t>(e[1]) << 16); w.y = e[2] | (static_cast<uint32_t>(e[3]) << 16);
      w.z = e[4] | (static_cast<uint32_t>(e[5]) << 16); w.w = e[6] | (static_cast<uint32_t>(e[7]) << 16);
      *reinterpret_cast<uint4*>(px) = w;
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (col + i < a.cols) px[i] = e[i];
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    nz |= (col + i < a.cols) ? (e[i] & 0x7FFFu) : 0u;
    v[i] = static_cast<short>(e[i]);
  }
  return v;
}

__device__ __forceinline__ bf16x8s b16_tload(const uint16_t* tt, int Kp, int c, int k) {
  // panel rows are Kp (a multiple of 32) long and zero past K: 16-byte aligned runs
  return *reinterpret_cast<const bf16x8s*>(tt + static_cast<long>(c) * Kp + k);
}

constexpr int kB16RW = 4;                // 16-row output blocks per wave
constexpr int kB16BO = 64 * kB16RW;      // output rows per block (4 waves)

// out = X T (row mode: out_rows = rows, K = cols) or X^T T (column mode:
// out_rows = cols, K = rows).  Block = 4 waves x 4 x 16 output rows, blockIdx.y =
// K-chunk, blockIdx.z = matrix; each K-step's thin-operand run is loaded once per
// wave and reused by its 4 row blocks.  Row mode reads its MFMA A operand straight
// from X (8 consecutive columns per lane); column mode stages a 32 x 256 tile of X
// through LDS (512-byte row segments in, one column per lane out).
template <bool COL, int RB, int GDT>
__global__ void __launch_bounds__(256) b16_proj_kernel(const B16ProjArgs a) {
  constexpr int RW = kB16RW, BO = kB16BO;
  __shared__ uint16_t tile[COL ? 32 : 1][COL ? BO + 8 : 1];
  const int b = blockIdx.z, kc = blockIdx.y;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int t = lane & 15, g = lane >> 4;
  const int o0 = blockIdx.x * BO + wave * 16 * RW;  // first output row of this wave
  const int k_begin = kc * a.kchunk;
  const int k_end = min(a.K, k_begin + a.kchunk);
  const uint16_t* tt = a.tt + static_cast<long>(b) * a.rpad * a.Kp;
  f32x4 acc[RW][RB];
#pragma unroll
  for (int rw = 0; rw < RW; ++rw)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) acc[rw][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint32_t nz = 0;
  for (int k0 = k_begin; k0 < k_end; k0 += 32) {
    bf16x8s A[RW];
    if constexpr (!COL) {
      // chunk bounds are multiples of 32, so an 8-run never straddles two chunks
      // (each element is accumulated by exactly one block)
#pragma unroll
      for (int rw = 0; rw < RW; ++rw) {
        A[rw] = bf16x8s{0, 0, 0, 0, 0, 0, 0, 0};
        if (k0 + 8 * g < k_end) A[rw] = b16_xload<GDT>(a, b, o0 + 16 * rw + t, k0 + 8 * g, nz);
      }
    } else {
      // tile rows = X rows k0 .. k0+31, tile columns = X columns blockIdx.x*BO .. +BO-1
#pragma unroll
      for (int it = 0; it < (32 * BO / 8) / 256; ++it) {
        const int chunk = tid + 256 * it;
        const int tr = chunk / (BO / 8), tc = (chunk % (BO / 8)) * 8;
        bf16x8s v = bf16x8s{0, 0, 0, 0, 0, 0, 0, 0};
        if (k0 + tr < k_end) v = b16_xload<GDT>(a, b, k0 + tr, blockIdx.x * BO + tc, nz);
        *reinterpret_cast<bf16x8s*>(&tile[tr][tc]) = v;
      }
      __syncthreads();
#pragma unroll
      for (int rw = 0; rw < RW; ++rw)
#pragma unroll
        for (int i = 0; i < 8; ++i) A[rw][i] = static_cast<short>(tile[8 * g + i][wave * 16 * RW + 16 * rw + t]);
      __syncthreads();
    }
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) {
      const bf16x8s B = (k0 + 8 * g < k_end) ? b16_tload(tt, a.Kp, 16 * cb + t, k0 + 8 * g)
                                             : bf16x8s{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int rw = 0; rw < RW; ++rw) acc[rw][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[rw], B, acc[rw][cb], 0, 0, 0);
    }
  }
  float* out = a.slab + (static_cast<long>(b) * a.nchunk + kc) * a.out_rows * a.r;
#pragma unroll
  for (int rw = 0; rw < RW; ++rw)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int orow = o0 + 16 * rw + 4 * g + q, c = 16 * cb + t;
        if (orow < a.out_rows && c < a.r) out[static_cast<long>(orow) * a.r + c] = acc[rw][cb][q];
      }
  if (a.nonzero != nullptr && __any(nz != 0u) && lane == 0) atomicMax(&a.nonzero[b], kAbsUnknown);
}

// tt[b][c][k] = c < r ? bf16(T_b[k][c]) : 0  for k < K (zero up to the stride Kp)
struct B16ThinArgs {
  const void* src[MAXB];  // per matrix: K x r, bf16 (src_bf16) or fp32
  uint16_t* tt;
  int K, Kp, r, rpad, src_bf16;
};

// one 64 (k) x 64 (c) tile per block through LDS: coalesced row reads of T (c contiguous),
// coalesced row writes of tt (k contiguous)
__global__ void __launch_bounds__(256) b16_thin_kernel(const B16ThinArgs a) {
  __shared__ uint16_t tile[64][66];
  const int b = blockIdx.z;
  const int k0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const int tid = threadIdx.x;
#pragma unroll 4
  for (int i = tid; i < 64 * 64; i += 256) {
    const int kk = i >> 6, cc = i & 63, k = k0 + kk, c = c0 + cc;
    uint16_t v = 0;
    if (c < a.r && k < a.K) {
      const long s = static_cast<long>(k) * a.r + c;
      v = a.src_bf16 ? static_cast<const uint16_t*>(a.src[b])[s] : f32_to_bf16_rne(static_cast<const float*>(a.src[b])[s]);
    }
    tile[kk][cc] = v;
  }
  __syncthreads();
  uint16_t* tt = a.tt + static_cast<long>(b) * a.rpad * a.Kp;
#pragma unroll 4
  for (int i = tid; i < 64 * 64; i += 256) {
    const int cc = i >> 6, kk = i & 63, c = c0 + cc, k = k0 + kk;
    if (c < a.rpad && k < a.Kp) tt[static_cast<long>(c) * a.Kp + k] = tile[kk][cc];
  }
}

// out[b][e] = rne_bf16(sum_k slab[b][k][e]) in fixed k order
__global__ void __launch_bounds__(256) b16_reduce_round_kernel(float* __restrict__ out, const float* __restrict__ slab,
                                                               int nchunk, long per_entry, int batch) {
  const long total = per_entry * batch;
  for (long idx = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; idx < total;
       idx += static_cast<long>(gridDim.x) * blockDim.x) {
    const long b = idx / per_entry, e = idx - b * per_entry;
    const float* s = slab + b * nchunk * per_entry + e;
    float v = 0.f;
    for (int k = 0; k < nchunk; ++k) v += s[k * per_entry];
    out[idx] = bf16_round(v);
  }
}

__global__ void __launch_bounds__(256) b16_round_kernel(float* __restrict__ x, long n) {
  for (long i = static_cast<long>(blockIdx.x) * 256 + threadIdx.x; i < n; i += static_cast<long>(gridDim.x) * 256)
    x[i] = bf16_round(x[i]);
}

// ----------------------------------------------------------------------------- streaming projections
// The two projection geometries for shapes made of whole blocks (b16_fast_*_ok), HBM-bound:
// every M / G access is a whole 128-byte line with the non-temporal policy, the next step's
// lines are in flight while a step computes (register double buffer), and the thin operand's
// 32-k run of every 16-column block is staged ONCE per block per step in LDS, in the MFMA
// operand order (double-buffered, one barrier per step).  The thin operand is the MFMA A
// operand (lane (t, g): T column 16 cb + t, k-run 8 g .. 8 g + 7, from the tt panel), X the
// B operand, so D[T column][X row / column] lands as four consecutive output values per lane.
// Same per-element arithmetic as b16_proj_kernel: M = rne(M + G), exact bf16 products summed
// in fp32 (in MFMA order), the K-chunk slabs summed in fixed order and rounded once.
constexpr int kB16RowBlk = 128;  // row mode: 4 waves x 32 rows per block, 64-column steps
constexpr int kB16ColBlk = 256;  // column mode: 4 waves x 64 columns per block, 32-row steps

__device__ __forceinline__ uint32_t b16_add2(uint32_t m, uint32_t g) {
  return f32x2_to_bf16x2_rne(__uint_as_float(m << 16) + __uint_as_float(g << 16),
                             __uint_as_float(m & 0xFFFF0000u) + __uint_as_float(g & 0xFFFF0000u));
}

// one step's thin-operand runs: item (s, cb, lane) = tt[16 cb + lane % 16][k0 + 32 s + 8 (lane / 16) ..]
template <int NS, int RB>
struct B16Stage {
  static constexpr int kItems = NS * RB * 64;
  static constexpr int kPer = (kItems + 255) / 256;
  u32x4 v[kPer];
  __device__ __forceinline__ void load(const uint16_t* tt, long Kp, int k0, int tid) {
#pragma unroll
    for (int it = 0; it < kPer; ++it) {
      const int item = tid + 256 * it;
      if (kItems % 256 == 0 || item < kItems) {
        const int s = item / (RB * 64), rem = item - s * (RB * 64), cb = rem >> 6, ln = rem & 63;
        v[it] = *reinterpret_cast<const u32x4*>(tt + static_cast<long>(16 * cb + (ln & 15)) * Kp + k0 + 32 * s +
                                                8 * (ln >> 4));
      }
    }
  }
  __device__ __forceinline__ void store(u32x4* dst, int tid) const {
#pragma unroll
    for (int it = 0; it < kPer; ++it) {
      const int item = tid + 256 * it;
      if (kItems % 256 == 0 || item < kItems) dst[item] = v[it];
    }
  }
};

// row mode: out (rows, r) = X (rows x K) T; wave = 32 rows, step = 64 columns.  Lane l loads
// row 8 q + l / 8, 16 bytes at column 8 (l % 8) of the step (four instructions, each 8 whole
// lines); the operand layout (lane (t, g): row t, columns 8 g ..) comes from the wave's LDS
// tile (xt_swz swizzle, conflict-free reads).
template <int RB, int GDT>
__global__ void __launch_bounds__(256, 2) b16_row_kernel(const B16ProjArgs a) {
  constexpr int NI = 2 * RB * 64;
  __shared__ u32x4 tp[2][NI];
  __shared__ u32x4 xt[4][32 * 8];
  const BlockXYZ blk = xcd_block();
  const int b = blk.z, kc = blk.y;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int t = lane & 15, g = lane >> 4;
  const int lr = lane >> 3, lc = lane & 7;
  const int r0 = blk.x * kB16RowBlk + wave * 32;
  const int k_begin = kc * a.kchunk, k_end = min(a.K, k_begin + a.kchunk);
  uint16_t* X = a.x[b] + static_cast<long>(r0 + lr) * a.ld_x + 8 * lc;
  const uint16_t* G = GDT == DION_DTYPE_BF16
                          ? static_cast<const uint16_t*>(a.g[b]) + static_cast<long>(r0 + lr) * a.ld_g + 8 * lc
                          : nullptr;
  const uint16_t* tt = a.tt + static_cast<long>(b) * a.rpad * a.Kp;
  u32x4 xs[2][4], gs[2][4];
  auto load = [&](int s, int j) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      xs[s][q] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(X + static_cast<long>(8 * q) * a.ld_x + j));
      if constexpr (GDT == DION_DTYPE_BF16)
        gs[s][q] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(G + static_cast<long>(8 * q) * a.ld_g + j));
    }
  };
  f32x4 acc[2][RB];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) acc[rb][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint32_t nz = 0;
  B16Stage<2, RB> T;
  if (k_begin < k_end) {
    load(0, k_begin);
    T.load(tt, a.Kp, k_begin, tid);
    T.store(tp[0], tid);
  }
  __syncthreads();
  // one 64-column step on ring slot S (a compile-time index: the two-step loop body below)
  auto step = [&](auto Sc, int j, int cur) -> bool {
    constexpr int S = decltype(Sc)::value;
    const bool more = j + 64 < k_end;
    if (more) {
      T.load(tt, a.Kp, j + 64, tid);
      load(S ^ 1, j + 64);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if constexpr (GDT == DION_DTYPE_BF16) {
        u32x4 o;
#pragma unroll
        for (int d = 0; d < 4; ++d) o[d] = b16_add2(xs[S][q][d], gs[S][q][d]);
        xs[S][q] = o;
        __builtin_nontemporal_store(o, reinterpret_cast<u32x4*>(X + static_cast<long>(8 * q) * a.ld_x + j));
      }
      nz |= (xs[S][q][0] | xs[S][q][1] | xs[S][q][2] | xs[S][q][3]) & 0x7FFF7FFFu;
    }
    u32x4* xw = xt[wave];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = 8 * q + lr;
      xw[row * 8 + (lc ^ xt_swz(row))] = xs[S][q];
    }
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      bf16x8s B[2];
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        const int row = 16 * rb + t;
        B[rb] = __builtin_bit_cast(bf16x8s, xw[row * 8 + ((4 * ss + g) ^ xt_swz(row))]);
      }
#pragma unroll
      for (int cb = 0; cb < RB; ++cb) {
        const bf16x8s A = __builtin_bit_cast(bf16x8s, tp[cur][(ss * RB + cb) * 64 + lane]);
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, B[rb], acc[rb][cb], 0, 0, 0);
      }
    }
    if (!more) return false;
    T.store(tp[cur ^ 1], tid);
    __syncthreads();
    return true;
  };
  for (int j = k_begin; j < k_end; j += 128) {
    if (!step(std::integral_constant<int, 0>{}, j, 0)) break;
    if (!step(std::integral_constant<int, 1>{}, j + 64, 1)) break;
  }
  // lane (t, g): rows 16 rb + t, T columns 16 cb + 4 g .. + 3
  float* out = a.slab + (static_cast<long>(b) * a.nchunk + kc) * a.out_rows * a.r;
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb)
      *reinterpret_cast<f32x4*>(out + static_cast<long>(r0 + 16 * rb + t) * a.r + 16 * cb + 4 * g) = acc[rb][cb];
  if (a.nonzero != nullptr && __any(nz != 0u) && lane == 0) atomicMax(&a.nonzero[b], kAbsUnknown);
}

// column mode: out (cols, r) = X^T T, X rows = K; wave = 64 columns, step = 32 rows.  Lane
// (t, g) loads columns 4 t .. 4 t + 3 of the wave's 64 (8 bytes) of rows 8 g + e, e < 8
// (eight instructions, each 4 whole lines); the B operand of column c is the lane's 8 rows
// of that column, regrouped in registers (16-bit lanes of the 8 loads).
template <int RB, int GDT>
__global__ void __launch_bounds__(256, 2) b16_col_kernel(const B16ProjArgs a) {
  constexpr int NI = RB * 64;
  __shared__ u32x4 tp[2][NI];
  const BlockXYZ blk = xcd_block();
  const int b = blk.z, kc = blk.y;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int t = lane & 15, g = lane >> 4;
  const int c0 = blk.x * kB16ColBlk + wave * 64 + 4 * t;
  const int k_begin = kc * a.kchunk, k_end = min(a.K, k_begin + a.kchunk);
  uint16_t* X = a.x[b] + static_cast<long>(8 * g) * a.ld_x + c0;
  const uint16_t* G = GDT == DION_DTYPE_BF16
                          ? static_cast<const uint16_t*>(a.g[b]) + static_cast<long>(8 * g) * a.ld_g + c0
                          : nullptr;
  const uint16_t* tt = a.tt + static_cast<long>(b) * a.rpad * a.Kp;
  u32x2_ xs[2][8], gs[2][8];
  auto load = [&](int s, int i) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      xs[s][e] = __builtin_nontemporal_load(reinterpret_cast<const u32x2_*>(X + static_cast<long>(i + e) * a.ld_x));
      if constexpr (GDT == DION_DTYPE_BF16)
        gs[s][e] = __builtin_nontemporal_load(reinterpret_cast<const u32x2_*>(G + static_cast<long>(i + e) * a.ld_g));
    }
  };
  f32x4 acc[4][RB];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) acc[c][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint32_t nz = 0;
  B16Stage<1, RB> T;
  if (k_begin < k_end) {
    load(0, k_begin);
    T.load(tt, a.Kp, k_begin, tid);
    T.store(tp[0], tid);
  }
  __syncthreads();
  auto step = [&](auto Sc, int i, int cur) -> bool {
    constexpr int S = decltype(Sc)::value;
    const bool more = i + 32 < k_end;
    if (more) {
      T.load(tt, a.Kp, i + 32, tid);
      load(S ^ 1, i + 32);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if constexpr (GDT == DION_DTYPE_BF16) {
        const u32x2_ o{b16_add2(xs[S][e][0], gs[S][e][0]), b16_add2(xs[S][e][1], gs[S][e][1])};
        xs[S][e] = o;
        __builtin_nontemporal_store(o, reinterpret_cast<u32x2_*>(X + static_cast<long>(i + e) * a.ld_x));
      }
      nz |= (xs[S][e][0] | xs[S][e][1]) & 0x7FFF7FFFu;
    }
    // column c of the lane's 8 rows: 16-bit lane c % 2 of dword c / 2 of each row's load
    bf16x8s B[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      u32x4 v;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const uint32_t x0 = xs[S][2 * d][c >> 1], x1 = xs[S][2 * d + 1][c >> 1];
        v[d] = (c & 1) ? ((x0 >> 16) | (x1 & 0xFFFF0000u)) : ((x0 & 0xFFFFu) | (x1 << 16));
      }
      B[c] = __builtin_bit_cast(bf16x8s, v);
    }
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) {
      const bf16x8s A = __builtin_bit_cast(bf16x8s, tp[cur][cb * 64 + lane]);
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, B[c], acc[c][cb], 0, 0, 0);
    }
    if (!more) return false;
    T.store(tp[cur ^ 1], tid);
    __syncthreads();
    return true;
  };
  for (int i = k_begin; i < k_end; i += 64) {
    if (!step(std::integral_constant<int, 0>{}, i, 0)) break;
    if (!step(std::integral_constant<int, 1>{}, i + 32, 1)) break;
  }
  // lane (t, g): output rows (X columns) c0 + c, T columns 16 cb + 4 g .. + 3
  float* out = a.slab + (static_cast<long>(b) * a.nchunk + kc) * a.out_rows * a.r;
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb)
      *reinterpret_cast<f32x4*>(out + static_cast<long>(c0 + c) * a.r + 16 * cb + 4 * g) = acc[c][cb];
  if (a.nonzero != nullptr && __any(nz != 0u) && lane == 0) atomicMax(&a.nonzero[b], kAbsUnknown);
}

// ----------------------------------------------------------------------------- deferred EF
// The previous step's error feedback folded into this step's pass A (the fp32 mode's
// schedule, dion_project_p_ef): for every element, before the gradient,
//   M = rne(M + rne(alpha rne(u))),  u = sum_c P'[i][c] R'[j][c]   (R'[i] P'[j] transposed)
// -- the eager update's formula (b16_ef, kernels.py:54-83) on the same M value, applied one
// pass later -- then M = rne(M + rne(G)) and P = rne(X Q) as in b16_row_kernel / b16_col_kernel.
// The step's u tile comes from v_mfma_f32_16x16x32_bf16 (exact bf16 products summed in fp32;
// K = r in steps of 32), is rounded to the bf16 EF increment in the MFMA layout, and reaches
// the load layout of M through the wave's LDS tile.  P' and R' are the bf16 panels the host
// packs from the pending fp32 buffers (bf16 values).  Saves the eager update's M read + write
// (4 of 20 bytes per element).
struct B16EfArgs {
  B16ProjArgs p;
  const uint16_t* ep;  // (batch, m_P, r) bf16: P' of each entry's pending error feedback
  const uint16_t* er;  // (batch, n_Q, r) bf16: R'
  int has[MAXB];       // entry has a pending error feedback
  float alpha;
};

// one step's R' fragments: item (nb, kk, lane) = er[(j0 + 16 nb + lane % 16) r + 32 kk + 8 (lane / 16) ..]
template <int NB, int KK>
struct B16EfStage {
  static constexpr int kItems = NB * KK * 64;
  static constexpr int kPer = (kItems + 255) / 256;
  u32x4 v[kPer];
  __device__ __forceinline__ void load(const uint16_t* er, int r, int j0, int tid) {
#pragma unroll
    for (int it = 0; it < kPer; ++it) {
      const int item = tid + 256 * it;
      if (kItems % 256 == 0 || item < kItems) {
        const int nb = item / (KK * 64), rem = item - nb * (KK * 64), kk = rem >> 6, ln = rem & 63;
        v[it] = *reinterpret_cast<const u32x4*>(er + static_cast<long>(j0 + 16 * nb + (ln & 15)) * r + 32 * kk +
                                                8 * (ln >> 4));
      }
    }
  }
  __device__ __forceinline__ void store(u32x4* dst, int tid) const {
#pragma unroll
    for (int it = 0; it < kPer; ++it) {
      const int item = tid + 256 * it;
      if (kItems % 256 == 0 || item < kItems) dst[item] = v[it];
    }
  }
};

// the EF increments of four accumulator values, packed: rne(alpha rne(u))
__device__ __forceinline__ u32x2_ b16_ef_pack(const f32x4& u, float alpha) {
  const uint32_t r01 = f32x2_to_bf16x2_rne(u[0], u[1]), r23 = f32x2_to_bf16x2_rne(u[2], u[3]);
  return u32x2_{f32x2_to_bf16x2_rne(alpha * __uint_as_float(r01 << 16), alpha * __uint_as_float(r01 & 0xFFFF0000u)),
                f32x2_to_bf16x2_rne(alpha * __uint_as_float(r23 << 16), alpha * __uint_as_float(r23 & 0xFFFF0000u))};
}

// row mode (not transposed): b16_row_kernel + the EF.  u's lane (t, g) of tile (rb, jb) is
// row 16 rb + t, columns 16 jb + 4 g .. + 3 of the wave's 32 x 64 step (D = R'_tile P'_tile^T:
// A = R' rows of the step's columns, staged per step; B = P' of the wave's rows, in registers);
// it goes into the transpose tile xt (16-B slots, 8-B halves) and comes back in the load layout.
template <int RB, int GDT>
__global__ void __launch_bounds__(256, 2) b16_row_ef_kernel(const B16EfArgs e) {
  const B16ProjArgs& a = e.p;
  constexpr int KK = RB / 2;
  constexpr int NI = 2 * RB * 64;
  constexpr int NE = 4 * KK * 64;
  __shared__ u32x4 tp[2][NI];
  __shared__ u32x4 rs[2][NE];
  __shared__ u32x4 xt[4][32 * 8];
  const BlockXYZ blk = xcd_block();
  const int b = blk.z, kc = blk.y;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int t = lane & 15, g = lane >> 4;
  const int lr = lane >> 3, lc = lane & 7;
  const int r0 = blk.x * kB16RowBlk + wave * 32;
  const int k_begin = kc * a.kchunk, k_end = min(a.K, k_begin + a.kchunk);
  uint16_t* X = a.x[b] + static_cast<long>(r0 + lr) * a.ld_x + 8 * lc;
  const uint16_t* G = GDT == DION_DTYPE_BF16
                          ? static_cast<const uint16_t*>(a.g[b]) + static_cast<long>(r0 + lr) * a.ld_g + 8 * lc
                          : nullptr;
  const uint16_t* tt = a.tt + static_cast<long>(b) * a.rpad * a.Kp;
  const bool ef_on = e.has[b] != 0;  // uniform over the block
  const uint16_t* er = e.er + static_cast<long>(b) * a.cols * a.r;
  bf16x8s Pf[2][KK];
  if (ef_on) {
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
        Pf[rb][kk] = *reinterpret_cast<const bf16x8s*>(e.ep + (static_cast<long>(b) * a.rows + r0 + 16 * rb + t) * a.r +
                                                       32 * kk + 8 * g);
  }
  u32x4 xs[2][4], gs[2][4];
  auto load = [&](int s, int j) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      xs[s][q] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(X + static_cast<long>(8 * q) * a.ld_x + j));
      if constexpr (GDT == DION_DTYPE_BF16)
        gs[s][q] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(G + static_cast<long>(8 * q) * a.ld_g + j));
    }
  };
  f32x4 acc[2][RB];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) acc[rb][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint32_t nz = 0;
  B16Stage<2, RB> T;
  B16EfStage<4, KK> RS;
  if (k_begin < k_end) {
    load(0, k_begin);
    T.load(tt, a.Kp, k_begin, tid);
    T.store(tp[0], tid);
    if (ef_on) {
      RS.load(er, a.r, k_begin, tid);
      RS.store(rs[0], tid);
    }
  }
  __syncthreads();
  auto step = [&](auto Sc, int j, int cur) -> bool {
    constexpr int S = decltype(Sc)::value;
    const bool more = j + 64 < k_end;
    if (more) {
      T.load(tt, a.Kp, j + 64, tid);
      if (ef_on) RS.load(er, a.r, j + 64, tid);
      load(S ^ 1, j + 64);
    }
    u32x4* xw = xt[wave];
    if (ef_on) {
      u32x2_* xe = reinterpret_cast<u32x2_*>(xw);
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) {
          f32x4 u = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kk = 0; kk < KK; ++kk)
            u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8s, rs[cur][(jb * KK + kk) * 64 + lane]),
                                                        Pf[rb][kk], u, 0, 0, 0);
          const int row = 16 * rb + t, cg = 2 * jb + (g >> 1);
          xe[(row * 8 + (cg ^ xt_swz(row))) * 2 + (g & 1)] = b16_ef_pack(u, e.alpha);
        }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 8 * q + lr;
        const u32x4 ev = xw[row * 8 + (lc ^ xt_swz(row))];
#pragma unroll
        for (int d = 0; d < 4; ++d) xs[S][q][d] = b16_add2(xs[S][q][d], ev[d]);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if constexpr (GDT == DION_DTYPE_BF16) {
        u32x4 o;
#pragma unroll
        for (int d = 0; d < 4; ++d) o[d] = b16_add2(xs[S][q][d], gs[S][q][d]);
        xs[S][q] = o;
      }
      if (GDT == DION_DTYPE_BF16 || ef_on)
        __builtin_nontemporal_store(xs[S][q], reinterpret_cast<u32x4*>(X + static_cast<long>(8 * q) * a.ld_x + j));
      nz |= (xs[S][q][0] | xs[S][q][1] | xs[S][q][2] | xs[S][q][3]) & 0x7FFF7FFFu;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = 8 * q + lr;
      xw[row * 8 + (lc ^ xt_swz(row))] = xs[S][q];
    }
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      bf16x8s B[2];
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        const int row = 16 * rb + t;
        B[rb] = __builtin_bit_cast(bf16x8s, xw[row * 8 + ((4 * ss + g) ^ xt_swz(row))]);
      }
#pragma unroll
      for (int cb = 0; cb < RB; ++cb) {
        const bf16x8s A = __builtin_bit_cast(bf16x8s, tp[cur][(ss * RB + cb) * 64 + lane]);
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, B[rb], acc[rb][cb], 0, 0, 0);
      }
    }
    if (!more) return false;
    T.store(tp[cur ^ 1], tid);
    if (ef_on) RS.store(rs[cur ^ 1], tid);
    __syncthreads();
    return true;
  };
  for (int j = k_begin; j < k_end; j += 128) {
    if (!step(std::integral_constant<int, 0>{}, j, 0)) break;
    if (!step(std::integral_constant<int, 1>{}, j + 64, 1)) break;
  }
  float* out = a.slab + (static_cast<long>(b) * a.nchunk + kc) * a.out_rows * a.r;
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb)
      *reinterpret_cast<f32x4*>(out + static_cast<long>(r0 + 16 * rb + t) * a.r + 16 * cb + 4 * g) = acc[rb][cb];
  if (a.nonzero != nullptr && __any(nz != 0u) && lane == 0) atomicMax(&a.nonzero[b], kAbsUnknown);
}

// column mode (transposed storage): b16_col_kernel + the EF.  u = R'[i] P'[j]: D = P'_tile
// R'_tile^T (A = P' of the wave's 64 columns, in registers; B = R' rows of the step, staged);
// lane (t, g) of tile (ib, jb) holds row 16 ib + t, columns 16 jb + 4 g .. + 3, written to the
// wave's padded LDS tile and read back as the load layout's rows 8 g + e, columns 4 t .. + 3.
constexpr int kB16EfLd = 17;  // u32x2 slots per row of the column kernel's EF tile (16 + 1 pad)
template <int RB, int GDT>
__global__ void __launch_bounds__(256, 2) b16_col_ef_kernel(const B16EfArgs e) {
  const B16ProjArgs& a = e.p;
  constexpr int KK = RB / 2;
  constexpr int NI = RB * 64;
  constexpr int NE = 2 * KK * 64;
  __shared__ u32x4 tp[2][NI];
  __shared__ u32x4 rs[2][NE];
  __shared__ u32x2_ et[4][32 * kB16EfLd];
  const BlockXYZ blk = xcd_block();
  const int b = blk.z, kc = blk.y;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int t = lane & 15, g = lane >> 4;
  const int wc = blk.x * kB16ColBlk + wave * 64;
  const int c0 = wc + 4 * t;
  const int k_begin = kc * a.kchunk, k_end = min(a.K, k_begin + a.kchunk);
  uint16_t* X = a.x[b] + static_cast<long>(8 * g) * a.ld_x + c0;
  const uint16_t* G = GDT == DION_DTYPE_BF16
                          ? static_cast<const uint16_t*>(a.g[b]) + static_cast<long>(8 * g) * a.ld_g + c0
                          : nullptr;
  const uint16_t* tt = a.tt + static_cast<long>(b) * a.rpad * a.Kp;
  const bool ef_on = e.has[b] != 0;
  const uint16_t* er = e.er + static_cast<long>(b) * a.rows * a.r;
  bf16x8s Pf[4][KK];
  if (ef_on) {
#pragma unroll
    for (int jb = 0; jb < 4; ++jb)
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
        Pf[jb][kk] = *reinterpret_cast<const bf16x8s*>(e.ep + (static_cast<long>(b) * a.cols + wc + 16 * jb + t) * a.r +
                                                       32 * kk + 8 * g);
  }
  u32x2_ xs[2][8], gs[2][8];
  auto load = [&](int s, int i) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      xs[s][q] = __builtin_nontemporal_load(reinterpret_cast<const u32x2_*>(X + static_cast<long>(i + q) * a.ld_x));
      if constexpr (GDT == DION_DTYPE_BF16)
        gs[s][q] = __builtin_nontemporal_load(reinterpret_cast<const u32x2_*>(G + static_cast<long>(i + q) * a.ld_g));
    }
  };
  f32x4 acc[4][RB];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) acc[c][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint32_t nz = 0;
  B16Stage<1, RB> T;
  B16EfStage<2, KK> RS;
  if (k_begin < k_end) {
    load(0, k_begin);
    T.load(tt, a.Kp, k_begin, tid);
    T.store(tp[0], tid);
    if (ef_on) {
      RS.load(er, a.r, k_begin, tid);
      RS.store(rs[0], tid);
    }
  }
  __syncthreads();
  auto step = [&](auto Sc, int i, int cur) -> bool {
    constexpr int S = decltype(Sc)::value;
    const bool more = i + 32 < k_end;
    if (more) {
      T.load(tt, a.Kp, i + 32, tid);
      if (ef_on) RS.load(er, a.r, i + 32, tid);
      load(S ^ 1, i + 32);
    }
    if (ef_on) {
      u32x2_* ew = et[wave];
#pragma unroll
      for (int ib = 0; ib < 2; ++ib)
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) {
          f32x4 u = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kk = 0; kk < KK; ++kk)
            u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Pf[jb][kk],
                                                        __builtin_bit_cast(bf16x8s, rs[cur][(ib * KK + kk) * 64 + lane]), u,
                                                        0, 0, 0);
          ew[(16 * ib + t) * kB16EfLd + 4 * jb + g] = b16_ef_pack(u, e.alpha);
        }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const u32x2_ ev = ew[(8 * g + q) * kB16EfLd + t];
        xs[S][q] = u32x2_{b16_add2(xs[S][q][0], ev[0]), b16_add2(xs[S][q][1], ev[1])};
      }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if constexpr (GDT == DION_DTYPE_BF16)
        xs[S][q] = u32x2_{b16_add2(xs[S][q][0], gs[S][q][0]), b16_add2(xs[S][q][1], gs[S][q][1])};
      if (GDT == DION_DTYPE_BF16 || ef_on)
        __builtin_nontemporal_store(xs[S][q], reinterpret_cast<u32x2_*>(X + static_cast<long>(i + q) * a.ld_x));
      nz |= (xs[S][q][0] | xs[S][q][1]) & 0x7FFF7FFFu;
    }
    bf16x8s B[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      u32x4 v;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const uint32_t x0 = xs[S][2 * d][c >> 1], x1 = xs[S][2 * d + 1][c >> 1];
        v[d] = (c & 1) ? ((x0 >> 16) | (x1 & 0xFFFF0000u)) : ((x0 & 0xFFFFu) | (x1 << 16));
      }
      B[c] = __builtin_bit_cast(bf16x8s, v);
    }
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) {
      const bf16x8s A = __builtin_bit_cast(bf16x8s, tp[cur][cb * 64 + lane]);
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, B[c], acc[c][cb], 0, 0, 0);
    }
    if (!more) return false;
    T.store(tp[cur ^ 1], tid);
    if (ef_on) RS.store(rs[cur ^ 1], tid);
    __syncthreads();
    return true;
  };
  for (int i = k_begin; i < k_end; i += 64) {
    if (!step(std::integral_constant<int, 0>{}, i, 0)) break;
    if (!step(std::integral_constant<int, 1>{}, i + 32, 1)) break;
  }
  float* out = a.slab + (static_cast<long>(b) * a.nchunk + kc) * a.out_rows * a.r;
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb)
      *reinterpret_cast<f32x4*>(out + static_cast<long>(c0 + c) * a.r + 16 * cb + 4 * g) = acc[c][cb];
  if (a.nonzero != nullptr && __any(nz != 0u) && lane == 0) atomicMax(&a.nonzero[b], kAbsUnknown);
}

// fp32 buffers of bf16 values -> bf16 panels (exact), entries with a null source skipped
struct B16PackArgs {
  const float* src[2 * MAXB];
  uint16_t* dst[2 * MAXB];
  long count[2 * MAXB];
};
__global__ void __launch_bounds__(256) b16_pack_kernel(const B16PackArgs a) {
  const int s = blockIdx.y;
  const float* src = a.src[s];
  if (src == nullptr) return;
  uint16_t* dst = a.dst[s];
  const long n8 = a.count[s] / 8;
  for (long i = static_cast<long>(blockIdx.x) * 256 + threadIdx.x; i < n8; i += static_cast<long>(gridDim.x) * 256) {
    const f32x4 x0 = reinterpret_cast<const f32x4*>(src)[2 * i];
    const f32x4 x1 = reinterpret_cast<const f32x4*>(src)[2 * i + 1];
    u32x4 o;
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      o[d] = f32_to_bf16_rne(x0[2 * d]) | (static_cast<uint32_t>(f32_to_bf16_rne(x0[2 * d + 1])) << 16);
      o[2 + d] = f32_to_bf16_rne(x1[2 * d]) | (static_cast<uint32_t>(f32_to_bf16_rne(x1[2 * d + 1])) << 16);
    }
    reinterpret_cast<u32x4*>(dst)[i] = o;
  }
}

// ----------------------------------------------------------------------------- updates
// For every element (i, j) of the m x n storage:
//   u = sum_c RF_u[i][c] CF_u[j][c];   M = rne(M + rne(alpha rne(u)))      (error feedback)
//   d = sum_c RF_w[i][c] CF_w[j][c];   W = fma(beta, rne(d), W decay)      (weight update)
// not transposed: RF_u = RF_w = P (m x r), CF_u = R (n x r), CF_w = Qn (n x r)
// transposed:     RF_u = R, RF_w = Qn (m x r),  CF_u = CF_w = P (n x r)
// The MFMA computes the transposed tile (rows j, columns i) so a lane's four
// accumulator values are four adjacent columns of one storage row.  A wave owns
// 64 columns and walks 16-row steps down its block's row range.
struct B16UpdArgs {
  uint16_t* m[MAXB];         // bf16 momentum or null (weight update only)
  float* w[MAXB];            // fp32 weights or null (error feedback only)
  const void* rf_u[MAXB];    // fp32 (P/R buffers)
  const void* cf_u[MAXB];
  const void* rf_w[MAXB];    // fp32 (P) or bf16 (Qn)
  const void* cf_w[MAXB];
  int rfw_bf16, cfw_bf16;
  int vec;                   // 8-byte M / 16-byte W runs (cols, strides multiple of 4, aligned bases)
  int fvec;                  // 16-byte factor loads (r % 8 == 0, aligned factors)
  int rows, cols, r, rows_per_block;
  long ld_m, ld_w;
  float alpha, beta, decay;
};

template <int KS>
__device__ __forceinline__ void b16_factor(bf16x8s (&o)[KS], const void* base, bool is_bf16, bool vec, int row,
                                           int nrows, int r, int g) {
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    bf16x8s v = {0, 0, 0, 0, 0, 0, 0, 0};
    const int c0 = 32 * s + 8 * g;
    if (row < nrows && c0 < r) {
      const long idx = static_cast<long>(row) * r + c0;
      if (vec) {  // r % 8 == 0 and 16-byte aligned factors: one or two 16-byte loads
        if (is_bf16) {
          v = *reinterpret_cast<const bf16x8s*>(static_cast<const uint16_t*>(base) + idx);
        } else {
          const f32x4 x0 = *reinterpret_cast<const f32x4*>(static_cast<const float*>(base) + idx);
          const f32x4 x1 = *reinterpret_cast<const f32x4*>(static_cast<const float*>(base) + idx + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = static_cast<short>(f32_to_bf16_rne(x0[e]));
            v[4 + e] = static_cast<short>(f32_to_bf16_rne(x1[e]));
          }
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (c0 + e < r)
            v[e] = static_cast<short>(is_bf16 ? static_cast<const uint16_t*>(base)[idx + e]
                                              : f32_to_bf16_rne(static_cast<const float*>(base)[idx + e]));
      }
    }
    o[s] = v;
  }
}

__device__ __forceinline__ uint16_t b16_ef(uint16_t m, float u, float alpha) {
  return f32_to_bf16_rne(bf16_to_f32(m) + bf16_round(alpha * bf16_round(u)));
}

template <int KS>
__global__ void __launch_bounds__(256) b16_update_kernel(const B16UpdArgs a) {
  const int b = blockIdx.z;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int t = lane & 15, g = lane >> 4;
  const int j0 = blockIdx.x * 256 + wave * 64;
  const int i_begin = blockIdx.y * a.rows_per_block;
  const int i_end = min(a.rows, i_begin + a.rows_per_block);
  uint16_t* M = a.m[b];
  float* W = a.w[b];
  const bool fvec = a.fvec != 0;
  // column factors of this wave's 64 columns: 4 blocks of 16 columns, operand rows j = j0 + 16 jb + t
  bf16x8s cu[4][KS], cw[4][KS];
#pragma unroll
  for (int jb = 0; jb < 4; ++jb) {
    if (M) b16_factor<KS>(cu[jb], a.cf_u[b], false, fvec, j0 + 16 * jb + t, a.cols, a.r, g);
    if (W) b16_factor<KS>(cw[jb], a.cf_w[b], a.cfw_bf16 != 0, fvec, j0 + 16 * jb + t, a.cols, a.r, g);
  }
  for (int i0 = i_begin; i0 < i_end; i0 += 16) {
    const int i = i0 + t;  // the storage row of this lane's accumulator column
    const bool row_ok = i < i_end;
    bf16x8s ru[KS], rw[KS];
    if (M) b16_factor<KS>(ru, a.rf_u[b], false, fvec, i, a.rows, a.r, g);
    if (W) b16_factor<KS>(rw, a.rf_w[b], a.rfw_bf16 != 0, fvec, i, a.rows, a.r, g);
    if (a.vec) {
      // cols % 4 == 0: a lane's four columns are one 8-byte M run and one 16-byte W run;
      // all loads of the step are issued before the products
      uint2 mv[4];
      f32x4 wv[4];
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const int j = j0 + 16 * jb + 4 * g;
        const bool ok = row_ok && j < a.cols;
        if (M) mv[jb] = ok ? *reinterpret_cast<const uint2*>(M + static_cast<long>(i) * a.ld_m + j) : uint2{0u, 0u};
        if (W) wv[jb] = ok ? *reinterpret_cast<const f32x4*>(W + static_cast<long>(i) * a.ld_w + j)
                           : f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const int j = j0 + 16 * jb + 4 * g;
        const bool ok = row_ok && j < a.cols;
        if (M) {
          f32x4 u = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < KS; ++s) u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cu[jb][s], ru[s], u, 0, 0, 0);
          if (ok) {
            const uint32_t lo = b16_ef(mv[jb].x & 0xFFFFu, u[0], a.alpha) |
                                (static_cast<uint32_t>(b16_ef(mv[jb].x >> 16, u[1], a.alpha)) << 16);
            const uint32_t hi = b16_ef(mv[jb].y & 0xFFFFu, u[2], a.alpha) |
                                (static_cast<uint32_t>(b16_ef(mv[jb].y >> 16, u[3], a.alpha)) << 16);
            *reinterpret_cast<uint2*>(M + static_cast<long>(i) * a.ld_m + j) = uint2{lo, hi};
          }
        }
        if (W) {
          f32x4 d = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < KS; ++s) d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cw[jb][s], rw[s], d, 0, 0, 0);
          if (ok) {
            f32x4 w = wv[jb];
#pragma unroll
            for (int q = 0; q < 4; ++q) w[q] = fmaf(a.beta, bf16_round(d[q]), w[q] * a.decay);
            *reinterpret_cast<f32x4*>(W + static_cast<long>(i) * a.ld_w + j) = w;
          }
        }
      }
      continue;
    }
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
      const int j = j0 + 16 * jb + 4 * g;  // first of this lane's four columns
      if (M) {
        f32x4 u = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s) u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cu[jb][s], ru[s], u, 0, 0, 0);
        if (row_ok) {
          uint16_t* pm = M + static_cast<long>(i) * a.ld_m + j;
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (j + q < a.cols) pm[q] = b16_ef(pm[q], u[q], a.alpha);
        }
      }
      if (W) {
        f32x4 d = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s) d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cw[jb][s], rw[s], d, 0, 0, 0);
        if (row_ok) {
          float* pw = W + static_cast<long>(i) * a.ld_w + j;
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (j + q < a.cols) pw[q] = fmaf(a.beta, bf16_round(d[q]), pw[q] * a.decay);
        }
      }
    }
  }
}

// The same update in rank_stream_kernel's geometry (dion_codec.hip): NW-wave blocks, a
// wave owns a 32-column strip of the storage and walks 32-row steps; the column factors
// of the strip sit in registers (bf16, v_mfma_f32_32x32x16_bf16 B operand), the step's
// row factors are converted to bf16 once per block into LDS (A operand); M (bf16) and W
// (fp32) move as 32 x 32 tiles in the accumulator layout with nt buffer loads / stores
// (a W load instruction is two whole 128-B rows), two tiles in flight.  Same per-element
// arithmetic as b16_update_kernel; the fp32 sums of the bf16 products run in the 32x32
// MFMA's order.  TR (transposed storage): RF_u = R, RF_w = Qn (two staged factors),
// CF_u = CF_w = P (one register factor); otherwise RF_u = RF_w = P, CF_u = R, CF_w = Qn.
struct B16StreamArgs {
  uint16_t* m[MAXB];
  float* w[MAXB];
  const void* cf_u[MAXB];
  const void* cf_w[MAXB];
  const void* rf_u[MAXB];
  const void* rf_w[MAXB];
  int cfw_bf16, rfw_bf16;  // Qn is the bf16 Q tensor; P and R are fp32 buffers of bf16 values
  int rows, cols, r, s_len;
  long ld_m, ld_w;
  float alpha, beta, decay;
};

// 8 consecutive factor values (row `row`, columns c0 .. c0 + 7) as bf16 (exact: bf16 values)
__device__ __forceinline__ bf16x8s b16_run8(const void* base, bool is_bf16, long idx) {
  if (is_bf16) return *reinterpret_cast<const bf16x8s*>(static_cast<const uint16_t*>(base) + idx);
  const f32x4 x0 = *reinterpret_cast<const f32x4*>(static_cast<const float*>(base) + idx);
  const f32x4 x1 = *reinterpret_cast<const f32x4*>(static_cast<const float*>(base) + idx + 4);
  bf16x8s v;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = static_cast<short>(f32_to_bf16_rne(x0[e]));
    v[4 + e] = static_cast<short>(f32_to_bf16_rne(x1[e]));
  }
  return v;
}

template <int RU, int NW, bool TR>
__global__ void __launch_bounds__(64 * NW, NW >= 8 ? 1 : 2) b16_stream_kernel(const B16StreamArgs a) {
  constexpr int NT = 64 * NW;
  constexpr int NF = TR ? 2 : 1;                 // staged row factors
  constexpr int kGroups = NF * RU * 64;          // 8-value groups of one 32-row step
  constexpr int kPer = (kGroups + NT - 1) / NT;
  __shared__ bf16x8s sp[2][NF * RU * 64];
  const int b = blockIdx.z;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(tid >> 6));
  const int lane = tid & 63;
  const int t = lane & 31;
  const int h = lane >> 5;
  const int R = a.r;
  const int fbase = blockIdx.x * (32 * NW) + wave * 32;
  const bool active = fbase < a.cols;
  const int s_begin = blockIdx.y * a.s_len;
  const int s_end = min(a.rows, s_begin + a.s_len);
  uint16_t* M = a.m[b];
  float* W = a.w[b];
  const bool has_m = M != nullptr, has_w = W != nullptr;
  const __amdgpu_buffer_rsrc_t rm = __builtin_amdgcn_make_buffer_rsrc(
      has_m ? static_cast<void*>(M) : static_cast<void*>(W), static_cast<short>(0),
      static_cast<int>(min(static_cast<long>(a.rows) * a.ld_m * 2, 0x7FFFFFF0L)), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      has_w ? static_cast<void*>(W) : static_cast<void*>(M), static_cast<short>(0),
      static_cast<int>(min(static_cast<long>(a.rows) * a.ld_w * 4, 0x7FFFFFF0L)), 0x00020000);
  int vrow[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) vrow[q] = (q & 3) + 8 * (q >> 2) + 4 * h;

  // column factors of this lane's column fbase + t: k-run 16 u + 8 h .. + 7
  bf16x8s Fu[RU], Fw[TR ? 1 : RU];
  if (active) {
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const long idx = static_cast<long>(fbase + t) * R + 16 * u + 8 * h;
      if (TR || has_m) Fu[u] = b16_run8(a.cf_u[b], false, idx);  // R or P: fp32 buffers
      if constexpr (!TR) {
        if (has_w) Fw[u] = b16_run8(a.cf_w[b], a.cfw_bf16 != 0, idx);
      }
    }
  }
  // staging of one step's row factors: item g -> (f, u, l): factor f, row s0 + l % 32,
  // columns 16 u + 8 (l / 32) .. + 7
  bf16x8s pv[kPer];
  auto p_load = [&](int s0) {
#pragma unroll
    for (int it = 0; it < kPer; ++it) {
      const int g = tid + NT * it;
      if (g < kGroups) {
        const int f = g / (RU * 64), rem = g - f * RU * 64;
        const int u = rem >> 6, l = rem & 63;
        const long idx = static_cast<long>(s0 + (l & 31)) * R + 16 * u + 8 * (l >> 5);
        pv[it] = (f == 0) ? b16_run8(a.rf_u[b], false, idx) : b16_run8(a.rf_w[b], a.rfw_bf16 != 0, idx);
      }
    }
  };
  auto p_store = [&](bf16x8s* dst) {
#pragma unroll
    for (int it = 0; it < kPer; ++it) {
      const int g = tid + NT * it;
      if (g < kGroups) dst[g] = pv[it];
    }
  };
  struct Tile {
    float w[16];
    uint32_t m[16];
  };
  Tile X[2];
  auto x_load = [&](int s0, Tile& T) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int row = s0 + vrow[q];
      if (has_m)
        T.m[q] = __builtin_amdgcn_raw_buffer_load_b16(rm, static_cast<int>((static_cast<long>(row) * a.ld_m + fbase + t) * 2), 0,
                                                      kStreamAux);
      if (has_w)
        T.w[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
            rw, static_cast<int>((static_cast<long>(row) * a.ld_w + fbase + t) * 4), 0, kStreamAux));
    }
  };
  auto compute_store = [&](int s0, const Tile& T, const bf16x8s* src) {
    if (has_m) {
      f32x16 acc;
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[q] = 0.f;
#pragma unroll
      for (int u = 0; u < RU; ++u) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
          __builtin_bit_cast(bf16x8, src[u * 64 + lane]), __builtin_bit_cast(bf16x8, Fu[u]), acc, 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const uint16_t v = b16_ef(static_cast<uint16_t>(T.m[q]), acc[q], a.alpha);
        __builtin_amdgcn_raw_buffer_store_b16(v, rm, static_cast<int>((static_cast<long>(s0 + vrow[q]) * a.ld_m + fbase + t) * 2),
                                              0, kStreamAux);
      }
    }
    if (has_w) {
      f32x16 acc;
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[q] = 0.f;
#pragma unroll
      for (int u = 0; u < RU; ++u) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
          __builtin_bit_cast(bf16x8, src[((TR ? 1 : 0) * RU + u) * 64 + lane]),
          __builtin_bit_cast(bf16x8, TR ? Fu[u] : Fw[TR ? 0 : u]), acc, 0, 0, 0);
      // W = fma(beta, rne(d), W decay), two values per instruction (v_cvt_pk_bf16_f32,
      // v_pk_mul_f32, v_pk_fma_f32): the same per-element operations
#pragma unroll
      for (int q = 0; q < 16; q += 2) {
        const uint32_t d2 = f32x2_to_bf16x2_rne(acc[q], acc[q + 1]);
        const f32x2v dv{__uint_as_float(d2 << 16), __uint_as_float(d2 & 0xFFFF0000u)};
        const f32x2v wd = f32x2v{T.w[q], T.w[q + 1]} * a.decay;
        const f32x2v v = __builtin_elementwise_fma(f32x2v{a.beta, a.beta}, dv, wd);
#pragma unroll
        for (int e = 0; e < 2; ++e)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[e]), rw,
                                                static_cast<int>((static_cast<long>(s0 + vrow[q + e]) * a.ld_w + fbase + t) * 4),
                                                0, kStreamAux);
      }
    }
  };

  p_load(s_begin);
  if (active) x_load(s_begin, X[0]);
  p_store(sp[0]);
  __syncthreads();
  int cur = 0;
  for (int s0 = s_begin; s0 < s_end; s0 += 64) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int s = s0 + 32 * k;
      if (s >= s_end) break;
      const bool more = s + 32 < s_end;
      if (more) p_load(s + 32);
      if (active && more) x_load(s + 32, X[k ^ 1]);
      if (active) compute_store(s, X[k], sp[cur]);
      if (!more) break;
      p_store(sp[cur ^ 1]);
      __syncthreads();
      cur ^= 1;
    }
  }
}

// ----------------------------------------------------------------------------- host side
namespace b16 {

// the update on b16_stream_kernel (rank-stream geometry) where the shapes allow
constexpr bool kB16Stream = true;


int rpad_of(int r) { return (r + 15) / 16 * 16; }
long kpad_of(int K) { return (K + 31) / 32 * 32; }

Geo geo(int out_rows, int K, int batch) {
  Geo g;
  g.gx = static_cast<int>(ceil_div(out_rows, kB16BO));
  long want = ceil_div(kTargetBlocks, static_cast<long>(g.gx) * (batch > 0 ? batch : 1));
  long maxc = ceil_div(K, 256);
  long nc = want < maxc ? want : maxc;
  if (nc < 1) nc = 1;
  g.kchunk = round_up(ceil_div(K, nc), 32);
  g.nchunk = static_cast<int>(ceil_div(K, g.kchunk));
  g.out_rows = out_rows;
  return g;
}

// the streaming kernels (b16_row_kernel / b16_col_kernel): whole blocks, r a multiple of 16,
// bf16 or no gradient (shape rules here; pointer alignment is checked at launch).  Measured
// and not kept: 8-wave blocks for the read-only pass B (column 0.42 -> 0.49 ms, row equal),
// and dword-paired bf16 M accesses in b16_stream_kernel (2.15 -> 2.28 ms; round 3)
constexpr bool kB16Fast = true;
bool fast_ok(bool row_mode, int m, int n, int r, int gdt) {
  if (!kB16Fast || r % 16 != 0 || r > 128 || (gdt != DION_DTYPE_NONE && gdt != DION_DTYPE_BF16)) return false;
  return row_mode ? (m % kB16RowBlk == 0 && n % 64 == 0) : (n % kB16ColBlk == 0 && m % 32 == 0);
}

// split-K geometry of the streaming kernels: K chunks of whole steps, about kTargetBlocks blocks
Geo fast_geo(bool row_mode, int out_rows, int K, int batch) {
  Geo g;
  const int blk = row_mode ? kB16RowBlk : kB16ColBlk, step = row_mode ? 64 : 32;
  g.gx = static_cast<int>(ceil_div(out_rows, blk));
  long want = ceil_div(kTargetBlocks, static_cast<long>(g.gx) * (batch > 0 ? batch : 1));
  long maxc = ceil_div(K, 256);
  long nc = want < maxc ? want : maxc;
  if (nc < 1) nc = 1;
  g.kchunk = round_up(ceil_div(K, nc), step);
  g.nchunk = static_cast<int>(ceil_div(K, g.kchunk));
  g.out_rows = out_rows;
  return g;
}

// the EF panels (P' and R' in bf16) after the thin panel, when the pass carries the error feedback
size_t ef_panel_bytes(int m, int n, int r, int batch) {
  return (sizeof(uint16_t) * static_cast<size_t>(batch) * (static_cast<size_t>(m) + n) * r + 255) / 256 * 256;
}

size_t proj_ws(int m, int n, int r, int batch, bool row_mode, bool with_ef = false) {
  const int out_rows = row_mode ? m : n, K = row_mode ? n : m;
  const Geo g = geo(out_rows, K, batch);
  const Geo f = fast_geo(row_mode, out_rows, K, batch);
  const int nchunk = g.nchunk > f.nchunk ? g.nchunk : f.nchunk;  // either kernel may run (alignment)
  const size_t slab = (sizeof(float) * static_cast<size_t>(batch) * nchunk * out_rows * r + 255) / 256 * 256;
  const size_t thin = (sizeof(uint16_t) * static_cast<size_t>(batch) * rpad_of(r) * kpad_of(K) + 255) / 256 * 256;
  return slab + thin + (with_ef ? ef_panel_bytes(m, n, r, batch) : 0);
}

// the deferred-EF pass A exists for the streaming kernels' shapes with r = 32 or 64 (r = 96 / 128
// spill past 256 VGPRs) and a bf16 (or no) gradient
bool ef_ok(bool row_mode, int m, int n, int r, int gdt) {
  return (r == 32 || r == 64) && fast_ok(row_mode, m, n, r, gdt);
}

// one projection of up to MAXB matrices: out (batch, out_rows, r) = rne(X T) or rne(X^T T); with
// `efP` (pass A only) each entry whose efP[b] is set first takes its pending error feedback
// M = rne(M + rne(alpha rne(P' R'^T)))
int project(bool row_mode, int m, int n, int r, int nb, const void* const* G, int gdt, uint16_t* const* X, long ld_x,
            long ld_g, const void* const* thin, bool thin_bf16, float* out, uint32_t* nonzero, void* ws,
            size_t ws_bytes, hipStream_t st, const float* const* efP = nullptr, const float* const* efR = nullptr,
            float alpha = 0.f) {
  if (r > 128) return fail(DION_E_UNSUPPORTED, "bf16 path: r=%d > 128", r);
  const int out_rows = row_mode ? m : n, K = row_mode ? n : m;
  const Geo g = geo(out_rows, K, nb);
  const bool with_ef = efP != nullptr;
  const size_t need = proj_ws(m, n, r, nb, row_mode, with_ef);
  if (ws == nullptr || ws_bytes < need) return fail(DION_E_WORKSPACE, "bf16 projection needs %zu workspace bytes, got %zu", need, ws_bytes);
  const size_t slab_b = (sizeof(float) * static_cast<size_t>(nb) * g.nchunk * out_rows * r + 255) / 256 * 256;
  float* slab = static_cast<float*>(ws);
  uint16_t* tt = reinterpret_cast<uint16_t*>(static_cast<char*>(ws) + slab_b);
  const int rp = rpad_of(r);
  const long Kp = kpad_of(K);
  {
    B16ThinArgs ta;
    memset(&ta, 0, sizeof(ta));
    for (int b = 0; b < nb; ++b) ta.src[b] = thin[b];
    ta.tt = tt;
    ta.K = K;
    ta.Kp = static_cast<int>(Kp);
    ta.r = r;
    ta.rpad = rp;
    ta.src_bf16 = thin_bf16 ? 1 : 0;
    const dim3 tgrid(static_cast<unsigned>(ceil_div(Kp, 64)), static_cast<unsigned>(ceil_div(rp, 64)), nb);
    hipLaunchKernelGGL(b16_thin_kernel, tgrid, dim3(256), 0, st, ta);
    int rc = check_launch("b16_thin");
    if (rc != DION_OK) return rc;
  }
  B16ProjArgs a;
  memset(&a, 0, sizeof(a));
  for (int b = 0; b < nb; ++b) {
    a.x[b] = X[b];
    a.g[b] = G ? G[b] : nullptr;
    if (X[b] == nullptr || (gdt != DION_DTYPE_NONE && a.g[b] == nullptr)) return fail(DION_E_INVALID, "null matrix at %d", b);
  }
  a.tt = tt;
  a.slab = slab;
  a.nonzero = nonzero;
  a.rows = m;
  a.cols = n;
  a.r = r;
  a.rpad = rp;
  a.kchunk = g.kchunk;
  a.nchunk = g.nchunk;
  a.out_rows = out_rows;
  a.K = K;
  a.Kp = static_cast<int>(Kp);
  a.ld_x = ld_x;
  a.ld_g = ld_g;
  {
    bool vec = ld_x % 8 == 0 && (gdt == DION_DTYPE_NONE || ld_g % 8 == 0);
    for (int b = 0; b < nb && vec; ++b)
      vec = (reinterpret_cast<uintptr_t>(X[b]) & 15u) == 0 &&
            (gdt == DION_DTYPE_NONE || (reinterpret_cast<uintptr_t>(G[b]) & 15u) == 0);
    a.vec = vec ? 1 : 0;
  }
  bool fast = fast_ok(row_mode, m, n, r, gdt) && a.vec;
  const Geo fg = fast_geo(row_mode, out_rows, K, nb);
  if (fast) {
    a.kchunk = fg.kchunk;
    a.nchunk = fg.nchunk;
  }
  const dim3 grid = fast ? dim3(fg.gx, fg.nchunk, nb) : dim3(g.gx, g.nchunk, nb);
  B16EfArgs e;
  if (with_ef) {
    if (!fast || !ef_ok(row_mode, m, n, r, gdt))
      return fail(DION_E_UNSUPPORTED, "no deferred-EF bf16 pass A for %dx%d r=%d", m, n, r);
    const int mp = row_mode ? m : n, nq = row_mode ? n : m;
    memset(&e, 0, sizeof(e));
    e.p = a;
    uint16_t* ep = reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(tt) +
                                               (sizeof(uint16_t) * static_cast<size_t>(nb) * rp * Kp + 255) / 256 * 256);
    uint16_t* er = ep + static_cast<long>(nb) * mp * r;
    B16PackArgs pk;
    memset(&pk, 0, sizeof(pk));
    for (int b = 0; b < nb; ++b) {
      if ((efP[b] == nullptr) != (efR[b] == nullptr))
        return fail(DION_E_INVALID, "pending EF of entry %d has only one factor", b);
      if (efP[b] && ((reinterpret_cast<uintptr_t>(efP[b]) & 15u) || (reinterpret_cast<uintptr_t>(efR[b]) & 15u)))
        return fail(DION_E_UNSUPPORTED, "deferred-EF pass A needs 16-byte aligned factors (entry %d)", b);
      e.has[b] = efP[b] != nullptr;
      pk.src[b] = efP[b];
      pk.dst[b] = ep + static_cast<long>(b) * mp * r;
      pk.count[b] = static_cast<long>(mp) * r;
      pk.src[nb + b] = efR[b];
      pk.dst[nb + b] = er + static_cast<long>(b) * nq * r;
      pk.count[nb + b] = static_cast<long>(nq) * r;
    }
    long pblocks = ceil_div(static_cast<long>(mp > nq ? mp : nq) * r / 8, 256);
    if (pblocks > 1024) pblocks = 1024;
    hipLaunchKernelGGL(b16_pack_kernel, dim3(static_cast<unsigned>(pblocks), 2 * nb), dim3(256), 0, st, pk);
    int rc = check_launch("b16_pack");
    if (rc != DION_OK) return rc;
    e.ep = ep;
    e.er = er;
    e.alpha = alpha;
  }
  auto launch = [&](auto RBc) {
    constexpr int RB = decltype(RBc)::value;
    return dispatch_gdt(gdt, [&](auto Gc) {
      constexpr int GD = decltype(Gc)::value;
      if constexpr (RB % 2 == 0 && GD != DION_DTYPE_F32) {
        if (with_ef) {
          if (row_mode)
            hipLaunchKernelGGL((b16_row_ef_kernel<RB, GD>), grid, dim3(256), 0, st, e);
          else
            hipLaunchKernelGGL((b16_col_ef_kernel<RB, GD>), grid, dim3(256), 0, st, e);
          return check_launch("b16_proj_ef");
        }
      }
      if (with_ef) return fail(DION_E_UNSUPPORTED, "no deferred-EF bf16 pass A for r=%d", r);
      if constexpr (GD == DION_DTYPE_F32) {
        if (row_mode)
          hipLaunchKernelGGL((b16_proj_kernel<false, RB, GD>), grid, dim3(256), 0, st, a);
        else
          hipLaunchKernelGGL((b16_proj_kernel<true, RB, GD>), grid, dim3(256), 0, st, a);
      } else if (fast && row_mode) {
        hipLaunchKernelGGL((b16_row_kernel<RB, GD>), grid, dim3(256), 0, st, a);
      } else if (fast) {
        hipLaunchKernelGGL((b16_col_kernel<RB, GD>), grid, dim3(256), 0, st, a);
      } else if (row_mode) {
        hipLaunchKernelGGL((b16_proj_kernel<false, RB, GD>), grid, dim3(256), 0, st, a);
      } else {
        hipLaunchKernelGGL((b16_proj_kernel<true, RB, GD>), grid, dim3(256), 0, st, a);
      }
      return check_launch("b16_proj");
    });
  };
  int rc;
  switch (rp / 16) {
    case 1: rc = launch(std::integral_constant<int, 1>{}); break;
    case 2: rc = launch(std::integral_constant<int, 2>{}); break;
    case 3: rc = launch(std::integral_constant<int, 3>{}); break;
    case 4: rc = launch(std::integral_constant<int, 4>{}); break;
    case 5: rc = launch(std::integral_constant<int, 5>{}); break;
    case 6: rc = launch(std::integral_constant<int, 6>{}); break;
    case 7: rc = launch(std::integral_constant<int, 7>{}); break;
    default: rc = launch(std::integral_constant<int, 8>{}); break;
  }
  if (rc != DION_OK) return rc;
  const long per = static_cast<long>(out_rows) * r;
  long blocks = ceil_div(per * nb, 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(b16_reduce_round_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, st, out, slab, a.nchunk,
                     per, nb);
  return check_launch("b16_reduce_round");
}

int round_buffer(float* x, long n, hipStream_t st) {
  if (n <= 0) return DION_OK;
  long blocks = ceil_div(n, 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(b16_round_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, st, x, n);
  return check_launch("b16_round");
}

int update(const DionBatchDesc* d, uint16_t* const* M, float* const* W, const float* P, const float* R,
           const uint16_t* const* Qn, float alpha, float beta, float decay, hipStream_t st) {
  const int mp = d->transposed ? d->n : d->m;
  const int nq = d->transposed ? d->m : d->n;
  const int r = d->r;
  for (int b0 = 0; b0 < d->batch; b0 += MAXB) {
    const int nb = d->batch - b0 < MAXB ? d->batch - b0 : MAXB;
    if (kB16Stream && d->m % 32 == 0 && d->n % 32 == 0 && r % 16 == 0 && r <= 128) {
      // the rank-stream geometry (b16_stream_kernel)
      B16StreamArgs sa;
      memset(&sa, 0, sizeof(sa));
      bool ok = (reinterpret_cast<uintptr_t>(P) & 15u) == 0 && (reinterpret_cast<uintptr_t>(R) & 15u) == 0;
      for (int b = 0; b < nb && ok; ++b) {
        const float* Pb = P + static_cast<long>(b0 + b) * mp * r;
        const float* Rb = R + static_cast<long>(b0 + b) * nq * r;
        sa.m[b] = M ? M[b0 + b] : nullptr;
        sa.w[b] = W ? W[b0 + b] : nullptr;
        if ((M && sa.m[b] == nullptr) || (W && sa.w[b] == nullptr) || Qn[b0 + b] == nullptr)
          return fail(DION_E_INVALID, "null pointer at entry %d", b0 + b);
        ok = (reinterpret_cast<uintptr_t>(Qn[b0 + b]) & 15u) == 0;
        if (!d->transposed) {
          sa.rf_u[b] = Pb; sa.rf_w[b] = Pb; sa.cf_u[b] = Rb; sa.cf_w[b] = Qn[b0 + b];
        } else {
          sa.rf_u[b] = Rb; sa.rf_w[b] = Qn[b0 + b]; sa.cf_u[b] = Pb; sa.cf_w[b] = Pb;
        }
      }
      if (ok) {
        sa.cfw_bf16 = d->transposed ? 0 : 1;
        sa.rfw_bf16 = d->transposed ? 1 : 0;
        sa.rows = d->m;
        sa.cols = d->n;
        sa.r = r;
        sa.s_len = 512;
        sa.ld_m = ldv(d->ld_m, d->n);
        sa.ld_w = ldv(d->ld_w, d->n);
        sa.alpha = alpha;
        sa.beta = beta;
        sa.decay = decay;
        constexpr int NW = 8;
        const dim3 grid(static_cast<unsigned>(ceil_div(d->n, 32 * NW)), static_cast<unsigned>(ceil_div(d->m, sa.s_len)), nb);
        auto go = [&](auto RUc) {
          constexpr int RU = decltype(RUc)::value;
          if (d->transposed)
            hipLaunchKernelGGL((b16_stream_kernel<RU, NW, true>), grid, dim3(64 * NW), 0, st, sa);
          else
            hipLaunchKernelGGL((b16_stream_kernel<RU, NW, false>), grid, dim3(64 * NW), 0, st, sa);
        };
        switch (r / 16) {
          case 1: go(std::integral_constant<int, 1>{}); break;
          case 2: go(std::integral_constant<int, 2>{}); break;
          case 3: go(std::integral_constant<int, 3>{}); break;
          case 4: go(std::integral_constant<int, 4>{}); break;
          case 5: go(std::integral_constant<int, 5>{}); break;
          case 6: go(std::integral_constant<int, 6>{}); break;
          case 7: go(std::integral_constant<int, 7>{}); break;
          default: go(std::integral_constant<int, 8>{}); break;
        }
        const int rc = check_launch("b16_stream");
        if (rc != DION_OK) return rc;
        continue;
      }
    }
    B16UpdArgs a;
    memset(&a, 0, sizeof(a));
    for (int b = 0; b < nb; ++b) {
      const float* Pb = P + static_cast<long>(b0 + b) * mp * r;
      const float* Rb = R + static_cast<long>(b0 + b) * nq * r;
      a.m[b] = M ? M[b0 + b] : nullptr;
      a.w[b] = W ? W[b0 + b] : nullptr;
      if ((M && a.m[b] == nullptr) || (W && a.w[b] == nullptr) || Qn[b0 + b] == nullptr)
        return fail(DION_E_INVALID, "null pointer at entry %d", b0 + b);
      if (!d->transposed) {
        a.rf_u[b] = Pb; a.cf_u[b] = Rb; a.rf_w[b] = Pb; a.cf_w[b] = Qn[b0 + b];
      } else {
        a.rf_u[b] = Rb; a.cf_u[b] = Pb; a.rf_w[b] = Qn[b0 + b]; a.cf_w[b] = Pb;
      }
    }
    a.ld_m = ldv(d->ld_m, d->n);
    a.ld_w = ldv(d->ld_w, d->n);
    {
      bool vec = d->n % 4 == 0 && a.ld_m % 4 == 0 && a.ld_w % 4 == 0;
      bool fvec = r % 8 == 0;
      for (int b = 0; b < nb; ++b) {
        if (a.m[b]) vec = vec && (reinterpret_cast<uintptr_t>(a.m[b]) & 7u) == 0;
        if (a.w[b]) vec = vec && (reinterpret_cast<uintptr_t>(a.w[b]) & 15u) == 0;
        for (const void* f : {a.rf_u[b], a.cf_u[b], a.rf_w[b], a.cf_w[b]})
          fvec = fvec && (reinterpret_cast<uintptr_t>(f) & 15u) == 0;
      }
      a.vec = vec ? 1 : 0;
      a.fvec = fvec ? 1 : 0;
    }
    a.rfw_bf16 = d->transposed ? 1 : 0;
    a.cfw_bf16 = d->transposed ? 0 : 1;
    a.rows = d->m;
    a.cols = d->n;
    a.r = r;
    a.rows_per_block = 256;
    a.alpha = alpha;
    a.beta = beta;
    a.decay = decay;
    const dim3 grid(static_cast<unsigned>(ceil_div(d->n, 256)), static_cast<unsigned>(ceil_div(d->m, a.rows_per_block)), nb);
    const int ks = (r + 31) / 32;
    if (ks == 1) hipLaunchKernelGGL(b16_update_kernel<1>, grid, dim3(256), 0, st, a);
    else if (ks == 2) hipLaunchKernelGGL(b16_update_kernel<2>, grid, dim3(256), 0, st, a);
    else if (ks == 3) hipLaunchKernelGGL(b16_update_kernel<3>, grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(b16_update_kernel<4>, grid, dim3(256), 0, st, a);
    int rc = check_launch("b16_update");
    if (rc != DION_OK) return rc;
  }
  return DION_OK;
}

}  // namespace b16
