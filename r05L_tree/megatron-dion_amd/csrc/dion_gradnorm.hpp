// dion_gradnorm.hpp -- sum of squares of the Dion gradients in fp64, on device.
//
// Replaces the Dion term of the grad-norm computation Megatron runs before the
// optimizer step when gradient clipping is on:
//   /root/reference/megatron/core/optimizer/distrib_dion/grad_norm.py:54-68
//   (_grad_sum_sq_fp64: chunked .to(float64), square, sum) as called by
//   _dion_grad_norm_sq (:144-258) on the local (W = 1) or replica-reduced gradients.
// Every square of a bf16 / fp32 value is exact in fp64; the sums are fp64 and run in
// a fixed order (per-thread, then wave, then block partials, then one block that
// reduces the partials), so the result is bitwise reproducible run to run.  It
// differs from the reference's chunked torch sum only by fp64 summation order.
//
// One read of G (2 B per element for bf16 gradients), no write.

struct SumSqArgs {
  const void* g[MAXB];
  double* part;  // (batch, gridDim.x) block partials
  int rows, cols;
  long ld;
  int vec;       // 16-byte runs (cols % 8 == 0, ld % 8 == 0, aligned bases)
};

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ double block_sum_f64(double v, double* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v = wave_sum_f64(v);
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0)
    for (int w = 0; w < static_cast<int>(blockDim.x >> 6); ++w) s += red[w];
  return s;
}

// block x of matrix b: rows x, x + gridDim.x, ...; threads stride over the columns
template <int GDT>
__global__ void __launch_bounds__(256) sumsq_partial_kernel(const SumSqArgs a) {
  __shared__ double red[4];
  const int b = blockIdx.y;
  double acc = 0.0;
  for (int row = blockIdx.x; row < a.rows; row += gridDim.x) {
    if constexpr (GDT == DION_DTYPE_BF16) {
      const uint16_t* p = static_cast<const uint16_t*>(a.g[b]) + static_cast<long>(row) * a.ld;
      if (a.vec) {
        for (int c = threadIdx.x * 8; c < a.cols; c += 256 * 8) {
          const uint4 q = *reinterpret_cast<const uint4*>(p + c);
          const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const double lo = __uint_as_float(w[i] << 16), hi = __uint_as_float(w[i] & 0xFFFF0000u);
            acc = fma(lo, lo, acc);
            acc = fma(hi, hi, acc);
          }
        }
      } else {
        for (int c = threadIdx.x; c < a.cols; c += 256) {
          const double x = bf16_to_f32(p[c]);
          acc = fma(x, x, acc);
        }
      }
    } else {
      const float* p = static_cast<const float*>(a.g[b]) + static_cast<long>(row) * a.ld;
      if (a.vec) {
        for (int c = threadIdx.x * 4; c < a.cols; c += 256 * 4) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(p + c);
#pragma unroll
          for (int i = 0; i < 4; ++i) acc = fma(static_cast<double>(v[i]), static_cast<double>(v[i]), acc);
        }
      } else {
        for (int c = threadIdx.x; c < a.cols; c += 256) {
          const double x = p[c];
          acc = fma(x, x, acc);
        }
      }
    }
  }
  const double s = block_sum_f64(acc, red);
  if (threadIdx.x == 0) a.part[static_cast<long>(b) * gridDim.x + blockIdx.x] = s;
}

// out[0] += sum of the n partials, fixed order (one block)
__global__ void __launch_bounds__(256) sumsq_final_kernel(const double* __restrict__ part, long n,
                                                          double* __restrict__ out) {
  __shared__ double red[4];
  double acc = 0.0;
  for (long i = threadIdx.x; i < n; i += 256) acc += part[i];
  const double s = block_sum_f64(acc, red);
  if (threadIdx.x == 0) out[0] += s;
}

namespace gnorm {

constexpr int kMaxRowBlocks = 512;

int row_blocks(int rows, int batch) {
  long want = ceil_div(4096, batch > 0 ? batch : 1);
  if (want > rows) want = rows;
  if (want > kMaxRowBlocks) want = kMaxRowBlocks;
  return static_cast<int>(want < 1 ? 1 : want);
}

size_t ws_bytes(int rows, int batch) {
  const int chunk = batch < MAXB ? batch : MAXB;
  return sizeof(double) * static_cast<size_t>(chunk > 0 ? chunk : 1) * row_blocks(rows, chunk);
}

int run(const DionBatchDesc* d, const void* const* G, double* out, void* ws, size_t wsb, hipStream_t st) {
  if (d->g_dtype != DION_DTYPE_BF16 && d->g_dtype != DION_DTYPE_F32)
    return fail(DION_E_UNSUPPORTED, "grad dtype %d", d->g_dtype);
  const long ld = ldv(d->ld_g, d->n);
  for (int b0 = 0; b0 < d->batch; b0 += MAXB) {
    const int nb = d->batch - b0 < MAXB ? d->batch - b0 : MAXB;
    const int gx = row_blocks(d->m, nb);
    const size_t need = sizeof(double) * static_cast<size_t>(nb) * gx;
    if (ws == nullptr || wsb < need) return fail(DION_E_WORKSPACE, "grad sum-sq needs %zu workspace bytes", need);
    SumSqArgs a;
    memset(&a, 0, sizeof(a));
    bool vec = d->n % 8 == 0 && ld % 8 == 0;
    for (int b = 0; b < nb; ++b) {
      a.g[b] = G[b0 + b];
      if (a.g[b] == nullptr) return fail(DION_E_INVALID, "null gradient at %d", b0 + b);
      vec = vec && (reinterpret_cast<uintptr_t>(a.g[b]) & 15u) == 0;
    }
    a.part = static_cast<double*>(ws);
    a.rows = d->m;
    a.cols = d->n;
    a.ld = ld;
    a.vec = vec ? 1 : 0;
    if (d->g_dtype == DION_DTYPE_BF16)
      hipLaunchKernelGGL(sumsq_partial_kernel<DION_DTYPE_BF16>, dim3(gx, nb), dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL(sumsq_partial_kernel<DION_DTYPE_F32>, dim3(gx, nb), dim3(256), 0, st, a);
    int rc = check_launch("sumsq_partial");
    if (rc != DION_OK) return rc;
    hipLaunchKernelGGL(sumsq_final_kernel, dim3(1), dim3(256), 0, st, a.part, static_cast<long>(nb) * gx, out);
    rc = check_launch("sumsq_final");
    if (rc != DION_OK) return rc;
  }
  return DION_OK;
}

}  // namespace gnorm
