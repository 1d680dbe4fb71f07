// Dev microbenchmark (not product): the HBM ceiling for pass A's traffic mix on this box.
// Pass A moves 10 B per element: M (fp32) read and written back, G (bf16) read.  Here the
// same mix with no arithmetic beyond M += G (mix), next to a plain fp32 copy (8 B/elem, read 4 +
// write 4) and a pure fp32 read (4 B/elem, a sum kept live), each over 1 GiB of M in one-shot
// grids (one tile per thread) and grid-stride grids, with plain and nontemporal accesses.
// Prints the best rate of each kind: the rate pass A's roofline fraction should be read against.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o scripts/ubench/hbm_mix scripts/ubench/hbm_mix.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CKU(x)                                                                        \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

template <bool NT, typename T>
__device__ __forceinline__ T ld(const T* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT, typename T>
__device__ __forceinline__ void st(T* p, const T& v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

__device__ __forceinline__ f32x4 add_bf16(f32x4 x, u32x2 g) {
  x[0] += __uint_as_float(g[0] << 16);
  x[1] += __uint_as_float(g[0] & 0xFFFF0000u);
  x[2] += __uint_as_float(g[1] << 16);
  x[3] += __uint_as_float(g[1] & 0xFFFF0000u);
  return x;
}

// kind 0: mix (M += G in place, 10 B/elem), 1: copy (8 B/elem), 2: read (4 B/elem),
// 3: mix out of place (D = M + G, 10 B/elem), 4: in-place scale (M *= 1.0001, 8 B/elem)
template <int KIND, int U, bool NT>
__global__ void __launch_bounds__(256) stream_kernel(f32x4* __restrict__ M, const u32x2* __restrict__ G,
                                                     f32x4* __restrict__ D, long n4, float* sink) {
  const long stride = static_cast<long>(gridDim.x) * 256 * U;
  float s = 0.f;
  for (long base = static_cast<long>(blockIdx.x) * 256 * U + threadIdx.x; base < n4; base += stride) {
    f32x4 x[U];
    u32x2 g[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = base + 256L * u;
      x[u] = i < n4 ? ld<NT>(M + i) : f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (KIND == 0 || KIND == 3) g[u] = i < n4 ? ld<NT>(G + i) : u32x2{0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = base + 256L * u;
      if (i >= n4) continue;
      if constexpr (KIND == 0) st<NT>(M + i, add_bf16(x[u], g[u]));
      else if constexpr (KIND == 1) st<NT>(D + i, x[u]);
      else if constexpr (KIND == 3) st<NT>(D + i, add_bf16(x[u], g[u]));
      else if constexpr (KIND == 4) st<NT>(M + i, x[u] * 1.0001f);
      else s += x[u][0] + x[u][1] + x[u][2] + x[u][3];
    }
  }
  if constexpr (KIND == 2)
    if (s == 1234.5f) sink[threadIdx.x] = s;  // keeps the loads live
}

static const char* kKind[5] = {"mix in place (M rw, G bf16 r, 10 B/elem)", "copy (fp32 r + w, 8 B/elem)",
                               "read (fp32 r, 4 B/elem)", "mix out of place (D = M + G, 10 B/elem)",
                               "scale in place (M rw, 8 B/elem)"};
static const double kBytes[5] = {10.0, 8.0, 4.0, 10.0, 8.0};

template <int KIND, int U, bool NT>
double run(f32x4* M, const u32x2* G, f32x4* D, long n4, float* sink, int blocks, int iters) {
  hipEvent_t a, b;
  CKU(hipEventCreate(&a));
  CKU(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) stream_kernel<KIND, U, NT><<<blocks, 256>>>(M, G, D, n4, sink);
  CKU(hipGetLastError());
  CKU(hipEventRecord(a));
  for (int it = 0; it < iters; ++it) stream_kernel<KIND, U, NT><<<blocks, 256>>>(M, G, D, n4, sink);
  CKU(hipEventRecord(b));
  CKU(hipEventSynchronize(b));
  float ms = 0.f;
  CKU(hipEventElapsedTime(&ms, a, b));
  CKU(hipEventDestroy(a));
  CKU(hipEventDestroy(b));
  const double sec = ms * 1e-3 / iters;
  return kBytes[KIND] * 4.0 * n4 / sec / 1e9;  // GB/s (1e9 B)
}

template <int KIND, int U, bool NT>
void sweep(f32x4* M, const u32x2* G, f32x4* D, long n4, float* sink, double* best) {
  const long one_shot = (n4 + 256L * U - 1) / (256L * U);
  const long grids[4] = {one_shot, 256L * 8, 256L * 16, 256L * 32};
  for (long gb : grids) {
    const double r = run<KIND, U, NT>(M, G, D, n4, sink, static_cast<int>(gb), 20);
    printf("  %-40s U=%d nt=%d blocks=%-8ld %8.1f GB/s\n", kKind[KIND], U, NT ? 1 : 0, gb, r);
    if (r > best[KIND]) best[KIND] = r;
  }
}

int main() {
  const long n = 1L << 28;  // 1 GiB of fp32 M
  const long n4 = n / 4;
  f32x4 *M, *D;
  u32x2* G;
  float* sink;
  CKU(hipMalloc(&M, n * 4));
  CKU(hipMalloc(&D, n * 4));
  CKU(hipMalloc(&G, n * 2));
  CKU(hipMalloc(&sink, 1024));
  CKU(hipMemset(M, 0, n * 4));
  CKU(hipMemset(D, 0, n * 4));
  CKU(hipMemset(G, 0, n * 2));
  double best[5] = {0, 0, 0, 0, 0};
  sweep<0, 1, false>(M, G, D, n4, sink, best);
  sweep<0, 2, false>(M, G, D, n4, sink, best);
  sweep<0, 4, false>(M, G, D, n4, sink, best);
  sweep<0, 1, true>(M, G, D, n4, sink, best);
  sweep<0, 2, true>(M, G, D, n4, sink, best);
  sweep<0, 4, true>(M, G, D, n4, sink, best);
  sweep<1, 1, false>(M, G, D, n4, sink, best);
  sweep<1, 2, false>(M, G, D, n4, sink, best);
  sweep<1, 4, true>(M, G, D, n4, sink, best);
  sweep<1, 2, true>(M, G, D, n4, sink, best);
  sweep<2, 2, false>(M, G, D, n4, sink, best);
  sweep<2, 4, false>(M, G, D, n4, sink, best);
  sweep<2, 4, true>(M, G, D, n4, sink, best);
  sweep<3, 2, true>(M, G, D, n4, sink, best);
  sweep<3, 4, true>(M, G, D, n4, sink, best);
  sweep<3, 2, false>(M, G, D, n4, sink, best);
  sweep<4, 2, true>(M, G, D, n4, sink, best);
  sweep<4, 4, true>(M, G, D, n4, sink, best);
  sweep<4, 2, false>(M, G, D, n4, sink, best);
  for (int k = 0; k < 5; ++k) printf("best %-40s %8.1f GB/s = %.3f of 8 TB/s\n", kKind[k], best[k], best[k] / 8000.0);
  CKU(hipFree(M));
  CKU(hipFree(D));
  CKU(hipFree(G));
  CKU(hipFree(sink));
  return 0;
}
