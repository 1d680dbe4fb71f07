// Micro-benchmark (dev tool, not product): read-only access patterns a pass-B kernel can use
// over a batch of fp32 matrices (rows x cols, row-major), no arithmetic besides a sum that
// keeps the loads alive.  Every pattern reads every element exactly once.
//   flat     : grid-stride 16-byte loads over the whole buffer (the ceiling)
//   strip    : block = NW waves; wave w owns a 16 * CT * 4-byte column segment of a
//              NW-wide strip; lane (t, g) reads CT floats of column 16 CT w + CT t of rows
//              8 g + e (e < 8) per 32-row step (the pass-B column kernel's geometry),
//              D steps in flight; blocks walk KC rows (split over blockIdx.y)
//   stripL   : as strip, but every load instruction reads ONE row's 64 x 16 B = 1 KB
//              (lane l: 16 B at 16 l of the wave's 256-column segment), 16 rows per step
//   rowwalk  : block = 4 waves x 32 rows, step = SC columns (SC * 4 bytes of each row),
//              lane l reads rows 8 q + l / 8 ... whole 128-B lines (the pass-B row kernel)
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <typename T>
__device__ __forceinline__ T ldnt(const T* p) { return __builtin_nontemporal_load(p); }

__global__ void __launch_bounds__(256) flat(const f32x4* __restrict__ x, long n4, float* out) {
  f32x4 acc = {0, 0, 0, 0};
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) acc += ldnt(x + i);
  if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.f) out[0] = 1.f;
}

template <int NW, int CT, int D>
__global__ void __launch_bounds__(64 * NW) strip(const float* __restrict__ M, int rows, int cols, int kc, float* out) {
  typedef float vec __attribute__((ext_vector_type(CT)));
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, t = lane & 15, g = lane >> 4;
  const long mat = (long)rows * cols;
  const float* base = M + blockIdx.z * mat + (long)(8 * g) * cols + blockIdx.x * (16 * CT * NW) + 16 * CT * w + CT * t;
  const int i0 = blockIdx.y * kc, i1 = min(rows, i0 + kc);
  vec ring[D][8];
  vec acc = {};
  auto load = [&](vec* r, int i) {
#pragma unroll
    for (int e = 0; e < 8; ++e) r[e] = ldnt(reinterpret_cast<const vec*>(base + (long)(i + e) * cols));
  };
#pragma unroll
  for (int k = 0; k < D - 1; ++k)
    if (i0 + 32 * k < i1) load(ring[k], i0 + 32 * k);
  for (int i = i0; i < i1; i += 32 * D) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const int ii = i + 32 * k;
      if (ii >= i1) break;
      if (ii + 32 * (D - 1) < i1) load(ring[(k + D - 1) % D], ii + 32 * (D - 1));
#pragma unroll
      for (int e = 0; e < 8; ++e) acc += ring[k][e];
    }
  }
  float s = 0;
#pragma unroll
  for (int c = 0; c < CT; ++c) s += acc[c];
  if (s == 12345.f) out[0] = 1.f;
}

template <int NW, int D>
__global__ void __launch_bounds__(64 * NW) stripL(const float* __restrict__ M, int rows, int cols, int kc, float* out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long mat = (long)rows * cols;
  const float* base = M + blockIdx.z * mat + blockIdx.x * (256 * NW) + 256 * w + 4 * lane;
  const int i0 = blockIdx.y * kc, i1 = min(rows, i0 + kc);
  f32x4 ring[D][16];
  f32x4 acc = {};
#pragma unroll
  for (int k = 0; k < D - 1; ++k)
    if (i0 + 16 * k < i1)
#pragma unroll
      for (int e = 0; e < 16; ++e) ring[k][e] = ldnt(reinterpret_cast<const f32x4*>(base + (long)(i0 + 16 * k + e) * cols));
  for (int i = i0; i < i1; i += 16 * D) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const int ii = i + 16 * k;
      if (ii >= i1) break;
      if (ii + 16 * (D - 1) < i1)
#pragma unroll
        for (int e = 0; e < 16; ++e)
          ring[(k + D - 1) % D][e] = ldnt(reinterpret_cast<const f32x4*>(base + (long)(ii + 16 * (D - 1) + e) * cols));
#pragma unroll
      for (int e = 0; e < 16; ++e) acc += ring[k][e];
    }
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.f) out[0] = 1.f;
}

template <int SC, int D>
__global__ void __launch_bounds__(256) rowwalk(const float* __restrict__ M, int rows, int cols, int kc, float* out) {
  constexpr int NL = 32 * SC / 4 / 64;  // 16-B loads per lane per step (32 rows x SC floats)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int LPR = SC / 4;           // lanes per row
  constexpr int RPI = 64 / LPR;         // rows per instruction
  const long mat = (long)rows * cols;
  const float* base = M + blockIdx.z * mat + (long)(blockIdx.x * 128 + 32 * w + lane / LPR) * cols + 4 * (lane % LPR);
  const int j0 = blockIdx.y * kc, j1 = min(cols, j0 + kc);
  f32x4 ring[D][NL];
  f32x4 acc = {};
  auto load = [&](f32x4* r, int j) {
#pragma unroll
    for (int q = 0; q < NL; ++q) r[q] = ldnt(reinterpret_cast<const f32x4*>(base + (long)(RPI * q) * cols + j));
  };
#pragma unroll
  for (int k = 0; k < D - 1; ++k)
    if (j0 + SC * k < j1) load(ring[k], j0 + SC * k);
  for (int j = j0; j < j1; j += SC * D) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const int jj = j + SC * k;
      if (jj >= j1) break;
      if (jj + SC * (D - 1) < j1) load(ring[(k + D - 1) % D], jj + SC * (D - 1));
#pragma unroll
      for (int q = 0; q < NL; ++q) acc += ring[k][q];
    }
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.f) out[0] = 1.f;
}

template <typename F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  // the pass-B shapes: fc1 group (16 x 28672 x 4096, column kernel) and fc2 group
  // (16 x 4096 x 14336, row kernel), fp32
  const int nb = 16;
  float* out;
  hipMalloc(&out, 64);
  {
    const int rows = 28672, cols = 4096;
    const long n = (long)rows * cols * nb;
    float* M;
    hipMalloc(&M, n * 4);
    hipMemset(M, 0, n * 4);
    auto rep = [&](const char* name, float ms) {
      printf("%-32s %8.3f ms  %7.3f TB/s\n", name, ms, 4.0 * n / ms / 1e9);
      fflush(stdout);
    };
    rep("flat", timeit([&] { flat<<<8192, 256>>>((const f32x4*)M, n / 4, out); }, 10));
#define S(NW, CT, D, NC) rep("strip NW" #NW " CT" #CT " D" #D " nc" #NC, timeit([&] { strip<NW, CT, D><<<dim3(cols / (16 * CT * NW), NC, nb), 64 * NW>>>(M, rows, cols, rows / NC, out); }, 10));
    S(4, 2, 2, 8) S(4, 4, 2, 8) S(4, 4, 3, 8) S(8, 4, 2, 4) S(4, 4, 2, 4) S(4, 4, 2, 16) S(2, 4, 2, 16) S(4, 2, 3, 8)
#define L(NW, D, NC) rep("stripL NW" #NW " D" #D " nc" #NC, timeit([&] { stripL<NW, D><<<dim3(cols / (256 * NW), NC, nb), 64 * NW>>>(M, rows, cols, rows / NC, out); }, 10));
    L(4, 2, 8) L(2, 2, 16) L(1, 2, 32) L(4, 1, 8)
    hipFree(M);
  }
  {
    const int rows = 4096, cols = 14336;
    const long n = (long)rows * cols * nb;
    float* M;
    hipMalloc(&M, n * 4);
    hipMemset(M, 0, n * 4);
    auto rep = [&](const char* name, float ms) {
      printf("%-32s %8.3f ms  %7.3f TB/s\n", name, ms, 4.0 * n / ms / 1e9);
      fflush(stdout);
    };
    rep("flat (fc2)", timeit([&] { flat<<<8192, 256>>>((const f32x4*)M, n / 4, out); }, 10));
#define W(SC, D, NC) rep("rowwalk SC" #SC " D" #D " nc" #NC, timeit([&] { rowwalk<SC, D><<<dim3(rows / 128, NC, nb), 256>>>(M, rows, cols, cols / NC, out); }, 10));
    W(32, 2, 4) W(32, 3, 4) W(64, 2, 4) W(128, 2, 4) W(32, 2, 8) W(64, 2, 8) W(128, 2, 8) W(32, 4, 4)
    hipFree(M);
  }
  return 0;
}
