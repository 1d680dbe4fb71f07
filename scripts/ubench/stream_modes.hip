// Micro-benchmark (dev tool, not product): HBM ceilings of the stream shapes the codec
// passes have, in place vs out of place, default vs non-temporal cache policy.
//   inplace  X = X*d        (the weight update shape, 8 B/elem)
//   copy     Y = X*d        (same bytes, read and write different buffers)
//   passA    M = M + G      (bf16 G; 10 B/elem; in place and out of place)
//   read     sum(X)         (pass B shape, 4 B/elem)
// Every thread moves U float4 per iteration (a wave moves U KiB contiguous), loads all
// U first, then stores all U.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7FFFFFF0, 0x00020000);
}

// chunk = 64 lanes * U * 16 B; block b handles chunks b, b + grid, ...; offsets fit in 31 bits per
// 1 GiB window, so the base pointer moves per chunk
template <int U, int LP, int SP>
__global__ void __launch_bounds__(256) scale(const float* __restrict__ x, float* y, long n4, float d) {
  const int lane = threadIdx.x & 63;
  const long wave = (blockIdx.x * 4L + (threadIdx.x >> 6));
  const long nw = gridDim.x * 4L;
  for (long c = wave; c * 64 * U < n4; c += nw) {
    const float* xs = x + c * 64 * U * 4;
    float* ys = y + c * 64 * U * 4;
    auto rx = rsrc(xs);
    auto ry = rsrc(ys);
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rx, (u * 64 + lane) * 16, 0, LP);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f32x4 f = __builtin_bit_cast(f32x4, v[u]) * d;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, f), ry, (u * 64 + lane) * 16, 0, SP);
    }
  }
}

// M (fp32) += G (bf16): thread owns 4 consecutive elements per unit
template <int U, int LP, int SP>
__global__ void __launch_bounds__(256) passa(const float* __restrict__ m, const unsigned short* __restrict__ g,
                                             float* mo, long n4) {
  const int lane = threadIdx.x & 63;
  const long wave = (blockIdx.x * 4L + (threadIdx.x >> 6));
  const long nw = gridDim.x * 4L;
  for (long c = wave; c * 64 * U < n4; c += nw) {
    auto rm = rsrc(m + c * 64 * U * 4);
    auto rg = rsrc(g + c * 64 * U * 4);
    auto ro = rsrc(mo + c * 64 * U * 4);
    u32x4 v[U];
    u32x2 w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v[u] = __builtin_amdgcn_raw_buffer_load_b128(rm, (u * 64 + lane) * 16, 0, LP);
      w[u] = __builtin_amdgcn_raw_buffer_load_b64(rg, (u * 64 + lane) * 8, 0, LP);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f32x4 f = __builtin_bit_cast(f32x4, v[u]);
      f[0] += __uint_as_float(w[u][0] << 16);
      f[1] += __uint_as_float(w[u][0] & 0xFFFF0000u);
      f[2] += __uint_as_float(w[u][1] << 16);
      f[3] += __uint_as_float(w[u][1] & 0xFFFF0000u);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, f), ro, (u * 64 + lane) * 16, 0, SP);
    }
  }
}

template <int U, int LP>
__global__ void __launch_bounds__(256) readsum(const float* __restrict__ x, float* out, long n4) {
  const int lane = threadIdx.x & 63;
  const long wave = (blockIdx.x * 4L + (threadIdx.x >> 6));
  const long nw = gridDim.x * 4L;
  f32x4 s = {0, 0, 0, 0};
  for (long c = wave; c * 64 * U < n4; c += nw) {
    auto rx = rsrc(x + c * 64 * U * 4);
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rx, (u * 64 + lane) * 16, 0, LP);
#pragma unroll
    for (int u = 0; u < U; ++u) s += __builtin_bit_cast(f32x4, v[u]);
  }
  if (s[0] + s[1] + s[2] + s[3] == 12345.f) out[0] = s[0];
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
  const long n = 28672L * 4096 * 4;  // 470 M elements: 1.88 GB fp32
  float *x, *y, *o;
  unsigned short* g;
  hipMalloc(&x, n * 4);
  hipMalloc(&y, n * 4);
  hipMalloc(&g, n * 2);
  hipMalloc(&o, 64);
  hipMemset(x, 0, n * 4);
  hipMemset(y, 0, n * 4);
  hipMemset(g, 0, n * 2);
  const long n4 = n / 4;
  auto rep = [&](const char* name, double bpe, float ms) {
    printf("%-36s %8.3f ms  %7.3f TB/s\n", name, ms, bpe * n / ms / 1e9);
    fflush(stdout);
  };
  char nm[96];
  for (int grid : {2048, 8192}) {
#define SC(U, LP, SP)                                                                              \
  snprintf(nm, 96, "inplace U%d lp%d sp%d g%d", U, LP, SP, grid);                                  \
  rep(nm, 8, timeit([&] { scale<U, LP, SP><<<grid, 256>>>(x, x, n4, 1.0f); }, 10));                \
  snprintf(nm, 96, "copy    U%d lp%d sp%d g%d", U, LP, SP, grid);                                  \
  rep(nm, 8, timeit([&] { scale<U, LP, SP><<<grid, 256>>>(x, y, n4, 1.0f); }, 10));
    SC(1, 0, 0) SC(4, 0, 0) SC(8, 0, 0) SC(4, 2, 2) SC(4, 0, 2) SC(8, 2, 2) SC(8, 0, 2)
#define PA(U, LP, SP)                                                                              \
  snprintf(nm, 96, "passA in  U%d lp%d sp%d g%d", U, LP, SP, grid);                                \
  rep(nm, 10, timeit([&] { passa<U, LP, SP><<<grid, 256>>>(x, g, x, n4); }, 10));                   \
  snprintf(nm, 96, "passA out U%d lp%d sp%d g%d", U, LP, SP, grid);                                \
  rep(nm, 10, timeit([&] { passa<U, LP, SP><<<grid, 256>>>(x, g, y, n4); }, 10));
    PA(1, 0, 0) PA(4, 0, 0) PA(4, 2, 2) PA(4, 0, 2) PA(8, 0, 2)
#define RS(U, LP)                                                                                  \
  snprintf(nm, 96, "read    U%d lp%d g%d", U, LP, grid);                                           \
  rep(nm, 4, timeit([&] { readsum<U, LP><<<grid, 256>>>(x, o, n4); }, 10));
    RS(1, 0) RS(4, 0) RS(8, 0) RS(4, 2) RS(8, 2)
  }
  hipFree(x);
  hipFree(y);
  hipFree(g);
  hipFree(o);
  return 0;
}
