// Micro-benchmark: in-place X = X*d streaming with the access shapes the
// rank-update kernels use (dev tool; not part of the product).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__global__ void lin4(float* x, long n4, float d) {
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  long stride = (long)gridDim.x * blockDim.x;
  f32x4* p = (f32x4*)x;
  for (; i < n4; i += stride) { f32x4 v = p[i]; p[i] = v * d; }
}

// tile pattern: wave strip of 32*W cols (lane t owns W consecutive cols), 32-row tiles,
// DEPTH tiles in flight.  Block = 4 waves side by side.  STREAM rows per block.
template <int W, int DEPTH>
__global__ void __launch_bounds__(256) tiles(float* x, int rows, int cols, int stream, float d) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, t = lane & 31, h = lane >> 5;
  const int c0 = (blockIdx.x * 4 + wave) * 32 * W + W * t;
  const int r_begin = blockIdx.y * stream;
  const int r_end = min(rows, r_begin + stream);
  const float* mat = x + (long)blockIdx.z * rows * cols;
  __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)mat, (short)0, 0x7FFFFFF0, 0x00020000);
  int voff[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) voff[q] = (((q & 3) + 8 * (q >> 2) + 4 * h) * cols + c0) * 4;
  typedef float vt __attribute__((ext_vector_type(W)));
  vt buf[DEPTH][16];
  auto ld = [&](int r0, vt* b) {
    const int so = r0 * cols * 4;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      if constexpr (W == 1) b[q][0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rx, voff[q], so, 0));
      else if constexpr (W == 2) { auto u = __builtin_amdgcn_raw_buffer_load_b64(rx, voff[q], so, 0); b[q] = __builtin_bit_cast(vt, u); }
      else { auto u = __builtin_amdgcn_raw_buffer_load_b128(rx, voff[q], so, 0); b[q] = __builtin_bit_cast(vt, u); }
    }
  };
  auto st = [&](int r0, vt* b) {
    const int so = r0 * cols * 4;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      vt v = b[q] * d;
      if constexpr (W == 1) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[0]), rx, voff[q], so, 0);
      else if constexpr (W == 2) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, v), rx, voff[q], so, 0);
      else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), rx, voff[q], so, 0);
    }
  };
  // prologue
#pragma unroll
  for (int k = 0; k < DEPTH - 1; ++k)
    if (r_begin + 32 * k < r_end) ld(r_begin + 32 * k, buf[k]);
  for (int r0 = r_begin; r0 < r_end; r0 += 32 * DEPTH) {
#pragma unroll
    for (int k = 0; k < DEPTH; ++k) {
      const int cur = r0 + 32 * k;
      if (cur >= r_end) break;
      const int nxt = cur + 32 * (DEPTH - 1);
      if (nxt < r_end) ld(nxt, buf[(k + DEPTH - 1) % DEPTH]);
      st(cur, buf[k]);
    }
  }
}

template <typename F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  const int rows = 28672, cols = 4096, nb = 4;
  const long n = (long)rows * cols * nb;
  float* x; hipMalloc(&x, n * 4);
  hipMemset(x, 0, n * 4);
  const double bytes = 8.0 * n;
  auto rep = [&](const char* name, float ms) { printf("%-28s %8.3f ms  %7.3f TB/s\n", name, ms, bytes / ms / 1e9); };
  rep("lin4 grid 4096x256", timeit([&] { lin4<<<4096, 256>>>(x, n / 4, 1.0f); }, 10));
  rep("lin4 grid 16384x256", timeit([&] { lin4<<<16384, 256>>>(x, n / 4, 1.0f); }, 10));
  for (int stream : {256, 512, 1024, 2048}) {
#define RUN(W, D)                                                                                   \
  {                                                                                                 \
    dim3 g(cols / (128 * W), rows / stream, nb);                                                    \
    char nm[64]; snprintf(nm, 64, "tiles W%d D%d s%d", W, D, stream);                              \
    rep(nm, timeit([&] { tiles<W, D><<<g, 256>>>(x, rows, cols, stream, 1.0f); }, 10));          \
    snprintf(nm, 64, "tiles W%d D%d s%d occ2", W, D, stream);                                       \
    rep(nm, timeit([&] { tiles<W, D><<<g, 256, 60000>>>(x, rows, cols, stream, 1.0f); }, 10));   \
  }
    RUN(1, 2) RUN(1, 3) RUN(1, 4) RUN(2, 2) RUN(2, 3) RUN(4, 2) RUN(4, 3)
  }
  hipFree(x);
  return 0;
}
