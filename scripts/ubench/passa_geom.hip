// Micro-benchmark (dev tool, not product): candidate geometries for the pass-A stream
// M += G (fp32 M in place, bf16 G; 10 B per element), no arithmetic besides the add.
// Every block-row variant keeps 128 rows per block (4 stacked waves of 32 rows) so a
// block shares one staged copy of the thin operand per column step, as pass A needs.
//   cur   : the product's loads: M whole lines (lane: row 8q + l/8, 16 B at 4 (l%8)), G in
//           the MFMA layout (lane (t, g): rows 16 rb + t, 8 B at 16 c + 4 g): 32-col steps
//   gtj   : as cur, G whole half-lines (lane: row 16q + l/4, 16 B at 8 (l%4))
//   w64   : 64-col steps: M lane row 4q + l/16, 16 B at 4 (l%16); G lane row 8q + l/8,
//           16 B at 8 (l%8) (every G instruction = 8 whole 128-B lines)
//   w64b  : as w64 with buffer loads/stores (nt aux bits)
//   strip : rank_stream geometry: 8 waves side by side (256 columns), 32-row steps down
//           the rows, 32x32 accumulator layout (b32 loads, 2 rows x 128 B per instruction)
//   flat  : grid-stride float4 M + 8-B G (the ceiling)
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <typename T>
__device__ __forceinline__ T ld(const T* p) { return __builtin_nontemporal_load(p); }
template <typename T>
__device__ __forceinline__ void st(T* p, T v) { __builtin_nontemporal_store(v, p); }
template <typename T, bool NT>
__device__ __forceinline__ T ldp(const T* p) { if constexpr (NT) return __builtin_nontemporal_load(p); else return *p; }

__device__ __forceinline__ f32x4 add_lo(f32x4 f, u32x2 g) {
  f[0] += __uint_as_float(g[0] << 16);
  f[1] += __uint_as_float(g[0] & 0xFFFF0000u);
  f[2] += __uint_as_float(g[1] << 16);
  f[3] += __uint_as_float(g[1] & 0xFFFF0000u);
  return f;
}

// ---- cur / gtj: 32-col steps, D-deep register ring
template <int GMODE, int D>
__global__ void __launch_bounds__(256, 2) walk32(float* Mb, const unsigned short* Gb, int rows, int cols) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long mat = (long)rows * cols;
  float* M = Mb + blockIdx.z * mat;
  const unsigned short* G = Gb + blockIdx.z * mat;
  const int r0 = blockIdx.x * 128 + wave * 32;
  f32x4 x[D][4];
  u32x2 g2[D][4];
  u32x4 g4[D][2];
  auto load = [&](int k, int j) {
#pragma unroll
    for (int q = 0; q < 4; ++q) x[k][q] = ld(reinterpret_cast<const f32x4*>(M + (long)(r0 + 8 * q + (lane >> 3)) * cols + j + 4 * (lane & 7)));
    if constexpr (GMODE == 0 || GMODE == 2) {
#pragma unroll
      for (int v = 0; v < 4; ++v)
        g2[k][v] = ldp<u32x2, GMODE == 2>(reinterpret_cast<const u32x2*>(G + (long)(r0 + 16 * (v >> 1) + (lane & 15)) * cols + j + 16 * (v & 1) + 4 * (lane >> 4)));
    } else {
#pragma unroll
      for (int q = 0; q < 2; ++q)
        g4[k][q] = ld(reinterpret_cast<const u32x4*>(G + (long)(r0 + 16 * q + (lane >> 2)) * cols + j + 8 * (lane & 3)));
    }
  };
  auto store = [&](int k, int j) {
    // the add pairs M chunks with G chunks of other lanes in the product (LDS transpose);
    // here any lane-consistent pairing keeps the byte stream the same
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      u32x2 gg = GMODE != 1 ? g2[k][q] : u32x2{g4[k][q >> 1][2 * (q & 1)], g4[k][q >> 1][2 * (q & 1) + 1]};
      st(reinterpret_cast<f32x4*>(M + (long)(r0 + 8 * q + (lane >> 3)) * cols + j + 4 * (lane & 7)), add_lo(x[k][q], gg));
    }
  };
#pragma unroll
  for (int k = 0; k < D - 1; ++k) load(k, 32 * k);
  for (int j0 = 0; j0 < cols; j0 += 32 * D) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const int j = j0 + 32 * k;
      if (j >= cols) break;
      if (j + 32 * (D - 1) < cols) load((k + D - 1) % D, j + 32 * (D - 1));
      store(k, j);
    }
  }
}

// ---- w64: 64-col steps
template <int D, bool GNT>
__global__ void __launch_bounds__(256, 2) walk64(float* Mb, const unsigned short* Gb, int rows, int cols) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long mat = (long)rows * cols;
  float* M = Mb + blockIdx.z * mat;
  const unsigned short* G = Gb + blockIdx.z * mat;
  const int r0 = blockIdx.x * 128 + wave * 32;
  f32x4 x[D][8];
  u32x4 g[D][4];
  auto load = [&](int k, int j) {
#pragma unroll
    for (int q = 0; q < 8; ++q) x[k][q] = ld(reinterpret_cast<const f32x4*>(M + (long)(r0 + 4 * q + (lane >> 4)) * cols + j + 4 * (lane & 15)));
#pragma unroll
    for (int q = 0; q < 4; ++q) g[k][q] = ldp<u32x4, GNT>(reinterpret_cast<const u32x4*>(G + (long)(r0 + 8 * q + (lane >> 3)) * cols + j + 8 * (lane & 7)));
  };
  auto store = [&](int k, int j) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      u32x2 gg{g[k][q >> 1][2 * (q & 1)], g[k][q >> 1][2 * (q & 1) + 1]};
      st(reinterpret_cast<f32x4*>(M + (long)(r0 + 4 * q + (lane >> 4)) * cols + j + 4 * (lane & 15)), add_lo(x[k][q], gg));
    }
  };
#pragma unroll
  for (int k = 0; k < D - 1; ++k) load(k, 64 * k);
  for (int j0 = 0; j0 < cols; j0 += 64 * D) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const int j = j0 + 64 * k;
      if (j >= cols) break;
      if (j + 64 * (D - 1) < cols) load((k + D - 1) % D, j + 64 * (D - 1));
      store(k, j);
    }
  }
}

// ---- strip: rank_stream geometry (8 waves x 32 columns, 32-row steps, D = 2)
__global__ void __launch_bounds__(512) strip(float* Mb, const unsigned short* Gb, int rows, int cols, int sl) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, t = lane & 31, h = lane >> 5;
  const long mat = (long)rows * cols;
  float* M = Mb + blockIdx.z * mat;
  const unsigned short* G = Gb + blockIdx.z * mat;
  const int c0 = blockIdx.x * 256 + wave * 32 + t;
  const int i_begin = blockIdx.y * sl, i_end = min(rows, i_begin + sl);
  float x[2][16];
  unsigned short g[2][16];
  auto row = [&](int q) { return (q & 3) + 8 * (q >> 2) + 4 * h; };
  auto load = [&](int k, int i) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      x[k][q] = ld(M + (long)(i + row(q)) * cols + c0);
      g[k][q] = ld(G + (long)(i + row(q)) * cols + c0);
    }
  };
  auto store = [&](int k, int i) {
#pragma unroll
    for (int q = 0; q < 16; ++q) st(M + (long)(i + row(q)) * cols + c0, x[k][q] + __uint_as_float((unsigned)g[k][q] << 16));
  };
  load(0, i_begin);
  for (int i = i_begin; i < i_end; i += 64) {
    if (i + 32 < i_end) load(1, i + 32);
    store(0, i);
    if (i + 32 >= i_end) break;
    if (i + 64 < i_end) load(0, i + 64);
    store(1, i + 32);
  }
}

__global__ void __launch_bounds__(256) flat(f32x4* M, const u32x2* G, long n4) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) st(M + i, add_lo(ld(M + i), ld(G + i)));
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
  const int nb = 8;
  const int shapes[2][2] = {{28672, 4096}, {6144, 4096}};
  for (auto& sh : shapes) {
    const int rows = sh[0], cols = sh[1];
    const long n = (long)rows * cols * nb;
    float* M;
    unsigned short* G;
    hipMalloc(&M, n * 4);
    hipMalloc(&G, n * 2);
    hipMemset(M, 0, n * 4);
    hipMemset(G, 0, n * 2);
    printf("--- %d x %d x %d (%.2f GB per call)\n", nb, rows, cols, 10.0 * n / 1e9);
    auto rep = [&](const char* name, float ms) {
      printf("%-24s %8.3f ms  %7.3f TB/s\n", name, ms, 10.0 * n / ms / 1e9);
      fflush(stdout);
    };
    for (int round = 0; round < 2; ++round) {
      rep("flat", timeit([&] { flat<<<4096, 256>>>((f32x4*)M, (const u32x2*)G, n / 4); }, 10));
      rep("cur D2", timeit([&] { walk32<0, 2><<<dim3(rows / 128, 1, nb), 256>>>(M, G, rows, cols); }, 10));
      rep("cur D3", timeit([&] { walk32<0, 3><<<dim3(rows / 128, 1, nb), 256>>>(M, G, rows, cols); }, 10));
      rep("cur gnt D2", timeit([&] { walk32<2, 2><<<dim3(rows / 128, 1, nb), 256>>>(M, G, rows, cols); }, 10));
      rep("gtj D2", timeit([&] { walk32<1, 2><<<dim3(rows / 128, 1, nb), 256>>>(M, G, rows, cols); }, 10));
      rep("gtj D3", timeit([&] { walk32<1, 3><<<dim3(rows / 128, 1, nb), 256>>>(M, G, rows, cols); }, 10));
      rep("w64 D2 gnt", timeit([&] { walk64<2, true><<<dim3(rows / 128, 1, nb), 256>>>(M, G, rows, cols); }, 10));
      rep("w64 D2 gdef", timeit([&] { walk64<2, false><<<dim3(rows / 128, 1, nb), 256>>>(M, G, rows, cols); }, 10));
      rep("w64 D3 gnt", timeit([&] { walk64<3, true><<<dim3(rows / 128, 1, nb), 256>>>(M, G, rows, cols); }, 10));
      rep("strip sl1024", timeit([&] { strip<<<dim3(cols / 256, rows / 1024, nb), 512>>>(M, G, rows, cols, 1024); }, 10));
      rep("strip sl2048", timeit([&] { strip<<<dim3(cols / 256, rows / 2048, nb), 512>>>(M, G, rows, cols, 2048); }, 10));
    }
    hipFree(M);
    hipFree(G);
  }
  return 0;
}
