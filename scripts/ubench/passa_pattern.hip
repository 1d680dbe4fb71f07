// Micro-benchmark (dev tool, not product): the access patterns a pass-A row kernel can
// use for the in-place M += G stream (fp32 M, bf16 G), no arithmetic besides the add.
// Block = 4 waves, wave = 32 rows, a block streams 128 rows across all columns, one
// step of registers in flight (double buffer), like rowproj_ef_kernel.
//   pat 0: lane (t, g) rows t, t + 16; columns 16 c + 4 g .. +3, c < C (C = 2: 32-col steps)
//   pat 1: lane l: row (l / 8) + 8 i (i < 4); columns 4 (l % 8) .. +3 of a 32-col step
//          (every instruction covers 8 full 128-B lines)
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

template <typename T, bool NT>
__device__ __forceinline__ T ld(const T* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <typename T, bool NT>
__device__ __forceinline__ void st(T* p, T v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <int PAT, int C, bool NT>
__global__ void __launch_bounds__(256, 2) rowpat(float* Mb, const unsigned short* Gb, int rows, int cols) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int b = blockIdx.z;
  float* M = Mb + (long)b * rows * cols;
  const unsigned short* G = Gb + (long)b * rows * cols;
  const int row_base = blockIdx.x * 128 + wave * 32;
  constexpr int NV = PAT == 0 ? 2 * C : 4;  // f32x4 per lane per step
  constexpr int STEP = PAT == 0 ? 16 * C : 32;
  long off[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    if constexpr (PAT == 0) {
      const int rb = v / C, c = v % C;
      off[v] = (long)(row_base + 16 * rb + (lane & 15)) * cols + 16 * c + 4 * (lane >> 4);
    } else {
      off[v] = (long)(row_base + (lane >> 3) + 8 * v) * cols + 4 * (lane & 7);
    }
  }
  f32x4 xa[NV], xb[NV];
  u32x2 ga[NV], gb[NV];
  auto load = [&](int j, f32x4* x, u32x2* g) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      x[v] = ld<f32x4, NT>(reinterpret_cast<const f32x4*>(M + off[v] + j));
      g[v] = ld<u32x2, NT>(reinterpret_cast<const u32x2*>(G + off[v] + j));
    }
  };
  auto store = [&](int j, f32x4* x, u32x2* g) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      f32x4 f = x[v];
      f[0] += __uint_as_float(g[v][0] << 16);
      f[1] += __uint_as_float(g[v][0] & 0xFFFF0000u);
      f[2] += __uint_as_float(g[v][1] << 16);
      f[3] += __uint_as_float(g[v][1] & 0xFFFF0000u);
      st<f32x4, NT>(reinterpret_cast<f32x4*>(M + off[v] + j), f);
    }
  };
  load(0, xa, ga);
  for (int j = 0; j < cols; j += 2 * STEP) {
    if (j + STEP < cols) load(j + STEP, xb, gb);
    store(j, xa, ga);
    if (j + STEP >= cols) break;
    if (j + 2 * STEP < cols) load(j + 2 * STEP, xa, ga);
    store(j + STEP, xb, gb);
  }
}

// band pattern: block = NW waves over a band of BR rows; at step s wave w covers columns
// 32 w + 32 NW s (the block covers 32 NW contiguous columns = 128 NW bytes of each row);
// lane (t, g): rows 16 rb + t, columns 16 c + 4 g .. +3 (c = 0, 1) of the wave's 32
template <int NW, int BR, bool NT>
__global__ void __launch_bounds__(64 * NW) bandpat(float* Mb, const unsigned short* Gb, int rows, int cols) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int b = blockIdx.z;
  float* M = Mb + (long)b * rows * cols;
  const unsigned short* G = Gb + (long)b * rows * cols;
  constexpr int NRB = BR / 16;
  constexpr int NV = 2 * NRB;
  long off[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int rb = v / 2, c = v % 2;
    off[v] = (long)(blockIdx.x * BR + 16 * rb + (lane & 15)) * cols + 32 * wave + 16 * c + 4 * (lane >> 4);
  }
  constexpr int STEP = 32 * NW;
  f32x4 xa[NV], xb[NV];
  u32x2 ga[NV], gb[NV];
  auto load = [&](int j, f32x4* x, u32x2* g) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      x[v] = ld<f32x4, NT>(reinterpret_cast<const f32x4*>(M + off[v] + j));
      g[v] = ld<u32x2, NT>(reinterpret_cast<const u32x2*>(G + off[v] + j));
    }
  };
  auto store = [&](int j, f32x4* x, u32x2* g) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      f32x4 f = x[v];
      f[0] += __uint_as_float(g[v][0] << 16);
      f[1] += __uint_as_float(g[v][0] & 0xFFFF0000u);
      f[2] += __uint_as_float(g[v][1] << 16);
      f[3] += __uint_as_float(g[v][1] & 0xFFFF0000u);
      st<f32x4, NT>(reinterpret_cast<f32x4*>(M + off[v] + j), f);
    }
  };
  load(0, xa, ga);
  for (int j = 0; j < cols; j += 2 * STEP) {
    if (j + STEP < cols) load(j + STEP, xb, gb);
    store(j, xa, ga);
    if (j + STEP >= cols) break;
    if (j + 2 * STEP < cols) load(j + 2 * STEP, xa, ga);
    store(j + STEP, xb, gb);
  }
}

// row walk with depth: block = NW stacked waves, wave = 16 RB rows; step = 32 columns;
// DEPTH steps in flight per wave (register ring)
template <int NW, int RB, int DEPTH, int MINB>
__global__ void __launch_bounds__(64 * NW, MINB) walkpat(float* Mb, const unsigned short* Gb, int rows, int cols) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int b = blockIdx.z;
  float* M = Mb + (long)b * rows * cols;
  const unsigned short* G = Gb + (long)b * rows * cols;
  constexpr int NV = 2 * RB;
  long off[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int rb = v / 2, c = v % 2;
    off[v] = (long)(blockIdx.x * (16 * RB * NW) + wave * 16 * RB + 16 * rb + (lane & 15)) * cols + 16 * c + 4 * (lane >> 4);
  }
  f32x4 x[DEPTH][NV];
  u32x2 g[DEPTH][NV];
  auto load = [&](int j, f32x4* xx, u32x2* gg) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      xx[v] = *reinterpret_cast<const f32x4*>(M + off[v] + j);
      gg[v] = *reinterpret_cast<const u32x2*>(G + off[v] + j);
    }
  };
  auto store = [&](int j, f32x4* xx, u32x2* gg) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      f32x4 f = xx[v];
      f[0] += __uint_as_float(gg[v][0] << 16);
      f[1] += __uint_as_float(gg[v][0] & 0xFFFF0000u);
      f[2] += __uint_as_float(gg[v][1] << 16);
      f[3] += __uint_as_float(gg[v][1] & 0xFFFF0000u);
      *reinterpret_cast<f32x4*>(M + off[v] + j) = f;
    }
  };
#pragma unroll
  for (int k = 0; k < DEPTH - 1; ++k) load(32 * k, x[k], g[k]);
  for (int j0 = 0; j0 < cols; j0 += 32 * DEPTH) {
#pragma unroll
    for (int k = 0; k < DEPTH; ++k) {
      const int j = j0 + 32 * k;
      if (j >= cols) break;
      if (j + 32 * (DEPTH - 1) < cols) load(j + 32 * (DEPTH - 1), x[(k + DEPTH - 1) % DEPTH], g[(k + DEPTH - 1) % DEPTH]);
      store(j, x[k], g[k]);
    }
  }
}

// strip walk: block = NW waves side by side (wave w: 32 columns 32 w of the block's 32 NW),
// walking DOWN a range of SL rows in 32-row steps; lane (t, g) rows 16 rb + t, cols 16 c + 4 g
template <int NW, int SL, bool NT>
__global__ void __launch_bounds__(64 * NW) stripwalk(float* Mb, const unsigned short* Gb, int rows, int cols) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int b = blockIdx.z;
  float* M = Mb + (long)b * rows * cols;
  const unsigned short* G = Gb + (long)b * rows * cols;
  long off[4];
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int rb = v / 2, c = v % 2;
    off[v] = (long)(blockIdx.y * SL + 16 * rb + (lane & 15)) * cols + blockIdx.x * 32 * NW + 32 * wave + 16 * c + 4 * (lane >> 4);
  }
  f32x4 xa[4], xb[4];
  u32x2 ga[4], gb[4];
  auto load = [&](long i, f32x4* x, u32x2* g) {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      x[v] = ld<f32x4, NT>(reinterpret_cast<const f32x4*>(M + off[v] + i * cols));
      g[v] = ld<u32x2, NT>(reinterpret_cast<const u32x2*>(G + off[v] + i * cols));
    }
  };
  auto store = [&](long i, f32x4* x, u32x2* g) {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      f32x4 f = x[v];
      f[0] += __uint_as_float(g[v][0] << 16);
      f[1] += __uint_as_float(g[v][0] & 0xFFFF0000u);
      f[2] += __uint_as_float(g[v][1] << 16);
      f[3] += __uint_as_float(g[v][1] & 0xFFFF0000u);
      st<f32x4, NT>(reinterpret_cast<f32x4*>(M + off[v] + i * cols), f);
    }
  };
  load(0, xa, ga);
  for (int i = 0; i < SL; i += 64) {
    if (i + 32 < SL) load(i + 32, xb, gb);
    store(i, xa, ga);
    if (i + 32 >= SL) break;
    if (i + 64 < SL) load(i + 64, xa, ga);
    store(i + 32, xb, gb);
  }
}

// row walk with a per-block rotated start column (partition-camping test): block = 4 stacked
// waves of 32 rows, 32-col steps, start at column (blockIdx.x * ROT) mod cols, wrap around
template <int ROT>
__global__ void __launch_bounds__(256, 2) rotwalk(float* Mb, const unsigned short* Gb, int rows, int cols) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int b = blockIdx.z;
  float* M = Mb + (long)b * rows * cols;
  const unsigned short* G = Gb + (long)b * rows * cols;
  long off[4];
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int rb = v / 2, c = v % 2;
    off[v] = (long)(blockIdx.x * 128 + wave * 32 + 16 * rb + (lane & 15)) * cols + 16 * c + 4 * (lane >> 4);
  }
  const int j0 = (int)(((long)(blockIdx.x + 7 * blockIdx.z) * ROT) % cols) & ~31;
  f32x4 xa[4], xb[4];
  u32x2 ga[4], gb[4];
  auto load = [&](int j, f32x4* x, u32x2* g) {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      x[v] = *reinterpret_cast<const f32x4*>(M + off[v] + j);
      g[v] = *reinterpret_cast<const u32x2*>(G + off[v] + j);
    }
  };
  auto store = [&](int j, f32x4* x, u32x2* g) {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      f32x4 f = x[v];
      f[0] += __uint_as_float(g[v][0] << 16);
      f[1] += __uint_as_float(g[v][0] & 0xFFFF0000u);
      f[2] += __uint_as_float(g[v][1] << 16);
      f[3] += __uint_as_float(g[v][1] & 0xFFFF0000u);
      *reinterpret_cast<f32x4*>(M + off[v] + j) = f;
    }
  };
  auto col = [&](int k) { int j = j0 + 32 * k; return j >= cols ? j - cols : j; };
  const int nsteps = cols / 32;
  load(col(0), xa, ga);
  for (int k = 0; k < nsteps; k += 2) {
    if (k + 1 < nsteps) load(col(k + 1), xb, gb);
    store(col(k), xa, ga);
    if (k + 1 >= nsteps) break;
    if (k + 2 < nsteps) load(col(k + 2), xa, ga);
    store(col(k + 1), xb, gb);
  }
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
  const int rows = 28672, cols = 4096, nb = 8;
  const long n = (long)rows * cols * nb;
  float* M;
  unsigned short* G;
  hipMalloc(&M, n * 4);
  hipMalloc(&G, n * 2);
  hipMemset(M, 0, n * 4);
  hipMemset(G, 0, n * 2);
  auto rep = [&](const char* name, float ms) {
    printf("%-28s %8.3f ms  %7.3f TB/s\n", name, ms, 10.0 * n / ms / 1e9);
    fflush(stdout);
  };
  dim3 grid(rows / 128, 1, nb);
#define R(P, C, NT) rep("pat" #P " C" #C " nt" #NT, timeit([&] { rowpat<P, C, NT><<<grid, 256>>>(M, G, rows, cols); }, 10));
  R(0, 2, false) R(1, 2, false)
#define RW(ROT) rep("rotwalk " #ROT, timeit([&] { rotwalk<ROT><<<dim3(rows / 128, 1, nb), 256>>>(M, G, rows, cols); }, 10));
  RW(0) RW(32) RW(96) RW(256) RW(544) RW(1056)
#define S(NW, SL, NT) rep("strip NW" #NW " SL" #SL " nt" #NT, timeit([&] { stripwalk<NW, SL, NT><<<dim3(cols / (32 * NW), rows / SL, nb), 64 * NW>>>(M, G, rows, cols); }, 10));
  S(16, 256, false) S(8, 256, false)
#define W(NW, RB, D, MB) rep("walk NW" #NW " RB" #RB " D" #D " mb" #MB, timeit([&] { walkpat<NW, RB, D, MB><<<dim3(rows / (16 * RB * NW), 1, nb), 64 * NW>>>(M, G, rows, cols); }, 10));

#define B(NW, BR, NT) rep("band NW" #NW " BR" #BR " nt" #NT, timeit([&] { bandpat<NW, BR, NT><<<dim3(rows / BR, 1, nb), 64 * NW>>>(M, G, rows, cols); }, 10));

  B(8, 16, false) B(8, 16, true) B(16, 32, false) B(16, 32, true)
  hipFree(M);
  hipFree(G);
  return 0;
}
