// Micro-benchmark (dev tool, not product): the pass-A byte stream M += G (fp32 M in place, bf16 G,
// 10 B per element) under block/wave geometries a projection kernel could use, with the product's
// per-step structure (issue the step's loads, wait, add, store nt) and its occupancy (LDS pad).
//   block = WR x WC waves; a wave owns RW rows x CWB columns of every step; the block walks
//   along the rows (COLWALK = 0: steps advance by WC*CWB columns, the row walk of pass A) or down
//   the columns (COLWALK = 1: steps advance by WR*RW rows, rank_stream's strip walk).
//   K > 1 (row walk): the block's column range is split over K blocks, interleaved step by step
//   (block kc takes steps kc, kc + K, ...) so the K blocks of a row range touch adjacent bytes.
//   PD = 2: the next step's loads are issued before the current step's stores.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

template <typename T>
__device__ __forceinline__ T ldnt(const T* p) { return __builtin_nontemporal_load(p); }
template <typename T>
__device__ __forceinline__ void stnt(T* p, T v) { __builtin_nontemporal_store(v, p); }

__device__ __forceinline__ f32x4 addg4(f32x4 f, u32x2 g) {
  f[0] += __uint_as_float(g[0] << 16);
  f[1] += __uint_as_float(g[0] & 0xFFFF0000u);
  f[2] += __uint_as_float(g[1] << 16);
  f[3] += __uint_as_float(g[1] & 0xFFFF0000u);
  return f;
}

// CWB = columns per wave-step (32 or 64); RW = rows per wave (16 or 32)
template <int WR, int WC, int RW, int CWB, int COLWALK, int PD, int LDSPAD>
__global__ void __launch_bounds__(64 * WR * WC) geo(float* Mb, const uint16_t* Gb, int rows, int cols, int K,
                                                    int kchunk) {
  __shared__ char pad[LDSPAD];
  constexpr int NW = WR * WC;
  constexpr int MI = RW * CWB * 4 / 1024;  // M 16-B-lane instructions per wave-step
  constexpr int GI = RW * CWB * 2 / 1024;  // G instructions
  constexpr int MRPI = 1024 / (CWB * 4);   // rows per M instruction
  constexpr int GRPI = 1024 / (CWB * 2);   // rows per G instruction
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave / WC, wc = wave % WC;
  const long mat = (long)rows * cols;
  float* M = Mb + blockIdx.z * mat;
  const uint16_t* G = Gb + blockIdx.z * mat;
  if (LDSPAD > 16 && lane == 0 && rows < 0) pad[wave] = 1;  // keep the LDS allocation
  // per-lane offsets inside the wave's RW x CWB tile
  const int mr = lane / (CWB / 4), mc = 4 * (lane % (CWB / 4));
  const int gr = lane / (CWB / 8), gc = 8 * (lane % (CWB / 8));
  int r0, c0, nsteps;
  long rstep, cstep;
  if (COLWALK == 0) {
    r0 = blockIdx.x * (WR * RW) + wr * RW;
    c0 = wc * CWB;
    rstep = 0;
    cstep = WC * CWB;
    const int kc = blockIdx.y;
    nsteps = kchunk / (WC * CWB);
    if (K > 1) {
      c0 += kc * WC * CWB;
      cstep *= K;
    } else {
      c0 += kc * kchunk;
    }
  } else {
    r0 = blockIdx.y * kchunk + wr * RW;
    c0 = blockIdx.x * (WC * CWB) + wc * CWB;
    rstep = WR * RW;
    cstep = 0;
    nsteps = kchunk / (WR * RW);
  }
  f32x4 x[PD][MI];
  f32x4 y[MI];
  u32x4 g[PD][GI];
  auto load = [&](int k, int s) {
    const long rr = r0 + s * rstep;
    const long cc = c0 + s * cstep;
#pragma unroll
    for (int i = 0; i < MI; ++i) x[k][i] = ldnt(reinterpret_cast<const f32x4*>(M + (rr + MRPI * i + mr) * cols + cc + mc));
#pragma unroll
    for (int i = 0; i < GI; ++i) g[k][i] = ldnt(reinterpret_cast<const u32x4*>(G + (rr + GRPI * i + gr) * cols + cc + gc));
  };
  auto store = [&](int k, int s) {
    const long rr = r0 + s * rstep;
    const long cc = c0 + s * cstep;
    // pairing of M and G chunks: any lane-consistent pairing keeps the byte stream
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const u32x4 gg = g[k][i / 2];
      y[i] = addg4(x[k][i], (i & 1) ? u32x2{gg[2], gg[3]} : u32x2{gg[0], gg[1]});
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) stnt(reinterpret_cast<f32x4*>(M + (rr + MRPI * i + mr) * cols + cc + mc), y[i]);
  };
  if (PD == 1) {
    for (int s = 0; s < nsteps; ++s) {
      load(0, s);
      store(0, s);
      if (NW > 1) __syncthreads();
    }
  } else {
    load(0, 0);
    for (int s = 0; s < nsteps; s += 2) {
      if (s + 1 < nsteps) load(1, s + 1);
      store(0, s);
      if (NW > 1) __syncthreads();
      if (s + 1 >= nsteps) break;
      if (s + 2 < nsteps) load(0, s + 2);
      store(1, s + 1);
      if (NW > 1) __syncthreads();
    }
  }
}

template <typename F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  f();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int i = 0; i < reps; ++i) f();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

__global__ void fill(float* x, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) x[i] = 1e-3f * (float)(i % 1000);
}

int main() {
  const int nb = 16, rows = 28672, cols = 4096;
  const long n = (long)rows * cols * nb;
  float* M;
  uint16_t* G;
  (void)hipMalloc(&M, n * 4);
  (void)hipMalloc(&G, n * 2);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, M, n);
  (void)hipMemset(G, 0x3b, n * 2);
  (void)hipDeviceSynchronize();
  const double bytes = 10.0 * n;
  auto rep = [&](const char* name, float ms) {
    printf("%-44s %8.3f ms  %6.3f TB/s\n", name, ms, bytes / ms / 1e9);
    fflush(stdout);
  };
  const int reps = 4;
  // LDS pads: 48 KB -> 3 blocks per CU (the product's pass A), 0 -> limited by waves/VGPRs
  for (int round = 0; round < 2; ++round) {
    printf("=== round %d: %d x %d x %d\n", round, nb, rows, cols);
    // A: product geometry, row walk, 4 waves x 32 rows, 32-col steps, whole row per block
    rep("A  rowwalk 4x1 r32 c32 PD1 3blk", timeit([&] { geo<4, 1, 32, 32, 0, 1, 49152><<<dim3(rows / 128, 1, nb), 256>>>(M, G, rows, cols, 1, cols); }, reps));
    rep("A2 rowwalk 4x1 r32 c32 PD2 2blk", timeit([&] { geo<4, 1, 32, 32, 0, 2, 65536><<<dim3(rows / 128, 1, nb), 256>>>(M, G, rows, cols, 1, cols); }, reps));
    rep("A3 rowwalk 4x1 r32 c32 PD1 4blk", timeit([&] { geo<4, 1, 32, 32, 0, 1, 36864><<<dim3(rows / 128, 1, nb), 256>>>(M, G, rows, cols, 1, cols); }, reps));
    // K-interleaved chunks
    rep("E  rowwalk 4x1 r32 c32 PD1 3blk K2", timeit([&] { geo<4, 1, 32, 32, 0, 1, 49152><<<dim3(rows / 128, 2, nb), 256>>>(M, G, rows, cols, 2, cols / 2); }, reps));
    rep("E4 rowwalk 4x1 r32 c32 PD1 3blk K4", timeit([&] { geo<4, 1, 32, 32, 0, 1, 49152><<<dim3(rows / 128, 4, nb), 256>>>(M, G, rows, cols, 4, cols / 4); }, reps));
    rep("Ec rowwalk 4x1 r32 c32 PD1 3blk chunk4", timeit([&] { geo<4, 1, 32, 32, 0, 1, 49152><<<dim3(rows / 128, 4, nb), 256>>>(M, G, rows, cols, 1, cols / 4); }, reps));
    // wider steps
    rep("D  rowwalk 4x1 r32 c64 PD1 3blk", timeit([&] { geo<4, 1, 32, 64, 0, 1, 49152><<<dim3(rows / 128, 1, nb), 256>>>(M, G, rows, cols, 1, cols); }, reps));
    rep("D2 rowwalk 4x1 r16 c64 PD1 3blk", timeit([&] { geo<4, 1, 16, 64, 0, 1, 49152><<<dim3(rows / 64, 1, nb), 256>>>(M, G, rows, cols, 1, cols); }, reps));
    // waves side by side on the same rows
    rep("B  rowwalk 1x4 r32 c32 PD1 3blk", timeit([&] { geo<1, 4, 32, 32, 0, 1, 49152><<<dim3(rows / 32, 1, nb), 256>>>(M, G, rows, cols, 1, cols); }, reps));
    rep("C  rowwalk 2x2 r32 c32 PD1 3blk", timeit([&] { geo<2, 2, 32, 32, 0, 1, 49152><<<dim3(rows / 64, 1, nb), 256>>>(M, G, rows, cols, 1, cols); }, reps));
    rep("F  rowwalk 1x8 r32 c32 PD1 1blk", timeit([&] { geo<1, 8, 32, 32, 0, 1, 81920><<<dim3(rows / 32, 1, nb), 512>>>(M, G, rows, cols, 1, cols); }, reps));
    rep("F2 rowwalk 1x8 r32 c32 PD1 2blk", timeit([&] { geo<1, 8, 32, 32, 0, 1, 65536><<<dim3(rows / 32, 1, nb), 512>>>(M, G, rows, cols, 1, cols); }, reps));
    // strip (rank_stream's walk): 8 waves x 32 cols, 32-row steps, kchunk rows per block
    rep("S  strip 1x8 r32 c32 PD2 2blk kc1024", timeit([&] { geo<1, 8, 32, 32, 1, 2, 65536><<<dim3(cols / 256, rows / 1024, nb), 512>>>(M, G, rows, cols, 1, 1024); }, reps));
    rep("S1 strip 1x8 r32 c32 PD1 2blk kc1024", timeit([&] { geo<1, 8, 32, 32, 1, 1, 65536><<<dim3(cols / 256, rows / 1024, nb), 512>>>(M, G, rows, cols, 1, 1024); }, reps));
    rep("S4 strip 1x4 r32 c32 PD1 3blk kc1024", timeit([&] { geo<1, 4, 32, 32, 1, 1, 49152><<<dim3(cols / 128, rows / 1024, nb), 256>>>(M, G, rows, cols, 1, 1024); }, reps));
  }
  (void)hipFree(M);
  (void)hipFree(G);
  return 0;
}
