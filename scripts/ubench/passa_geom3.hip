// Micro-benchmark (dev tool, not product): the pass-A byte stream M += G (fp32 M in place, bf16 G,
// 10 B per element) under block/wave geometries, with the product's per-step structure (issue the
// step's loads, wait, add, store nt, barrier) and controlled occupancy (LDS pad).
//   block = WR x WC waves; a wave owns 32 rows x CWB columns of a step; the block walks along the
//   rows (row walk: a step advances WC*CWB columns).  Access shapes per wave-instruction:
//     MF = 0: M whole tile rows (8 rows x 128 B at CWB = 32);  MF = 1: MFMA fragments (16 rows x 64 B)
//     GF = 0: G tile rows, 16 B per lane (half lines at CWB = 32); GF = 1: fragments (16 rows x 32 B,
//             8 B per lane, the product's pass A)
//     GNT: nt policy on G (else default: a partial line then stays in L2 for its other half)
//   STRIP = 1: rank_stream's walk instead (the block owns WC*CWB columns and steps down the rows).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

template <typename T, bool NT>
__device__ __forceinline__ T ld(const T* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <typename T>
__device__ __forceinline__ void stnt(T* p, T v) { __builtin_nontemporal_store(v, p); }

__device__ __forceinline__ f32x4 addg4(f32x4 f, u32x2 g) {
  f[0] += __uint_as_float(g[0] << 16);
  f[1] += __uint_as_float(g[0] & 0xFFFF0000u);
  f[2] += __uint_as_float(g[1] << 16);
  f[3] += __uint_as_float(g[1] & 0xFFFF0000u);
  return f;
}

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
template <int WR, int WC, int CWB, int MF, int GF, bool GNT, int STRIP, int PD, int LDSPAD, int CMP = 0>
__global__ void __launch_bounds__(64 * WR * WC) geo(float* Mb, const uint16_t* Gb, int rows, int cols, int kchunk) {
  __shared__ char pad[LDSPAD];
  constexpr int RW = 32;
  constexpr int NM = RW * CWB * 4 / 1024;  // M instructions per wave-step (16 B per lane)
  constexpr int NG = GF ? RW * CWB * 2 / 512 : RW * CWB * 2 / 1024;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave / WC, wc = wave % WC;
  const long mat = (long)rows * cols;
  float* M = Mb + blockIdx.z * mat;
  const uint16_t* G = Gb + blockIdx.z * mat;
  if (lane == 0 && rows < 0) pad[wave] = 1;
  // per-lane (row, col) of M instruction i and G instruction i inside the wave's 32 x CWB tile
  auto mpos = [&](int i, int& r, int& c) {
    if (MF == 0) {
      const int lpr = CWB / 4;  // lanes per tile row
      r = (64 / lpr) * i + lane / lpr;
      c = 4 * (lane % lpr);
    } else {  // 16 rows x 64 B per instruction: i = (row half, 16-col group)
      const int ncg = CWB / 16;
      r = 16 * (i / ncg) + (lane & 15);
      c = 16 * (i % ncg) + 4 * (lane >> 4);
    }
  };
  auto gpos = [&](int i, int& r, int& c) {
    if (GF == 0) {
      const int lpr = CWB / 8;
      r = (64 / lpr) * i + lane / lpr;
      c = 8 * (lane % lpr);
    } else {  // 16 rows x 32 B (4 lanes x 8 B per row)
      const int ncg = CWB / 16;
      r = 16 * (i / ncg) + (lane & 15);
      c = 16 * (i % ncg) + 4 * (lane >> 4);
    }
  };
  long r0, c0, rstep, cstep;
  int nsteps;
  if (STRIP == 0) {
    r0 = blockIdx.x * (WR * RW) + wr * RW;
    c0 = (long)blockIdx.y * kchunk + wc * CWB;
    rstep = 0;
    cstep = WC * CWB;
    nsteps = kchunk / (WC * CWB);
  } else {
    r0 = (long)blockIdx.y * kchunk + wr * RW;
    c0 = blockIdx.x * (WC * CWB) + wc * CWB;
    rstep = WR * RW;
    cstep = 0;
    nsteps = kchunk / (WR * RW);
  }
  f32x4 x[PD][NM];
  u32x4 g4[PD][GF ? 1 : NG];
  u32x2 g2[PD][GF ? NG : 1];
  auto load = [&](int k, int s) {
    const long rr = r0 + s * rstep, cc = c0 + s * cstep;
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      int r, c;
      mpos(i, r, c);
      x[k][i] = ld<f32x4, true>(reinterpret_cast<const f32x4*>(M + (rr + r) * cols + cc + c));
    }
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      int r, c;
      gpos(i, r, c);
      if (GF) g2[k][i] = ld<u32x2, GNT>(reinterpret_cast<const u32x2*>(G + (rr + r) * cols + cc + c));
      else g4[k][i] = ld<u32x4, GNT>(reinterpret_cast<const u32x4*>(G + (rr + r) * cols + cc + c));
    }
  };
  auto store = [&](int k, int s) {
    const long rr = r0 + s * rstep, cc = c0 + s * cstep;
    if constexpr (CMP > 0) {
      // stand-in for the projection: CMP data-dependent 16x16x32 f16 MFMAs on the step's tile
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const f16x8 a = __builtin_bit_cast(f16x8, x[k][0]);
      const f16x8 b = __builtin_bit_cast(f16x8, x[k][NM - 1]);
#pragma unroll
      for (int q = 0; q < CMP; ++q) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc, 0, 0, 0);
      x[k][0][0] += acc[0] * 1e-38f;
    }
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      u32x2 gg;
      if (GF) gg = g2[k][i % NG];
      else {
        const u32x4 q = g4[k][(i / 2) % NG];
        gg = (i & 1) ? u32x2{q[2], q[3]} : u32x2{q[0], q[1]};
      }
      int r, c;
      mpos(i, r, c);
      stnt(reinterpret_cast<f32x4*>(M + (rr + r) * cols + cc + c), addg4(x[k][i], gg));
    }
  };
  if (PD == 1) {
    for (int s = 0; s < nsteps; ++s) {
      load(0, s);
      store(0, s);
      __syncthreads();
    }
  } else {
    load(0, 0);
    for (int s = 0; s < nsteps; s += 2) {
      if (s + 1 < nsteps) load(1, s + 1);
      store(0, s);
      __syncthreads();
      if (s + 1 >= nsteps) break;
      if (s + 2 < nsteps) load(0, s + 2);
      store(1, s + 1);
      __syncthreads();
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
    printf("%-52s %8.3f ms  %6.3f TB/s\n", name, ms, bytes / ms / 1e9);
    fflush(stdout);
  };
  const int reps = 4;
  for (int round = 0; round < 2; ++round) {
    printf("=== round %d: %d x %d x %d\n", round, nb, rows, cols);
    // the product's pass A: 4 waves x 32 rows, 32-col steps, M lines, G fragments default, 3 blocks/CU
    rep("A   row 4x1 c32 Mline Gfrag-def 3blk", timeit([&] { geo<4, 1, 32, 0, 1, false, 0, 1, 49152><<<dim3(rows / 128, 1, nb), 256>>>(M, G, rows, cols, cols); }, reps));
    rep("A1  row 4x1 c32 Mline Ghalf-def 3blk", timeit([&] { geo<4, 1, 32, 0, 0, false, 0, 1, 49152><<<dim3(rows / 128, 1, nb), 256>>>(M, G, rows, cols, cols); }, reps));
    rep("A2  row 4x1 c32 Mfrag Gfrag-def 3blk", timeit([&] { geo<4, 1, 32, 1, 1, false, 0, 1, 49152><<<dim3(rows / 128, 1, nb), 256>>>(M, G, rows, cols, cols); }, reps));
    rep("A3  row 4x1 c32 Mline Gfrag-def PD2 2blk", timeit([&] { geo<4, 1, 32, 0, 1, false, 0, 2, 65536><<<dim3(rows / 128, 1, nb), 256>>>(M, G, rows, cols, cols); }, reps));
    // 64-col wave steps (G whole lines)
    rep("D   row 4x1 c64 Mline Gline-nt 3blk", timeit([&] { geo<4, 1, 64, 0, 0, true, 0, 1, 49152><<<dim3(rows / 128, 1, nb), 256>>>(M, G, rows, cols, cols); }, reps));
    rep("D1  row 4x1 c64 Mline Gline-nt 2blk", timeit([&] { geo<4, 1, 64, 0, 0, true, 0, 1, 65536><<<dim3(rows / 128, 1, nb), 256>>>(M, G, rows, cols, cols); }, reps));
    // waves side by side on the same rows
    rep("B   row 1x4 c32 Mline Gfrag-def 3blk", timeit([&] { geo<1, 4, 32, 0, 1, false, 0, 1, 49152><<<dim3(rows / 32, 1, nb), 256>>>(M, G, rows, cols, cols); }, reps));
    rep("B1  row 1x4 c32 Mline Ghalf-def 3blk", timeit([&] { geo<1, 4, 32, 0, 0, false, 0, 1, 49152><<<dim3(rows / 32, 1, nb), 256>>>(M, G, rows, cols, cols); }, reps));
    rep("H   row 3x4 c32 Mfrag Gfrag-def 1blk(12w)", timeit([&] { geo<3, 4, 32, 1, 1, false, 0, 1, 98304><<<dim3(rows / 96, 1, nb), 768>>>(M, G, rows, cols, cols); }, reps));
    rep("H1  row 3x4 c32 Mline Gfrag-def 1blk(12w)", timeit([&] { geo<3, 4, 32, 0, 1, false, 0, 1, 98304><<<dim3(rows / 96, 1, nb), 768>>>(M, G, rows, cols, cols); }, reps));
    rep("H2  row 2x4 c32 Mline Gfrag-def 1blk(8w)", timeit([&] { geo<2, 4, 32, 0, 1, false, 0, 1, 98304><<<dim3(rows / 64, 1, nb), 512>>>(M, G, rows, cols, cols); }, reps));
    rep("F   row 1x8 c32 Mline Gfrag-def 2blk", timeit([&] { geo<1, 8, 32, 0, 1, false, 0, 1, 65536><<<dim3(rows / 32, 1, nb), 512>>>(M, G, rows, cols, cols); }, reps));
    // with a stand-in for the projection work (48 MFMAs per wave-step)
    rep("Ac  row 4x1 c32 Mline Gfrag-def 3blk +48mfma", timeit([&] { geo<4, 1, 32, 0, 1, false, 0, 1, 49152, 48><<<dim3(rows / 128, 1, nb), 256>>>(M, G, rows, cols, cols); }, reps));
    rep("H1c row 3x4 c32 Mline Gfrag-def 1blk(12w) +48mfma", timeit([&] { geo<3, 4, 32, 0, 1, false, 0, 1, 98304, 48><<<dim3(rows / 96, 1, nb), 768>>>(M, G, rows, cols, cols); }, reps));
    rep("H3c row 4x2 c32 Mline Gfrag-def 1blk(8w) +48mfma", timeit([&] { geo<4, 2, 32, 0, 1, false, 0, 1, 98304, 48><<<dim3(rows / 128, 1, nb), 512>>>(M, G, rows, cols, cols); }, reps));
    rep("H4c row 2x4 c32 Mline Gfrag-def 2blk(8w) +48mfma", timeit([&] { geo<2, 4, 32, 0, 1, false, 0, 1, 65536, 48><<<dim3(rows / 64, 1, nb), 512>>>(M, G, rows, cols, cols); }, reps));
    rep("Bc  row 1x4 c32 Mline Gfrag-def 3blk +48mfma", timeit([&] { geo<1, 4, 32, 0, 1, false, 0, 1, 49152, 48><<<dim3(rows / 32, 1, nb), 256>>>(M, G, rows, cols, cols); }, reps));
    rep("H5  row 3x4 c32 Mline Gfrag-def 1blk(12w) kc2", timeit([&] { geo<3, 4, 32, 0, 1, false, 0, 1, 98304><<<dim3(rows / 96, 2, nb), 768>>>(M, G, rows, cols, cols / 2); }, reps));
    // rank_stream's strip walk (reference point)
    rep("S   strip 1x8 c32 Mline Gfrag-def PD2 2blk", timeit([&] { geo<1, 8, 32, 0, 1, false, 1, 2, 65536><<<dim3(cols / 256, rows / 1024, nb), 512>>>(M, G, rows, cols, 1024); }, reps));
    rep("S1  strip 1x8 c32 Mline Gfrag-def PD1 2blk", timeit([&] { geo<1, 8, 32, 0, 1, false, 1, 1, 65536><<<dim3(cols / 256, rows / 1024, nb), 512>>>(M, G, rows, cols, 1024); }, reps));
    rep("S2  strip 1x4 c32 Mline Gfrag-def PD1 3blk", timeit([&] { geo<1, 4, 32, 0, 1, false, 1, 1, 49152><<<dim3(cols / 128, rows / 1024, nb), 256>>>(M, G, rows, cols, 1024); }, reps));
  }
  (void)hipFree(M);
  (void)hipFree(G);
  return 0;
}
