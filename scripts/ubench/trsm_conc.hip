// Dev microbenchmark (not product): the triangular solve P <- P R^-1 (m_P x 64 panels, 16 per
// launch group) alone and beside a streaming kernel on another stream, which is how the two-stream
// step runs it.  Marginal cost of a solve variant = t(copy + 10 solves, concurrent) - t(copy alone).
//   A   trsm_right_kernel<64>: one row per lane, factor from LDS
//   A2  two rows per lane (rows i, i + 256 of a 512-row block), factor from LDS
//   L   trsm_lds_kernel<64, false>: rows staged by LDS-DMA, factor from LDS
//   B   one row per lane, factor by scalar loads
//   M   tsolve_mfma_kernel: X = P T with T = R^-1 (fp64 on the host), fp16x3 MFMA
// and at r = 128: A against M.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include -o scripts/ubench/trsm_conc scripts/ubench/trsm_conc.hip
#include "../../megatron-dion_amd/csrc/dion_codec.hip"

#include <vector>

#define CKU(x)                                                                        \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

constexpr int RT = 64;  // the hand-written variants below

__global__ void __launch_bounds__(256) trsm_two_rows_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                            const float* __restrict__ Rf, int mp) {
  __shared__ f32x4 Rs4[(RT * RT + RT) / 4];
  const int b = blockIdx.y;
  {
    const f32x4* Rg = reinterpret_cast<const f32x4*>(Rf + static_cast<long>(b) * (RT * RT + RT));
    for (int i = threadIdx.x; i < (RT * RT + RT) / 4; i += 256) Rs4[i] = Rg[i];
    __syncthreads();
  }
  const float* R = reinterpret_cast<const float*>(Rs4);
  const long row0 = static_cast<long>(blockIdx.x) * 512 + threadIdx.x;
  const long row1 = row0 + 256;
  if (row0 >= mp) return;
  const bool two = row1 < mp;
  const float* p0 = src + (static_cast<long>(b) * mp + row0) * RT;
  const float* p1 = src + (static_cast<long>(b) * mp + (two ? row1 : row0)) * RT;
  float x[RT], y[RT];
#pragma unroll
  for (int j = 0; j < RT; j += 4) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(p0 + j);
    const f32x4 w = *reinterpret_cast<const f32x4*>(p1 + j);
    x[j] = v[0], x[j + 1] = v[1], x[j + 2] = v[2], x[j + 3] = v[3];
    y[j] = w[0], y[j + 1] = w[1], y[j + 2] = w[2], y[j + 3] = w[3];
  }
#pragma unroll
  for (int k = 0; k < RT; ++k) {
    const float d = R[RT * RT + k];
    x[k] *= d;
    y[k] *= d;
#pragma unroll
    for (int j = k + 1; j < RT; ++j) {
      const float u = R[k * RT + j];
      x[j] = fmaf(-x[k], u, x[j]);
      y[j] = fmaf(-y[k], u, y[j]);
    }
  }
  float* q0 = dst + (static_cast<long>(b) * mp + row0) * RT;
  float* q1 = dst + (static_cast<long>(b) * mp + row1) * RT;
#pragma unroll
  for (int j = 0; j < RT; j += 4) {
    *reinterpret_cast<f32x4*>(q0 + j) = f32x4{x[j], x[j + 1], x[j + 2], x[j + 3]};
    if (two) *reinterpret_cast<f32x4*>(q1 + j) = f32x4{y[j], y[j + 1], y[j + 2], y[j + 3]};
  }
}

__global__ void __launch_bounds__(256) trsm_scalar_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                          const float* __restrict__ Rf, int mp) {
  const int b = blockIdx.y;
  const float* R = Rf + static_cast<long>(b) * (RT * RT + RT);
  const long row = static_cast<long>(blockIdx.x) * 256 + threadIdx.x;
  if (row >= mp) return;
  const float* p = src + (static_cast<long>(b) * mp + row) * RT;
  float x[RT];
#pragma unroll
  for (int j = 0; j < RT; j += 4) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(p + j);
    x[j] = v[0], x[j + 1] = v[1], x[j + 2] = v[2], x[j + 3] = v[3];
  }
#pragma unroll
  for (int k = 0; k < RT; ++k) {
    x[k] *= R[RT * RT + k];
#pragma unroll
    for (int j = k + 1; j < RT; ++j) x[j] = fmaf(-x[k], R[k * RT + j], x[j]);
  }
  float* q = dst + (static_cast<long>(b) * mp + row) * RT;
#pragma unroll
  for (int j = 0; j < RT; j += 4) *reinterpret_cast<f32x4*>(q + j) = f32x4{x[j], x[j + 1], x[j + 2], x[j + 3]};
}

// the streaming neighbour: y = x (16-byte loads / stores, grid-stride, ~2 blocks per CU)
__global__ void __launch_bounds__(256) copy_kernel(const f32x4* __restrict__ x, f32x4* __restrict__ y, long n) {
  for (long i = static_cast<long>(blockIdx.x) * 256 + threadIdx.x; i < n; i += static_cast<long>(gridDim.x) * 256)
    y[i] = x[i];
}

template <int T_RT>
void run_rt(int mp, const f32x4* cx, f32x4* cy, long cn, float tcopy, hipStream_t s0, hipStream_t s1) {
  constexpr int R = T_RT;
  const int B = 16;
  const long n = static_cast<long>(B) * mp * R;
  std::vector<float> hP(n), hR(static_cast<long>(B) * (R * R + R)), hT(static_cast<long>(B) * R * R);
  srand(1);
  for (auto& v : hP) v = (rand() / (float)RAND_MAX - 0.5f);
  for (int b = 0; b < B; ++b) {
    float* Rm = &hR[static_cast<long>(b) * (R * R + R)];
    for (int i = 0; i < R; ++i)
      for (int j = 0; j < R; ++j)
        Rm[i * R + j] = j < i ? 0.f : (j == i ? 1.f + 0.1f * (i % 7) : 0.05f * ((i * 31 + j * 17) % 11 - 5) / 5.f / (R / 64));
    for (int i = 0; i < R; ++i) Rm[R * R + i] = 1.f / Rm[i * R + i];
    std::vector<double> X(R * R, 0.0);
    for (int c = 0; c < R; ++c)
      for (int i = c; i >= 0; --i) {
        double acc = (i == c) ? 1.0 : 0.0;
        for (int k = i + 1; k <= c; ++k) acc -= (double)Rm[i * R + k] * X[k * R + c];
        X[i * R + c] = acc / Rm[i * R + i];
      }
    for (int i = 0; i < R * R; ++i) hT[static_cast<long>(b) * R * R + i] = (float)X[i];
  }
  float *dP, *dO, *dR, *dT;
  CKU(hipMalloc(&dP, n * 4));
  CKU(hipMalloc(&dO, n * 4));
  CKU(hipMalloc(&dR, hR.size() * 4));
  CKU(hipMalloc(&dT, hT.size() * 4));
  CKU(hipMemcpy(dP, hP.data(), n * 4, hipMemcpyHostToDevice));
  CKU(hipMemcpy(dR, hR.data(), hR.size() * 4, hipMemcpyHostToDevice));
  CKU(hipMemcpy(dT, hT.data(), hT.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CKU(hipEventCreate(&e0));
  CKU(hipEventCreate(&e1));
  auto copy = [&](hipStream_t s) { hipLaunchKernelGGL(copy_kernel, dim3(512), dim3(256), 0, s, cx, cy, cn); };
  const int nv = R == 64 ? 5 : 2;
  auto solve = [&](int v, hipStream_t s) {
    const dim3 grid(static_cast<unsigned>((mp + 255) / 256), B);
    if (v == 0) hipLaunchKernelGGL((trsm_right_kernel<R>), grid, dim3(256), 0, s, dP, dO, dR, mp, R, nullptr);
    if (R == 64 && v == 1)
      hipLaunchKernelGGL(trsm_two_rows_kernel, dim3(static_cast<unsigned>((mp + 511) / 512), B), dim3(256), 0, s, dP, dO,
                         dR, mp);
    if (R == 64 && v == 2) {
      TrsmArgs ta{dP, dO, dR, nullptr, nullptr, 0, mp, 0};
      hipLaunchKernelGGL((trsm_lds_kernel<R == 64 ? 64 : 32, false>),
                         dim3(static_cast<unsigned>((mp + 64 * kTrsmWaves - 1) / (64 * kTrsmWaves)), B),
                         dim3(64 * kTrsmWaves), 0, s, ta);
    }
    if (R == 64 && v == 3) hipLaunchKernelGGL(trsm_scalar_kernel, grid, dim3(256), 0, s, dP, dO, dR, mp);
    if ((R == 64 && v == 4) || (R == 128 && v == 1)) {
      TrsmArgs ta{dP, dO, dT, nullptr, nullptr, 0, mp, 0};
      constexpr int NW = tsolve_img<R, false, false>() ? kTgWavesImg : kTgWavesDirect;
      hipLaunchKernelGGL((tsolve_mfma_kernel<R, false>), dim3(static_cast<unsigned>((mp + 64 * NW - 1) / (64 * NW)), B),
                         dim3(64 * NW), 0, s, ta);
    }
  };
  auto timed = [&](auto&& body) {
    CKU(hipDeviceSynchronize());
    CKU(hipEventRecord(e0, s0));
    body();
    CKU(hipEventRecord(e1, s0));
    CKU(hipEventSynchronize(e1));
    float ms;
    CKU(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3f;
  };
  const char* names64[5] = {"A  (lds factor, 1 row)", "A2 (lds factor, 2 rows)", "L  (lds rows + lds factor)",
                            "B  (scalar factor)", "M  (T = R^-1, h3 MFMA)"};
  const char* names128[2] = {"A  (lds factor, 1 row)", "M  (T = R^-1, h3 MFMA)"};
  std::vector<float> ref(n), out(n);
  for (int v = 0; v < nv; ++v) {
    solve(v, s0);
    CKU(hipDeviceSynchronize());
    CKU(hipMemcpy(out.data(), dO, n * 4, hipMemcpyDeviceToHost));
    if (v == 0) ref = out;
    long nd = 0;
    double md = 0, mx = 0;
    for (long i = 0; i < n; ++i) {
      nd += out[i] != ref[i];
      md = fmax(md, fabs((double)out[i] - ref[i]));
      mx = fmax(mx, fabs((double)ref[i]));
    }
    const float talone = timed([&] {
      for (int i = 0; i < 10; ++i) solve(v, s0);
    }) / 10.f;
    const float tconc = timed([&] {
      CKU(hipStreamWaitEvent(s1, e0, 0));
      copy(s0);
      for (int i = 0; i < 10; ++i) solve(v, s1);
      hipEvent_t d;
      CKU(hipEventCreateWithFlags(&d, hipEventDisableTiming));
      CKU(hipEventRecord(d, s1));
      CKU(hipStreamWaitEvent(s0, d, 0));
      CKU(hipEventDestroy(d));
    });
    printf("r=%d mp=%d %-28s alone %.1f us/launch (%.2f TB/s); copy + 10 concurrent %.1f us -> marginal %.1f us/launch; "
           "vs A: %ld entries differ, maxrel %.2e\n",
           R, mp, R == 64 ? names64[v] : names128[v], talone, 2.0 * n * 4 / (talone * 1e-6) / 1e12, tconc,
           (tconc - tcopy) / 10.f, nd, md / mx);
  }
  CKU(hipFree(dP));
  CKU(hipFree(dO));
  CKU(hipFree(dR));
  CKU(hipFree(dT));
}

int main() {
  const long cn = 1L << 28;  // 4 GiB each way
  f32x4 *cx, *cy;
  CKU(hipMalloc(&cx, cn * 16));
  CKU(hipMalloc(&cy, cn * 16));
  CKU(hipMemset(cx, 0, cn * 16));
  hipStream_t s0, s1;
  CKU(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CKU(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CKU(hipEventCreate(&e0));
  CKU(hipEventCreate(&e1));
  hipLaunchKernelGGL(copy_kernel, dim3(512), dim3(256), 0, s0, cx, cy, cn);
  CKU(hipDeviceSynchronize());
  CKU(hipEventRecord(e0, s0));
  hipLaunchKernelGGL(copy_kernel, dim3(512), dim3(256), 0, s0, cx, cy, cn);
  CKU(hipEventRecord(e1, s0));
  CKU(hipEventSynchronize(e1));
  float ms;
  CKU(hipEventElapsedTime(&ms, e0, e1));
  const float tcopy = ms * 1e3f;
  printf("copy alone: %.1f us (%.2f TB/s)\n", tcopy, 2.0 * cn * 16 / (tcopy * 1e-6) / 1e12);
  run_rt<64>(14336, cx, cy, cn, tcopy, s0, s1);
  run_rt<64>(4096, cx, cy, cn, tcopy, s0, s1);
  run_rt<128>(14336, cx, cy, cn, tcopy, s0, s1);
  return 0;
}
