// Dev microbenchmark (not product): P <- P R^-1 for a batch of tall m_P x 64 panels, the two
// triangular solves of the randomised Cholesky QR.  Variants:
//   A  trsm_right_kernel<64> of the codec (one row per lane, factor from LDS)
//   B  the same with the factor read by wave-uniform global (scalar) loads
//   C  factor from LDS, two columns per v_pk_fma_f32 (diagonal zeroed in the LDS copy)
//   E  explicit T = R^-1 and P T on v_mfma_f32_16x16x4f32 (a streaming GEMM; other rounding)
//   X  B with an XCD-contiguous block order
// and at r = 128: the codec's LDS-factor solve against scalar loads in three 64 x 64 factor blocks
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include -o scripts/ubench/trsm_ab scripts/ubench/trsm_ab.hip
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

constexpr int RT = 64;

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

__global__ void __launch_bounds__(256) trsm_pk_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                      const float* __restrict__ Rf, int mp) {
  __shared__ f32x2 Rs[RT * RT / 2];
  __shared__ float dg[RT];
  const int b = blockIdx.y;
  const float* Rg = Rf + static_cast<long>(b) * (RT * RT + RT);
  for (int i = threadIdx.x; i < RT * RT / 2; i += 256) {
    const int k = (2 * i) / RT, j = (2 * i) % RT;
    Rs[i] = f32x2{j == k ? 0.f : Rg[k * RT + j], j + 1 == k ? 0.f : Rg[k * RT + j + 1]};
  }
  for (int i = threadIdx.x; i < RT; i += 256) dg[i] = Rg[RT * RT + i];
  __syncthreads();
  const long row = static_cast<long>(blockIdx.x) * 256 + threadIdx.x;
  if (row >= mp) return;
  const float* p = src + (static_cast<long>(b) * mp + row) * RT;
  f32x2 x[RT / 2];
#pragma unroll
  for (int j = 0; j < RT; j += 4) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(p + j);
    x[j / 2] = f32x2{v[0], v[1]};
    x[j / 2 + 1] = f32x2{v[2], v[3]};
  }
#pragma unroll
  for (int k = 0; k < RT; ++k) {
    float xk = x[k / 2][k & 1] * dg[k];
    x[k / 2][k & 1] = xk;
    const f32x2 nx{-xk, -xk};
#pragma unroll
    for (int j2 = k / 2; j2 < RT / 2; ++j2) {
      if (j2 == k / 2 && (k & 1)) continue;  // pair (k-1, k): both already final
      x[j2] = __builtin_elementwise_fma(nx, Rs[k * (RT / 2) + j2], x[j2]);
    }
  }
  float* q = dst + (static_cast<long>(b) * mp + row) * RT;
#pragma unroll
  for (int j = 0; j < RT; j += 4)
    *reinterpret_cast<f32x4*>(q + j) = f32x4{x[j / 2][0], x[j / 2][1], x[j / 2 + 1][0], x[j / 2 + 1][1]};
}

// P T with T (64 x 64, row-major) on fp32 MFMA: a wave owns 16 rows, lane (t, g) loads A[row t][k 4s + g]
__global__ void __launch_bounds__(256) gemm_t_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                     const float* __restrict__ Tf, int mp) {
  __shared__ float Ts[RT * RT];
  const int b = blockIdx.y;
  for (int i = threadIdx.x; i < RT * RT; i += 256) Ts[i] = Tf[static_cast<long>(b) * RT * RT + i];
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, t = lane & 15, g = lane >> 4;
  const long row0 = (static_cast<long>(blockIdx.x) * 4 + wave) * 16;
  if (row0 >= mp) return;
  const float* p = src + (static_cast<long>(b) * mp + row0) * RT;
  f32x4 acc[RT / 16];
#pragma unroll
  for (int c = 0; c < RT / 16; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < RT / 4; ++s) {
    const float a = p[t * RT + 4 * s + g];
#pragma unroll
    for (int c = 0; c < RT / 16; ++c)
      acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, Ts[(4 * s + g) * RT + 16 * c + t], acc[c], 0, 0, 0);
  }
  float* q = dst + (static_cast<long>(b) * mp + row0) * RT;
#pragma unroll
  for (int c = 0; c < RT / 16; ++c)
#pragma unroll
    for (int e = 0; e < 4; ++e) q[(4 * g + e) * RT + 16 * c + t] = acc[c][e];
}

// B2: variant B with an XCD-contiguous block order (the blocks that share a factor run on one
// XCD, so fewer distinct factors compete for each CU's scalar cache)
__global__ void __launch_bounds__(256) trsm_scalar_xcd_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                              const float* __restrict__ Rf, int mp) {
  const BlockXYZ blk = xcd_block();
  const int b = blk.y;
  const float* R = Rf + static_cast<long>(b) * (RT * RT + RT);
  const long row = static_cast<long>(blk.x) * 256 + threadIdx.x;
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

// r = 128 by scalar factor loads in three 64 x 64 blocks (U11, U12, U22): the same fma order
// per x_j as the right-looking loop, but each phase reads one 16 KB block of the factor
template <bool XCD>
__global__ void __launch_bounds__(256) trsm128_blocked_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                              const float* __restrict__ Rf, int mp) {
  constexpr int T = 128, H = 64;
  const BlockXYZ blk = XCD ? xcd_block() : BlockXYZ{static_cast<int>(blockIdx.x), static_cast<int>(blockIdx.y), 0, 0};
  const int b = blk.y;
  const float* R = Rf + static_cast<long>(b) * (T * T + T);
  const long row = static_cast<long>(blk.x) * 256 + threadIdx.x;
  if (row >= mp) return;
  const float* p = src + (static_cast<long>(b) * mp + row) * T;
  float x[T];
#pragma unroll
  for (int j = 0; j < T; j += 4) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(p + j);
    x[j] = v[0], x[j + 1] = v[1], x[j + 2] = v[2], x[j + 3] = v[3];
  }
#pragma unroll
  for (int k = 0; k < H; ++k) {
    x[k] *= R[T * T + k];
#pragma unroll
    for (int j = k + 1; j < H; ++j) x[j] = fmaf(-x[k], R[k * T + j], x[j]);
  }
#pragma unroll
  for (int k = 0; k < H; ++k)
#pragma unroll
    for (int j = H; j < T; ++j) x[j] = fmaf(-x[k], R[k * T + j], x[j]);
#pragma unroll
  for (int k = H; k < T; ++k) {
    x[k] *= R[T * T + k];
#pragma unroll
    for (int j = k + 1; j < T; ++j) x[j] = fmaf(-x[k], R[k * T + j], x[j]);
  }
  float* q = dst + (static_cast<long>(b) * mp + row) * T;
#pragma unroll
  for (int j = 0; j < T; j += 4) *reinterpret_cast<f32x4*>(q + j) = f32x4{x[j], x[j + 1], x[j + 2], x[j + 3]};
}

// a test factor: unit-ish diagonal, small bounded off-diagonal
static void make_factor(float* R, int rt) {
  for (int i = 0; i < rt; ++i)
    for (int j = 0; j < rt; ++j)
      R[i * rt + j] = j < i ? 0.f : (j == i ? 1.f + 0.1f * (i % 7) : 0.05f * ((i * 31 + j * 17) % 11 - 5) / 5.f / (rt / 64));
  for (int i = 0; i < rt; ++i) R[rt * rt + i] = 1.f / R[i * rt + i];
}

static void run128() {
  constexpr int T = 128;
  const int B = 16;
  for (int mp : {14336, 28672}) {
    const long n = static_cast<long>(B) * mp * T;
    std::vector<float> hP(n), hR(static_cast<long>(B) * (T * T + T));
    srand(2);
    for (auto& v : hP) v = (rand() / (float)RAND_MAX - 0.5f);
    for (int b = 0; b < B; ++b) make_factor(&hR[static_cast<long>(b) * (T * T + T)], T);
    float *dP, *dO, *dR;
    CKU(hipMalloc(&dP, n * 4));
    CKU(hipMalloc(&dO, n * 4));
    CKU(hipMalloc(&dR, hR.size() * 4));
    CKU(hipMemcpy(dP, hP.data(), n * 4, hipMemcpyHostToDevice));
    CKU(hipMemcpy(dR, hR.data(), hR.size() * 4, hipMemcpyHostToDevice));
    std::vector<float> ref(n), out(n);
    hipEvent_t e0, e1;
    CKU(hipEventCreate(&e0));
    CKU(hipEventCreate(&e1));
    const dim3 grid(static_cast<unsigned>((mp + 255) / 256), B);
    for (int v = 0; v < 3; ++v) {
      auto go = [&]() {
        if (v == 0) hipLaunchKernelGGL((trsm_right_kernel<128>), grid, dim3(256), 0, 0, dP, dO, dR, mp, T, nullptr);
        if (v == 1) hipLaunchKernelGGL((trsm128_blocked_kernel<false>), grid, dim3(256), 0, 0, dP, dO, dR, mp);
        if (v == 2) hipLaunchKernelGGL((trsm128_blocked_kernel<true>), grid, dim3(256), 0, 0, dP, dO, dR, mp);
      };
      go();
      CKU(hipDeviceSynchronize());
      CKU(hipMemcpy(out.data(), dO, n * 4, hipMemcpyDeviceToHost));
      if (v == 0) ref = out;
      long ndiff = 0;
      for (long i = 0; i < n; ++i) ndiff += out[i] != ref[i];
      CKU(hipEventRecord(e0));
      const int it = 20;
      for (int i = 0; i < it; ++i) go();
      CKU(hipEventRecord(e1));
      CKU(hipEventSynchronize(e1));
      float ms;
      CKU(hipEventElapsedTime(&ms, e0, e1));
      printf("r128 mp %d variant %s: %.1f us per launch (%.2f TB/s of P in+out), entries differing from LDS %ld\n", mp,
             v == 0 ? "A128(lds)" : (v == 1 ? "F128(scalar 3-block)" : "G128(scalar 3-block, xcd)"), 1e3 * ms / it,
             2.0 * n * 4 / (1e-3 * ms / it) / 1e12, ndiff);
    }
    CKU(hipFree(dP));
    CKU(hipFree(dO));
    CKU(hipFree(dR));
  }
}

int main() {
  const int B = 16;
  for (int mp : {6144, 28672}) {
    const long n = static_cast<long>(B) * mp * RT;
    std::vector<float> hP(n), hR(static_cast<long>(B) * (RT * RT + RT)), hT(static_cast<long>(B) * RT * RT, 0.f);
    srand(1);
    for (auto& v : hP) v = (rand() / (float)RAND_MAX - 0.5f);
    for (int b = 0; b < B; ++b) {
      float* R = &hR[static_cast<long>(b) * (RT * RT + RT)];
      for (int i = 0; i < RT; ++i)
        for (int j = 0; j < RT; ++j) R[i * RT + j] = j < i ? 0.f : (j == i ? 1.f + 0.1f * (i % 7) : 0.05f * ((i * 31 + j * 17) % 11 - 5) / 5.f);
      for (int i = 0; i < RT; ++i) R[RT * RT + i] = 1.f / R[i * RT + i];
      // T = R^-1 (back substitution, double)
      std::vector<double> X(RT * RT, 0.0);
      for (int c = 0; c < RT; ++c)
        for (int i = c; i >= 0; --i) {
          double acc = (i == c) ? 1.0 : 0.0;
          for (int k = i + 1; k <= c; ++k) acc -= (double)R[i * RT + k] * X[k * RT + c];
          X[i * RT + c] = acc / R[i * RT + i];
        }
      for (int i = 0; i < RT * RT; ++i) hT[static_cast<long>(b) * RT * RT + i] = (float)X[i];
    }
    float *dP, *dO, *dR, *dT;
    CKU(hipMalloc(&dP, n * 4));
    CKU(hipMalloc(&dO, n * 4));
    CKU(hipMalloc(&dR, hR.size() * 4));
    CKU(hipMalloc(&dT, hT.size() * 4));
    CKU(hipMemcpy(dP, hP.data(), n * 4, hipMemcpyHostToDevice));
    CKU(hipMemcpy(dR, hR.data(), hR.size() * 4, hipMemcpyHostToDevice));
    CKU(hipMemcpy(dT, hT.data(), hT.size() * 4, hipMemcpyHostToDevice));
    std::vector<float> ref(n), out(n);
    hipEvent_t e0, e1;
    CKU(hipEventCreate(&e0));
    CKU(hipEventCreate(&e1));
    const dim3 grid(static_cast<unsigned>((mp + 255) / 256), B);
    const dim3 gridE(static_cast<unsigned>((mp + 63) / 64), B);
    for (int v = 0; v < 5; ++v) {
      auto go = [&]() {
        if (v == 0) hipLaunchKernelGGL((trsm_right_kernel<64>), grid, dim3(256), 0, 0, dP, dO, dR, mp, RT, nullptr);
        if (v == 1) hipLaunchKernelGGL(trsm_scalar_kernel, grid, dim3(256), 0, 0, dP, dO, dR, mp);
        if (v == 2) hipLaunchKernelGGL(trsm_pk_kernel, grid, dim3(256), 0, 0, dP, dO, dR, mp);
        if (v == 3) hipLaunchKernelGGL(gemm_t_kernel, gridE, dim3(256), 0, 0, dP, dO, dT, mp);
        if (v == 4) hipLaunchKernelGGL(trsm_scalar_xcd_kernel, grid, dim3(256), 0, 0, dP, dO, dR, mp);
      };
      go();
      CKU(hipDeviceSynchronize());
      CKU(hipMemcpy(out.data(), dO, n * 4, hipMemcpyDeviceToHost));
      if (v == 0) ref = out;
      double md = 0, mx = 0;
      for (long i = 0; i < n; ++i) {
        md = fmax(md, fabs((double)out[i] - ref[i]));
        mx = fmax(mx, fabs((double)ref[i]));
      }
      CKU(hipEventRecord(e0));
      const int it = 20;
      for (int i = 0; i < it; ++i) go();
      CKU(hipEventRecord(e1));
      CKU(hipEventSynchronize(e1));
      float ms;
      CKU(hipEventElapsedTime(&ms, e0, e1));
      printf("mp %d variant %c: %.1f us per launch (%.2f TB/s of P in+out), maxrel vs A %.2e\n", mp, "ABCEX"[v],
             1e3 * ms / it, 2.0 * n * 4 / (1e-3 * ms / it) / 1e12, md / mx);
    }
    CKU(hipFree(dP));
    CKU(hipFree(dO));
    CKU(hipFree(dR));
    CKU(hipFree(dT));
  }
  run128();
  return 0;
}
