// Precision of fp16 hi/lo ("h3") products on the two gfx950 fp16 MFMA shapes.
// One wave computes D = A B (32x32x16 and 16x16x32) from two-limb splits of random fp32
// A, B with the three products lo*hi + hi*lo + hi*hi, and each product alone; the host
// compares with the fp64 product.  Build: hipcc --offload-arch=gfx950 -O3 -o mfma_f16_limbs mfma_f16_limbs.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ void split(const float* x, float s, f16x8& hi, f16x8& lo) {
#pragma clang fp contract(off)
  for (int j = 0; j < 8; ++j) {
    const float v = x[j] * s;
    const _Float16 h = static_cast<_Float16>(v);
    hi[j] = h;
    lo[j] = static_cast<_Float16>(v - static_cast<float>(h));
  }
}

// mode: 0 = all three, 1 = hi*hi, 2 = lo*hi, 3 = hi*lo
__global__ void k32(const float* A, const float* B, float* D, float sa, float sb, int mode) {
  const int l = threadIdx.x, t = l & 31, h = l >> 5;
  float a[8], b[8];
  for (int j = 0; j < 8; ++j) {
    a[j] = A[t * 16 + 8 * h + j];  // A row-major 32 x 16
    b[j] = B[t * 16 + 8 * h + j];  // B stored as col-major: B^T row-major 32 x 16
  }
  f16x8 ah, al, bh, bl;
  split(a, sa, ah, al);
  split(b, sb, bh, bl);
  f32x16 acc;
  for (int q = 0; q < 16; ++q) acc[q] = 0.f;
  if (mode == 0 || mode == 2) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc, 0, 0, 0);
  if (mode == 0 || mode == 3) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc, 0, 0, 0);
  if (mode == 0 || mode == 1) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc, 0, 0, 0);
  for (int q = 0; q < 16; ++q) D[((q & 3) + 8 * (q >> 2) + 4 * h) * 32 + t] = acc[q] / (sa * sb);
}

__global__ void k16(const float* A, const float* B, float* D, float sa, float sb, int mode) {
  const int l = threadIdx.x, t = l & 15, g = l >> 4;
  float a[8], b[8];
  for (int j = 0; j < 8; ++j) {
    a[j] = A[t * 32 + 8 * g + j];  // A row-major 16 x 32
    b[j] = B[t * 32 + 8 * g + j];  // B^T row-major 16 x 32
  }
  f16x8 ah, al, bh, bl;
  split(a, sa, ah, al);
  split(b, sb, bh, bl);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (mode == 0 || mode == 2) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc, 0, 0, 0);
  if (mode == 0 || mode == 3) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc, 0, 0, 0);
  if (mode == 0 || mode == 1) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc, 0, 0, 0);
  for (int q = 0; q < 4; ++q) D[(4 * g + q) * 16 + t] = acc[q] / (sa * sb);
}

int main() {
  srand(1);
  const char* names[4] = {"lo*hi+hi*lo+hi*hi", "hi*hi", "lo*hi", "hi*lo"};
  for (int shape = 0; shape < 2; ++shape) {
    const int M = shape == 0 ? 32 : 16, K = shape == 0 ? 16 : 32;
    std::vector<float> A(M * K), B(M * K), D(M * M);
    for (auto& v : A) v = (rand() / (float)RAND_MAX - 0.5f) * 0.1f;
    for (auto& v : B) v = (rand() / (float)RAND_MAX - 0.5f) * 0.1f;
    float *dA, *dB, *dD;
    hipMalloc(&dA, A.size() * 4);
    hipMalloc(&dB, B.size() * 4);
    hipMalloc(&dD, D.size() * 4);
    hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
    double mx = 0;
    std::vector<double> E(M * M);
    for (int i = 0; i < M; ++i)
      for (int j = 0; j < M; ++j) {
        double s = 0;
        for (int k = 0; k < K; ++k) s += (double)A[i * K + k] * B[j * K + k];
        E[i * M + j] = s;
        mx = fmax(mx, fabs(s));
      }
    for (int mode = 0; mode < 4; ++mode) {
      const float sa = 8192.f, sb = 8192.f;
      if (shape == 0)
        hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, dA, dB, dD, sa, sb, mode);
      else
        hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, dA, dB, dD, sa, sb, mode);
      hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
      double err = 0, mag = 0;
      for (int i = 0; i < M * M; ++i) {
        err = fmax(err, fabs(D[i] - E[i]));
        mag = fmax(mag, fabs(D[i]));
      }
      printf("%s %-20s max|D| %.3e  max|D - exact| / max|exact| %.3e\n", shape == 0 ? "32x32x16" : "16x16x32",
             names[mode], mag, err / mx);
    }
    hipFree(dA);
    hipFree(dB);
    hipFree(dD);
  }
  return 0;
}
