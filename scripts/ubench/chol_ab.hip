// Dev microbenchmark (not product): chol_reg_kernel<RP, NT> (the Cholesky of the RCQR's Gram, one
// block per matrix, 16 matrices per launch) over block sizes NT.  Every NT runs the same per-element
// arithmetic in the same order, so the factors must agree bitwise.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include -o scripts/ubench/chol_ab scripts/ubench/chol_ab.hip
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

template <int RP, int NT>
float run(const float* dG, float* dF, int B, std::vector<float>& out) {
  hipEvent_t e0, e1;
  CKU(hipEventCreate(&e0));
  CKU(hipEventCreate(&e1));
  hipLaunchKernelGGL((chol_reg_kernel<RP, NT>), dim3(B), dim3(NT), 0, 0, dG, dF, RP);
  CKU(hipDeviceSynchronize());
  CKU(hipEventRecord(e0));
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL((chol_reg_kernel<RP, NT>), dim3(B), dim3(NT), 0, 0, dG, dF, RP);
  CKU(hipEventRecord(e1));
  CKU(hipEventSynchronize(e1));
  float ms;
  CKU(hipEventElapsedTime(&ms, e0, e1));
  out.resize(static_cast<size_t>(B) * (RP * RP + RP));
  CKU(hipMemcpy(out.data(), dF, out.size() * 4, hipMemcpyDeviceToHost));
  return ms * 1e3f / 20.f;
}

template <int RP>
void sweep() {
  const int B = 16;
  // G = X^T X / rows + I/8 for a random X: symmetric positive definite, unit-ish diagonal
  std::vector<float> hG(static_cast<size_t>(B) * RP * RP);
  srand(3);
  const int rows = 4 * RP;
  std::vector<double> X(static_cast<size_t>(rows) * RP);
  for (int b = 0; b < B; ++b) {
    for (auto& v : X) v = rand() / (double)RAND_MAX - 0.5;
    for (int i = 0; i < RP; ++i)
      for (int j = 0; j < RP; ++j) {
        double s = 0;
        for (int k = 0; k < rows; ++k) s += X[k * RP + i] * X[k * RP + j];
        hG[(static_cast<size_t>(b) * RP + i) * RP + j] = static_cast<float>(s / rows + (i == j ? 0.125 : 0.0));
      }
  }
  float *dG, *dF;
  CKU(hipMalloc(&dG, hG.size() * 4));
  CKU(hipMalloc(&dF, static_cast<size_t>(B) * (RP * RP + RP) * 4));
  CKU(hipMemcpy(dG, hG.data(), hG.size() * 4, hipMemcpyHostToDevice));
  std::vector<float> ref, out;
  auto report = [&](int nt, float us) {
    long nd = 0;
    for (size_t i = 0; i < ref.size(); ++i) nd += (out[i] != ref[i]) && !(out[i] != out[i] && ref[i] != ref[i]);
    printf("chol RP=%d NT=%4d: %.1f us per 16-matrix launch, entries differing from the first %ld\n", RP, nt, us, nd);
  };
  if constexpr (RP == 64) {
    float t = run<64, 256>(dG, dF, B, ref);
    out = ref;
    report(256, t);
    t = run<64, 64>(dG, dF, B, out);
    report(64, t);
    t = run<64, 128>(dG, dF, B, out);
    report(128, t);
    t = run<64, 512>(dG, dF, B, out);
    report(512, t);
  } else {
    float t = run<128, 1024>(dG, dF, B, ref);
    out = ref;
    report(1024, t);
    t = run<128, 128>(dG, dF, B, out);
    report(128, t);
    t = run<128, 256>(dG, dF, B, out);
    report(256, t);
    t = run<128, 512>(dG, dF, B, out);
    report(512, t);
  }
  CKU(hipFree(dG));
  CKU(hipFree(dF));
}

int main() {
  sweep<64>();
  sweep<128>();
  return 0;
}
