// Dev microbenchmark (not product): sketch_qr_inv_kernel<RPL, CPW, XT, false, NWQ> (the Householder
// QR of the K x r sketch product, one block per matrix, 16 matrices per launch) over its wave
// count NWQ.  Every column runs the same arithmetic whichever wave owns it, so the factors must
// agree bitwise.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include -o scripts/ubench/qr_ab scripts/ubench/qr_ab.hip
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

template <int RPL, int CPW, typename XT, int NWQ>
float run(const float* dSP, float* dF, int K, int r, int B, std::vector<float>& out) {
  const int rt = trsm_rt(r);
  const size_t lds = ((sizeof(float) * (520 + static_cast<size_t>(r) * (r + 1)) + 15) / 16) * 16 +
                     sizeof(XT) * static_cast<size_t>(r) * r;
  if (allow_lds(sketch_qr_inv_kernel<RPL, CPW, XT, false, NWQ>, lds) != DION_OK) exit(1);
  auto go = [&] {
    hipLaunchKernelGGL((sketch_qr_inv_kernel<RPL, CPW, XT, false, NWQ>), dim3(B), dim3(64 * NWQ), lds, 0, dSP, dF, K,
                       r, rt);
  };
  go();
  CKU(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CKU(hipEventCreate(&e0));
  CKU(hipEventCreate(&e1));
  CKU(hipEventRecord(e0));
  for (int i = 0; i < 20; ++i) go();
  CKU(hipEventRecord(e1));
  CKU(hipEventSynchronize(e1));
  float ms;
  CKU(hipEventElapsedTime(&ms, e0, e1));
  out.resize(static_cast<size_t>(B) * (rt * rt + rt));
  CKU(hipMemcpy(out.data(), dF, out.size() * 4, hipMemcpyDeviceToHost));
  return ms * 1e3f / 20.f;
}

template <int K, int R, int RPL, typename XT>
void sweep() {
  const int B = 16;
  std::vector<float> h(static_cast<size_t>(B) * K * R);
  srand(5);
  for (auto& v : h) v = rand() / (float)RAND_MAX - 0.5f;
  float *dSP, *dF;
  CKU(hipMalloc(&dSP, h.size() * 4));
  CKU(hipMalloc(&dF, static_cast<size_t>(B) * (trsm_rt(R) * trsm_rt(R) + trsm_rt(R)) * 4));
  CKU(hipMemcpy(dSP, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  std::vector<float> ref, out;
  auto report = [&](int nwq, float us) {
    long nd = 0;
    for (size_t i = 0; i < ref.size(); ++i) nd += out[i] != ref[i];
    printf("sketch QR K=%d r=%d NWQ=%2d: %.1f us per 16-matrix launch, entries differing from NWQ=4: %ld\n", K, R, nwq,
           us, nd);
  };
  float t = run<RPL, R / 4, XT, 4>(dSP, dF, K, R, B, ref);
  out = ref;
  report(4, t);
  t = run<RPL, R / 8, XT, 8>(dSP, dF, K, R, B, out);
  report(8, t);
  t = run<RPL, R / 16, XT, 16>(dSP, dF, K, R, B, out);
  report(16, t);
  // tri_inv_kernel on the factor: time, and max |T F - I| on the host
  {
    constexpr int RT = R;
    float* dT;
    CKU(hipMalloc(&dT, static_cast<size_t>(B) * RT * RT * 4));
    hipLaunchKernelGGL((tri_inv_kernel<RT>), dim3(B), dim3(RT * tri_inv_tip<RT>()), 0, 0, dF, dT);
    CKU(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CKU(hipEventCreate(&e0));
    CKU(hipEventCreate(&e1));
    CKU(hipEventRecord(e0));
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL((tri_inv_kernel<RT>), dim3(B), dim3(RT * tri_inv_tip<RT>()), 0, 0, dF, dT);
    CKU(hipEventRecord(e1));
    CKU(hipEventSynchronize(e1));
    float ms;
    CKU(hipEventElapsedTime(&ms, e0, e1));
    std::vector<float> hT(static_cast<size_t>(B) * RT * RT);
    CKU(hipMemcpy(hT.data(), dT, hT.size() * 4, hipMemcpyDeviceToHost));
    double worst = 0;
    for (int b = 0; b < B; ++b) {
      const float* F = &ref[static_cast<size_t>(b) * (RT * RT + RT)];
      const float* T = &hT[static_cast<size_t>(b) * RT * RT];
      for (int i = 0; i < RT; ++i)
        for (int j = 0; j < RT; ++j) {
          double acc = 0;
          for (int k = 0; k < RT; ++k) acc += (double)T[i * RT + k] * F[k * RT + j];
          worst = fmax(worst, fabs(acc - (i == j ? 1.0 : 0.0)));
        }
    }
    printf("tri_inv r=%d: %.1f us per 16-matrix launch, max |T F - I| %.2e\n", R, ms * 1e3f / 20.f, worst);
    CKU(hipFree(dT));
  }
  CKU(hipFree(dSP));
  CKU(hipFree(dF));
}

int main() {
  sweep<128, 64, 2, double>();
  sweep<256, 128, 4, float>();
  return 0;
}
