// dion_elementwise.hpp -- the elementwise (non-Dion) branch of MegatronDion.step on
// device: AdamW and Lion for the parameters the adapter routes as
// ElementwiseStepParam (embeddings, norms, biases, the output layer).
//
// Replaces /root/reference/megatron/core/optimizer/dion/elementwise_opts.py:45-107
// (_adamw_update_foreach_chunk, _lion_update_foreach_chunk), which the reference
// runs as a chain of torch._foreach_* calls -- one HBM pass per call.  Here one
// multi-tensor launch reads W, G and the moments once and writes W and the moments
// once (AdamW fp32: 16 B read + 12 B written per element with an fp32 gradient).
// The per-element arithmetic follows the foreach chain operation by operation, each
// result rounded to fp32 (no contraction into FMAs except where torch's own lerp
// uses one: start + w (end - start) for |w| < 0.5, else end + (w - 1)(end - start)).
#pragma clang fp contract(off)

struct EwArgs {
  float* w[MAXB];
  const void* g[MAXB];
  void* m1[MAXB];    // first moment (fp32, or bf16 in the mixed-precision mode)
  void* m2[MAXB];    // second moment (AdamW) or null
  long numel[MAXB];
  float lerp1, lerp2;    // 1 - beta1, 1 - beta2
  float bc2_sqrt;        // sqrt(1 - beta2^step)
  float eps;
  float step_size;       // lr / (1 - beta1^step)  (AdamW) or lr (Lion)
  float decay;           // 1 - lr wd
  int has_decay;
};

__device__ __forceinline__ float torch_lerp(float start, float end, float w) {
  // ATen lerp: small weights from the start, large weights from the end
  return (fabsf(w) < 0.5f) ? fmaf(w, end - start, start) : fmaf(w - 1.0f, end - start, end);
}

__device__ __forceinline__ float torch_sign(float x) {
  if (x != x) return x;
  return (x > 0.f) ? 1.f : ((x < 0.f) ? -1.f : 0.f);
}

// every foreach result lands in the moment dtype: rounded to bf16 in the
// mixed-precision mode (torch computes bf16 elementwise ops in fp32 and rounds once)
template <int MDT>
__device__ __forceinline__ float rnd(float x) {
  if constexpr (MDT == DION_DTYPE_BF16) return bf16_round(x);
  else return x;
}

template <int MDT>
__device__ __forceinline__ float ld_moment(const void* p, long i) {
  if constexpr (MDT == DION_DTYPE_BF16) return bf16_to_f32(static_cast<const uint16_t*>(p)[i]);
  else return static_cast<const float*>(p)[i];
}

template <int MDT>
__device__ __forceinline__ void st_moment(void* p, long i, float v) {
  if constexpr (MDT == DION_DTYPE_BF16) static_cast<uint16_t*>(p)[i] = f32_to_bf16_rne(v);
  else static_cast<float*>(p)[i] = v;
}

template <int GDT, int M1, int M2, bool LION>
__global__ void __launch_bounds__(256) elementwise_kernel(const EwArgs a) {
  // torch's type promotion of first_moments / denom: bf16 only when both moments are bf16
  constexpr int UDT = (M1 == DION_DTYPE_BF16 && M2 == DION_DTYPE_BF16) ? DION_DTYPE_BF16 : DION_DTYPE_F32;
  const int b = blockIdx.y;
  const long n = a.numel[b];
  float* __restrict__ W = a.w[b];
  for (long i = static_cast<long>(blockIdx.x) * 256 + threadIdx.x; i < n; i += static_cast<long>(gridDim.x) * 256) {
    float g;
    if constexpr (GDT == DION_DTYPE_BF16) g = bf16_to_f32(static_cast<const uint16_t*>(a.g[b])[i]);
    else g = static_cast<const float*>(a.g[b])[i];
    g = rnd<M1>(g);  // grad.to(first_moment.dtype)
    float w = W[i];
    const float m = ld_moment<M1>(a.m1[b], i);
    if constexpr (LION) {
      // elementwise_opts.py:88-105
      float u = torch_sign(rnd<M1>(torch_lerp(m, g, a.lerp1)));
      st_moment<M1>(a.m1[b], i, torch_lerp(m, g, a.lerp2));
      u = rnd<M1>(u * a.step_size);
      if (a.has_decay) w = w * a.decay;
      W[i] = w - u;
    } else {
      // elementwise_opts.py:45-80: the first moment's ops in its dtype, the squared
      // gradient cast to the second moment's dtype, the denominator in that dtype
      const float m_new = rnd<M1>(torch_lerp(m, g, a.lerp1));
      const float gsq = rnd<M2>(rnd<M1>(g * g));
      const float v_new = rnd<M2>(torch_lerp(ld_moment<M2>(a.m2[b], i), gsq, a.lerp2));
      st_moment<M1>(a.m1[b], i, m_new);
      st_moment<M2>(a.m2[b], i, v_new);
      float denom = rnd<M2>(sqrtf(v_new));
      denom = rnd<M2>(denom / a.bc2_sqrt);
      denom = rnd<M2>(denom + a.eps);
      float u = rnd<UDT>(m_new / denom);
      u = rnd<UDT>(u * a.step_size);
      if (a.has_decay) w = w * a.decay;
      W[i] = w - u;
    }
  }
}

#pragma clang fp contract(on)

namespace ew {

int run(int n_tensors, const int64_t* numels, float* const* W, const void* const* G, int g_dtype, int m1_dtype,
        int m2_dtype, void* const* m1, void* const* m2, bool lion, float lerp1, float lerp2, float bc2_sqrt, float eps, float step_size,
        float decay, int has_decay, hipStream_t st) {
  if (n_tensors < 0) return fail(DION_E_INVALID, "n_tensors=%d", n_tensors);
  if (n_tensors > 0 && (numels == nullptr || W == nullptr || G == nullptr || m1 == nullptr || (!lion && m2 == nullptr)))
    return fail(DION_E_INVALID, "null argument");
  if (g_dtype != DION_DTYPE_F32 && g_dtype != DION_DTYPE_BF16) return fail(DION_E_UNSUPPORTED, "grad dtype %d", g_dtype);
  if (m1_dtype != DION_DTYPE_F32 && m1_dtype != DION_DTYPE_BF16) return fail(DION_E_UNSUPPORTED, "moment dtype %d", m1_dtype);
  if (!lion && m2_dtype != DION_DTYPE_F32 && m2_dtype != DION_DTYPE_BF16)
    return fail(DION_E_UNSUPPORTED, "second moment dtype %d", m2_dtype);
  for (int t0 = 0; t0 < n_tensors; t0 += MAXB) {
    const int nt = n_tensors - t0 < MAXB ? n_tensors - t0 : MAXB;
    EwArgs a;
    memset(&a, 0, sizeof(a));
    long maxn = 0;
    for (int t = 0; t < nt; ++t) {
      a.w[t] = W[t0 + t];
      a.g[t] = G[t0 + t];
      a.m1[t] = m1[t0 + t];
      a.m2[t] = lion ? nullptr : m2[t0 + t];
      a.numel[t] = numels[t0 + t];
      if (a.numel[t] < 0 || (a.numel[t] > 0 && (!a.w[t] || !a.g[t] || !a.m1[t] || (!lion && !a.m2[t]))))
        return fail(DION_E_INVALID, "bad tensor %d", t0 + t);
      if (a.numel[t] > maxn) maxn = a.numel[t];
    }
    if (maxn == 0) continue;
    a.lerp1 = lerp1;
    a.lerp2 = lerp2;
    a.bc2_sqrt = bc2_sqrt;
    a.eps = eps;
    a.step_size = step_size;
    a.decay = decay;
    a.has_decay = has_decay;
    long gx = ceil_div(maxn, 256 * 4);
    if (gx > 2048) gx = 2048;
    const dim3 grid(static_cast<unsigned>(gx), nt);
    auto launch = [&](auto Gc, auto M1c, auto M2c) {
      constexpr int GD = decltype(Gc)::value, MD1 = decltype(M1c)::value, MD2 = decltype(M2c)::value;
      if (lion) hipLaunchKernelGGL((elementwise_kernel<GD, MD1, MD1, true>), grid, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((elementwise_kernel<GD, MD1, MD2, false>), grid, dim3(256), 0, st, a);
    };
    using F32 = std::integral_constant<int, DION_DTYPE_F32>;
    using B16 = std::integral_constant<int, DION_DTYPE_BF16>;
    auto with_m2 = [&](auto Gc, auto M1c) {
      if (!lion && m2_dtype != m1_dtype) {
        if (m2_dtype == DION_DTYPE_BF16) launch(Gc, M1c, B16{}); else launch(Gc, M1c, F32{});
      } else {
        launch(Gc, M1c, M1c);
      }
    };
    auto with_m1 = [&](auto Gc) {
      if (m1_dtype == DION_DTYPE_BF16) with_m2(Gc, B16{}); else with_m2(Gc, F32{});
    };
    if (g_dtype == DION_DTYPE_BF16) with_m1(B16{}); else with_m1(F32{});
    const int rc = check_launch(lion ? "elementwise(lion)" : "elementwise(adamw)");
    if (rc != DION_OK) return rc;
  }
  return DION_OK;
}

}  // namespace ew
