// Micro-benchmark (dev tool, not product): what the HBM streams of one Dion step can reach on
// MI355X when nothing but the bytes is in the way.
//   read4  : x read once (pass B's M read, 4 B/elem)
//   copy   : y = x (guide reference: 6.29 TB/s)
//   rmw8   : x = x * a + b in place (the weight update, 8 B/elem)
//   rmw10  : M += G, fp32 M in place, bf16 G (pass A, 10 B/elem); lane = 8 elements
//            (two 16-B M loads + one 16-B G load + two 16-B M stores)
// Each: grid-stride, U independent lane-groups in flight per iteration, nt or default policy,
// grid = CUs x blocks-per-CU.
// The "mall" section asks whether M written by one pass and read right after by the next
// (pass A then pass B of one matrix) is served from the 256 MiB Infinity Cache: read time of
// a freshly written S-byte buffer vs the same read after 4 GB of unrelated traffic.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

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

template <int U, bool NT>
__global__ void __launch_bounds__(256) read4(const f32x4* __restrict__ x, long n4, float* out) {
  f32x4 acc = {0, 0, 0, 0};
  const long stride = (long)gridDim.x * 256;
  long i = blockIdx.x * 256L + threadIdx.x;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<f32x4, NT>(x + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  for (; i < n4; i += stride) acc += ld<f32x4, NT>(x + i);
  if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.f) out[0] = 1.f;
}

template <int U, bool NT>
__global__ void __launch_bounds__(256) copy(const f32x4* __restrict__ x, f32x4* __restrict__ y, long n4) {
  const long stride = (long)gridDim.x * 256;
  long i = blockIdx.x * 256L + threadIdx.x;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<f32x4, NT>(x + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) st<f32x4, NT>(y + i + u * stride, v[u]);
  }
  for (; i < n4; i += stride) st<f32x4, NT>(y + i, ld<f32x4, NT>(x + i));
}

template <int U, bool NT>
__global__ void __launch_bounds__(256) rmw8(f32x4* __restrict__ x, long n4, float a) {
  const long stride = (long)gridDim.x * 256;
  long i = blockIdx.x * 256L + threadIdx.x;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<f32x4, NT>(x + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) st<f32x4, NT>(x + i + u * stride, v[u] * a + 1.f);
  }
  for (; i < n4; i += stride) st<f32x4, NT>(x + i, ld<f32x4, NT>(x + i) * a + 1.f);
}

__device__ __forceinline__ void addg(f32x4& lo, f32x4& hi, u32x4 g) {
  lo[0] += __uint_as_float(g[0] << 16);
  lo[1] += __uint_as_float(g[0] & 0xFFFF0000u);
  lo[2] += __uint_as_float(g[1] << 16);
  lo[3] += __uint_as_float(g[1] & 0xFFFF0000u);
  hi[0] += __uint_as_float(g[2] << 16);
  hi[1] += __uint_as_float(g[2] & 0xFFFF0000u);
  hi[2] += __uint_as_float(g[3] << 16);
  hi[3] += __uint_as_float(g[3] & 0xFFFF0000u);
}

// n8 groups of 8 elements: M[2 i], M[2 i + 1] (f32x4), G[i] (8 bf16)
template <int U, bool NT>
__global__ void __launch_bounds__(256) rmw10(f32x4* __restrict__ M, const u32x4* __restrict__ G, long n8) {
  const long stride = (long)gridDim.x * 256;
  long i = blockIdx.x * 256L + threadIdx.x;
  for (; i + (U - 1) * stride < n8; i += U * stride) {
    f32x4 lo[U], hi[U];
    u32x4 g[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      lo[u] = ld<f32x4, NT>(M + 2 * (i + u * stride));
      hi[u] = ld<f32x4, NT>(M + 2 * (i + u * stride) + 1);
      g[u] = ld<u32x4, NT>(G + i + u * stride);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      addg(lo[u], hi[u], g[u]);
      st<f32x4, NT>(M + 2 * (i + u * stride), lo[u]);
      st<f32x4, NT>(M + 2 * (i + u * stride) + 1, hi[u]);
    }
  }
  for (; i < n8; i += stride) {
    f32x4 lo = ld<f32x4, NT>(M + 2 * i), hi = ld<f32x4, NT>(M + 2 * i + 1);
    addg(lo, hi, ld<u32x4, NT>(G + i));
    st<f32x4, NT>(M + 2 * i, lo);
    st<f32x4, NT>(M + 2 * i + 1, hi);
  }
}

// the same M += G but coalesced per wave-instruction: lane l of a wave-instruction takes
// M 16 B at 16 l (1 KB contiguous per instruction) and G 16 B at 16 l for the 8 elements of
// the wave's two M instructions (lane pairing differs; the bytes are the same)
template <int U, bool NT>
__global__ void __launch_bounds__(256) rmw10c(float* __restrict__ M, const unsigned short* __restrict__ G, long n) {
  // unit = 512 elements per wave (2 KB M, 1 KB G)
  const int lane = threadIdx.x & 63;
  const long wave = (blockIdx.x * 256L + threadIdx.x) >> 6;
  const long nw = (long)gridDim.x * 4;
  const long units = n / 512;
  long w = wave;
  for (; w + (U - 1) * nw < units; w += U * nw) {
    f32x4 a[U], b[U];
    u32x4 g[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long e = (w + u * nw) * 512;
      a[u] = ld<f32x4, NT>(reinterpret_cast<const f32x4*>(M + e) + lane);
      b[u] = ld<f32x4, NT>(reinterpret_cast<const f32x4*>(M + e + 256) + lane);
      g[u] = ld<u32x4, NT>(reinterpret_cast<const u32x4*>(G + e) + lane);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long e = (w + u * nw) * 512;
      addg(a[u], b[u], g[u]);
      st<f32x4, NT>(reinterpret_cast<f32x4*>(M + e) + lane, a[u]);
      st<f32x4, NT>(reinterpret_cast<f32x4*>(M + e + 256) + lane, b[u]);
    }
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
  hipEventDestroy(a);
  hipEventDestroy(b);
  return ms / reps;
}

static void rep(const char* name, int grid, double bytes, float ms) {
  printf("%-22s grid %5d  %8.3f ms  %6.3f TB/s\n", name, grid, ms, bytes / ms / 1e9);
  fflush(stdout);
}

int main(int argc, char** argv) {
  // 1.5 G elements: M 6 GB, G 3 GB, copy target 6 GB
  const long n = 1536L << 20;
  float *M, *Y, *out;
  unsigned short* G;
  hipMalloc(&M, n * 4);
  hipMalloc(&Y, n * 4);
  hipMalloc(&G, n * 2);
  hipMalloc(&out, 64);
  // non-zero data (DVFS: zeros run a different clock)
  hipMemset(M, 0x3c, n * 4);
  hipMemset(Y, 0x3c, n * 4);
  hipMemset(G, 0x3b, n * 2);
  const int reps = 5;
  const int grids[] = {512, 1024, 2048, 4096};
  for (int round = 0; round < 2; ++round) {
    printf("=== round %d (n = %ld elements)\n", round, n);
    for (int gr : grids) {
      rep("read4 U2 nt", gr, 4.0 * n, timeit([&] { read4<2, true><<<gr, 256>>>((const f32x4*)M, n / 4, out); }, reps));
      rep("read4 U4 nt", gr, 4.0 * n, timeit([&] { read4<4, true><<<gr, 256>>>((const f32x4*)M, n / 4, out); }, reps));
      rep("read4 U4 def", gr, 4.0 * n, timeit([&] { read4<4, false><<<gr, 256>>>((const f32x4*)M, n / 4, out); }, reps));
      rep("copy U2 nt", gr, 8.0 * n, timeit([&] { copy<2, true><<<gr, 256>>>((const f32x4*)M, (f32x4*)Y, n / 4); }, reps));
      rep("copy U4 nt", gr, 8.0 * n, timeit([&] { copy<4, true><<<gr, 256>>>((const f32x4*)M, (f32x4*)Y, n / 4); }, reps));
      rep("copy U4 def", gr, 8.0 * n, timeit([&] { copy<4, false><<<gr, 256>>>((const f32x4*)M, (f32x4*)Y, n / 4); }, reps));
      rep("rmw8 U2 nt", gr, 8.0 * n, timeit([&] { rmw8<2, true><<<gr, 256>>>((f32x4*)Y, n / 4, 0.999f); }, reps));
      rep("rmw8 U4 nt", gr, 8.0 * n, timeit([&] { rmw8<4, true><<<gr, 256>>>((f32x4*)Y, n / 4, 0.999f); }, reps));
      rep("rmw8 U4 def", gr, 8.0 * n, timeit([&] { rmw8<4, false><<<gr, 256>>>((f32x4*)Y, n / 4, 0.999f); }, reps));
      rep("rmw10 U1 nt", gr, 10.0 * n, timeit([&] { rmw10<1, true><<<gr, 256>>>((f32x4*)M, (const u32x4*)G, n / 8); }, reps));
      rep("rmw10 U2 nt", gr, 10.0 * n, timeit([&] { rmw10<2, true><<<gr, 256>>>((f32x4*)M, (const u32x4*)G, n / 8); }, reps));
      rep("rmw10 U4 nt", gr, 10.0 * n, timeit([&] { rmw10<4, true><<<gr, 256>>>((f32x4*)M, (const u32x4*)G, n / 8); }, reps));
      rep("rmw10 U2 def", gr, 10.0 * n, timeit([&] { rmw10<2, false><<<gr, 256>>>((f32x4*)M, (const u32x4*)G, n / 8); }, reps));
      rep("rmw10c U2 nt", gr, 10.0 * n, timeit([&] { rmw10c<2, true><<<gr, 256>>>(M, G, n); }, reps));
      rep("rmw10c U4 nt", gr, 10.0 * n, timeit([&] { rmw10c<4, true><<<gr, 256>>>(M, G, n); }, reps));
    }
  }

  // ---- Infinity Cache: read right after write
  printf("=== mall: read of a buffer just written vs after 4 GB of other traffic\n");
  const long sizes_mb[] = {32, 64, 128, 192, 256, 384, 768};
  for (long smb : sizes_mb) {
    const long s4 = (smb << 20) / 16;  // f32x4 units
    const int gr = 2048;
    for (int pol = 0; pol < 2; ++pol) {
      float hot = 0.f, cold = 0.f;
      const int R = 5;
      for (int r = 0; r < R; ++r) {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        // evict: 4 GB read of Y elsewhere
        read4<4, true><<<gr, 256>>>((const f32x4*)Y, (1024L << 20) / 4, out);
        // write the buffer (pass A's store policy), then read it
        if (pol == 0) rmw8<2, true><<<gr, 256>>>((f32x4*)M, s4, 0.999f);
        else rmw8<2, false><<<gr, 256>>>((f32x4*)M, s4, 0.999f);
        hipEventRecord(e0);
        read4<4, true><<<gr, 256>>>((const f32x4*)M, s4, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        hot += ms;
        read4<4, true><<<gr, 256>>>((const f32x4*)Y, (1024L << 20) / 4, out);
        hipEventRecord(e0);
        read4<4, true><<<gr, 256>>>((const f32x4*)M, s4, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        cold += ms;
        hipEventDestroy(e0);
        hipEventDestroy(e1);
      }
      hot /= R;
      cold /= R;
      printf("mall %4ld MB writer %-3s  hot read %7.3f ms %6.3f TB/s   cold read %7.3f ms %6.3f TB/s\n", smb,
             pol == 0 ? "nt" : "def", hot, (smb << 20) / hot / 1e9, cold, (smb << 20) / cold / 1e9);
      fflush(stdout);
    }
  }
  hipFree(M);
  hipFree(Y);
  hipFree(G);
  hipFree(out);
  return 0;
}
