// copylab.hip — streaming-copy variants on one 1 GiB buffer pair (the
// roofline's copy ceiling).  Standalone lab binary:
//   hipcc --offload-arch=gfx950 -O3 -o tools/copylab tools/copylab.hip
// Prints one JSON line per variant and round (GB/s = read + written bytes).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                   \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const f4 gcf4;
typedef __attribute__((address_space(1))) f4 gf4;

template <bool NT>
__device__ __forceinline__ f4 ld(const float* p, int64_t v) {
  if constexpr (NT) return __builtin_nontemporal_load((gcf4*)p + v);
  else return ((gcf4*)p)[v];
}
template <bool NT>
__device__ __forceinline__ void st(float* p, int64_t v, f4 x) {
  if constexpr (NT) __builtin_nontemporal_store(x, (gf4*)p + v);
  else ((gf4*)p)[v] = x;
}

// grid-stride, one float4 per lane per trip
template <bool NT>
__global__ __launch_bounds__(256) void gs1(const float* s, float* d, int64_t nv) {
  for (int64_t v = blockIdx.x * 256ll + threadIdx.x; v < nv; v += (int64_t)gridDim.x * 256)
    st<NT>(d, v, ld<NT>(s, v));
}
// grid-stride, U float4 per lane in flight before the stores
template <bool NT, int U>
__global__ __launch_bounds__(256) void gsu(const float* s, float* d, int64_t nv) {
  const int64_t str = (int64_t)gridDim.x * 256;
  int64_t v = blockIdx.x * 256ll + threadIdx.x;
  for (; v + (U - 1) * str < nv; v += U * str) {
    f4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = ld<NT>(s, v + u * str);
#pragma unroll
    for (int u = 0; u < U; ++u) st<NT>(d, v + u * str, x[u]);
  }
  for (; v < nv; v += str) st<NT>(d, v, ld<NT>(s, v));
}
// one tile of U*256 float4 per workgroup (the reduce kernel's shape)
template <bool NT, int U>
__global__ __launch_bounds__(256) void tile(const float* s, float* d, int64_t nv) {
  const int64_t b = (int64_t)blockIdx.x * U * 256 + threadIdx.x;
  f4 x[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (b + u * 256 < nv) x[u] = ld<NT>(s, b + u * 256);
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (b + u * 256 < nv) st<NT>(d, b + u * 256, x[u]);
}

template <class F>
float time_ms(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  const int64_t n = 256ll * 1024 * 1024;  // floats: 1 GiB
  const int64_t nv = n / 4;
  float *s, *d;
  CK(hipMalloc(&s, n * 4));
  CK(hipMalloc(&d, n * 4));
  CK(hipMemset(s, 0, n * 4));
  CK(hipMemset(d, 0, n * 4));
  auto rep = [&](const char* name, float ms) {
    printf("{\"variant\": \"%s\", \"us\": %.1f, \"GBps\": %.1f}\n", name, ms * 1e3,
           2.0 * n * 4 / (ms * 1e-3) / 1e9);
    fflush(stdout);
  };
  for (int r = 0; r < 3; ++r) {
    rep("gs1_nt_4096", time_ms([&] { gs1<true><<<4096, 256>>>(s, d, nv); }, 10));
    rep("gs1_plain_4096", time_ms([&] { gs1<false><<<4096, 256>>>(s, d, nv); }, 10));
    rep("gsu4_nt_2048", time_ms([&] { gsu<true, 4><<<2048, 256>>>(s, d, nv); }, 10));
    rep("gsu4_plain_2048", time_ms([&] { gsu<false, 4><<<2048, 256>>>(s, d, nv); }, 10));
    rep("gsu4_nt_8192", time_ms([&] { gsu<true, 4><<<8192, 256>>>(s, d, nv); }, 10));
    rep("gsu2_nt_4096", time_ms([&] { gsu<true, 2><<<4096, 256>>>(s, d, nv); }, 10));
    rep("tile1_nt", time_ms([&] { tile<true, 1><<<nv / 256, 256>>>(s, d, nv); }, 10));
    rep("tile1_plain", time_ms([&] { tile<false, 1><<<nv / 256, 256>>>(s, d, nv); }, 10));
    rep("tile2_nt", time_ms([&] { tile<true, 2><<<nv / 512, 256>>>(s, d, nv); }, 10));
    rep("tile2_plain", time_ms([&] { tile<false, 2><<<nv / 512, 256>>>(s, d, nv); }, 10));
    rep("tile4_nt", time_ms([&] { tile<true, 4><<<nv / 1024, 256>>>(s, d, nv); }, 10));
    rep("tile4_plain", time_ms([&] { tile<false, 4><<<nv / 1024, 256>>>(s, d, nv); }, 10));
  }
  CK(hipFree(s));
  CK(hipFree(d));
  return 0;
}
