// roundlab.hip — which kernel carries the round's back-to-back penalty?
// (r04)  The cfg2 round's broadcast runs ~20 us slower
// right after the reduce than back to back with itself, while the write lab's
// plain kernels (tools/writelab.hip) lose only ~3 us the same way.  This lab
// crosses the product's two launches (libfedagg.so: fa_reduce, then
// fa_reduce(FA_F_BCAST_ONLY)) with the lab's plain read and broadcast kernels
// over the SAME 20 + 1 buckets (one slab, hashed data, one fp32 tensor of the
// wrn16_8 size), and times every kernel of an alternating sequence with
// events between the kernels.
//   hipcc --offload-arch=gfx950 -O3 -I include -o tools/roundlab tools/roundlab.hip \
//         -L feddct_amd -lfedagg -Wl,-rpath,'$ORIGIN/../feddct_amd'
// One JSON line per (pair, pass).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "fedagg.h"

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)
#define FA(x)                                                                  \
  do {                                                                         \
    if ((x) != FA_OK) {                                                        \
      fprintf(stderr, "%s: %s\n", #x, fa_last_error());                        \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const f4 gcf4;
typedef __attribute__((address_space(1))) f4 gf4;

constexpr int kN = 20;
struct Dst {
  float* d[kN];
};

// SP: the result's store policy — 0 nt, 1 sc1 (write-through, drops the
// line from L2), 2 plain, 3 sc0 sc1
template <int SP>
__device__ __forceinline__ void st(float* base, int64_t v, f4 x) {
  if constexpr (SP == 0) {
    __builtin_nontemporal_store(x, (gf4*)base + v);
  } else if constexpr (SP == 2) {
    ((gf4*)base)[v] = x;
  } else {
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(x, r, (int)(16 * v), 0, SP == 1 ? 16 : 17);
  }
}
// LP: the source loads' policy — 0 plain, 1 nt, 2 sc1, 3 sc0 sc1
template <int LP>
__device__ __forceinline__ f4 ld(const float* base, int64_t v) {
  if constexpr (LP == 0) return ((gcf4*)base)[v];
  else if constexpr (LP == 1) return __builtin_nontemporal_load((gcf4*)base + v);
  else {
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7fffffff, 0x00020000);
    return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(16 * v), 0,
                                                                      LP == 2 ? 16 : 17));
  }
}

template <int SP = 0>
__global__ __launch_bounds__(256) void read20(Dst d, float* out, int64_t nv) {
  const int64_t b = (int64_t)blockIdx.x * 512;
  const int t = threadIdx.x;
  f4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
#pragma unroll 4
  for (int c = 0; c < kN; ++c) {
    if (b + t < nv) a0 += __builtin_nontemporal_load((gcf4*)d.d[c] + b + t);
    if (b + t + 256 < nv) a1 += __builtin_nontemporal_load((gcf4*)d.d[c] + b + t + 256);
  }
  if (b + t < nv) st<SP>(out + 4 * b, t, a0 * 0.05f);
  if (b + t + 256 < nv) st<SP>(out + 4 * b, t + 256, a1 * 0.05f);
}

template <int U, int G, int LP = 0>
__global__ __launch_bounds__(256) void bcast(const float* s, Dst d, int64_t nv) {
  constexpr int NG = (kN + G - 1) / G;
  const int g = (int)(blockIdx.x % NG);
  const int64_t b = (int64_t)(blockIdx.x / NG) * U * 256 + threadIdx.x;
  const int64_t b0 = (int64_t)(blockIdx.x / NG) * U * 256;
  f4 x[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (b + u * 256 < nv) x[u] = ld<LP>(s + 4 * b0, threadIdx.x + u * 256);
#pragma unroll
  for (int i = 0; i < G; ++i) {
    const int c = g * G + i;
    if (c >= kN) break;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (b + u * 256 < nv) __builtin_nontemporal_store(x[u], (gf4*)d.d[c] + b + u * 256);
  }
}

// persistent: a grid of resident workgroups striding over (part, group), the
// NEXT item's source loads issued before the current item's stores, so the
// source's read latency hides behind the stores
template <int U, int G>
__global__ __launch_bounds__(256) void bcast_persist(const float* s, Dst d, int64_t nv) {
  constexpr int NG = (kN + G - 1) / G;
  const uint32_t parts = (uint32_t)((nv + U * 256 - 1) / (U * 256));
  const uint32_t total = parts * NG;
  uint32_t v = blockIdx.x;
  if (v >= total) return;
  f4 x[U];
  {
    const int64_t b = (int64_t)(v / NG) * U * 256 + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (b + u * 256 < nv) x[u] = ((gcf4*)s)[b + u * 256];
  }
  for (; v < total; v += gridDim.x) {
    const int g = (int)(v % NG);
    const int64_t b = (int64_t)(v / NG) * U * 256 + threadIdx.x;
    const uint32_t vn = v + gridDim.x;
    f4 y[U];
    if (vn < total) {
      const int64_t bn = (int64_t)(vn / NG) * U * 256 + threadIdx.x;
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (bn + u * 256 < nv) y[u] = ((gcf4*)s)[bn + u * 256];
    }
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int c = g * G + i;
      if (c >= kN) break;
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (b + u * 256 < nv) __builtin_nontemporal_store(x[u], (gf4*)d.d[c] + b + u * 256);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = y[u];
  }
}

// one wave that idles `us` microseconds (s_memrealtime: 100 MHz)
__global__ void spin(int us) {
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < (uint64_t)us * 100) __builtin_amdgcn_s_sleep(8);
}

__device__ __forceinline__ uint32_t mix(uint32_t x);
// write-only: fresh hashed values (seed) in the U1 / groups-of-10 shape
__global__ __launch_bounds__(256) void fill(Dst d, int64_t nv, uint32_t seed) {
  const int g = (int)(blockIdx.x % 2);
  const int64_t b = (int64_t)(blockIdx.x / 2) * 256 + threadIdx.x;
  if (b >= nv) return;
  const uint32_t h = (uint32_t)(4 * b) ^ seed;
  f4 x;
  x.x = (float)(int32_t)(mix(h) >> 8) * (1.0f / 8388608.0f) - 1.0f;
  x.y = (float)(int32_t)(mix(h + 1) >> 8) * (1.0f / 8388608.0f) - 1.0f;
  x.z = (float)(int32_t)(mix(h + 2) >> 8) * (1.0f / 8388608.0f) - 1.0f;
  x.w = (float)(int32_t)(mix(h + 3) >> 8) * (1.0f / 8388608.0f) - 1.0f;
#pragma unroll
  for (int i = 0; i < 10; ++i) __builtin_nontemporal_store(x, (gf4*)d.d[g * 10 + i] + b);
}

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
__global__ void hash_fill(float* p, int64_t n, uint32_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = (float)(int32_t)(mix((uint32_t)i * 2654435761u ^ seed) >> 8) * (1.0f / 8388608.0f) - 1.0f;
}

int main(int argc, char** argv) {
  const int passes = argc > 1 ? atoi(argv[1]) : 3;
  const int64_t n = 10972184;
  const int64_t nv = n / 4;
  const int64_t stride = (n * 4 + 65535) / 65536 * 65536;
  char* slab;
  CK(hipMalloc(&slab, stride * (kN + 2)));
  float* src2 = (float*)(slab + stride * (kN + 1));  // a source no kernel writes
  Dst d;
  const float* c32[kN];
  for (int c = 0; c < kN; ++c) {
    d.d[c] = (float*)(slab + stride * c);
    c32[c] = d.d[c];
  }
  float* out = (float*)(slab + stride * kN);
  for (int c = 0; c <= kN + 1; ++c) hash_fill<<<4096, 256>>>((float*)(slab + stride * c), n, 17u + c);
  CK(hipDeviceSynchronize());
  fa_seg seg{0, n};
  fa_plan* plan = nullptr;
  FA(fa_plan_create(&seg, 1, n, nullptr, 0, 0, 0, FA_PLAN_GAPS_ARE_PADDING, &plan));
  hipStream_t st = nullptr;
  uint32_t seed = 1;
  const uint32_t p1 = (uint32_t)((nv + 255) / 256), p2 = (uint32_t)((nv + 511) / 512);
  std::vector<std::pair<std::string, std::function<void()>>> R = {
      {"prod_reduce", [&] { FA(fa_reduce(plan, c32, nullptr, kN, nullptr, out, nullptr, 0, st)); }},
      {"lab_read20", [&] { read20<0><<<p2, 256>>>(d, out, nv); }},
      {"lab_read20_st_sc1", [&] { read20<1><<<p2, 256>>>(d, out, nv); }},
      {"lab_read20_st_plain", [&] { read20<2><<<p2, 256>>>(d, out, nv); }},
      {"lab_read20_st_sc0sc1", [&] { read20<3><<<p2, 256>>>(d, out, nv); }},
  };
  std::vector<std::pair<std::string, std::function<void()>>> B = {
      {"prod_bcast", [&] {
         FA(fa_reduce(plan, c32, nullptr, kN, nullptr, out, nullptr, FA_F_BCAST_ONLY, st));
       }},
      {"lab_bcast_U1_G10", [&] { bcast<1, 10><<<p1 * 2, 256>>>(out, d, nv); }},
      {"lab_bcast_U2_G10", [&] { bcast<2, 10><<<p2 * 2, 256>>>(out, d, nv); }},
      {"lab_bcast_U1_G10_oldsrc", [&] { bcast<1, 10><<<p1 * 2, 256>>>(src2, d, nv); }},
      {"lab_bcast_U1_G10_ldnt", [&] { bcast<1, 10, 1><<<p1 * 2, 256>>>(out, d, nv); }},
      {"lab_bcast_U1_G10_ldsc1", [&] { bcast<1, 10, 2><<<p1 * 2, 256>>>(out, d, nv); }},
      {"lab_bcast_U1_G10_ldsc0sc1", [&] { bcast<1, 10, 3><<<p1 * 2, 256>>>(out, d, nv); }},
      {"lab_bcast_U2_G10_ldsc1", [&] { bcast<2, 10, 2><<<p2 * 2, 256>>>(out, d, nv); }},
  };
  const int K = 20;
  std::vector<hipEvent_t> ev(2 * K + 1);
  for (auto& e : ev) CK(hipEventCreate(&e));
  auto pair = [&](const std::string& rn, std::function<void()>& r, const std::string& bn,
                  std::function<void()>& b, int pass) {
    for (int i = 0; i < 3; ++i) {
      r();
      b();
    }
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(ev[0], st));
    for (int i = 0; i < K; ++i) {
      r();
      CK(hipEventRecord(ev[2 * i + 1], st));
      b();
      CK(hipEventRecord(ev[2 * i + 2], st));
    }
    CK(hipEventSynchronize(ev[2 * K]));
    double tr = 0, tb = 0;
    for (int i = 0; i < K; ++i) {
      float a, c;
      CK(hipEventElapsedTime(&a, ev[2 * i], ev[2 * i + 1]));
      CK(hipEventElapsedTime(&c, ev[2 * i + 1], ev[2 * i + 2]));
      tr += a;
      tb += c;
    }
    printf("{\"lab\": \"round\", \"reduce\": \"%s\", \"bcast\": \"%s\", \"pass\": %d, "
           "\"reduce_us\": %.2f, \"bcast_us\": %.2f}\n",
           rn.c_str(), bn.c_str(), pass, tr / K * 1e3, tb / K * 1e3);
    fflush(stdout);
  };
  auto alone = [&](const std::string& nm, std::function<void()>& f, int pass) {
    for (int i = 0; i < 3; ++i) f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(ev[0], st));
    for (int i = 0; i < K; ++i) f();
    CK(hipEventRecord(ev[1], st));
    CK(hipEventSynchronize(ev[1]));
    float ms;
    CK(hipEventElapsedTime(&ms, ev[0], ev[1]));
    printf("{\"lab\": \"round\", \"alone\": \"%s\", \"pass\": %d, \"us\": %.2f}\n", nm.c_str(), pass,
           ms / K * 1e3);
    fflush(stdout);
  };
  for (int pass = 0; pass < passes; ++pass) {
    for (auto& r : R) alone(r.first, r.second, pass);
    for (auto& b : B) alone(b.first, b.second, pass);
    for (auto& r : R)
      for (auto& b : B) pair(r.first, r.second, b.first, b.second, pass);
  }
  FA(fa_plan_destroy(plan));
  CK(hipFree(slab));
  return 0;
}
