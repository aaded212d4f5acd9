// writelab.hip — the write side of the round (train_fedavg.py:148-149: every
// client slot <- the global) as a standalone lab, r04:
// what does this chip write per second when the values are real data, and how
// close is the broadcast to that?  N = 20 destination buckets of the wrn16_8
// size (10,972,184 floats, 43.9 MB) carved from ONE allocation (the product's
// slab placement), every buffer pre-filled with hashed non-zero values.
//   hipcc --offload-arch=gfx950 -O3 -o tools/writelab tools/writelab.hip
// One JSON line per variant and pass.  "GBps" = algorithmic bytes / time:
// fills count N*B written, broadcasts B read + N*B written, read20 N*B read +
// B written.  "in_round" lines time each kernel of an alternating
// read20 -> broadcast sequence with events between the kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

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

constexpr int kN = 20;
struct Dst {
  float* d[kN];
};

__device__ __forceinline__ f4 ldnt(const float* p, int64_t v) {
  return __builtin_nontemporal_load((gcf4*)p + v);
}
__device__ __forceinline__ f4 ldp(const float* p, int64_t v) { return ((gcf4*)p)[v]; }
__device__ __forceinline__ void stnt(float* p, int64_t v, f4 x) {
  __builtin_nontemporal_store(x, (gf4*)p + v);
}
__device__ __forceinline__ void stp(float* p, int64_t v, f4 x) { ((gf4*)p)[v] = x; }

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// a float in (-1, 1) with a full random mantissa: real-data-like bits
__device__ __forceinline__ float hval(uint32_t i) {
  return (float)(int32_t)(mix(i) >> 8 | 0u) * (1.0f / 8388608.0f) - 1.0f;
}
__device__ __forceinline__ f4 hvec(int64_t v, uint32_t salt) {
  const uint32_t b = (uint32_t)(4 * v) ^ salt;
  return f4{hval(b), hval(b + 1), hval(b + 2), hval(b + 3)};
}

// (part, group) of block v: groups fastest (the product's consecutive form),
// or a part's groups on blocks b, b+8, ... (one XCD under round-robin dispatch)
template <bool XCD>
__device__ __forceinline__ bool part_of(uint32_t v, uint32_t nparts, uint32_t groups,
                                        uint32_t* p, uint32_t* g) {
  if (XCD) {
    const uint32_t q = v / 8;
    *g = q % groups;
    *p = (q / groups) * 8 + v % 8;
    return *p < nparts;
  }
  *p = v / groups;
  *g = v % groups;
  return true;
}

// MODE 0: constant {1,2,3,4}; 1: hashed by position (every client the same
// values, as a broadcast writes); 2: hashed by position and client
template <int U, int G, int MODE, bool XCD>
__global__ __launch_bounds__(256) void fill(Dst d, int64_t nv, uint32_t nparts) {
  constexpr uint32_t NG = (kN + G - 1) / G;
  uint32_t p, g;
  if (!part_of<XCD>(blockIdx.x, nparts, NG, &p, &g)) return;
  const int64_t b = (int64_t)p * U * 256 + threadIdx.x;
  f4 x[U];
#pragma unroll
  for (int u = 0; u < U; ++u) x[u] = MODE == 0 ? f4{1.f, 2.f, 3.f, 4.f} : hvec(b + u * 256, 0);
#pragma unroll
  for (int i = 0; i < G; ++i) {
    const int c = (int)g * G + i;
    if (c >= kN) break;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (MODE == 2) x[u] = hvec(b + u * 256, 0x9e3779b9u * (c + 1));
      if (b + u * 256 < nv) stnt(d.d[c], b + u * 256, x[u]);
    }
  }
}

// the product's broadcast shape: one workgroup per (part of U*1024 floats,
// group of G clients); the part's loads before the G*U stores
template <int U, int G, bool XCD, bool NT>
__global__ __launch_bounds__(256) void bcast(const float* s, Dst d, int64_t nv, uint32_t nparts) {
  constexpr uint32_t NG = (kN + G - 1) / G;
  uint32_t p, g;
  if (!part_of<XCD>(blockIdx.x, nparts, NG, &p, &g)) return;
  const int64_t b = (int64_t)p * U * 256 + threadIdx.x;
  f4 x[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (b + u * 256 < nv) x[u] = ldp(s, b + u * 256);
#pragma unroll
  for (int i = 0; i < G; ++i) {
    const int c = (int)g * G + i;
    if (c >= kN) break;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (b + u * 256 < nv) {
        if (NT) stnt(d.d[c], b + u * 256, x[u]);
        else stp(d.d[c], b + u * 256, x[u]);
      }
  }
}

// persistent: grid of resident workgroups striding over (part, group), the
// next item's source loads issued before the current item's stores
template <int U, int G>
__global__ __launch_bounds__(256) void bcast_persist(const float* s, Dst d, int64_t nv,
                                                     uint32_t nparts) {
  constexpr uint32_t NG = (kN + G - 1) / G;
  const uint32_t total = nparts * NG;
  uint32_t v = blockIdx.x;
  if (v >= total) return;
  f4 x[U];
  {
    const int64_t b = (int64_t)(v / NG) * U * 256 + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (b + u * 256 < nv) x[u] = ldp(s, b + u * 256);
  }
  for (; v < total; v += gridDim.x) {
    const uint32_t p = v / NG, g = v % NG;
    const int64_t b = (int64_t)p * U * 256 + threadIdx.x;
    const uint32_t vn = v + gridDim.x;
    f4 y[U];
    if (vn < total) {
      const int64_t bn = (int64_t)(vn / NG) * U * 256 + threadIdx.x;
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (bn + u * 256 < nv) y[u] = ldp(s, bn + u * 256);
    }
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int c = (int)g * G + i;
      if (c >= kN) break;
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (b + u * 256 < nv) stnt(d.d[c], b + u * 256, x[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = y[u];
  }
}

// the reduce's stream shape (order irrelevant here): one workgroup per
// 2048-float tile, 16-client batches of 2 nt loads per lane each, result nt
template <bool NTLD>
__global__ __launch_bounds__(256) void read20(Dst d, float* out, int64_t nv) {
  const int64_t b = (int64_t)blockIdx.x * 512 + threadIdx.x;
  f4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
#pragma unroll 4
  for (int c = 0; c < kN; ++c) {
    if (b < nv) a0 += NTLD ? ldnt(d.d[c], b) : ldp(d.d[c], b);
    if (b + 256 < nv) a1 += NTLD ? ldnt(d.d[c], b + 256) : ldp(d.d[c], b + 256);
  }
  if (b < nv) stnt(out, b, a0);
  if (b + 256 < nv) stnt(out, b + 256, a1);
}

__global__ void hash_fill(float* p, int64_t n, uint32_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = hval((uint32_t)i * 2654435761u ^ seed);
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
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / reps;
}

// argv: PASSES [PLACEMENTS] [full]: one slab per placement letter, in order
// (m: hipMalloc; c: hipExtMallocWithFlags(hipDeviceMallocContiguous);
// f: hipMalloc after allocation churn that leaves the free memory
// fragmented), each measured then freed; "full" runs every variant, else
// the short set.
int main(int argc, char** argv) {
  const int passes = argc > 1 ? atoi(argv[1]) : 3;
  const char* placements = argc > 2 ? argv[2] : "m";
  const bool full = argc > 3;
  const int64_t n = 10972184;  // wrn16_8 C10 fp32 bucket, whole float4s
  const int64_t nv = n / 4;
  const int64_t stride = (n * 4 + 65535) / 65536 * 65536;  // 64 KiB-aligned slots
  for (const char* pl = placements; *pl; ++pl) {
  std::vector<void*> churn;
  if (*pl == 'f') {
    // 400 x 6 MiB, free every other one: the slab's pages come from the holes
    for (int i = 0; i < 400; ++i) {
      void* q;
      CK(hipMalloc(&q, 6 << 20));
      churn.push_back(q);
    }
    for (size_t i = 0; i < churn.size(); i += 2) CK(hipFree(churn[i]));
  }
  char* slab;
  if (*pl == 'c')
    CK(hipExtMallocWithFlags((void**)&slab, stride * (kN + 2), hipDeviceMallocContiguous));
  else
    CK(hipMalloc(&slab, stride * (kN + 2)));
  const char ptag[2] = {*pl, 0};
  float* s = (float*)(slab + stride * kN);
  float* out = (float*)(slab + stride * (kN + 1));
  Dst d;
  for (int c = 0; c < kN; ++c) d.d[c] = (float*)(slab + stride * c);
  for (int c = 0; c < kN + 2; ++c) hash_fill<<<4096, 256>>>((float*)(slab + stride * c), n, 17u + c);
  CK(hipDeviceSynchronize());
  const double B = n * 4.0;
  const double wbytes = kN * B, bbytes = (kN + 1) * B, rbytes = (kN + 1) * B;
  auto rep = [&](const char* name, float ms, double bytes, int pass) {
    printf("{\"lab\": \"write\", \"alloc\": \"%s\", \"variant\": \"%s\", \"pass\": %d, \"us\": %.2f, \"GBps\": %.1f}\n",
           ptag, name, pass, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
  };
  auto parts = [&](int U) { return (uint32_t)((nv + U * 256 - 1) / (U * 256)); };
  auto blocks = [&](int U, int G, bool xcd) {
    const uint32_t ng = (kN + G - 1) / G, np = parts(U);
    return (xcd ? (np + 7) / 8 * 8 : np) * ng;
  };
  const int R = 20;
  // the round emulation: read20 then a broadcast form, each timed with
  // events between the kernels
  auto in_round = [&](const char* name, auto bc, int pass) {
    std::vector<hipEvent_t> ev(2 * R + 1);
    for (auto& ev1 : ev) CK(hipEventCreate(&ev1));
    for (int i = 0; i < 3; ++i) {
      read20<true><<<parts(2), 256>>>(d, out, nv);
      bc();
    }
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(ev[0]));
    for (int i = 0; i < R; ++i) {
      read20<true><<<parts(2), 256>>>(d, out, nv);
      CK(hipEventRecord(ev[2 * i + 1]));
      bc();
      CK(hipEventRecord(ev[2 * i + 2]));
    }
    CK(hipEventSynchronize(ev[2 * R]));
    double tr = 0, tb = 0;
    for (int i = 0; i < R; ++i) {
      float a, b2;
      CK(hipEventElapsedTime(&a, ev[2 * i], ev[2 * i + 1]));
      CK(hipEventElapsedTime(&b2, ev[2 * i + 1], ev[2 * i + 2]));
      tr += a;
      tb += b2;
    }
    float tot;
    CK(hipEventElapsedTime(&tot, ev[0], ev[2 * R]));
    printf("{\"lab\": \"write\", \"alloc\": \"%s\", \"variant\": \"in_round_%s\", \"pass\": %d, \"read20_us\": %.2f, "
           "\"bcast_us\": %.2f, \"round_us\": %.2f, \"round_GBps\": %.1f}\n",
           ptag, name, pass, tr / R * 1e3, tb / R * 1e3, tot / R * 1e3,
           (rbytes + bbytes) / (tot / R * 1e-3) / 1e9);
    fflush(stdout);
    for (auto& ev1 : ev) CK(hipEventDestroy(ev1));
  };
#define FILL(U, G, M, X)                                                                   \
  rep("fill_" #M "_U" #U "_G" #G "_xcd" #X,                                                \
      time_ms([&] { fill<U, G, M, X><<<blocks(U, G, X), 256>>>(d, nv, parts(U)); }, R), wbytes, \
      pass)
#define BC(U, G, X, NT)                                                                    \
  rep("bcast_U" #U "_G" #G "_xcd" #X "_nt" #NT,                                            \
      time_ms([&] { bcast<U, G, X, NT><<<blocks(U, G, X), 256>>>(s, d, nv, parts(U)); }, R), \
      bbytes, pass)
  for (int pass = 0; pass < passes && !full; ++pass) {
    FILL(1, 1, 1, 0);
    FILL(2, 10, 1, 0);
    BC(2, 10, 0, 1);
    BC(1, 20, 0, 1);
    BC(1, 10, 0, 1);
    rep("read20_nt", time_ms([&] { read20<true><<<parts(2), 256>>>(d, out, nv); }, R), rbytes,
        pass);
    in_round("U2_G10", [&] { bcast<2, 10, false, true><<<blocks(2, 10, false), 256>>>(s, d, nv, parts(2)); }, pass);
    in_round("U1_G20", [&] { bcast<1, 20, false, true><<<blocks(1, 20, false), 256>>>(s, d, nv, parts(1)); }, pass);
    in_round("fill_hash_U2_G10", [&] { fill<2, 10, 1, false><<<blocks(2, 10, false), 256>>>(d, nv, parts(2)); }, pass);
  }
  for (int pass = 0; pass < passes && full; ++pass) {
    // pure writes (the ceiling): constant, hashed, hashed per client
    FILL(1, 1, 0, 0);
    FILL(2, 10, 0, 0);
    FILL(1, 1, 1, 0);
    FILL(2, 1, 1, 0);
    FILL(2, 10, 1, 0);
    FILL(2, 20, 1, 0);
    FILL(2, 10, 2, 0);
    FILL(1, 10, 1, 0);
    FILL(4, 10, 1, 0);
    // broadcasts
    BC(2, 10, 0, 1);  // the product's form
    BC(2, 10, 1, 1);
    BC(2, 20, 0, 1);
    BC(2, 20, 1, 1);
    BC(2, 5, 0, 1);
    BC(1, 10, 0, 1);
    BC(1, 20, 0, 1);
    BC(2, 10, 0, 0);
    BC(4, 10, 0, 1);
    for (int gr : {1024, 2048, 4096}) {
      char nm[64];
      snprintf(nm, sizeof nm, "bcast_persist_U2_G10_grid%d", gr);
      rep(nm, time_ms([&] { bcast_persist<2, 10><<<gr, 256>>>(s, d, nv, parts(2)); }, R), bbytes,
          pass);
    }
    rep("read20_nt", time_ms([&] { read20<true><<<parts(2), 256>>>(d, out, nv); }, R), rbytes,
        pass);
    in_round("U2_G10", [&] { bcast<2, 10, false, true><<<blocks(2, 10, false), 256>>>(s, d, nv, parts(2)); }, pass);
    in_round("U2_G20", [&] { bcast<2, 20, false, true><<<blocks(2, 20, false), 256>>>(s, d, nv, parts(2)); }, pass);
    in_round("U1_G20", [&] { bcast<1, 20, false, true><<<blocks(1, 20, false), 256>>>(s, d, nv, parts(1)); }, pass);
    in_round("U1_G10", [&] { bcast<1, 10, false, true><<<blocks(1, 10, false), 256>>>(s, d, nv, parts(1)); }, pass);
    in_round("U2_G10_xcd", [&] { bcast<2, 10, true, true><<<blocks(2, 10, true), 256>>>(s, d, nv, parts(2)); }, pass);
    in_round("fill_hash_U2_G10", [&] { fill<2, 10, 1, false><<<blocks(2, 10, false), 256>>>(d, nv, parts(2)); }, pass);
    in_round("none", [&] {}, pass);
  }
  CK(hipFree(slab));
  for (size_t i = 1; i < churn.size(); i += 2) CK(hipFree(churn[i]));
  }
  return 0;
}
