// bcastlab.hip — the round's broadcast (train_fedavg.py:148-149: every client
// slot <- global) as a standalone lab: N = 20 destination buckets of the
// wrn16_8 size (10,972,186 floats, 43.9 MB) from one source bucket, against
// the pure-write ceiling of the same bytes.  Standalone binary:
//   hipcc --offload-arch=gfx950 -O3 -o tools/bcastlab tools/bcastlab.hip
// One JSON line per variant and round; GB/s = (B read + N*B written) / time
// (the bench's bytes for the broadcast; "fill" counts its N*B written only).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>

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

// pure writes: one float4 per lane, U per lane, one tile per workgroup,
// destination-major (workgroup b writes tile b % T of client b / T)
template <int U>
__global__ __launch_bounds__(256) void fill(Dst d, int64_t nv, int64_t tiles) {
  const int c = (int)(blockIdx.x / tiles);
  const int64_t b = (int64_t)(blockIdx.x % tiles) * U * 256 + threadIdx.x;
  const f4 x = {1.f, 2.f, 3.f, 4.f};
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (b + u * 256 < nv) stnt(d.d[c], b + u * 256, x);
}

// the product's shape: a workgroup per source tile of U*256 float4, its
// loads before the N*U stores
template <int U>
__global__ __launch_bounds__(256) void tile_major(const float* s, Dst d, int64_t nv) {
  const int64_t b = (int64_t)blockIdx.x * U * 256 + threadIdx.x;
  f4 x[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (b + u * 256 < nv) x[u] = ldnt(s, b + u * 256);
  for (int c = 0; c < kN; ++c)
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (b + u * 256 < nv) stnt(d.d[c], b + u * 256, x[u]);
}

// a workgroup per (tile, group of G clients), clients fastest: the G-groups
// of one tile run side by side, the source tile is re-read from L2
template <int U, int G>
__global__ __launch_bounds__(256) void split(const float* s, Dst d, int64_t nv) {
  constexpr int NG = (kN + G - 1) / G;
  const int g = (int)(blockIdx.x % NG);
  const int64_t b = (int64_t)(blockIdx.x / NG) * U * 256 + threadIdx.x;
  f4 x[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (b + u * 256 < nv) x[u] = ldp(s, b + u * 256);
#pragma unroll
  for (int i = 0; i < G; ++i) {
    const int c = g * G + i;
    if (c >= kN) break;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (b + u * 256 < nv) stnt(d.d[c], b + u * 256, x[u]);
  }
}

// split_U1_G1 as the product writes it: runtime client count (scalar
// division), a grid-stride loop, the source base offset per part
__global__ __launch_bounds__(256) void split_rt(const float* s, Dst d, int64_t nv, uint32_t n,
                                                uint32_t parts) {
  const uint32_t total = parts * n;
  for (uint32_t v = blockIdx.x; v < total; v += gridDim.x) {
    const uint32_t p = v / n;
    const int c = (int)(v - p * n);
    const int64_t base = (int64_t)p * 256;
    if (base + threadIdx.x < nv) stnt(d.d[c] + 4 * base, threadIdx.x, ldp(s + 4 * base, threadIdx.x));
  }
}

// ... plus a 16-B descriptor per part read from a table first (the tiled
// product's dependent fetch)
struct Desc {
  int64_t start;
  int32_t count, kind;
};
__global__ __launch_bounds__(256) void split_rt_table(const float* s, Dst d, const Desc* t,
                                                      uint32_t n, uint32_t parts) {
  const uint32_t total = parts * n;
  for (uint32_t v = blockIdx.x; v < total; v += gridDim.x) {
    const uint32_t p = v / n;
    const int c = (int)(v - p * n);
    const Desc x = t[p];
    if ((int)threadIdx.x * 4 < x.count)
      stnt(d.d[c] + x.start, threadIdx.x, ldp(s + x.start, threadIdx.x));
  }
}

// non-zero, non-repeating data (an integer hash per element)
__global__ void hash_fill(float* p, int64_t n, uint32_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 15;
    x *= 2246822519u;
    x ^= x >> 13;
    p[i] = (float)(x & 0xFFFFFF) * (1.0f / 16777216.0f) - 0.5f;
  }
}

// client-major: workgroup b copies tile b % T into client b / T (the source
// is re-read from the Infinity Cache, 43.9 MB << 256 MiB)
template <int U>
__global__ __launch_bounds__(256) void client_major(const float* s, Dst d, int64_t nv,
                                                    int64_t tiles) {
  const int c = (int)(blockIdx.x / tiles);
  const int64_t b = (int64_t)(blockIdx.x % tiles) * U * 256 + threadIdx.x;
  f4 x[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (b + u * 256 < nv) x[u] = ldp(s, b + u * 256);
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (b + u * 256 < nv) stnt(d.d[c], b + u * 256, x[u]);
}

template <class F>
float time_ms(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 5; ++i) f();
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

int main() {
  const int64_t n = 10972186 / 4 * 4;  // wrn16_8 C10 floats, vector part
  const int64_t nv = n / 4;
  float* s;
  CK(hipMalloc(&s, n * 4));
  CK(hipMemset(s, 0, n * 4));
  Dst d;
  for (int c = 0; c < kN; ++c) {
    CK(hipMalloc(&d.d[c], n * 4));
    CK(hipMemset(d.d[c], 0, n * 4));
  }
  const double bytes = (1.0 + kN) * n * 4, wbytes = 1.0 * kN * n * 4;
  auto rep = [&](const char* name, float ms, double b) {
    printf("{\"variant\": \"%s\", \"us\": %.1f, \"GBps\": %.1f}\n", name, ms * 1e3,
           b / (ms * 1e-3) / 1e9);
    fflush(stdout);
  };
  auto T = [&](int U) { return (nv + U * 256 - 1) / (U * 256); };
  const uint32_t parts = (uint32_t)((nv + 255) / 256);
  Desc* hd = (Desc*)malloc(parts * sizeof(Desc));
  for (uint32_t p = 0; p < parts; ++p)
    hd[p] = Desc{(int64_t)p * 1024, (int32_t)std::min<int64_t>(1024, n - (int64_t)p * 1024), 0};
  Desc* dd;
  CK(hipMalloc(&dd, parts * sizeof(Desc)));
  CK(hipMemcpy(dd, hd, parts * sizeof(Desc), hipMemcpyHostToDevice));
  for (int r = 0; r < 3; ++r) {
    rep("split_rt", time_ms([&] { split_rt<<<parts * kN, 256>>>(s, d, nv, kN, parts); }, 20),
        bytes);
    rep("split_rt_table",
        time_ms([&] { split_rt_table<<<parts * kN, 256>>>(s, d, dd, kN, parts); }, 20), bytes);
    rep("fill_U1", time_ms([&] { fill<1><<<T(1) * kN, 256>>>(d, nv, T(1)); }, 20), wbytes);
    rep("fill_U2", time_ms([&] { fill<2><<<T(2) * kN, 256>>>(d, nv, T(2)); }, 20), wbytes);
    rep("tile_major_U2", time_ms([&] { tile_major<2><<<T(2), 256>>>(s, d, nv); }, 20), bytes);
    rep("tile_major_U1", time_ms([&] { tile_major<1><<<T(1), 256>>>(s, d, nv); }, 20), bytes);
    rep("split_U1_G1", time_ms([&] { split<1, 1><<<T(1) * 20, 256>>>(s, d, nv); }, 20), bytes);
    rep("split_U1_G2", time_ms([&] { split<1, 2><<<T(1) * 10, 256>>>(s, d, nv); }, 20), bytes);
    rep("split_U1_G4", time_ms([&] { split<1, 4><<<T(1) * 5, 256>>>(s, d, nv); }, 20), bytes);
    rep("split_U2_G4", time_ms([&] { split<2, 4><<<T(2) * 5, 256>>>(s, d, nv); }, 20), bytes);
    rep("split_U2_G5", time_ms([&] { split<2, 5><<<T(2) * 4, 256>>>(s, d, nv); }, 20), bytes);
    rep("split_U2_G10", time_ms([&] { split<2, 10><<<T(2) * 2, 256>>>(s, d, nv); }, 20), bytes);
    rep("client_major_U1",
        time_ms([&] { client_major<1><<<T(1) * kN, 256>>>(s, d, nv, T(1)); }, 20), bytes);
    rep("client_major_U2",
        time_ms([&] { client_major<2><<<T(2) * kN, 256>>>(s, d, nv, T(2)); }, 20), bytes);
  }
  // the same variants with non-zero data in the source and every destination
  hash_fill<<<4096, 256>>>(s, n, 7u);
  for (int c = 0; c < kN; ++c) hash_fill<<<4096, 256>>>(d.d[c], n, 100u + c);
  CK(hipDeviceSynchronize());
  for (int r = 0; r < 2; ++r) {
    rep("rand_split_U1_G2", time_ms([&] { split<1, 2><<<T(1) * 10, 256>>>(s, d, nv); }, 20), bytes);
    rep("rand_split_U1_G4", time_ms([&] { split<1, 4><<<T(1) * 5, 256>>>(s, d, nv); }, 20), bytes);
    rep("rand_split_U1_G7", time_ms([&] { split<1, 7><<<T(1) * 3, 256>>>(s, d, nv); }, 20), bytes);
    rep("rand_split_U1_G10", time_ms([&] { split<1, 10><<<T(1) * 2, 256>>>(s, d, nv); }, 20), bytes);
    rep("rand_split_U2_G2", time_ms([&] { split<2, 2><<<T(2) * 10, 256>>>(s, d, nv); }, 20), bytes);
    rep("rand_split_U2_G4", time_ms([&] { split<2, 4><<<T(2) * 5, 256>>>(s, d, nv); }, 20), bytes);
    rep("rand_split_U2_G7", time_ms([&] { split<2, 7><<<T(2) * 3, 256>>>(s, d, nv); }, 20), bytes);
    rep("rand_split_U2_G10", time_ms([&] { split<2, 10><<<T(2) * 2, 256>>>(s, d, nv); }, 20), bytes);
    rep("rand_split_U4_G4", time_ms([&] { split<4, 4><<<T(4) * 5, 256>>>(s, d, nv); }, 20), bytes);
    rep("rand_split_U4_G10", time_ms([&] { split<4, 10><<<T(4) * 2, 256>>>(s, d, nv); }, 20), bytes);
    rep("rand_fill_U1", time_ms([&] { fill<1><<<T(1) * kN, 256>>>(d, nv, T(1)); }, 20), wbytes);
  }
  for (int r = 0; r < 3; ++r) {
    rep("rand_split_rt", time_ms([&] { split_rt<<<parts * kN, 256>>>(s, d, nv, kN, parts); }, 20),
        bytes);
    rep("rand_split_U2_G5", time_ms([&] { split<2, 5><<<T(2) * 4, 256>>>(s, d, nv); }, 20), bytes);
    rep("rand_tile_major_U2", time_ms([&] { tile_major<2><<<T(2), 256>>>(s, d, nv); }, 20),
        bytes);
  }
  CK(hipFree(s));
  for (int c = 0; c < kN; ++c) CK(hipFree(d.d[c]));
  return 0;
}
