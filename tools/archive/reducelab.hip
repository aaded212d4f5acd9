// reducelab.hip — where the write stream's cost comes from in an N-client
// tile reduction (cfg3: N=5, cfg2: N=20), against the copy kernel on the
// same allocation scheme.  Standalone lab binary (not the product):
//   hipcc --offload-arch=gfx950 -O3 -o tools/reducelab tools/reducelab.hip
// One JSON line per (variant, N, round); GB/s counts N inputs + 1 output.
// `reducelab hashed [pipe]`: every buffer filled with non-zero hashed values first
// (zero-filled buffers stream faster on this chip than real data,
// tools/bcastlab.hip; the r02 numbers before this option were on zeros).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
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

constexpr int MAXN = 20;
struct Ptrs {
  const float* c[MAXN];
};

__device__ __forceinline__ f4 ld(const float* p, int64_t v) {
  return __builtin_nontemporal_load((gcf4*)p + v);
}
__device__ __forceinline__ void st(float* p, int64_t v, f4 x) {
  __builtin_nontemporal_store(x, (gf4*)p + v);
}

// MODE 0: client by client (U loads, wait, add); 1: all N*U loads issued
// first; 2: like 0 but no store (read-only); 3: like 0 with the tile order
// strided across the grid (block b -> tile (b * S) mod T).
template <int N, int U, int MODE>
__global__ __launch_bounds__(256) void nsum(Ptrs p, float* out, int64_t nv, int ntiles, int S) {
  int t = blockIdx.x;
  if constexpr (MODE == 3) t = (int)(((int64_t)blockIdx.x * S) % ntiles);
  const int64_t b = (int64_t)t * U * 256 + threadIdx.x;
  f4 acc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) acc[u] = f4{0, 0, 0, 0};
  if constexpr (MODE == 1) {
    f4 x[N][U];
#pragma unroll
    for (int c = 0; c < N; ++c)
#pragma unroll
      for (int u = 0; u < U; ++u) x[c][u] = ld(p.c[c], b + u * 256);
#pragma unroll
    for (int c = 0; c < N; ++c)
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] += x[c][u];
  } else {
#pragma unroll
    for (int c = 0; c < N; ++c) {
      f4 x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) x[u] = ld(p.c[c], b + u * 256);
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] += x[u];
    }
  }
  if constexpr (MODE == 2) {
    // keep the sum live without storing it (one lane of 2^20 writes)
    f4 all = acc[0];
#pragma unroll
    for (int u = 1; u < U; ++u) all += acc[u];
    if (all.x == 1.2345e-30f && all.y == 6.789e-31f) st(out, b, all);
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u) st(out, b + u * 256, acc[u]);
  }
}

// G consecutive tiles per workgroup (U=1: 1024 floats each); each tile's
// result parked in LDS, the G results stored back to back after the last
// tile's reads (writes clustered in time, reads unchanged).
template <int N, int G>
__global__ __launch_bounds__(256) void nsum_park(Ptrs p, float* out, int64_t nv, int ntiles) {
  __shared__ f4 park[G][256];
  const int t0 = blockIdx.x * G;
#pragma unroll 1
  for (int g = 0; g < G; ++g) {
    const int t = t0 + g;
    if (t >= ntiles) break;
    const int64_t b = (int64_t)t * 256 + threadIdx.x;
    f4 acc = f4{0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < N; ++c) acc += ld(p.c[c], b);
    park[g][threadIdx.x] = acc;
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int t = t0 + g;
    if (t >= ntiles) break;
    st(out, (int64_t)t * 256 + threadIdx.x, park[g][threadIdx.x]);
  }
}

// r03: G consecutive tiles per workgroup, software-
// pipelined across tiles — tile g's loads (all N*U) are issued, THEN tile
// g-1's result is stored, so every store leaves behind a full tile of loads
// in flight (the write does not wait behind its own tile's reads).
template <int N, int U, int G>
__global__ __launch_bounds__(256) void nsum_pipe(Ptrs p, float* out, int64_t nv, int ntiles) {
  const int t0 = blockIdx.x * G;
  f4 prev[U];
  int64_t prevb = -1;
#pragma unroll 1
  for (int g = 0; g < G; ++g) {
    const int t = t0 + g;
    if (t >= ntiles) break;
    const int64_t b = (int64_t)t * U * 256 + threadIdx.x;
    f4 x[N][U];
#pragma unroll
    for (int c = 0; c < N; ++c)
#pragma unroll
      for (int u = 0; u < U; ++u) x[c][u] = ld(p.c[c], b + u * 256);
    if (prevb >= 0) {
#pragma unroll
      for (int u = 0; u < U; ++u) st(out, prevb + u * 256, prev[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f4 acc = f4{0, 0, 0, 0};
#pragma unroll
      for (int c = 0; c < N; ++c) acc += x[c][u];
      prev[u] = acc;
    }
    prevb = b;
  }
  if (prevb >= 0) {
#pragma unroll
    for (int u = 0; u < U; ++u) st(out, prevb + u * 256, prev[u]);
  }
}

__global__ __launch_bounds__(256) void copy1(const float* s, float* d, int64_t nv) {
  const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (v < nv) st(d, v, ld(s, v));
}

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

template <class F>
float time_us(F f, int reps) {
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
  return ms * 1e3f / reps;
}

int main(int argc, char** argv) {
  const bool hashed = argc > 1 && strcmp(argv[1], "hashed") == 0;
  const int64_t m = 10971136;  // floats per client: ~ the wrn16_8 bucket, 4096-aligned
  const int64_t nv = m / 4;
  std::vector<float*> bufs(MAXN);
  for (auto& q : bufs) {
    CK(hipMalloc(&q, m * 4));
    CK(hipMemset(q, 0, m * 4));
  }
  float* out;
  CK(hipMalloc(&out, m * 4));
  CK(hipMemset(out, 0, m * 4));
  Ptrs p;
  for (int c = 0; c < MAXN; ++c) p.c[c] = bufs[c];
  auto rep = [&](const char* name, int n, float us, int nw) {
    double bytes = (double)m * 4 * (n + nw);
    printf("{\"variant\": \"%s\", \"n\": %d, \"data\": \"%s\", \"us\": %.2f, "
           "\"GBps\": %.1f}\n", name, n, hashed ? "hashed" : "zeros", us,
           bytes / (us * 1e-6) / 1e9);
    fflush(stdout);
  };
  const int t1 = (int)(nv / 256), t2 = (int)(nv / 512);
  // a second, disjoint set for rotation (the bench's cfg3 form: 2 sets > MALL)
  std::vector<float*> bufs2(MAXN);
  for (auto& q : bufs2) {
    CK(hipMalloc(&q, m * 4));
    CK(hipMemset(q, 0, m * 4));
  }
  float* out2;
  CK(hipMalloc(&out2, m * 4));
  Ptrs p2;
  for (int c = 0; c < MAXN; ++c) p2.c[c] = bufs2[c];
  if (hashed) {
    uint32_t seed = 1;
    for (auto* q : bufs) hash_fill<<<4096, 256>>>(q, m, seed++);
    for (auto* q : bufs2) hash_fill<<<4096, 256>>>(q, m, seed++);
    hash_fill<<<4096, 256>>>(out, m, seed++);
    hash_fill<<<4096, 256>>>(out2, m, seed++);
    CK(hipDeviceSynchronize());
  }
  int flip = 0;
#define RUN(N)                                                                                   \
  rep("rw_U1", N, time_us([&] { nsum<N, 1, 0><<<t1, 256>>>(p, out, nv, t1, 1); }, 20), 1);       \
  rep("rw_U2", N, time_us([&] { nsum<N, 2, 0><<<t2, 256>>>(p, out, nv, t2, 1); }, 20), 1);       \
  rep("issue_all_U1", N, time_us([&] { nsum<N, 1, 1><<<t1, 256>>>(p, out, nv, t1, 1); }, 20), 1); \
  rep("ro_U1", N, time_us([&] { nsum<N, 1, 2><<<t1, 256>>>(p, out, nv, t1, 1); }, 20), 0);       \
  rep("ro_U2", N, time_us([&] { nsum<N, 2, 2><<<t2, 256>>>(p, out, nv, t2, 1); }, 20), 0);       \
  rep("strided_U1_S257", N,                                                                      \
      time_us([&] { nsum<N, 1, 3><<<t1, 256>>>(p, out, nv, t1, 257); }, 20), 1);                 \
  rep("strided_U1_S9", N, time_us([&] { nsum<N, 1, 3><<<t1, 256>>>(p, out, nv, t1, 9); }, 20), 1); \
  rep("rw_U1_rot2", N, time_us([&] {                                                             \
        flip ^= 1;                                                                               \
        nsum<N, 1, 0><<<t1, 256>>>(flip ? p2 : p, flip ? out2 : out, nv, t1, 1);                 \
      }, 20), 1);                                                                                \
  rep("rw_U2_rot2", N, time_us([&] {                                                             \
        flip ^= 1;                                                                               \
        nsum<N, 2, 0><<<t2, 256>>>(flip ? p2 : p, flip ? out2 : out, nv, t2, 1);                 \
      }, 20), 1);
#define PARK(N, G)                                                                               \
  rep("park_G" #G, N,                                                                            \
      time_us([&] { nsum_park<N, G><<<(t1 + G - 1) / G, 256>>>(p, out, nv, t1); }, 20), 1);
#define PIPE(N, U, G, T)                                                                         \
  rep("pipe_U" #U "_G" #G "_rot2", N, time_us([&] {                                              \
        flip ^= 1;                                                                               \
        nsum_pipe<N, U, G><<<(T + G - 1) / G, 256>>>(flip ? p2 : p, flip ? out2 : out, nv, T);   \
      }, 20), 1);
  if (argc > 2 && strcmp(argv[2], "pipe") == 0) {   // r03: the cross-tile pipeline A/B only
    for (int r = 0; r < 3; ++r) {
      rep("rw_U1_rot2", 5, time_us([&] {
            flip ^= 1;
            nsum<5, 1, 0><<<t1, 256>>>(flip ? p2 : p, flip ? out2 : out, nv, t1, 1);
          }, 20), 1);
      rep("rw_U2_rot2", 5, time_us([&] {
            flip ^= 1;
            nsum<5, 2, 0><<<t2, 256>>>(flip ? p2 : p, flip ? out2 : out, nv, t2, 1);
          }, 20), 1);
      PIPE(5, 1, 2, t1) PIPE(5, 1, 4, t1) PIPE(5, 1, 8, t1)
      PIPE(5, 2, 2, t2) PIPE(5, 2, 4, t2)
      PIPE(20, 1, 2, t1) PIPE(20, 2, 2, t2)
      rep("rw_U2_rot2", 20, time_us([&] {
            flip ^= 1;
            nsum<20, 2, 0><<<t2, 256>>>(flip ? p2 : p, flip ? out2 : out, nv, t2, 1);
          }, 20), 1);
    }
    return 0;
  }
  for (int r = 0; r < 2; ++r) {
    rep("copy1", 1, time_us([&] { copy1<<<t1, 256>>>(bufs[0], out, nv); }, 20), 1);
    RUN(5) RUN(20)
    if (!hashed) {
      PARK(20, 1) PARK(20, 2) PARK(20, 4) PARK(20, 8) PARK(20, 16)
      PARK(5, 1) PARK(5, 4) PARK(5, 16)
    }
  }
  return 0;
}
