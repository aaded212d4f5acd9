// bwlab.hip — standalone bandwidth lab (tools only, not the product):
// what HBM rate do N-stream reductions reach on this chip, with and without
// the output stream, against a single-stream read and a copy?
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bwlab tools/bwlab.hip
// Run:   tools/bwlab [n_clients=20] [floats_per_client=10972160]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

__device__ __forceinline__ f4 ld(const float* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const f4*>(p));
}
__device__ __forceinline__ void st(float* p, f4 v) {
  __builtin_nontemporal_store(v, reinterpret_cast<f4*>(p));
}

// N streams (client i at base + i*stride), tile of U*1024 floats per
// workgroup, loads in batches of NB clients; WRITE: store the sum, else only
// a never-true guarded store (keeps the loads alive).
template <int U, int NB, bool WRITE>
__global__ __launch_bounds__(256) void nstream(const float* __restrict__ base, int64_t stride,
                                               int n, float* __restrict__ out) {
  const int64_t t0 = (int64_t)blockIdx.x * U * 1024;
  f4 acc[U];
  int64_t off[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    off[u] = t0 + 4 * (int64_t)(threadIdx.x + u * 256);
    acc[u] = f4{0.f, 0.f, 0.f, 0.f};
  }
  int b0 = 0;
  for (; b0 + NB <= n; b0 += NB) {
    f4 x[NB][U];
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int u = 0; u < U; ++u) x[b][u] = ld(base + (b0 + b) * stride + off[u]);
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] += x[b][u];
  }
  for (; b0 < n; ++b0)
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] += ld(base + b0 * stride + off[u]);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (WRITE) st(out + off[u], acc[u]);
    else if (acc[u].x == 1234.5f && acc[u].y == -1.f) st(out + off[u], acc[u]);
  }
}

// Buffer-op variant with explicit cache-policy bits (gfx950 aux: 1 = sc0,
// 2 = nt, 16 = sc1) on the loads (LA) and the store (SA).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, 0x7fffffff,
                                           0x00020000);
}
template <int U, int NB, int LA, int SA>
__global__ __launch_bounds__(256) void nstream_pol(const float* __restrict__ base,
                                                   int64_t stride, int n,
                                                   float* __restrict__ out) {
  const int64_t t0 = (int64_t)blockIdx.x * U * 1024;
  f4 acc[U];
  int voff[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    voff[u] = 16 * (threadIdx.x + u * 256);
    acc[u] = f4{0.f, 0.f, 0.f, 0.f};
  }
  int b0 = 0;
  for (; b0 + NB <= n; b0 += NB) {
    f4 x[NB][U];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const __amdgpu_buffer_rsrc_t r = rsrc(base + (b0 + b) * stride + t0);
#pragma unroll
      for (int u = 0; u < U; ++u) x[b][u] = __builtin_amdgcn_raw_buffer_load_b128(r, voff[u], 0, LA);
    }
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] += x[b][u];
  }
  for (; b0 < n; ++b0) {
    const __amdgpu_buffer_rsrc_t r = rsrc(base + b0 * stride + t0);
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] += __builtin_amdgcn_raw_buffer_load_b128(r, voff[u], 0, LA);
  }
  const __amdgpu_buffer_rsrc_t ro = rsrc(out + t0);
#pragma unroll
  for (int u = 0; u < U; ++u) __builtin_amdgcn_raw_buffer_store_b128(acc[u], ro, voff[u], 0, SA);
}

// Deferred writes: each workgroup reduces K consecutive tiles, keeping the K
// results in registers, and stores them all at the end (writes cluster in
// time instead of trickling between other workgroups' reads).
template <int U, int NB, int K>
__global__ __launch_bounds__(256) void nstream_defer(const float* __restrict__ base,
                                                     int64_t stride, int n,
                                                     float* __restrict__ out) {
  f4 acc[K][U];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int64_t t0 = ((int64_t)blockIdx.x * K + k) * U * 1024;
    int64_t off[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      off[u] = t0 + 4 * (int64_t)(threadIdx.x + u * 256);
      acc[k][u] = f4{0.f, 0.f, 0.f, 0.f};
    }
    int b0 = 0;
    for (; b0 + NB <= n; b0 += NB) {
      f4 x[NB][U];
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int u = 0; u < U; ++u) x[b][u] = ld(base + (b0 + b) * stride + off[u]);
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int u = 0; u < U; ++u) acc[k][u] += x[b][u];
    }
    for (; b0 < n; ++b0)
#pragma unroll
      for (int u = 0; u < U; ++u) acc[k][u] += ld(base + b0 * stride + off[u]);
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int64_t t0 = ((int64_t)blockIdx.x * K + k) * U * 1024;
#pragma unroll
    for (int u = 0; u < U; ++u) st(out + t0 + 4 * (int64_t)(threadIdx.x + u * 256), acc[k][u]);
  }
}

// Persistent park: each workgroup of TPB threads reduces S sub-tiles of
// TPB*4 floats (contiguous range, or interleaved with the other workgroups:
// sub-tile s of workgroup g at s*G + g), keeps the S results in registers and
// stores them all at the end (PARK), so writes come in one burst after reads.
template <int S, int NB, int TPB, bool PARK, bool INTER>
__global__ __launch_bounds__(TPB) void persist(const float* __restrict__ base, int64_t stride,
                                               int n, float* __restrict__ out) {
  f4 park[S];
#pragma unroll
  for (int sidx = 0; sidx < S; ++sidx) {
    const int64_t tile = INTER ? (int64_t)sidx * gridDim.x + blockIdx.x
                               : (int64_t)blockIdx.x * S + sidx;
    const int64_t off = tile * TPB * 4 + 4 * (int64_t)threadIdx.x;
    f4 acc = f4{0.f, 0.f, 0.f, 0.f};
    int b0 = 0;
    for (; b0 + NB <= n; b0 += NB) {
      f4 x[NB];
#pragma unroll
      for (int b = 0; b < NB; ++b) x[b] = ld(base + (b0 + b) * stride + off);
#pragma unroll
      for (int b = 0; b < NB; ++b) acc += x[b];
    }
    for (; b0 < n; ++b0) acc += ld(base + b0 * stride + off);
    if (PARK) park[sidx] = acc;
    else st(out + off, acc);
  }
  if (PARK) {
#pragma unroll
    for (int sidx = 0; sidx < S; ++sidx) {
      const int64_t tile = INTER ? (int64_t)sidx * gridDim.x + blockIdx.x
                                 : (int64_t)blockIdx.x * S + sidx;
      st(out + tile * TPB * 4 + 4 * (int64_t)threadIdx.x, park[sidx]);
    }
  }
}

// Rolling window: at most W clients' loads (W*U per lane) in flight; the load
// of client b+W is issued right after client b is consumed.  SERIAL: the
// old product shape (issue U loads, wait for them, add, next client).
template <int U, int W>
__global__ __launch_bounds__(256) void nstream_win(const float* __restrict__ base,
                                                   int64_t stride, int n,
                                                   float* __restrict__ out) {
  const int64_t t0 = (int64_t)blockIdx.x * U * 1024;
  f4 acc[U];
  int64_t off[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    off[u] = t0 + 4 * (int64_t)(threadIdx.x + u * 256);
    acc[u] = f4{0.f, 0.f, 0.f, 0.f};
  }
  f4 x[W][U];
#pragma unroll
  for (int w = 0; w < W; ++w)
#pragma unroll
    for (int u = 0; u < U; ++u) x[w][u] = w < n ? ld(base + w * stride + off[u]) : f4{0, 0, 0, 0};
  int b = 0;
  for (; b + W <= n; b += W) {
#pragma unroll
    for (int w = 0; w < W; ++w) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        acc[u] += x[w][u];
        if (b + w + W < n) x[w][u] = ld(base + (b + w + W) * stride + off[u]);
      }
    }
  }
#pragma unroll
  for (int w = 0; w < W; ++w)
    if (b + w < n)
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] += x[w][u];
#pragma unroll
  for (int u = 0; u < U; ++u) st(out + off[u], acc[u]);
}

__global__ __launch_bounds__(256) void copy4(const float* __restrict__ s, float* __restrict__ d,
                                             int64_t nv) {
  for (int64_t v = blockIdx.x * 256ll + threadIdx.x; v < nv; v += (int64_t)gridDim.x * 256)
    st(d + 4 * v, ld(s + 4 * v));
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

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 20;
  int64_t m = argc > 2 ? atoll(argv[2]) : 10972160;  // wrn16_8 C10 fp32, 2048-multiple
  m = (m + 8191) / 8192 * 8192;
  const int64_t stride = m + 64 * 1024;  // 256 KiB gap between clients
  float *base, *out;
  CK(hipMalloc(&base, (size_t)(n * stride) * 4));
  CK(hipMalloc(&out, (size_t)m * 4));
  CK(hipMemset(base, 0, (size_t)(n * stride) * 4));
  const double rbytes = (double)n * m * 4, wbytes = (double)m * 4;
  auto rep = [&](const char* name, float ms, double bytes) {
    printf("{\"variant\": \"%s\", \"n\": %d, \"us\": %.2f, \"GBps\": %.1f}\n", name, n, ms * 1e3,
           bytes / (ms * 1e-3) / 1e9);
  };
  for (int round = 0; round < 5; ++round) {
    rep("n_stream_read_write_U2B16",
        time_ms([&] { nstream<2, 16, true><<<m / 2048, 256>>>(base, stride, n, out); }, 20),
        rbytes + wbytes);
    rep("n_stream_read_only_U2B16",
        time_ms([&] { nstream<2, 16, false><<<m / 2048, 256>>>(base, stride, n, out); }, 20),
        rbytes);
    rep("n_stream_read_write_U4B8",
        time_ms([&] { nstream<4, 8, true><<<m / 4096, 256>>>(base, stride, n, out); }, 20),
        rbytes + wbytes);
    rep("n_stream_read_only_U4B8",
        time_ms([&] { nstream<4, 8, false><<<m / 4096, 256>>>(base, stride, n, out); }, 20),
        rbytes);
    // one stream over the same bytes: n*m floats as one "client"
    const int64_t big = (int64_t)n * stride / 4096 * 4096;
    rep("one_stream_read_only_U2",
        time_ms([&] { nstream<2, 1, false><<<big / 2048, 256>>>(base, 0, 1, out); }, 20),
        (double)big * 4);
    rep("one_stream_read_only_U8",
        time_ms([&] { nstream<8, 1, false><<<big / 8192, 256>>>(base, 0, 1, out); }, 20),
        (double)big * 4);
#define POL(LA, SA)                                                                    \
  rep("pol_ld" #LA "_st" #SA,                                                          \
      time_ms([&] { nstream_pol<2, 16, LA, SA><<<m / 2048, 256>>>(base, stride, n, out); }, \
              20),                                                                     \
      rbytes + wbytes)
#define WIN(U, W)                                                                         \
  rep("win_U" #U "_W" #W,                                                                 \
      time_ms([&] { nstream_win<U, W><<<m / (U * 1024), 256>>>(base, stride, n, out); }, 20), \
      rbytes + wbytes)
    WIN(2, 1); WIN(2, 2); WIN(2, 3); WIN(2, 4); WIN(2, 6); WIN(2, 8); WIN(2, 16);
    WIN(1, 1); WIN(1, 2); WIN(1, 4); WIN(1, 8); WIN(4, 1); WIN(4, 2);
    const int64_t half = big / 2;
    rep("copy_float4",
        time_ms([&] { copy4<<<4096, 256>>>(base, base + half, half / 4); }, 20),
        (double)half * 8);
  }
  CK(hipFree(base));
  CK(hipFree(out));
  return 0;
}
