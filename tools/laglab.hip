// laglab.hip — can ONE launch do the whole round (reduce + broadcast) faster
// than the product's two?  (r05)  r04's single pass
// (every workgroup broadcasting its own tile right after reducing it) lost on
// every layout: the broadcast read a line the same launch had just written.
// Here the broadcast of tile j is done LAG tiles later in the grid: workgroup
// w reduces tile w (w < T) and then broadcasts tile w - LAG (0 <= w - LAG <
// T), after that tile's reducer has published it.  LAG = T is the split grid
// (reducers first, then broadcasters, one launch).
//
// Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, the sc1 table's
// first row): the reducer stores its result sc1 (write-through, as the
// product's reduce does), every storing wave waits vmcnt(0), a workgroup
// barrier, then one lane stores the tile's flag sc1 (the launch's epoch); the
// broadcaster's lane 0 polls the flag with sc1 loads (bounded: a poll that
// times out counts an error and the tile is skipped, so a launch always
// drains), a workgroup barrier, then every load of the result is an sc1
// buffer load.
//
// Everything is compared in ONE process on the same buckets (hashed data,
// each client set in one slab, sets rotated past the 256 MiB MALL as
// bench.py other_configs): the lab reduce, the lab broadcast, the two as
// separate launches, the single launch at several lags, and the product's
// round (fa_reduce(FA_F_BCAST) on a one-segment gap-padded plan).  Layout
// sizes are the BASELINE layouts' fp32 bytes as one flat tensor (DESIGN §4.4:
// within 5 % of the real layouts).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I include -o tools/laglab \
//         tools/laglab.hip -L feddct_amd -lfedagg -Wl,-rpath,'$ORIGIN/../feddct_amd'
// One JSON line per (layout, variant).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

constexpr int kMaxN = 32;
constexpr int kTile = 2048;  // floats per tile (the product's default width)
struct Args {
  const float* c[kMaxN];
  float* out;
  unsigned* flags;
  unsigned* err;
  int n;
  int ntiles;
  int lag;
  unsigned epoch;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff,
                                           0x00020000);
}
// cache policy bits of the buffer ops: 16 = sc1, 18 = sc1 nt
__device__ __forceinline__ void st_sc1(float* base, int v, f4 x) {
  __builtin_amdgcn_raw_buffer_store_b128(x, rsrc(base), 16 * v, 0, 16);
}
__device__ __forceinline__ void st_sc1nt(float* base, int v, f4 x) {
  __builtin_amdgcn_raw_buffer_store_b128(x, rsrc(base), 16 * v, 0, 18);
}
__device__ __forceinline__ f4 ld_sc1(const float* base, int v) {
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rsrc(base), 16 * v, 0, 16));
}
__device__ __forceinline__ f4 ld_nt(const float* base, int v) {
  return __builtin_nontemporal_load((gcf4*)base + v);
}

// the reduce of tile t: per client 2 x 16-B nt loads per lane behind one
// vmcnt wait (the product's paced rhythm), the sum in client order, / n,
// result stored sc1 (the product's policy)
__device__ __forceinline__ void reduce_tile(const Args& a, int t) {
  const float* base[1];
  const int v0 = threadIdx.x, v1 = threadIdx.x + 256;
  f4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0;
  for (int i = 0; i < a.n; ++i) {
    base[0] = a.c[i] + (size_t)t * kTile;
    const f4 x0 = ld_nt(base[0], v0), x1 = ld_nt(base[0], v1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    s0 += x0;
    s1 += x1;
  }
  const float fn = (float)a.n;
  s0 = f4{s0.x / fn, s0.y / fn, s0.z / fn, s0.w / fn};
  s1 = f4{s1.x / fn, s1.y / fn, s1.z / fn, s1.w / fn};
  float* o = a.out + (size_t)t * kTile;
  st_sc1(o, v0, s0);
  st_sc1(o, v1, s1);
}

// the broadcast of tile t from the result (sc1 loads), every client, sc1 nt
// stores (the product broadcast's policy)
__device__ __forceinline__ void bcast_tile(const Args& a, int t) {
  const float* o = a.out + (size_t)t * kTile;
  const int v0 = threadIdx.x, v1 = threadIdx.x + 256;
  const f4 r0 = ld_sc1(o, v0), r1 = ld_sc1(o, v1);
  for (int i = 0; i < a.n; ++i) {
    float* d = const_cast<float*>(a.c[i]) + (size_t)t * kTile;
    st_sc1nt(d, v0, r0);
    st_sc1nt(d, v1, r1);
  }
}

__global__ __launch_bounds__(256) void reduce_k(Args a) { reduce_tile(a, blockIdx.x); }
__global__ __launch_bounds__(256) void bcast_k(Args a) { bcast_tile(a, blockIdx.x); }

__global__ __launch_bounds__(256) void lagged_k(Args a) {
  const int w = blockIdx.x;
  __shared__ int go;
  if (w < a.ntiles) {
    reduce_tile(a, w);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave
    __syncthreads();
    if (threadIdx.x == 0)
      __builtin_amdgcn_raw_buffer_store_b32(a.epoch, rsrc(a.flags), 4 * w, 0, 16);
  }
  const int j = w - a.lag;
  if (j < 0 || j >= a.ntiles) return;
  if (threadIdx.x == 0) {
    int ok = 0;
    for (int it = 0; it < (1 << 16); ++it) {  // bounded: the launch always drains
      const unsigned f = __builtin_amdgcn_raw_buffer_load_b32(rsrc(a.flags), 4 * j, 0, 16);
      if (f == a.epoch) {
        ok = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (!ok) atomicAdd(a.err, 1u);
    go = ok;
  }
  __syncthreads();
  if (go) bcast_tile(a, j);
}

// split grid with a bounded number of broadcasters (deadlock-free whatever
// the dispatch order: P < the resident slots, so spinning broadcasters can
// never hold every slot a pending reducer needs): blocks T .. T+P-1 each
// broadcast tiles j = b - T, b - T + P, ... in a loop
__global__ __launch_bounds__(256) void persist_k(Args a) {
  const int w = blockIdx.x;
  __shared__ int go;
  if (w < a.ntiles) {
    reduce_tile(a, w);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
      __builtin_amdgcn_raw_buffer_store_b32(a.epoch, rsrc(a.flags), 4 * w, 0, 16);
    return;
  }
  for (int j = w - a.ntiles; j < a.ntiles; j += a.lag) {
    if (threadIdx.x == 0) {
      int ok = 0;
      for (int it = 0; it < (1 << 16); ++it) {
        const unsigned f = __builtin_amdgcn_raw_buffer_load_b32(rsrc(a.flags), 4 * j, 0, 16);
        if (f == a.epoch) {
          ok = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      if (!ok) atomicAdd(a.err, 1u);
      go = ok;
    }
    __syncthreads();
    if (go) bcast_tile(a, j);
    __syncthreads();
  }
}

// r06: the publish deferred by one tile.  R persistent
// reducers (blocks 0..R-1) take tiles w, w + R, ...; after storing tile t's
// result a reducer issues tile t + R's FIRST client's loads, then waits only
// until the older operations — tile t's result stores — have completed
// (vmcnt(2): the two new loads may stay in flight), then a bare workgroup
// barrier (no fence: a workgroup-scope release would wait for the new loads
// too) and one lane publishes tile t's flag sc1.  P broadcasters (blocks R ..
// R+P-1) poll the flags in tile order as persist_k does.  So each reducer
// keeps the chip's reads going while its stores drain, instead of idling for
// the stores' write-through latency (the r05 bisect: +1.4 us per round of
// resident workgroups).
__device__ __forceinline__ void reduce_tile_from(const Args& a, int t, f4 x0, f4 x1) {
  const int v0 = threadIdx.x, v1 = threadIdx.x + 256;
  f4 s0 = x0, s1 = x1;   // client 0's values, loaded ahead
  for (int i = 1; i < a.n; ++i) {
    const float* b = a.c[i] + (size_t)t * kTile;
    const f4 y0 = ld_nt(b, v0), y1 = ld_nt(b, v1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    s0 += y0;
    s1 += y1;
  }
  const float fn = (float)a.n;
  s0 = f4{s0.x / fn, s0.y / fn, s0.z / fn, s0.w / fn};
  s1 = f4{s1.x / fn, s1.y / fn, s1.z / fn, s1.w / fn};
  float* o = a.out + (size_t)t * kTile;
  st_sc1(o, v0, s0);
  st_sc1(o, v1, s1);
}

__global__ __launch_bounds__(256) void defer_k(Args a, int R) {
  const int w = blockIdx.x;
  __shared__ int go;
  const int v0 = threadIdx.x, v1 = threadIdx.x + 256;
  if (w < R) {
    int t = w;
    if (t >= a.ntiles) return;
    f4 x0 = ld_nt(a.c[0] + (size_t)t * kTile, v0), x1 = ld_nt(a.c[0] + (size_t)t * kTile, v1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (;;) {
      reduce_tile_from(a, t, x0, x1);
      const int nt = t + R;
      if (nt < a.ntiles) {
        x0 = ld_nt(a.c[0] + (size_t)nt * kTile, v0);
        x1 = ld_nt(a.c[0] + (size_t)nt * kTile, v1);
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");   // the stores, not the new loads
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      if (threadIdx.x == 0)
        __builtin_amdgcn_raw_buffer_store_b32(a.epoch, rsrc(a.flags), 4 * t, 0, 16);
      if (nt >= a.ntiles) return;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // the next tile's first loads
      t = nt;
    }
  }
  const int P = gridDim.x - R;
  for (int j = w - R; j < a.ntiles; j += P) {
    if (threadIdx.x == 0) {
      int ok = 0;
      for (int it = 0; it < (1 << 16); ++it) {
        const unsigned f = __builtin_amdgcn_raw_buffer_load_b32(rsrc(a.flags), 4 * j, 0, 16);
        if (f == a.epoch) {
          ok = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      if (!ok) atomicAdd(a.err, 1u);
      go = ok;
    }
    __syncthreads();
    if (go) bcast_tile(a, j);
    __syncthreads();
  }
}

__global__ void hash_fill(float* p, int64_t n, uint32_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 0x9E3779B9u ^ seed;
    h ^= h >> 16;
    h *= 0x7feb352du;
    h ^= h >> 15;
    p[i] = ((float)(int32_t)(h >> 8) - 8388608.0f) * (1.0f / 8388608.0f);
  }
}

struct Layout {
  const char* name;
  int n;
  int64_t floats;  // per client (rounded to whole tiles)
  int rot;
};

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 30;
  std::vector<Layout> lays = {{"cfg2", 20, 10972416, 1},
                              {"cfg3", 5, 11017320, 2},
                              {"sf32", 3, 5832256, 6},
                              {"r110", 25, 1249264, 4}};
  for (Layout& L : lays) L.floats = (L.floats + kTile - 1) / kTile * kTile;
  unsigned *flags, *err;
  int64_t maxt = 0;
  for (const Layout& L : lays) maxt = std::max(maxt, L.floats / kTile);
  CK(hipMalloc(&flags, maxt * 4));
  CK(hipMemset(flags, 0, maxt * 4));
  CK(hipMalloc(&err, 4));
  CK(hipMemset(err, 0, 4));
  unsigned epoch = 0;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const Layout& L : lays) {
    const int T = (int)(L.floats / kTile);
    // R sets of N + 1 buckets, each set in one slab
    std::vector<float*> slab(L.rot);
    std::vector<Args> args(L.rot);
    for (int r = 0; r < L.rot; ++r) {
      CK(hipMalloc(&slab[r], (size_t)(L.n + 1) * L.floats * 4));
      hipLaunchKernelGGL(hash_fill, dim3(4096), dim3(256), 0, 0, slab[r],
                         (int64_t)(L.n + 1) * L.floats, 1000u + r);
      Args& a = args[r];
      memset(&a, 0, sizeof a);
      for (int i = 0; i < L.n; ++i) a.c[i] = slab[r] + (size_t)i * L.floats;
      a.out = slab[r] + (size_t)L.n * L.floats;
      a.flags = flags;
      a.err = err;
      a.n = L.n;
      a.ntiles = T;
    }
    CK(hipDeviceSynchronize());
    // the product's round over the same buckets: one gap-padded segment
    fa_plan* plan = nullptr;
    fa_seg seg{0, L.floats};
    FA(fa_plan_create(&seg, 1, L.floats, nullptr, 0, 0, 0, FA_PLAN_GAPS_ARE_PADDING, &plan));
    const int64_t B = L.floats * 4;
    const double red_bytes = (double)(L.n + 1) * B, round_bytes = 2.0 * (L.n + 1) * B;
    struct V {
      std::string name;
      int lag;  // -1: two lab launches; -2: product; -3 reduce only; -4 bcast only
    };
    std::vector<V> vs = {{"lab_reduce", -3},       {"lab_bcast", -4},
                         {"lab_two_launches", -1}, {"product_round", -2},
                         {"lag_split_grid", T},    {"lag_1024", 1024},
                         {"persist_quarter", -12},
                         // r06: the publish deferred by one tile (defer_k),
                         // P = slots / 4, 8, 16 broadcasters
                         {"defer_P4", -20},        {"defer_P8", -21},
                         {"defer_P16", -22}};
    int occ = 0, cus = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(persist_k),
                                                    256, 0));
    int occ_d = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ_d, reinterpret_cast<const void*>(defer_k),
                                                    256, 0));
    occ = std::min(occ, occ_d);
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int slots = occ * cus;
    int ctr = 0;
    auto run = [&](const V& v) {
      Args a = args[ctr++ % L.rot];
      if (v.lag == -3) {
        hipLaunchKernelGGL(reduce_k, dim3(T), dim3(256), 0, 0, a);
      } else if (v.lag == -4) {
        hipLaunchKernelGGL(bcast_k, dim3(T), dim3(256), 0, 0, a);
      } else if (v.lag == -1) {
        hipLaunchKernelGGL(reduce_k, dim3(T), dim3(256), 0, 0, a);
        hipLaunchKernelGGL(bcast_k, dim3(T), dim3(256), 0, 0, a);
      } else if (v.lag == -2) {
        FA(fa_reduce(plan, a.c, nullptr, L.n, nullptr, a.out, nullptr, FA_F_BCAST, nullptr));
      } else if (v.lag <= -20) {
        const int P = std::max(1, slots / (v.lag == -20 ? 4 : v.lag == -21 ? 8 : 16));
        const int R = std::max(1, slots - P);
        a.epoch = ++epoch;
        hipLaunchKernelGGL(defer_k, dim3(R + P), dim3(256), 0, 0, a, R);
      } else if (v.lag <= -10) {
        const int P = std::max(1, std::min(T, v.lag == -10 ? slots - 1
                                              : v.lag == -11 ? slots / 2 : slots / 4));
        a.lag = P;
        a.epoch = ++epoch;
        hipLaunchKernelGGL(persist_k, dim3(T + P), dim3(256), 0, 0, a);
      } else {
        a.lag = std::min(v.lag, T);
        a.epoch = ++epoch;
        hipLaunchKernelGGL(lagged_k, dim3(T + a.lag), dim3(256), 0, 0, a);
      }
    };
    // interleaved passes: each variant timed over `reps` launches per pass
    std::vector<std::vector<float>> ts(vs.size());
    for (int pass = 0; pass < 5; ++pass)
      for (size_t k = 0; k < vs.size(); ++k) {
        for (int i = 0; i < 3; ++i) run(vs[k]);
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < reps; ++i) run(vs[k]);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ts[k].push_back(ms * 1e3f / reps);
      }
    CK(hipGetLastError());
    unsigned herr = 0;
    CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    // bits: the lagged round leaves every client = the lab reduce's result
    bool same = true;
    {
      Args a = args[0];
      hipLaunchKernelGGL(hash_fill, dim3(4096), dim3(256), 0, 0, slab[0],
                         (int64_t)(L.n + 1) * L.floats, 77u);
      hipLaunchKernelGGL(reduce_k, dim3(T), dim3(256), 0, 0, a);
      std::vector<float> want(L.floats), got(L.floats);
      CK(hipMemcpy(want.data(), a.out, B, hipMemcpyDeviceToHost));
      hipLaunchKernelGGL(hash_fill, dim3(4096), dim3(256), 0, 0, slab[0],
                         (int64_t)(L.n + 1) * L.floats, 77u);
      a.lag = std::min(1024, T);
      a.epoch = ++epoch;
      hipLaunchKernelGGL(lagged_k, dim3(T + a.lag), dim3(256), 0, 0, a);
      CK(hipDeviceSynchronize());
      for (int i = 0; i <= L.n && same; ++i) {
        CK(hipMemcpy(got.data(), i < L.n ? a.c[i] : a.out, B, hipMemcpyDeviceToHost));
        same = memcmp(got.data(), want.data(), B) == 0;
      }
      // and the deferred-publish round
      hipLaunchKernelGGL(hash_fill, dim3(4096), dim3(256), 0, 0, slab[0],
                         (int64_t)(L.n + 1) * L.floats, 77u);
      a.epoch = ++epoch;
      const int P = std::max(1, slots / 8);
      hipLaunchKernelGGL(defer_k, dim3(std::max(1, slots - P) + P), dim3(256), 0, 0, a,
                         std::max(1, slots - P));
      CK(hipDeviceSynchronize());
      for (int i = 0; i <= L.n && same; ++i) {
        CK(hipMemcpy(got.data(), i < L.n ? a.c[i] : a.out, B, hipMemcpyDeviceToHost));
        same = memcmp(got.data(), want.data(), B) == 0;
      }
    }
    for (size_t k = 0; k < vs.size(); ++k) {
      std::vector<float> t = ts[k];
      std::sort(t.begin(), t.end());
      const double us = t[t.size() / 2];
      const double bytes = vs[k].lag == -3 ? red_bytes : vs[k].lag == -4 ? red_bytes : round_bytes;
      printf("{\"exp\": \"laglab\", \"layout\": \"%s\", \"n\": %d, \"tiles\": %d, \"variant\": "
             "\"%s\", \"us_median\": %.2f, \"us_min\": %.2f, \"bytes\": %.0f, \"frac\": %.4f, "
             "\"poll_timeouts\": %u, \"lagged_bits_equal\": %s, \"slots\": %d}\n",
             L.name, L.n, T, vs[k].name.c_str(), us, (double)t[0], bytes,
             bytes / (us * 1e-6) / 8e12, herr, same ? "true" : "false", slots);
      fflush(stdout);
    }
    FA(fa_plan_destroy(plan));
    for (float* s : slab) CK(hipFree(s));
  }
  return 0;
}
