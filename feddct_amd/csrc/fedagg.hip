// fedagg.hip — MI355X (gfx950) kernels + C ABI for server-side parameter
// aggregation (the reference's server_aggregate, train_fedavg.py:138-149,
// train_fedprox.py:143-154, train_feddct.py:34-56, train_splitfed.py:34-56).
//
// The work is a bandwidth-bound column reduction: for every element of the
// flat per-client bucket, sum the N client values in exactly the order torch's
// CPU SumKernel uses (cascade / ILP-4 / 8-lane inner, see include/fedagg.h and
// DESIGN.md §2), then divide by N.  Each thread owns its columns and walks the
// clients serially, so the order costs nothing: there is no cross-lane or LDS
// reduction over clients (that would re-associate the sum).  The bucket is cut
// on the host into a tile table; one 256-thread workgroup streams one tile:
// per client, one coalesced 16-B load per lane per vector (1 KiB per wave
// instruction), loads for a batch of clients issued before their adds.
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared
// (no fast-math, no FTZ: the sum must be IEEE round-to-nearest-even, no FMA).

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <queue>
#include <string>
#include <vector>

#include "common.h"

#define FA_VERSION_STR "fedagg 0.1.0 gfx950"

// ---------------------------------------------------------------- errors --
namespace {
thread_local std::string g_last_error;
}  // namespace

int fa::set_err(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

#include "reduce_impl.h"

// the reduce kernels' launchers are instantiated in the fedagg_k*.hip units
FA_K_UNITS(extern)

namespace {
using fa::set_err;
using namespace fa_k;
#define HIP_TRY(expr) FA_HIP_TRY(expr)


// ------------------------------------------------------ small kernels ----
__global__ void div_f32_kernel(const float* __restrict__ x, float d, float* __restrict__ out,
                               int64_t numel) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < numel;
       j += (int64_t)gridDim.x * blockDim.x)
    out[j] = __fdiv_rn(x[j], d);
}
__global__ void div_trunc_i64_kernel(const float* __restrict__ x, float d,
                                     int64_t* __restrict__ out, int64_t numel) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < numel;
       j += (int64_t)gridDim.x * blockDim.x)
    out[j] = (int64_t)__fdiv_rn(x[j], d);
}

// The round's broadcast (train_fedavg.py:148-149) after the reduce: one
// workgroup per (part, group of <= G consecutive clients), groups fastest
// (consecutive blocks), so a part's groups run side by side and its source
// is fetched once.  (r01-r03 forms — one workgroup per tile writing every
// client, 2048-float parts in groups of <= 10, per-client pointer loads
// behind a vmcnt(0) wait, XCD-contiguous groups, the broadcast fused into
// the reduce — measured and dropped; tools/bcastlab.hip,
// tools/writelab.hip, tools/roundlab.hip keep them for A/B.)
__device__ __forceinline__ void bcast_part(uint32_t v, uint32_t groups, uint32_t* p,
                                           uint32_t* g) {
  *p = v / groups;
  *g = v % groups;
}
constexpr int kBcastGroupMax = 24;  // clients per broadcast workgroup

// r04: the round's broadcast with every client pointer a scalar load
// (sptr32) and a group's G stores back to back.  The r02/r03 kernels fetched
// each destination through cptr32, which the compiler serves with an
// `s_waitcnt vmcnt(0)` before every client's stores — a wave's previous
// client's stores had to complete first (ISA checked; vmcnt counts stores on
// CDNA).  Measured on one box (tools/writelab.hip, 20 x 43.9 MB destinations
// in one slab, hashed data, profiles/r04_writelab.jsonl): a lab kernel of
// this shape 127.4 us at U = 1 with all 20 clients in one workgroup (one
// source fetch: 7.23 TB/s of B read + N*B written; a pure write of the same
// N*B 124 us = 7.08 TB/s), 134.3 us at U = 2 in groups of 10, against
// 156.2 us for the r03 product kernel of the U = 2, groups-of-10 shape.
// One workgroup per (part of 1024 floats, group of <= G clients); G is the
// template bound, the host's group size `gsize` <= G.  The int64 bucket is
// one more part.  Destination stores sc1 nt (a buffer store with those
// cache-policy bits: sc1 writes through and drops the line from the XCD's
// L2, so the launch ends with no dirty lines to write back; against nt
// stores r110 47.3 vs 47.9 us, cfg3 79.5 vs 79.8, the rest within 0.3 %).
__device__ __forceinline__ void st_bc(float* base, uint32_t vidx, f4 v) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)(16 * vidx), 0, 18);
}
template <int G>
__global__ __launch_bounds__(kBlock) void bcast_flat2_kernel(ReduceArgs args, uint32_t parts,
                                                             uint32_t groups, uint32_t gsize,
                                                             int64_t f32_numel,
                                                             int64_t i64_numel) {
  (void)args;
  constexpr int U = 1;
  KArgs& a = *(KArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  uint32_t p, g;
  bcast_part(blockIdx.x, groups, &p, &g);
  const int c0 = (int)(g * gsize);
  const int cnt = min(a.n - c0, (int)gsize);
  if (p < parts) {
    const int64_t nv = f32_numel / 4;
    const int64_t vb = (int64_t)p * U * kBlock;  // the part's first float4
    const float* src = a.out32 + 4 * vb;
    f4 r[U];
    if (vb + U * kBlock <= nv) {
      // a whole part (all but possibly the last): no per-lane predicate, and
      // client 0's stores unconditional (cnt >= 1), so the source loads are
      // waited for once there and no later store carries a vmcnt wait (the
      // waitcnt pass merges pending loads across a skipped branch)
#pragma unroll
      for (int u = 0; u < U; ++u) r[u] = ldg4<false>(src, threadIdx.x + u * kBlock);
#pragma unroll
      for (int i = 0; i < G; ++i) {
        if (i == 0 || i < cnt) {
          float* d = sptr32(a, c0 + i) + 4 * vb;
#pragma unroll
          for (int u = 0; u < U; ++u) st_bc(d, threadIdx.x + u * kBlock, r[u]);
        }
      }
    } else {
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        ok[u] = vb + threadIdx.x + u * kBlock < nv;
        if (ok[u]) r[u] = ldg4<false>(src, threadIdx.x + u * kBlock);
      }
      for (int i = 0; i < cnt; ++i) {
        float* d = sptr32(a, c0 + i) + 4 * vb;
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (ok[u]) stg4<true>(d, threadIdx.x + u * kBlock, r[u]);
      }
    }
    // the last part also copies the f32_numel % 4 trailing floats
    if (p == parts - 1 && (int64_t)threadIdx.x < f32_numel - 4 * nv) {
      const float x = a.out32[4 * nv + threadIdx.x];
      for (int i = 0; i < cnt; ++i) sptr32(a, c0 + i)[4 * nv + threadIdx.x] = x;
    }
  } else {
    for (int64_t e = threadIdx.x; e < i64_numel; e += kBlock) {
      const int64_t x = a.out64[e];
      for (int i = 0; i < cnt; ++i) sptr64(a, c0 + i)[e] = x;
    }
  }
}

// The same over the plan's tile table (plans whose segments do not cover
// the bucket, and torch-GPU-order rounds): one workgroup per (tile, group of
// <= G clients); a vector tile's U <= 4 float4 per lane load before the
// group's stores.
template <int G>
__global__ __launch_bounds__(kBlock) void bcast_group2_kernel(ReduceArgs args, uint32_t groups,
                                                              uint32_t gsize) {
  (void)args;
  KArgs& a = *(KArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  uint32_t ti, g;
  bcast_part(blockIdx.x, groups, &ti, &g);
  const int c0 = (int)(g * gsize);
  const int cnt = min(a.n - c0, (int)gsize);
  const Tile t = a.tiles[ti];
  const int kb = t.kind & 0xFF;
  if (kb == K_F32_VEC || kb == K_F32_TGPU_V || kb == K_F32_TGPU_W) {
    const uint32_t nv = (uint32_t)t.count / 4;
    f4 r[4];
    if (nv == 2 * kBlock) {
      // a full 2048-float tile (the default width): unpredicated, client 0's
      // stores unconditional (see bcast_flat2_kernel)
#pragma unroll
      for (int u = 0; u < 2; ++u) r[u] = ldg4<false>(a.out32 + t.start, threadIdx.x + u * kBlock);
#pragma unroll
      for (int i = 0; i < G; ++i) {
        if (i == 0 || i < cnt) {
          float* d = sptr32(a, c0 + i) + t.start;
#pragma unroll
          for (int u = 0; u < 2; ++u) st_bc(d, threadIdx.x + u * kBlock, r[u]);
        }
      }
      return;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t vi = threadIdx.x + u * kBlock;
      if (vi < nv) r[u] = ldg4<false>(a.out32 + t.start, vi);
    }
    for (int i = 0; i < cnt; ++i) {
      float* d = sptr32(a, c0 + i) + t.start;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t vi = threadIdx.x + u * kBlock;
        if (vi < nv) stg4<true>(d, vi, r[u]);
      }
    }
  } else if ((int)threadIdx.x < t.count) {
    int64_t e = t.start + threadIdx.x;
    bool is64 = kind_is64(t.kind);
    if (kb == K_SCALAR_PACKED) {  // a packed column: its element and kind
      const int64_t ent = a.sidx[e];
      e = ent >> 4;
      is64 = kind_is64((int)(ent & 15));
    }
    if (!is64) {
      const float x = a.out32[e];
      for (int i = 0; i < cnt; ++i) sptr32(a, c0 + i)[e] = x;
    } else {
      const int64_t x = a.out64[e];
      for (int i = 0; i < cnt; ++i) sptr64(a, c0 + i)[e] = x;
    }
  }
}

// ---------------------------------------------- torch-ROCm's GPU order ----
// The reduction torch-ROCm itself performs for stack(list, 0).mean(0) on
// device tensors (ATen/native/hip/Reduce.cuh as built into this torch:
// setReduceConfig, thread_reduce_impl, block_y_reduce / block_x_reduce;
// MeanOps: project = acc * factor) — the order of the reference's original
// GPU runs (train_fedavg.py:244-250 place the models on the GPU before
// server_aggregate).  Opt-in (fa_plan_create_order); the default order is
// torch's CPU one.
//   outer (M >= 2): rows split S ways (S = 1 or the block height bh when
//     N >= min(16*bh, 256)); part y takes rows y, y+S, ... round-robin into
//     4 accumulators from +0, combined ((a0+a1)+a2)+a3; the S parts meet in
//     block_y_reduce's halving tree; times the factor.  One element/thread.
//   inner (M == 1): lane l < bw = last_pow2(N) takes rows l, l+bw (the same
//     4-accumulator thread order), then the intra-wave tree with increasing
//     shuffle offsets (ROCm's), lane 0's value times the factor.  One
//     element per wave.
template <class Src, int S>
__device__ __forceinline__ float tgpu_outer(const Src& src, int64_t e, int n) {
  float v[S];
#pragma unroll
  for (int y = 0; y < S; ++y) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int r = y;
    for (; r + 3 * S < n; r += 4 * S) {
      a0 = __fadd_rn(a0, src(r, e));
      a1 = __fadd_rn(a1, src(r + S, e));
      a2 = __fadd_rn(a2, src(r + 2 * S, e));
      a3 = __fadd_rn(a3, src(r + 3 * S, e));
    }
    if (r < n) a0 = __fadd_rn(a0, src(r, e));
    if (r + S < n) a1 = __fadd_rn(a1, src(r + S, e));
    if (r + 2 * S < n) a2 = __fadd_rn(a2, src(r + 2 * S, e));
    v[y] = __fadd_rn(__fadd_rn(__fadd_rn(a0, a1), a2), a3);
  }
#pragma unroll
  for (int off = S / 2; off > 0; off /= 2)
#pragma unroll
    for (int y = 0; y < off; ++y) v[y] = __fadd_rn(v[y], v[y + off]);
  return v[0];
}

// The same order for 4 consecutive elements of one tensor per lane (the
// order depends only on (N, M), so the 4 lanes of a float4 are 4 independent
// copies of it): 16-B non-temporal loads, up to eight rows' loads (two
// round-robin steps) in flight per lane.  Vector adds are per-component IEEE
// adds (no multiply feeds them, so contraction cannot apply).
template <int S>
__device__ __forceinline__ f4 tgpu_outer4(KArgs& a, int64_t start, uint32_t v, int n) {
  f4 val[S];
#pragma unroll
  for (int y = 0; y < S; ++y) {
    // part y's p-th row is y + p*S; row p goes into accumulator p % 4.  Rows
    // are loaded B at a time, then added in row order, so every accumulator
    // still sees its rows in increasing order.
    const f4 z = {0.f, 0.f, 0.f, 0.f};
    f4 acc[4] = {z, z, z, z};
    const int np = (n - y + S - 1) / S;
    constexpr int B = S >= 8 ? 4 : 8;  // rows in flight (register budget of val[S])
    int p = 0;
    for (; p + B <= np; p += B) {
      f4 x[B];
#pragma unroll
      for (int i = 0; i < B; ++i) x[i] = ldg4<true>(cptr32(a, y + (p + i) * S) + start, v);
#pragma unroll
      for (int i = 0; i < B; ++i) acc[i & 3] += x[i];
    }
    if (p < np) {  // p % 4 == 0 here: row p + i goes into accumulator i & 3
      f4 x[B];
#pragma unroll
      for (int i = 0; i < B; ++i)
        if (p + i < np) x[i] = ldg4<true>(cptr32(a, y + (p + i) * S) + start, v);
#pragma unroll
      for (int i = 0; i < B; ++i)
        if (p + i < np) acc[i & 3] += x[i];
    }
    val[y] = ((acc[0] + acc[1]) + acc[2]) + acc[3];
  }
#pragma unroll
  for (int off = S / 2; off > 0; off /= 2)
#pragma unroll
    for (int y = 0; y < off; ++y) val[y] = val[y] + val[y + off];
  return val[0];
}

// S = 1 (no row split: every BASELINE config's tensors) over 2048-element
// tiles, the default kernel's load shape: U = 2 float4 per lane per row, rows
// in batches of B (a multiple of 4, so row b of a batch feeds accumulator
// b & 3 statically), loads through the same pointer accessor as the default
// reduce.  Row p goes into accumulator p % 4 in increasing row order, then
// ((a0 + a1) + a2) + a3 — torch's thread order, per component.
template <int U, int B, bool FULL, int PIPE = 0>
__device__ __forceinline__ void tgpu_wide(KArgs& a, int64_t start, int count, float fac,
                                          bool sum_only) {
  static_assert(B % 4 == 0, "batch must keep the accumulator index static");
  const f4 z = {0.f, 0.f, 0.f, 0.f};
  f4 acc[4][U];
  uint32_t vi[U];
  bool ok[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    vi[u] = threadIdx.x + u * kBlock;
    ok[u] = FULL || (int)(4 * vi[u]) < count;
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k][u] = z;
  }
  const int n = a.n;
  int b0 = 0;
  if constexpr (PIPE != 0 && FULL) {
    // the client loop (as reduce_impl.h pipe2_clients): row b + 1's loads
    // before row b's adds; four rows per pass keep row b's accumulator
    // index (b & 3) static.  The rows' order per accumulator is unchanged.
    // Pointers through scalar loads only (sptr32): cptr32's table arm is a
    // vector load, and the compiler then waited for the current row's data
    // before issuing the next row's loads (ISA read; same process -0.3 ..
    // -0.9 % on cfg2 / cfg3 / cfg5, profiles/r05_ab_lib_tgpu_sptr.jsonl).
    // Same process, r05: cfg2 order 139.9 -> 136.7 us, cfg5 169.9 -> 166.6,
    // N = 17 / 28 -2.8 / -2.5 %, cfg3 and N = 2..16 -1.3 .. +0.1 %, unlike
    // the default kernel's rule: both batch sizes take it
    f4 cur[U], nxt[U];
    {
      const float* p = sptr32(a, 0) + start;
#pragma unroll
      for (int u = 0; u < U; ++u) cur[u] = ldg4<true>(p, vi[u]);
    }
    for (; b0 < n; b0 += 4) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int b = b0 + k;
        if (b < n) {
          if (b + 1 < n) {
            const float* p = sptr32(a, b + 1) + start;
#pragma unroll
            for (int u = 0; u < U; ++u) nxt[u] = ldg4<true>(p, vi[u]);
          }
#pragma unroll
          for (int u = 0; u < U; ++u) {
            acc[k][u] += cur[u];
            cur[u] = nxt[u];
          }
        }
      }
    }
  }
  for (; b0 + B <= n; b0 += B) {
    f4 x[B][U];
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const float* p = cptr32(a, b0 + b) + start;
#pragma unroll
      for (int u = 0; u < U; ++u)
        x[b][u] = (FULL || ok[u]) ? ldg4<true>(p, vi[u]) : z;
    }
#pragma unroll
    for (int b = 0; b < B; ++b)
#pragma unroll
      for (int u = 0; u < U; ++u) acc[b & 3][u] += x[b][u];
  }
  if (b0 < n) {  // b0 % 4 == 0 here
    const int nb = n - b0;
    f4 x[B][U];
#pragma unroll
    for (int b = 0; b < B; ++b) {
      if (b < nb) {
        const float* p = cptr32(a, b0 + b) + start;
  #pragma unroll
        for (int u = 0; u < U; ++u)
          x[b][u] = (FULL || ok[u]) ? ldg4<true>(p, vi[u]) : z;
      }
    }
#pragma unroll
    for (int b = 0; b < B; ++b)
      if (b < nb)
#pragma unroll
        for (int u = 0; u < U; ++u) acc[b & 3][u] += x[b][u];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (!FULL && !ok[u]) continue;
    f4 r = ((acc[0][u] + acc[1][u]) + acc[2][u]) + acc[3][u];
    if (!sum_only)
      r = f4{__fmul_rn(r.x, fac), __fmul_rn(r.y, fac), __fmul_rn(r.z, fac), __fmul_rn(r.w, fac)};
    st_out<5>(a.out32, start, vi[u], r);  // sc1: see reduce_impl.h st_out
  }
}

// S = 1 or 2 (torch's row split for N >= 32 over the large tensors) over
// 2048-element tiles with the client loop: rows in slot order, row r into
// part r % S and that part's accumulator (r / S) % 4 — part y's p-th row
// (y + S p) into accumulator p % 4, as tgpu_outer4<S> — then each part's
// ((a0 + a1) + a2) + a3 and, for S = 2, part 0 + part 1.  4 S rows per pass
// keep the accumulator index static.  The S = 2 launch runs its S = 1 tiles
// through it too (tgpu_kernel<1>).
// FA_TGPU_LOOP_DEPTH: rows in flight ahead of the add (1: row b + 1's loads
// before row b's adds).  2 and 3 (same 130 VGPRs, three workgroups per CU)
// measured within +-0.4 % of 1 at N = 32 / 48 / 64 (r06,
// profiles/r06_ab_lib_tgpu_runs.jsonl): the launch is not short of loads in
// flight.
#ifndef FA_TGPU_LOOP_DEPTH
#define FA_TGPU_LOOP_DEPTH 1
#endif
template <int U, int S, bool FULL>
__device__ __forceinline__ void tgpu_wide_loop(KArgs& a, int64_t start, int count, float fac,
                                               bool sum_only) {
  static_assert(S == 1 || S == 2, "row split of the wide loop");
  constexpr int R = 4 * S;
  constexpr int D = FA_TGPU_LOOP_DEPTH;
  const f4 z = {0.f, 0.f, 0.f, 0.f};
  f4 acc[R][U];
  uint32_t vi[U];
  bool ok[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    vi[u] = threadIdx.x + u * kBlock;
    ok[u] = FULL || (int)(4 * vi[u]) < count;
#pragma unroll
    for (int k = 0; k < R; ++k) acc[k][u] = z;
  }
  const int n = a.n;
  f4 row[D + 1][U];   // row[0]: the row being added; row[d]: d rows ahead
#pragma unroll
  for (int d = 0; d < D; ++d) {
    if (d < n) {
      const float* p = sptr32(a, d) + start;
#pragma unroll
      for (int u = 0; u < U; ++u) row[d][u] = (FULL || ok[u]) ? ldg4<true>(p, vi[u]) : z;
    }
  }
  for (int b0 = 0; b0 < n; b0 += R) {
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int b = b0 + k;
      if (b < n) {
        if (b + D < n) {
          const float* p = sptr32(a, b + D) + start;
#pragma unroll
          for (int u = 0; u < U; ++u) row[D][u] = (FULL || ok[u]) ? ldg4<true>(p, vi[u]) : z;
        }
        const int ai = (k % S) * 4 + ((k / S) & 3);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          acc[ai][u] += row[0][u];
#pragma unroll
          for (int d = 0; d < D; ++d) row[d][u] = row[d + 1][u];
        }
      }
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (!FULL && !ok[u]) continue;
    f4 r = ((acc[0][u] + acc[1][u]) + acc[2][u]) + acc[3][u];
    if constexpr (S == 2) r = r + (((acc[4][u] + acc[5][u]) + acc[6][u]) + acc[7][u]);
    if (!sum_only)
      r = f4{__fmul_rn(r.x, fac), __fmul_rn(r.y, fac), __fmul_rn(r.z, fac), __fmul_rn(r.w, fac)};
    st_out<5>(a.out32, start, vi[u], r);
  }
}

// lane value of the inner order; the wave then runs the shuffle tree
template <class Src>
__device__ __forceinline__ float tgpu_inner(const Src& src, int64_t e, int n, int bw, int lane) {
  float a0 = 0.f, a1 = 0.f;
  if (lane < n) a0 = __fadd_rn(a0, src(lane, e));
  if (lane + bw < n) a1 = __fadd_rn(a1, src(lane + bw, e));
  float v = __fadd_rn(__fadd_rn(__fadd_rn(a0, a1), 0.f), 0.f);
  for (int off = 1; off < bw; off <<= 1) v = __fadd_rn(v, __shfl_down(v, off, 64));
  return v;
}

// M == 1 with N >= 128: torch vectorises along the input (setReduceConfig's
// "vectorize along input": dim0 = N / 4 >= 32), so the block is bw =
// last_pow2(N / 4) (at most 512) threads; thread x sums the 4-element
// vectors x, x+bw, ... into 4 accumulators, one per vector component, then
// the <= 3 trailing rows N - N%4 + x into accumulator 0, and combines
// ((v0 + v1) + v2) + v3 (input_vectorized_thread_reduce_impl).  The threads
// meet in block_x_reduce: the shared-memory halving tree for offsets bw/2
// down to 64, then the intra-wave tree with increasing offsets.  One wave per
// element here: lane l plays threads l + 64 j (j < bw / 64), and the halving
// over j is the shared-memory tree.
template <class Src>
__device__ __forceinline__ float tgpu_inner_vec(const Src& src, int64_t e, int n, int bw,
                                                int lane) {
  const int J = bw >= 64 ? bw / 64 : 1;
  const int tail = n - n % 4;
  float t[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    t[j] = 0.f;
    const int x = lane + 64 * j;
    if (j >= J || x >= bw) continue;
    float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;
    for (int q = x; 4 * q + 3 < n; q += bw) {
      v0 = __fadd_rn(v0, src(4 * q, e));
      v1 = __fadd_rn(v1, src(4 * q + 1, e));
      v2 = __fadd_rn(v2, src(4 * q + 2, e));
      v3 = __fadd_rn(v3, src(4 * q + 3, e));
    }
    if (tail + x < n) v0 = __fadd_rn(v0, src(tail + x, e));
    t[j] = __fadd_rn(__fadd_rn(__fadd_rn(v0, v1), v2), v3);
  }
  if (J >= 8) {
#pragma unroll
    for (int j = 0; j < 4; ++j) t[j] = __fadd_rn(t[j], t[j + 4]);
  }
  if (J >= 4) {
#pragma unroll
    for (int j = 0; j < 2; ++j) t[j] = __fadd_rn(t[j], t[j + 2]);
  }
  if (J >= 2) t[0] = __fadd_rn(t[0], t[1]);
  float v = t[0];
  const int dx = bw >= 64 ? 64 : bw;
  for (int off = 1; off < dx; off <<= 1) v = __fadd_rn(v, __shfl_down(v, off, 64));
  return v;
}

// A V tile (4 elements per lane) and a scalar tile (one element per lane)
// of row split S.
template <int S>
__device__ __forceinline__ void tgpu_v_tile(KArgs& a, const Tile& t, float fac, bool sum_only) {
  const uint32_t v = threadIdx.x;
  if ((int)(v * 4) >= t.count) return;
  f4 r = tgpu_outer4<S>(a, t.start, v, a.n);
  if (!sum_only)
    r = f4{__fmul_rn(r.x, fac), __fmul_rn(r.y, fac), __fmul_rn(r.z, fac), __fmul_rn(r.w, fac)};
  st_out<5>(a.out32, t.start, v, r);
}
template <int S>
__device__ __forceinline__ void tgpu_scalar_tile(KArgs& a, const Tile& t, float fac,
                                                 bool sum_only) {
  const int j = threadIdx.x;
  if (j >= t.count) return;
  const int64_t e = t.start + j;
  if ((t.kind & 0xFF) == K_F32_TGPU) {
    const float s = tgpu_outer<SrcF32, S>(SrcF32{a, false}, e, a.n);
    a.out32[e] = sum_only ? s : __fmul_rn(s, fac);
  } else {
    a.out64[e] = (int64_t)__fmul_rn(tgpu_outer<SrcI64, S>(SrcI64{a}, e, a.n), fac);
  }
}

// One instantiation per row split S = 1 << LS (the plan groups its tiles by
// S and launches each group): a single S per kernel keeps the register
// budget of the parts' values to that S (a runtime switch over S = 1..16 in
// one kernel needed 300 VGPRs and spilled).  Inner tiles (M == 1) ride in
// the LS = 0 group; their own field is the lane count exponent.  r05: when
// the S = 2 group is the largest (N >= 32 over the large tensors) the S = 1
// and S = 4 tiles and the inner tiles ride in its launch (their own S from
// the tile's field; fa_plan_create_order), so the small groups cost no
// launch of their own.
template <int LS, int WB = 16, int PIPE = 0>
__global__ __launch_bounds__(kBlock) void tgpu_kernel(ReduceArgs args) {
  (void)args;
  constexpr int S = 1 << LS;
  KArgs& a = *(KArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  const Tile t = a.tiles[blockIdx.x];
  const float fac = a.tfac[blockIdx.x];
  const int base = t.kind & 0xFF, ls = (t.kind >> 8) & 0xFF;
  const bool sum_only = a.flags & FA_F_SUM_ONLY;
  const int n = a.n;
  const bool inner = base == K_F32_TGPU_IN || base == K_I64_TGPU_IN;
  if constexpr (LS == 0) {
    if (base == K_F32_TGPU_W) {
      if (t.count == 8 * kBlock) tgpu_wide<2, WB, true, PIPE>(a, t.start, t.count, fac, sum_only);
      else tgpu_wide<2, WB, false>(a, t.start, t.count, fac, sum_only);
      return;
    }
  }
  if constexpr (LS == 1) {
    if (base == K_F32_TGPU_W) {
      if (ls == 0) {
        if (t.count == 8 * kBlock) tgpu_wide_loop<2, 1, true>(a, t.start, t.count, fac, sum_only);
        else tgpu_wide_loop<2, 1, false>(a, t.start, t.count, fac, sum_only);
      } else {
        if (t.count == 8 * kBlock) tgpu_wide_loop<2, 2, true>(a, t.start, t.count, fac, sum_only);
        else tgpu_wide_loop<2, 2, false>(a, t.start, t.count, fac, sum_only);
      }
      return;
    }
    if (!inner && ls != 1) {  // a rider: S = 1 or 4
      if (base == K_F32_TGPU_V) tgpu_v_tile<4>(a, t, fac, sum_only);
      else if (ls == 0) tgpu_scalar_tile<1>(a, t, fac, sum_only);
      else tgpu_scalar_tile<4>(a, t, fac, sum_only);
      return;
    }
  }
  if (base == K_F32_TGPU_V) {
    tgpu_v_tile<S>(a, t, fac, sum_only);
    return;
  }
  if (base == K_F32_TGPU || base == K_I64_TGPU) {
    tgpu_scalar_tile<S>(a, t, fac, sum_only);
    return;
  }
  // inner: one element per wave
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (w >= t.count) return;
  const int64_t e = t.start + w;
  const int bw = 1 << ls;
  const bool vec = (t.kind >> 16) & 1;   // N >= 128: input-vectorised form
  if (base == K_F32_TGPU_IN) {
    const float s = vec ? tgpu_inner_vec(SrcF32{a, false}, e, n, bw, lane)
                        : tgpu_inner(SrcF32{a, false}, e, n, bw, lane);
    if (lane == 0) a.out32[e] = sum_only ? s : __fmul_rn(s, fac);
  } else {
    const float s = vec ? tgpu_inner_vec(SrcI64{a}, e, n, bw, lane)
                        : tgpu_inner(SrcI64{a}, e, n, bw, lane);
    if (lane == 0) a.out64[e] = (int64_t)__fmul_rn(s, fac);
  }
}

// fa_broadcast_f32: up to kBcastInline destinations per launch, pointers in
// the kernel arguments (more destinations: consecutive launches, each
// re-reading the source)
constexpr int kBcastInline = 256;
struct BcastArgs {
  const float* src;
  int n;
  float* dst[kBcastInline];
};
// One workgroup per (2048-float part, group of <= kBcastGroupMax
// destinations), groups fastest; the last part also copies the numel % 4
// tail.
__global__ __launch_bounds__(kBlock) void bcast_kernel(BcastArgs a, int64_t numel,
                                                       uint32_t parts, uint32_t groups,
                                                       uint32_t gsize) {
  const int64_t nv = numel / 4;
  const uint32_t total = parts * groups;
  for (uint32_t v = blockIdx.x; v < total; v += gridDim.x) {
    uint32_t p, g;
    bcast_part(v, groups, &p, &g);
    const int c0 = (int)(g * gsize);
    const int c1 = min(a.n, c0 + (int)gsize);
    const int64_t v0 = (int64_t)p * 2 * kBlock + threadIdx.x, v1 = v0 + kBlock;
    f4 r0 = {0.f, 0.f, 0.f, 0.f}, r1 = r0;
    if (v0 < nv) r0 = ld4<false>(a.src + 4 * v0);
    if (v1 < nv) r1 = ld4<false>(a.src + 4 * v1);
    for (int c = c0; c < c1; ++c) {
      if (v0 < nv) st4<true>(a.dst[c] + 4 * v0, r0);
      if (v1 < nv) st4<true>(a.dst[c] + 4 * v1, r1);
    }
    if (p == parts - 1 && threadIdx.x < numel - 4 * nv)
      for (int c = c0; c < c1; ++c) a.dst[c][4 * nv + threadIdx.x] = a.src[4 * nv + threadIdx.x];
  }
}

// Streaming copy (the roofline's calibration): one 16-B non-temporal load and
// store per lane, one 256-lane tile per workgroup, no loop — the fastest of
// the copy forms measured (tools/archive/copylab.hip, profiles/r02_copylab.jsonl:
// 6.62-6.66 TB/s on 1 GiB, against 5.0 TB/s for a grid-stride loop with one
// float4 per lane and 4.4-5.2 TB/s with four in flight per lane).
__global__ __launch_bounds__(kBlock) void copy_kernel(const float* __restrict__ src,
                                                      float* __restrict__ dst, int64_t numel) {
  const int64_t nv = numel / 4;
  const int64_t v = blockIdx.x * (int64_t)kBlock + threadIdx.x;
  if (v < nv) st4<true>(dst + 4 * v, ld4<true>(src + 4 * v));
  if (blockIdx.x == 0 && threadIdx.x < numel - 4 * nv)
    dst[4 * nv + threadIdx.x] = src[4 * nv + threadIdx.x];
}

// Read-only streaming probe: per workgroup sum of its float4s (calibrates the
// read-bandwidth ceiling the reduce kernel, 95 % reads, is measured against).
__global__ __launch_bounds__(kBlock) void read_probe_kernel(const float* __restrict__ src,
                                                            int64_t nv, float* __restrict__ out) {
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
  int64_t v = blockIdx.x * (int64_t)kBlock + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (; v + 3 * stride < nv; v += 4 * stride) {
    const f4 a = ld4<true>(src + 4 * v), b = ld4<true>(src + 4 * (v + stride));
    const f4 c = ld4<true>(src + 4 * (v + 2 * stride)), d = ld4<true>(src + 4 * (v + 3 * stride));
    acc += (a + b) + (c + d);
  }
  for (; v < nv; v += stride) acc += ld4<true>(src + 4 * v);
  float s = acc.x + acc.y + acc.z + acc.w;
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(out + blockIdx.x, s);
}

// Write-only probe in the round broadcast's own shape (fa_write_probe_f32,
// r04): one workgroup per (1024-float part, group of <= kBcastGroupMax
// destinations, as bcast_flat2_kernel), one 16-B store per lane per
// destination with the broadcast's sc1 nt policy, the
// values non-zero and non-repeating (an integer hash of the element index
// and `seed`, computed in registers: nothing is read).  Zero-filled or
// constant stores are no write ceiling on this chip.
__device__ __forceinline__ float probe_val(uint32_t i) {
  i ^= i >> 16;
  i *= 0x7feb352du;
  i ^= i >> 15;
  i *= 0x846ca68bu;
  i ^= i >> 16;
  return __fmul_rn((float)(int32_t)((i >> 8) | 1u) - 8388608.0f, 1.0f / 8388608.0f);
}
__global__ __launch_bounds__(kBlock) void write_probe_kernel(BcastArgs a, int64_t numel,
                                                             uint32_t parts, uint32_t groups,
                                                             uint32_t gsize, uint32_t seed) {
  uint32_t p, g;
  bcast_part(blockIdx.x, groups, &p, &g);
  const int c0 = (int)(g * gsize);
  const int c1 = min(a.n, c0 + (int)gsize);
  const int64_t nv = numel / 4;
  const int64_t v = (int64_t)p * kBlock + threadIdx.x;
  if (v >= nv) return;
  const uint32_t b = (uint32_t)(4 * v) ^ seed;
  const f4 x = {probe_val(b), probe_val(b + 1), probe_val(b + 2), probe_val(b + 3)};
  // based at the part's start, as bcast_flat2_kernel: the buffer offset is
  // 32-bit, so a bucket-based offset would wrap past 2^28 float4s
  for (int c = c0; c < c1; ++c) st_bc(a.dst[c] + 4 * (int64_t)p * kBlock, threadIdx.x, x);
}

// Read-only probe in the reduce's own shape (grid = 0 in fa_read_probe_f32):
// one tile of 2 x 1024 floats per workgroup, 2 independent 16-B
// non-temporal loads per lane, no loop, and no store unless the tile's sum
// hits a sentinel value (so nothing but the reads reaches HBM).  The lab's
// fastest read-only form (tools/archive/bwlab.hip one_stream_read_only_U2: 7.0-7.1
// TB/s, profiles/r01_bwlab.jsonl) — the read ceiling of a box, which the
// reduce (95 % reads) is compared with; the grid-stride form above runs
// ~10 % slower.
__global__ __launch_bounds__(kBlock) void read_tile_kernel(const float* __restrict__ src,
                                                           int64_t nv, float* __restrict__ out) {
  const int64_t v0 = blockIdx.x * (int64_t)(2 * kBlock) + threadIdx.x, v1 = v0 + kBlock;
  f4 a = f4{0.f, 0.f, 0.f, 0.f}, b = a;
  if (v0 < nv) a = ld4<true>(src + 4 * v0);
  if (v1 < nv) b = ld4<true>(src + 4 * v1);
  const f4 s = a + b;
  if (s.x == 1234.5f && s.y == -1.0f && s.z == 7.0f) out[threadIdx.x] = s.w;
}

// ------------------------------------------- synthetic state (synth.py) --
__device__ __forceinline__ uint64_t hash64(uint64_t seed, uint64_t idx) {
  uint64_t z = seed * 0x9E3779B97F4A7C15ull + idx * 0xD1B54A32D192ED03ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ float sym_unit(uint64_t h) {
  const int64_t v = (int64_t)(h >> 40) - (1 << 23);
  return __fmul_rn((float)v, 1.0f / 8388608.0f);
}
constexpr uint64_t kBaseSeed = 7, kClientSeed0 = 1000;
constexpr int kKeyShift = 36;

__global__ void synth_f32_kernel(float* dst, int64_t numel, int key, int client,
                                 float mu, float sigma, float dsig, int mode) {
  const uint64_t kb = (uint64_t)key << kKeyShift;
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < numel;
       j += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t idx = kb | (uint64_t)j;
    const uint64_t hc = hash64(kClientSeed0 + client, idx);
    float x;
    if (mode == 1) {
      const int ex = (int)((hc >> 8) % 41ull) - 20;
      x = __fmul_rn(sym_unit(hc), ldexpf(1.0f, ex));
    } else {
      const float base = __fadd_rn(mu, __fmul_rn(sigma, sym_unit(hash64(kBaseSeed, idx))));
      x = __fadd_rn(base, __fmul_rn(dsig, sym_unit(hc)));
    }
    dst[j] = x;
  }
}
__global__ void synth_i64_kernel(int64_t* dst, int64_t numel, int key, int client, int mode) {
  const uint64_t kb = (uint64_t)key << kKeyShift;
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < numel;
       j += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t hc = hash64(kClientSeed0 + client, kb | (uint64_t)j);
    dst[j] = mode == 1 ? (int64_t)(hc % (1ull << 26)) - (1ll << 25)
                       : (int64_t)(19 * 5) + (int64_t)(hc % 7ull);
  }
}

// ------------------------------------------------------------ host plan --
int grid_for(int64_t work, int per_block) {
  int64_t g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > 256 * 16) g = 256 * 16;
  return (int)g;
}

}  // namespace

struct fa_plan {
  int device = 0;
  Tile* d_tiles = nullptr;
  fa_plan_info info{};
  int vec_u = kDefaultU;
  // auto plans (tile_elems == 0) also carry a 1024-float table, used for
  // unweighted reductions over >= 64 clients (tools/tune.py sweep)
  Tile* d_tiles_alt = nullptr;
  int ntiles_alt = 0;
  int nscalar_alt = 0;
  // the device tables' own counts: their scalar tiles are packed (r03,
  // K_SCALAR_PACKED; info.* keep the host view of the layout's tiles)
  int nt_dev = 0, ns_dev = 0, nt_alt_dev = 0, ns_alt_dev = 0;
  int64_t* d_sidx = nullptr;  // packed scalar columns: (element << 4) | kind, -1 unused
  int64_t sidx_alt_off = 0;   // the alt table's region of d_sidx
  // balanced tables (r03): the vector tiles re-cut so that packed + vector
  // tiles fill whole rounds of `slots` resident workgroups (balance_vec);
  // their packed tiles are the main table's (same scalar index region)
  struct BalTable {
    int u = 0, slots = 0;
    int batch = 16;  // clients per load batch of the kernel it was cut for
    Tile* d = nullptr;
    int nt = 0;
    bool alt = false;  // cut from the alt (1024-float) table: its scalar index region
  };
  std::vector<BalTable> bal;
  unsigned flags = 0;
  bool has32 = false;  // the tile table touches the fp32 bucket
  bool has64 = false;  // ... the int64 bucket
  int order = FA_ORDER_TORCH_CPU;
  int order_n = 0;        // FA_ORDER_TORCH_GPU: the client count it was cut for
  int tgpu_batch = 16;    // ... rows per load batch of its S = 1 tiles (8 for N < 16)
  size_t tgpu_s2_lds = 0;  // ... the S = 2 launch's LDS reservation (tgpu_s2_lds)
  float* d_fac = nullptr; // ... and its per-tile mean factors
  int tg_lo[6] = {0, 0, 0, 0, 0, 0};  // ... tiles grouped by row split S = 1..16
  // cut from a segment list with FA_PLAN_GAPS_ARE_PADDING: every byte of
  // the buckets is a tensor's or padding, so the broadcast may copy them flat
  bool flat_bcast = false;
};

namespace {
void set_kinds(fa_plan* p, const std::vector<Tile>& t) {
  for (const Tile& x : t) {
    if (x.kind >= K_I64_CASC) p->has64 = true;
    else p->has32 = true;
  }
}
}  // namespace

namespace {

inline int64_t body_len(int64_t M) {
  if (M >= 8) return (M / 32) * 32;
  if (M >= 2) return (M / 4) * 4;
  return 0;
}

int check_segs(const fa_seg* s, int ns, int64_t numel, const char* what,
               std::vector<fa_seg>* sorted) {
  if (ns < 0 || (ns > 0 && !s)) return set_err(FA_E_INVAL, "%s: bad segment array", what);
  sorted->assign(s, s + ns);
  std::stable_sort(sorted->begin(), sorted->end(),
                   [](const fa_seg& x, const fa_seg& y) { return x.offset < y.offset; });
  int64_t end = 0;
  for (const fa_seg& g : *sorted) {
    if (g.offset < 0 || g.numel < 0 || g.offset + g.numel > numel)
      return set_err(FA_E_INVAL, "%s: segment [%lld,+%lld) outside bucket of %lld", what,
                     (long long)g.offset, (long long)g.numel, (long long)numel);
    if (g.numel > 0 && g.offset < end)
      return set_err(FA_E_INVAL, "%s: overlapping segments at %lld", what, (long long)g.offset);
    if (g.numel > 0) end = g.offset + g.numel;
  }
  return FA_OK;
}

// May the broadcast copy the buckets flat?  Only when the caller declared the
// gaps padding (FA_PLAN_GAPS_ARE_PADDING) AND the segments, with that
// padding, cover the whole bucket: no gap (leading, between, trailing) of
// `pad` elements or more, i.e. no room for a key the plan does not own.  A
// plan over some of a layout's keys (a column chunk) keeps the tile-table
// broadcast, which writes its own tiles only.
bool covers_with_padding(const std::vector<fa_seg>& s, int64_t numel, int64_t pad) {
  int64_t pos = 0;
  for (const fa_seg& g : s) {
    if (g.numel == 0) continue;
    if (g.offset - pos >= pad) return false;
    pos = g.offset + g.numel;
  }
  return numel - pos < pad;
}

bool flat_bcast_ok(unsigned flags, const std::vector<fa_seg>& s32, int64_t f32_numel,
                   const std::vector<fa_seg>& s64, int64_t i64_numel) {
  return (flags & FA_PLAN_GAPS_ARE_PADDING) && covers_with_padding(s32, f32_numel, 64) &&
         covers_with_padding(s64, i64_numel, 1);
}

// Every element belongs to at most one tile: two tiles over one element would
// race two summation orders (and two stores) into the same output.
int check_disjoint(std::vector<Tile> t, const char* who) {
  std::sort(t.begin(), t.end(), [](const Tile& x, const Tile& y) {
    const bool x64 = kind_is64(x.kind), y64 = kind_is64(y.kind);
    return x64 != y64 ? y64 : x.start < y.start;
  });
  for (size_t i = 1; i < t.size(); ++i)
    if (kind_is64(t[i - 1].kind) == kind_is64(t[i].kind) &&
        t[i - 1].start + t[i - 1].count > t[i].start)
      return set_err(FA_E_INVAL, "%s: tiles overlap at %s element %lld", who,
                     kind_is64(t[i].kind) ? "int64" : "fp32", (long long)t[i].start);
  return FA_OK;
}

void push_scalar(std::vector<Tile>* t, int64_t start, int64_t count, int kind) {
  for (int64_t c = 0; c < count; c += kBlock)
    t->push_back(Tile{start + c, (int32_t)std::min<int64_t>(kBlock, count - c), kind});
}

int build_tiles(const std::vector<fa_seg>& s32, const std::vector<fa_seg>& s64, int tile_elems,
                unsigned flags, std::vector<Tile>* out, fa_plan_info* info) {
  std::vector<Tile> vec, tail;
  // Maximal runs of cascade-order elements, 4-aligned (vectorisable).
  int64_t run_s = -1, run_e = -1;
  auto flush = [&]() {
    if (run_s < 0) return;
    for (int64_t c = run_s; c < run_e; c += tile_elems)
      vec.push_back(Tile{c, (int32_t)std::min<int64_t>(tile_elems, run_e - c), K_F32_VEC});
    info->cascade_elems += run_e - run_s;
    run_s = run_e = -1;
  };
  for (const fa_seg& g : s32) {
    const int64_t M = g.numel;
    if (M == 0) continue;
    if (M == 1) {
      // the scalar breaks the run: a later aligned segment must not extend
      // the open vector run across this element (it would be covered twice)
      flush();
      push_scalar(&tail, g.offset, 1, K_F32_INNER);
      info->tail_elems += 1;
      continue;
    }
    const int64_t b = body_len(M);
    if (b > 0) {
      if (g.offset % 4 == 0) {
        const bool extend = run_s >= 0 && (run_e == g.offset ||
                                           ((flags & FA_PLAN_GAPS_ARE_PADDING) && run_e <= g.offset));
        if (!extend) flush();
        if (run_s < 0) run_s = g.offset;
        run_e = g.offset + b;
      } else {
        flush();
        push_scalar(&tail, g.offset, b, K_F32_CASC_S);
        info->tail_elems += b;
      }
    }
    if (b < M) {
      flush();  // the tail breaks the run
      push_scalar(&tail, g.offset + b, M - b, K_F32_ILP4);
      info->tail_elems += M - b;
    }
  }
  flush();
  for (const fa_seg& g : s64) {
    const int64_t M = g.numel;
    if (M == 0) continue;
    if (M == 1) { push_scalar(&tail, g.offset, 1, K_I64_INNER); continue; }
    const int64_t b = body_len(M);
    if (b) push_scalar(&tail, g.offset, b, K_I64_CASC);
    if (b < M) push_scalar(&tail, g.offset + b, M - b, K_I64_ILP4);
  }
  std::vector<Tile> all(vec);
  all.insert(all.end(), tail.begin(), tail.end());
  const int rc = check_disjoint(all, "tile planner");
  if (rc) return rc;
  // Scalar tiles first: their few long-latency workgroups start early and
  // finish under the vector stream instead of trailing it.
  out->clear();
  out->insert(out->end(), tail.begin(), tail.end());
  out->insert(out->end(), vec.begin(), vec.end());
  info->ntiles = (int32_t)out->size();
  info->ntiles_cascade = (int32_t)vec.size();
  info->ntiles_tail = (int32_t)tail.size();
  return FA_OK;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// Clients per load batch of the reduce kernel a call runs (launch_reduce).
// r06: the 16-client kernels (three workgroups per CU) from 12 clients, with
// the client loop (pipe_rule): same process (profiles/r06_ab_lib_mid_n.jsonl)
// N = 12 / 14 / 16 -1.8 / -2.7 / -0.3 %, weighted N = 12 -1.4 / -1.5 % (C10 /
// C100); at N = 10 +1.0 %, so below 12 the 8-client kernels stay.
#ifndef FA_B16_MIN
#define FA_B16_MIN 12
#endif
int pick_batch(int n, int vec_u, unsigned pflags) {
  const int b = (pflags & FA_PLAN_TUNE_BATCH8)    ? 8
                : (pflags & FA_PLAN_TUNE_BATCH16) ? 16 : (n < FA_B16_MIN ? 8 : 16);
  return (vec_u == 4 && b == 16) ? 8 : b;  // no 16-client kernels at U = 4
}

// ------------------------------------------------------ balanced tables --
// One workgroup per tile: a launch of T equal tiles over `slots` resident
// workgroups (CUs x workgroups per CU) runs ceil(T / slots) rounds, and a
// part-filled round costs nearly a whole one while the launch is only one or
// two rounds long — measured r03 on one fp32 tensor of T x 2048 floats
// (tools/archive/exp_batch_cross.py, profiles/r03_exp_batch_cross*.jsonl), N = 20,
// 16-client kernel on 768 slots: 384 tiles 16.1 us, re-cut to 768 13.4 us;
// 768 tiles 22.7 us; 1,024 tiles 33.5 us, on the 8-client kernel's 1,280
// slots (one round) 28.3 us.  Past two rounds the tail is a small share and
// a re-cut (smaller, partial tiles) costs more than it saves: cfg4 weighted
// 144.2 vs 142.0 us, cfg5 185.5 vs 181.4 us, cfg3 43.7 vs 43.5 us re-cut vs
// plain (profiles/r03_exp_tune_balance.jsonl).  So a call of N >= 16
// clients whose plain table (a) part-fills ONE round of the 16-client kernel
// runs a table re-cut to fill it, (b) needs two rounds of the 16-client
// kernel but one of the 8-client kernel runs the 8-client kernel (resnet110sl
// sf4 N = 25, 923 tiles: 23.0 vs 26.3 us plain, 23.9 re-cut), (c) spills a
// few tiles past its last full round: the tail split below (split_tail), and
// (d) runs the plain table otherwise.  N < 16 (8-client kernel already) always runs
// plain: at N = 5 a re-cut is no gain (384 tiles 7.8 vs 9.0 us).
constexpr double kKeepFill = 0.97;  // the round at least this full: keep the plain table
constexpr int64_t kMinTile = 256;   // never cut vector tiles below this (elements)

// Resident workgroups of the reduce kernel (U, B, deep, weighted) on device
// `dev`, queried once per process (0: unknown -> the plain table).
int kernel_slots(int dev, int u, int b, bool deep, bool w) {
  static std::mutex mu;
  static std::map<int64_t, int> cache;
  const int64_t key = ((((int64_t)dev * 8 + u) * 32 + b) * 2 + deep) * 2 + w;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int occ = 0;
  switch (u * 100 + b) {
    case 108: occ = occupancy_u<1, 8>(deep, w); break;
    case 116: occ = occupancy_u<1, 16>(deep, w); break;
    case 208: occ = occupancy_u<2, 8>(deep, w); break;
    case 216: occ = occupancy_u<2, 16>(deep, w); break;
    case 408: occ = occupancy_u<4, 8>(deep, w); break;
    default: break;
  }
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 0;
  const int slots = occ > 0 && cus > 0 ? occ * cus : 0;
  cache[key] = slots;
  return slots;
}

// The slot count a plain (non-chain) reduce call runs on; 0 for a plan that
// launches its tiles as given (FA_PLAN_TUNE_NO_BALANCE).
int call_slots(int dev, int n, int vec_u, bool w, unsigned pflags) {
  if (pflags & FA_PLAN_TUNE_NO_BALANCE) return 0;
  return kernel_slots(dev, vec_u, pick_batch(n, vec_u, pflags), n >= 256, w);
}

// Case (b) above: the batch a plain call of n clients runs with, given the
// plain table's tile count — 8 instead of 16 when that turns two rounds into
// one.  Explicit batch tuning flags and grid-shaping flags keep their batch.
int round_batch(int dev, int n, int vec_u, bool w, unsigned pflags, int ntiles) {
  const int b = pick_batch(n, vec_u, pflags);
  if (b != 16 || (pflags & (FA_PLAN_TUNE_BATCH16 | FA_PLAN_TUNE_NO_BALANCE))) return b;
  const int s16 = kernel_slots(dev, vec_u, 16, n >= 256, w);
  const int s8 = kernel_slots(dev, vec_u, 8, n >= 256, w);
  return (s16 > 0 && s8 > s16 && ntiles > s16 && ntiles <= s8) ? 8 : 16;
}

// A multi-round launch whose last round holds only r << slots tiles (r03
// session 4, tools/archive/exp_round_quant.py, profiles/r03_exp_round_quant.jsonl):
// those r tiles run alone, latency-bound, ~7-8 us after the last full round
// at N = 20 — cfg2's layout plus 16 / 18 / 25 extra 2048-float tiles (r = 1
// / 3 / 10 past 7 rounds of 768) reads 139.0 / 142.3 / 143.9 us against
// 136.3 us at 6.99 rounds, while 300 extra tiles cost only 146.4 us.  So the
// LAST slots - r vector tiles are split in halves (64-element lines): the
// table then fills exactly k rounds, its last round made of half tiles, and
// every earlier tile keeps the full width (re-cutting the whole table
// instead was slower, see above).  Same process, weighted, split vs plain
// (profiles/r03_exp_round_quant_tail_split*.jsonl): r = 10 137.9 vs 143.8
// us, r = 85 139.5 vs 144.0, r = 135 141.5 vs 144.8, r = 285 144.8 vs 146.3,
// r = 335 145.4 vs 147.6 — a gain at every r measured, up to 0.44 slots,
// so it is applied for 0 < r <= 0.44 slots (r03 applied it up to
// slots / 2, past the measured range).  A tile too small to halve (< 2 *
// kMinTile / 2 elements: ragged ends of runs) is left whole, so such a table
// may end up a few tiles short of exactly k rounds; the bits never change.
constexpr int64_t kTailMaxPct = 44;
std::vector<Tile> split_tail(const std::vector<Tile>& tiles, int64_t r, int slots) {
  if (r <= 0 || r * 100 > kTailMaxPct * (int64_t)slots) return {};
  std::vector<Tile> vec;
  for (const Tile& x : tiles)
    if (x.kind == K_F32_VEC) vec.push_back(x);
  const int64_t m = slots - r;  // tiles to split
  if ((int64_t)vec.size() < m) return {};
  std::vector<Tile> out;
  out.reserve(vec.size() + (size_t)m);
  const size_t first = vec.size() - (size_t)m;
  for (size_t i = 0; i < vec.size(); ++i) {
    const Tile& x = vec[i];
    const int64_t h = ((int64_t)x.count / 2) & ~(int64_t)63;
    if (i < first || h < kMinTile / 2) {
      out.push_back(x);
      continue;
    }
    out.push_back(Tile{x.start, (int32_t)h, K_F32_VEC});
    out.push_back(Tile{x.start + h, (int32_t)(x.count - h), K_F32_VEC});
  }
  return out;
}

// The vector tiles of `tiles` (cut at cmax elements), re-cut for `slots`:
// only when they part-fill a single round (k = 1: slots - nscalar vector tiles),
// handed out run by run (a run = adjacent vector tiles) to the run whose
// tiles are largest, boundaries on 64-element (256 B) lines, no tile above
// cmax or (when split further) below kMinTile.  Empty: keep the plain table.
std::vector<Tile> balance_vec(const std::vector<Tile>& tiles, int cmax, int nscalar, int slots,
                              bool tail_only = false) {
  std::vector<std::pair<int64_t, int64_t>> runs;  // [start, end)
  int64_t t0 = 0;
  for (const Tile& x : tiles) {
    if (x.kind != K_F32_VEC) continue;
    ++t0;
    if (!runs.empty() && runs.back().second == x.start) runs.back().second += x.count;
    else runs.emplace_back(x.start, x.start + x.count);
  }
  if (t0 == 0 || slots <= 0) return {};
  const int64_t have = t0 + nscalar;
  const int64_t k = (have + slots - 1) / slots;
  if (k > 1) return split_tail(tiles, have - (k - 1) * slots, slots);
  if (tail_only || (double)have >= kKeepFill * (double)(k * slots)) return {};
  const int64_t target = k * slots - nscalar;
  std::vector<int64_t> m(runs.size());
  std::priority_queue<std::pair<double, size_t>> pq;  // (tile size, run), largest first
  int64_t total = 0;
  for (size_t r = 0; r < runs.size(); ++r) {
    const int64_t len = runs[r].second - runs[r].first;
    m[r] = (len + cmax - 1) / cmax;
    total += m[r];
    pq.emplace((double)len / (double)m[r], r);
  }
  while (total < target && !pq.empty()) {
    const size_t r = pq.top().second;
    pq.pop();
    const int64_t len = runs[r].second - runs[r].first;
    if ((double)len / (double)(m[r] + 1) < (double)kMinTile) break;  // every run is as small
    ++m[r];
    ++total;
    pq.emplace((double)len / (double)m[r], r);
  }
  if (total == t0) return {};
  std::vector<Tile> out;
  out.reserve((size_t)total + 16);
  for (size_t r = 0; r < runs.size(); ++r) {
    const int64_t s = runs[r].first, e = runs[r].second, len = e - s;
    for (int64_t mm = m[r];; ++mm) {
      const size_t mark = out.size();
      int64_t prev = s;
      bool ok = true;
      for (int64_t j = 1; j <= mm; ++j) {
        const int64_t b = j == mm ? e : ((s + j * len / mm) & ~(int64_t)63);
        if (b <= prev) continue;  // (a boundary rounded onto the previous one)
        if (b - prev > cmax) {
          ok = false;
          break;
        }
        out.push_back(Tile{prev, (int32_t)(b - prev), K_F32_VEC});
        prev = b;
      }
      if (ok) break;
      out.resize(mark);  // rounding pushed a tile past cmax: one more tile
    }
  }
  return out;
}

hipError_t launch_chain(const ReduceArgs& a, int ntiles, int vec_u, hipStream_t st) {
  const bool deep = a.n_total >= 256;
  const bool w = a.flags & 0x100u;
  if (vec_u == 1) return launch_chain_ub<1, 8>(a, ntiles, deep, w, st);
  if (vec_u == 4) return launch_chain_ub<4, 8>(a, ntiles, deep, w, st);
  if (w || a.n < 16) return launch_chain_ub<2, 8>(a, ntiles, deep, w, st);
  return launch_chain_ub<2, 16>(a, ntiles, deep, w, st);
}


hipError_t launch_reduce(const ReduceArgs& a, int ntiles, int vec_u, unsigned pflags,
                         hipStream_t st, int batch = 0, int pipe = 0) {
  // DEEP (n >= 256): cascade levels 2-3 and the constant-space table loads.
  // Weighted reductions take the mean's 16-client batches too since the
  // batch's weights are read once up front (r02 sweep, same box: weighted
  // U2xB16 140.5 us vs U2xB8 143.3 us, unweighted 143.0 us).
  const bool deep = a.n >= 256;
  const bool w = a.flags & 0x100u;  // internal: weighted
  const int b = batch > 0 ? batch : pick_batch(a.n, vec_u, pflags);
  switch (vec_u) {
    case 1: return b == 16 ? launch_u<1, 16>(a, ntiles, deep, w, 0, st)
                           : launch_u<1, 8>(a, ntiles, deep, w, 0, st);
    case 4: return launch_u<4, 8>(a, ntiles, deep, w, 0, st);
    default: return b == 16 ? launch_u<2, 16>(a, ntiles, deep, w, pipe, st)
                            : launch_u<2, 8>(a, ntiles, deep, w, pipe, st);
  }
}

// Stateless-API plan cache, keyed by device + layout.
std::mutex g_cache_mu;
std::map<std::string, fa_plan*> g_cache;

int cached_plan(const fa_seg* s32, int n32, int64_t numel32, const fa_seg* s64, int n64,
                int64_t numel64, fa_plan** out) {
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  std::string key((const char*)&dev, sizeof dev);
  key.append((const char*)&numel32, sizeof numel32);
  key.append((const char*)&numel64, sizeof numel64);
  key.append((const char*)&n32, sizeof n32);
  if (n32 > 0) key.append((const char*)s32, sizeof(fa_seg) * n32);
  if (n64 > 0) key.append((const char*)s64, sizeof(fa_seg) * n64);
  std::lock_guard<std::mutex> lk(g_cache_mu);
  auto it = g_cache.find(key);
  if (it != g_cache.end()) { *out = it->second; return FA_OK; }
  fa_plan* p = nullptr;
  int rc = fa_plan_create(s32, n32, numel32, s64, n64, numel64, 0, 0, &p);
  if (rc) return rc;
  g_cache[key] = p;
  *out = p;
  return FA_OK;
}

}  // namespace

// =================================================================== ABI ==
namespace {
// Client pointer tables (N > kInline) come from a private stream-ordered pool
// whose freed blocks are reused only by the stream that freed them: cross-
// stream reuse (opportunistic or internal-dependency) is switched off, so a
// table still read by a kernel on one stream can never be handed to another
// stream (the executor in fedcomm.hip drives two).  The loopback test of the
// multi-rank rounds saw payload corruption with cross-stream frees on the
// default pool (tests/loopback/loopccl.hip).
hipError_t table_alloc(void** p, size_t bytes, hipStream_t st) {
  static std::mutex mu;
  static std::map<int, hipMemPool_t> pools;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  hipMemPool_t pool = nullptr;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = pools.find(dev);
    if (it != pools.end()) {
      pool = it->second;
    } else {
      hipMemPoolProps props{};
      props.allocType = hipMemAllocationTypePinned;
      props.location.type = hipMemLocationTypeDevice;
      props.location.id = dev;
      e = hipMemPoolCreate(&pool, &props);
      if (e != hipSuccess) return e;
      int off = 0;
      for (hipMemPoolAttr a : {hipMemPoolReuseFollowEventDependencies,
                               hipMemPoolReuseAllowOpportunistic,
                               hipMemPoolReuseAllowInternalDependencies})
        if ((e = hipMemPoolSetAttribute(pool, a, &off)) != hipSuccess) return e;
      uint64_t keep = UINT64_MAX;  // keep freed blocks for the next round
      if ((e = hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep)) != hipSuccess)
        return e;
      pools[dev] = pool;
    }
  }
  return hipMallocFromPoolAsync(p, bytes, pool, st);
}

// A caller-owned pointer table (fa_reduce_tab) is written by kernels whose
// arguments carry the words by value: no host memcpy, no allocation, so the
// call can be captured into a graph and replayed (the table's contents are
// the kernel arguments, frozen at capture).
constexpr int kFillWords = 400;
struct FillArgs {
  uint64_t* dst;
  int count;
  uint64_t w[kFillWords];
};
__global__ void table_fill_kernel(FillArgs a) {
  for (int i = threadIdx.x; i < a.count; i += blockDim.x) a.dst[i] = a.w[i];
}
hipError_t table_fill(void* dst, const std::vector<char>& host, hipStream_t st) {
  const size_t words = (host.size() + 7) / 8;
  for (size_t w0 = 0; w0 < words; w0 += kFillWords) {
    FillArgs f;
    memset(&f, 0, sizeof f);
    f.dst = (uint64_t*)dst + w0;
    f.count = (int)std::min<size_t>(kFillWords, words - w0);
    memcpy(f.w, host.data() + w0 * 8, std::min<size_t>(f.count * 8, host.size() - w0 * 8));
    hipLaunchKernelGGL(table_fill_kernel, dim3(1), dim3(256), 0, st, f);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
}  // namespace

namespace {
// The device form of a host tile table: its scalar tiles' columns, sorted by
// kind (a wave then mostly runs one order), packed kPackCols per K_SCALAR_PACKED
// tile with their entries appended to `sidx`; the vector tiles follow
// unchanged.  *nscalar = packed tiles (they lead the table, as the scalar
// tiles did).
std::vector<Tile> pack_scalar(const std::vector<Tile>& t, std::vector<int64_t>* sidx,
                              int* nscalar, unsigned flags) {
  (void)flags;
  const int pack = kPackCols;
  std::vector<std::pair<int, int64_t>> cols;
  std::vector<Tile> vec;
  for (const Tile& x : t) {
    if (x.kind == K_F32_VEC) {
      vec.push_back(x);
      continue;
    }
    for (int32_t c = 0; c < x.count; ++c) cols.emplace_back(x.kind, x.start + c);
  }
  std::stable_sort(cols.begin(), cols.end(),
                   [](const std::pair<int, int64_t>& u, const std::pair<int, int64_t>& v) {
                     return u.first < v.first;
                   });
  std::vector<Tile> out;
  for (size_t c = 0; c < cols.size(); c += pack) {
    const int cnt = (int)std::min<size_t>(pack, cols.size() - c);
    out.push_back(Tile{(int64_t)sidx->size(), cnt, K_SCALAR_PACKED});
    for (int i = 0; i < kPackCols; ++i)
      sidx->push_back(i < cnt ? (cols[c + i].second << 4) | cols[c + i].first : -1);
  }
  *nscalar = (int)out.size();
  out.insert(out.end(), vec.begin(), vec.end());
  return out;
}

// Upload a CPU-order plan's device tables (main + optional alt) and the
// shared scalar index.
hipError_t upload_tables(fa_plan* p, const std::vector<Tile>& tiles,
                         const std::vector<Tile>& alt) {
  std::vector<int64_t> sidx;
  const std::vector<Tile> dm = pack_scalar(tiles, &sidx, &p->ns_dev, p->flags);
  p->nt_dev = (int)dm.size();
  std::vector<Tile> da;
  if (!alt.empty()) {
    // the alt table's packed tiles index their own region of the scalar
    // index (the kernels get its base: tile k's entries at base + k * kPackCols)
    std::vector<int64_t> sa;
    da = pack_scalar(alt, &sa, &p->ns_alt_dev, p->flags);
    p->sidx_alt_off = (int64_t)sidx.size();
    sidx.insert(sidx.end(), sa.begin(), sa.end());
    p->nt_alt_dev = (int)da.size();
  }
  hipError_t e = hipSuccess;
  if (!dm.empty()) {
    e = hipMalloc(&p->d_tiles, dm.size() * sizeof(Tile));
    if (e == hipSuccess)
      e = hipMemcpy(p->d_tiles, dm.data(), dm.size() * sizeof(Tile), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess && !da.empty()) {
    e = hipMalloc(&p->d_tiles_alt, da.size() * sizeof(Tile));
    if (e == hipSuccess)
      e = hipMemcpy(p->d_tiles_alt, da.data(), da.size() * sizeof(Tile), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess && !sidx.empty()) {
    e = hipMalloc(&p->d_sidx, sidx.size() * sizeof(int64_t));
    if (e == hipSuccess)
      e = hipMemcpy(p->d_sidx, sidx.data(), sidx.size() * sizeof(int64_t), hipMemcpyHostToDevice);
  }
  // balanced tables for every slot count a call on this plan may run on
  // (main table: the 16-client kernels, deep or not, weighted or not; the
  // alt table: its unweighted 16-client kernels)
  if (e != hipSuccess || (p->flags & FA_PLAN_TUNE_NO_BALANCE)) return e;
  struct Req {
    int u, slots, batch;
    const std::vector<Tile>* host;
    const std::vector<Tile>* dev;
    int ns;
  };
  std::vector<Req> reqs;
  auto want = [&](int u, int slots, int batch, const std::vector<Tile>* host,
                  const std::vector<Tile>* dev, int ns) {
    if (slots <= 0) return;
    for (const Req& q : reqs)
      if (q.u == u && q.slots == slots && q.batch == batch && q.dev == dev) return;
    reqs.push_back(Req{u, slots, batch, host, dev, ns});
  };
  // the 16-client kernels' calls: the whole rule; the calls of N < 16 (the
  // 8-client kernels): the tail split only (tools/archive/exp_tail_small_n.py: N = 5
  // / 8 / 12, 1.1-2.9 us per launch; a one-round re-cut is no gain there)
  for (int deep = 0; deep < 2; ++deep)
    for (int w = 0; w < 2; ++w) {
      if (pick_batch(16, p->vec_u, p->flags) == 16)
        want(p->vec_u, kernel_slots(p->device, p->vec_u, 16, deep != 0, w != 0), 16, &tiles,
             &dm, p->ns_dev);
      const int b8 = pick_batch(8, p->vec_u, p->flags);
      if (deep == 0)
        want(p->vec_u, kernel_slots(p->device, p->vec_u, b8, false, w != 0), b8, &tiles, &dm,
             p->ns_dev);
    }
  if (!da.empty())
    for (int deep = 0; deep < 2; ++deep)
      want(1, kernel_slots(p->device, 1, pick_batch(64, 1, p->flags), deep != 0, false),
           pick_batch(64, 1, p->flags), &alt, &da, p->ns_alt_dev);
  for (const Req& q : reqs) {
    const std::vector<Tile> v =
        balance_vec(*q.host, q.u * 4 * kBlock, q.ns, q.slots, q.batch < 16);
    if (v.empty()) continue;
    std::vector<Tile> t(q.dev->begin(), q.dev->begin() + q.ns);  // the packed tiles lead
    t.insert(t.end(), v.begin(), v.end());
    fa_plan::BalTable b;
    b.u = q.u;
    b.slots = q.slots;
    b.batch = q.batch;
    b.nt = (int)t.size();
    b.alt = q.dev == &da;
    e = hipMalloc(&b.d, t.size() * sizeof(Tile));
    if (e == hipSuccess)
      e = hipMemcpy(b.d, t.data(), t.size() * sizeof(Tile), hipMemcpyHostToDevice);
    if (b.d) p->bal.push_back(b);
    if (e != hipSuccess) return e;
  }
  return e;
}
}  // namespace

extern "C" {

const char* fa_version(void) { return FA_VERSION_STR; }
const char* fa_last_error(void) { return g_last_error.c_str(); }

int fa_plan_create(const fa_seg* seg32, int nseg32, int64_t f32_numel, const fa_seg* seg64,
                   int nseg64, int64_t i64_numel, int tile_elems, unsigned flags,
                   fa_plan** out) {
  if (!out) return set_err(FA_E_INVAL, "fa_plan_create: out is NULL");
  *out = nullptr;
  if (flags & ~(unsigned)FA_PLAN_FLAGS_KNOWN)
    return set_err(FA_E_INVAL, "fa_plan_create: unknown flag bits 0x%x (removed tuning flags?)",
                   flags & ~(unsigned)FA_PLAN_FLAGS_KNOWN);
  if (f32_numel < 0 || i64_numel < 0) return set_err(FA_E_INVAL, "negative bucket size");
  const bool autosel = tile_elems == 0;
  if (tile_elems == 0) tile_elems = 4 * kBlock * kDefaultU;
  if (tile_elems != 4 * kBlock && tile_elems != 8 * kBlock && tile_elems != 16 * kBlock)
    return set_err(FA_E_INVAL, "tile_elems must be 1024, 2048 or 4096 (got %d)", tile_elems);
  std::vector<fa_seg> s32, s64;
  int rc = check_segs(seg32, nseg32, f32_numel, "fp32", &s32);
  if (rc) return rc;
  rc = check_segs(seg64, nseg64, i64_numel, "int64", &s64);
  if (rc) return rc;
  fa_plan* p = new fa_plan();
  p->info.f32_numel = f32_numel;
  p->info.i64_numel = i64_numel;
  p->info.tile_elems = tile_elems;
  p->vec_u = tile_elems / (4 * kBlock);
  p->flags = flags;
  p->flat_bcast = flat_bcast_ok(flags, s32, f32_numel, s64, i64_numel);
  std::vector<Tile> tiles, alt;
  rc = build_tiles(s32, s64, tile_elems, flags, &tiles, &p->info);
  if (rc) {
    delete p;
    return rc;
  }
  set_kinds(p, tiles);
  if (autosel) {
    fa_plan_info ia{};
    rc = build_tiles(s32, s64, 4 * kBlock, flags, &alt, &ia);
    if (rc) {
      delete p;
      return rc;
    }
    p->ntiles_alt = (int)alt.size();
    p->nscalar_alt = ia.ntiles_tail;
  }
  hipError_t e = hipGetDevice(&p->device);
  if (e == hipSuccess) e = upload_tables(p, tiles, alt);
  if (e != hipSuccess) {
    (void)fa_plan_destroy(p);  // frees whatever was uploaded
    return set_err(FA_E_HIP, "fa_plan_create: %s", hipGetErrorString(e));
  }
  *out = p;
  return FA_OK;
}

int fa_torch_gpu_config(int n, int64_t m, int* stride) {
  if (n < 2 || m < 1) return 0;
  auto last_pow2 = [](int64_t v) {
    int64_t p = 1;
    while (p * 2 <= v) p *= 2;
    return p;
  };
  auto div_up = [](int64_t a, int64_t b) { return (a + b - 1) / b; };
  int64_t S;
  if (m == 1) {
    // a 0-dim key stacked to [N]: lanes over the N values; from N >= 128 on
    // torch vectorises the input (tgpu_inner_vec), and N <= FA_MAX_CLIENTS
    // keeps values per thread below the cross-block threshold (N / 512 <
    // 256).  `stride` is the block width.
    S = n < 128 ? last_pow2(n) : std::min<int64_t>(last_pow2(n / 4), 512);
  } else {
    // setReduceConfig, "vectorize along output" ([N, M] reduced over dim 0,
    // iter.ndim() == 2), set_block_dimension with MAX_NUM_THREADS 512
    const int64_t ovs = m % 4 == 0 ? 4 : (m % 2 == 0 ? 2 : 1);
    const int64_t mnt = 512 / ovs, dim0 = m / ovs;
    const int64_t d0 = dim0 < mnt ? last_pow2(dim0) : mnt;
    const int64_t d1 = n < mnt ? last_pow2(n) : mnt;
    const int64_t bw0 = std::min<int64_t>(d0, 64);
    const int64_t bh = std::min<int64_t>(d1, mnt / bw0);
    const int64_t bw = std::min<int64_t>(d0, mnt / bh);
    const bool split = n >= std::min<int64_t>(bh * 16, 256);
    S = split ? bh : 1;
    if (S > 16) return 0;  // kernel limit (tgpu_kernel<LS>, LS <= 4)
    const int64_t vpt = div_up(n, S);
    if (split && vpt >= 256) {
      // the cross-block ("global") split: only when the output grid is
      // small against the target grid (kTorchNumCU CUs; max threads per CU
      // 256 for a 2-D iterator, the device's own for a single block —
      // ROCm's `uses_a_single_block` reads grid.x == 1)
      const int64_t grid = div_up(dim0, bw);
      const int64_t tpm = grid == 1 ? kTorchMaxThreadsPerCU : 256;
      const int64_t target = kTorchNumCU * (tpm / (bw * bh));
      if (grid <= target) {
        int64_t c = std::max(std::min(div_up(target, grid), div_up(vpt, 16)), div_up(vpt, 256));
        if (c > kTorchNumCU) c = kTorchNumCU;
        else if (c > div_up(kTorchNumCU, 2)) c = div_up(kTorchNumCU, 2);
        else if (c < 16) c = 1;
        if (c > 1) return 0;  // global_reduce: not restated
      }
    }
  }
  if (stride) *stride = (int)S;
  return 1;
}

namespace {
// Resident workgroups of tgpu_kernel<0> (the S = 1 group's launch) on `dev`,
// queried once per process (0: unknown).
int tgpu_slots(int dev, int batch) {
  static std::mutex mu;
  static std::map<int, int> cache;
  std::lock_guard<std::mutex> lk(mu);
  const int key = dev * 2 + (batch == 8);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int occ = 0, cus = 0;
  const hipError_t e =
      batch == 8 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, tgpu_kernel<0, 8, 1>, kBlock, 0)
                 : hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, tgpu_kernel<0, 16, 1>, kBlock, 0);
  if (e != hipSuccess) occ = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 0;
  return cache[key] = occ > 0 && cus > 0 ? occ * cus : 0;
}

// The dynamic LDS the S = 2 launch reserves (and never uses) so that at most
// kTgpuS2Resident of its workgroups share a CU.  Measured r05
// (profiles/r05_ab_lib_tgpu_s2.jsonl, same process) on the kernel before its
// S = 4 riders (100 VGPRs, five per CU): three per CU 3-4 % faster than five,
// two 10 % slower (a reservation of exactly a third of the CU's LDS admitted
// only two: the allocation rounds up).  With the riders' paths it holds 130
// VGPRs, three per CU by itself; the reservation keeps the measured count if
// that changes.  The default reduce's 8-client kernels capped the same way
// ran 20-25 % slower (r05_ab_lib_occupancy_cap.jsonl).  0 when the device
// cannot say.
#ifndef FA_TGPU_S2_RESIDENT
#define FA_TGPU_S2_RESIDENT 3
#endif
constexpr int kTgpuS2Resident = FA_TGPU_S2_RESIDENT;
size_t tgpu_s2_lds(int dev) {
  static std::mutex mu;
  static std::map<int, size_t> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  int per_cu = 0;
  if (hipDeviceGetAttribute(&per_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) !=
      hipSuccess)
    per_cu = 0;
  // per_cu / (resident + 1/2): the allocation granularity may round the
  // request up, and per_cu / resident exactly would then admit one fewer
  return cache[dev] =
             per_cu > 0 ? (size_t)(2 * (int64_t)per_cu / (2 * kTgpuS2Resident + 1)) & ~(size_t)1023
                        : 0;
}

// Rows per load batch of the S = 1 tiles for a plan cut for n clients: 8
// below 16 clients (as the default reduce's 8-client kernel; the 8-row form
// holds 102 VGPRs against 164, five workgroups per CU against three):
// measured r04 (tools/tgpu_speed.py, profiles/r04_tgpu_batch.jsonl) cfg3
// N = 5 40.8 vs 45.8 us, but cfg2 N = 20 146.7 vs 140.9, cfg5 N = 24 173.9
// vs 167.3.
// r06: from 10 clients the 16-row form (three workgroups per CU) since the
// client loop: same process (profiles/r06_ab_lib_tgpu_batch.jsonl) N = 10 / 12
// -1.7 / -2.5 %, N = 2 / 5 / sf32 (N = 3) +1.3 / +3.8 / +1.6 %.
#ifndef FA_TGPU_B16_MIN
#define FA_TGPU_B16_MIN 10
#endif
int tgpu_batch_for(int n) { return n < FA_TGPU_B16_MIN ? 8 : 16; }

// The tail round of launch group gi (the S = 1 group, r04; the default
// plan's split_tail, §4.3 of DESIGN.md):
// its scalar and inner tiles first; and when its T tiles spill
// 0 < r <= 0.44 slots past k - 1 full rounds, the last slots - r wide tiles
// are halved (64-element lines), so the table fills exactly k rounds with a
// last round of half tiles instead of r tiles running alone.  cfg2 at N = 20: ~5,400 tiles on
// 768 slots = 7.03 rounds.  Per-column arithmetic: the bits never change.
void tgpu_split_tail(std::vector<Tile>* t, std::vector<float>* fac, int lo[6], int gi, int slots) {
  const int64_t T = lo[gi + 1] - lo[gi];
  const int64_t k = slots > 0 ? (T + slots - 1) / slots : 0;
  const int64_t r = T - (k - 1) * slots;
  // m: the wide tiles to halve (0: none; the group is still reordered so
  // its scalar and inner tiles — the int64 keys' one-wave latency chains —
  // run in the first round, as the default plan places its scalar tiles)
  const int64_t m = (k > 1 && r > 0 && r * 100 <= kTailMaxPct * (int64_t)slots) ? slots - r : 0;
  std::vector<Tile> nw, wd;
  std::vector<float> fnw, fwd;
  for (int64_t i = lo[gi]; i < lo[gi + 1]; ++i) {
    const bool w = ((*t)[i].kind & 0xFF) == K_F32_TGPU_W;
    (w ? wd : nw).push_back((*t)[i]);
    (w ? fwd : fnw).push_back((*fac)[i]);
  }
  std::vector<Tile> g(t->begin(), t->begin() + lo[gi]);
  std::vector<float> f(fac->begin(), fac->begin() + lo[gi]);
  g.insert(g.end(), nw.begin(), nw.end());
  f.insert(f.end(), fnw.begin(), fnw.end());
  const size_t first = (int64_t)wd.size() < m ? wd.size() : wd.size() - (size_t)m;
  for (size_t j = 0; j < wd.size(); ++j) {
    const Tile& x = wd[j];
    const int64_t h = ((int64_t)x.count / 2) & ~(int64_t)63;
    if (j < first || h < 64) {
      g.push_back(x);
      f.push_back(fwd[j]);
      continue;
    }
    g.push_back(Tile{x.start, (int32_t)h, x.kind});
    g.push_back(Tile{x.start + h, (int32_t)(x.count - h), x.kind});
    f.push_back(fwd[j]);
    f.push_back(fwd[j]);
  }
  const int add = (int)((int64_t)g.size() - lo[gi] - T);
  g.insert(g.end(), t->begin() + lo[gi + 1], t->end());
  f.insert(f.end(), fac->begin() + lo[gi + 1], fac->end());
  t->swap(g);
  fac->swap(f);
  for (int i = gi + 1; i < 6; ++i) lo[i] += add;
}
}  // namespace

int fa_plan_create_order(const fa_seg* seg32, int nseg32, int64_t f32_numel, const fa_seg* seg64,
                         int nseg64, int64_t i64_numel, int n, int order, unsigned flags,
                         fa_plan** out) {
  if (flags & ~(unsigned)FA_PLAN_FLAGS_KNOWN)
    return set_err(FA_E_INVAL, "fa_plan_create_order: unknown flag bits 0x%x",
                   flags & ~(unsigned)FA_PLAN_FLAGS_KNOWN);
  if (order == FA_ORDER_TORCH_CPU)
    return fa_plan_create(seg32, nseg32, f32_numel, seg64, nseg64, i64_numel, 0, flags, out);
  if (!out) return set_err(FA_E_INVAL, "fa_plan_create_order: out is NULL");
  *out = nullptr;
  if (order != FA_ORDER_TORCH_GPU)
    return set_err(FA_E_INVAL, "fa_plan_create_order: order %d", order);
  if (n < 2 || n > FA_MAX_CLIENTS)
    return set_err(FA_E_RANGE, "fa_plan_create_order: n=%d outside 2..%d", n, FA_MAX_CLIENTS);
  std::vector<fa_seg> s32, s64;
  int rc = check_segs(seg32, nseg32, f32_numel, "fp32", &s32);
  if (rc) return rc;
  rc = check_segs(seg64, nseg64, i64_numel, "int64", &s64);
  if (rc) return rc;
  std::vector<Tile> t;
  std::vector<float> fac;
  std::vector<int> order_groups_tmp;
  // Wide S = 1 runs.  With S = 1 every M > 1 tensor has the same per-element
  // order (row p into accumulator p % 4, then ((a0 + a1) + a2) + a3), so the
  // 4-aligned bodies of adjacent such tensors with the same factor (bit for
  // bit) share one run cut into 2048-element tiles across key boundaries, as
  // the default plan's vector runs are: no partial tile per key (cfg2: 5432
  // -> ~5381 tiles).  Gaps join a run only when declared padding.
  // r06: runs of every row split S (the order depends on (N, S) only, as for
  // S = 1; S <= 2 in 2048-element W tiles, S >= 4 in 1024-element V tiles),
  // and adjacent one-element keys of one kind packed a wave each into one
  // tile: wrn16_8 C10 at N = 32 / 48 / 64 then fills 7 rounds of the S = 2
  // launch's 768 slots (5,372 / 5,372 / 5,370 tiles) where per-key tiles
  // spilled past them (5,417 / 5,417 / 5,432)
  int64_t run_s = -1, run_e = -1;
  int run_ls = 0;
  float run_f = 0.f;
  auto flush = [&]() {
    if (run_s < 0) return;
    const int64_t te = run_ls <= 1 ? 8 * kBlock : 4 * kBlock;
    const int kind = (run_ls <= 1 ? K_F32_TGPU_W : K_F32_TGPU_V) | (run_ls << 8);
    for (int64_t c = run_s; c < run_e; c += te) {
      t.push_back(Tile{c, (int32_t)std::min<int64_t>(te, run_e - c), kind});
      fac.push_back(run_f);
    }
    run_s = run_e = -1;
  };
  for (int pass = 0; pass < 2; ++pass) {
    flush();
    for (const fa_seg& g : pass ? s64 : s32) {
      if (g.numel == 0) continue;
      int S = 1;
      if (!fa_torch_gpu_config(n, g.numel, &S))
        return set_err(FA_E_RANGE,
                       "torch-GPU order: N=%d over a %lld-element tensor is outside the "
                       "restated configurations (cross-block split)", n, (long long)g.numel);
      int ls = 0;
      while ((1 << ls) < S) ++ls;
      // torch's factor: float(num_outputs) / numel, in float
      const float f = (float)g.numel / (float)((int64_t)n * g.numel);
      if (g.numel == 1) {
        flush();
        const int vec = n >= 128 ? 1 << 16 : 0;  // input-vectorised (tgpu_inner_vec)
        const int kind = (pass ? K_I64_TGPU_IN : K_F32_TGPU_IN) | (ls << 8) | vec;
        if (!t.empty() && t.back().kind == kind && fac.back() == f &&
            t.back().start + t.back().count == g.offset && t.back().count < kBlock / 64) {
          t.back().count++;   // one wave per element (tgpu_kernel's inner form)
          continue;
        }
        t.push_back(Tile{g.offset, 1, kind});
        fac.push_back(f);
        continue;
      }
      auto scalar = [&](int64_t lo, int64_t hi) {
        for (int64_t c = lo; c < hi; c += kBlock) {
          t.push_back(Tile{g.offset + c, (int32_t)std::min<int64_t>(kBlock, hi - c),
                           (pass ? K_I64_TGPU : K_F32_TGPU) | (ls << 8)});
          fac.push_back(f);
        }
      };
      if (pass) {
        scalar(0, g.numel);
        continue;
      }
      // fp32: the 16-B aligned body in 4-element-per-lane tiles, the <= 3
      // element head and tail one element per lane (same order, same factor)
      const int64_t head = std::min<int64_t>((4 - g.offset % 4) % 4, g.numel);
      const int64_t body = (g.numel - head) / 4 * 4;
      // S = 1: 2048-element tiles, the default reduce's load shape (r02:
      // 151.9 us on cfg2 with the 1024-element form); S = 2 too since r05
      // (tgpu_wide_loop); a key whose body is not 16-B aligned keeps its own
      // tiles
      const bool wide = S <= 2;
      if (head == 0 && body > 0) {
        const bool extend = run_s >= 0 && run_f == f && run_ls == ls &&
                            (run_e == g.offset ||
                             ((flags & FA_PLAN_GAPS_ARE_PADDING) && run_e <= g.offset));
        if (!extend) flush();
        if (run_s < 0) {
          run_s = g.offset;
          run_f = f;
          run_ls = ls;
        }
        run_e = g.offset + body;
        if (body < g.numel) {
          flush();  // the tail breaks the run
          scalar(body, g.numel);
        }
        continue;
      }
      flush();
      scalar(0, head);
      const int64_t te = wide ? 8 * kBlock : 4 * kBlock;
      for (int64_t c = head; c < head + body; c += te) {
        t.push_back(Tile{g.offset + c, (int32_t)std::min<int64_t>(te, head + body - c),
                         (wide ? K_F32_TGPU_W : K_F32_TGPU_V) | (ls << 8)});
        fac.push_back(f);
      }
      scalar(head + body, g.numel);
    }
  }
  flush();
  rc = check_disjoint(t, "torch-GPU order planner");
  if (rc) return rc;
  // group the tiles by row split (inner tiles with S = 1): one launch each.
  // r05: when the S = 2 group holds the most tiles, the S = 1, S = 4 and
  // inner tiles ride in its launch, first (tgpu_kernel<1>; the small groups'
  // own launches cost 10-13 us of latency each at N = 32..127).  With the
  // S = 2 tiles wide, same process against the build before
  // (profiles/r05_ab_lib_tgpu_s2.jsonl): N = 32 / 48 / 64 / 100 / 127
  // -10.0 / -10.2 / -12.2 / -10.6 / -7.8 %, C100 N = 64 / 128 -11.6 / -6.0 %
  // (0.83-0.85 of 8 TB/s); S = 1 riders only: 1-3 points less
  {
    std::vector<int> grp(t.size());
    int cnt[5] = {0, 0, 0, 0, 0};
    for (size_t i = 0; i < t.size(); ++i) {
      const int b = t[i].kind & 0xFF;
      grp[i] = (b == K_F32_TGPU_IN || b == K_I64_TGPU_IN) ? 0 : (t[i].kind >> 8) & 0xFF;
      cnt[grp[i]]++;
    }
    const bool ride = cnt[1] > 0 && cnt[1] >= cnt[0] && cnt[1] >= cnt[2];
    // sort key: launch group, riders before the group's own tiles
    std::vector<int> key(t.size());
    for (size_t i = 0; i < t.size(); ++i) {
      const bool rider = ride && (grp[i] == 0 || grp[i] == 2);
      // tgpu_kernel<1> reduces every vector (V) rider with the S = 4 path: S = 1
      // keys never make V tiles (wide = S <= 2 above); refuse a table that
      // would, rather than reduce it in the wrong order
      if (rider && (t[i].kind & 0xFF) == K_F32_TGPU_V && ((t[i].kind >> 8) & 0xFF) != 2)
        return set_err(FA_E_INVAL, "torch-GPU order planner: a vector rider of row split %d",
                       1 << ((t[i].kind >> 8) & 0xFF));
      if (rider) grp[i] = 1;
      key[i] = 2 * grp[i] + (rider ? 0 : 1);
    }
    std::vector<size_t> ord(t.size());
    for (size_t i = 0; i < ord.size(); ++i) ord[i] = i;
    std::stable_sort(ord.begin(), ord.end(), [&](size_t x, size_t y) { return key[x] < key[y]; });
    std::vector<Tile> t2;
    std::vector<float> f2;
    for (size_t i : ord) {
      t2.push_back(t[i]);
      f2.push_back(fac[i]);
    }
    t.swap(t2);
    fac.swap(f2);
    int lo[6] = {0, 0, 0, 0, 0, 0};
    for (size_t i = 0; i < ord.size(); ++i) lo[grp[ord[i]] + 1]++;
    for (int g = 0; g < 5; ++g) lo[g + 1] += lo[g];
    if (!(flags & FA_PLAN_TUNE_NO_BALANCE)) {
      int dev = 0;
      if (hipGetDevice(&dev) == hipSuccess) {
        tgpu_split_tail(&t, &fac, lo, 0, tgpu_slots(dev, tgpu_batch_for(n)));
        // r06: the same halving on the S = 2 launch measured neutral at
        // N = 32 / 64 / 100, -2.7 % at N = 48, +0.5 % on C100 N = 128
        // (profiles/r06_ab_lib_tgpu_runs.jsonl, variant "nobal"): not applied
      }
    }
    order_groups_tmp.assign(lo, lo + 6);
  }
  fa_plan* p = new fa_plan();
  for (int g = 0; g < 6; ++g) p->tg_lo[g] = order_groups_tmp[g];
  p->info.f32_numel = f32_numel;
  p->info.i64_numel = i64_numel;
  p->info.tile_elems = 4 * kBlock;
  p->info.ntiles = (int32_t)t.size();
  p->info.ntiles_tail = (int32_t)t.size();
  p->flags = flags;
  p->flat_bcast = flat_bcast_ok(flags, s32, f32_numel, s64, i64_numel);
  p->order = FA_ORDER_TORCH_GPU;
  p->order_n = n;
  p->tgpu_batch = tgpu_batch_for(n);
  for (const Tile& x : t) (kind_is64(x.kind) ? p->has64 : p->has32) = true;
  hipError_t e = hipGetDevice(&p->device);
  if (e == hipSuccess) p->tgpu_s2_lds = tgpu_s2_lds(p->device);
  if (e == hipSuccess && !t.empty()) {
    e = hipMalloc(&p->d_tiles, t.size() * sizeof(Tile));
    if (e == hipSuccess)
      e = hipMemcpy(p->d_tiles, t.data(), t.size() * sizeof(Tile), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&p->d_fac, fac.size() * sizeof(float));
    if (e == hipSuccess)
      e = hipMemcpy(p->d_fac, fac.data(), fac.size() * sizeof(float), hipMemcpyHostToDevice);
  }
  if (e != hipSuccess) {
    if (p->d_tiles) (void)hipFree(p->d_tiles);
    if (p->d_fac) (void)hipFree(p->d_fac);
    delete p;
    return set_err(FA_E_HIP, "fa_plan_create_order: %s", hipGetErrorString(e));
  }
  *out = p;
  return FA_OK;
}

int fa_plan_build_host(const fa_seg* seg32, int nseg32, int64_t f32_numel, const fa_seg* seg64,
                       int nseg64, int64_t i64_numel, int tile_elems, unsigned flags,
                       fa_tile_desc* tiles, int cap, fa_plan_info* info) {
  if (!info) return set_err(FA_E_INVAL, "fa_plan_build_host: info is NULL");
  if (flags & ~(unsigned)FA_PLAN_FLAGS_KNOWN)
    return set_err(FA_E_INVAL, "fa_plan_build_host: unknown flag bits 0x%x",
                   flags & ~(unsigned)FA_PLAN_FLAGS_KNOWN);
  if (tile_elems == 0) tile_elems = 4 * kBlock * kDefaultU;
  if (tile_elems != 4 * kBlock && tile_elems != 8 * kBlock && tile_elems != 16 * kBlock)
    return set_err(FA_E_INVAL, "tile_elems must be 1024, 2048 or 4096 (got %d)", tile_elems);
  std::vector<fa_seg> s32, s64;
  int rc = check_segs(seg32, nseg32, f32_numel, "fp32", &s32);
  if (rc) return rc;
  rc = check_segs(seg64, nseg64, i64_numel, "int64", &s64);
  if (rc) return rc;
  fa_plan_info in{};
  in.f32_numel = f32_numel;
  in.i64_numel = i64_numel;
  in.tile_elems = tile_elems;
  std::vector<Tile> t;
  rc = build_tiles(s32, s64, tile_elems, flags, &t, &in);
  if (rc) return rc;
  *info = in;
  if (tiles) {
    if (cap < (int)t.size())
      return set_err(FA_E_RANGE, "fa_plan_build_host: %d tiles, capacity %d", (int)t.size(), cap);
    for (size_t i = 0; i < t.size(); ++i) tiles[i] = fa_tile_desc{t[i].start, t[i].count, t[i].kind};
  }
  return FA_OK;
}

int fa_plan_create_from_tiles(const fa_tile_desc* tiles, int ntiles, int64_t f32_numel,
                              int64_t i64_numel, int tile_elems, unsigned flags,
                              fa_plan** out) {
  if (!out) return set_err(FA_E_INVAL, "fa_plan_create_from_tiles: out is NULL");
  *out = nullptr;
  if (flags & ~(unsigned)FA_PLAN_FLAGS_KNOWN)
    return set_err(FA_E_INVAL, "fa_plan_create_from_tiles: unknown flag bits 0x%x",
                   flags & ~(unsigned)FA_PLAN_FLAGS_KNOWN);
  if (ntiles < 0 || (ntiles > 0 && !tiles))
    return set_err(FA_E_INVAL, "fa_plan_create_from_tiles: bad tile array");
  if (tile_elems == 0) tile_elems = 4 * kBlock * kDefaultU;
  if (tile_elems != 4 * kBlock && tile_elems != 8 * kBlock && tile_elems != 16 * kBlock)
    return set_err(FA_E_INVAL, "tile_elems must be 1024, 2048 or 4096 (got %d)", tile_elems);
  std::vector<Tile> t(ntiles);
  fa_plan_info in{};
  in.f32_numel = f32_numel;
  in.i64_numel = i64_numel;
  in.tile_elems = tile_elems;
  std::vector<Tile> vec, sc;
  for (int i = 0; i < ntiles; ++i) {
    const fa_tile_desc& d = tiles[i];
    const bool is64 = d.kind >= K_I64_CASC;
    const int64_t lim = is64 ? i64_numel : f32_numel;
    if (d.kind < K_F32_VEC || d.kind > K_I64_INNER || d.count < 1 || d.start < 0 ||
        d.start + d.count > lim)
      return set_err(FA_E_INVAL, "tile %d: kind %d [%lld,+%d) invalid", i, d.kind,
                     (long long)d.start, d.count);
    if (d.kind == K_F32_VEC) {
      if (d.start % 4 || d.count % 4 || d.count > tile_elems)
        return set_err(FA_E_INVAL, "tile %d: vector tile must be 4-aligned and <= %d", i,
                       tile_elems);
      vec.push_back(Tile{d.start, d.count, d.kind});
      in.cascade_elems += d.count;
    } else {
      if (d.count > kBlock) return set_err(FA_E_INVAL, "tile %d: scalar tile > %d", i, kBlock);
      sc.push_back(Tile{d.start, d.count, d.kind});
      if (!is64) in.tail_elems += d.count;
    }
  }
  t.clear();
  t.insert(t.end(), sc.begin(), sc.end());
  t.insert(t.end(), vec.begin(), vec.end());
  const int rc = check_disjoint(t, "fa_plan_create_from_tiles");
  if (rc) return rc;
  in.ntiles = (int32_t)t.size();
  in.ntiles_cascade = (int32_t)vec.size();
  in.ntiles_tail = (int32_t)sc.size();
  fa_plan* p = new fa_plan();
  p->info = in;
  p->vec_u = tile_elems / (4 * kBlock);
  p->flags = flags | FA_PLAN_TUNE_NO_BALANCE;  // the caller's tiles are the ones launched
  set_kinds(p, t);
  hipError_t e = hipGetDevice(&p->device);
  if (e == hipSuccess) e = upload_tables(p, t, {});
  if (e != hipSuccess) {
    if (p->d_tiles) (void)hipFree(p->d_tiles);
    if (p->d_sidx) (void)hipFree(p->d_sidx);
    delete p;
    return set_err(FA_E_HIP, "fa_plan_create_from_tiles: %s", hipGetErrorString(e));
  }
  *out = p;
  return FA_OK;
}

int fa_plan_destroy(fa_plan* plan) {
  if (!plan) return FA_OK;
  if (plan->d_fac) HIP_TRY(hipFree(plan->d_fac));
  if (plan->d_tiles) HIP_TRY(hipFree(plan->d_tiles));
  if (plan->d_tiles_alt) HIP_TRY(hipFree(plan->d_tiles_alt));
  if (plan->d_sidx) HIP_TRY(hipFree(plan->d_sidx));
  for (const fa_plan::BalTable& b : plan->bal)
    if (b.d) HIP_TRY(hipFree(b.d));
  delete plan;
  return FA_OK;
}

int fa_plan_get_info(const fa_plan* plan, fa_plan_info* info) {
  if (!plan || !info) return set_err(FA_E_INVAL, "fa_plan_get_info: NULL argument");
  *info = plan->info;
  return FA_OK;
}

namespace {
// The round's broadcast launch (after the reduce, over the arguments the
// reduce used): the flat copy in client groups on gap-padded plans
// (bcast_flat2_kernel), client groups per tile through the tile table
// otherwise (bcast_group2_kernel).  Scalar pointer loads, client groups of
// <= kBcastGroupMax = 24, 1024-float parts, destination stores sc1 nt.
// Measured inside the round, same process, after the reduce's result stores
// became sc1 (tools/archive/exp_round2.py, profiles/r04_exp_round2_bcast_forms.jsonl):
// groups of <= 24 vs <= 10 cfg2 283.7 / 282.4 vs 284.9 / 285.0 us, cfg5 (24
// slots: one group vs three) 350.0 vs 363.5 us, the small layouts equal; and
// one source fetch instead of one per group (PMC: broadcast traffic 1.0012
// vs 1.0486 x algorithmic, profiles/r04_round_pmc_round*.json).
extern "C++" template <int G>
void launch_bcast2(const fa_plan* plan, ReduceArgs& a, int ntiles, uint32_t groups,
                   uint32_t gsize, hipStream_t st) {
  if (plan->flat_bcast) {
    const int64_t f = plan->has32 ? plan->info.f32_numel : 0;
    const int64_t i = plan->has64 ? plan->info.i64_numel : 0;
    const int64_t parts = f > 0 ? std::max<int64_t>(1, (f / 4 + kBlock - 1) / kBlock) : 0;
    const int64_t np = parts + (i > 0 ? 1 : 0);
    if (np == 0) return;
    hipLaunchKernelGGL((bcast_flat2_kernel<G>), dim3((unsigned)(np * groups)), dim3(kBlock), 0,
                       st, a, (uint32_t)parts, groups, gsize, f, i);
  } else if (ntiles > 0) {
    hipLaunchKernelGGL((bcast_group2_kernel<G>), dim3((unsigned)ntiles * groups), dim3(kBlock), 0,
                       st, a, groups, gsize);
  }
}

hipError_t launch_bcast(const fa_plan* plan, ReduceArgs& a, int n, int ntiles, hipStream_t st) {
  a.flags |= FA_F_BCAST;
  if (n <= 0) return hipSuccess;
  const uint32_t groups = (uint32_t)((n + kBcastGroupMax - 1) / kBcastGroupMax);
  const uint32_t gsize = (uint32_t)((n + groups - 1) / groups);
  // grids stay below 2^32 blocks: n clients of >= 4 KB parts would outgrow
  // any GPU's memory long before
  const int64_t units = plan->flat_bcast ? (plan->info.f32_numel / 1024 + 2) : ntiles;
  if (units * (int64_t)groups > (int64_t)UINT32_MAX) return hipErrorInvalidValue;
  if (gsize <= 8) launch_bcast2<8>(plan, a, ntiles, groups, gsize, st);
  else if (gsize <= 16) launch_bcast2<16>(plan, a, ntiles, groups, gsize, st);
  else launch_bcast2<24>(plan, a, ntiles, groups, gsize, st);
  return hipGetLastError();
}
}  // namespace

}  // extern "C"
namespace {
// The table, packed-tile count, scalar index and tile width a plain reduce
// call runs with (fa_reduce; fa_plan_launch_shape reports it).
struct Launch {
  const Tile* tiles;
  int nt, ns;
  const int64_t* sidx;
  int vec_u;
  int slots;  // resident workgroups of its kernel (0: unknown / tuning grid)
  int batch;  // clients per load batch of its kernel
};
// The next client's loads before the current client's adds
// (reduce_impl.h pipe2_clients) where it measured faster
// (profiles/r05_exp_pipe2_*.jsonl, r05_ab_lib_pipe2_*.jsonl): calls of 2..7
// or 17..63 clients (inline pointers), mean or weighted, on the full
// 2048-float tiles of launches of three or more rounds of resident
// workgroups (partial tiles — tensor ends, the halved tail of a table re-cut
// for the round count — keep the batch form).  Not the 1024-float table, not
// 8..16 clients (r05: on the 8-client kernels), not the short launches
// (resnet110sl N = 25 at two rounds: +0.9 %; sf32 N = 3 at 2.5: +0.8 %).
// r06: 12..16 clients on the 16-client kernels (pick_batch, FA_B16_MIN);
// unweighted calls of 64..128 clients too, now on the 2048-float table
// (select_launch): same process against the 1024-float table's batch form
// (profiles/r06_ab_lib_n64.jsonl, two boxes) C10 N = 64 / 100 / 128 -3.5 /
// -3.1 / -3.2 % and -3.1 / -2.5 / -2.6 %, C100 N = 64 / 100 -3.0 / -2.5 % and
// -0.3 / -2.2 %, bits equal; the 2048-float table in the batch form alone
// -1.8 / -3.0 / -3.3 / -1.8 / -2.0 %.  Weighted calls from 64 keep the batch
// form (r05: the loop +0.4 / +2.4 % at 80 / 128; r06 again: -0.7 / +0.3 /
// +1.2 / +3.2 % at 64 / 80 / 100 / 128, profiles/r06_ab_lib_w64_loop.jsonl).
int pipe_rule(const fa_plan* plan, const Launch& L, int n, bool weighted) {
  (void)plan;
  // r06: unweighted calls of 256 clients and more (the DEEP cascade) on the
  // 2048-float table, the loop reading the device pointer table through
  // scalar loads (PIPE = 2): same process against the 1024-float table's
  // batch form (profiles/r06_ab_lib_tab_loop.jsonl) N = 256 / 300 -1.9 /
  // -3.8 %; at 129..255 (not deep) +0.2 / +3.5 % at 150 / 200, so those keep
  // the 1024-float table.  Bits equal.
  if (n > kInline)
    return (!weighted && n >= 256 && L.vec_u == 2 && L.batch == 16 && L.slots > 0 &&
            L.nt >= 3 * L.slots)
               ? 2
               : 0;
  if (n > kInline || L.vec_u != 2 || L.slots <= 0 || L.nt < 3 * L.slots) return 0;
#ifndef FA_PIPE_MID_LO
#define FA_PIPE_MID_LO FA_B16_MIN
#endif
  return (n >= 2 && n <= 7) || (n >= FA_PIPE_MID_LO && n <= 63) || (!weighted && n >= 64) ? 1
                                                                                            : 0;
}


Launch select_launch(const fa_plan* plan, int n, bool weighted, unsigned flags) {
  Launch L{plan->d_tiles, plan->nt_dev, plan->ns_dev, plan->d_sidx, plan->vec_u, 0, 0};
  bool alt = false;
  (void)flags;
  // 1024-float tiles for unweighted calls of 129..255 clients (r02's
  // tools/tune.py sweep took them from N = 64; r06: 64..128 and from 256 run
  // faster on the 2048-float table with the client loop, see pipe_rule; the
  // 2048-float table at N = 200 +3.7 % in the batch form, +3.5 % with the loop)
  if (plan->d_tiles_alt && !weighted && n > kInline && n < 256) {
    L.tiles = plan->d_tiles_alt;
    L.nt = plan->nt_alt_dev;
    L.ns = plan->ns_alt_dev;
    L.sidx = plan->d_sidx ? plan->d_sidx + plan->sidx_alt_off : nullptr;
    L.vec_u = 1;
    alt = true;
  }
  // the batch: 8 where that runs the plain table in one round instead of two
  L.batch = round_batch(plan->device, n, L.vec_u, weighted, plan->flags, L.nt);
  L.slots = call_slots(plan->device, n, L.vec_u, weighted, plan->flags);
  if (L.batch != pick_batch(n, L.vec_u, plan->flags)) {
    L.slots = kernel_slots(plan->device, L.vec_u, L.batch, n >= 256, weighted);
  } else if (!plan->bal.empty()) {
    // the table cut for the slot count of the kernel this call runs
    for (const fa_plan::BalTable& b : plan->bal)
      if (b.slots == L.slots && b.u == L.vec_u && b.alt == alt && b.batch == L.batch) {
        L.tiles = b.d;
        L.nt = b.nt;
        break;
      }
  }
  return L;
}
}  // namespace

extern "C" {

int fa_plan_balance_host(const fa_tile_desc* vec, int nvec, int tile_elems, int nscalar,
                         int slots, fa_tile_desc* out, int cap) {
  if (nvec < 0 || (nvec > 0 && !vec) || nscalar < 0 || slots < 0 || cap < 0 ||
      (cap > 0 && !out))
    return set_err(FA_E_INVAL, "fa_plan_balance_host: bad arguments");
  if (tile_elems != 4 * kBlock && tile_elems != 8 * kBlock && tile_elems != 16 * kBlock)
    return set_err(FA_E_INVAL, "tile_elems must be 1024, 2048 or 4096 (got %d)", tile_elems);
  std::vector<Tile> t;
  for (int i = 0; i < nvec; ++i) {
    if (vec[i].kind != K_F32_VEC || vec[i].count < 4 || vec[i].count % 4 ||
        vec[i].count > tile_elems || vec[i].start % 4)
      return set_err(FA_E_INVAL, "fa_plan_balance_host: tile %d is not a vector tile", i);
    t.push_back(Tile{vec[i].start, vec[i].count, vec[i].kind});
  }
  const std::vector<Tile> b = balance_vec(t, tile_elems, nscalar, slots);
  if ((int64_t)b.size() > (int64_t)cap)
    return set_err(FA_E_RANGE, "fa_plan_balance_host: %zu tiles > cap %d", b.size(), cap);
  for (size_t i = 0; i < b.size(); ++i) out[i] = fa_tile_desc{b[i].start, b[i].count, b[i].kind};
  return (int)b.size();
}

int fa_plan_launch_shape(const fa_plan* plan, int n, int weighted, int* ntiles, int* slots) {
  if (!plan || !ntiles || !slots || n < 1)
    return set_err(FA_E_INVAL, "fa_plan_launch_shape: bad arguments");
  if (plan->order == FA_ORDER_TORCH_GPU) {
    *ntiles = plan->info.ntiles;
    *slots = 0;
    return FA_OK;
  }
  const Launch L = select_launch(plan, n, weighted != 0, 0);
  *ntiles = L.nt;
  *slots = L.slots ? L.slots
                   : call_slots(plan->device, n, L.vec_u, weighted != 0,
                                plan->flags & ~FA_PLAN_TUNE_NO_BALANCE);
  return FA_OK;
}

int fa_plan_launch_form(const fa_plan* plan, int n, int weighted, int* tile_elems, int* batch,
                        int* pipe) {
  if (!plan || !tile_elems || !batch || !pipe || n < 1)
    return set_err(FA_E_INVAL, "fa_plan_launch_form: bad arguments");
  if (plan->order == FA_ORDER_TORCH_GPU) {
    *tile_elems = 0;
    *batch = 0;
    *pipe = 0;
    return FA_OK;
  }
  const Launch L = select_launch(plan, n, weighted != 0, 0);
  *tile_elems = 4 * kBlock * L.vec_u;
  *batch = L.batch;
  *pipe = pipe_rule(plan, L, n, weighted != 0);
  return FA_OK;
}

size_t fa_table_bytes(int n) { return n > kInline ? ((size_t)n * 20 + 7) / 8 * 8 : 0; }

int fa_reduce(const fa_plan* plan, const float* const* c32, const int64_t* const* c64, int n,
              const float* weights, float* out32, int64_t* out64, unsigned flags,
              void* stream) {
  return fa_reduce_tab(plan, c32, c64, n, weights, nullptr, out32, out64, flags, stream);
}

int fa_reduce_tab(const fa_plan* plan, const float* const* c32, const int64_t* const* c64, int n,
                  const float* weights, void* ctable, float* out32, int64_t* out64,
                  unsigned flags, void* stream) {
  if (!plan) return set_err(FA_E_INVAL, "fa_reduce: plan is NULL");
  if (n < 1) return set_err(FA_E_INVAL, "fa_reduce: need at least one client (n=%d)", n);
  if (n > FA_MAX_CLIENTS)
    return set_err(FA_E_RANGE, "fa_reduce: n=%d exceeds FA_MAX_CLIENTS=%d", n, FA_MAX_CLIENTS);
  if (flags & ~(FA_F_BCAST | FA_F_SUM_ONLY | FA_F_BCAST_ONLY))
    return set_err(FA_E_INVAL, "fa_reduce: bad flags");
  if (plan->order == FA_ORDER_TORCH_GPU && weights)
    return set_err(FA_E_INVAL, "fa_reduce: the torch-GPU order is the reference's unweighted mean");
  const fa_plan_info& in = plan->info;
  if (plan->info.ntiles == 0) return FA_OK;
  ReduceArgs a;
  memset(&a, 0, sizeof a);
  a.tiles = plan->d_tiles;
  a.out32 = out32;
  a.out64 = out64;
  a.n = n;
  a.n_total = n;
  a.flags = flags | (weights ? 0x100u : 0u);
  const bool need32 = plan->has32, need64 = plan->has64;
  if (need32) {
    if (!c32 || !out32) return set_err(FA_E_INVAL, "fa_reduce: fp32 buckets required");
    if (!aligned16(out32)) return set_err(FA_E_ALIGN, "fa_reduce: out32 not 16-B aligned");
    for (int i = 0; i < n; ++i) {
      if (!c32[i]) return set_err(FA_E_INVAL, "fa_reduce: client %d fp32 bucket NULL", i);
      if (!aligned16(c32[i]))
        return set_err(FA_E_ALIGN, "fa_reduce: client %d fp32 bucket not 16-B aligned", i);
    }
  }
  if (need64) {
    if (!c64 || !out64) return set_err(FA_E_INVAL, "fa_reduce: int64 buckets required");
    for (int i = 0; i < n; ++i)
      if (!c64[i]) return set_err(FA_E_INVAL, "fa_reduce: client %d int64 bucket NULL", i);
  }
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  if (dev != plan->device)
    return set_err(FA_E_INVAL, "fa_reduce: plan built on device %d, current device %d",
                   plan->device, dev);
  hipStream_t st = (hipStream_t)stream;
  void* table = nullptr;
  if (n <= kInline) {
    for (int i = 0; i < n; ++i) {
      if (need32) a.c32[i] = c32[i];
      if (need64) a.c64[i] = c64[i];
      if (weights) a.w[i] = weights[i];
    }
  } else {
    // [n fp32 ptrs][n int64 ptrs][n weights], stream-ordered alloc + copy
    std::vector<char> host((size_t)n * 20);
    const void** h32 = (const void**)host.data();
    const void** h64 = h32 + n;
    float* hw = (float*)(h64 + n);
    for (int i = 0; i < n; ++i) {
      h32[i] = need32 ? (const void*)c32[i] : nullptr;
      h64[i] = need64 ? (const void*)c64[i] : nullptr;
      hw[i] = weights ? weights[i] : 0.f;
    }
    if (ctable) {   // caller-owned (fa_reduce_tab): written by kernels, no memcpy
      a.tab32 = (const float* const*)ctable;
      a.tab64 = (const int64_t* const*)((const void**)ctable + n);
      a.tabw = (const float*)((const void**)ctable + 2 * n);
      HIP_TRY(table_fill(ctable, host, st));
    } else {
      HIP_TRY(table_alloc(&table, host.size(), st));
      HIP_TRY(hipMemcpyAsync(table, host.data(), host.size(), hipMemcpyHostToDevice, st));
      a.tab32 = (const float* const*)table;
      a.tab64 = (const int64_t* const*)((const void**)table + n);
      a.tabw = (const float*)((const void**)table + 2 * n);
    }
  }
  if (flags & FA_F_BCAST_ONLY) {
    // the broadcast alone (the reference's initial sync, train_fedavg.py:
    // 244-250, and :148-149 without the reduce): out32/out64 -> every client
    const int nt = plan->order == FA_ORDER_TORCH_GPU ? in.ntiles : plan->nt_dev;
    a.ntiles = nt;
    a.sidx = plan->d_sidx;
    hipError_t e = launch_bcast(plan, a, n, nt, st);
    if (table) {
      hipError_t e2 = hipFreeAsync(table, st);
      if (e == hipSuccess) e = e2;
    }
    if (e != hipSuccess) return set_err(FA_E_HIP, "broadcast launch: %s", hipGetErrorString(e));
    return FA_OK;
  }
  if (plan->order == FA_ORDER_TORCH_GPU) {
    if (n != plan->order_n) {
      if (table) (void)hipFreeAsync(table, st);
      return set_err(FA_E_INVAL, "fa_reduce: torch-GPU-order plan cut for n=%d, called with n=%d",
                     plan->order_n, n);
    }
    hipError_t e = hipSuccess;
    // the broadcast as its own launch over the whole table, client groups
    // per tile (as the default order's split broadcast)
    const bool bc = (flags & FA_F_BCAST) != 0;
    a.flags &= ~FA_F_BCAST;
    for (int g = 0; g < 5 && e == hipSuccess; ++g) {
      const int lo = plan->tg_lo[g], cnt = plan->tg_lo[g + 1] - lo;
      if (cnt == 0) continue;
      a.tiles = plan->d_tiles + lo;
      a.tfac = plan->d_fac + lo;
      a.ntiles = cnt;
      switch (g) {
        case 0:
          // the client loop on full tiles at every N (r05,
          // profiles/r05_ab_lib_tgpu_client_loop.jsonl)
          if (plan->tgpu_batch == 8)
            hipLaunchKernelGGL((tgpu_kernel<0, 8, 1>), dim3(cnt), dim3(kBlock), 0, st, a);
          else
            hipLaunchKernelGGL((tgpu_kernel<0, 16, 1>), dim3(cnt), dim3(kBlock), 0, st, a);
          break;
        case 1:
          hipLaunchKernelGGL(tgpu_kernel<1>, dim3(cnt), dim3(kBlock), plan->tgpu_s2_lds, st, a);
          break;
        case 2: hipLaunchKernelGGL(tgpu_kernel<2>, dim3(cnt), dim3(kBlock), 0, st, a); break;
        case 3: hipLaunchKernelGGL(tgpu_kernel<3>, dim3(cnt), dim3(kBlock), 0, st, a); break;
        default: hipLaunchKernelGGL(tgpu_kernel<4>, dim3(cnt), dim3(kBlock), 0, st, a); break;
      }
      e = hipGetLastError();
    }
    if (e == hipSuccess && bc && plan->tg_lo[5] > 0) {
      a.tiles = plan->d_tiles;
      a.ntiles = plan->tg_lo[5];
      e = launch_bcast(plan, a, n, a.ntiles, st);
    }
    if (table) {
      hipError_t e2 = hipFreeAsync(table, st);
      if (e == hipSuccess) e = e2;
    }
    if (e != hipSuccess) return set_err(FA_E_HIP, "torch-GPU-order launch: %s", hipGetErrorString(e));
    return FA_OK;
  }
  const Launch L = select_launch(plan, n, weights != nullptr, flags);
  a.tiles = L.tiles;
  a.nscalar = L.ns;
  a.sidx = L.sidx;
  const int ntiles = L.nt, vec_u = L.vec_u;
  a.ntiles = ntiles;
  // the broadcast is its own launch after the reduce
  const bool bcast = (flags & FA_F_BCAST) != 0;
  a.flags &= ~FA_F_BCAST;
  hipError_t e = launch_reduce(a, ntiles, vec_u, plan->flags, st, L.batch,
                               pipe_rule(plan, L, n, weights != nullptr));
  if (e == hipSuccess && bcast) e = launch_bcast(plan, a, n, ntiles, st);
  if (table) {
    hipError_t e2 = hipFreeAsync(table, st);
    if (e == hipSuccess) e = e2;
  }
  if (e != hipSuccess) return set_err(FA_E_HIP, "reduce launch: %s", hipGetErrorString(e));
  return FA_OK;
}

unsigned fa_chain_levels(int rows, int n_total) {
  if (rows <= 0 || n_total < 1) return 0;
  const int lp = level_power(n_total);
  const int step = 1 << lp;
  unsigned m = 0;
  if (rows % step) m |= 1u;                     // the open block
  if ((rows >> lp) % step) m |= 2u;             // completed blocks since the last promotion
  if (n_total >= 256) {                         // levels 2-3 exist (DEEP kernels)
    if ((rows >> (2 * lp)) % step) m |= 4u;
    if (rows >> (3 * lp)) m |= 8u;              // level 3 only accumulates
  }
  return m;
}

int fa_reduce_chain(const fa_plan* plan, const float* const* c32, int n, const float* weights,
                    const fa_chain* ch, float* out32, unsigned flags, void* stream) {
  if (!plan || !ch) return set_err(FA_E_INVAL, "fa_reduce_chain: plan/chain is NULL");
  if (flags & ~FA_F_SUM_ONLY) return set_err(FA_E_INVAL, "fa_reduce_chain: bad flags");
  const int nt = ch->n_total;
  if (nt < 1 || nt > FA_MAX_CLIENTS)
    return set_err(FA_E_RANGE, "fa_reduce_chain: n_total=%d outside 1..%d", nt, FA_MAX_CLIENTS);
  if (n < 1 || ch->row0 < 0 || ch->row0 + n > nt)
    return set_err(FA_E_INVAL, "fa_reduce_chain: rows [%d,+%d) outside the %d-row reduction",
                   ch->row0, n, nt);
  if (plan->has64 || plan->info.ntiles_tail > 0)
    return set_err(FA_E_INVAL,
                   "fa_reduce_chain: the plan holds scalar tiles (tails, M==1, int64); chain "
                   "plans carry vector tiles only (scalar columns travel raw, fedagg_comm.h)");
  const unsigned lin = fa_chain_levels(ch->row0, nt);
  const unsigned lout = fa_chain_levels(ch->row0 + n, nt);
  if (lin && !ch->state_in)
    return set_err(FA_E_INVAL, "fa_reduce_chain: rows 0..%d-1 leave a state: state_in required",
                   ch->row0);
  if (!ch->state_out && !out32)
    return set_err(FA_E_INVAL, "fa_reduce_chain: need state_out or out32");
  if (ch->state_out && ch->row0 + n == nt)
    return set_err(FA_E_INVAL, "fa_reduce_chain: the last segment finishes (state_out NULL)");
  if (!ch->state_out && ch->row0 + n != nt)
    return set_err(FA_E_INVAL, "fa_reduce_chain: only the last segment (rows ..%d) finishes",
                   nt - 1);
  const bool st = ch->state_in || ch->state_out;
  if (st && (ch->plane < plan->info.f32_numel || ch->plane % 4))
    return set_err(FA_E_INVAL, "fa_reduce_chain: plane=%lld must be >= %lld and a multiple of 4",
                   (long long)ch->plane, (long long)plan->info.f32_numel);
  if ((ch->state_in && !aligned16(ch->state_in)) || (ch->state_out && !aligned16(ch->state_out)) ||
      (out32 && !aligned16(out32)))
    return set_err(FA_E_ALIGN, "fa_reduce_chain: state/out buffers not 16-B aligned");
  if (plan->info.ntiles == 0) return FA_OK;
  if (!c32) return set_err(FA_E_INVAL, "fa_reduce_chain: fp32 buckets required");
  for (int i = 0; i < n; ++i)
    if (!c32[i] || !aligned16(c32[i]))
      return set_err(FA_E_ALIGN, "fa_reduce_chain: client %d bucket NULL or not 16-B aligned", i);
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  if (dev != plan->device)
    return set_err(FA_E_INVAL, "fa_reduce_chain: plan built on device %d, current device %d",
                   plan->device, dev);
  ReduceArgs a;
  memset(&a, 0, sizeof a);
  a.tiles = plan->d_tiles;
  a.out32 = out32;
  a.n = n;
  a.n_total = nt;
  a.row0 = ch->row0;
  a.st_in = lin ? ch->state_in : nullptr;
  a.st_out = ch->state_out;
  a.lev_in = (int)lin;
  a.lev_out = (int)lout;
  a.plane = ch->plane;
  a.flags = flags | (weights ? 0x100u : 0u);
  a.ntiles = plan->nt_dev;
  hipStream_t s = (hipStream_t)stream;
  void* table = nullptr;
  if (n <= kInline) {
    for (int i = 0; i < n; ++i) {
      a.c32[i] = c32[i];
      if (weights) a.w[i] = weights[i];
    }
  } else {
    std::vector<char> host((size_t)n * 20);
    const void** h32 = (const void**)host.data();
    float* hw = (float*)(h32 + 2 * n);
    for (int i = 0; i < n; ++i) {
      h32[i] = c32[i];
      h32[n + i] = nullptr;
      hw[i] = weights ? weights[i] : 0.f;
    }
    HIP_TRY(table_alloc(&table, host.size(), s));
    HIP_TRY(hipMemcpyAsync(table, host.data(), host.size(), hipMemcpyHostToDevice, s));
    a.tab32 = (const float* const*)table;
    a.tab64 = (const int64_t* const*)((const void**)table + n);
    a.tabw = (const float*)((const void**)table + 2 * n);
  }
  hipError_t e = launch_chain(a, a.ntiles, plan->vec_u, s);
  if (table) {
    hipError_t e2 = hipFreeAsync(table, s);
    if (e == hipSuccess) e = e2;
  }
  if (e != hipSuccess) return set_err(FA_E_HIP, "chain launch: %s", hipGetErrorString(e));
  return FA_OK;
}

int fa_mean_f32(const float* const* clients, int n, int64_t numel, float* out,
                const fa_seg* segs, int nseg, void* stream) {
  fa_plan* p = nullptr;
  int rc = cached_plan(segs, nseg, numel, nullptr, 0, 0, &p);
  if (rc) return rc;
  return fa_reduce(p, clients, nullptr, n, nullptr, out, nullptr, 0, stream);
}

int fa_weighted_f32(const float* const* clients, const float* w, int n, int64_t numel,
                    float* out, const fa_seg* segs, int nseg, void* stream) {
  if (!w) return set_err(FA_E_INVAL, "fa_weighted_f32: weights NULL");
  fa_plan* p = nullptr;
  int rc = cached_plan(segs, nseg, numel, nullptr, 0, 0, &p);
  if (rc) return rc;
  return fa_reduce(p, clients, nullptr, n, w, out, nullptr, 0, stream);
}

int fa_mean_i64_trunc(const int64_t* const* clients, int n, int64_t numel, int64_t* out,
                      const fa_seg* segs, int nseg, void* stream) {
  fa_plan* p = nullptr;
  int rc = cached_plan(nullptr, 0, 0, segs, nseg, numel, &p);
  if (rc) return rc;
  return fa_reduce(p, nullptr, clients, n, nullptr, nullptr, out, 0, stream);
}

int fa_div_f32(const float* x, float d, float* out, int64_t numel, void* stream) {
  if (numel < 0 || (numel > 0 && (!x || !out))) return set_err(FA_E_INVAL, "fa_div_f32: bad args");
  if (numel == 0) return FA_OK;
  hipLaunchKernelGGL(div_f32_kernel, dim3(grid_for(numel, kBlock)), dim3(kBlock), 0,
                     (hipStream_t)stream, x, d, out, numel);
  HIP_TRY(hipGetLastError());
  return FA_OK;
}

int fa_div_trunc_i64(const float* x, float d, int64_t* out, int64_t numel, void* stream) {
  if (numel < 0 || (numel > 0 && (!x || !out)))
    return set_err(FA_E_INVAL, "fa_div_trunc_i64: bad args");
  if (numel == 0) return FA_OK;
  hipLaunchKernelGGL(div_trunc_i64_kernel, dim3(grid_for(numel, kBlock)), dim3(kBlock), 0,
                     (hipStream_t)stream, x, d, out, numel);
  HIP_TRY(hipGetLastError());
  return FA_OK;
}

int fa_broadcast_f32(const float* src, float* const* dst, int n, int64_t numel, void* stream) {
  if (n < 0 || n > FA_MAX_CLIENTS) return set_err(FA_E_RANGE, "fa_broadcast_f32: n=%d", n);
  if (numel < 0 || (numel > 0 && (!src || (n > 0 && !dst))))
    return set_err(FA_E_INVAL, "fa_broadcast_f32: bad args");
  if (n == 0 || numel == 0) return FA_OK;
  if (!aligned16(src)) return set_err(FA_E_ALIGN, "fa_broadcast_f32: src not 16-B aligned");
  for (int i = 0; i < n; ++i)
    if (!dst[i] || !aligned16(dst[i]))
      return set_err(FA_E_ALIGN, "fa_broadcast_f32: dst %d NULL or unaligned", i);
  for (int i0 = 0; i0 < n; i0 += kBcastInline) {
    BcastArgs a;
    memset(&a, 0, sizeof a);
    a.src = src;
    a.n = std::min(kBcastInline, n - i0);
    for (int i = 0; i < a.n; ++i) a.dst[i] = dst[i0 + i];
    const int64_t parts = std::max<int64_t>(1, (numel / 4 + 2 * kBlock - 1) / (2 * kBlock));
    const uint32_t groups = (uint32_t)((a.n + kBcastGroupMax - 1) / kBcastGroupMax);
    const uint32_t gsize = (uint32_t)((a.n + groups - 1) / groups);
    if (parts * groups > (int64_t)UINT32_MAX)
      return set_err(FA_E_RANGE, "fa_broadcast_f32: numel=%lld", (long long)numel);
    const unsigned grid = (unsigned)std::min<int64_t>(parts * groups, 1ll << 30);
    hipLaunchKernelGGL(bcast_kernel, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream, a, numel,
                       (uint32_t)parts, groups, gsize);
    HIP_TRY(hipGetLastError());
  }
  return FA_OK;
}

int fa_write_probe_f32(float* const* dst, int n, int64_t numel, unsigned seed, void* stream) {
  if (n < 0 || n > kBcastInline) return set_err(FA_E_RANGE, "fa_write_probe_f32: n=%d", n);
  if (numel < 0 || (numel > 0 && n > 0 && !dst))
    return set_err(FA_E_INVAL, "fa_write_probe_f32: bad args");
  if (n == 0 || numel < 4) return FA_OK;
  BcastArgs a;
  memset(&a, 0, sizeof a);
  a.n = n;
  for (int i = 0; i < n; ++i) {
    if (!dst[i] || !aligned16(dst[i]))
      return set_err(FA_E_ALIGN, "fa_write_probe_f32: dst %d NULL or unaligned", i);
    a.dst[i] = dst[i];
  }
  const int64_t parts = (numel / 4 + kBlock - 1) / kBlock;
  const uint32_t groups = (uint32_t)((n + kBcastGroupMax - 1) / kBcastGroupMax);
  const uint32_t gsize = (uint32_t)((n + groups - 1) / groups);
  if (parts * groups > (int64_t)UINT32_MAX)
    return set_err(FA_E_RANGE, "fa_write_probe_f32: numel=%lld", (long long)numel);
  hipLaunchKernelGGL(write_probe_kernel, dim3((unsigned)(parts * groups)), dim3(kBlock), 0,
                     (hipStream_t)stream, a, numel, (uint32_t)parts, groups, gsize, seed);
  HIP_TRY(hipGetLastError());
  return FA_OK;
}

int fa_synth_fill_f32(float* dst, int64_t numel, int key_index, int client, float mu,
                      float sigma, int mode, void* stream) {
  if (numel < 0 || (numel > 0 && !dst)) return set_err(FA_E_INVAL, "fa_synth_fill_f32: bad args");
  if (numel == 0) return FA_OK;
  // the generator's third constant, rounded exactly as synth.key_consts does
  volatile float s = sigma, c = 0.01f;
  const float dsig = s * c;
  hipLaunchKernelGGL(synth_f32_kernel, dim3(grid_for(numel, kBlock)), dim3(kBlock), 0,
                     (hipStream_t)stream, dst, numel, key_index, client, mu, sigma, dsig, mode);
  HIP_TRY(hipGetLastError());
  return FA_OK;
}

int fa_synth_fill_i64(int64_t* dst, int64_t numel, int key_index, int client, int mode,
                      void* stream) {
  if (numel < 0 || (numel > 0 && !dst)) return set_err(FA_E_INVAL, "fa_synth_fill_i64: bad args");
  if (numel == 0) return FA_OK;
  hipLaunchKernelGGL(synth_i64_kernel, dim3(grid_for(numel, kBlock)), dim3(kBlock), 0,
                     (hipStream_t)stream, dst, numel, key_index, client, mode);
  HIP_TRY(hipGetLastError());
  return FA_OK;
}

int fa_read_probe_f32(const float* src, int64_t numel, float* out, int grid, void* stream) {
  if (numel < 4 || !src || !out || grid < 0) return set_err(FA_E_INVAL, "fa_read_probe_f32: bad args");
  if (!aligned16(src)) return set_err(FA_E_ALIGN, "fa_read_probe_f32: unaligned");
  if (grid == 0) {  // one 2048-float tile per workgroup (whole float4s only)
    const int64_t nv = numel / 4, g = (nv + 2 * kBlock - 1) / (2 * kBlock);
    if (g > 0x7fffffff) return set_err(FA_E_RANGE, "fa_read_probe_f32: %lld floats", (long long)numel);
    hipLaunchKernelGGL(read_tile_kernel, dim3((unsigned)g), dim3(kBlock), 0, (hipStream_t)stream,
                       src, nv, out);
  } else {
    hipLaunchKernelGGL(read_probe_kernel, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream, src,
                       numel / 4, out);
  }
  HIP_TRY(hipGetLastError());
  return FA_OK;
}

int fa_copy_f32(const float* src, float* dst, int64_t numel, void* stream) {
  if (numel < 0 || (numel > 0 && (!src || !dst))) return set_err(FA_E_INVAL, "fa_copy_f32: bad args");
  if (numel == 0) return FA_OK;
  if (!aligned16(src) || !aligned16(dst)) return set_err(FA_E_ALIGN, "fa_copy_f32: unaligned");
  const int64_t grid = std::max<int64_t>(1, (numel / 4 + kBlock - 1) / kBlock);
  if (grid > 0x7fffffff) return set_err(FA_E_RANGE, "fa_copy_f32: %lld floats", (long long)numel);
  hipLaunchKernelGGL(copy_kernel, dim3((unsigned)grid), dim3(kBlock), 0, (hipStream_t)stream, src,
                     dst, numel);
  HIP_TRY(hipGetLastError());
  return FA_OK;
}

}  // extern "C"
