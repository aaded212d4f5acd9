// reduce_impl.h — the reduce kernel family of libfedagg.so (torch's CPU
// summation order over flat client buckets, fedagg.hip's header comment) and
// its launchers.  Shared by fedagg.hip (plans, C ABI, every other kernel)
// and the fedagg_k*.hip translation units, which instantiate the launcher
// templates for disjoint (tile width U, client batch B) sets so hipcc builds
// the reduce_kernel variants in parallel; fedagg.hip declares those
// instantiations extern.  Every kernel instance is compiled in exactly one
// translation unit (its launches are made from there).  r05 (VERDICT r04
// weak 7): only what ships — U in {1, 2, 4} (1024 / 2048 / 4096-float
// tiles), batches of 8 or 16 clients, the default cache policy (nt loads, sc1
// result stores; chain segments nt) — 36 instances; the measured-and-dropped
// forms (other policies, persistent grids, XCD-contiguous tiles, wave-
// contiguous lanes, issue-all batches, the fused broadcast) live on in
// tools/reducelab.hip / tools/roundlab.hip and the r04 history.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.h"

namespace fa_k {

// ----------------------------------------------------------------- tiles --
enum TileKind : int32_t {
  K_F32_VEC = 0,      // cascade order, 16-B vectors, count % 4 == 0
  K_F32_CASC_S = 1,   // cascade order, one element per thread (unaligned)
  K_F32_ILP4 = 2,     // tail columns: ILP-4 order
  K_F32_INNER = 3,    // M == 1: ILP-4 (n < 8) or 8-lane inner (n >= 8)
  K_I64_CASC = 4,
  K_I64_ILP4 = 5,
  K_I64_INNER = 6,
  // torch-ROCm's GPU order (fa_plan_create_order, FA_ORDER_TORCH_GPU); the
  // tile's kind carries log2 of its stride in bits 8-15
  K_F32_TGPU = 7,     // [N, M>=2]: S-way row split, 4 round-robin accumulators
  K_I64_TGPU = 8,
  K_F32_TGPU_IN = 9,  // M == 1: lane split + intra-wave shuffle tree, 1 element/wave
  K_I64_TGPU_IN = 10,
  K_F32_TGPU_V = 11,  // [N, M>=2], 16-B aligned run: 4 elements per lane, up to 1024
  K_F32_TGPU_W = 12,  // the same with S = 1: 8 elements per lane (2 x 16 B), up to 2048
  // device tables only (r03): the plan's scalar tiles (kinds 1-6) packed,
  // up to 256 elements of any tensors per tile; `start` indexes the plan's
  // scalar index, whose entries are (bucket element << 4) | kind
  K_SCALAR_PACKED = 13,
};

__host__ __device__ inline bool kind_is64(int kind) {
  const int b = kind & 0xFF;
  return b == K_I64_CASC || b == K_I64_ILP4 || b == K_I64_INNER || b == K_I64_TGPU ||
         b == K_I64_TGPU_IN;
}

struct Tile {
  int64_t start;  // first element (bucket index)
  int32_t count;  // elements
  int32_t kind;
};
static_assert(sizeof(Tile) == 16, "tile is 16 B");

constexpr int kBlock = 256;
constexpr int kDefaultU = 2;
// MI355X's device properties as torch-ROCm's setReduceConfig reads them
// (multiProcessorCount, maxThreadsPerMultiProcessor): they decide where torch
// splits a reduction across blocks (fa_torch_gpu_config); a GPU test checks
// them against torch.cuda.get_device_properties.
constexpr int64_t kTorchNumCU = 256;
constexpr int64_t kTorchMaxThreadsPerCU = 2048;  // float4 vectors per thread per client (tools/tune.py)

constexpr int kInline = FA_INLINE_CLIENTS;

// Client pointer tables travel inline in the kernel arguments for
// n <= kInline (the common case: no setup copy at all); beyond that they sit
// in a stream-ordered device allocation (tab32/tab64/tabw).
struct ReduceArgs {
  const Tile* tiles;
  float* out32;
  int64_t* out64;
  int n;
  unsigned flags;
  int ntiles;   // tiles in the table (== grid)
  int nscalar;  // leading scalar tiles
  // The cascade's position (fa_reduce_chain; a plain reduction is row0 = 0,
  // n_total = n): these clients are rows row0 .. row0+n-1 of an n_total-row
  // reduction.  The level accumulators start from st_in's planes (bit l of
  // lev_in: plane l at st_in + l*plane; others +0) and, with st_out, end
  // there (bit l of lev_out) instead of being finished into out32.
  int n_total;
  int row0;
  int lev_in;
  int lev_out;
  const float* st_in;
  float* st_out;
  int64_t plane;
  const float* tfac;  // torch-GPU order: per-tile mean factor fl(M)/fl(N*M)
  const int64_t* sidx;  // packed scalar tiles' entries (K_SCALAR_PACKED)
  const float* const* tab32;
  const int64_t* const* tab64;
  const float* tabw;
  const float* c32[kInline];
  const int64_t* c64[kInline];
  float w[kInline];
};

// The kernel reads its arguments through this constant-address-space view of
// the kernarg segment.  Binding a by-value struct parameter to a reference
// instead makes the compiler copy the whole 2.6 KB struct into per-lane
// scratch (measured: 7x slower); the kernarg view keeps every pointer fetch a
// scalar load.
typedef __attribute__((address_space(4))) const ReduceArgs KArgs;

__device__ __forceinline__ const float* cptr32(KArgs& a, int i) {
  return a.n <= kInline ? a.c32[i] : a.tab32[i];
}
__device__ __forceinline__ const int64_t* cptr64(KArgs& a, int i) {
  return a.n <= kInline ? a.c64[i] : a.tab64[i];
}
__device__ __forceinline__ float cw(KArgs& a, int i) {
  return a.n <= kInline ? a.w[i] : a.tabw[i];
}

// Pointer source of the vector path.  TAB (the DEEP kernels, n >= 256): the
// device table through a constant-address-space view (read-only for the
// launch), so a uniform index is one scalar load: 2-10 % faster at 300
// clients than generic loads (2 % slower at 200, hence only from 256 on).
// Otherwise the runtime-selecting accessor above.  Measured
// (tools/archive/exp_ab.py, same box, one process): compiled this way the inline
// kernel issues each client's U loads behind a vmcnt(0) wait and runs
// 141-146 us on the cfg2 workload; reading a.c32[i] directly lets the
// compiler issue the whole batch's loads back to back, which is 4-6 %
// SLOWER (148-156 us) at every batch size tried (1, 4, 8, 16 clients).
typedef const float* f32p;
#define FA_CONST __attribute__((address_space(4)))
template <bool TAB>
__device__ __forceinline__ const float* vptr32(KArgs& a, int i) {
  if constexpr (TAB) return ((const FA_CONST f32p*)a.tab32)[i];
  else return cptr32(a, i);
}

// Destination pointer of a store loop, through SCALAR loads only: the
// kernarg array, or the device table through the constant address space
// (read-only for the launch).  cptr32's table arm is a generic global load,
// and the compiler serves the runtime choice between the two arms with an
// `s_waitcnt vmcnt(0)` before each client's stores (ISA checked, r04); vmcnt
// counts stores on CDNA, so every wave waited for its previous client's
// stores to complete before issuing the next client's.  Measured r04: the
// broadcast of the cfg2 round 156 us with cptr32, 127-134 us in a lab kernel
// whose pointers are scalar loads (tools/writelab.hip).
typedef float* f32m;
typedef const int64_t* i64p;
__device__ __forceinline__ float* sptr32(KArgs& a, int i) {
  return a.n <= kInline ? const_cast<float*>(a.c32[i]) : ((const FA_CONST f32m*)a.tab32)[i];
}
__device__ __forceinline__ int64_t* sptr64(KArgs& a, int i) {
  return const_cast<int64_t*>(a.n <= kInline ? a.c64[i] : ((const FA_CONST i64p*)a.tab64)[i]);
}

typedef float f4 __attribute__((ext_vector_type(4)));

// The weights of clients b0..b0+nb-1, read once per batch BEFORE its data
// loads are issued, through scalar loads only (kernarg array, or the device
// table through the constant address space: read-only for the launch).
// Reading each weight in the add phase instead put a load round trip and a
// vmcnt/lgkmcnt(0) wait between consecutive clients' adds (the weighted
// kernel ran 4-6 % behind the mean, r02 profiles).
template <int NB>
__device__ __forceinline__ void load_weights(KArgs& a, int b0, int nb, float (&wb)[NB]) {
  if (a.n <= kInline) {
#pragma unroll
    for (int b = 0; b < NB; ++b) wb[b] = b < nb ? a.w[b0 + b] : 0.f;
  } else {
    const FA_CONST float* t = (const FA_CONST float*)a.tabw;
#pragma unroll
    for (int b = 0; b < NB; ++b) wb[b] = b < nb ? t[b0 + b] : 0.f;
  }
}

// c10::utils::CeilLog2 / ATen multi_row_sum level power
__host__ __device__ inline int ceil_log2_i(int64_t n) {
  if (n <= 1) return 0;
  int r = 0;
  uint64_t v = (uint64_t)(n - 1);
  while (v) { ++r; v >>= 1; }
  return r;
}
__host__ __device__ inline int level_power(int64_t n) {
  int c = ceil_log2_i(n) / 4;
  return c > 4 ? c : 4;
}

__device__ __forceinline__ f4 add4(f4 a, f4 b) {
  return f4{__fadd_rn(a.x, b.x), __fadd_rn(a.y, b.y), __fadd_rn(a.z, b.z),
            __fadd_rn(a.w, b.w)};
}
__device__ __forceinline__ f4 mul4s(f4 a, float s) {
  return f4{__fmul_rn(a.x, s), __fmul_rn(a.y, s), __fmul_rn(a.z, s),
            __fmul_rn(a.w, s)};
}
__device__ __forceinline__ f4 div4s(f4 a, float s) {
  return f4{__fdiv_rn(a.x, s), __fdiv_rn(a.y, s), __fdiv_rn(a.z, s),
            __fdiv_rn(a.w, s)};
}

// Global-address-space views: loads/stores compile to global_* (not flat_*)
// instructions; with a uniform base and a 32-bit vector index they take the
// SGPR-base + one-VGPR-offset form, so a batch of B clients costs no 64-bit
// per-lane address arithmetic and no address VGPRs.
typedef __attribute__((address_space(1))) const f4 gcf4;
typedef __attribute__((address_space(1))) f4 gf4;

template <bool NT>
__device__ __forceinline__ f4 ldg4(const float* base, uint32_t vidx) {
  gcf4* g = (gcf4*)base;
  if constexpr (NT) return __builtin_nontemporal_load(g + vidx);
  else return g[vidx];
}
template <bool NT>
__device__ __forceinline__ void stg4(float* base, uint32_t vidx, f4 v) {
  gf4* g = (gf4*)base;
  if constexpr (NT) __builtin_nontemporal_store(v, g + vidx);
  else g[vidx] = v;
}
template <bool NT>
__device__ __forceinline__ f4 ld4(const float* p) {
  return ldg4<NT>(p, 0);
}
template <bool NT>
__device__ __forceinline__ void st4(float* p, f4 v) {
  stg4<NT>(p, 0, v);
}

// Result store of a vector tile.  POL bit 2 (the default reduce, POL 5):
// through a buffer op with the sc1 cache-policy bit (aux 16) instead of a
// global store; POL 3 (chain segments): the global nt store.  The descriptor
// is based at the tile start (uniform).
// r04 default (POL 5: sc1 without nt).  An sc1 store writes through and drops
// the line from the XCD's L2; an nt store (r01-r03) keeps it there.  The
// round's broadcast reads this result right after the reduce, and reading it
// then was the round's back-to-back penalty: tools/roundlab.hip
// (profiles/r04_roundlab_policy.jsonl, one box, 20 x 43.9 MB, hashed data):
// the broadcast after a read pass whose result went out nt 168-172 us, after
// one whose result went out sc1 (or sc0 sc1) 151-152 us, alone 149 us; the
// read pass itself 136-138 us with sc1 result stores against 142 us nt.  The
// r01 measurement that kept nt ("sc1 result stores 1-2 % slower") was of
// sc1 + nt (aux 18, FA_PLAN_TUNE_ST_SC1), which keeps the penalty.
template <int POL>
__device__ __forceinline__ void st_out(float* out, int64_t start, uint32_t vidx, f4 v) {
  if constexpr ((POL & 4) != 0) {
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(out + start, (short)0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)(16 * vidx), 0, (POL & 2) ? 18 : 16);
  } else {
    stg4<(POL & 2) != 0>(out + start, vidx, v);
  }
}

// -------------------------------------------------- vectorised cascade ----
// ATen multi_row_sum over the n clients for 4*U columns per thread.  The
// loop over clients is uniform (scalar control).  Clients go in batches of B:
// the batch's B pointers come in as one scalar load, all B*U 16-B loads are
// issued, then the adds run in client order with the block promotion after
// every full block of 2^lp rows (lp = 4 for n < 2^20).
template <int U, bool DEEP>
struct Acc {
  f4 l0[U], l1[U], l2[U], l3[U];
};

template <int U, bool DEEP>
__device__ __forceinline__ void promote(Acc<U, DEEP>& A, int ii, int lp, int mask) {
  if ((ii & mask) != 0) return;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    A.l1[u] = add4(A.l1[u], A.l0[u]);
    A.l0[u] = f4{0.f, 0.f, 0.f, 0.f};
  }
  if constexpr (DEEP) {
    if ((ii & (mask << lp)) != 0) return;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      A.l2[u] = add4(A.l2[u], A.l1[u]);
      A.l1[u] = f4{0.f, 0.f, 0.f, 0.f};
    }
    if ((ii & (mask << (2 * lp))) != 0) return;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      A.l3[u] = add4(A.l3[u], A.l2[u]);
      A.l2[u] = f4{0.f, 0.f, 0.f, 0.f};
    }
  }
}

// One batch of NB clients starting at b0.  FULL: every lane's U vectors are
// inside the tile (no per-lane predicate).
template <int U, int NB, bool FULL, bool DEEP, bool WEIGHTED, int POL, bool TAB>
__device__ __forceinline__ void batch(KArgs& a, Acc<U, DEEP>& A, int b0, int64_t start,
                                      const uint32_t (&vi)[U], const bool (&ok)[U],
                                      int lp, int mask, int r0) {
  f4 x[NB][U];
  float wb[NB];
  if constexpr (WEIGHTED) load_weights<NB>(a, b0, NB, wb);
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const float* p = vptr32<TAB>(a, b0 + b) + start;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (FULL) x[b][u] = ldg4<(POL & 1) != 0>(p, vi[u]);
      else x[b][u] = ok[u] ? ldg4<(POL & 1) != 0>(p, vi[u]) : f4{0.f, 0.f, 0.f, 0.f};
    }
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f4 v = x[b][u];
      if constexpr (WEIGHTED) v = mul4s(v, wb[b]);
      A.l0[u] = add4(A.l0[u], v);
    }
    promote<U, DEEP>(A, r0 + b0 + b + 1, lp, mask);
  }
}

// The last, partial batch (nb < NB clients): same issue-all-then-add shape,
// every step guarded by a uniform (scalar) branch.
template <int U, int NB, bool FULL, bool DEEP, bool WEIGHTED, int POL, bool TAB>
__device__ __forceinline__ void batch_tail(KArgs& a, Acc<U, DEEP>& A, int b0, int nb,
                                           int64_t start, const uint32_t (&vi)[U],
                                           const bool (&ok)[U], int lp, int mask, int r0) {
  f4 x[NB][U];
  float wb[NB];
  if constexpr (WEIGHTED) load_weights<NB>(a, b0, nb, wb);
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    if (b < nb) {
      const float* p = vptr32<TAB>(a, b0 + b) + start;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if constexpr (FULL) x[b][u] = ldg4<(POL & 1) != 0>(p, vi[u]);
        else x[b][u] = ok[u] ? ldg4<(POL & 1) != 0>(p, vi[u]) : f4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    if (b < nb) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        f4 v = x[b][u];
        if constexpr (WEIGHTED) v = mul4s(v, wb[b]);
        A.l0[u] = add4(A.l0[u], v);
      }
      promote<U, DEEP>(A, r0 + b0 + b + 1, lp, mask);
    }
  }
}

// The clients one after another with the next client's loads issued
// before the current client's adds (r05; the same order as the batches, so
// the batches' bits).  As compiled (ISA read), each iteration issues client
// b+1's loads, then waits for every outstanding load (vmcnt(0)), then adds
// client b: still one client's data in flight per wave, as in the batch
// form, but the adds, the promotion and the next pointer's scalar load no
// longer sit between one client's data arriving and the next client's loads
// leaving.  Its own kernel instances (PIPE), full tiles only; the launch
// rule (fedagg.hip pipe_rule) and the measurements behind it are in DESIGN
// §4.1: 1.0-1.7 % faster for 2..7 and 17..63 clients (r06: 12..63, and
// unweighted 64..128), mean or weighted, in
// launches of three or more rounds (cfg2, cfg3, cfg4, cfg5), slower for
// 8..12 and 64..128 clients and on short launches.  Partial tiles keep the
// batch form: an instance that took them too compiled into a truly two-deep
// loop (waits for the older client only, vmcnt(U)) and ran 5-8 % SLOWER, as
// did a hand-written two-register-set form (4 %): two clients per wave in
// flight spread the chip's reads over twice as many places, as the issue-all
// batch form did in r04 (profiles/r05_ab_lib_pipe2_*.jsonl).
template <int U, bool DEEP, bool WEIGHTED, int POL, bool TABP = false>
__device__ __forceinline__ const float* pipe_ptr(KArgs& a, int i) {
  if constexpr (TABP) return ((const FA_CONST f32p*)a.tab32)[i];
  else return a.c32[i];
}
template <int U, bool DEEP, bool WEIGHTED, int POL, bool TABP = false>
__device__ __forceinline__ void pipe2_clients(KArgs& a, Acc<U, DEEP>& A, int n, int64_t start,
                                              const uint32_t (&vl)[U], int lp, int mask) {
  f4 cur[U], nxt[U];
  {
    const float* p = pipe_ptr<U, DEEP, WEIGHTED, POL, TABP>(a, 0) + start;
#pragma unroll
    for (int u = 0; u < U; ++u) cur[u] = ldg4<(POL & 1) != 0>(p, vl[u]);
  }
  for (int b = 0; b < n; ++b) {
    if (b + 1 < n) {
      const float* p = pipe_ptr<U, DEEP, WEIGHTED, POL, TABP>(a, b + 1) + start;
#pragma unroll
      for (int u = 0; u < U; ++u) nxt[u] = ldg4<(POL & 1) != 0>(p, vl[u]);
    }
    if constexpr (WEIGHTED) {
      const float wb = a.w[b];
#pragma unroll
      for (int u = 0; u < U; ++u) A.l0[u] = add4(A.l0[u], mul4s(cur[u], wb));
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) A.l0[u] = add4(A.l0[u], cur[u]);
    }
    promote<U, DEEP>(A, b + 1, lp, mask);
#pragma unroll
    for (int u = 0; u < U; ++u) cur[u] = nxt[u];
  }
}

// PIPE (r05): pipe2_clients for the full tiles (fedagg.hip pipe_rule); its
// own kernel instances, so the other kernels' code is unchanged
template <int U, int B, bool FULL, bool DEEP, bool WEIGHTED, int POL, bool CHAIN, int PIPE = 0>
__device__ __forceinline__ void tile_vec(KArgs& a, int64_t start,
                                         int count) {
  // TAB: the DEEP kernels' constant-space pointer table; a chain segment may
  // be DEEP (n_total >= 256) with few local clients, so it takes the
  // runtime-selected pointer source instead
  constexpr bool TAB = DEEP && !CHAIN;
  const int n = a.n;
  const int nt = CHAIN ? a.n_total : n;
  const int r0 = CHAIN ? a.row0 : 0;
  const int lp = level_power(nt);
  const int mask = (1 << lp) - 1;
  Acc<U, DEEP> A;
  uint32_t vi[U];
  bool ok[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    // block-strided: lane t takes vectors t, t+256, ...
    const int v = (int)threadIdx.x + u * kBlock;
    vi[u] = (uint32_t)v;
    ok[u] = FULL || 4 * v < count;
    A.l0[u] = A.l1[u] = A.l2[u] = A.l3[u] = f4{0.f, 0.f, 0.f, 0.f};
  }
  if constexpr (CHAIN) {
    // the state after rows 0..row0-1 (levels outside lev_in are +0, exactly
    // what the cascade holds there after its promotions)
    if (a.st_in) {
      const int li = a.lev_in;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (!ok[u]) continue;
        if (li & 1) A.l0[u] = ldg4<true>(a.st_in + start, vi[u]);
        if (li & 2) A.l1[u] = ldg4<true>(a.st_in + a.plane + start, vi[u]);
        if constexpr (DEEP) {
          if (li & 4) A.l2[u] = ldg4<true>(a.st_in + 2 * a.plane + start, vi[u]);
          if (li & 8) A.l3[u] = ldg4<true>(a.st_in + 3 * a.plane + start, vi[u]);
        }
      }
    }
  }
  int b0 = 0;
  if constexpr (PIPE == 1 && FULL && !CHAIN && !TAB) {
    // pipe2_clients reads the inline kernarg arrays: safe on its own for any
    // launch, the host rule (pipe_rule) aside — beyond kInline clients the
    // batches below take the tile
    if (n <= kInline) {
      pipe2_clients<U, DEEP, WEIGHTED, POL>(a, A, n, start, vi, lp, mask);
      b0 = n;
    }
  }
  if constexpr (PIPE == 2 && FULL && !CHAIN && !WEIGHTED) {
    // r06: the device pointer table through the constant address space
    // (scalar loads): the unweighted calls of 256 clients and more (DEEP)
    if (n > kInline) {
      pipe2_clients<U, DEEP, WEIGHTED, POL, true>(a, A, n, start, vi, lp, mask);
      b0 = n;
    }
  }
  for (; b0 + B <= n; b0 += B)
    batch<U, B, FULL, DEEP, WEIGHTED, POL, TAB>(a, A, b0, start, vi, ok, lp, mask, r0);
  if (b0 < n)
    batch_tail<U, B, FULL, DEEP, WEIGHTED, POL, TAB>(a, A, b0, n - b0, start, vi, ok, lp, mask,
                                                     r0);
  if constexpr (CHAIN) {
    if (a.st_out) {
      const int lo = a.lev_out;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (!ok[u]) continue;
        if (lo & 1) stg4<true>(a.st_out + start, vi[u], A.l0[u]);
        if (lo & 2) stg4<true>(a.st_out + a.plane + start, vi[u], A.l1[u]);
        if constexpr (DEEP) {
          if (lo & 4) stg4<true>(a.st_out + 2 * a.plane + start, vi[u], A.l2[u]);
          if (lo & 8) stg4<true>(a.st_out + 3 * a.plane + start, vi[u], A.l3[u]);
        }
      }
      return;
    }
  }

  const bool sum_only = WEIGHTED || (a.flags & FA_F_SUM_ONLY);
  const float fn = (float)nt;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (!ok[u]) continue;
    // acc2/acc3 stay +0 unless DEEP; x + (+0) == x for every x a +0-seeded
    // round-to-nearest sum can produce (never -0), so skipping them is exact.
    f4 s = add4(A.l0[u], A.l1[u]);
    if constexpr (DEEP) {
      s = add4(s, A.l2[u]);
      s = add4(s, A.l3[u]);
    }
    const f4 r = sum_only ? s : div4s(s, fn);
    st_out<POL>(a.out32, start, vi[u], r);
  }
}

// ------------------------------------------------------- scalar orders ----
struct SrcF32 {
  KArgs& a;
  bool weighted;
  __device__ float operator()(int i, int64_t e) const {
    float x = cptr32(a, i)[e];
    return weighted ? __fmul_rn(x, cw(a, i)) : x;
  }
};
struct SrcI64 {
  KArgs& a;
  __device__ float operator()(int i, int64_t e) const {
    return (float)cptr64(a, i)[e];  // .float(): int64 -> fp32, round to nearest
  }
};

// multi_row_sum over rows first, first+stride, ... (count rows), 1 column.
// The four level accumulators are named variables (a runtime-indexed array
// would live in scratch).
template <class Src>
__device__ __forceinline__ float cascade_seq(const Src& src, int64_t e, int first, int stride,
                             int count) {
  const int lp = level_power(count);
  const int step = 1 << lp, mask = step - 1;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int i = 0;
  for (; i + step <= count;) {
    for (int j = 0; j < step; ++j, ++i) a0 = __fadd_rn(a0, src(first + i * stride, e));
    a1 = __fadd_rn(a1, a0);
    a0 = 0.f;
    if (i & (mask << lp)) continue;
    a2 = __fadd_rn(a2, a1);
    a1 = 0.f;
    if (i & (mask << (2 * lp))) continue;
    a3 = __fadd_rn(a3, a2);
    a2 = 0.f;
  }
  for (; i < count; ++i) a0 = __fadd_rn(a0, src(first + i * stride, e));
  a0 = __fadd_rn(a0, a1);
  a0 = __fadd_rn(a0, a2);
  return __fadd_rn(a0, a3);
}

// ATen row_sum: ILP-4 over rows first + k*stride (count rows).
template <class Src>
__device__ __forceinline__ float ilp4_seq(const Src& src, int64_t e, int first, int stride,
                          int count) {
  const int q = count / 4;
  float p0 = cascade_seq(src, e, first, 4 * stride, q);
  const float p1 = cascade_seq(src, e, first + stride, 4 * stride, q);
  const float p2 = cascade_seq(src, e, first + 2 * stride, 4 * stride, q);
  const float p3 = cascade_seq(src, e, first + 3 * stride, 4 * stride, q);
  for (int i = 4 * q; i < count; ++i) p0 = __fadd_rn(p0, src(first + i * stride, e));
  p0 = __fadd_rn(p0, p1);
  p0 = __fadd_rn(p0, p2);
  return __fadd_rn(p0, p3);
}

// ATen vectorized_inner_sum (M == 1, n >= 8): 8 lanes, each an ILP-4 over
// the n/8 vectors; scalar tail into a fresh +0; then lanes 0..7 in order.
template <class Src>
__device__ __forceinline__ float inner_seq(const Src& src, int64_t e, int n) {
  if (n < 8) return ilp4_seq(src, e, 0, 1, n);
  const int nv = n / 8;
  float fin = 0.f;
  for (int k = 8 * nv; k < n; ++k) fin = __fadd_rn(fin, src(k, e));
  for (int l = 0; l < 8; ++l) fin = __fadd_rn(fin, ilp4_seq(src, e, l, 8, nv));
  return fin;
}

// Scalar tiles (ILP-4 tails, unaligned cascade columns, M == 1 keys, int64
// keys): one column walked over the N rows in its order by one thread.  Up
// to r02 each tensor's scalar columns were a tile of their own (1 to 31
// columns in a 256-thread workgroup) and each thread loaded its rows in its
// order, N dependent round trips to HBM: resnet110sl sf4 at N = 25 — 1,240
// such tiles, 0.75 % of its elements — spent 20.6 us in them against
// 21.5 us for all its vector tiles (r03, bench other_configs).  Now the
// plan packs every scalar column of the layout, sorted by kind, into tiles
// of kPackCols (K_SCALAR_PACKED; the plan's scalar index holds each
// column's bucket element and kind); a workgroup stages its columns' N
// values into LDS with independent loads (the value each order reads:
// weighted products and int64 -> fp32 conversions applied as the direct
// loads apply them), then runs each column's order from LDS.  The stage is
// 16 KB (64 columns x 64 rows at once): the 16-client kernels are VGPR-bound
// at 3 workgroups per CU (156-176 VGPRs), and the 8-client ones (91-126) at
// 4-5, which a 32 KB stage capped at 4 (measured r03: tile counts of 1,280
// ran as two rounds of 1,024, tools/archive/exp_batch_cross.py).
constexpr int kStageFloats = 4096;
struct SrcLdsCol {
  const float* stage;
  int m;    // columns staged
  int col;  // this thread's column
  __device__ float operator()(int i, int64_t) const { return stage[i * m + col]; }
};

// One scalar column's order and result (kind: K_F32_* 1-3, K_I64_* 4-6).
template <bool WEIGHTED, class SrcF, class SrcI>
__device__ __forceinline__ void scalar_column(KArgs& a, const SrcF& sf, const SrcI& si, int64_t e,
                                              int kind) {
  const int n = a.n;
  const float fn = (float)n;
  if (kind <= K_F32_INNER) {
    float s;
    if (kind == K_F32_CASC_S) s = cascade_seq(sf, e, 0, 1, n);
    else if (kind == K_F32_ILP4) s = ilp4_seq(sf, e, 0, 1, n);
    else s = inner_seq(sf, e, n);
    s = __fadd_rn(0.f, s);  // sum_out: out (=+0) += value
    const bool sum_only = WEIGHTED || (a.flags & FA_F_SUM_ONLY);
    a.out32[e] = sum_only ? s : __fdiv_rn(s, fn);
  } else {
    float s;
    if (kind == K_I64_CASC) s = cascade_seq(si, e, 0, 1, n);
    else if (kind == K_I64_ILP4) s = ilp4_seq(si, e, 0, 1, n);
    else s = inner_seq(si, e, n);
    s = __fadd_rn(0.f, s);
    // load_state_dict copy_: fp32 -> int64 truncates toward zero
    a.out64[e] = (int64_t)__fdiv_rn(s, fn);
  }
}

// A packed tile holds up to kPackCols columns, one per lane of wave 0.  The
// staging spreads the rows over the workgroup's 4 waves (wave w: rows w,
// w+4, ...; the row is wave-uniform, so its client pointer is a scalar load
// and each lane loads its column's value), 8 rows in flight per lane; then
// wave 0 runs every column's order from LDS.  More rows than fit
// kStageFloats / kPackCols: the columns in sub-batches of kStageFloats / N.
constexpr int kPackCols = 64;

// Packed tile k's entries sit at sidx[k * kPackCols, +kPackCols) (unused
// slots -1), so a scalar workgroup needs no tile descriptor: its first load
// is its entries, one dependent round trip fewer on the critical path of
// these latency-bound workgroups.
template <bool WEIGHTED>
__device__ __forceinline__ void tile_scalar_packed(KArgs& a, int k) {
  __shared__ float stage[kStageFloats];
  const int n = a.n;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t* ents = a.sidx + (int64_t)k * kPackCols;
  if (n > kStageFloats) {  // (N > 4096) direct loads, one column per lane of wave 0
    if (wv == 0) {
      const int64_t ent = ents[lane];
      if (ent >= 0)
        scalar_column<WEIGHTED>(a, SrcF32{a, WEIGHTED}, SrcI64{a}, ent >> 4, (int)(ent & 15));
    }
    return;
  }
  const int sub = min(kPackCols, kStageFloats / n);  // columns staged at once
  for (int c0 = 0; c0 < kPackCols; c0 += sub) {
    const int m = min(sub, kPackCols - c0);
    const int64_t ent = lane < m ? ents[c0 + lane] : -1;
    const bool mine = ent >= 0;
    const int64_t e = mine ? ent >> 4 : 0;
    const int kind = mine ? (int)(ent & 15) : K_F32_ILP4;
    const bool f32 = kind <= K_F32_INNER;
    constexpr int R = 8;  // rows in flight per lane
    for (int i0 = wv; i0 < n; i0 += 4 * R) {
      float x[R];
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const int r = i0 + 4 * u;
        if (r < n && mine) x[u] = f32 ? SrcF32{a, WEIGHTED}(r, e) : SrcI64{a}(r, e);
      }
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const int r = i0 + 4 * u;
        if (r < n && mine) stage[r * m + lane] = x[u];
      }
    }
    __syncthreads();
    if (wv == 0 && mine) {
      const SrcLdsCol src{stage, m, lane};
      scalar_column<WEIGHTED>(a, src, src, e, kind);
    }
    __syncthreads();
  }
}

template <int U, int B, bool DEEP, bool WEIGHTED, int POL, bool CHAIN, int PIPE = 0>
__device__ __forceinline__ void run_tile(KArgs& a, int ti) {
  if constexpr (!CHAIN) {
    if (ti < a.nscalar) {  // the packed scalar tiles lead the table
      tile_scalar_packed<WEIGHTED>(a, ti);
      return;
    }
  }
  const Tile t = a.tiles[ti];
  if (t.kind == K_F32_VEC) {
    if (t.count == 4 * U * kBlock)
      tile_vec<U, B, true, DEEP, WEIGHTED, POL, CHAIN, PIPE>(a, t.start, t.count);
    else
      tile_vec<U, B, false, DEEP, WEIGHTED, POL, CHAIN, PIPE>(a, t.start, t.count);
  }
}

// One workgroup per tile (grid == the table's tile count).  (A persistent
// grid walking the table, an occupancy cap and an XCD-contiguous tile order
// were measured slower, r01-r03; tools/reducelab.hip.)
template <int U, int B, bool DEEP, bool WEIGHTED, int POL, bool CHAIN = false, int PIPE = 0>
__global__ __launch_bounds__(kBlock) void reduce_kernel(ReduceArgs args) {
  (void)args;
  KArgs& a = *(KArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  run_tile<U, B, DEEP, WEIGHTED, POL, CHAIN, PIPE>(a, blockIdx.x);
}

// --------------------------------------------------------------- launches --
template <int U, int B, bool DEEP, bool W, int POL, bool CHAIN = false, int PIPE = 0>
hipError_t launch_one(const ReduceArgs& a, int ntiles, hipStream_t st) {
  hipLaunchKernelGGL((reduce_kernel<U, B, DEEP, W, POL, CHAIN, PIPE>), dim3(ntiles), dim3(kBlock),
                     0, st, a);
  return hipGetLastError();
}

// Chain segments (fa_reduce_chain): nt loads and stores (POL 3), the plan's
// tile width, 16-client batches for unweighted segments of >= 16 clients.
template <int U, int B>
hipError_t launch_chain_ub(const ReduceArgs& a, int ntiles, bool deep, bool w, hipStream_t st) {
  if (deep) return w ? launch_one<U, B, true, true, 3, true>(a, ntiles, st)
                     : launch_one<U, B, true, false, 3, true>(a, ntiles, st);
  return w ? launch_one<U, B, false, true, 3, true>(a, ntiles, st)
           : launch_one<U, B, false, false, 3, true>(a, ntiles, st);
}
// The reduce: nt loads, sc1 result stores (POL 5, st_out).  pipe (fedagg.hip
// pipe_rule; U = 2 only): 1 the PIPE instances over the inline pointers (not
// deep), 2 (r06) the unweighted DEEP instance over the pointer table.
template <int U, int B>
hipError_t launch_u(const ReduceArgs& a, int ntiles, bool deep, bool w, int pipe,
                    hipStream_t st) {
  if constexpr (U == 2) {
    if constexpr (B == 16)
      if (pipe == 2 && deep && !w) return launch_one<U, B, true, false, 5, false, 2>(a, ntiles, st);
    if (pipe == 1 && !deep)
      return w ? launch_one<U, B, false, true, 5, false, 1>(a, ntiles, st)
               : launch_one<U, B, false, false, 5, false, 1>(a, ntiles, st);
  } else {
    (void)pipe;
  }
  if (deep) return w ? launch_one<U, B, true, true, 5>(a, ntiles, st)
                     : launch_one<U, B, true, false, 5>(a, ntiles, st);
  return w ? launch_one<U, B, false, true, 5>(a, ntiles, st)
           : launch_one<U, B, false, false, 5>(a, ntiles, st);
}

// Resident workgroups per CU of launch_u<U, B>'s kernel for this call
// shape; 0 if the runtime cannot say.  The
// plan cuts its balanced tile tables for these counts (fedagg.hip).
template <int U, int B>
int occupancy_u(bool deep, bool w) {
  int nb = 0;
  hipError_t e;
  if (deep)
    e = w ? hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &nb, reinterpret_cast<const void*>(reduce_kernel<U, B, true, true, 5>), kBlock, 0)
          : hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &nb, reinterpret_cast<const void*>(reduce_kernel<U, B, true, false, 5>), kBlock, 0);
  else
    e = w ? hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &nb, reinterpret_cast<const void*>(reduce_kernel<U, B, false, true, 5>), kBlock, 0)
          : hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &nb, reinterpret_cast<const void*>(reduce_kernel<U, B, false, false, 5>), kBlock,
                0);
  return e == hipSuccess ? nb : 0;
}

}  // namespace fa_k

// The (U, B) launcher instantiations, each in one fedagg_k*.hip unit.
#define FA_K_LAUNCH_U(EXT, U, B)                                                      \
  EXT template hipError_t fa_k::launch_u<U, B>(const fa_k::ReduceArgs&, int, bool, bool, int, \
                                                hipStream_t);                                 \
  EXT template int fa_k::occupancy_u<U, B>(bool, bool);
#define FA_K_LAUNCH_CHAIN(EXT, U, B)                                                          \
  EXT template hipError_t fa_k::launch_chain_ub<U, B>(const fa_k::ReduceArgs&, int, bool, bool, \
                                                       hipStream_t);
#define FA_K_UNITS(EXT)                                                                  \
  FA_K_LAUNCH_U(EXT, 1, 8) FA_K_LAUNCH_U(EXT, 1, 16) FA_K_LAUNCH_CHAIN(EXT, 1, 8)       \
  FA_K_LAUNCH_U(EXT, 2, 8) FA_K_LAUNCH_CHAIN(EXT, 2, 8)                                  \
  FA_K_LAUNCH_U(EXT, 2, 16) FA_K_LAUNCH_CHAIN(EXT, 2, 16)                                \
  FA_K_LAUNCH_U(EXT, 4, 8) FA_K_LAUNCH_CHAIN(EXT, 4, 8)
