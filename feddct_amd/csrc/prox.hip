// prox.hip — FedProx proximal term on flat buckets.
//
// The reference adds, every training step of every FedProx client
// (train_fedprox.py:113-116),
//
//     proximal_term = 0.0
//     for w, w_t in zip(client_model.parameters(), global_model.parameters()):
//         proximal_term += (w - w_t).norm(2)
//     total_loss = total_loss + (mu / 2) * proximal_term
//
// i.e. one norm kernel launch (+ its backward) per parameter tensor.  Here
// the client's and the global's parameters are views of flat buckets
// (arena.py), so the whole term is two launches forward and one backward:
//
//   prox_partials : per chunk (<= 4096 floats of ONE tensor; one chunk per
//                   workgroup) the sum of (a-b)^2 with 16-B loads, wave +
//                   LDS reduction;
//   prox_finish   : one workgroup: per tensor the chunk partials in a fixed
//                   order -> sqrt -> norms[k]; sum of norms -> total
//                   (deterministic: no atomics);
//   prox_grad     : d/dw ||w - w_t|| = (w - w_t)/||w - w_t|| (0 where the
//                   norm is 0, as torch's norm backward), scaled by the
//                   incoming gradient; the global side gets the negation.
//
// HBM-bound: forward reads 2 B per element pair, backward reads 2 and writes
// 1-2.  fp32 throughout (the reference runs it in fp32 on the GPU, whose
// reduction order is not torch-CPU-defined): results agree with torch to
// fp32 rounding, not bitwise.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "common.h"

namespace {

constexpr int kBlk = 256;
constexpr int kChunk = 4096;  // floats per workgroup (4 float4 per lane)

struct NormChunk {
  int64_t start;
  int32_t count;
  int32_t seg;
};

typedef float f4 __attribute__((ext_vector_type(4)));

// Cache policy (measured, tools/archive/exp_prox_ab.py, profiles/r01_experiments.jsonl
// "prox_ab"): the forward reads the two buckets with plain loads, so the
// backward — which in a training step runs right after it (the proximal term
// is next to the loss, the first node loss.backward() reaches) — finds them
// in the 256 MB MALL; the backward reads non-temporally and writes the
// gradients non-temporally (the optimizer consumes them much later).
// Forward + backward: 43.7 us vs 54.0 us with plain loads and stores, vs
// 50.7-51.3 us with non-temporal loads in both.
constexpr bool kNtLoadFwd = false, kNtLoadBwd = true, kNtStore = true;

template <bool NT>
__device__ __forceinline__ f4 ld4(const f4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
__device__ __forceinline__ void st4(f4* p, f4 v) {
  if constexpr (kNtStore) __builtin_nontemporal_store(v, p);
  else *p = v;
}
// The gradient stores' cache policy (r04 tuning, fa_tune_prox_store): 0 nt
// (default), 1 sc1 — write-through, the line leaves the XCD's L2 (what the
// reduce's result stores use since r04, reduce_impl.h st_out).
template <int SP>
__device__ __forceinline__ void st_grad(f4* base, int i, f4 v) {
  if constexpr (SP == 0) {
    st4(base + i, v);
  } else {  // the descriptor on the uniform chunk base, the lane's offset in a VGPR
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(v, r, 16 * i, 0, 16);
  }
}
thread_local int t_prox_store = 0;
thread_local int t_prox_cpw = 0;  // tuning: chunks per forward workgroup (0: the default)

__device__ __forceinline__ float wave_sum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}


// Every lane owns kVec float4 of the chunk (lane t: vectors t, t+256, ...);
// all of them are loaded before any arithmetic, so a workgroup keeps its
// whole 2 x 16 KiB in flight.  Chunk starts are 16-B aligned (tensors start
// on 256-B boundaries in the bucket, chunks are 4096 floats); a count that is
// not a multiple of 4 finishes with scalar elements.
constexpr int kVec = kChunk / (4 * kBlk);

// The finish: per tensor the chunk partials in a fixed order -> sqrt ->
// norms[k]; the norms summed the same way -> total.  Its latency is the point
// (the work is a few thousand floats): the chunk partials and the tensor
// boundaries come in with ONE round of independent loads into LDS (when they
// fit, else they are read from global memory in the same order); then wave w
// sums tensors w, w+W, ... (lane l: partials l, l+64, ... of the tensor, then
// a shuffle tree) -> norms[k], and wave 0 sums the norms.  The order depends
// on neither the wave count nor which workgroup runs it: deterministic, no
// atomics in the arithmetic.
constexpr int kFinBlk = 1024;
constexpr int kFinLoads = 8;

// per tensor k (wave w: k = w, w + W, ...): sqrt of its partials' sum ->
// norms[k] (and NL[k] when NL is in LDS); then wave 0 sums NL -> total
template <int BLK, bool NL_LDS>
__device__ __forceinline__ void finish_compute(const float* P, const int* F, float* NL, int nseg,
                                               float* __restrict__ norms,
                                               float* __restrict__ total) {
  constexpr int kWaves = BLK / 64;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int k = wave; k < nseg; k += kWaves) {
    float sq = 0.f;
    for (int i = F[k] + lane; i < F[k + 1]; i += 64) sq += P[i];
    sq = wave_sum(sq);
    if (lane == 0) {
      const float n = sqrtf(sq);
      norms[k] = n;
      if constexpr (NL_LDS) NL[k] = n;
    }
  }
  __syncthreads();  // NL[] written by this workgroup's waves
  // the norms (a few hundred) summed by wave 0 alone: no second barrier
  if (wave == 0) {
    float t = 0.f;
    for (int k = lane; k < nseg; k += 64) t += NL[k];
    t = wave_sum(t);
    if (lane == 0) *total = t;
  }
}

template <int BLK, bool LDS>
__device__ __forceinline__ void finish_body(float* dyn, const int* __restrict__ seg_first,
                                            int nseg, int nchunks,
                                            const float* __restrict__ partials,
                                            float* __restrict__ norms, float* __restrict__ total) {
  // LDS: [nchunks partials][nseg + 1 boundaries][nseg norms]
  if constexpr (LDS) {
    float* sp = dyn;
    int* sf = reinterpret_cast<int*>(dyn + nchunks);
    // the boundaries' loads issued with the first batch of partials: one
    // round trip for both when they fit (r04)
    const int f0 = threadIdx.x <= nseg ? seg_first[threadIdx.x] : 0;
    for (int base = 0; base < nchunks; base += BLK * kFinLoads) {
      float x[kFinLoads];
#pragma unroll
      for (int i = 0; i < kFinLoads; ++i) {
        const int j = base + threadIdx.x + i * BLK;
        x[i] = j < nchunks ? partials[j] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < kFinLoads; ++i) {
        const int j = base + threadIdx.x + i * BLK;
        if (j < nchunks) sp[j] = x[i];
      }
    }
    if (threadIdx.x <= nseg) sf[threadIdx.x] = f0;
    for (int j = threadIdx.x + BLK; j <= nseg; j += BLK) sf[j] = seg_first[j];
    __syncthreads();
    finish_compute<BLK, true>(sp, sf, reinterpret_cast<float*>(sf + nseg + 1), nseg, norms,
                              total);
  } else {
    finish_compute<BLK, false>(partials, seg_first, norms, nseg, norms, total);
  }
}

// The finish: one workgroup of kFinBlk threads, the partials staged in LDS
// when they fit (else read from global memory in the same order)
template <bool LDS>
__global__ __launch_bounds__(kFinBlk) void prox_finish(const int* __restrict__ seg_first,
                                                       int nseg, int nchunks,
                                                       const float* __restrict__ partials,
                                                       float* __restrict__ norms,
                                                       float* __restrict__ total) {
  extern __shared__ float dyn[];
  finish_body<kFinBlk, LDS>(dyn, seg_first, nseg, nchunks, partials, norms, total);
}

// r04: each workgroup sums CPW consecutive chunks (each chunk's partial its
// own, so the partials — and the norms — are the same bits for every CPW),
// all CPW x 2 x 16 KiB loads in flight before any arithmetic.  CPW = 2 puts
// the 2,688-chunk grid of the wrn16_8 layout in one round of resident
// workgroups, and is slower (16.4 vs 14.7 us): default 1, the knob
// (fa_tune_prox_cpw) for other layouts.  Tried and dropped (r04): the forward as
// ONE launch whose last workgroup runs the finish — a returning atomic per
// workgroup on one counter 46 us, sharded over 8 words 24 us, partials
// tagged with a launch epoch and polled by an extra workgroup 22.6 us, the
// same poller finishing each tensor as soon as its chunks are in 24.2 us
// (partials staged in dynamic LDS) / 27.8 us (none: each poll pass is a
// chain of dependent round trips, and the poller falls behind), an
// agent-scope fence per workgroup 137 us — against 15 + 4.8 us for the two
// launches.
template <int CPW>
__global__ __launch_bounds__(kBlk) void prox_partials(const NormChunk* __restrict__ chunks,
                                                      int nchunks, const float* __restrict__ a,
                                                      const float* __restrict__ b,
                                                      float* __restrict__ partials) {
  __shared__ float lds[CPW][kBlk / 64];
  const int c0 = blockIdx.x * CPW;
  NormChunk c[CPW];
  f4 xa[CPW][kVec], xb[CPW][kVec];
#pragma unroll
  for (int k = 0; k < CPW; ++k) {
    c[k] = c0 + k < nchunks ? chunks[c0 + k] : NormChunk{0, 0, 0};
    const int nv = c[k].count / 4;
    const f4* pa = reinterpret_cast<const f4*>(a + c[k].start);
    const f4* pb = reinterpret_cast<const f4*>(b + c[k].start);
#pragma unroll
    for (int u = 0; u < kVec; ++u) {
      const int v = threadIdx.x + u * kBlk;
      const bool ok = v < nv;
      xa[k][u] = ok ? ld4<kNtLoadFwd>(pa + v) : f4{0.f, 0.f, 0.f, 0.f};
      xb[k][u] = ok ? ld4<kNtLoadFwd>(pb + v) : f4{0.f, 0.f, 0.f, 0.f};
    }
  }
  float acc[CPW];
#pragma unroll
  for (int k = 0; k < CPW; ++k) {
    acc[k] = 0.f;
#pragma unroll
    for (int u = 0; u < kVec; ++u) {
      const f4 d = xa[k][u] - xb[k][u];
      acc[k] += d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w;
    }
    for (int j = 4 * (c[k].count / 4) + threadIdx.x; j < c[k].count; j += kBlk) {
      const float d = a[c[k].start + j] - b[c[k].start + j];
      acc[k] += d * d;
    }
  }
  // the block sums, as block_sum: wave sums, then thread 0 adds the waves'
#pragma unroll
  for (int k = 0; k < CPW; ++k) acc[k] = wave_sum(acc[k]);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0)
#pragma unroll
    for (int k = 0; k < CPW; ++k) lds[k][w] = acc[k];
  __syncthreads();
  if (threadIdx.x < CPW && c0 + (int)threadIdx.x < nchunks) {
    float r = 0.f;
    for (int i = 0; i < kBlk / 64; ++i) r += lds[threadIdx.x][i];
    partials[c0 + threadIdx.x] = r;
  }
}

constexpr size_t kFinLdsMax = 64 * 1024;  // the default dynamic-LDS limit
constexpr int kCpwDefault = 1;  // chunks per forward workgroup (2: 16.4 vs 14.7 us, r04)

// ACC: the gradients are added to what the buckets hold (grad += d, one
// rounding — what autograd's AccumulateGrad does in place), for parameters
// whose .grad are views of the buckets (prox.py's one-node backward).
template <bool ACC, bool ACCB, int SP = 0>
__global__ __launch_bounds__(kBlk) void prox_grad(const NormChunk* __restrict__ chunks,
                                                  const float* __restrict__ a,
                                                  const float* __restrict__ b,
                                                  const float* __restrict__ norms,
                                                  const float* __restrict__ gout, float alpha,
                                                  float* __restrict__ ga, float* __restrict__ gb) {
  const NormChunk c = chunks[blockIdx.x];
  const float nk = norms[c.seg];
  const float g = nk > 0.f ? (*gout) * alpha / nk : 0.f;
  const int nv = c.count / 4;
  const f4* pa = reinterpret_cast<const f4*>(a + c.start);
  const f4* pb = reinterpret_cast<const f4*>(b + c.start);
  f4* qa = reinterpret_cast<f4*>(ga + c.start);
  f4* qb = reinterpret_cast<f4*>(gb + c.start);
  f4 xa[kVec], xb[kVec];
#pragma unroll
  for (int u = 0; u < kVec; ++u) {
    const int v = threadIdx.x + u * kBlk;
    const bool ok = v < nv;
    xa[u] = ok ? ld4<kNtLoadBwd>(pa + v) : f4{0.f, 0.f, 0.f, 0.f};
    xb[u] = ok ? ld4<kNtLoadBwd>(pb + v) : f4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int u = 0; u < kVec; ++u) {
    const int v = threadIdx.x + u * kBlk;
    if (v < nv) {
      const f4 d = g * (xa[u] - xb[u]);
      if constexpr (ACC) st_grad<SP>(qa, v, ld4<kNtLoadBwd>(qa + v) + d);
      else st_grad<SP>(qa, v, d);
      if constexpr (ACCB) {
        if (gb) st_grad<SP>(qb, v, ld4<kNtLoadBwd>(qb + v) - d);
      } else {
        if (gb) st_grad<SP>(qb, v, -d);
      }
    }
  }
  for (int j = 4 * nv + threadIdx.x; j < c.count; j += kBlk) {
    const int64_t e = c.start + j;
    const float d = g * (a[e] - b[e]);
    ga[e] = ACC ? ga[e] + d : d;
    if (gb) gb[e] = ACCB ? gb[e] - d : -d;
  }
}

}  // namespace

struct fa_norm_plan {
  int device = 0;
  int nseg = 0;
  int nchunks = 0;
  int64_t numel = 0;
  NormChunk* d_chunks = nullptr;
  int* d_seg_first = nullptr;
  float* d_partials = nullptr;
};

extern "C" {

int fa_norm_plan_create(const fa_seg* segs, int nseg, int64_t numel, fa_norm_plan** out) {
  if (!out) return fa::set_err(FA_E_INVAL, "fa_norm_plan_create: out is NULL");
  *out = nullptr;
  if (nseg < 0 || (nseg > 0 && !segs) || numel < 0)
    return fa::set_err(FA_E_INVAL, "fa_norm_plan_create: bad segments");
  std::vector<NormChunk> ch;
  std::vector<int> first(nseg + 1, 0);
  for (int k = 0; k < nseg; ++k) {
    first[k] = (int)ch.size();
    if (segs[k].offset < 0 || segs[k].numel < 0 || segs[k].offset + segs[k].numel > numel)
      return fa::set_err(FA_E_INVAL, "fa_norm_plan_create: segment %d outside bucket", k);
    if (segs[k].offset % 4)
      return fa::set_err(FA_E_ALIGN, "fa_norm_plan_create: segment %d not 16-B aligned", k);
    for (int64_t c = 0; c < segs[k].numel; c += kChunk)
      ch.push_back(NormChunk{segs[k].offset + c, (int32_t)std::min<int64_t>(kChunk, segs[k].numel - c), k});
  }
  first[nseg] = (int)ch.size();
  fa_norm_plan* p = new fa_norm_plan();
  p->nseg = nseg;
  p->nchunks = (int)ch.size();
  p->numel = numel;
  hipError_t e = hipGetDevice(&p->device);
  if (e == hipSuccess && !ch.empty()) e = hipMalloc(&p->d_chunks, ch.size() * sizeof(NormChunk));
  if (e == hipSuccess) e = hipMalloc(&p->d_seg_first, first.size() * sizeof(int));
  if (e == hipSuccess && !ch.empty()) e = hipMalloc(&p->d_partials, ch.size() * sizeof(float));
  if (e == hipSuccess && !ch.empty())
    e = hipMemcpy(p->d_chunks, ch.data(), ch.size() * sizeof(NormChunk), hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = hipMemcpy(p->d_seg_first, first.data(), first.size() * sizeof(int), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(p->d_chunks);
    (void)hipFree(p->d_seg_first);
    (void)hipFree(p->d_partials);
    delete p;
    return fa::set_err(FA_E_HIP, "fa_norm_plan_create: %s", hipGetErrorString(e));
  }
  *out = p;
  return FA_OK;
}

int fa_norm_plan_destroy(fa_norm_plan* p) {
  if (!p) return FA_OK;
  FA_HIP_TRY(hipFree(p->d_chunks));
  FA_HIP_TRY(hipFree(p->d_seg_first));
  FA_HIP_TRY(hipFree(p->d_partials));
  delete p;
  return FA_OK;
}

int fa_prox_norms(const fa_norm_plan* p, const float* a, const float* b, float* norms,
                  float* total, void* stream) {
  if (!p || !a || !b || !norms || !total) return fa::set_err(FA_E_INVAL, "fa_prox_norms: NULL argument");
  if (((uintptr_t)a | (uintptr_t)b) & 15u)
    return fa::set_err(FA_E_ALIGN, "fa_prox_norms: buckets must be 16-B aligned");
  hipStream_t st = (hipStream_t)stream;
  if (p->nchunks > 0) {
    const int cpw = t_prox_cpw > 0 ? t_prox_cpw : kCpwDefault;
    const unsigned grid = (unsigned)((p->nchunks + cpw - 1) / cpw);
    switch (cpw) {
      case 1: hipLaunchKernelGGL(prox_partials<1>, dim3(grid), dim3(kBlk), 0, st, p->d_chunks,
                                 p->nchunks, a, b, p->d_partials); break;
      case 3: hipLaunchKernelGGL(prox_partials<3>, dim3(grid), dim3(kBlk), 0, st, p->d_chunks,
                                 p->nchunks, a, b, p->d_partials); break;
      case 4: hipLaunchKernelGGL(prox_partials<4>, dim3(grid), dim3(kBlk), 0, st, p->d_chunks,
                                 p->nchunks, a, b, p->d_partials); break;
      default: hipLaunchKernelGGL(prox_partials<2>, dim3(grid), dim3(kBlk), 0, st, p->d_chunks,
                                  p->nchunks, a, b, p->d_partials); break;
    }
    FA_HIP_TRY(hipGetLastError());
  }
  const size_t lds = (size_t)(p->nchunks + 2 * p->nseg + 1) * 4;
  if (lds <= kFinLdsMax)
    hipLaunchKernelGGL(prox_finish<true>, dim3(1), dim3(kFinBlk), lds, st, p->d_seg_first,
                       p->nseg, p->nchunks, p->d_partials, norms, total);
  else
    hipLaunchKernelGGL(prox_finish<false>, dim3(1), dim3(kFinBlk), 0, st, p->d_seg_first,
                       p->nseg, p->nchunks, p->d_partials, norms, total);
  FA_HIP_TRY(hipGetLastError());
  return FA_OK;
}

int fa_tune_prox_cpw(int cpw) {
  if (cpw < 0 || cpw > 4) return fa::set_err(FA_E_INVAL, "fa_tune_prox_cpw: %d", cpw);
  const int old = t_prox_cpw;
  t_prox_cpw = cpw;
  return old;
}

int fa_tune_prox_store(int policy) {
  if (policy < 0 || policy > 1) return fa::set_err(FA_E_INVAL, "fa_tune_prox_store: %d", policy);
  const int old = t_prox_store;
  t_prox_store = policy;
  return old;
}

int fa_prox_grad(const fa_norm_plan* p, const float* a, const float* b, const float* norms,
                 const float* gout, float alpha, float* grad_a, float* grad_b, void* stream) {
  return fa_prox_grad_ex(p, a, b, norms, gout, alpha, grad_a, grad_b, 0, stream);
}

int fa_prox_grad_ex(const fa_norm_plan* p, const float* a, const float* b, const float* norms,
                    const float* gout, float alpha, float* grad_a, float* grad_b,
                    unsigned flags, void* stream) {
  if (!p || !a || !b || !norms || !gout || !grad_a)
    return fa::set_err(FA_E_INVAL, "fa_prox_grad: NULL argument");
  if (flags & ~(FA_PROX_ACCUMULATE | FA_PROX_ACCUMULATE_A | FA_PROX_ACCUMULATE_B))
    return fa::set_err(FA_E_INVAL, "fa_prox_grad_ex: bad flags");
  if (((uintptr_t)a | (uintptr_t)b | (uintptr_t)grad_a | (uintptr_t)grad_b) & 15u)
    return fa::set_err(FA_E_ALIGN, "fa_prox_grad: buckets must be 16-B aligned");
  if (p->nchunks == 0) return FA_OK;
  // per side: accumulate into the bound .grad, or overwrite (a side whose
  // .grad were all None: no memset of its bucket first)
  const bool acc_a = flags & (FA_PROX_ACCUMULATE | FA_PROX_ACCUMULATE_A);
  const bool acc_b = flags & (FA_PROX_ACCUMULATE | FA_PROX_ACCUMULATE_B);
  auto k = acc_a ? (acc_b ? prox_grad<true, true> : prox_grad<true, false>)
                 : (acc_b ? prox_grad<false, true> : prox_grad<false, false>);
  if (t_prox_store == 1)
    k = acc_a ? (acc_b ? prox_grad<true, true, 1> : prox_grad<true, false, 1>)
              : (acc_b ? prox_grad<false, true, 1> : prox_grad<false, false, 1>);
  hipLaunchKernelGGL(k, dim3(p->nchunks), dim3(kBlk), 0, (hipStream_t)stream, p->d_chunks, a, b,
                     norms, gout, alpha, grad_a, grad_b);
  FA_HIP_TRY(hipGetLastError());
  return FA_OK;
}

}  // extern "C"
