// fedcomm.hip — libfedagg_comm.so: aggregation across the GPUs of one node
// over RCCL (include/fedagg_comm.h; SURVEY.md §8 b, e1, e2).
//
// Layering: this library uses only libfedagg.so's public ABI for the
// arithmetic (fa_plan_build_host to enumerate the layout's tiles,
// fa_plan_create_from_tiles for tile subsets, fa_reduce for the reductions,
// fa_div_f32 for the /N finish) and adds the exchanges:
//   e1 (fa_reduce_sharded): one ncclReduce / ncclAllReduce per column chunk
//      on an internal communication stream, issued as soon as the kernel
//      over that chunk is done, so the exchange of chunk c overlaps the
//      reduction of chunk c+1;
//   e2 (fa_reduce_striped): grouped ncclSend/ncclRecv move every client's
//      values for rank r's column stripe to rank r, which reduces its stripe
//      over all clients in the exact order; the stripes then travel to the
//      root (or to every rank).  Bit-identical to one GPU.
// RCCL resolves to the librccl.so.1 torch has already loaded (same soname),
// so a process holds one RCCL.

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../../include/fedagg_comm.h"
#include "common.h"

static_assert(sizeof(ncclUniqueId) == FA_COMM_UID_BYTES, "unique id size");

using fa::set_err;

#define NCCL_TRY(expr)                                                          \
  do {                                                                          \
    ncclResult_t r_ = (expr);                                                   \
    if (r_ != ncclSuccess)                                                      \
      return set_err(FA_E_COMM, "%s: %s", #expr, ncclGetErrorString(r_));      \
  } while (0)

struct fa_comm {
  ncclComm_t nc = nullptr;
  int nranks = 0, rank = 0, device = 0;
  hipStream_t cs = nullptr;  // communication stream
};

namespace {

// ------------------------------------------------------------ int64 keys --
// The int64 keys (num_batches_tracked) are a few bytes per client: every
// rank's buckets are stacked into rows, all-gathered raw, and the result
// ranks reduce all n_total rows exactly (slot order = rank order).
constexpr int kStackPtrs = 64;
struct StackArgs {
  const int64_t* src[kStackPtrs];
  int64_t* dst;
  int64_t width;
  int rows;
};
__global__ void stack_i64_kernel(StackArgs a) {
  const int r = blockIdx.y;
  if (r >= a.rows) return;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < a.width;
       e += (int64_t)gridDim.x * blockDim.x)
    a.dst[r * a.width + e] = a.src[r][e];
}

struct I64Part {
  fa_plan* plan = nullptr;  // the int64 tiles (nullptr: no int64 keys)
  int64_t* stack = nullptr;   // nmax rows of width
  int64_t* gather = nullptr;  // nranks * nmax rows
  std::vector<const int64_t*> rows;  // the n_total real rows, slot order
  int nmax = 0;
  int64_t width = 0;

  int init(const fa_comm* c, const std::vector<fa_tile_desc>& t64, const int* counts,
           int64_t f32_numel, int64_t i64_numel, unsigned flags) {
    if (t64.empty()) return FA_OK;
    int rc = fa_plan_create_from_tiles(t64.data(), (int)t64.size(), f32_numel, i64_numel, 0,
                                       flags, &plan);
    if (rc) return rc;
    width = i64_numel;
    for (int r = 0; r < c->nranks; ++r) nmax = std::max(nmax, counts[r]);
    const size_t row = (size_t)width * 8;
    FA_HIP_TRY(hipMalloc(&stack, std::max<size_t>(1, (size_t)nmax * row)));
    FA_HIP_TRY(hipMalloc(&gather, std::max<size_t>(1, (size_t)nmax * c->nranks * row)));
    for (int r = 0; r < c->nranks; ++r)
      for (int j = 0; j < counts[r]; ++j)
        rows.push_back(gather + ((size_t)r * nmax + j) * width);
    return FA_OK;
  }
  void release() {
    fa_plan_destroy(plan);
    if (stack) (void)hipFree(stack);
    if (gather) (void)hipFree(gather);
    plan = nullptr;
    stack = gather = nullptr;
  }
  // stack this rank's n_local buckets on stream s
  int stack_local(const int64_t* const* c64, int n_local, hipStream_t s) {
    for (int j0 = 0; j0 < n_local; j0 += kStackPtrs) {
      StackArgs a;
      memset(&a, 0, sizeof a);
      a.rows = std::min(kStackPtrs, n_local - j0);
      for (int j = 0; j < a.rows; ++j) a.src[j] = c64[j0 + j];
      a.dst = stack + (size_t)j0 * width;
      a.width = width;
      const int gx = (int)std::min<int64_t>(64, (width + 255) / 256);
      hipLaunchKernelGGL(stack_i64_kernel, dim3(gx, a.rows), dim3(256), 0, s, a);
      FA_HIP_TRY(hipGetLastError());
    }
    return FA_OK;
  }
};

// ------------------------------------------------------------ tile cuts --
// The layout's fp32 tiles sorted by start, and its int64 tiles.
int layout_tiles(const fa_seg* seg32, int nseg32, int64_t f32_numel, const fa_seg* seg64,
                 int nseg64, int64_t i64_numel, unsigned flags, std::vector<fa_tile_desc>* t32,
                 std::vector<fa_tile_desc>* t64) {
  fa_plan_info info{};
  int rc = fa_plan_build_host(seg32, nseg32, f32_numel, seg64, nseg64, i64_numel, 0, flags,
                              nullptr, 0, &info);
  if (rc) return rc;
  std::vector<fa_tile_desc> tiles(std::max(1, info.ntiles));
  rc = fa_plan_build_host(seg32, nseg32, f32_numel, seg64, nseg64, i64_numel, 0, flags,
                          tiles.data(), info.ntiles, &info);
  if (rc) return rc;
  tiles.resize(info.ntiles);
  for (const fa_tile_desc& t : tiles) (t.kind >= 4 ? t64 : t32)->push_back(t);
  std::sort(t32->begin(), t32->end(),
            [](const fa_tile_desc& a, const fa_tile_desc& b) { return a.start < b.start; });
  return FA_OK;
}

// k contiguous groups of the sorted fp32 tiles with equal shares of the
// elements, cut only before a vector tile on a 256-B boundary (so every
// group's byte range starts aligned); exactly k groups, trailing ones may be
// empty.  Group g = tiles [cut[g], cut[g+1]), byte range [lo[g], lo[g+1])
// with lo[0] = 0 and lo[k] = f32_numel (the padding between tensors is
// covered, FA_PLAN_GAPS_ARE_PADDING).
void cut_tiles(const std::vector<fa_tile_desc>& t32, int k, int64_t f32_numel,
               std::vector<size_t>* cut, std::vector<int64_t>* lo) {
  int64_t total = 0;
  for (const fa_tile_desc& t : t32) total += t.count;
  cut->assign(1, 0);
  int64_t acc = 0;
  for (size_t i = 0; i < t32.size(); ++i) {
    const int c = (int)cut->size();
    if (c < k && i > 0 && acc >= total * c / k && t32[i].kind == 0 && t32[i].start % 64 == 0)
      cut->push_back(i);
    acc += t32[i].count;
  }
  while ((int)cut->size() < k + 1) cut->push_back(t32.size());
  lo->assign(k + 1, f32_numel);
  (*lo)[0] = 0;
  for (int g = 1; g < k; ++g)
    (*lo)[g] = (*cut)[g] < t32.size() ? t32[(*cut)[g]].start : f32_numel;
}

struct DeviceGuard {
  int prev = -1;
  DeviceGuard() { (void)hipGetDevice(&prev); }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

int make_comm(ncclComm_t nc, int device, fa_comm** out) {
  fa_comm* c = new fa_comm();
  c->nc = nc;
  c->device = device;
  ncclResult_t r = ncclCommCount(nc, &c->nranks);
  if (r == ncclSuccess) r = ncclCommUserRank(nc, &c->rank);
  if (r != ncclSuccess) {
    delete c;
    return set_err(FA_E_COMM, "ncclCommCount/UserRank: %s", ncclGetErrorString(r));
  }
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->cs, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    return set_err(FA_E_HIP, "comm stream: %s", hipGetErrorString(e));
  }
  *out = c;
  return FA_OK;
}

int slot_layout(const fa_comm* comm, const int* counts, int* n_total, int* lo_slot,
                const char* who) {
  *n_total = 0;
  *lo_slot = 0;
  for (int r = 0; r < comm->nranks; ++r) {
    if (counts[r] < 0) return set_err(FA_E_INVAL, "%s: counts[%d]=%d", who, r, counts[r]);
    if (r < comm->rank) *lo_slot += counts[r];
    *n_total += counts[r];
  }
  if (*n_total < 1 || *n_total > FA_MAX_CLIENTS)
    return set_err(FA_E_RANGE, "%s: %d clients in total", who, *n_total);
  return FA_OK;
}

int make_events(std::vector<hipEvent_t>* ev, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    hipEvent_t e;
    FA_HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ev->push_back(e);
  }
  return FA_OK;
}

}  // namespace

struct fa_shard_plan {
  fa_comm* comm = nullptr;
  int64_t f32_numel = 0, i64_numel = 0;
  int n_local = 0, n_total = 0, lo_slot = 0;
  std::vector<fa_plan*> chunk;                     // tile subset per column chunk
  std::vector<std::pair<int64_t, int64_t>> range;  // [lo, hi) of each chunk
  float* partial = nullptr;                        // f32_numel (library scratch)
  I64Part i64;
  std::vector<hipEvent_t> ev;  // per chunk (+ int64, + done)
};

struct fa_stripe_plan {
  fa_comm* comm = nullptr;
  int64_t f32_numel = 0, i64_numel = 0;
  int n_local = 0, n_total = 0, lo_slot = 0;
  std::vector<int> counts, first_slot;  // per rank
  std::vector<int64_t> lo;              // nranks + 1 stripe bounds
  fa_plan* stripe = nullptr;            // this rank's stripe tiles (nullptr: empty)
  int64_t row = 0;                      // recv row stride (floats, 64-aligned)
  float* recv = nullptr;                // n_total rows of the stripe
  float* sbuf = nullptr;                // the reduced stripe
  std::vector<const float*> ptrs;       // the n_total source pointers (see create)
  I64Part i64;
  std::vector<hipEvent_t> ev;  // start, int64, done
};

namespace {
void free_shard(fa_shard_plan* p) {
  if (!p) return;
  DeviceGuard g;
  if (p->comm) (void)hipSetDevice(p->comm->device);
  for (fa_plan* c : p->chunk) fa_plan_destroy(c);
  if (p->partial) (void)hipFree(p->partial);
  p->i64.release();
  for (hipEvent_t e : p->ev) (void)hipEventDestroy(e);
  delete p;
}
void free_stripe(fa_stripe_plan* p) {
  if (!p) return;
  DeviceGuard g;
  if (p->comm) (void)hipSetDevice(p->comm->device);
  fa_plan_destroy(p->stripe);
  if (p->recv) (void)hipFree(p->recv);
  if (p->sbuf) (void)hipFree(p->sbuf);
  p->i64.release();
  for (hipEvent_t e : p->ev) (void)hipEventDestroy(e);
  delete p;
}

// int64 keys after the local buckets are stacked on stream s: all-gather
// (grouped over the local GPUs by the caller) happens in run_i64_exchange.
int i64_exchange(I64Part* const* parts, const fa_comm* const* comms, int nlocal) {
  NCCL_TRY(ncclGroupStart());
  for (int d = 0; d < nlocal; ++d) {
    (void)hipSetDevice(comms[d]->device);
    ncclResult_t r = ncclAllGather(parts[d]->stack, parts[d]->gather,
                                   (size_t)parts[d]->nmax * parts[d]->width, ncclInt64,
                                   comms[d]->nc, comms[d]->cs);
    if (r != ncclSuccess) {
      ncclGroupEnd();
      return set_err(FA_E_COMM, "int64 all-gather: %s", ncclGetErrorString(r));
    }
  }
  NCCL_TRY(ncclGroupEnd());
  return FA_OK;
}
}  // namespace

// fa_mean_f32_multi's shard plans, by (communicator, layout, counts); a
// communicator's entries go with it (fa_comm_destroy).
namespace {
std::mutex g_multi_mu;
std::map<std::string, fa_shard_plan*> g_multi;
}  // namespace

extern "C" {

int fa_comm_unique_id(unsigned char* id, int len) {
  if (!id || len < FA_COMM_UID_BYTES)
    return set_err(FA_E_INVAL, "fa_comm_unique_id: need a %d-byte buffer", FA_COMM_UID_BYTES);
  ncclUniqueId u;
  NCCL_TRY(ncclGetUniqueId(&u));
  memcpy(id, &u, sizeof u);
  return FA_OK;
}

int fa_comm_init_rank(int nranks, int rank, const unsigned char* id, int len, fa_comm** out) {
  if (!out) return set_err(FA_E_INVAL, "fa_comm_init_rank: out is NULL");
  *out = nullptr;
  if (!id || len < FA_COMM_UID_BYTES || nranks < 1 || rank < 0 || rank >= nranks)
    return set_err(FA_E_INVAL, "fa_comm_init_rank: bad arguments (nranks=%d rank=%d)", nranks,
                   rank);
  int dev = 0;
  FA_HIP_TRY(hipGetDevice(&dev));
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  ncclComm_t nc = nullptr;
  NCCL_TRY(ncclCommInitRank(&nc, nranks, u, rank));
  const int rc = make_comm(nc, dev, out);
  if (rc) ncclCommDestroy(nc);
  return rc;
}

int fa_comm_init(int ndev, const int* devs, fa_comm** comms) {
  if (ndev < 1 || !devs || !comms) return set_err(FA_E_INVAL, "fa_comm_init: bad arguments");
  DeviceGuard g;
  std::vector<ncclComm_t> nc(ndev, nullptr);
  NCCL_TRY(ncclCommInitAll(nc.data(), ndev, devs));
  for (int i = 0; i < ndev; ++i) comms[i] = nullptr;
  for (int i = 0; i < ndev; ++i) {
    const int rc = make_comm(nc[i], devs[i], &comms[i]);
    if (rc) {
      for (int j = 0; j < ndev; ++j) {
        if (comms[j]) fa_comm_destroy(comms[j]), comms[j] = nullptr;
        else if (j >= i) ncclCommDestroy(nc[j]);
      }
      return rc;
    }
  }
  return FA_OK;
}

int fa_comm_destroy(fa_comm* c) {
  if (!c) return FA_OK;
  {
    std::lock_guard<std::mutex> lk(g_multi_mu);
    for (auto it = g_multi.begin(); it != g_multi.end();) {
      if (it->second->comm == c) {
        free_shard(it->second);
        it = g_multi.erase(it);
      } else {
        ++it;
      }
    }
  }
  DeviceGuard g;
  (void)hipSetDevice(c->device);
  if (c->cs) (void)hipStreamDestroy(c->cs);
  ncclResult_t r = c->nc ? ncclCommDestroy(c->nc) : ncclSuccess;
  delete c;
  if (r != ncclSuccess) return set_err(FA_E_COMM, "ncclCommDestroy: %s", ncclGetErrorString(r));
  return FA_OK;
}

int fa_comm_info(const fa_comm* c, int* nranks, int* rank, int* device) {
  if (!c) return set_err(FA_E_INVAL, "fa_comm_info: comm is NULL");
  if (nranks) *nranks = c->nranks;
  if (rank) *rank = c->rank;
  if (device) *device = c->device;
  return FA_OK;
}

// ============================================================== e1 ========
int fa_shard_plan_create(fa_comm* comm, const fa_seg* seg32, int nseg32, int64_t f32_numel,
                         const fa_seg* seg64, int nseg64, int64_t i64_numel, const int* counts,
                         int nchunks, unsigned flags, fa_shard_plan** out) {
  if (!out) return set_err(FA_E_INVAL, "fa_shard_plan_create: out is NULL");
  *out = nullptr;
  if (!comm || !counts) return set_err(FA_E_INVAL, "fa_shard_plan_create: NULL comm/counts");
  if (!(flags & FA_PLAN_GAPS_ARE_PADDING))
    return set_err(FA_E_INVAL,
                   "fa_shard_plan_create: the layout must allow writes to its padding "
                   "(FA_PLAN_GAPS_ARE_PADDING): chunk exchanges span it");
  if (nchunks == 0) nchunks = 8;
  if (nchunks < 1 || nchunks > FA_COMM_MAX_CHUNKS)
    return set_err(FA_E_INVAL, "fa_shard_plan_create: nchunks=%d", nchunks);
  int n_total = 0, lo_slot = 0;
  int rc = slot_layout(comm, counts, &n_total, &lo_slot, "fa_shard_plan_create");
  if (rc) return rc;
  DeviceGuard g;
  FA_HIP_TRY(hipSetDevice(comm->device));
  std::vector<fa_tile_desc> t32, t64;
  rc = layout_tiles(seg32, nseg32, f32_numel, seg64, nseg64, i64_numel, flags, &t32, &t64);
  if (rc) return rc;

  fa_shard_plan* p = new fa_shard_plan();
  p->comm = comm;
  p->f32_numel = f32_numel;
  p->i64_numel = i64_numel;
  p->n_local = counts[comm->rank];
  p->n_total = n_total;
  p->lo_slot = lo_slot;
  if (!t32.empty()) {
    std::vector<size_t> cut;
    std::vector<int64_t> lo;
    cut_tiles(t32, nchunks, f32_numel, &cut, &lo);
    for (int c = 0; c < nchunks; ++c) {
      if (cut[c] == cut[c + 1]) continue;  // empty trailing group
      fa_plan* sub = nullptr;
      rc = fa_plan_create_from_tiles(t32.data() + cut[c], (int)(cut[c + 1] - cut[c]),
                                     f32_numel, i64_numel, 0, flags, &sub);
      if (rc) {
        free_shard(p);
        return rc;
      }
      p->chunk.push_back(sub);
      // the last non-empty chunk's exchange runs to the end of the bucket
      p->range.emplace_back(lo[c], lo[c + 1]);
    }
    p->range.back().second = f32_numel;
    hipError_t e = hipMalloc(&p->partial, (size_t)f32_numel * 4);
    if (e == hipSuccess) e = hipMemset(p->partial, 0, (size_t)f32_numel * 4);
    if (e != hipSuccess) {
      free_shard(p);
      return set_err(FA_E_HIP, "fa_shard_plan_create: %s", hipGetErrorString(e));
    }
  }
  rc = p->i64.init(comm, t64, counts, f32_numel, i64_numel, flags);
  if (!rc) rc = make_events(&p->ev, p->chunk.size() + 2);
  if (rc) {
    free_shard(p);
    return rc;
  }
  *out = p;
  return FA_OK;
}

int fa_shard_plan_destroy(fa_shard_plan* p) {
  free_shard(p);
  return FA_OK;
}

int fa_reduce_sharded(fa_shard_plan* const* plans, int nlocal, const fa_shard_io* io, int root) {
  if (nlocal < 1 || !plans || !io) return set_err(FA_E_INVAL, "fa_reduce_sharded: bad arguments");
  const bool weighted = io[0].weights != nullptr;
  for (int d = 0; d < nlocal; ++d) {
    const fa_shard_plan* p = plans[d];
    if (!p) return set_err(FA_E_INVAL, "fa_reduce_sharded: plan %d is NULL", d);
    if (root >= p->comm->nranks) return set_err(FA_E_INVAL, "fa_reduce_sharded: root=%d", root);
    if ((io[d].weights != nullptr) != weighted)
      return set_err(FA_E_INVAL, "fa_reduce_sharded: weights on some GPUs only");
    const bool result = root < 0 || root == p->comm->rank;
    if (p->n_local > 0 && !p->chunk.empty() && !io[d].c32)
      return set_err(FA_E_INVAL, "fa_reduce_sharded: fp32 buckets required (GPU %d)", d);
    if (p->n_local > 0 && p->i64.plan && !io[d].c64)
      return set_err(FA_E_INVAL, "fa_reduce_sharded: int64 buckets required (GPU %d)", d);
    if (result && ((!p->chunk.empty() && !io[d].out32) || (p->i64.plan && !io[d].out64)))
      return set_err(FA_E_INVAL, "fa_reduce_sharded: result buckets required on rank %d",
                     p->comm->rank);
    if (p->chunk.size() != plans[0]->chunk.size())
      return set_err(FA_E_INVAL, "fa_reduce_sharded: plans of different layouts");
  }
  DeviceGuard g;
  const size_t nch = plans[0]->chunk.size();
  for (size_t c = 0; c < nch; ++c) {
    // partial sums of chunk c on every local GPU, then its exchange
    for (int d = 0; d < nlocal; ++d) {
      fa_shard_plan* p = plans[d];
      hipStream_t s = (hipStream_t)io[d].stream;
      FA_HIP_TRY(hipSetDevice(p->comm->device));
      if (p->n_local > 0) {
        const int rc = fa_reduce(p->chunk[c], io[d].c32, nullptr, p->n_local, io[d].weights,
                                 p->partial, nullptr, FA_F_SUM_ONLY, s);
        if (rc) return rc;
      }
      FA_HIP_TRY(hipEventRecord(p->ev[c], s));
      FA_HIP_TRY(hipStreamWaitEvent(p->comm->cs, p->ev[c], 0));
    }
    NCCL_TRY(ncclGroupStart());
    for (int d = 0; d < nlocal; ++d) {
      fa_shard_plan* p = plans[d];
      (void)hipSetDevice(p->comm->device);
      const int64_t lo = p->range[c].first, cnt = p->range[c].second - lo;
      const bool result = root < 0 || root == p->comm->rank;
      float* dst = result ? io[d].out32 + lo : p->partial + lo;
      ncclResult_t r = root < 0
          ? ncclAllReduce(p->partial + lo, dst, (size_t)cnt, ncclFloat32, ncclSum, p->comm->nc,
                          p->comm->cs)
          : ncclReduce(p->partial + lo, dst, (size_t)cnt, ncclFloat32, ncclSum, root,
                       p->comm->nc, p->comm->cs);
      if (r != ncclSuccess) {
        ncclGroupEnd();
        return set_err(FA_E_COMM, "chunk %zu exchange: %s", c, ncclGetErrorString(r));
      }
    }
    NCCL_TRY(ncclGroupEnd());
    if (!weighted) {
      for (int d = 0; d < nlocal; ++d) {
        fa_shard_plan* p = plans[d];
        if (!(root < 0 || root == p->comm->rank)) continue;
        FA_HIP_TRY(hipSetDevice(p->comm->device));
        const int64_t lo = p->range[c].first, cnt = p->range[c].second - lo;
        const int rc = fa_div_f32(io[d].out32 + lo, (float)p->n_total, io[d].out32 + lo, cnt,
                                  p->comm->cs);
        if (rc) return rc;
      }
    }
  }
  if (plans[0]->i64.plan) {
    std::vector<I64Part*> parts;
    std::vector<const fa_comm*> comms;
    for (int d = 0; d < nlocal; ++d) {
      fa_shard_plan* p = plans[d];
      hipStream_t s = (hipStream_t)io[d].stream;
      FA_HIP_TRY(hipSetDevice(p->comm->device));
      int rc = p->i64.stack_local(io[d].c64, p->n_local, s);
      if (rc) return rc;
      FA_HIP_TRY(hipEventRecord(p->ev[nch], s));
      FA_HIP_TRY(hipStreamWaitEvent(p->comm->cs, p->ev[nch], 0));
      parts.push_back(&p->i64);
      comms.push_back(p->comm);
    }
    int rc = i64_exchange(parts.data(), comms.data(), nlocal);
    if (rc) return rc;
    for (int d = 0; d < nlocal; ++d) {
      fa_shard_plan* p = plans[d];
      if (!(root < 0 || root == p->comm->rank)) continue;
      FA_HIP_TRY(hipSetDevice(p->comm->device));
      rc = fa_reduce(p->i64.plan, nullptr, p->i64.rows.data(), p->n_total, nullptr, nullptr,
                     io[d].out64, 0, p->comm->cs);
      if (rc) return rc;
    }
  }
  // the caller's stream joins the communication stream
  for (int d = 0; d < nlocal; ++d) {
    fa_shard_plan* p = plans[d];
    FA_HIP_TRY(hipSetDevice(p->comm->device));
    hipEvent_t done = p->ev[nch + 1];
    FA_HIP_TRY(hipEventRecord(done, p->comm->cs));
    FA_HIP_TRY(hipStreamWaitEvent((hipStream_t)io[d].stream, done, 0));
  }
  return FA_OK;
}

// Stateless form (SURVEY.md §8 b's fa_mean_f32_multi): fp32 segments only,
// shard plans cached per (communicator, layout, counts); 8 chunks.
int fa_mean_f32_multi(fa_comm* comm, const float* const* clients, const int* counts,
                      int64_t numel, float* out, const fa_seg* segs, int nseg, int root,
                      void* stream) {
  if (!comm || !counts) return set_err(FA_E_INVAL, "fa_mean_f32_multi: NULL comm/counts");
  if (nseg < 0 || (nseg > 0 && !segs)) return set_err(FA_E_INVAL, "fa_mean_f32_multi: segs");
  std::string key((const char*)&comm, sizeof comm);
  key.append((const char*)&numel, sizeof numel);
  key.append((const char*)counts, sizeof(int) * comm->nranks);
  if (nseg > 0) key.append((const char*)segs, sizeof(fa_seg) * nseg);
  fa_shard_plan* plan = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_multi_mu);
    auto it = g_multi.find(key);
    if (it != g_multi.end()) {
      plan = it->second;
    } else {
      const int rc = fa_shard_plan_create(comm, segs, nseg, numel, nullptr, 0, 0, counts, 8,
                                          FA_PLAN_GAPS_ARE_PADDING, &plan);
      if (rc) return rc;
      g_multi[key] = plan;
    }
  }
  fa_shard_io io{};
  io.c32 = clients;
  io.out32 = out;
  io.stream = stream;
  return fa_reduce_sharded(&plan, 1, &io, root);
}

// ============================================================== e2 ========
int fa_stripe_plan_create(fa_comm* comm, const fa_seg* seg32, int nseg32, int64_t f32_numel,
                          const fa_seg* seg64, int nseg64, int64_t i64_numel, const int* counts,
                          unsigned flags, fa_stripe_plan** out) {
  if (!out) return set_err(FA_E_INVAL, "fa_stripe_plan_create: out is NULL");
  *out = nullptr;
  if (!comm || !counts) return set_err(FA_E_INVAL, "fa_stripe_plan_create: NULL comm/counts");
  if (!(flags & FA_PLAN_GAPS_ARE_PADDING))
    return set_err(FA_E_INVAL,
                   "fa_stripe_plan_create: the layout must allow writes to its padding "
                   "(FA_PLAN_GAPS_ARE_PADDING): stripe exchanges span it");
  int n_total = 0, lo_slot = 0;
  int rc = slot_layout(comm, counts, &n_total, &lo_slot, "fa_stripe_plan_create");
  if (rc) return rc;
  DeviceGuard g;
  FA_HIP_TRY(hipSetDevice(comm->device));
  std::vector<fa_tile_desc> t32, t64;
  rc = layout_tiles(seg32, nseg32, f32_numel, seg64, nseg64, i64_numel, flags, &t32, &t64);
  if (rc) return rc;

  fa_stripe_plan* p = new fa_stripe_plan();
  p->comm = comm;
  p->f32_numel = f32_numel;
  p->i64_numel = i64_numel;
  p->n_local = counts[comm->rank];
  p->n_total = n_total;
  p->lo_slot = lo_slot;
  p->counts.assign(counts, counts + comm->nranks);
  int s0 = 0;
  for (int r = 0; r < comm->nranks; ++r) {
    p->first_slot.push_back(s0);
    s0 += counts[r];
  }
  std::vector<size_t> cut;
  cut_tiles(t32, comm->nranks, f32_numel, &cut, &p->lo);
  const int me = comm->rank;
  const int64_t L = p->lo[me + 1] - p->lo[me];
  hipError_t e = hipSuccess;
  if (cut[me] < cut[me + 1]) {
    rc = fa_plan_create_from_tiles(t32.data() + cut[me], (int)(cut[me + 1] - cut[me]),
                                   f32_numel, i64_numel, 0, flags, &p->stripe);
    if (rc) {
      free_stripe(p);
      return rc;
    }
    // one row per client slot (local rows unused), 256-B aligned rows; the
    // stripe starts on a 64-float boundary, so (row - lo) stays aligned
    p->row = (L + 63) / 64 * 64;
    e = hipMalloc(&p->recv, (size_t)n_total * p->row * 4);
    if (e == hipSuccess) e = hipMalloc(&p->sbuf, (size_t)p->row * 4);
    if (e == hipSuccess) e = hipMemset(p->sbuf, 0, (size_t)p->row * 4);
    for (int k = 0; e == hipSuccess && k < n_total; ++k)
      p->ptrs.push_back(p->recv + (size_t)k * p->row - p->lo[me]);  // element e at [e - lo]
  }
  if (e != hipSuccess) {
    free_stripe(p);
    return set_err(FA_E_HIP, "fa_stripe_plan_create: %s", hipGetErrorString(e));
  }
  rc = p->i64.init(comm, t64, counts, f32_numel, i64_numel, flags);
  if (!rc) rc = make_events(&p->ev, 3);
  if (rc) {
    free_stripe(p);
    return rc;
  }
  *out = p;
  return FA_OK;
}

int fa_stripe_plan_destroy(fa_stripe_plan* p) {
  free_stripe(p);
  return FA_OK;
}

int fa_reduce_striped(fa_stripe_plan* const* plans, int nlocal, const fa_shard_io* io,
                      int root) {
  if (nlocal < 1 || !plans || !io) return set_err(FA_E_INVAL, "fa_reduce_striped: bad arguments");
  for (int d = 0; d < nlocal; ++d) {
    const fa_stripe_plan* p = plans[d];
    if (!p) return set_err(FA_E_INVAL, "fa_reduce_striped: plan %d is NULL", d);
    if (root >= p->comm->nranks) return set_err(FA_E_INVAL, "fa_reduce_striped: root=%d", root);
    if (io[d].weights)
      return set_err(FA_E_INVAL, "fa_reduce_striped: the exact mode takes no weights");
    const bool result = root < 0 || root == p->comm->rank;
    if (p->n_local > 0 && !io[d].c32)
      return set_err(FA_E_INVAL, "fa_reduce_striped: fp32 buckets required (GPU %d)", d);
    if (p->n_local > 0 && p->i64.plan && !io[d].c64)
      return set_err(FA_E_INVAL, "fa_reduce_striped: int64 buckets required (GPU %d)", d);
    if (result && (!io[d].out32 || (p->i64.plan && !io[d].out64)))
      return set_err(FA_E_INVAL, "fa_reduce_striped: result buckets required on rank %d",
                     p->comm->rank);
  }
  DeviceGuard g;
  // the inputs are ready on the caller's streams
  for (int d = 0; d < nlocal; ++d) {
    fa_stripe_plan* p = plans[d];
    FA_HIP_TRY(hipSetDevice(p->comm->device));
    FA_HIP_TRY(hipEventRecord(p->ev[0], (hipStream_t)io[d].stream));
    FA_HIP_TRY(hipStreamWaitEvent(p->comm->cs, p->ev[0], 0));
  }
  // 1. every client's values for stripe r go to rank r
  NCCL_TRY(ncclGroupStart());
  for (int d = 0; d < nlocal; ++d) {
    fa_stripe_plan* p = plans[d];
    (void)hipSetDevice(p->comm->device);
    const int me = p->comm->rank;
    const int64_t Lme = p->lo[me + 1] - p->lo[me];
    for (int r = 0; r < p->comm->nranks; ++r) {
      if (r == me) continue;
      const int64_t Lr = p->lo[r + 1] - p->lo[r];
      ncclResult_t x = ncclSuccess;
      for (int j = 0; x == ncclSuccess && Lr > 0 && j < p->n_local; ++j)
        x = ncclSend(io[d].c32[j] + p->lo[r], (size_t)Lr, ncclFloat32, r, p->comm->nc,
                     p->comm->cs);
      for (int k = 0; x == ncclSuccess && Lme > 0 && k < p->counts[r]; ++k)
        x = ncclRecv(p->recv + (size_t)(p->first_slot[r] + k) * p->row, (size_t)Lme,
                     ncclFloat32, r, p->comm->nc, p->comm->cs);
      if (x != ncclSuccess) {
        ncclGroupEnd();
        return set_err(FA_E_COMM, "stripe exchange: %s", ncclGetErrorString(x));
      }
    }
  }
  NCCL_TRY(ncclGroupEnd());
  // 2. each rank reduces its stripe over all n_total clients, exact order
  for (int d = 0; d < nlocal; ++d) {
    fa_stripe_plan* p = plans[d];
    if (!p->stripe) continue;
    FA_HIP_TRY(hipSetDevice(p->comm->device));
    std::vector<const float*> src(p->ptrs);
    for (int j = 0; j < p->n_local; ++j) src[p->lo_slot + j] = io[d].c32[j];
    const int rc = fa_reduce(p->stripe, src.data(), nullptr, p->n_total, nullptr,
                             p->sbuf - p->lo[p->comm->rank], nullptr, 0, p->comm->cs);
    if (rc) return rc;
  }
  // 3. the stripes to the result ranks
  NCCL_TRY(ncclGroupStart());
  for (int d = 0; d < nlocal; ++d) {
    fa_stripe_plan* p = plans[d];
    (void)hipSetDevice(p->comm->device);
    const int me = p->comm->rank;
    const bool result = root < 0 || root == me;
    const int64_t Lme = p->lo[me + 1] - p->lo[me];
    ncclResult_t x = ncclSuccess;
    for (int r = 0; x == ncclSuccess && r < p->comm->nranks; ++r) {
      if (r == me) continue;
      const int64_t Lr = p->lo[r + 1] - p->lo[r];
      if (Lme > 0 && (root < 0 || r == root))
        x = ncclSend(p->sbuf, (size_t)Lme, ncclFloat32, r, p->comm->nc, p->comm->cs);
      if (x == ncclSuccess && Lr > 0 && result)
        x = ncclRecv(io[d].out32 + p->lo[r], (size_t)Lr, ncclFloat32, r, p->comm->nc,
                     p->comm->cs);
    }
    if (x != ncclSuccess) {
      ncclGroupEnd();
      return set_err(FA_E_COMM, "stripe gather: %s", ncclGetErrorString(x));
    }
  }
  NCCL_TRY(ncclGroupEnd());
  for (int d = 0; d < nlocal; ++d) {
    fa_stripe_plan* p = plans[d];
    const int me = p->comm->rank;
    const int64_t Lme = p->lo[me + 1] - p->lo[me];
    if (!(root < 0 || root == me) || Lme == 0) continue;
    FA_HIP_TRY(hipSetDevice(p->comm->device));
    FA_HIP_TRY(hipMemcpyAsync(io[d].out32 + p->lo[me], p->sbuf, (size_t)Lme * 4,
                              hipMemcpyDeviceToDevice, p->comm->cs));
  }
  // 4. int64 keys as in e1
  if (plans[0]->i64.plan) {
    std::vector<I64Part*> parts;
    std::vector<const fa_comm*> comms;
    for (int d = 0; d < nlocal; ++d) {
      fa_stripe_plan* p = plans[d];
      FA_HIP_TRY(hipSetDevice(p->comm->device));
      int rc = p->i64.stack_local(io[d].c64, p->n_local, p->comm->cs);
      if (rc) return rc;
      parts.push_back(&p->i64);
      comms.push_back(p->comm);
    }
    int rc = i64_exchange(parts.data(), comms.data(), nlocal);
    if (rc) return rc;
    for (int d = 0; d < nlocal; ++d) {
      fa_stripe_plan* p = plans[d];
      if (!(root < 0 || root == p->comm->rank)) continue;
      FA_HIP_TRY(hipSetDevice(p->comm->device));
      rc = fa_reduce(p->i64.plan, nullptr, p->i64.rows.data(), p->n_total, nullptr, nullptr,
                     io[d].out64, 0, p->comm->cs);
      if (rc) return rc;
    }
  }
  for (int d = 0; d < nlocal; ++d) {
    fa_stripe_plan* p = plans[d];
    FA_HIP_TRY(hipSetDevice(p->comm->device));
    FA_HIP_TRY(hipEventRecord(p->ev[2], p->comm->cs));
    FA_HIP_TRY(hipStreamWaitEvent((hipStream_t)io[d].stream, p->ev[2], 0));
  }
  return FA_OK;
}

}  // extern "C"
