// fedcomm.hip — libfedagg_comm.so: client-sharded aggregation across the GPUs
// of one node over RCCL (include/fedagg_comm.h; SURVEY.md §8 b, e1).
//
// Layering: this library uses only libfedagg.so's public ABI for the
// arithmetic (fa_plan_build_host to enumerate the layout's tiles,
// fa_plan_create_from_tiles for the per-chunk tile subsets, fa_reduce with
// FA_F_SUM_ONLY for the per-rank partial sums, fa_div_f32 for the /N finish)
// and adds the exchange: one ncclReduce / ncclAllReduce per column chunk on an
// internal communication stream, issued as soon as the kernel over that chunk
// is done, so the exchange of chunk c overlaps the reduction of chunk c+1.
// RCCL resolves to the librccl.so.1 torch has already loaded (same soname),
// so a process holds one RCCL.

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
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

struct fa_shard_plan {
  fa_comm* comm = nullptr;
  int64_t f32_numel = 0, i64_numel = 0;
  int n_local = 0, n_total = 0, nmax = 0, lo_slot = 0;
  std::vector<fa_plan*> chunk;               // tile subset per column chunk
  std::vector<std::pair<int64_t, int64_t>> range;  // [lo, hi) of each chunk
  fa_plan* plan64 = nullptr;                 // the int64 tiles
  float* partial = nullptr;                  // f32_numel (library scratch)
  int64_t* stack64 = nullptr;                // nmax rows of i64_numel
  int64_t* gather64 = nullptr;               // nranks * nmax rows
  std::vector<const int64_t*> rows64;        // n_total real rows, slot order
  std::vector<hipEvent_t> ev;                // per chunk (+ int64, + done)
};

namespace {

// Stack the rank's int64 buckets into contiguous rows for the all-gather.
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

void free_plan(fa_shard_plan* p) {
  if (!p) return;
  DeviceGuard g;
  if (p->comm) (void)hipSetDevice(p->comm->device);
  for (fa_plan* c : p->chunk) fa_plan_destroy(c);
  fa_plan_destroy(p->plan64);
  if (p->partial) (void)hipFree(p->partial);
  if (p->stack64) (void)hipFree(p->stack64);
  if (p->gather64) (void)hipFree(p->gather64);
  for (hipEvent_t e : p->ev) (void)hipEventDestroy(e);
  delete p;
}

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
  int n_total = 0, nmax = 0, lo_slot = 0;
  for (int r = 0; r < comm->nranks; ++r) {
    if (counts[r] < 0) return set_err(FA_E_INVAL, "counts[%d]=%d", r, counts[r]);
    if (r < comm->rank) lo_slot += counts[r];
    n_total += counts[r];
    nmax = std::max(nmax, counts[r]);
  }
  if (n_total < 1 || n_total > FA_MAX_CLIENTS)
    return set_err(FA_E_RANGE, "fa_shard_plan_create: %d clients in total", n_total);
  DeviceGuard g;
  FA_HIP_TRY(hipSetDevice(comm->device));
  fa_plan_info info{};
  int rc = fa_plan_build_host(seg32, nseg32, f32_numel, seg64, nseg64, i64_numel, 0, flags,
                              nullptr, 0, &info);
  if (rc) return rc;
  std::vector<fa_tile_desc> tiles(std::max(1, info.ntiles));
  rc = fa_plan_build_host(seg32, nseg32, f32_numel, seg64, nseg64, i64_numel, 0, flags,
                          tiles.data(), info.ntiles, &info);
  if (rc) return rc;
  tiles.resize(info.ntiles);
  std::vector<fa_tile_desc> t32, t64;
  for (const fa_tile_desc& t : tiles) (t.kind >= 4 ? t64 : t32).push_back(t);
  std::sort(t32.begin(), t32.end(),
            [](const fa_tile_desc& a, const fa_tile_desc& b) { return a.start < b.start; });

  fa_shard_plan* p = new fa_shard_plan();
  p->comm = comm;
  p->f32_numel = f32_numel;
  p->i64_numel = i64_numel;
  p->n_local = counts[comm->rank];
  p->n_total = n_total;
  p->nmax = nmax;
  p->lo_slot = lo_slot;
  hipError_t e = hipSuccess;
  // chunks: equal shares of the summed elements, cut only before a vector
  // tile on a 256-B boundary so every exchange starts aligned
  if (!t32.empty()) {
    int64_t total = 0;
    for (const fa_tile_desc& t : t32) total += t.count;
    std::vector<size_t> cuts{0};
    int64_t acc = 0;
    for (size_t i = 0; i < t32.size(); ++i) {
      const int c = (int)cuts.size();
      if (c < nchunks && i > 0 && acc >= total * c / nchunks && t32[i].kind == 0 &&
          t32[i].start % 64 == 0)
        cuts.push_back(i);
      acc += t32[i].count;
    }
    cuts.push_back(t32.size());
    for (size_t c = 0; c + 1 < cuts.size(); ++c) {
      const int64_t lo = c == 0 ? 0 : t32[cuts[c]].start;
      const int64_t hi = c + 2 == cuts.size() ? f32_numel : t32[cuts[c + 1]].start;
      fa_plan* sub = nullptr;
      rc = fa_plan_create_from_tiles(t32.data() + cuts[c], (int)(cuts[c + 1] - cuts[c]),
                                     f32_numel, i64_numel, 0, flags, &sub);
      if (rc) {
        free_plan(p);
        return rc;
      }
      p->chunk.push_back(sub);
      p->range.emplace_back(lo, hi);
    }
    e = hipMalloc(&p->partial, (size_t)f32_numel * 4);
    if (e == hipSuccess) e = hipMemset(p->partial, 0, (size_t)f32_numel * 4);
  }
  if (e == hipSuccess && !t64.empty()) {
    rc = fa_plan_create_from_tiles(t64.data(), (int)t64.size(), f32_numel, i64_numel, 0, flags,
                                   &p->plan64);
    if (rc) {
      free_plan(p);
      return rc;
    }
    const size_t row = (size_t)i64_numel * 8;
    e = hipMalloc(&p->stack64, std::max<size_t>(1, (size_t)nmax * row));
    if (e == hipSuccess)
      e = hipMalloc(&p->gather64, std::max<size_t>(1, (size_t)nmax * comm->nranks * row));
    if (e == hipSuccess) {
      for (int r = 0; r < comm->nranks; ++r)
        for (int j = 0; j < counts[r]; ++j)
          p->rows64.push_back(p->gather64 + ((size_t)r * nmax + j) * i64_numel);
    }
  }
  for (size_t i = 0; e == hipSuccess && i < p->chunk.size() + 2; ++i) {
    hipEvent_t ev;
    e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e == hipSuccess) p->ev.push_back(ev);
  }
  if (e != hipSuccess) {
    free_plan(p);
    return set_err(FA_E_HIP, "fa_shard_plan_create: %s", hipGetErrorString(e));
  }
  *out = p;
  return FA_OK;
}

int fa_shard_plan_destroy(fa_shard_plan* p) {
  free_plan(p);
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
    if (p->n_local > 0 && p->plan64 && !io[d].c64)
      return set_err(FA_E_INVAL, "fa_reduce_sharded: int64 buckets required (GPU %d)", d);
    if (result && ((!p->chunk.empty() && !io[d].out32) || (p->plan64 && !io[d].out64)))
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
  if (plans[0]->plan64) {
    const size_t k64 = nch;  // event slot of the int64 stack
    for (int d = 0; d < nlocal; ++d) {
      fa_shard_plan* p = plans[d];
      hipStream_t s = (hipStream_t)io[d].stream;
      FA_HIP_TRY(hipSetDevice(p->comm->device));
      for (int j0 = 0; j0 < p->n_local; j0 += kStackPtrs) {
        StackArgs a;
        memset(&a, 0, sizeof a);
        a.rows = std::min(kStackPtrs, p->n_local - j0);
        for (int j = 0; j < a.rows; ++j) a.src[j] = io[d].c64[j0 + j];
        a.dst = p->stack64 + (size_t)j0 * p->i64_numel;
        a.width = p->i64_numel;
        const int gx = (int)std::min<int64_t>(64, (p->i64_numel + 255) / 256);
        hipLaunchKernelGGL(stack_i64_kernel, dim3(gx, a.rows), dim3(256), 0, s, a);
        FA_HIP_TRY(hipGetLastError());
      }
      FA_HIP_TRY(hipEventRecord(p->ev[k64], s));
      FA_HIP_TRY(hipStreamWaitEvent(p->comm->cs, p->ev[k64], 0));
    }
    NCCL_TRY(ncclGroupStart());
    for (int d = 0; d < nlocal; ++d) {
      fa_shard_plan* p = plans[d];
      (void)hipSetDevice(p->comm->device);
      ncclResult_t r = ncclAllGather(p->stack64, p->gather64, (size_t)p->nmax * p->i64_numel,
                                     ncclInt64, p->comm->nc, p->comm->cs);
      if (r != ncclSuccess) {
        ncclGroupEnd();
        return set_err(FA_E_COMM, "int64 all-gather: %s", ncclGetErrorString(r));
      }
    }
    NCCL_TRY(ncclGroupEnd());
    for (int d = 0; d < nlocal; ++d) {
      fa_shard_plan* p = plans[d];
      if (!(root < 0 || root == p->comm->rank)) continue;
      FA_HIP_TRY(hipSetDevice(p->comm->device));
      const int rc = fa_reduce(p->plan64, nullptr, p->rows64.data(), p->n_total, nullptr,
                               nullptr, io[d].out64, 0, p->comm->cs);
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

}  // extern "C"
