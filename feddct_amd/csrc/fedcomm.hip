// fedcomm.hip — libfedagg_comm.so: aggregation across the GPUs of one node
// over RCCL (include/fedagg_comm.h; SURVEY.md §8 b, e1, e2).
//
// Layering: this library uses only libfedagg.so's public ABI for the
// arithmetic (fa_plan_build_host to enumerate the layout's tiles,
// fa_plan_create_from_tiles for tile subsets, fa_reduce / fa_reduce_chain for
// the reductions, fa_div_f32 for the /N finish) and adds the exchanges.
//
// Every round is a SCHEDULE: a host-built list of operations per rank
// (fa_xfer: sends, receives, collectives, kernels), built by pure host code
// from the layout, the shard counts and the rank — the same list
// fa_describe_round returns without a GPU, so the multi-rank schedules are
// testable on a CPU (tests/test_schedule.py replays all ranks' lists with the
// oracle as the arithmetic).  The executor walks the list: the comm ops of
// one step form one RCCL group, on the plan's communication stream; kernels
// that read exchanged data run there too, the others on the caller's stream
// (event-joined), so a rank's arithmetic overlaps its exchanges.
//   e1 sharded (fa_reduce_sharded): per column chunk, the partial sum of the
//      rank's clients, then ncclReduce / ncclAllReduce — or ncclReduceScatter
//      (in place) + ncclGather / ncclAllGather, spreading the exchange over
//      every link — and the /N; re-associates the cross-rank sum;
//   e2 striped (fa_reduce_striped): pairwise rounds of grouped sends and
//      receives move every client's values for rank r's column stripe to
//      rank r, which reduces it over all clients; the stripes then travel to
//      the result ranks.  Bit-identical to one GPU;
//   chained (fa_reduce_chained): the client shards stay put; the cascade's
//      accumulator state (fa_reduce_chain) travels rank to rank in slot order,
//      chunk by chunk, so chunk c's hop overlaps chunk c+1's reduction; the
//      scalar columns (ILP-4 tails, M==1, int64) are all-gathered raw.
//      Bit-identical to one GPU.
// RCCL resolves to the librccl.so.1 torch has already loaded (same soname),
// so a process holds one RCCL.

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <list>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../../include/fedagg_comm.h"
#include "common.h"

static_assert(sizeof(ncclUniqueId) == FA_COMM_UID_BYTES, "unique id size");
static_assert(sizeof(fa_xfer) == 56, "fa_xfer is 56 B");

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
  bool graphs = false;       // replay rounds from captured HIP graphs (fa_comm_set_graphs)
  bool profile = false;      // time every group and kernel of a round (fa_comm_set_profile)
};

namespace {

// ------------------------------------------------------------ small kernels --
// Stacks of the scalar columns: local client j's values at idx[0..width) as
// row j (fp32: times the client's weight when weighted, the product rounded
// exactly as the weighted kernel rounds it, so the root can reduce the rows
// unweighted with FA_F_SUM_ONLY and get the weighted order's bits).
constexpr int kStackPtrs = 64;
struct StackArgs {
  const void* src[kStackPtrs];
  float w[kStackPtrs];
  void* dst;
  const int64_t* idx;  // fp32 tails: bucket index of each column (NULL: 0..width)
  int64_t width;
  int64_t stride;      // row stride of dst (elements)
  int rows;
  int weighted;
};
__global__ void stack_i64_kernel(StackArgs a) {
  const int r = blockIdx.y;
  if (r >= a.rows) return;
  const int64_t* s = (const int64_t*)a.src[r];
  int64_t* d = (int64_t*)a.dst + r * a.stride;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < a.width;
       e += (int64_t)gridDim.x * blockDim.x)
    d[e] = s[e];
}
__global__ void stack_f32_kernel(StackArgs a) {
  const int r = blockIdx.y;
  if (r >= a.rows) return;
  const float* s = (const float*)a.src[r];
  float* d = (float*)a.dst + r * a.stride;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < a.width;
       e += (int64_t)gridDim.x * blockDim.x) {
    const float x = s[a.idx[e]];
    d[e] = a.weighted ? __fmul_rn(x, a.w[r]) : x;
  }
}
__global__ void scatter_f32_kernel(const float* __restrict__ src, const int64_t* __restrict__ idx,
                                   float* __restrict__ dst, int64_t width) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < width;
       e += (int64_t)gridDim.x * blockDim.x)
    dst[idx[e]] = src[e];
}

// Weighted striped rounds (r06): local client j's columns [off, off + count)
// times its weight, the product rounded as the weighted reduce rounds it
// (__fmul_rn, no contraction), into staging row j.  The receivers reduce
// these rows with weight 1 (x * 1 == x exactly), their own clients with
// their weights: the one-GPU weighted order's bits.
struct ScaleArgs {
  const float* src[kStackPtrs];
  float w[kStackPtrs];
  float* dst;
  int64_t plane;  // staging row stride (floats)
  int64_t off, count;
  int rows;
  int vec;        // every row's src + off and dst + off 16-B aligned
};
__global__ void scale_rows_kernel(ScaleArgs a) {
  const int r = blockIdx.y;
  if (r >= a.rows) return;
  const float* s = a.src[r] + a.off;
  float* d = a.dst + r * a.plane + a.off;
  const float w = a.w[r];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t e0 = 0;
  if (a.vec) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const int64_t nv = a.count / 4;
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < nv; v += stride) {
      f4v x = ((const f4v*)s)[v];
      x.x = __fmul_rn(x.x, w);
      x.y = __fmul_rn(x.y, w);
      x.z = __fmul_rn(x.z, w);
      x.w = __fmul_rn(x.w, w);
      ((f4v*)d)[v] = x;
    }
    e0 = 4 * nv;
  }
  for (int64_t e = e0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < a.count; e += stride)
    d[e] = __fmul_rn(s[e], w);
}

// Blocked mode: an owner's fold of the block sums of its column stripe, in
// block order, with the cascade's promotions after every 2^lp-th block
// (levels 1-3 of fa_reduce's accumulators: the block after row i = (k+1)<<lp
// promotes exactly as reduce_kernel's `promote` does at row i), then the
// finish ((rem + l1) + l2) + l3 and the division.  blk: nblk + has_rem rows
// of `row` floats (the remainder block's partial last).
// Up to kFoldPtrs pieces each piece's stripe is read where it lies (r03):
// src[k] is the stripe's first element — the owner's receive row for a
// remote piece, or this rank's own block-sum / continuation plane, which the
// schedule's K_COPY into the receive row would have duplicated (the executor
// binds the row to the copy's source instead, FA_X_K_COPY below).  More
// pieces: rows of blk, copies made.
constexpr int kFoldPtrs = 256;
struct FoldArgs {
  const float* blk;
  int64_t row;
  int64_t count;
  float* out;
  int nblk;
  int has_rem;
  int lp;
  int n_total;
  int divide;
  int bound;  // src[] holds every piece's stripe
  const float* src[kFoldPtrs];
};
__device__ __forceinline__ float fold_at(const FoldArgs& a, int k, int64_t e) {
  return a.bound ? a.src[k][e] : a.blk[(size_t)k * a.row + e];
}
__global__ void fold_kernel(FoldArgs a) {
  const int mask = (1 << a.lp) - 1;
  const float fn = (float)a.n_total;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < a.count;
       e += (int64_t)gridDim.x * blockDim.x) {
    float l1 = 0.f, l2 = 0.f, l3 = 0.f;
    for (int k = 0; k < a.nblk; ++k) {
      l1 = __fadd_rn(l1, fold_at(a, k, e));
      const int i = (k + 1) << a.lp;
      if ((i & (mask << a.lp)) != 0) continue;
      l2 = __fadd_rn(l2, l1);
      l1 = 0.f;
      if ((i & (mask << (2 * a.lp))) != 0) continue;
      l3 = __fadd_rn(l3, l2);
      l2 = 0.f;
    }
    const float l0 = a.has_rem ? fold_at(a, a.nblk, e) : 0.f;
    const float s = __fadd_rn(__fadd_rn(__fadd_rn(l0, l1), l2), l3);
    a.out[e] = a.divide ? __fdiv_rn(s, fn) : s;
  }
}

int launch_stack(bool f32, const void* const* src, const float* w, int n_local, void* dst,
                 const int64_t* idx, int64_t width, int64_t stride, hipStream_t s) {
  for (int j0 = 0; j0 < n_local; j0 += kStackPtrs) {
    StackArgs a;
    memset(&a, 0, sizeof a);
    a.rows = std::min(kStackPtrs, n_local - j0);
    for (int j = 0; j < a.rows; ++j) {
      a.src[j] = src[j0 + j];
      a.w[j] = w ? w[j0 + j] : 1.f;
    }
    a.weighted = w != nullptr;
    a.dst = (char*)dst + (size_t)j0 * stride * (f32 ? 4 : 8);
    a.idx = idx;
    a.width = width;
    a.stride = stride;
    const int gx = (int)std::min<int64_t>(64, (width + 255) / 256);
    if (f32) hipLaunchKernelGGL(stack_f32_kernel, dim3(gx, a.rows), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(stack_i64_kernel, dim3(gx, a.rows), dim3(256), 0, s, a);
    FA_HIP_TRY(hipGetLastError());
  }
  return FA_OK;
}

// ------------------------------------------------------------- geometry ----
// Everything a schedule depends on, host-only (no device, no communicator).
struct Geo {
  int nranks = 1, rank = 0;
  std::vector<int> counts, first;  // per rank: slots held, first slot
  int n_total = 0, n_local = 0, lo_slot = 0, nmax = 0;
  int64_t f32_numel = 0, i64_numel = 0;
  unsigned flags = 0;
  std::vector<fa_tile_desc> t32, t64;  // fp32 tiles sorted by start; int64 tiles
};

int make_geo(int nranks, int rank, const int* counts, const fa_seg* seg32, int nseg32,
             int64_t f32_numel, const fa_seg* seg64, int nseg64, int64_t i64_numel,
             unsigned flags, const char* who, Geo* g) {
  if (!counts) return set_err(FA_E_INVAL, "%s: counts is NULL", who);
  if (nranks < 1 || rank < 0 || rank >= nranks)
    return set_err(FA_E_INVAL, "%s: rank %d of %d", who, rank, nranks);
  if (!(flags & FA_PLAN_GAPS_ARE_PADDING))
    return set_err(FA_E_INVAL,
                   "%s: the layout must allow writes to its padding "
                   "(FA_PLAN_GAPS_ARE_PADDING): exchanges span it",
                   who);
  g->nranks = nranks;
  g->rank = rank;
  g->counts.assign(counts, counts + nranks);
  g->first.clear();
  g->n_total = 0;
  g->nmax = 0;
  for (int r = 0; r < nranks; ++r) {
    if (counts[r] < 0) return set_err(FA_E_INVAL, "%s: counts[%d]=%d", who, r, counts[r]);
    g->first.push_back(g->n_total);
    g->n_total += counts[r];
    g->nmax = std::max(g->nmax, counts[r]);
  }
  if (g->n_total < 1 || g->n_total > FA_MAX_CLIENTS)
    return set_err(FA_E_RANGE, "%s: %d clients in total", who, g->n_total);
  g->n_local = counts[rank];
  g->lo_slot = g->first[rank];
  g->f32_numel = f32_numel;
  g->i64_numel = i64_numel;
  g->flags = flags;
  fa_plan_info info{};
  int rc = fa_plan_build_host(seg32, nseg32, f32_numel, seg64, nseg64, i64_numel, 0, flags,
                              nullptr, 0, &info);
  if (rc) return rc;
  std::vector<fa_tile_desc> tiles(std::max(1, info.ntiles));
  rc = fa_plan_build_host(seg32, nseg32, f32_numel, seg64, nseg64, i64_numel, 0, flags,
                          tiles.data(), info.ntiles, &info);
  if (rc) return rc;
  tiles.resize(info.ntiles);
  g->t32.clear();
  g->t64.clear();
  for (const fa_tile_desc& t : tiles) (t.kind >= 4 ? g->t64 : g->t32).push_back(t);
  std::sort(g->t32.begin(), g->t32.end(),
            [](const fa_tile_desc& a, const fa_tile_desc& b) { return a.start < b.start; });
  return FA_OK;
}

// k contiguous groups of sorted tiles with equal shares of the elements, cut
// only before a vector tile on a 256-B boundary; exactly k groups, trailing
// ones may be empty.  Group g = tiles [cut[g], cut[g+1]).
void cut_tiles(const std::vector<fa_tile_desc>& t, int k, std::vector<size_t>* cut) {
  int64_t total = 0;
  for (const fa_tile_desc& x : t) total += x.count;
  cut->assign(1, 0);
  int64_t acc = 0;
  for (size_t i = 0; i < t.size(); ++i) {
    const int c = (int)cut->size();
    if (c < k && i > 0 && acc >= total * c / k && t[i].kind == 0 && t[i].start % 64 == 0)
      cut->push_back(i);
    acc += t[i].count;
  }
  while ((int)cut->size() < k + 1) cut->push_back(t.size());
}

// Group g's bucket range: [lo[g], lo[g+1]) with lo[0] = 0 and lo[k] =
// f32_numel — the groups tile the whole bucket (padding included).
std::vector<int64_t> cut_bounds(const std::vector<fa_tile_desc>& t,
                                const std::vector<size_t>& cut, int64_t f32_numel) {
  const int k = (int)cut.size() - 1;
  std::vector<int64_t> lo(k + 1, f32_numel);
  lo[0] = 0;
  for (int g = 1; g < k; ++g) lo[g] = cut[g] < t.size() ? t[cut[g]].start : f32_numel;
  return lo;
}

// ------------------------------------------------------------- schedules ---
inline bool is_comm(int op) { return op >= FA_X_SEND && op <= FA_X_BCAST; }

struct Sched {
  std::vector<fa_xfer> ops;
  int step = 0;
  void add(int op, int peer, int src, int si, int dst, int di, int64_t off, int64_t cnt,
           int chunk = -1, int row0 = 0, int nrows = 0) {
    fa_xfer x;
    memset(&x, 0, sizeof x);
    x.step = step;
    x.op = op;
    x.peer = peer;
    x.chunk = chunk;
    x.src = src;
    x.src_index = si;
    x.dst = dst;
    x.dst_index = di;
    x.offset = off;
    x.count = cnt;
    x.row0 = row0;
    x.nrows = nrows;
    ops.push_back(x);
  }
  void next() { ++step; }
};

// The striped round's default column chunks per stripe (fa_stripe_plan_create,
// nchunks 0): the chunk c + 1 exchange overlaps chunk c's stripe reduce and
// the chunk c - 1 results; fa_multi_select_layout picks the count by the model.
constexpr int kStripeChunks = 4;

// The int64 keys (num_batches_tracked) of every client, gathered raw and
// reduced exactly by the result ranks; with `tails`, the fp32 scalar columns
// (ILP-4 tails, M==1) too.  stack -> all-gather -> (result ranks) reduce.
void sched_raw_gather(Sched* S, const Geo& g, int64_t t32_width, bool tails, bool result) {
  const bool i64 = !g.t64.empty();
  if (!i64 && !(tails && t32_width)) return;
  if (g.n_local > 0) S->add(FA_X_K_STACK, -1, FA_B_CLIENT, -1, FA_B_STACK, -1, 0, 0, -1,
                            g.lo_slot, g.n_local);
  S->next();
  if (tails && t32_width)
    S->add(FA_X_ALLGATHER, -1, FA_B_STACK, 0, FA_B_GATHER, 0, 0, (int64_t)g.nmax * t32_width);
  if (i64)
    S->add(FA_X_ALLGATHER, -1, FA_B_STACK, 1, FA_B_GATHER, 1, 0,
           (int64_t)g.nmax * g.i64_numel);
  S->next();
  if (result) S->add(FA_X_K_TAILS, -1, FA_B_GATHER, -1, FA_B_OUT, -1, 0, 0, -1, 0, g.n_total);
  S->next();
}

// e1: chunked partial sums + RCCL reduce (or reduce-scatter + gather).
void sched_sharded(const Geo& g, const std::vector<std::pair<int64_t, int64_t>>& range, int xchg,
                   int root, bool weighted, Sched* S) {
  const int me = g.rank, W = g.nranks;
  const bool result = root < 0 || root == me;
  for (size_t c = 0; c < range.size(); ++c) {
    const int64_t lo = range[c].first, L = range[c].second - lo;
    if (g.n_local > 0)
      S->add(FA_X_K_SUM, -1, FA_B_CLIENT, -1, FA_B_PARTIAL, -1, lo, L, (int)c, g.lo_slot,
             g.n_local);
    else
      S->add(FA_X_K_ZERO, -1, FA_B_NONE, -1, FA_B_PARTIAL, -1, lo, L, (int)c);
    S->next();
    const int64_t q = xchg == FA_XCHG_RS_GATHER ? L / W : 0;
    if (q > 0) {
      // in place: rank r's share of the sum lands at partial[lo + r*q, +q)
      S->add(FA_X_REDUCE_SCATTER, -1, FA_B_PARTIAL, -1, FA_B_PARTIAL, -1, lo, q * W);
      S->next();
      if (root < 0)
        S->add(FA_X_ALLGATHER, -1, FA_B_PARTIAL, -1, FA_B_OUT, -1, lo, q * W);
      else
        S->add(FA_X_GATHER, root, FA_B_PARTIAL, -1, result ? FA_B_OUT : FA_B_NONE, -1, lo,
               q * W);
    }
    const int64_t rlo = lo + q * W, rl = L - q * W;  // (all of it for a plain reduce)
    if (rl > 0) {
      if (root < 0)
        S->add(FA_X_ALLREDUCE, -1, FA_B_PARTIAL, -1, FA_B_OUT, -1, rlo, rl);
      else
        S->add(FA_X_REDUCE, root, FA_B_PARTIAL, -1, result ? FA_B_OUT : FA_B_PARTIAL, -1, rlo,
               rl);
    }
    S->next();
    if (result && !weighted) S->add(FA_X_K_DIV, -1, FA_B_OUT, -1, FA_B_OUT, -1, lo, L, (int)c);
    S->next();
  }
  sched_raw_gather(S, g, 0, false, result);
}

// e2: column stripes, cut into column chunks; every peer in one group per
// chunk (r06, VERDICT r05 next 1: r02-r05 ran one RCCL group per partner, so
// a rank used one of its xGMI links at a time).  clo[r][c .. c+1]: chunk c of
// rank r's stripe.  Step 2 + j carries, in ONE group, chunk j's client
// exchange with every peer and the finished chunk j - 2 to the result ranks,
// and — on the caller's stream, concurrent with that group — the stripe
// reduce of chunk j - 1, whose rows arrived in the previous step's group
// (the executor starts a compute-stream kernel that reads exchanged data
// after the exchanges of the steps BEFORE its own: reads_exchanged below).
// Per pair, the sender posts its client rows then its result chunk and the
// receiver its receives in the same order (RCCL matches a pair's sends and
// receives in posting order).  Weighted: the rows sent are the local
// clients' pre-multiplied values (FA_X_K_SCALE into WSTAGE, step 0).
void sched_striped(const Geo& g, const std::vector<std::vector<int64_t>>& clo, int root,
                   bool weighted, Sched* S) {
  const int me = g.rank, W = g.nranks;
  const int C = (int)clo[0].size() - 1;
  const bool result = root < 0 || root == me;
  const bool i64 = !g.t64.empty();
  auto len = [&](int r, int c) { return clo[r][c + 1] - clo[r][c]; };
  // step 0: the int64 keys stacked; weighted: the local clients' values
  // outside this rank's stripe (what the peers receive) pre-multiplied
  if (i64 && g.n_local > 0)
    S->add(FA_X_K_STACK, -1, FA_B_CLIENT, -1, FA_B_STACK, -1, 0, 0, -1, g.lo_slot, g.n_local);
  const int64_t mlo = clo[me][0], mhi = clo[me][C];
  if (weighted && g.n_local > 0) {
    if (mlo > 0)
      S->add(FA_X_K_SCALE, -1, FA_B_CLIENT, -1, FA_B_WSTAGE, -1, 0, mlo, -1, 0, g.n_local);
    if (mhi < g.f32_numel)
      S->add(FA_X_K_SCALE, -1, FA_B_CLIENT, -1, FA_B_WSTAGE, -1, mhi, g.f32_numel - mhi, -1, 0,
             g.n_local);
  }
  S->next();
  // step 1: the int64 keys of every rank (a few bytes)
  if (i64)
    S->add(FA_X_ALLGATHER, -1, FA_B_STACK, 1, FA_B_GATHER, 1, 0, (int64_t)g.nmax * g.i64_numel);
  S->next();
  const int src = weighted ? FA_B_WSTAGE : FA_B_CLIENT;
  for (int j = 0; j <= C + 1; ++j) {
    for (int q = 1; q < W; ++q) {  // peers in a rotated order: rank me + q first
      const int r = (me + q) % W;
      if (j < C) {
        if (len(r, j) > 0)
          for (int k = 0; k < g.n_local; ++k)
            S->add(FA_X_SEND, r, src, k, FA_B_NONE, -1, clo[r][j], len(r, j), j);
        if (len(me, j) > 0)
          for (int k = 0; k < g.counts[r]; ++k)
            S->add(FA_X_RECV, r, FA_B_NONE, -1, FA_B_RECV, g.first[r] + k, clo[me][j],
                   len(me, j), j);
      }
      const int c = j - 2;
      if (c >= 0 && c < C) {
        if (len(me, c) > 0 && (root < 0 || root == r))
          S->add(FA_X_SEND, r, result ? FA_B_OUT : FA_B_STRIPE, -1, FA_B_NONE, -1, clo[me][c],
                 len(me, c), c);
        if (len(r, c) > 0 && result)
          S->add(FA_X_RECV, r, FA_B_NONE, -1, FA_B_OUT, -1, clo[r][c], len(r, c), c);
      }
    }
    const int k = j - 1;
    if (k >= 0 && k < C && len(me, k) > 0)
      S->add(FA_X_K_STRIPE, -1, FA_B_RECV, -1, result ? FA_B_OUT : FA_B_STRIPE, -1, clo[me][k],
             len(me, k), k, 0, g.n_total);
    S->next();
  }
  if (i64 && result)
    S->add(FA_X_K_TAILS, -1, FA_B_GATHER, -1, FA_B_OUT, -1, 0, 0, -1, 0, g.n_total);
  S->next();
}

// Chained: state hops rank to rank, chunk by chunk.
struct ChainGeo {
  std::vector<std::pair<int64_t, int64_t>> range;  // vector-tile chunks [lo, hi)
  int finisher = 0;                                // last rank holding clients
  unsigned lev_in = 0, lev_out = 0;
  int64_t t32_width = 0;                           // scalar fp32 columns
  int64_t t32_row = 0;                             // their stack row stride (64-aligned)
};

// Blocked mode geometry (host-only, the same on every rank).  Pieces are the
// cascade's blocks of 2^lp slots (0..K-1) and the remainder block (K, when
// n_total % 2^lp); a piece's slots lie on its starter and holder ranks.
struct BlockGeo {
  int lp = 4;
  int K = 0, P = 0;                       // complete blocks, pieces (K + remainder)
  std::vector<int> s0, s1;                // piece rows [s0, s1)
  std::vector<int> starter, holder;       // first / last row's rank
  std::vector<int> bsum_slot;             // local pieces: BSUM index on the holder (-1: spans)
  std::vector<int> plane;                 // spanning complete blocks: CONT plane of the sum
  int tail_piece = -1, head_piece = -1;   // this rank's spanning piece it starts / ends
  int nbsum = 0;                          // local pieces of this rank
  std::vector<int64_t> slo, shi;          // owner column stripes (vector tiles)
  int64_t row = 0;                        // stripe row stride (floats, 64-aligned)
};

void sched_chained(const Geo& g, const ChainGeo& cg, int root, Sched* S) {
  const int me = g.rank, F = cg.finisher;
  const bool result = root < 0 || root == me;
  // the raw scalar columns first: their gather overlaps the chain
  const int64_t C = (int64_t)cg.range.size();
  const bool i64 = !g.t64.empty();
  if (i64 || cg.t32_width) {
    if (g.n_local > 0)
      S->add(FA_X_K_STACK, -1, FA_B_CLIENT, -1, FA_B_STACK, -1, 0, 0, -1, g.lo_slot, g.n_local);
    S->next();
    if (cg.t32_width)
      S->add(FA_X_ALLGATHER, -1, FA_B_STACK, 0, FA_B_GATHER, 0, 0, (int64_t)g.nmax * cg.t32_row);
    if (i64)
      S->add(FA_X_ALLGATHER, -1, FA_B_STACK, 1, FA_B_GATHER, 1, 0,
             (int64_t)g.nmax * g.i64_numel);
    S->next();
  }
  if (me <= F) {
    const bool pred = me > 0 && cg.lev_in, succ = me < F && cg.lev_out;
    auto planes = [&](int op, int peer, unsigned lev, int64_t c) {
      for (int l = 0; l < 4; ++l)
        if (lev & (1u << l)) {
          const int64_t lo = cg.range[c].first, L = cg.range[c].second - lo;
          if (op == FA_X_SEND) S->add(op, peer, FA_B_STATE, l, FA_B_NONE, -1, lo, L, (int)c);
          else S->add(op, peer, FA_B_NONE, -1, FA_B_STATE, l, lo, L, (int)c);
        }
    };
    const int fin = me < F ? FA_B_STATE : (result ? FA_B_OUT : FA_B_FIN);
    for (int64_t c = 0; c <= C; ++c) {
      if (succ && c > 0) planes(FA_X_SEND, me + 1, cg.lev_out, c - 1);
      if (pred && c < C) planes(FA_X_RECV, me - 1, cg.lev_in, c);
      S->next();
      if (c < C && g.n_local > 0) {
        const int64_t lo = cg.range[c].first, L = cg.range[c].second - lo;
        S->add(FA_X_K_CHAIN, -1, pred ? FA_B_STATE : FA_B_NONE, -1, fin, -1, lo, L, (int)c,
               g.lo_slot, g.n_local);
      }
      S->next();
    }
  } else {
    S->step += 2 * (int)(C + 1);
  }
  // the finished vector columns to the result ranks
  if (C > 0) {
    const int64_t lo = cg.range[0].first, L = cg.range[C - 1].second - lo;
    if (root < 0) {
      S->add(FA_X_BCAST, F, me == F ? FA_B_OUT : FA_B_NONE, -1, FA_B_OUT, -1, lo, L);
    } else if (root != F) {
      if (me == F) S->add(FA_X_SEND, root, FA_B_FIN, -1, FA_B_NONE, -1, lo, L);
      if (me == root) S->add(FA_X_RECV, F, FA_B_NONE, -1, FA_B_OUT, -1, lo, L);
    }
  }
  S->next();
  if (result && (i64 || cg.t32_width))
    S->add(FA_X_K_TAILS, -1, FA_B_GATHER, -1, FA_B_OUT, -1, 0, 0, -1, 0, g.n_total);
  S->next();
}

// Blocked: block sums where they lie, spanning blocks' partials relayed
// through the stripe owners, block sums to the owners, fold, results out.
void sched_blocked(const Geo& g, const ChainGeo& cg, const BlockGeo& bg, int root, Sched* S) {
  const int me = g.rank, W = g.nranks;
  const bool result = root < 0 || root == me;
  const bool i64 = !g.t64.empty();
  auto w_of = [&](int s) { return bg.shi[s] - bg.slo[s]; };
  const bool vec = !cg.range.empty();  // a layout of scalar columns only has no blocks
  // step 0: the partial a neighbour waits for, alone
  if ((i64 || cg.t32_width) && g.n_local > 0)
    S->add(FA_X_K_STACK, -1, FA_B_CLIENT, -1, FA_B_STACK, -1, 0, 0, -1, g.lo_slot, g.n_local);
  if (vec && bg.tail_piece >= 0) {
    const int i = bg.tail_piece;
    S->add(FA_X_K_PART, -1, FA_B_PIN, -1, FA_B_TAILP, 0, 0, 0, -1, bg.s0[i],
           g.lo_slot + g.n_local - bg.s0[i]);
  }
  S->next();
  // step 1: raw columns gathered; each spanning partial split into stripes,
  // to its holder directly (the starter's and the holder's own stripes) or
  // to the stripe's owner
  if (cg.t32_width)
    S->add(FA_X_ALLGATHER, -1, FA_B_STACK, 0, FA_B_GATHER, 0, 0, (int64_t)g.nmax * cg.t32_row);
  if (i64)
    S->add(FA_X_ALLGATHER, -1, FA_B_STACK, 1, FA_B_GATHER, 1, 0, (int64_t)g.nmax * g.i64_numel);
  for (int i = 0; i < bg.P; ++i) {
    const int r1 = bg.starter[i], r2 = bg.holder[i];
    if (r1 == r2) continue;
    for (int s = 0; s < W; ++s) {
      const int64_t w = w_of(s);
      if (w == 0) continue;
      const int64_t off = bg.slo[s];
      const bool direct = s == r1 || s == r2;
      if (me == r1) S->add(FA_X_SEND, direct ? r2 : s, FA_B_TAILP, 0, FA_B_NONE, -1, off, w);
      if (direct && me == r2) S->add(FA_X_RECV, r1, FA_B_NONE, -1, FA_B_PIN, 0, off, w);
      if (!direct && me == s) S->add(FA_X_RECV, r1, FA_B_NONE, -1, FA_B_RELAY, r1, off, w);
    }
  }
  // the local block sums on the compute stream, behind the partial's
  // scatter and overlapping it and the forwarding step (which reads only
  // relayed data)
  for (int i = 0; i < bg.P && vec; ++i)
    if (bg.bsum_slot[i] >= 0)
      S->add(FA_X_K_BLOCK, -1, FA_B_CLIENT, -1, FA_B_BSUM, bg.bsum_slot[i], 0, 0, i, bg.s0[i],
             bg.s1[i] - bg.s0[i]);
  S->next();
  // step 2: the owners forward their stripes of the partials
  for (int i = 0; i < bg.P; ++i) {
    const int r1 = bg.starter[i], r2 = bg.holder[i];
    if (r1 == r2) continue;
    for (int s = 0; s < W; ++s) {
      const int64_t w = w_of(s);
      if (w == 0 || s == r1 || s == r2) continue;
      if (me == s) S->add(FA_X_SEND, r2, FA_B_RELAY, r1, FA_B_NONE, -1, bg.slo[s], w);
      if (me == r2) S->add(FA_X_RECV, s, FA_B_NONE, -1, FA_B_PIN, 0, bg.slo[s], w);
    }
  }
  S->next();
  // step 3: the holder finishes the spanning block (or the remainder)
  if (vec && bg.head_piece >= 0) {
    const int i = bg.head_piece;
    S->add(FA_X_K_CONT, -1, FA_B_PIN, -1, FA_B_CONT, bg.plane[i], 0, 0, i, g.lo_slot,
           bg.s1[i] - g.lo_slot);
  }
  S->next();
  // step 4: every piece's stripes to their owners, in piece order
  for (int i = 0; i < bg.P; ++i) {
    const int h = bg.holder[i];
    const bool local = bg.starter[i] == h;
    for (int s = 0; s < W; ++s) {
      const int64_t w = w_of(s);
      if (w == 0 || s == h) continue;
      if (me == h) {
        if (local) S->add(FA_X_SEND, s, FA_B_BSUM, bg.bsum_slot[i], FA_B_NONE, -1, bg.slo[s], w);
        else S->add(FA_X_SEND, s, FA_B_CONT, bg.plane[i], FA_B_NONE, -1, bg.slo[s], w);
      }
      if (me == s) S->add(FA_X_RECV, h, FA_B_NONE, -1, FA_B_BLK, i, bg.slo[s], w);
    }
  }
  S->next();
  // step 5: own pieces into the stripe, then the fold
  const int64_t wme = w_of(me);
  if (vec && wme > 0) {
    for (int i = 0; i < bg.P; ++i) {
      if (bg.holder[i] != me) continue;
      if (bg.bsum_slot[i] >= 0)
        S->add(FA_X_K_COPY, -1, FA_B_BSUM, bg.bsum_slot[i], FA_B_BLK, i, bg.slo[me], wme);
      else
        S->add(FA_X_K_COPY, -1, FA_B_CONT, bg.plane[i], FA_B_BLK, i, bg.slo[me], wme);
    }
    S->add(FA_X_K_FOLD, -1, FA_B_BLK, -1, result ? FA_B_OUT : FA_B_FIN, -1, bg.slo[me], wme, me,
           0, bg.P);
  }
  S->next();
  // step 6: the folded stripes to the result ranks
  for (int s = 0; s < W; ++s) {
    const int64_t w = w_of(s);
    if (w == 0) continue;
    for (int r = 0; r < W; ++r) {
      if (r == s || !(root < 0 || root == r)) continue;
      const bool s_result = root < 0 || root == s;
      if (me == s)
        S->add(FA_X_SEND, r, s_result ? FA_B_OUT : FA_B_FIN, -1, FA_B_NONE, -1, bg.slo[s], w);
      if (me == r) S->add(FA_X_RECV, s, FA_B_NONE, -1, FA_B_OUT, -1, bg.slo[s], w);
    }
  }
  S->next();
  if (result && (i64 || cg.t32_width))
    S->add(FA_X_K_TAILS, -1, FA_B_GATHER, -1, FA_B_OUT, -1, 0, 0, -1, 0, g.n_total);
  S->next();
}

// The chained mode's cut of the layout: vector tiles chunked, scalar fp32
// columns compacted (their bucket index per compact column).
void chain_geo(const Geo& g, int nchunks, ChainGeo* cg, std::vector<fa_tile_desc>* vec,
               std::vector<size_t>* cut, std::vector<fa_tile_desc>* tails,
               std::vector<int64_t>* tidx) {
  vec->clear();
  tails->clear();
  tidx->clear();
  for (const fa_tile_desc& t : g.t32) {
    if (t.kind == 0) {
      vec->push_back(t);
    } else {
      fa_tile_desc c = t;
      c.start = (int64_t)tidx->size();  // compact coordinates
      tails->push_back(c);
      for (int32_t e = 0; e < t.count; ++e) tidx->push_back(t.start + e);
    }
  }
  cg->t32_width = (int64_t)tidx->size();
  cg->t32_row = (cg->t32_width + 63) / 64 * 64;
  cg->range.clear();
  cut_tiles(*vec, nchunks, cut);
  std::vector<size_t> keep(1, 0);
  for (int c = 0; c < nchunks; ++c) {
    if ((*cut)[c] == (*cut)[c + 1]) continue;
    const fa_tile_desc& a = (*vec)[(*cut)[c]];
    const fa_tile_desc& b = (*vec)[(*cut)[c + 1] - 1];
    cg->range.emplace_back(a.start, b.start + b.count);
    keep.push_back((*cut)[c + 1]);
  }
  *cut = keep;
  cg->finisher = 0;
  for (int r = 0; r < g.nranks; ++r)
    if (g.counts[r] > 0) cg->finisher = r;
  cg->lev_in = fa_chain_levels(g.lo_slot, g.n_total);
  cg->lev_out = fa_chain_levels(g.lo_slot + g.n_local, g.n_total);
}

int rank_of_row(const Geo& g, int i) {
  for (int r = 0; r < g.nranks; ++r)
    if (i >= g.first[r] && i < g.first[r] + g.counts[r]) return r;
  return -1;
}

// The cascade's level step for n rows (fa_reduce's lp: 16 below 2^16 rows).
int cascade_lp(int n) {
  int c = 0;
  while ((1ll << c) < n) ++c;
  return std::max(4, c / 4);
}

// The blocked round's condition from the counts alone: the first cascade
// block (slots [*a, *b)) whose slots lie on more than two of the ranks that
// hold slots (ranks without slots in between do not count), or -1 when every
// block fits.  block_geo and fa_multi_select share it.
int first_wide_block(int nranks, const int* counts, int* a_out, int* b_out) {
  int n = 0;
  std::vector<int> first(nranks);
  for (int r = 0; r < nranks; ++r) {
    first[r] = n;
    n += std::max(0, counts[r]);
  }
  const int Q = 1 << cascade_lp(n);
  for (int i = 0, a = 0; a < n; ++i, a += Q) {
    const int b = std::min(n, a + Q);
    int on = 0;
    for (int r = 0; r < nranks; ++r)
      if (counts[r] > 0 && first[r] < b && first[r] + counts[r] > a) ++on;
    if (on > 2) {
      if (a_out) *a_out = a;
      if (b_out) *b_out = b;
      return i;
    }
  }
  return -1;
}

int block_geo(const Geo& g, const std::vector<fa_tile_desc>& vec, BlockGeo* bg) {
  const int n = g.n_total;
  const int lp = cascade_lp(n);
  {
    int a = 0, b = 0;
    if (first_wide_block(g.nranks, g.counts.data(), &a, &b) >= 0)
      return set_err(FA_E_RANGE,
                     "blocked round: slots %d..%d (one cascade block) lie on more than two "
                     "ranks; use the chained round",
                     a, b - 1);
  }
  bg->lp = lp;
  const int Q = 1 << lp, mask = Q - 1;
  bg->K = n / Q;
  bg->P = bg->K + (n % Q ? 1 : 0);
  bg->s0.clear(); bg->s1.clear(); bg->starter.clear(); bg->holder.clear();
  bg->bsum_slot.clear(); bg->plane.clear();
  bg->tail_piece = bg->head_piece = -1;
  bg->nbsum = 0;
  for (int i = 0; i < bg->P; ++i) {
    const int a = i * Q, b = std::min(n, a + Q);
    // (first_wide_block above: the holder is the next rank holding slots
    // after the starter)
    const int r0 = rank_of_row(g, a), r1 = rank_of_row(g, b - 1);
    bg->s0.push_back(a);
    bg->s1.push_back(b);
    bg->starter.push_back(r0);
    bg->holder.push_back(r1);
    int j = 0;
    if (r0 != r1 && i < bg->K && b < n) {
      j = 1;
      if ((b & (mask << lp)) == 0) j = (b & (mask << (2 * lp))) == 0 ? 3 : 2;
    }
    bg->plane.push_back(j);  // 0: a finishing continuation writes CONT plane 0
    if (r0 == r1) {
      bg->bsum_slot.push_back(r1 == g.rank ? bg->nbsum++ : -1);
    } else {
      bg->bsum_slot.push_back(-1);
      if (r0 == g.rank) bg->tail_piece = i;
      if (r1 == g.rank) bg->head_piece = i;
    }
  }
  // owner stripes over the vector tiles
  std::vector<size_t> cut;
  cut_tiles(vec, g.nranks, &cut);
  bg->slo.assign(g.nranks, 0);
  bg->shi.assign(g.nranks, 0);
  int64_t w = 0;
  for (int s = 0; s < g.nranks; ++s) {
    if (cut[s] == cut[s + 1]) continue;
    bg->slo[s] = vec[cut[s]].start;
    const fa_tile_desc& t = vec[cut[s + 1] - 1];
    bg->shi[s] = t.start + t.count;
    w = std::max(w, bg->shi[s] - bg->slo[s]);
  }
  bg->row = (w + 63) / 64 * 64;
  return FA_OK;
}

// e1 chunk ranges over the whole bucket.
void shard_ranges(const Geo& g, int nchunks, std::vector<size_t>* cut_out,
                  std::vector<std::pair<int64_t, int64_t>>* range) {
  std::vector<size_t> cut;
  cut_tiles(g.t32, nchunks, &cut);
  const std::vector<int64_t> lo = cut_bounds(g.t32, cut, g.f32_numel);
  range->clear();
  cut_out->assign(1, 0);
  for (int c = 0; c < nchunks; ++c) {
    if (cut[c] == cut[c + 1]) continue;
    range->emplace_back(lo[c], lo[c + 1]);
    cut_out->push_back(cut[c + 1]);
  }
  if (!range->empty()) range->back().second = g.f32_numel;
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

}  // namespace

// =========================================================== round plans ==
// One plan type for the three modes: the schedule geometry plus the device
// resources its ops address.
struct fa_round_plan {
  int mode = 0;  // FA_MODE_*
  int xchg = 0;
  int req_chunks = 0;       // the column chunk count the plan was built for
  fa_comm* comm = nullptr;  // (may be destroyed before the plan: never read in free_round)
  int device = -1;          // the comm's device, for free_round
  Geo g;
  // e1: chunk plans + their ranges; chained: vector-tile chunk plans + ranges
  std::vector<fa_plan*> chunk;
  std::vector<std::pair<int64_t, int64_t>> range;
  float* partial = nullptr;  // e1 partial sums (f32_numel)
  // e2 (r06: every stripe cut into nchunks column chunks; `chunk` holds this
  // rank's chunk plans, NULL for an empty chunk)
  std::vector<int64_t> lo;   // nranks + 1 stripe bounds
  std::vector<std::vector<int64_t>> clo;  // per rank: nchunks + 1 chunk bounds
  int nchunks = 0;
  int64_t row = 0;           // receive row stride (floats)
  float* recv = nullptr;     // n_total rows
  float* sbuf = nullptr;     // the reduced stripe (a rank that is not a result rank)
  float* wstage = nullptr;   // weighted rounds: n_local pre-multiplied buckets
  std::vector<float> wfull;  // weighted rounds: the stripe kernel's n_total weights
  // chained
  ChainGeo cg;
  float* state = nullptr;    // nplanes * plane floats
  int64_t plane = 0;
  float* fin = nullptr;      // the finisher's result when it is not a result rank
  // blocked
  BlockGeo bg;
  float* pin = nullptr;      // 4 planes: incoming partial (plane 0), zero planes 1-3
  float* tailp = nullptr;    // 4 planes: outgoing partial
  float* cont = nullptr;     // 4 planes: the continuation's state / finished sum
  float* bsum = nullptr;     // nbsum planes: local block sums
  float* blk = nullptr;      // P stripe rows: the owner's stripe of every piece
  float* relay = nullptr;    // nranks stripe rows: partials in transit
  // raw scalar columns (int64 keys; chained: also the fp32 tails)
  fa_plan* plan64 = nullptr;
  fa_plan* plan_t32 = nullptr;  // compact tail tiles
  int64_t* tidx = nullptr;      // device: bucket index per compact tail column
  float* t32_stack = nullptr;
  float* t32_gather = nullptr;
  float* t32_out = nullptr;
  int64_t* i64_stack = nullptr;
  int64_t* i64_gather = nullptr;
  std::vector<const float*> t32_rows;
  std::vector<const int64_t*> i64_rows;
  std::vector<hipEvent_t> ev;  // start, compute join, done, comm join
  std::map<std::pair<int, int>, std::vector<fa_xfer>> sched;  // (root, weighted) -> ops
  // captured rounds (one process per GPU): the whole schedule of one
  // (root, weights, buffers) call as a HIP graph, replayed by one launch;
  // most recently used first, at most kGraphCache
  struct Graph {
    std::string key;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    std::vector<void*> tables;  // device pointer tables the graph's kernels read
  };
  std::list<Graph> graphs;
  hipStream_t gs = nullptr;     // capture stream
  bool graph_failed = false;    // capture refused once: this plan runs uncaptured
  // one rank (r04): every form is the plain single-GPU reduction of all the
  // slots, one fa_reduce call on this plan (no chunks, planes, copies or
  // empty exchanges)
  fa_plan* single = nullptr;
  // fa_comm_set_profile (r06): event pairs around every group (on the
  // communication stream) and kernel (on its stream) of the last round, and
  // around the whole round on the caller's stream
  struct ProfEv {
    hipEvent_t a = nullptr, b = nullptr;
    int kind = 0;   // 0 exchange group, 1 kernel on the comm stream, 2 on the caller's
  };
  std::vector<ProfEv> prof;
  size_t nprof = 0;
  hipEvent_t prof_t0 = nullptr, prof_t1 = nullptr;
  bool prof_valid = false;
};

namespace {

void free_round(fa_round_plan* p) {
  if (!p) return;
  DeviceGuard dg;
  if (p->device >= 0) (void)hipSetDevice(p->device);
  for (fa_plan* c : p->chunk) fa_plan_destroy(c);
  fa_plan_destroy(p->single);
  fa_plan_destroy(p->plan64);
  fa_plan_destroy(p->plan_t32);
  void* bufs[] = {p->partial,   p->recv,       p->sbuf,    p->state,     p->fin,
                  p->tidx,      p->t32_stack,  p->t32_gather, p->t32_out, p->i64_stack,
                  p->i64_gather, p->pin,       p->tailp,   p->cont,      p->bsum,
                  p->blk,       p->relay,      p->wstage};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  for (hipEvent_t e : p->ev) (void)hipEventDestroy(e);
  for (auto& pe : p->prof) {
    if (pe.a) (void)hipEventDestroy(pe.a);
    if (pe.b) (void)hipEventDestroy(pe.b);
  }
  if (p->prof_t0) (void)hipEventDestroy(p->prof_t0);
  if (p->prof_t1) (void)hipEventDestroy(p->prof_t1);
  for (auto& gr : p->graphs) {
    if (gr.exec) (void)hipGraphExecDestroy(gr.exec);
    if (gr.graph) (void)hipGraphDestroy(gr.graph);
    for (void* t : gr.tables) (void)hipFree(t);
  }
  if (p->gs) (void)hipStreamDestroy(p->gs);
  delete p;
}

// Host-only part of a plan: geometry and the cut.  With `dev`, also the
// device resources (tile plans, scratch, events) on the comm's device.
int build_round(fa_round_plan* p, int nchunks, std::vector<fa_tile_desc>* vec_out,
                std::vector<size_t>* cut_out, std::vector<fa_tile_desc>* tails_out,
                std::vector<int64_t>* tidx_out) {
  const Geo& g = p->g;
  if (p->mode == FA_MODE_SHARDED) {
    shard_ranges(g, nchunks, cut_out, &p->range);
  } else if (p->mode == FA_MODE_STRIPED) {
    // stripes, then each stripe's tiles cut into nchunks column chunks
    std::vector<size_t> cut;
    cut_tiles(g.t32, g.nranks, &cut);
    p->lo = cut_bounds(g.t32, cut, g.f32_numel);
    p->nchunks = nchunks;
    p->clo.assign(g.nranks, std::vector<int64_t>());
    cut_out->clear();
    for (int r = 0; r < g.nranks; ++r) {
      const std::vector<fa_tile_desc> sub(g.t32.begin() + cut[r], g.t32.begin() + cut[r + 1]);
      std::vector<size_t> sc;
      cut_tiles(sub, nchunks, &sc);
      std::vector<int64_t>& b = p->clo[r];
      b.assign(nchunks + 1, p->lo[r + 1]);
      b[0] = p->lo[r];
      for (int c = 1; c < nchunks; ++c)
        if (sc[c] < sub.size()) b[c] = sub[sc[c]].start;
      if (r == g.rank)   // this rank's chunk c = tiles [cut_out[c], cut_out[c + 1])
        for (size_t c = 0; c <= (size_t)nchunks; ++c) cut_out->push_back(cut[r] + sc[c]);
    }
  } else if (p->mode == FA_MODE_CHAINED) {
    chain_geo(g, nchunks, &p->cg, vec_out, cut_out, tails_out, tidx_out);
    p->range = p->cg.range;
  } else {
    chain_geo(g, 1, &p->cg, vec_out, cut_out, tails_out, tidx_out);
    p->range = p->cg.range;
    return block_geo(g, *vec_out, &p->bg);
  }
  return FA_OK;
}

int alloc(void** p, size_t bytes, bool zero) {
  FA_HIP_TRY(hipMalloc(p, std::max<size_t>(bytes, 16)));
  if (zero) FA_HIP_TRY(hipMemset(*p, 0, std::max<size_t>(bytes, 16)));
  return FA_OK;
}

int make_round(fa_comm* comm, int mode, const fa_seg* seg32, int nseg32, int64_t f32_numel,
               const fa_seg* seg64, int nseg64, int64_t i64_numel, const int* counts,
               int nchunks, int xchg, unsigned flags, const char* who, fa_round_plan** out) {
  if (!out) return set_err(FA_E_INVAL, "%s: out is NULL", who);
  *out = nullptr;
  if (!comm || !counts) return set_err(FA_E_INVAL, "%s: NULL comm/counts", who);
  if (nchunks == 0) nchunks = mode == FA_MODE_STRIPED ? kStripeChunks : 8;
  if (nchunks < 1 || nchunks > FA_COMM_MAX_CHUNKS)
    return set_err(FA_E_INVAL, "%s: nchunks=%d", who, nchunks);
  if (xchg != FA_XCHG_REDUCE && xchg != FA_XCHG_RS_GATHER)
    return set_err(FA_E_INVAL, "%s: exchange %d", who, xchg);
  fa_round_plan* p = new fa_round_plan();
  p->mode = mode;
  p->xchg = xchg;
  p->req_chunks = nchunks;
  p->comm = comm;
  p->device = comm->device;
  int rc = make_geo(comm->nranks, comm->rank, counts, seg32, nseg32, f32_numel, seg64, nseg64,
                    i64_numel, flags, who, &p->g);
  if (rc) {
    delete p;
    return rc;
  }
  DeviceGuard dg;
  hipError_t he = hipSetDevice(comm->device);
  if (he != hipSuccess) {
    delete p;
    return set_err(FA_E_HIP, "%s: %s", who, hipGetErrorString(he));
  }
  const Geo& g = p->g;
  std::vector<fa_tile_desc> vec, tails;
  std::vector<size_t> cut;
  std::vector<int64_t> tidx;
  auto fail = [&](int code) {
    free_round(p);
    return code;
  };
  if (g.nranks == 1) {
    // One rank (r04): the round IS the single-GPU
    // reduction — every form's own kernels (chunked chain segments, block
    // sums and their fold, stripe copies, partial sums) and its empty
    // exchanges cost 1.2-2.1x the plain launch on one rank
    // (profiles/r03_native_round_cost_nographs.jsonl), for the same bits.
    rc = fa_plan_create(seg32, nseg32, f32_numel, seg64, nseg64, i64_numel, 0, flags, &p->single);
    if (rc) return fail(rc);
    *out = p;
    return FA_OK;
  }
  if ((rc = build_round(p, nchunks, &vec, &cut, &tails, &tidx))) return fail(rc);
  // tile plans
  if (mode == FA_MODE_SHARDED) {
    for (size_t c = 0; c + 1 < cut.size(); ++c) {
      fa_plan* sub = nullptr;
      rc = fa_plan_create_from_tiles(g.t32.data() + cut[c], (int)(cut[c + 1] - cut[c]),
                                     f32_numel, i64_numel, 0, flags, &sub);
      if (rc) return fail(rc);
      p->chunk.push_back(sub);
    }
    if (!p->chunk.empty() && (rc = alloc((void**)&p->partial, (size_t)f32_numel * 4, true)))
      return fail(rc);
  } else if (mode == FA_MODE_STRIPED) {
    const int me = g.rank;
    const int64_t L = p->lo[me + 1] - p->lo[me];
    // cut: this rank's chunk c = tiles [cut[c], cut[c + 1]) (build_round)
    for (int c = 0; c < p->nchunks; ++c) {
      fa_plan* sub = nullptr;
      if (cut[c] < cut[c + 1]) {
        rc = fa_plan_create_from_tiles(g.t32.data() + cut[c], (int)(cut[c + 1] - cut[c]),
                                       f32_numel, i64_numel, 0, flags, &sub);
        if (rc) return fail(rc);
      }
      p->chunk.push_back(sub);
    }
    if (L > 0) {
      // one row per client slot, 256-B aligned; the stripe starts on a
      // 64-float boundary, so (row - lo) keeps the 16-B alignment
      p->row = (L + 63) / 64 * 64;
      if ((rc = alloc((void**)&p->recv, (size_t)g.n_total * p->row * 4, false))) return fail(rc);
      if ((rc = alloc((void**)&p->sbuf, (size_t)p->row * 4, true))) return fail(rc);
    }
    p->plane = (f32_numel + 63) / 64 * 64;   // WSTAGE row stride (allocated by a weighted round)
  } else {
    for (size_t c = 0; c + 1 < cut.size(); ++c) {
      fa_plan* sub = nullptr;
      rc = fa_plan_create_from_tiles(vec.data() + cut[c], (int)(cut[c + 1] - cut[c]), f32_numel,
                                     0, 0, flags, &sub);
      if (rc) return fail(rc);
      p->chunk.push_back(sub);
    }
    p->plane = (f32_numel + 63) / 64 * 64;
    if (mode == FA_MODE_CHAINED && !p->chunk.empty()) {
      const int nplanes = g.n_total >= 256 ? 4 : 2;
      if ((rc = alloc((void**)&p->state, (size_t)nplanes * p->plane * 4, true))) return fail(rc);
      if (g.rank == p->cg.finisher &&
          (rc = alloc((void**)&p->fin, (size_t)f32_numel * 4, true)))
        return fail(rc);
    }
    if (mode == FA_MODE_BLOCKED && !p->chunk.empty()) {
      const BlockGeo& bg = p->bg;
      const size_t pl = (size_t)p->plane * 4;
      if (bg.tail_piece >= 0 || bg.head_piece >= 0) {
        if ((rc = alloc((void**)&p->pin, 4 * pl, true))) return fail(rc);  // planes 1-3 stay 0
      }
      if (bg.tail_piece >= 0 && (rc = alloc((void**)&p->tailp, 4 * pl, true))) return fail(rc);
      if (bg.head_piece >= 0 && (rc = alloc((void**)&p->cont, 4 * pl, true))) return fail(rc);
      if (bg.nbsum > 0 && (rc = alloc((void**)&p->bsum, (size_t)bg.nbsum * pl, true)))
        return fail(rc);
      const size_t rowb = (size_t)bg.row * 4;
      if ((rc = alloc((void**)&p->blk, (size_t)std::max(1, bg.P) * rowb, true))) return fail(rc);
      if ((rc = alloc((void**)&p->relay, (size_t)g.nranks * rowb, true))) return fail(rc);
      if ((rc = alloc((void**)&p->fin, (size_t)f32_numel * 4, true))) return fail(rc);
    }
    if (!tails.empty()) {
      const int64_t T = p->cg.t32_width;
      rc = fa_plan_create_from_tiles(tails.data(), (int)tails.size(), T, 0, 0, 0, &p->plan_t32);
      if (rc) return fail(rc);
      if ((rc = alloc((void**)&p->tidx, (size_t)T * 8, false))) return fail(rc);
      he = hipMemcpy(p->tidx, tidx.data(), (size_t)T * 8, hipMemcpyHostToDevice);
      if (he != hipSuccess) return fail(set_err(FA_E_HIP, "%s: %s", who, hipGetErrorString(he)));
      const int64_t R = p->cg.t32_row;
      if ((rc = alloc((void**)&p->t32_stack, (size_t)g.nmax * R * 4, true))) return fail(rc);
      if ((rc = alloc((void**)&p->t32_gather, (size_t)g.nranks * g.nmax * R * 4, true)))
        return fail(rc);
      if ((rc = alloc((void**)&p->t32_out, (size_t)((T + 63) / 64 * 64) * 4, true)))
        return fail(rc);
      for (int r = 0; r < g.nranks; ++r)
        for (int j = 0; j < g.counts[r]; ++j)
          p->t32_rows.push_back(p->t32_gather + ((size_t)r * g.nmax + j) * R);
    }
  }
  if (!g.t64.empty()) {
    rc = fa_plan_create_from_tiles(g.t64.data(), (int)g.t64.size(), f32_numel, i64_numel, 0,
                                   flags, &p->plan64);
    if (rc) return fail(rc);
    const size_t rowb = (size_t)i64_numel * 8;
    if ((rc = alloc((void**)&p->i64_stack, (size_t)g.nmax * rowb, true))) return fail(rc);
    if ((rc = alloc((void**)&p->i64_gather, (size_t)g.nranks * g.nmax * rowb, true)))
      return fail(rc);
    for (int r = 0; r < g.nranks; ++r)
      for (int j = 0; j < g.counts[r]; ++j)
        p->i64_rows.push_back(p->i64_gather + ((size_t)r * g.nmax + j) * i64_numel);
  }
  for (int i = 0; i < 4; ++i) {   // start, compute join, done, comm join (striped)
    hipEvent_t e;
    he = hipEventCreateWithFlags(&e, hipEventDisableTiming);
    if (he != hipSuccess) return fail(set_err(FA_E_HIP, "%s: %s", who, hipGetErrorString(he)));
    p->ev.push_back(e);
  }
  *out = p;
  return FA_OK;
}

const std::vector<fa_xfer>& schedule(fa_round_plan* p, int root, bool weighted) {
  auto key = std::make_pair(root, weighted ? 1 : 0);
  auto it = p->sched.find(key);
  if (it != p->sched.end()) return it->second;
  Sched S;
  if (p->mode == FA_MODE_SHARDED) sched_sharded(p->g, p->range, p->xchg, root, weighted, &S);
  else if (p->mode == FA_MODE_STRIPED) sched_striped(p->g, p->clo, root, weighted, &S);
  else if (p->mode == FA_MODE_CHAINED) sched_chained(p->g, p->cg, root, &S);
  else sched_blocked(p->g, p->cg, p->bg, root, &S);
  return p->sched[key] = S.ops;
}

// ------------------------------------------------------------ executor ----
struct Local {
  fa_round_plan* p;
  const fa_shard_io* io;
  hipStream_t user;  // the caller's stream (compute)
  bool comp_dirty;   // compute-stream work the comm stream has not joined yet
  std::vector<const float*> src;  // e2 stripe sources
  // while capturing: the graph's own pointer tables for the kernels over
  // more than FA_INLINE_CLIENTS rows (fa_reduce_tab), taken in order
  const std::vector<void*>* tables = nullptr;
  size_t next_table = 0;
  // blocked fold: piece k's stripe where it lies (NULL: its receive row)
  std::vector<const float*> blk_src;
};

// The table of the next >FA_INLINE_CLIENTS-row kernel of a captured round
// (NULL when not capturing: fa_reduce's own pool).
void* take_table(Local& L) {
  if (!L.tables || L.next_table >= L.tables->size()) return nullptr;
  return (*L.tables)[L.next_table++];
}

ncclDataType_t dtype_of(int buf, int index) {
  return ((buf == FA_B_STACK || buf == FA_B_GATHER) && index == 1) ? ncclInt64 : ncclFloat32;
}

// Device address of (buffer, index, bucket offset).
void* addr(Local& L, int buf, int index, int64_t off) {
  fa_round_plan* p = L.p;
  const fa_shard_io* io = L.io;
  switch (buf) {
    case FA_B_CLIENT: return (void*)(io->c32[index] + off);
    case FA_B_OUT: return io->out32 ? (void*)(io->out32 + off) : nullptr;
    case FA_B_PARTIAL: return p->partial + off;
    case FA_B_RECV: return p->recv + (size_t)index * p->row + (off - p->lo[p->g.rank]);
    case FA_B_STRIPE: return p->sbuf + (off - p->lo[p->g.rank]);
    case FA_B_STATE: return p->state + (size_t)index * p->plane + off;
    case FA_B_FIN: return p->fin + off;
    case FA_B_STACK: return index == 1 ? (void*)(p->i64_stack + off) : (void*)(p->t32_stack + off);
    case FA_B_GATHER:
      return index == 1 ? (void*)(p->i64_gather + off) : (void*)(p->t32_gather + off);
    case FA_B_PIN: return p->pin + (size_t)index * p->plane + off;
    case FA_B_TAILP: return p->tailp + (size_t)index * p->plane + off;
    case FA_B_CONT: return p->cont + (size_t)index * p->plane + off;
    case FA_B_BSUM: return p->bsum + (size_t)index * p->plane + off;
    case FA_B_BLK: return p->blk + (size_t)index * p->bg.row + (off - p->bg.slo[p->g.rank]);
    case FA_B_RELAY: return p->relay + (size_t)index * p->bg.row + (off - p->bg.slo[p->g.rank]);
    case FA_B_WSTAGE: return p->wstage + (size_t)index * p->plane + off;
    default: return nullptr;
  }
}

bool on_comm_stream(const fa_xfer& x) {
  if (is_comm(x.op)) return true;
  switch (x.op) {
    case FA_X_K_SUM:
    case FA_X_K_ZERO:
    case FA_X_K_STACK:
    case FA_X_K_PART:                                // (the zero planes of PIN only)
    case FA_X_K_BLOCK:
    case FA_X_K_SCALE: return false;                 // read local inputs only
    case FA_X_K_STRIPE: return false;                // reads_exchanged: joined below
    case FA_X_K_CHAIN: return x.src == FA_B_STATE;   // after the state's hop
    default: return true;                            // read exchanged data
  }
}

// A compute-stream kernel that reads data exchanged in EARLIER steps (r06:
// the striped round's chunk reduce, beside the next chunk's exchange).  The
// executor records the communication stream's position at the start of the
// step — after the previous steps' groups, before this step's — and the
// caller's stream waits for it before the kernel, so the kernel overlaps
// this step's group.  A schedule must not give such a kernel data its own
// step's group writes (tests/schedsim.py checks it).
bool reads_exchanged(const fa_xfer& x) { return x.op == FA_X_K_STRIPE; }

// Buffers that kernels on the caller's (compute) stream write: partial sums,
// stacked raw columns, the blocked mode's outgoing partial and local block
// sums, and the state / result of a chain segment without a predecessor.
// An exchange or a comm-stream kernel that reads one of them waits for the
// compute stream first; the others (partials in transit, received planes,
// owners' block stripes, gathered rows, client buckets) need not, so they
// overlap the local kernels.  No exchange writes a buffer a compute-stream
// kernel reads or writes (received planes and stripes are comm-side only).
bool user_written(int b) {
  return b == FA_B_PARTIAL || b == FA_B_STACK || b == FA_B_TAILP || b == FA_B_BSUM ||
         b == FA_B_STATE || b == FA_B_OUT || b == FA_B_FIN || b == FA_B_STRIPE ||
         b == FA_B_WSTAGE;
}
bool needs_compute(const fa_xfer& x) { return user_written(x.src); }

int issue_comm(Local& L, const fa_xfer& x) {
  fa_comm* c = L.p->comm;
  const int64_t n = x.count;
  ncclResult_t r = ncclSuccess;
  switch (x.op) {
    case FA_X_SEND:
      r = ncclSend(addr(L, x.src, x.src_index, x.offset), (size_t)n, ncclFloat32, x.peer, c->nc,
                   c->cs);
      break;
    case FA_X_RECV:
      r = ncclRecv(addr(L, x.dst, x.dst_index, x.offset), (size_t)n, ncclFloat32, x.peer, c->nc,
                   c->cs);
      break;
    case FA_X_REDUCE:
      r = ncclReduce(addr(L, x.src, -1, x.offset),
                     x.dst == FA_B_NONE ? addr(L, x.src, -1, x.offset)
                                        : addr(L, x.dst, -1, x.offset),
                     (size_t)n, ncclFloat32, ncclSum, x.peer, c->nc, c->cs);
      break;
    case FA_X_ALLREDUCE:
      r = ncclAllReduce(addr(L, x.src, -1, x.offset), addr(L, x.dst, -1, x.offset), (size_t)n,
                        ncclFloat32, ncclSum, c->nc, c->cs);
      break;
    case FA_X_REDUCE_SCATTER: {
      const int64_t q = n / c->nranks;
      r = ncclReduceScatter(addr(L, x.src, -1, x.offset),
                            addr(L, x.dst, -1, x.offset + (int64_t)c->rank * q), (size_t)q,
                            ncclFloat32, ncclSum, c->nc, c->cs);
      break;
    }
    case FA_X_GATHER: {
      const int64_t q = n / c->nranks;
      // non-root ranks receive nothing; RCCL still gets a valid pointer
      void* dst = x.dst == FA_B_NONE ? addr(L, x.src, -1, x.offset) : addr(L, x.dst, -1, x.offset);
      r = ncclGather(addr(L, x.src, -1, x.offset + (int64_t)c->rank * q), dst, (size_t)q,
                     ncclFloat32, x.peer, c->nc, c->cs);
      break;
    }
    case FA_X_ALLGATHER: {
      if (x.src == FA_B_PARTIAL) {  // e1: every rank's share of the chunk
        const int64_t q = n / c->nranks;
        r = ncclAllGather(addr(L, x.src, -1, x.offset + (int64_t)c->rank * q),
                          addr(L, x.dst, -1, x.offset), (size_t)q, ncclFloat32, c->nc, c->cs);
      } else {                      // raw scalar columns: n = one rank's rows
        r = ncclAllGather(addr(L, x.src, x.src_index, x.offset),
                          addr(L, x.dst, x.dst_index, x.offset), (size_t)n,
                          dtype_of(x.src, x.src_index), c->nc, c->cs);
      }
      break;
    }
    case FA_X_BCAST: {
      void* b = addr(L, x.dst, -1, x.offset);
      r = ncclBroadcast(b, b, (size_t)n, ncclFloat32, x.peer, c->nc, c->cs);
      break;
    }
    default: return set_err(FA_E_INVAL, "schedule: op %d is not an exchange", x.op);
  }
  if (r != ncclSuccess) return set_err(FA_E_COMM, "op %d (peer %d, %lld floats): %s", x.op,
                                       x.peer, (long long)n, ncclGetErrorString(r));
  return FA_OK;
}

int issue_local(Local& L, const fa_xfer& x, hipStream_t s) {
  fa_round_plan* p = L.p;
  const fa_shard_io* io = L.io;
  const Geo& g = p->g;
  switch (x.op) {
    case FA_X_K_SUM:
      return fa_reduce(p->chunk[x.chunk], io->c32, nullptr, x.nrows, io->weights, p->partial,
                       nullptr, FA_F_SUM_ONLY, s);
    case FA_X_K_ZERO:
      FA_HIP_TRY(hipMemsetAsync(p->partial + x.offset, 0, (size_t)x.count * 4, s));
      return FA_OK;
    case FA_X_K_DIV:
      return fa_div_f32(io->out32 + x.offset, (float)g.n_total, io->out32 + x.offset, x.count,
                        s);
    case FA_X_K_COPY:
      // the blocked fold reads an own piece in its plane: bind, do not copy
      if (x.dst == FA_B_BLK && p->bg.P <= kFoldPtrs) {
        if (L.blk_src.size() < (size_t)p->bg.P) L.blk_src.assign(p->bg.P, nullptr);
        L.blk_src[x.dst_index] = (const float*)addr(L, x.src, x.src_index, x.offset);
        return FA_OK;
      }
      {
        // a copy kernel (capture-safe: a D2D hipMemcpyAsync inside a captured
        // round broke the capture, hipErrorStreamCaptureImplicit, r03)
        const float* src = (const float*)addr(L, x.src, x.src_index, x.offset);
        float* dst = (float*)addr(L, x.dst, x.dst_index, x.offset);
        if ((((uintptr_t)src | (uintptr_t)dst) & 15u) == 0)
          return fa_copy_f32(src, dst, x.count, s);
        FA_HIP_TRY(hipMemcpyAsync(dst, src, (size_t)x.count * 4, hipMemcpyDeviceToDevice, s));
      }
      return FA_OK;
    case FA_X_K_STRIPE: {
      // chunk x.chunk of this rank's stripe over all n_total clients: the
      // local clients from their buckets, the others from their receive
      // rows; written straight into the result bucket on a result rank
      fa_plan* cp = p->chunk[x.chunk];
      if (!cp) return FA_OK;
      L.src.assign(p->g.n_total, nullptr);
      for (int k = 0; k < g.n_total; ++k)
        L.src[k] = p->recv + (size_t)k * p->row - p->lo[g.rank];  // element e at [e - lo]
      for (int j = 0; j < g.n_local; ++j) L.src[g.lo_slot + j] = io->c32[j];
      const float* w = nullptr;
      if (io->weights) {   // received rows come pre-multiplied: weight 1
        p->wfull.assign(g.n_total, 1.0f);
        for (int j = 0; j < g.n_local; ++j) p->wfull[g.lo_slot + j] = io->weights[j];
        w = p->wfull.data();
      }
      void* tab = g.n_total > FA_INLINE_CLIENTS ? take_table(L) : nullptr;
      float* out = x.dst == FA_B_OUT ? io->out32 : p->sbuf - p->lo[g.rank];
      return fa_reduce_tab(cp, L.src.data(), nullptr, g.n_total, w, tab, out, nullptr, 0, s);
    }
    case FA_X_K_SCALE: {
      for (int j0 = 0; j0 < x.nrows; j0 += kStackPtrs) {
        ScaleArgs a;
        memset(&a, 0, sizeof a);
        a.rows = std::min(kStackPtrs, x.nrows - j0);
        bool al = ((uintptr_t)(p->wstage + x.offset) & 15u) == 0 && (p->plane & 3) == 0;
        for (int j = 0; j < a.rows; ++j) {
          a.src[j] = io->c32[j0 + j];
          a.w[j] = io->weights[j0 + j];
          al = al && ((uintptr_t)(io->c32[j0 + j] + x.offset) & 15u) == 0;
        }
        a.dst = p->wstage + (size_t)j0 * p->plane;
        a.plane = p->plane;
        a.off = x.offset;
        a.count = x.count;
        a.vec = al ? 1 : 0;
        const int gx = (int)std::min<int64_t>(1024, (x.count / 4 + 255) / 256 + 1);
        hipLaunchKernelGGL(scale_rows_kernel, dim3(gx, a.rows), dim3(256), 0, s, a);
        FA_HIP_TRY(hipGetLastError());
      }
      return FA_OK;
    }
    case FA_X_K_CHAIN: {
      fa_chain ch;
      ch.row0 = x.row0;
      ch.n_total = g.n_total;
      ch.state_in = x.src == FA_B_STATE ? p->state : nullptr;
      ch.state_out = x.dst == FA_B_STATE ? p->state : nullptr;
      ch.plane = p->plane;
      float* out = x.dst == FA_B_OUT ? io->out32 : (x.dst == FA_B_FIN ? p->fin : nullptr);
      return fa_reduce_chain(p->chunk[x.chunk], io->c32, x.nrows, io->weights, &ch, out, 0, s);
    }
    case FA_X_K_STACK: {
      if (p->plan64) {
        const int rc = launch_stack(false, (const void* const*)io->c64, nullptr, g.n_local,
                                    p->i64_stack, nullptr, g.i64_numel, g.i64_numel, s);
        if (rc) return rc;
      }
      if (p->plan_t32)
        return launch_stack(true, (const void* const*)io->c32, io->weights, g.n_local,
                            p->t32_stack, p->tidx, p->cg.t32_width, p->cg.t32_row, s);
      return FA_OK;
    }
    case FA_X_K_TAILS: {
      const bool big = g.n_total > FA_INLINE_CLIENTS;
      if (p->plan64) {
        const int rc = fa_reduce_tab(p->plan64, nullptr, p->i64_rows.data(), g.n_total, nullptr,
                                     big ? take_table(L) : nullptr, nullptr, io->out64, 0, s);
        if (rc) return rc;
      }
      if (p->plan_t32) {
        // pre-multiplied rows when weighted: their plain sum is the weighted order
        const int rc = fa_reduce_tab(p->plan_t32, p->t32_rows.data(), nullptr, g.n_total,
                                     nullptr, big ? take_table(L) : nullptr, p->t32_out,
                                     nullptr, io->weights ? FA_F_SUM_ONLY : 0, s);
        if (rc) return rc;
        const int64_t T = p->cg.t32_width;
        hipLaunchKernelGGL(scatter_f32_kernel, dim3((unsigned)std::min<int64_t>(64, (T + 255) / 256)),
                           dim3(256), 0, s, p->t32_out, p->tidx, io->out32, T);
        FA_HIP_TRY(hipGetLastError());
      }
      return FA_OK;
    }
    case FA_X_K_PART:
    case FA_X_K_CONT: {
      const int j = x.row0 - g.lo_slot;  // first local client of the rows
      fa_chain ch;
      ch.row0 = x.row0;
      ch.n_total = g.n_total;
      ch.state_in = p->pin;
      ch.plane = p->plane;
      const bool finishes = x.row0 + x.nrows == g.n_total;
      ch.state_out = x.op == FA_X_K_PART ? p->tailp : (finishes ? nullptr : p->cont);
      float* out = ch.state_out ? nullptr : p->cont;  // a finishing continuation: plane 0
      return fa_reduce_chain(p->chunk[0], io->c32 + j, x.nrows, io->weights ? io->weights + j
                                                                            : nullptr,
                             &ch, out, FA_F_SUM_ONLY, s);
    }
    case FA_X_K_BLOCK: {
      const int j = x.row0 - g.lo_slot;
      return fa_reduce(p->chunk[0], io->c32 + j, nullptr, x.nrows,
                       io->weights ? io->weights + j : nullptr,
                       p->bsum + (size_t)x.dst_index * p->plane, nullptr, FA_F_SUM_ONLY, s);
    }
    case FA_X_K_FOLD: {
      const BlockGeo& bg = p->bg;
      FoldArgs f;
      f.blk = p->blk;
      f.row = bg.row;
      f.count = x.count;
      f.out = (x.dst == FA_B_OUT ? io->out32 : p->fin) + x.offset;
      f.nblk = bg.K;
      f.has_rem = bg.P > bg.K;
      f.lp = bg.lp;
      f.n_total = g.n_total;
      f.divide = io->weights == nullptr;
      f.bound = bg.P <= kFoldPtrs;
      if (f.bound) {
        for (int k = 0; k < bg.P; ++k) {
          const float* own = k < (int)L.blk_src.size() ? L.blk_src[k] : nullptr;
          f.src[k] = own ? own : p->blk + (size_t)k * bg.row;
        }
        L.blk_src.assign(L.blk_src.size(), nullptr);
      }
      const unsigned grid = (unsigned)std::min<int64_t>(2048, (x.count + 255) / 256);
      hipLaunchKernelGGL(fold_kernel, dim3(std::max(1u, grid)), dim3(256), 0, s, f);
      FA_HIP_TRY(hipGetLastError());
      return FA_OK;
    }
    default: return set_err(FA_E_INVAL, "schedule: op %d is not local", x.op);
  }
}

// The next profiling event pair of a plan's round (fa_comm_set_profile).
int prof_pair(fa_round_plan* p, int kind, fa_round_plan::ProfEv** out) {
  if (p->nprof == p->prof.size()) {
    fa_round_plan::ProfEv e;
    FA_HIP_TRY(hipEventCreate(&e.a));
    FA_HIP_TRY(hipEventCreate(&e.b));
    p->prof.push_back(e);
  }
  *out = &p->prof[p->nprof++];
  (*out)->kind = kind;
  return FA_OK;
}

// Walk the local GPUs' schedules step by step: one RCCL group per step over
// every local GPU's exchanges, then the step's kernels.
int execute(std::vector<Local>& locals, const std::vector<const std::vector<fa_xfer>*>& scheds) {
  const size_t nl = locals.size();
  std::vector<size_t> pos(nl, 0);
  for (size_t d = 0; d < nl; ++d) {
    fa_round_plan* p = locals[d].p;
    FA_HIP_TRY(hipSetDevice(p->comm->device));
    if (p->comm->profile) {
      if (!p->prof_t0) FA_HIP_TRY(hipEventCreate(&p->prof_t0));
      if (!p->prof_t1) FA_HIP_TRY(hipEventCreate(&p->prof_t1));
      p->nprof = 0;
      p->prof_valid = false;
      FA_HIP_TRY(hipEventRecord(p->prof_t0, locals[d].user));
    }
    // the inputs are ready on the caller's stream
    FA_HIP_TRY(hipEventRecord(p->ev[0], locals[d].user));
    FA_HIP_TRY(hipStreamWaitEvent(p->comm->cs, p->ev[0], 0));
    locals[d].comp_dirty = false;
  }
  int step = 0;
  for (;;) {
    bool any = false, comm = false;
    std::vector<char> join(nl, 0), xread(nl, 0);
    for (size_t d = 0; d < nl; ++d) {
      const std::vector<fa_xfer>& o = *scheds[d];
      for (size_t i = pos[d]; i < o.size() && o[i].step == step; ++i) {
        any = true;
        if (is_comm(o[i].op)) {
          comm = true;
          join[d] |= needs_compute(o[i]);
        }
        xread[d] |= reads_exchanged(o[i]);
      }
      if (pos[d] < o.size()) any = true;
    }
    if (!any) break;
    // the communication stream's position before this step's group: what a
    // compute-stream kernel reading earlier steps' exchanges waits for
    for (size_t d = 0; d < nl; ++d) {
      if (!xread[d]) continue;
      FA_HIP_TRY(hipSetDevice(locals[d].p->comm->device));
      FA_HIP_TRY(hipEventRecord(locals[d].p->ev[3], locals[d].p->comm->cs));
    }
    // comm stream joins the compute stream before this step's exchanges when
    // one of them reads compute-stream output
    if (comm) {
      for (size_t d = 0; d < nl; ++d) {
        Local& L = locals[d];
        if (!L.comp_dirty || !join[d]) continue;
        FA_HIP_TRY(hipSetDevice(L.p->comm->device));
        FA_HIP_TRY(hipEventRecord(L.p->ev[1], L.user));
        FA_HIP_TRY(hipStreamWaitEvent(L.p->comm->cs, L.p->ev[1], 0));
        L.comp_dirty = false;
      }
      std::vector<fa_round_plan::ProfEv*> gev(nl, nullptr);
      for (size_t d = 0; d < nl; ++d) {
        fa_round_plan* p = locals[d].p;
        if (!p->comm->profile) continue;
        bool has = false;
        for (size_t i = pos[d]; i < scheds[d]->size() && (*scheds[d])[i].step == step; ++i)
          has |= is_comm((*scheds[d])[i].op);
        if (!has) continue;
        FA_HIP_TRY(hipSetDevice(p->comm->device));
        const int rc = prof_pair(p, 0, &gev[d]);
        if (rc) return rc;
        FA_HIP_TRY(hipEventRecord(gev[d]->a, p->comm->cs));
      }
      NCCL_TRY(ncclGroupStart());
      for (size_t d = 0; d < nl; ++d) {
        const std::vector<fa_xfer>& o = *scheds[d];
        (void)hipSetDevice(locals[d].p->comm->device);
        for (size_t i = pos[d]; i < o.size() && o[i].step == step; ++i) {
          if (!is_comm(o[i].op)) continue;
          const int rc = issue_comm(locals[d], o[i]);
          if (rc) {
            ncclGroupEnd();
            return rc;
          }
        }
      }
      NCCL_TRY(ncclGroupEnd());
      for (size_t d = 0; d < nl; ++d) {
        if (!gev[d]) continue;
        FA_HIP_TRY(hipSetDevice(locals[d].p->comm->device));
        FA_HIP_TRY(hipEventRecord(gev[d]->b, locals[d].p->comm->cs));
      }
    }
    for (size_t d = 0; d < nl; ++d) {
      Local& L = locals[d];
      const std::vector<fa_xfer>& o = *scheds[d];
      FA_HIP_TRY(hipSetDevice(L.p->comm->device));
      for (; pos[d] < o.size() && o[pos[d]].step == step; ++pos[d]) {
        const fa_xfer& x = o[pos[d]];
        if (is_comm(x.op)) continue;
        const bool cs = on_comm_stream(x);
        if (cs && L.comp_dirty && needs_compute(x)) {
          FA_HIP_TRY(hipEventRecord(L.p->ev[1], L.user));
          FA_HIP_TRY(hipStreamWaitEvent(L.p->comm->cs, L.p->ev[1], 0));
          L.comp_dirty = false;
        }
        if (!cs && reads_exchanged(x)) FA_HIP_TRY(hipStreamWaitEvent(L.user, L.p->ev[3], 0));
        const hipStream_t ks = cs ? L.p->comm->cs : L.user;
        fa_round_plan::ProfEv* kev = nullptr;
        if (L.p->comm->profile) {
          const int prc = prof_pair(L.p, cs ? 1 : 2, &kev);
          if (prc) return prc;
          FA_HIP_TRY(hipEventRecord(kev->a, ks));
        }
        const int rc = issue_local(L, x, ks);
        if (rc) return rc;
        if (kev) FA_HIP_TRY(hipEventRecord(kev->b, ks));
        if (!cs) L.comp_dirty = true;
      }
    }
    ++step;
  }
  // the caller's stream joins the communication stream
  for (size_t d = 0; d < nl; ++d) {
    Local& L = locals[d];
    FA_HIP_TRY(hipSetDevice(L.p->comm->device));
    FA_HIP_TRY(hipEventRecord(L.p->ev[2], L.p->comm->cs));
    FA_HIP_TRY(hipStreamWaitEvent(L.user, L.p->ev[2], 0));
    if (L.p->comm->profile) {
      FA_HIP_TRY(hipEventRecord(L.p->prof_t1, L.user));
      L.p->prof_valid = true;
    }
  }
  return FA_OK;
}

// ------------------------------------------------------ captured rounds ----
// One process per GPU: a round's whole schedule (its RCCL groups on the
// communication stream, its kernels on both streams, the event joins) is
// captured into a HIP graph once per (root, weights, buffers) and replayed by
// one hipGraphLaunch on the caller's stream — the executor issued ~12 µs of
// host calls per step (chained at 16 chunks: 190 µs of host issue per round,
// profiles/r02_native_round_cost.jsonl).  Measured r03 on one rank
// (profiles/r03_native_round_cost_{graphs,nographs}.jsonl): the replay's
// host time is still ~9 µs per node (chained_16 184 vs 192 µs: ROCm 7.0's
// graph launch submits node by node), and its GPU time gains on the blocked
// and striped rounds (244 vs 259, 188 vs 214 µs) but loses where the
// schedule overlaps its two streams (sharded 357 vs 290 µs, chained 181 vs
// 171 µs) — so it is off by default (fa_comm_set_graphs).  The capture runs on the plan's own
// stream (the caller's may be the legacy null stream, which cannot be
// captured); kernels over more than FA_INLINE_CLIENTS rows take pointer
// tables the graph owns (fa_reduce_tab).  A round whose other kernels exceed
// that row count, or a capture the runtime or RCCL refuses, runs uncaptured.
constexpr size_t kGraphCache = 4;

std::string graph_key(const Local& L, int root, bool weighted) {
  const Geo& g = L.p->g;
  const fa_shard_io* io = L.io;
  std::string k;
  auto put = [&](const void* p, size_t n) { k.append((const char*)p, n); };
  put(&root, sizeof root);
  put(&weighted, sizeof weighted);
  put(&io->out32, sizeof io->out32);
  put(&io->out64, sizeof io->out64);
  if (g.n_local > 0) {
    put(io->c32, sizeof(void*) * g.n_local);
    if (io->c64) put(io->c64, sizeof(void*) * g.n_local);
    if (io->weights) put(io->weights, sizeof(float) * g.n_local);
  }
  return k;
}

// Kernel ops other than the stripe / tails reductions take inline pointer
// lists only up to FA_INLINE_CLIENTS rows; count the tables those two need.
bool capturable(const fa_round_plan* p, const std::vector<fa_xfer>& ops, size_t* ntables) {
  *ntables = 0;
  const bool big = p->g.n_total > FA_INLINE_CLIENTS;
  for (const fa_xfer& x : ops) {
    // RCCL's ncclReduceScatter / ncclGather crash under stream capture (a
    // segfault in the capturing call, one-rank communicator, ROCm 7.2): the
    // reduce-scatter + gather exchange runs uncaptured
    if (x.op == FA_X_REDUCE_SCATTER || x.op == FA_X_GATHER) return false;
    if (is_comm(x.op)) continue;
    if (x.op == FA_X_K_STRIPE) {
      *ntables += big ? 1 : 0;
    } else if (x.op == FA_X_K_TAILS) {
      *ntables += big ? (p->plan64 ? 1 : 0) + (p->plan_t32 ? 1 : 0) : 0;
    } else if (x.nrows > FA_INLINE_CLIENTS ||
               (x.op == FA_X_K_SUM && p->g.n_local > FA_INLINE_CLIENTS)) {
      return false;
    }
  }
  return true;
}

// true: the round ran from a graph (rc = its status); false: run it uncaptured.
bool replay_graph(Local& L, const std::vector<fa_xfer>& ops, int root, bool weighted, int* rc) {
  fa_round_plan* p = L.p;
  size_t ntables = 0;
  if (!capturable(p, ops, &ntables)) return false;
  if (hipSetDevice(p->comm->device) != hipSuccess) return false;
  const std::string key = graph_key(L, root, weighted);
  for (auto it = p->graphs.begin(); it != p->graphs.end(); ++it) {
    if (it->key != key) continue;
    p->graphs.splice(p->graphs.begin(), p->graphs, it);
    const hipError_t e = hipGraphLaunch(p->graphs.front().exec, L.user);
    *rc = e == hipSuccess ? FA_OK
                          : set_err(FA_E_HIP, "hipGraphLaunch: %s", hipGetErrorString(e));
    return true;
  }
  if (!p->gs && hipStreamCreateWithFlags(&p->gs, hipStreamNonBlocking) != hipSuccess) {
    p->graph_failed = true;
    return false;
  }
  fa_round_plan::Graph gr;
  gr.key = key;
  const size_t tb = fa_table_bytes(p->g.n_total);
  for (size_t i = 0; i < ntables; ++i) {
    void* t = nullptr;
    if (hipMalloc(&t, std::max<size_t>(tb, 16)) != hipSuccess) {
      for (void* x : gr.tables) (void)hipFree(x);
      return false;
    }
    gr.tables.push_back(t);
  }
  auto drop = [&](fa_round_plan::Graph& x) {
    if (x.exec) (void)hipGraphExecDestroy(x.exec);
    if (x.graph) (void)hipGraphDestroy(x.graph);
    for (void* t : x.tables) (void)hipFree(t);
  };
  // capture on the plan's stream: the executor's "caller stream" is gs
  Local C = L;
  C.user = p->gs;
  C.tables = &gr.tables;
  C.next_table = 0;
  hipError_t e = hipStreamBeginCapture(p->gs, hipStreamCaptureModeRelaxed);
  if (e != hipSuccess) {
    drop(gr);
    p->graph_failed = true;
    return false;
  }
  std::vector<Local> one{C};
  std::vector<const std::vector<fa_xfer>*> sc{&ops};
  const int erc = execute(one, sc);
  e = hipStreamEndCapture(p->gs, &gr.graph);
  if (getenv("FA_GRAPH_DEBUG"))
    fprintf(stderr, "fedcomm capture: execute rc=%d (%s) end=%s graph=%p\n", erc,
            erc ? fa_last_error() : "", hipGetErrorString(e), (void*)gr.graph);
  if (erc != FA_OK || e != hipSuccess || !gr.graph) {
    drop(gr);
    (void)hipGetLastError();
    p->graph_failed = true;   // the runtime or RCCL refused: uncaptured from now on
    return false;
  }
  e = hipGraphInstantiate(&gr.exec, gr.graph, nullptr, nullptr, 0);
  if (e != hipSuccess) {
    drop(gr);
    p->graph_failed = true;
    return false;
  }
  p->graphs.push_front(std::move(gr));
  while (p->graphs.size() > kGraphCache) {
    drop(p->graphs.back());
    p->graphs.pop_back();
  }
  e = hipGraphLaunch(p->graphs.front().exec, L.user);
  *rc = e == hipSuccess ? FA_OK : set_err(FA_E_HIP, "hipGraphLaunch: %s", hipGetErrorString(e));
  return true;
}

int run_round(fa_round_plan* const* plans, int nlocal, const fa_shard_io* io, int root, int mode,
              const char* who) {
  if (nlocal < 1 || !plans || !io) return set_err(FA_E_INVAL, "%s: bad arguments", who);
  const bool weighted = io[0].weights != nullptr;
  std::vector<Local> locals;
  std::vector<const std::vector<fa_xfer>*> scheds;
  for (int d = 0; d < nlocal; ++d) {
    fa_round_plan* p = plans[d];
    if (!p) return set_err(FA_E_INVAL, "%s: plan %d is NULL", who, d);
    if (p->mode != mode) return set_err(FA_E_INVAL, "%s: plan %d is of another mode", who, d);
    if (root >= p->comm->nranks) return set_err(FA_E_INVAL, "%s: root=%d", who, root);
    if ((io[d].weights != nullptr) != weighted)
      return set_err(FA_E_INVAL, "%s: weights on some GPUs only", who);
    const Geo& g = p->g;
    const bool result = root < 0 || root == g.rank;
    if (g.n_local > 0 && !io[d].c32)
      return set_err(FA_E_INVAL, "%s: fp32 buckets required (GPU %d)", who, d);
    if (g.n_local > 0 && !g.t64.empty() && !io[d].c64)
      return set_err(FA_E_INVAL, "%s: int64 buckets required (GPU %d)", who, d);
    if (result && (!io[d].out32 || (!g.t64.empty() && !io[d].out64)))
      return set_err(FA_E_INVAL, "%s: result buckets required on rank %d", who, g.rank);
    if (p->g.n_total != plans[0]->g.n_total || p->range.size() != plans[0]->range.size())
      return set_err(FA_E_INVAL, "%s: plans of different layouts", who);
    if (p->single) {
      // one rank: the plain reduction (fa_reduce's own checks apply)
      if (nlocal != 1) return set_err(FA_E_INVAL, "%s: a one-rank plan drives one GPU", who);
      DeviceGuard dg1;
      const hipError_t he = hipSetDevice(p->device);
      if (he != hipSuccess) return set_err(FA_E_HIP, "%s: %s", who, hipGetErrorString(he));
      return fa_reduce(p->single, io[d].c32, io[d].c64, g.n_total, io[d].weights, io[d].out32,
                       io[d].out64, 0, io[d].stream);
    }
    if (weighted && mode == FA_MODE_STRIPED && !p->wstage && g.n_local > 0) {
      // the first weighted round: the staging buckets of the pre-multiplied
      // client rows (before any capture: no allocation inside a graph)
      DeviceGuard dg2;
      FA_HIP_TRY(hipSetDevice(p->device));
      const int rc = alloc((void**)&p->wstage, (size_t)g.n_local * p->plane * 4, false);
      if (rc) return rc;
    }
    Local L;
    L.p = p;
    L.io = &io[d];
    L.user = (hipStream_t)io[d].stream;
    L.comp_dirty = false;
    locals.push_back(L);
    scheds.push_back(&schedule(p, root, weighted));
  }
  DeviceGuard dg;
  if (nlocal == 1 && plans[0]->comm->graphs && !plans[0]->graph_failed &&
      !plans[0]->comm->profile) {
    int rc = FA_OK;
    if (replay_graph(locals[0], *scheds[0], root, weighted, &rc)) return rc;
  }
  return execute(locals, scheds);
}

// ============================================================ cost model ==
// (r06; fedagg_comm.h fa_round_model.)  Every
// rank's schedule replayed in virtual time under the executor's stream rules
// (execute above): per rank the communication stream (tc) and the caller's
// stream (tu).  tests/roundmodel.py restates it and checks it against this.
// The model's constants: fedagg_comm.h's FA_MODEL_* unless the process
// environment sets a positive FA_MODEL_LINK_GBPS / FA_MODEL_HBM_GBPS /
// FA_MODEL_GROUP_US / FA_MODEL_KERNEL_US (read once), so numbers measured on
// a multi-GPU node re-rank the forms without a rebuild.
struct ModelConst {
  double link_gbps, hbm_gbps, group_us, kernel_us;
};
double env_or(const char* name, double dflt, bool allow_zero) {
  const char* v = std::getenv(name);
  if (!v || !*v) return dflt;
  char* end = nullptr;
  const double x = std::strtod(v, &end);
  return (end && *end == '\0' && (x > 0.0 || (allow_zero && x == 0.0))) ? x : dflt;
}
const ModelConst& mc() {
  static const ModelConst c{env_or("FA_MODEL_LINK_GBPS", FA_MODEL_LINK_GBPS, false),
                            env_or("FA_MODEL_HBM_GBPS", FA_MODEL_HBM_GBPS, false),
                            env_or("FA_MODEL_GROUP_US", FA_MODEL_GROUP_US, true),
                            env_or("FA_MODEL_KERNEL_US", FA_MODEL_KERNEL_US, true)};
  return c;
}
inline double us_link(double bytes) { return bytes / (mc().link_gbps * 1e3); }
inline double us_hbm(double bytes) { return bytes / (mc().hbm_gbps * 1e3); }

int popc(unsigned v) { return __builtin_popcount(v); }

// HBM bytes a kernel op reads and writes (the columns it covers; count 0 =
// the vector columns, V elements); the scalar-column stacks and their
// reductions are a few KB and cost only their launch.
double kernel_bytes(const fa_xfer& x, int n_total, int64_t V) {
  const double b = 4.0 * (double)(x.count > 0 ? x.count : V);
  switch (x.op) {
    case FA_X_K_SUM:
    case FA_X_K_STRIPE:
    case FA_X_K_FOLD:
    case FA_X_K_PART:
    case FA_X_K_BLOCK: return (x.nrows + 1) * b;
    case FA_X_K_CONT: return (x.nrows + 2) * b;
    case FA_X_K_CHAIN: {
      const int lin = x.src == FA_B_STATE ? popc(fa_chain_levels(x.row0, n_total)) : 0;
      const int lout = x.dst == FA_B_STATE ? popc(fa_chain_levels(x.row0 + x.nrows, n_total)) : 1;
      return (x.nrows + lin + std::max(lout, 1)) * b;
    }
    case FA_X_K_COPY: return x.dst == FA_B_BLK ? 0.0 : 2 * b;
    case FA_X_K_DIV: return 2 * b;
    case FA_X_K_ZERO: return b;
    case FA_X_K_SCALE: return 2.0 * x.nrows * b;
    default: return 0.0;   // K_STACK, K_TAILS
  }
}

double elem_bytes(const fa_xfer& x) {
  const int buf = x.op == FA_X_RECV ? x.dst : x.src;
  const int idx = x.op == FA_X_RECV ? x.dst_index : x.src_index;
  return dtype_of(buf, idx) == ncclInt64 ? 8.0 : 4.0;
}

// A collective's bytes on each link direction of a rank (ring algorithms).
double coll_link_bytes(const fa_xfer& x, int W) {
  const double es = elem_bytes(x), n = (double)x.count * es;
  switch (x.op) {
    case FA_X_ALLGATHER:
      return x.src == FA_B_PARTIAL ? n * (W - 1) / W : n * (W - 1);
    case FA_X_BCAST: return n;
    case FA_X_ALLREDUCE: return 2.0 * n * (W - 1) / W;
    default: return n * (W - 1) / W;   // REDUCE, REDUCE_SCATTER, GATHER
  }
}

int model_schedules(const std::vector<std::vector<fa_xfer>>& sch, int n_total, int64_t V,
                    fa_round_cost* out) {
  const int W = (int)sch.size();
  std::vector<size_t> pos(W, 0);
  std::vector<char> posted(W, 0);
  std::vector<double> tc(W, 0.0), tu(W, 0.0), post(W, 0.0), ev3(W, 0.0);
  std::vector<double> hbm(W, 0.0);
  std::vector<std::vector<double>> lout(W, std::vector<double>(W, 0.0)),
      lin(W, std::vector<double>(W, 0.0));
  std::vector<int> groups(W, 0);
  // p2p matching: the post times of each channel's sends / receives in order
  std::map<std::pair<int, int>, std::vector<double>> sendt, recvt;
  std::map<uint64_t, std::vector<double>> collt;
  std::vector<uint64_t> cseq(W, 0);
  struct Pend {
    std::vector<std::pair<int, size_t>> p2p;  // (op index, channel position)
    std::vector<uint64_t> coll;
  };
  std::vector<Pend> pend(W);
  int steps = 0;
  for (;;) {
    bool progress = false, done = true;
    for (int r = 0; r < W; ++r) {
      const std::vector<fa_xfer>& o = sch[r];
      if (pos[r] >= o.size()) continue;
      done = false;
      const int step = o[pos[r]].step;
      size_t e = pos[r];
      while (e < o.size() && o[e].step == step) ++e;
      steps = std::max(steps, step + 1);
      if (!posted[r]) {
        ev3[r] = tc[r];
        bool join = false, comm = false;
        for (size_t i = pos[r]; i < e; ++i)
          if (is_comm(o[i].op)) {
            comm = true;
            join |= needs_compute(o[i]);
          }
        if (join) tc[r] = std::max(tc[r], tu[r]);
        post[r] = tc[r];
        pend[r] = Pend();
        for (size_t i = pos[r]; i < e; ++i) {
          const fa_xfer& x = o[i];
          if (x.op == FA_X_SEND) {
            auto& v = sendt[{r, x.peer}];
            pend[r].p2p.push_back({(int)i, v.size()});
            v.push_back(post[r]);
          } else if (x.op == FA_X_RECV) {
            auto& v = recvt[{x.peer, r}];
            pend[r].p2p.push_back({(int)i, v.size()});
            v.push_back(post[r]);
          } else if (is_comm(x.op)) {
            const uint64_t q = cseq[r]++;
            auto& v = collt[q];
            if (v.empty()) v.assign(W, -1.0);
            v[r] = post[r];
            pend[r].coll.push_back(q);
          }
        }
        if (comm) ++groups[r];
        posted[r] = 1;
        progress = true;
      }
      // complete once every peer has posted the matching operations
      double start = post[r];
      bool ok = true;
      for (const auto& pe : pend[r].p2p) {
        const fa_xfer& x = o[pe.first];
        const auto& v = x.op == FA_X_SEND ? recvt[{r, x.peer}] : sendt[{x.peer, r}];
        if (v.size() <= pe.second) {
          ok = false;
          break;
        }
        start = std::max(start, v[pe.second]);
      }
      for (uint64_t q : pend[r].coll) {
        if (!ok) break;
        for (double t : collt[q]) {
          if (t < 0) {
            ok = false;
            break;
          }
          start = std::max(start, t);
        }
      }
      if (!ok) continue;
      // the group
      std::vector<double> go(W, 0.0), gi(W, 0.0);
      double ghbm = 0.0, gcoll = 0.0;
      bool comm = false;
      for (size_t i = pos[r]; i < e; ++i) {
        const fa_xfer& x = o[i];
        if (!is_comm(x.op)) continue;
        comm = true;
        if (x.op == FA_X_SEND || x.op == FA_X_RECV) {
          const double b = (double)x.count * elem_bytes(x);
          (x.op == FA_X_SEND ? go : gi)[x.peer] += b;
          (x.op == FA_X_SEND ? lout : lin)[r][x.peer] += b;
          ghbm += b;
        } else {
          const double b = coll_link_bytes(x, W);
          gcoll += b;
          ghbm += 2.0 * b;
        }
      }
      if (comm) {
        double link = gcoll;
        for (int q = 0; q < W; ++q) link = std::max(link, std::max(go[q], gi[q]));
        tc[r] = start + mc().group_us + std::max(us_link(link), us_hbm(ghbm));
        hbm[r] += ghbm;
      }
      // the kernels
      for (size_t i = pos[r]; i < e; ++i) {
        const fa_xfer& x = o[i];
        if (is_comm(x.op)) continue;
        const double kb = kernel_bytes(x, n_total, V);
        const double dur = mc().kernel_us + us_hbm(kb);
        hbm[r] += kb;
        if (on_comm_stream(x)) {
          if (needs_compute(x)) tc[r] = std::max(tc[r], tu[r]);
          tc[r] += dur;
        } else {
          if (reads_exchanged(x)) tu[r] = std::max(tu[r], ev3[r]);
          tu[r] += dur;
        }
      }
      pos[r] = e;
      posted[r] = 0;
      progress = true;
    }
    if (done) break;
    if (!progress) return set_err(FA_E_INVAL, "fa_round_model: the schedules deadlock");
  }
  fa_round_cost c{};
  for (int r = 0; r < W; ++r) {
    c.model_us = std::max(c.model_us, std::max(tc[r], tu[r]));
    c.hbm_bytes_max = std::max(c.hbm_bytes_max, hbm[r]);
    for (int q = 0; q < W; ++q)
      c.link_bytes_max = std::max(c.link_bytes_max, std::max(lout[r][q], lin[r][q]));
    c.groups = std::max(c.groups, groups[r]);
  }
  c.steps = steps;
  *out = c;
  return FA_OK;
}

// Every rank's schedule of a form (host only), from one geometry.
int all_schedules(const Geo& base, int mode, int nchunks, int xchg, int root, bool weighted,
                  std::vector<std::vector<fa_xfer>>* sch, int64_t* V) {
  sch->assign(base.nranks, {});
  *V = 0;
  for (const fa_tile_desc& t : base.t32)
    if (t.kind == 0) *V += t.count;
  for (int r = 0; r < base.nranks; ++r) {
    fa_round_plan p;
    p.mode = mode;
    p.xchg = xchg;
    p.req_chunks = nchunks;
    p.g = base;
    p.g.rank = r;
    p.g.n_local = base.counts[r];
    p.g.lo_slot = base.first[r];
    std::vector<fa_tile_desc> vec, tails;
    std::vector<size_t> cut;
    std::vector<int64_t> tidx;
    const int rc = build_round(&p, nchunks, &vec, &cut, &tails, &tidx);
    if (rc) return rc;
    (*sch)[r] = schedule(&p, root, weighted);
  }
  return FA_OK;
}

// The default entry's choice (fa_multi_select_layout): the exact form and
// chunk count with the lowest modelled time; ties keep the earlier candidate
// (blocked, then chained, then striped, fewer chunks first).
int select_form(const Geo& base, unsigned mflags, int* mode, int* nchunks, double* us) {
  if (mflags & FA_MULTI_REASSOCIATE) {
    *mode = FA_MODE_SHARDED;
    *nchunks = 8;
    if (us) *us = -1.0;
    return FA_OK;
  }
  if (base.nranks == 1) {   // every form is the plain reduction (make_round)
    *mode = first_wide_block(1, base.counts.data(), nullptr, nullptr) < 0 ? FA_MODE_BLOCKED
                                                                         : FA_MODE_CHAINED;
    *nchunks = 1;
    // fa_round_model's one-rank cost: one kernel reading n_total buckets and
    // writing one
    if (us)
      *us = mc().kernel_us + us_hbm((double)(base.n_total + 1) *
                                        (4.0 * (double)base.f32_numel +
                                         8.0 * (double)base.i64_numel));
    return FA_OK;
  }
  int root = -1;
  if (!(mflags & FA_MULTI_ROOT_ALL))
    for (int r = 0; r < base.nranks; ++r)
      if (base.counts[r] > 0) root = r;
  struct Cand {
    int mode, nchunks;
  };
  std::vector<Cand> cand;
  if (first_wide_block(base.nranks, base.counts.data(), nullptr, nullptr) < 0)
    cand.push_back({FA_MODE_BLOCKED, 1});
  for (int c : {4, 8, 16, 32}) cand.push_back({FA_MODE_CHAINED, c});
  for (int c : {1, 2, 4, 8}) cand.push_back({FA_MODE_STRIPED, c});
  double best = 0.0;
  *mode = -1;
  for (const Cand& k : cand) {
    std::vector<std::vector<fa_xfer>> sch;
    int64_t V = 0;
    int rc = all_schedules(base, k.mode, k.nchunks, FA_XCHG_REDUCE, root, false, &sch, &V);
    if (rc) return rc;
    fa_round_cost c{};
    if ((rc = model_schedules(sch, base.n_total, V, &c))) return rc;
    if (*mode < 0 || c.model_us < best) {
      best = c.model_us;
      *mode = k.mode;
      *nchunks = k.nchunks;
    }
  }
  if (us) *us = best;
  return FA_OK;
}

// fa_mean_f32_multi's shard plans, by (communicator, layout, counts); a
// communicator's entries go with it (fa_comm_destroy).
std::mutex g_multi_mu;
std::map<std::string, fa_round_plan*> g_multi;

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
        free_round(it->second);
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

int fa_comm_set_graphs(fa_comm* c, int enable) {
  if (!c) return set_err(FA_E_INVAL, "fa_comm_set_graphs: NULL comm");
  c->graphs = enable != 0;
  return FA_OK;
}

int fa_comm_set_profile(fa_comm* c, int enable) {
  if (!c) return set_err(FA_E_INVAL, "fa_comm_set_profile: NULL comm");
  c->profile = enable != 0;
  return FA_OK;
}

int fa_round_plan_profile(const void* plan, fa_round_profile* out) {
  if (!plan || !out) return set_err(FA_E_INVAL, "fa_round_plan_profile: NULL argument");
  const fa_round_plan* p = (const fa_round_plan*)plan;
  memset(out, 0, sizeof *out);
  if (!p->prof_valid) return set_err(FA_E_INVAL, "fa_round_plan_profile: no profiled round");
  DeviceGuard dg;
  FA_HIP_TRY(hipSetDevice(p->device));
  FA_HIP_TRY(hipEventSynchronize(p->prof_t1));
  float ms = 0.f;
  FA_HIP_TRY(hipEventElapsedTime(&ms, p->prof_t0, p->prof_t1));
  out->wall_us = 1e3 * ms;
  for (size_t i = 0; i < p->nprof; ++i) {
    const fa_round_plan::ProfEv& e = p->prof[i];
    FA_HIP_TRY(hipEventElapsedTime(&ms, e.a, e.b));
    if (e.kind == 0) {
      out->exchange_us += 1e3 * ms;
      ++out->groups;
    } else {
      (e.kind == 1 ? out->comm_kernel_us : out->compute_kernel_us) += 1e3 * ms;
      ++out->kernels;
    }
  }
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
  return fa_shard_plan_create_ex(comm, seg32, nseg32, f32_numel, seg64, nseg64, i64_numel, counts,
                                 nchunks, FA_XCHG_REDUCE, flags, out);
}

int fa_shard_plan_create_ex(fa_comm* comm, const fa_seg* seg32, int nseg32, int64_t f32_numel,
                            const fa_seg* seg64, int nseg64, int64_t i64_numel, const int* counts,
                            int nchunks, int exchange, unsigned flags, fa_shard_plan** out) {
  return make_round(comm, FA_MODE_SHARDED, seg32, nseg32, f32_numel, seg64, nseg64, i64_numel,
                    counts, nchunks, exchange, flags, "fa_shard_plan_create",
                    (fa_round_plan**)out);
}

int fa_shard_plan_destroy(fa_shard_plan* p) {
  free_round((fa_round_plan*)p);
  return FA_OK;
}

int fa_reduce_sharded(fa_shard_plan* const* plans, int nlocal, const fa_shard_io* io, int root) {
  return run_round((fa_round_plan* const*)plans, nlocal, io, root, FA_MODE_SHARDED,
                   "fa_reduce_sharded");
}

// ================================================ default (r05, r06) ====
// The default multi-GPU entry: the exact form and chunk count with the lowest
// modelled time (select_form; r05: blocked if every cascade block lies on at
// most two ranks, else chained); e1 only on request (FA_MULTI_REASSOCIATE).
int fa_multi_select_layout(int nranks, const int* counts, const fa_seg* seg32, int nseg32,
                           int64_t f32_numel, const fa_seg* seg64, int nseg64, int64_t i64_numel,
                           unsigned flags, unsigned mflags, int* mode, int* nchunks,
                           double* model_us) {
  if (!mode || !nchunks) return set_err(FA_E_INVAL, "fa_multi_select: mode/nchunks is NULL");
  *mode = -1;
  *nchunks = 0;
  if (nranks < 1 || !counts) return set_err(FA_E_INVAL, "fa_multi_select: bad arguments");
  if (mflags & ~(unsigned)(FA_MULTI_REASSOCIATE | FA_MULTI_ROOT_ALL))
    return set_err(FA_E_INVAL, "fa_multi_select: unknown flags 0x%x", mflags);
  Geo g;
  const int rc = make_geo(nranks, 0, counts, seg32, nseg32, f32_numel, seg64, nseg64, i64_numel,
                          flags, "fa_multi_select", &g);
  if (rc) return rc;
  return select_form(g, mflags, mode, nchunks, model_us);
}

int fa_multi_select(int nranks, const int* counts, unsigned mflags, int* mode) {
  if (!mode) return set_err(FA_E_INVAL, "fa_multi_select: mode is NULL");
  // the nominal layout: one fp32 tensor of 2^24 elements
  const fa_seg seg{0, (int64_t)1 << 24};
  int nchunks = 0;
  return fa_multi_select_layout(nranks, counts, &seg, 1, seg.numel, nullptr, 0, 0,
                                FA_PLAN_GAPS_ARE_PADDING, mflags, mode, &nchunks, nullptr);
}

int fa_multi_plan_create(fa_comm* comm, const fa_seg* seg32, int nseg32, int64_t f32_numel,
                         const fa_seg* seg64, int nseg64, int64_t i64_numel, const int* counts,
                         int nchunks, unsigned flags, unsigned mflags, fa_multi_plan** out) {
  if (!out) return set_err(FA_E_INVAL, "fa_multi_plan_create: out is NULL");
  *out = nullptr;
  if (!comm) return set_err(FA_E_INVAL, "fa_multi_plan_create: NULL comm");
  int mode = -1, best = 0;
  int rc = fa_multi_select_layout(comm->nranks, counts, seg32, nseg32, f32_numel, seg64, nseg64,
                                  i64_numel, flags, mflags, &mode, &best, nullptr);
  if (rc) return rc;
  if (nchunks == 0) nchunks = best;
  if (mode == FA_MODE_BLOCKED) nchunks = 1;
  return make_round(comm, mode, seg32, nseg32, f32_numel, seg64, nseg64, i64_numel, counts,
                    nchunks, FA_XCHG_REDUCE, flags, "fa_multi_plan_create",
                    (fa_round_plan**)out);
}

int fa_multi_plan_chunks(const fa_multi_plan* plan, int* nchunks) {
  if (!plan || !nchunks) return set_err(FA_E_INVAL, "fa_multi_plan_chunks: NULL argument");
  *nchunks = ((const fa_round_plan*)plan)->req_chunks;
  return FA_OK;
}

int fa_multi_plan_mode(const fa_multi_plan* plan, int* mode) {
  if (!plan || !mode) return set_err(FA_E_INVAL, "fa_multi_plan_mode: NULL argument");
  *mode = ((const fa_round_plan*)plan)->mode;
  return FA_OK;
}

int fa_multi_plan_destroy(fa_multi_plan* p) {
  free_round((fa_round_plan*)p);
  return FA_OK;
}

int fa_reduce_multi(fa_multi_plan* const* plans, int nlocal, const fa_shard_io* io, int root) {
  if (nlocal < 1 || !plans || !plans[0])
    return set_err(FA_E_INVAL, "fa_reduce_multi: bad arguments");
  return run_round((fa_round_plan* const*)plans, nlocal, io, root,
                   ((const fa_round_plan*)plans[0])->mode, "fa_reduce_multi");
}

// Stateless form (SURVEY.md §8 b's fa_mean_f32_multi): fp32 segments only,
// the default (exact) round; plans cached per (communicator, layout, counts).
int fa_mean_f32_multi(fa_comm* comm, const float* const* clients, const int* counts,
                      int64_t numel, float* out, const fa_seg* segs, int nseg, int root,
                      void* stream) {
  return fa_mean_f32_multi_ex(comm, clients, counts, numel, out, segs, nseg, root, 0u, stream);
}

int fa_mean_f32_multi_ex(fa_comm* comm, const float* const* clients, const int* counts,
                         int64_t numel, float* out, const fa_seg* segs, int nseg, int root,
                         unsigned mflags, void* stream) {
  if (!comm || !counts) return set_err(FA_E_INVAL, "fa_mean_f32_multi: NULL comm/counts");
  if (nseg < 0 || (nseg > 0 && !segs)) return set_err(FA_E_INVAL, "fa_mean_f32_multi: segs");
  std::string key((const char*)&comm, sizeof comm);
  key.append((const char*)&mflags, sizeof mflags);
  key.append((const char*)&numel, sizeof numel);
  key.append((const char*)counts, sizeof(int) * comm->nranks);
  if (nseg > 0) key.append((const char*)segs, sizeof(fa_seg) * nseg);
  fa_multi_plan* plan = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_multi_mu);
    auto it = g_multi.find(key);
    if (it != g_multi.end()) {
      plan = (fa_multi_plan*)it->second;
    } else {
      const int rc = fa_multi_plan_create(comm, segs, nseg, numel, nullptr, 0, 0, counts, 0,
                                          FA_PLAN_GAPS_ARE_PADDING, mflags, &plan);
      if (rc) return rc;
      g_multi[key] = (fa_round_plan*)plan;
    }
  }
  fa_shard_io io{};
  io.c32 = clients;
  io.out32 = out;
  io.stream = stream;
  return fa_reduce_multi(&plan, 1, &io, root);
}

// ============================================================== e2 ========
int fa_stripe_plan_create(fa_comm* comm, const fa_seg* seg32, int nseg32, int64_t f32_numel,
                          const fa_seg* seg64, int nseg64, int64_t i64_numel, const int* counts,
                          unsigned flags, fa_stripe_plan** out) {
  return fa_stripe_plan_create_ex(comm, seg32, nseg32, f32_numel, seg64, nseg64, i64_numel,
                                  counts, 0, flags, out);
}

int fa_stripe_plan_create_ex(fa_comm* comm, const fa_seg* seg32, int nseg32, int64_t f32_numel,
                             const fa_seg* seg64, int nseg64, int64_t i64_numel, const int* counts,
                             int nchunks, unsigned flags, fa_stripe_plan** out) {
  return make_round(comm, FA_MODE_STRIPED, seg32, nseg32, f32_numel, seg64, nseg64, i64_numel,
                    counts, nchunks, FA_XCHG_REDUCE, flags, "fa_stripe_plan_create",
                    (fa_round_plan**)out);
}

int fa_stripe_plan_destroy(fa_stripe_plan* p) {
  free_round((fa_round_plan*)p);
  return FA_OK;
}

int fa_reduce_striped(fa_stripe_plan* const* plans, int nlocal, const fa_shard_io* io,
                      int root) {
  return run_round((fa_round_plan* const*)plans, nlocal, io, root, FA_MODE_STRIPED,
                   "fa_reduce_striped");
}

// =========================================================== chained ======
int fa_chain_plan_create(fa_comm* comm, const fa_seg* seg32, int nseg32, int64_t f32_numel,
                         const fa_seg* seg64, int nseg64, int64_t i64_numel, const int* counts,
                         int nchunks, unsigned flags, fa_chain_plan** out) {
  return make_round(comm, FA_MODE_CHAINED, seg32, nseg32, f32_numel, seg64, nseg64, i64_numel,
                    counts, nchunks, FA_XCHG_REDUCE, flags, "fa_chain_plan_create",
                    (fa_round_plan**)out);
}

int fa_chain_plan_destroy(fa_chain_plan* p) {
  free_round((fa_round_plan*)p);
  return FA_OK;
}

int fa_reduce_chained(fa_chain_plan* const* plans, int nlocal, const fa_shard_io* io, int root) {
  return run_round((fa_round_plan* const*)plans, nlocal, io, root, FA_MODE_CHAINED,
                   "fa_reduce_chained");
}

// =========================================================== blocked ======
int fa_block_plan_create(fa_comm* comm, const fa_seg* seg32, int nseg32, int64_t f32_numel,
                         const fa_seg* seg64, int nseg64, int64_t i64_numel, const int* counts,
                         unsigned flags, fa_block_plan** out) {
  return make_round(comm, FA_MODE_BLOCKED, seg32, nseg32, f32_numel, seg64, nseg64, i64_numel,
                    counts, 1, FA_XCHG_REDUCE, flags, "fa_block_plan_create",
                    (fa_round_plan**)out);
}

int fa_block_plan_destroy(fa_block_plan* p) {
  free_round((fa_round_plan*)p);
  return FA_OK;
}

int fa_reduce_blocked(fa_block_plan* const* plans, int nlocal, const fa_shard_io* io, int root) {
  return run_round((fa_round_plan* const*)plans, nlocal, io, root, FA_MODE_BLOCKED,
                   "fa_reduce_blocked");
}

// ====================================================== host-only view =====
int fa_describe_round(int mode, int nranks, int rank, const int* counts, const fa_seg* seg32,
                      int nseg32, int64_t f32_numel, const fa_seg* seg64, int nseg64,
                      int64_t i64_numel, int nchunks, int exchange, unsigned flags, int root,
                      int weighted, fa_xfer* ops, int cap, int* nops) {
  if (!nops) return set_err(FA_E_INVAL, "fa_describe_round: nops is NULL");
  *nops = 0;
  if (mode != FA_MODE_SHARDED && mode != FA_MODE_STRIPED && mode != FA_MODE_CHAINED &&
      mode != FA_MODE_BLOCKED)
    return set_err(FA_E_INVAL, "fa_describe_round: mode %d", mode);
  if (nchunks == 0) nchunks = mode == FA_MODE_STRIPED ? kStripeChunks : 8;
  if (nchunks < 1 || nchunks > FA_COMM_MAX_CHUNKS)
    return set_err(FA_E_INVAL, "fa_describe_round: nchunks=%d", nchunks);
  if (exchange != FA_XCHG_REDUCE && exchange != FA_XCHG_RS_GATHER)
    return set_err(FA_E_INVAL, "fa_describe_round: exchange %d", exchange);
  if (root >= nranks) return set_err(FA_E_INVAL, "fa_describe_round: root=%d", root);
  fa_round_plan p;
  p.mode = mode;
  p.xchg = exchange;
  p.req_chunks = nchunks;
  int rc = make_geo(nranks, rank, counts, seg32, nseg32, f32_numel, seg64, nseg64, i64_numel,
                    flags, "fa_describe_round", &p.g);
  if (rc) return rc;
  std::vector<fa_tile_desc> vec, tails;
  std::vector<size_t> cut;
  std::vector<int64_t> tidx;
  if ((rc = build_round(&p, nchunks, &vec, &cut, &tails, &tidx))) return rc;
  const std::vector<fa_xfer>& s = schedule(&p, root, weighted != 0);
  *nops = (int)s.size();
  if (ops) {
    if (cap < (int)s.size())
      return set_err(FA_E_RANGE, "fa_describe_round: %d ops, capacity %d", (int)s.size(), cap);
    std::copy(s.begin(), s.end(), ops);
  }
  return FA_OK;
}


int fa_model_constants(double* link_gbps, double* hbm_gbps, double* group_us,
                       double* kernel_us) {
  const ModelConst& c = mc();
  if (link_gbps) *link_gbps = c.link_gbps;
  if (hbm_gbps) *hbm_gbps = c.hbm_gbps;
  if (group_us) *group_us = c.group_us;
  if (kernel_us) *kernel_us = c.kernel_us;
  return FA_OK;
}

int fa_round_model(int mode, int nranks, const int* counts, const fa_seg* seg32, int nseg32,
                   int64_t f32_numel, const fa_seg* seg64, int nseg64, int64_t i64_numel,
                   int nchunks, int exchange, unsigned flags, int root, int weighted,
                   fa_round_cost* out) {
  if (!out) return set_err(FA_E_INVAL, "fa_round_model: out is NULL");
  if (mode != FA_MODE_SHARDED && mode != FA_MODE_STRIPED && mode != FA_MODE_CHAINED &&
      mode != FA_MODE_BLOCKED)
    return set_err(FA_E_INVAL, "fa_round_model: mode %d", mode);
  if (nchunks == 0) nchunks = mode == FA_MODE_STRIPED ? kStripeChunks : 8;
  if (nchunks < 1 || nchunks > FA_COMM_MAX_CHUNKS)
    return set_err(FA_E_INVAL, "fa_round_model: nchunks=%d", nchunks);
  if (exchange != FA_XCHG_REDUCE && exchange != FA_XCHG_RS_GATHER)
    return set_err(FA_E_INVAL, "fa_round_model: exchange %d", exchange);
  if (root >= nranks) return set_err(FA_E_INVAL, "fa_round_model: root=%d", root);
  Geo g;
  int rc = make_geo(nranks, 0, counts, seg32, nseg32, f32_numel, seg64, nseg64, i64_numel, flags,
                    "fa_round_model", &g);
  if (rc) return rc;
  if (nranks == 1) {
    // one rank: every form is the plain reduction (make_round), one kernel
    // reading n_total buckets and writing one
    fa_round_cost c{};
    c.hbm_bytes_max = (double)(g.n_total + 1) * (4.0 * (double)f32_numel + 8.0 * (double)i64_numel);
    c.model_us = mc().kernel_us + us_hbm(c.hbm_bytes_max);
    c.steps = 1;
    *out = c;
    return FA_OK;
  }
  std::vector<std::vector<fa_xfer>> sch;
  int64_t V = 0;
  if ((rc = all_schedules(g, mode, nchunks, exchange, root, weighted != 0, &sch, &V))) return rc;
  return model_schedules(sch, g.n_total, V, out);
}

}  // extern "C"
