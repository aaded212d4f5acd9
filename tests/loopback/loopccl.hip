// loopccl.hip — TEST INFRASTRUCTURE ONLY: an in-process loopback of the RCCL
// subset libfedagg_comm uses, so the native multi-rank rounds (fedcomm.hip:
// chained, striped, sharded, both e1 exchanges) run with W = 2..8 ranks on
// ONE GPU.  RCCL itself refuses two ranks on one device ("Duplicate GPU
// detected"), and the test pool has one GPU per box.
//
// libfedagg_comm_loop.so is fedcomm.hip compiled unchanged and linked against
// this library instead of librccl; tests/loopback/loop_round.cpp drives it
// with one thread per rank (the product's one-process-per-GPU model:
// fa_comm_init_rank) or one thread for all ranks (fa_comm_init).  Nothing in
// the product links or loads it.
//
// Semantics (RCCL's, as far as the executor can observe them):
//   - a group's ops are issued together; within a group every send is posted
//     before any receive waits, so pairwise exchanges cannot deadlock;
//   - p2p: the k-th send r->p pairs with the k-th receive at p from r, and
//     the receiver gets the send buffer's contents at the sender's stream
//     position of that send.  Sends are buffered (the payload is copied to
//     scratch on the sender's stream, which then moves on) and receives wait
//     on the host for their send to be posted: RCCL's rendezvous also lets a
//     single thread post a send in one group and its receive in a later one
//     (fa_comm_init's model), which a host-blocking send could not.  The
//     deadlock-freedom of the schedules under RCCL's rules is checked by
//     tests/schedsim.py; this library checks the data they move;
//   - a collective is the comm's k-th collective on every rank; the last rank
//     to arrive runs it on its stream after every rank's stream position,
//     reading every input into scratch before writing any output (in-place
//     forms are safe), and every rank's stream then waits for it;
//   - sums are float32, rank order 0..W-1 (RCCL's order is unspecified: the
//     sharded e1 result is compared with a tolerance, as on hardware);
//   - a wait that does not complete in FA_LOOP_TIMEOUT_S (default 60) seconds
//     fails the call (ncclInternalError) instead of hanging the test.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

namespace {

enum CollKind { C_ALLREDUCE, C_REDUCE, C_REDUCE_SCATTER, C_ALLGATHER, C_GATHER, C_BCAST };

struct SendRec {
  void* stage;  // the payload, copied on the sender's stream
  size_t bytes;
  hipEvent_t ready;
};

struct CollRec {
  int kind = -1, dtype = -1, root = -1;
  size_t count = 0;
  int arrived = 0, left = 0;
  std::vector<const void*> sbuf;
  std::vector<void*> rbuf;
  std::vector<hipEvent_t> ready;
  hipEvent_t done = nullptr;
  bool complete = false;
  int err = 0;
};

struct Clique {
  int n = 0, refs = 0;
  std::mutex mu;
  std::condition_variable cv;
  std::map<std::pair<int, int>, std::deque<SendRec*>> sends;  // (from, to)
  std::map<uint64_t, CollRec*> colls;
  std::vector<hipEvent_t> events;  // released with the clique
  std::vector<void*> scratch;      // staging / collective scratch, freed with the clique
};

std::mutex g_mu;
std::map<std::string, Clique*> g_cliques;

int timeout_s() {
  const char* e = getenv("FA_LOOP_TIMEOUT_S");
  return e ? atoi(e) : 60;
}

size_t dsize(int dtype) {
  switch (dtype) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 0;
  }
}

// Scratch lives until the clique is destroyed (plain hipMalloc: no
// stream-ordered reuse to reason about across the ranks' streams).
void* new_scratch(Clique* q, size_t bytes) {
  void* p = nullptr;
  if (hipMalloc(&p, bytes + 256) != hipSuccess) return nullptr;
  q->scratch.push_back(p);
  return p;
}

hipEvent_t new_event(Clique* q) {
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
  q->events.push_back(e);
  return e;
}

__global__ void add_f32(float* acc, const float* x, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    acc[i] = acc[i] + x[i];
}

}  // namespace

struct ncclComm {
  Clique* q;
  int rank;
  uint64_t coll_seq = 0;
};

namespace {

struct Op {
  int kind;  // 0 send, 1 recv, 2 collective
  ncclComm* comm;
  int peer;
  const void* sbuf;
  void* rbuf;
  size_t count;
  int dtype;
  int coll;
  hipStream_t st;
};

thread_local int t_depth = 0;
thread_local std::vector<Op> t_ops;

#define HT(x)                                                                   \
  do {                                                                          \
    if ((x) != hipSuccess) {                                                    \
      fprintf(stderr, "loopccl: %s failed\n", #x);                              \
      return ncclUnhandledCudaError;                                            \
    }                                                                           \
  } while (0)

// Run a complete collective on stream st (caller holds q->mu).
ncclResult_t run_coll(Clique* q, CollRec* c, hipStream_t st) {
  const int n = q->n;
  for (int j = 0; j < n; ++j) HT(hipStreamWaitEvent(st, c->ready[j], 0));
  const size_t es = dsize(c->dtype);
  const size_t cnt = c->count;
  size_t tmp_elems = cnt;
  if (c->kind == C_REDUCE_SCATTER || c->kind == C_ALLGATHER || c->kind == C_GATHER)
    tmp_elems = cnt * n;
  void* tmp = new_scratch(q, tmp_elems * es);
  if (!tmp) return ncclUnhandledCudaError;
  auto cp = [&](void* d, const void* s, size_t bytes) {
    return hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, st);
  };
  switch (c->kind) {
    case C_ALLREDUCE:
    case C_REDUCE:
    case C_REDUCE_SCATTER: {
      if (c->dtype != ncclFloat32) return ncclInvalidArgument;
      HT(cp(tmp, c->sbuf[0], tmp_elems * es));
      for (int j = 1; j < n; ++j)
        hipLaunchKernelGGL(add_f32, dim3(1024), dim3(256), 0, st, (float*)tmp,
                           (const float*)c->sbuf[j], tmp_elems);
      HT(hipGetLastError());
      if (c->kind == C_ALLREDUCE)
        for (int j = 0; j < n; ++j) HT(cp(c->rbuf[j], tmp, cnt * es));
      else if (c->kind == C_REDUCE)
        HT(cp(c->rbuf[c->root], tmp, cnt * es));
      else
        for (int j = 0; j < n; ++j) HT(cp(c->rbuf[j], (char*)tmp + j * cnt * es, cnt * es));
      break;
    }
    case C_ALLGATHER:
    case C_GATHER:
      for (int j = 0; j < n; ++j) HT(cp((char*)tmp + j * cnt * es, c->sbuf[j], cnt * es));
      if (c->kind == C_ALLGATHER)
        for (int j = 0; j < n; ++j) HT(cp(c->rbuf[j], tmp, n * cnt * es));
      else
        HT(cp(c->rbuf[c->root], tmp, n * cnt * es));
      break;
    case C_BCAST:
      HT(cp(tmp, c->sbuf[c->root], cnt * es));
      for (int j = 0; j < n; ++j) HT(cp(c->rbuf[j], tmp, cnt * es));
      break;
    default: return ncclInvalidArgument;
  }
  c->done = new_event(q);
  HT(hipEventRecord(c->done, st));
  return ncclSuccess;
}

bool wait_for(std::unique_lock<std::mutex>& lk, Clique* q, const char* what, int rank,
              const std::function<bool()>& pred) {
  if (q->cv.wait_for(lk, std::chrono::seconds(timeout_s()), pred)) return true;
  fprintf(stderr, "loopccl: rank %d timed out waiting for %s\n", rank, what);
  return false;
}

ncclResult_t flush(std::vector<Op>& ops) {
  std::vector<std::pair<CollRec*, Op*>> my_colls;
  // 1. post every send
  for (Op& o : ops) {
    if (o.kind != 0) continue;
    Clique* q = o.comm->q;
    std::lock_guard<std::mutex> lk(q->mu);
    SendRec* s = new SendRec{nullptr, o.count * dsize(o.dtype), new_event(q)};
    s->stage = new_scratch(q, s->bytes);
    if (!s->stage) return ncclUnhandledCudaError;
    if (s->bytes)
      HT(hipMemcpyAsync(s->stage, o.sbuf, s->bytes, hipMemcpyDeviceToDevice, o.st));
    HT(hipEventRecord(s->ready, o.st));
    q->sends[{o.comm->rank, o.peer}].push_back(s);
    q->cv.notify_all();
  }
  // 2. arrive at every collective (the last arrival runs it)
  for (Op& o : ops) {
    if (o.kind != 2) continue;
    Clique* q = o.comm->q;
    std::lock_guard<std::mutex> lk(q->mu);
    const uint64_t seq = o.comm->coll_seq++;
    CollRec*& c = q->colls[seq];
    if (!c) {
      c = new CollRec();
      c->kind = o.coll;
      c->dtype = o.dtype;
      c->count = o.count;
      c->root = o.peer;
      c->sbuf.assign(q->n, nullptr);
      c->rbuf.assign(q->n, nullptr);
      c->ready.assign(q->n, nullptr);
    }
    if (c->kind != o.coll || c->dtype != o.dtype || c->count != o.count || c->root != o.peer) {
      fprintf(stderr, "loopccl: collective %llu mismatch at rank %d (kind %d/%d count %zu/%zu)\n",
              (unsigned long long)seq, o.comm->rank, c->kind, o.coll, c->count, o.count);
      return ncclInvalidUsage;
    }
    c->sbuf[o.comm->rank] = o.sbuf;
    c->rbuf[o.comm->rank] = o.rbuf;
    c->ready[o.comm->rank] = new_event(q);
    HT(hipEventRecord(c->ready[o.comm->rank], o.st));
    if (++c->arrived == q->n) {
      const ncclResult_t r = run_coll(q, c, o.st);
      if (r != ncclSuccess) c->err = r;
      c->complete = true;
      q->cv.notify_all();
    }
    my_colls.push_back({c, &o});
  }
  // 3. receives: pair with the k-th send from the peer
  for (Op& o : ops) {
    if (o.kind != 1) continue;
    Clique* q = o.comm->q;
    std::unique_lock<std::mutex> lk(q->mu);
    auto& dq = q->sends[{o.peer, o.comm->rank}];
    if (!wait_for(lk, q, "a send", o.comm->rank, [&] { return !dq.empty(); }))
      return ncclInternalError;
    SendRec* s = dq.front();
    dq.pop_front();
    const size_t bytes = o.count * dsize(o.dtype);
    if (s->bytes != bytes) {
      fprintf(stderr, "loopccl: rank %d receives %zu B from %d, which sends %zu B\n",
              o.comm->rank, bytes, o.peer, s->bytes);
      return ncclInvalidUsage;
    }
    HT(hipStreamWaitEvent(o.st, s->ready, 0));
    if (bytes) HT(hipMemcpyAsync(o.rbuf, s->stage, bytes, hipMemcpyDeviceToDevice, o.st));
    delete s;
  }
  // 4. every participant's stream waits for the collective
  for (auto& pc : my_colls) {
    CollRec* c = pc.first;
    Op& o = *pc.second;
    Clique* q = o.comm->q;
    std::unique_lock<std::mutex> lk(q->mu);
    if (!wait_for(lk, q, "the other ranks of a collective", o.comm->rank,
                  [&] { return c->complete; }))
      return ncclInternalError;
    if (c->err) return (ncclResult_t)c->err;
    HT(hipStreamWaitEvent(o.st, c->done, 0));
    if (++c->left == q->n) {
      for (auto it = q->colls.begin(); it != q->colls.end(); ++it)
        if (it->second == c) {
          q->colls.erase(it);
          break;
        }
      delete c;
    }
  }
  return ncclSuccess;
}

ncclResult_t submit(const Op& o) {
  if (!o.comm) return ncclInvalidArgument;
  if (dsize(o.dtype) == 0) return ncclInvalidArgument;
  t_ops.push_back(o);
  if (t_depth > 0) return ncclSuccess;
  std::vector<Op> ops;
  ops.swap(t_ops);
  return flush(ops);
}

Clique* join(const std::string& key, int n) {
  std::lock_guard<std::mutex> lk(g_mu);
  Clique*& q = g_cliques[key];
  if (!q) {
    q = new Clique();
    q->n = n;
  }
  q->refs++;
  return q;
}

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  static std::atomic<unsigned long long> ctr{0};
  memset(id, 0, sizeof *id);
  snprintf(id->internal, sizeof id->internal, "loopccl:%d:%llu", (int)getpid(), ctr++);
  return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
  if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  std::string key(id.internal, strnlen(id.internal, sizeof id.internal));
  Clique* q = join(key, nranks);
  if (q->n != nranks) return ncclInvalidUsage;
  *comm = new ncclComm{q, rank};
  return ncclSuccess;
}

ncclResult_t ncclCommInitAll(ncclComm_t* comms, int ndev, const int* devlist) {
  (void)devlist;  // every rank may sit on the same device: that is the point
  if (!comms || ndev < 1) return ncclInvalidArgument;
  ncclUniqueId id;
  ncclGetUniqueId(&id);
  std::string key(id.internal);
  for (int r = 0; r < ndev; ++r) comms[r] = new ncclComm{join(key, ndev), r};
  return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  if (!comm) return ncclSuccess;
  Clique* q = comm->q;
  delete comm;
  std::lock_guard<std::mutex> lk(g_mu);
  if (--q->refs == 0) {
    for (auto it = g_cliques.begin(); it != g_cliques.end(); ++it)
      if (it->second == q) {
        g_cliques.erase(it);
        break;
      }
    (void)hipDeviceSynchronize();
    for (hipEvent_t e : q->events) (void)hipEventDestroy(e);
    for (void* p : q->scratch) (void)hipFree(p);
    delete q;
  }
  return ncclSuccess;
}

ncclResult_t ncclCommCount(const ncclComm_t comm, int* count) {
  if (!comm || !count) return ncclInvalidArgument;
  *count = comm->q->n;
  return ncclSuccess;
}

ncclResult_t ncclCommUserRank(const ncclComm_t comm, int* rank) {
  if (!comm || !rank) return ncclInvalidArgument;
  *rank = comm->rank;
  return ncclSuccess;
}

const char* ncclGetErrorString(ncclResult_t r) {
  switch (r) {
    case ncclSuccess: return "no error (loopccl)";
    case ncclUnhandledCudaError: return "HIP call failed (loopccl)";
    case ncclInternalError: return "timed out / internal (loopccl)";
    case ncclInvalidArgument: return "invalid argument (loopccl)";
    case ncclInvalidUsage: return "invalid usage: unmatched or mismatched op (loopccl)";
    default: return "error (loopccl)";
  }
}

ncclResult_t ncclGroupStart() {
  ++t_depth;
  return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
  if (t_depth <= 0) return ncclInvalidUsage;
  if (--t_depth > 0) return ncclSuccess;
  std::vector<Op> ops;
  ops.swap(t_ops);
  const ncclResult_t r = flush(ops);
  // FA_LOOP_SERIAL=1: drain the device after every group (tells a stream-
  // ordering race in the caller from a data-flow error)
  static const bool serial = getenv("FA_LOOP_SERIAL") && atoi(getenv("FA_LOOP_SERIAL"));
  if (serial) (void)hipDeviceSynchronize();
  return r;
}

ncclResult_t ncclSend(const void* sendbuff, size_t count, ncclDataType_t dt, int peer,
                      ncclComm_t comm, hipStream_t st) {
  return submit(Op{0, comm, peer, sendbuff, nullptr, count, (int)dt, -1, st});
}

ncclResult_t ncclRecv(void* recvbuff, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm,
                      hipStream_t st) {
  return submit(Op{1, comm, peer, nullptr, recvbuff, count, (int)dt, -1, st});
}

ncclResult_t ncclAllReduce(const void* s, void* r, size_t count, ncclDataType_t dt, ncclRedOp_t op,
                           ncclComm_t comm, hipStream_t st) {
  if (op != ncclSum) return ncclInvalidArgument;
  return submit(Op{2, comm, -1, s, r, count, (int)dt, C_ALLREDUCE, st});
}

ncclResult_t ncclReduce(const void* s, void* r, size_t count, ncclDataType_t dt, ncclRedOp_t op,
                        int root, ncclComm_t comm, hipStream_t st) {
  if (op != ncclSum) return ncclInvalidArgument;
  return submit(Op{2, comm, root, s, r, count, (int)dt, C_REDUCE, st});
}

ncclResult_t ncclReduceScatter(const void* s, void* r, size_t recvcount, ncclDataType_t dt,
                               ncclRedOp_t op, ncclComm_t comm, hipStream_t st) {
  if (op != ncclSum) return ncclInvalidArgument;
  return submit(Op{2, comm, -1, s, r, recvcount, (int)dt, C_REDUCE_SCATTER, st});
}

ncclResult_t ncclAllGather(const void* s, void* r, size_t sendcount, ncclDataType_t dt,
                           ncclComm_t comm, hipStream_t st) {
  return submit(Op{2, comm, -1, s, r, sendcount, (int)dt, C_ALLGATHER, st});
}

ncclResult_t ncclGather(const void* s, void* r, size_t sendcount, ncclDataType_t dt, int root,
                        ncclComm_t comm, hipStream_t st) {
  return submit(Op{2, comm, root, s, r, sendcount, (int)dt, C_GATHER, st});
}

ncclResult_t ncclBroadcast(const void* s, void* r, size_t count, ncclDataType_t dt, int root,
                           ncclComm_t comm, hipStream_t st) {
  return submit(Op{2, comm, root, s, r, count, (int)dt, C_BCAST, st});
}

}  // extern "C"
