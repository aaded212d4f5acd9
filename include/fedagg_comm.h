/*
 * fedagg_comm.h — C ABI of libfedagg_comm.so: the multi-GPU form of the
 * server-side aggregation (SURVEY.md §8 b "fa_comm_init / fa_mean_f32_multi",
 * §8 e1 and e2), natively over RCCL (xGMI inside one node).
 *
 * Reference: the round loops aggregate every client of a round into one
 * global model (train_fedavg.py:138-149, train_feddct.py:34-56); when the
 * clients' states do not fit one GPU, or were trained on several, the client
 * slots are sharded across the GPUs of the node — rank r holds a contiguous
 * run of slots, in slot order.
 *
 * THE DEFAULT ENTRY IS EXACT (r05): fa_multi_plan_create / fa_reduce_multi
 * (and the stateless fa_mean_f32_multi) run a round whose result is
 * bit-identical to one GPU's fa_reduce over all slots, i.e. to the
 * reference's single-process stack(...).mean(0) (train_feddct.py:42-50):
 * r06, the exact form — blocked (only when every cascade block of 16 slots
 * lies on at most two ranks), chained or striped — and chunk count with the
 * lowest time in the cost model below (fa_round_model; fa_multi_select_layout
 * names the choice, host only; r05 chose blocked-else-chained by geometry).  The re-associated e1 round (partial sums + an RCCL sum,
 * fa_reduce_sharded below) is opt-in (FA_MULTI_REASSOCIATE, or its own
 * plan type): it is NOT within the north_star's 1 ULP — measured r04 on
 * 2 x 20 wrn16_8 clients (profiles/r04_final_bench_n2_gloo_rehearsal.json):
 * max 22,938 ULP (near-cancelling sums), ULP histogram 0: 7,072,061,
 * 1: 2,990,526, 2: 892,989, 3-4: 15,239, 5-8: 642, 9-16: 342, 17+: 355
 * elements; within the forward error bound 2N * 2^-24 * sum|x_i| / N.
 *
 * The e1 round (fa_reduce_sharded) is
 *
 *   1. per rank, the torch-order sum of its own clients for every fp32 key
 *      (fa_reduce with FA_F_SUM_ONLY, over a column chunk at a time);
 *   2. an RCCL sum of those partial buckets — ncclReduce to the server rank
 *      (root >= 0), or ncclAllReduce (root < 0: every rank gets the global
 *      state, e.g. to reload its own client slots) — chunk c on an internal
 *      communication stream while the kernel sums chunk c+1;
 *   3. /N_total (IEEE division) on the ranks that hold the result.
 *   int64 keys (num_batches_tracked) are all-gathered raw and reduced exactly
 *   over all N_total clients, so they match the single-GPU result bit for bit.
 *
 * With one rank every form is the single-GPU reduction (bit-identical).
 *
 * Process models:
 *   - one process per GPU (the product's): rank 0 calls fa_comm_unique_id,
 *     ships the 128 bytes to every rank (e.g. a torch.distributed broadcast),
 *     each rank calls fa_comm_init_rank on its current device;
 *   - one process driving several GPUs: fa_comm_init(ndev, devs, comms).
 *   fa_reduce_sharded takes an array of local shard plans (one per GPU this
 *   process drives: 1 in the per-process model) and groups the RCCL calls.
 *
 * Conventions as in fedagg.h: caller-owned device buffers (zero-copy), 0 or a
 * negative FA_E* code, message in fa_last_error(); work is stream-ordered on
 * the caller's stream (the internal communication stream joins it before
 * fa_reduce_sharded returns).  Scratch (one partial bucket + the int64 gather
 * rows) lives in the shard plan.
 */
#ifndef FEDAGG_COMM_H
#define FEDAGG_COMM_H

#include <stdint.h>

#include "fedagg.h"

#ifdef __cplusplus
extern "C" {
#endif

#define FA_E_COMM (-6)          /* RCCL error (message in fa_last_error)      */
#define FA_COMM_UID_BYTES 128   /* == sizeof(ncclUniqueId)                     */
#define FA_COMM_MAX_CHUNKS 64

typedef struct fa_comm fa_comm;
typedef struct fa_shard_plan fa_shard_plan;

/* 128 opaque bytes identifying a new communicator (call on one rank). */
int fa_comm_unique_id(unsigned char *id, int len);
/* One process per GPU: rank `rank` of `nranks`, on the CURRENT device. */
int fa_comm_init_rank(int nranks, int rank, const unsigned char *id, int len,
                      fa_comm **out);
/* One process driving ndev GPUs (devs[i] becomes rank i): comms[ndev]. */
int fa_comm_init(int ndev, const int *devs, fa_comm **comms);
int fa_comm_destroy(fa_comm *comm);
int fa_comm_info(const fa_comm *comm, int *nranks, int *rank, int *device);
/* Captured rounds (default OFF; measured r03: a replay still costs ~9 µs of
 * host time per graph node on ROCm 7.0, and the replay loses the schedule's
 * two-stream overlap — faster for the blocked and striped rounds on one rank,
 * slower for the sharded and chained ones): in the
 * one-process-per-GPU model each
 * round's whole schedule — RCCL groups, kernels, stream joins — is captured
 * into a HIP graph the first time a plan runs with a given (root, weights,
 * buffer pointers) and replayed by one graph launch on the caller's stream
 * afterwards (up to 4 such graphs per plan, most recently used kept).  Off
 * (default): every round re-issues its schedule from the host.  Rounds whose kernels
 * cannot be captured (a rank holding more than FA_INLINE_CLIENTS slots) or
 * whose capture the runtime refuses run uncaptured either way. */
int fa_comm_set_graphs(fa_comm *comm, int enable);
/* Round profiles (r06; default OFF): with profiling on, every round a plan of
 * this communicator runs records event pairs around each of its RCCL groups
 * (on the communication stream) and each of its kernels (on the stream it
 * runs on), and around the whole round on the caller's stream (rounds are
 * then never replayed from graphs).  fa_round_plan_profile reads the last
 * profiled round of any plan of this library (an fa_multi_plan,
 * fa_chain_plan, fa_stripe_plan, fa_block_plan or fa_shard_plan; it waits for
 * the round): the sum of the groups' durations, of the kernels' on each
 * stream, the round's wall time on the caller's stream, and the counts — so
 * a multi-GPU run shows how much of a round is exchange, how much compute,
 * and how much of the two overlapped.  A one-rank plan (the plain reduction)
 * has no profile. */
typedef struct fa_round_profile {
  double exchange_us;         /* sum over the round's groups (communication stream) */
  double comm_kernel_us;      /* kernels on the communication stream            */
  double compute_kernel_us;   /* kernels on the caller's stream                 */
  double wall_us;             /* the whole round on the caller's stream         */
  int32_t groups;
  int32_t kernels;
} fa_round_profile;
int fa_comm_set_profile(fa_comm *comm, int enable);
int fa_round_plan_profile(const void *plan, fa_round_profile *out);

/* Shard plan of one rank for a bucket layout (as fa_plan_create; the layout
 * must be built with FA_PLAN_GAPS_ARE_PADDING: chunk exchanges span the
 * padding between tensors).  counts[r] = client slots held by rank r (all
 * ranks pass the same array); nchunks = column chunks of the exchange
 * (0 = 8).  Created on the comm's device. */
int fa_shard_plan_create(fa_comm *comm, const fa_seg *seg32, int nseg32,
                         int64_t f32_numel, const fa_seg *seg64, int nseg64,
                         int64_t i64_numel, const int *counts, int nchunks,
                         unsigned flags, fa_shard_plan **out);
int fa_shard_plan_destroy(fa_shard_plan *plan);

/* Per local GPU arguments of one round. */
typedef struct fa_shard_io {
  const float *const *c32;      /* this rank's counts[rank] fp32 buckets      */
  const int64_t *const *c64;    /* ... int64 buckets (NULL if no int64 keys)  */
  const float *weights;         /* NULL: mean; else per local client fp32 w   */
  float *out32;                 /* result (root / every rank); NULL elsewhere */
  int64_t *out64;
  void *stream;                 /* hipStream_t of the caller                  */
} fa_shard_io;

/* One e1 round across the ranks (re-associated: see the top of this file;
 * the default entry is fa_reduce_multi).  plans[d] / io[d]: the d-th GPU this process
 * drives (nlocal = 1 in the one-process-per-GPU model).  root >= 0: the
 * global state lands on rank `root` only (the north_star's final reduce);
 * root < 0: on every rank (all-reduce).  Weighted: fp32 keys = sum over all
 * clients of fp32(x_i * w_i) (no division); int64 keys always take the
 * mean-and-truncate path. */
int fa_reduce_sharded(fa_shard_plan *const *plans, int nlocal,
                      const fa_shard_io *io, int root);

/* ---- the default multi-GPU round (r05; chosen by a cost model since r06) ---
 * The default entry runs the EXACT form (blocked, chained or striped — all
 * bit-identical to one GPU) with the lowest modelled time (fa_round_model
 * below), and its chunk count; the blocked form only where its precondition
 * holds (every cascade block of 2^lp slots, 16 below 65,536 slots, on at
 * most two of the ranks holding slots).  FA_MODE_SHARDED (e1) only with
 * FA_MULTI_REASSOCIATE.
 * fa_multi_select_layout (host only, no communicator): that choice for a
 * layout — *mode, *nchunks (the candidates: chained 4/8/16/32, striped
 * 1/2/4/8, blocked 1) and the winner's modelled time in microseconds
 * (model_us may be NULL).  The model's root: every rank with
 * FA_MULTI_ROOT_ALL, else the last rank holding slots (the rounds may still
 * be run with any root: the flag only steers the choice).
 * fa_multi_select: the same for a nominal layout (one fp32 tensor of 2^24
 * elements, no int64 keys), from the counts alone.
 * fa_multi_plan_create builds the chosen form's plan (nchunks 0: the chosen
 * count; else the given count for whatever form is chosen); fa_reduce_multi
 * runs it (io / root as fa_reduce_sharded; weighted rounds: fp32 keys = sum
 * over all clients of fp32(x_i * w_i) in the torch order, also exact).
 * fa_multi_plan_mode reports the form, fa_multi_plan_chunks the count.
 * r05 chose by geometry alone (blocked if allowed, else chained). */
#define FA_MULTI_EXACT 0u          /* default: the fastest exact form            */
#define FA_MULTI_REASSOCIATE 1u    /* opt-in: e1, NOT bit-identical (above)      */
#define FA_MULTI_ROOT_ALL 2u       /* cost-model hint: results on every rank     */
typedef struct fa_multi_plan fa_multi_plan;
int fa_multi_select(int nranks, const int *counts, unsigned mflags, int *mode);
int fa_multi_select_layout(int nranks, const int *counts, const fa_seg *seg32,
                           int nseg32, int64_t f32_numel, const fa_seg *seg64,
                           int nseg64, int64_t i64_numel, unsigned flags,
                           unsigned mflags, int *mode, int *nchunks,
                           double *model_us);
int fa_multi_plan_chunks(const fa_multi_plan *plan, int *nchunks);
int fa_multi_plan_create(fa_comm *comm, const fa_seg *seg32, int nseg32,
                         int64_t f32_numel, const fa_seg *seg64, int nseg64,
                         int64_t i64_numel, const int *counts, int nchunks,
                         unsigned flags, unsigned mflags, fa_multi_plan **out);
int fa_multi_plan_mode(const fa_multi_plan *plan, int *mode);
int fa_multi_plan_destroy(fa_multi_plan *plan);
int fa_reduce_multi(fa_multi_plan *const *plans, int nlocal,
                    const fa_shard_io *io, int root);

/* Stateless fp32 form of the default round (SURVEY.md §8 b's
 * fa_mean_f32_multi): `clients` = this rank's counts[rank] buckets of numel
 * floats laid out by segs (as fa_mean_f32; gaps are treated as padding);
 * out = the mean over all ranks' clients on `root` (root < 0: every rank),
 * bit-identical to fa_mean_f32 over all clients on one GPU (r05; r01-r04 this
 * entry ran e1).  _ex takes FA_MULTI_* flags (FA_MULTI_REASSOCIATE: e1).  The
 * plan is cached per (comm, flags, layout, counts) and released with the
 * communicator (fa_comm_destroy). */
int fa_mean_f32_multi(fa_comm *comm, const float *const *clients,
                      const int *counts, int64_t numel, float *out,
                      const fa_seg *segs, int nseg, int root, void *stream);
int fa_mean_f32_multi_ex(fa_comm *comm, const float *const *clients,
                         const int *counts, int64_t numel, float *out,
                         const fa_seg *segs, int nseg, int root,
                         unsigned mflags, void *stream);

/* ---- exact mode: column stripes ----------------------
 * Rank r owns a contiguous column stripe [lo_r, lo_{r+1}) of the bucket (cut
 * before 256-B aligned vector tiles, equal shares of the elements), cut in
 * turn into nchunks column chunks.  A round (fa_reduce_striped), r06:
 *   1. per chunk c, ONE RCCL group with every peer: each rank sends every
 *      local client's values for chunk c of every other rank's stripe and
 *      receives every other rank's clients' values for chunk c of its own
 *      (n_local * (W-1)/W of a bucket out per rank over the round, spread
 *      over all W-1 links at once — r02-r05 exchanged with one partner per
 *      group, one link at a time);
 *   2. each rank reduces chunk c of its stripe over all n_total clients in
 *      the exact torch order (every tile keeps its column's order), on the
 *      caller's stream, while the group of chunk c+1 is in flight;
 *   3. the finished chunk c travels to the root (root >= 0) or to every rank
 *      in the group of chunk c+2 (beside that chunk's client exchange);
 *   int64 keys as in e1.  The result is bit-identical to one GPU's
 *   fa_reduce over all clients.  Weighted rounds (r06): each rank sends its
 *   clients' values pre-multiplied by their weights, rounded as the weighted
 *   kernel rounds the product (one staging pass over the columns it sends:
 *   a plan-owned buffer of n_local buckets, allocated by the first weighted
 *   round), and reduces its own clients with their weights and the received
 *   rows with weight 1 — the same bits as one GPU's weighted fa_reduce.
 * Same counts / io conventions as the sharded plan; the plan owns a receive
 * buffer of n_total stripe rows.  fa_stripe_plan_create: nchunks 0 (= 4);
 * _ex takes it (1..FA_COMM_MAX_CHUNKS, 0 = 4). */
typedef struct fa_stripe_plan fa_stripe_plan;
int fa_stripe_plan_create(fa_comm *comm, const fa_seg *seg32, int nseg32,
                          int64_t f32_numel, const fa_seg *seg64, int nseg64,
                          int64_t i64_numel, const int *counts, unsigned flags,
                          fa_stripe_plan **out);
int fa_stripe_plan_create_ex(fa_comm *comm, const fa_seg *seg32, int nseg32,
                             int64_t f32_numel, const fa_seg *seg64, int nseg64,
                             int64_t i64_numel, const int *counts, int nchunks,
                             unsigned flags, fa_stripe_plan **out);
int fa_stripe_plan_destroy(fa_stripe_plan *plan);
int fa_reduce_striped(fa_stripe_plan *const *plans, int nlocal,
                      const fa_shard_io *io, int root);

/* ---- e1 exchange options ---------------------------------------------------
 * FA_XCHG_REDUCE     : per chunk, one ncclReduce (root) / ncclAllReduce.
 * FA_XCHG_RS_GATHER  : per chunk, an in-place ncclReduceScatter (each rank
 *                      sums 1/W of the chunk) then ncclGather to the root /
 *                      ncclAllGather — every rank's links carry the exchange,
 *                      not one ring's; the chunk's last len % W floats take
 *                      the plain reduce.  Same arithmetic class as REDUCE
 *                      (re-associated across ranks). */
#define FA_XCHG_REDUCE 0
#define FA_XCHG_RS_GATHER 1
int fa_shard_plan_create_ex(fa_comm *comm, const fa_seg *seg32, int nseg32,
                            int64_t f32_numel, const fa_seg *seg64, int nseg64,
                            int64_t i64_numel, const int *counts, int nchunks,
                            int exchange, unsigned flags, fa_shard_plan **out);

/* ---- chained mode: client shards, exact order (fedagg.h fa_reduce_chain) ---
 * The client slots stay sharded as in e1 (rank r holds counts[r] slots, in
 * slot order), but instead of partial sums the cascade's accumulator STATE
 * travels: rank r continues rank r-1's state over its own clients, column
 * chunk by column chunk, and hands it to rank r+1 (ncclSend/ncclRecv of the
 * fa_chain_levels planes: one or two floats per element for N < 256), so
 * chunk c's hop overlaps chunk c+1's reduction.  The last rank holding
 * clients (the finisher) finishes the sum; the result then goes to `root`
 * (one send; none when root is the finisher) or to every rank (root < 0:
 * ncclBroadcast).  The scalar columns (ILP-4 tails, M==1 keys: a few hundred
 * floats) and the int64 keys are all-gathered raw and reduced in their own
 * orders by the result ranks (weighted: the fp32 rows are pre-multiplied).
 * The result is bit-identical to one GPU's fa_reduce over all clients, for
 * any counts.  Per hop: (1-2) * 4 B per vector element (4 planes for
 * N >= 256); no all-to-all of client state. */
typedef struct fa_chain_plan fa_chain_plan;
int fa_chain_plan_create(fa_comm *comm, const fa_seg *seg32, int nseg32,
                         int64_t f32_numel, const fa_seg *seg64, int nseg64,
                         int64_t i64_numel, const int *counts, int nchunks,
                         unsigned flags, fa_chain_plan **out);
int fa_chain_plan_destroy(fa_chain_plan *plan);
int fa_reduce_chained(fa_chain_plan *const *plans, int nlocal,
                      const fa_shard_io *io, int root);

/* ---- blocked mode: client shards, exact order, block sums to stripe owners -
 * torch's cascade sums the slots in blocks of 16 (level 0) and folds the
 * block sums in order (levels 1-3).  A block sum depends only on its own 16
 * rows, so every rank computes the block sums of the blocks it holds
 * entirely, independently; a block cut by a shard boundary needs the
 * level-0 partial of its first rank's rows (ONE plane) on the next rank,
 * which travels split into column stripes, each through the stripe's owner
 * (every link of a full xGMI mesh carries a share, not just r -> r+1).  The
 * block sums (and the remainder block's partial) then go to the column
 * stripe owners, which fold them in block order with torch's promotions
 * (fa_reduce's own arithmetic), divide, and send the result stripes to
 * `root` (or every rank).  Scalar columns and int64 keys as in the chained
 * mode.  Bit-identical to one GPU's fa_reduce over all clients; requires
 * every block's slots to lie on at most two ranks (fa_block_plan_create
 * returns FA_E_RANGE otherwise, e.g. for fewer than ~8 slots per rank: use
 * the chained round).  nchunks is unused (0). */
typedef struct fa_block_plan fa_block_plan;
int fa_block_plan_create(fa_comm *comm, const fa_seg *seg32, int nseg32,
                         int64_t f32_numel, const fa_seg *seg64, int nseg64,
                         int64_t i64_numel, const int *counts, unsigned flags,
                         fa_block_plan **out);
int fa_block_plan_destroy(fa_block_plan *plan);
int fa_reduce_blocked(fa_block_plan *const *plans, int nlocal,
                      const fa_shard_io *io, int root);

/* ---- schedules, host-only -------------------------------------------------
 * Every round above runs a schedule: a list of operations per rank, built on
 * the host from the layout, the counts and the rank.  fa_describe_round
 * returns rank `rank`'s list exactly as the executor issues it — no GPU, no
 * communicator — so the multi-rank schedules can be checked (and replayed)
 * on a CPU.  Ops with the same `step` are issued together: the exchanges of
 * a step form one RCCL group; a step's kernels follow its exchanges.
 * Offsets are bucket element offsets for CLIENT / OUT / PARTIAL / RECV /
 * STRIPE / STATE / FIN buffers, and element offsets into the stack for
 * STACK / GATHER (index 0: fp32 scalar columns, 1: int64 keys). */
#define FA_MODE_SHARDED 0
#define FA_MODE_STRIPED 1
#define FA_MODE_CHAINED 2
#define FA_MODE_BLOCKED 3

#define FA_X_SEND 1           /* ncclSend of src[offset, +count) to peer         */
#define FA_X_RECV 2           /* ncclRecv into dst[offset, +count) from peer     */
#define FA_X_REDUCE 3         /* ncclReduce to root `peer`                       */
#define FA_X_ALLREDUCE 4
#define FA_X_REDUCE_SCATTER 5 /* in place: rank r's sum at offset + r*count/W    */
#define FA_X_GATHER 6         /* every rank's count/W share to root `peer`       */
#define FA_X_ALLGATHER 7
#define FA_X_BCAST 8          /* from root `peer`                                */
#define FA_X_K_SUM 16         /* partial sum of the local clients, chunk `chunk`  */
#define FA_X_K_ZERO 17        /* zero dst[offset, +count) (a rank with no client) */
#define FA_X_K_DIV 18         /* dst[offset, +count) /= n_total                  */
#define FA_X_K_COPY 19
#define FA_X_K_STRIPE 20      /* this rank's stripe over all n_total clients     */
#define FA_X_K_CHAIN 21       /* fa_reduce_chain: rows row0..row0+nrows-1        */
#define FA_X_K_STACK 22       /* local clients' scalar columns / int64 keys      */
#define FA_X_K_TAILS 23       /* reduce the gathered rows into the result        */
#define FA_X_K_PART 24        /* blocked: level-0 partial of rows row0.. -> TAILP  */
#define FA_X_K_CONT 25        /* blocked: continue PIN over rows row0.. -> CONT    */
#define FA_X_K_BLOCK 26       /* blocked: block sum of local rows -> BSUM[dst_index] */
#define FA_X_K_FOLD 27        /* blocked: fold BLK[0..nrows) of this stripe       */
#define FA_X_K_SCALE 28       /* striped, weighted: WSTAGE[j] = fp32(client j * w_j)
                                 over [offset, +count), local rows 0..nrows-1    */

#define FA_B_NONE 0
#define FA_B_CLIENT 1         /* local client src_index's fp32 bucket            */
#define FA_B_OUT 2            /* the result buckets                              */
#define FA_B_PARTIAL 4        /* e1 partial sums                                 */
#define FA_B_RECV 5           /* e2 receive row of client slot `index`           */
#define FA_B_STRIPE 6         /* e2 this rank's reduced stripe                   */
#define FA_B_STATE 7          /* chained: cascade state plane `index`            */
#define FA_B_FIN 8            /* chained: the finisher's result (not a result rank) */
#define FA_B_STACK 9          /* raw scalar columns, this rank's rows            */
#define FA_B_GATHER 10        /* ... every rank's rows                           */
#define FA_B_PIN 11           /* blocked: incoming partial (plane 0; 1-3 stay 0) */
#define FA_B_TAILP 12         /* blocked: outgoing partial, plane `index`        */
#define FA_B_CONT 13          /* blocked: continuation result, plane `index`     */
#define FA_B_BSUM 14          /* blocked: local block sum `index`                */
#define FA_B_BLK 15           /* blocked: owner's stripe of block `index`        */
#define FA_B_RELAY 16         /* blocked: owner's relay of rank `index`'s partial */
#define FA_B_WSTAGE 17        /* striped, weighted: local client `index` pre-multiplied */

typedef struct fa_xfer {
  int32_t step;
  int32_t op;        /* FA_X_*                                                 */
  int32_t peer;      /* p2p: the other rank; rooted collectives: the root      */
  int32_t chunk;     /* kernels: chunk (chained/e1) or stripe (e2); else -1    */
  int32_t src, src_index; /* FA_B_* read, and its client / slot / plane index  */
  int32_t dst, dst_index; /* FA_B_* written                                    */
  int64_t offset;
  int64_t count;
  int32_t row0;      /* kernels: first client slot reduced                     */
  int32_t nrows;     /* kernels: clients reduced                               */
} fa_xfer;

/* mode FA_MODE_*; exchange FA_XCHG_* (e1 only); root as in the run call;
 * weighted != 0: the schedule of a weighted round.  ops == NULL: only *nops. */
int fa_describe_round(int mode, int nranks, int rank, const int *counts,
                      const fa_seg *seg32, int nseg32, int64_t f32_numel,
                      const fa_seg *seg64, int nseg64, int64_t i64_numel,
                      int nchunks, int exchange, unsigned flags, int root,
                      int weighted, fa_xfer *ops, int cap, int *nops);

/* ---- the round cost model (r06), host only ---------------------------------
 * Every rank's schedule (fa_describe_round) timed by a discrete-event replay
 * of the executor's rules: per rank a communication stream and the caller's
 * (compute) stream; a step's exchanges are one group, posted on the
 * communication stream once the compute-stream work it reads is done, and
 * complete when every peer has posted the matching operations; kernels that
 * read exchanged data run on the stream the executor puts them on, after the
 * exchanges they read.  Costs:
 *   a group: FA_MODEL_GROUP_US + max(the largest byte count on any one link
 *            direction of this rank / FA_MODEL_LINK_GBPS,
 *            the bytes its DMA moves in and out of HBM / FA_MODEL_HBM_GBPS),
 *            from the moment the last of its peers posted;
 *   a kernel: FA_MODEL_KERNEL_US + its HBM bytes / FA_MODEL_HBM_GBPS (reads
 *            and writes of the op's columns: rows read + planes written);
 *   collectives: ring traffic ((W-1)/W of the range per link direction, x2
 *            for an all-reduce, (W-1) x the range for an all-gather of
 *            per-rank rows; a broadcast the range), in and out of HBM.
 * The link rate is an assumption of this build until a multi-GPU node has
 * measured it (MI355X xGMI: 7 links per GPU, a full mesh of 8); the HBM rate
 * is this chip's measured float4 copy ceiling; the latencies
 * are round numbers for one RCCL group launch and one kernel launch's ramp
 * and drain.  bench.py --gpus N prints each form's modelled time beside its
 * measured time, so the first 8-GPU run checks the model.
 * fa_round_model: the round's modelled time (max over ranks, us), the
 * largest byte count on one link direction over the round (any rank, any
 * peer), the largest per-rank HBM byte count, and the busiest rank's group
 * count.  One rank: the plain reduction every form becomes (one kernel over
 * n_total + 1 buckets).  Errors as fa_describe_round. */
#define FA_MODEL_LINK_GBPS 64.0    /* GB/s per xGMI link direction (assumed)   */
#define FA_MODEL_HBM_GBPS 6500.0   /* GB/s: measured float4 copy ceiling       */
#define FA_MODEL_GROUP_US 15.0     /* one RCCL group: launch + completion      */
#define FA_MODEL_KERNEL_US 3.0     /* one kernel: launch gap + ramp / drain    */
/* The constants in effect: the defaults above unless the process
 * environment held a positive FA_MODEL_LINK_GBPS / FA_MODEL_HBM_GBPS (a
 * non-negative FA_MODEL_GROUP_US / FA_MODEL_KERNEL_US) when the model first
 * ran — read once per process — so rates measured on a multi-GPU node
 * re-rank the forms fa_multi_select_layout / fa_multi_plan_create pick
 * without a rebuild.  NULL outputs are skipped; always FA_OK. */
int fa_model_constants(double *link_gbps, double *hbm_gbps, double *group_us,
                       double *kernel_us);
typedef struct fa_round_cost {
  double model_us;
  double link_bytes_max;
  double hbm_bytes_max;
  int32_t groups;
  int32_t steps;
} fa_round_cost;
int fa_round_model(int mode, int nranks, const int *counts, const fa_seg *seg32,
                   int nseg32, int64_t f32_numel, const fa_seg *seg64, int nseg64,
                   int64_t i64_numel, int nchunks, int exchange, unsigned flags,
                   int root, int weighted, fa_round_cost *out);

#ifdef __cplusplus
}
#endif
#endif /* FEDAGG_COMM_H */
