/*
 * fedagg.h — C ABI of libfedagg.so, the MI355X (gfx950) server-side
 * parameter-aggregation engine.
 *
 * Drop-in boundary.  The reference has no native plugin/FFI API: its hot path
 * is the Python function
 *
 *     server_aggregate(global_model, client_models)
 *         train_fedavg.py:138-149  ==  train_fedprox.py:143-154
 *     server_aggregate(g_main, g_proxy, mains, proxies)
 *         train_feddct.py:34-56    ==  train_splitfed.py:34-56
 *
 * whose arithmetic is, per state_dict key k (train_fedavg.py:145-146),
 *
 *     torch.stack([client_models[i].state_dict()[k].float() for i], 0).mean(0)
 *
 * followed by load_state_dict into the global model (:147) and a broadcast of
 * the global state back into every client (:148-149).  The Python shim
 * feddct_amd.aggregate.server_aggregate keeps those signatures and side
 * effects and binds this ABI through ctypes; every entry
 * point below replaces one piece of that expression:
 *
 *   fa_reduce            stack(...).mean(0) for every key at once, over flat
 *                        per-client buckets (all fp32 keys + all int64 keys),
 *                        optionally followed by the :148-149 broadcast.
 *   fa_mean_f32          the same for fp32 keys only, stateless form.
 *   fa_weighted_f32      client-size-weighted extension.
 *   fa_mean_i64_trunc    int64 keys: .float() -> mean -> copy_ into int64
 *                        (truncation toward zero), train_fedavg.py:146-147.
 *
 * Summation order.  Results are bit-identical to torch's CPU
 * stack(...).mean(0) (ATen SumKernel cascade_sum, single-thread order; see
 * DESIGN.md §2): columns of a tensor with numel M are summed over the N
 * clients by the 4-level cascade (block 16) for the first (M/32)*32 columns
 * (M>=8) or (M/4)*4 columns (2<=M<8), by the ILP-4 interleaved order for the
 * remaining tail columns, and by the 8-lane inner order when M==1; the sum
 * starts from +0 and is divided by N with IEEE true division.
 *
 * Conventions
 *   - All buffers are caller-owned DEVICE pointers (PyTorch-ROCm tensors via
 *     data_ptr(), zero-copy).  The library never allocates or frees caller
 *     memory; plans own a small device-resident tile table.
 *   - Offsets and counts are in ELEMENTS of the bucket's dtype.
 *   - Return 0 on success or a negative FA_E* code; fa_last_error() returns a
 *     thread-local message for the last failure on the calling thread.
 *   - Calls are stream-ordered on the caller's stream (hipStream_t passed as
 *     void*, 0 = null stream) and never synchronise; reentrant.
 */
#ifndef FEDAGG_H
#define FEDAGG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FA_OK 0
#define FA_E_INVAL (-1)   /* bad argument (null pointer, n<1, overlap ...)   */
#define FA_E_RANGE (-2)   /* n exceeds FA_MAX_CLIENTS, size overflow          */
#define FA_E_ALIGN (-3)   /* a vectorised bucket pointer is not 16-B aligned */
#define FA_E_HIP (-4)     /* HIP runtime error (message in fa_last_error)     */
#define FA_E_NOMEM (-5)

/* Max clients per call (2^16: the cascade's four levels, promotions after
 * 16, 256 and 4096 rows, all exercised; 65,536 wrn16_8 clients would need
 * 2.9 TB, so one GPU's HBM, not this limit, bounds N).  Up to
 * FA_INLINE_CLIENTS the client pointer tables travel in the kernel
 * arguments; above, in a stream-ordered device table. */
#define FA_MAX_CLIENTS 65536
#define FA_INLINE_CLIENTS 128

/* fa_reduce flags */
#define FA_F_BCAST 1u    /* also write the result into every client bucket:
                            the plan's tiles (a second launch); a plan whose
                            segments cover the whole bucket up to padding
                            (FA_PLAN_GAPS_ARE_PADDING, no gap of >= 64 fp32 /
                            >= 1 int64 elements) copies [0, f32_numel) and
                            [0, i64_numel) flat instead                    */
#define FA_F_SUM_ONLY 2u /* fp32 keys: write the ordered sum, skip the /N   */
#define FA_F_BCAST_ONLY 4u /* no reduction: out32 / out64 (the global state)
                              written into every client bucket, as
                              FA_F_BCAST's launch (weights ignored)       */

/* Plan-build flags */
#define FA_PLAN_GAPS_ARE_PADDING 1u /* bytes between segments may be written
                                       (vector runs span them); with full
                                       coverage also FA_F_BCAST's flat copy */
#define FA_PLAN_TUNE_BATCH8 4u     /* force 8 clients per load batch          */
#define FA_PLAN_TUNE_BATCH16 8u    /* force 16 clients per load batch         */
#define FA_PLAN_TUNE_NO_BALANCE 0x10000000u /* launch the plain tile table with
                                               the default batch only (by
                                               default the launch shape follows
                                               the round count)    */
/* Every other bit is refused (FA_E_INVAL) since r05: the r01-r04 tuning
 * flags (cache policies, XCD / wave-contiguous tile orders, persistent grids,
 * occupancy caps, issue-all batches, fused / per-tile / r03 broadcasts,
 * packed-tile widths, ...) were measured, dropped and removed from the
 * library, and a caller still passing one gets an error, not a silently
 * different kernel. */
#define FA_PLAN_FLAGS_KNOWN \
  (FA_PLAN_GAPS_ARE_PADDING | FA_PLAN_TUNE_BATCH8 | FA_PLAN_TUNE_BATCH16 | FA_PLAN_TUNE_NO_BALANCE)

/* One tensor (state_dict key) inside a flat bucket: [offset, offset+numel). */
typedef struct fa_seg {
  int64_t offset;
  int64_t numel;
} fa_seg;

typedef struct fa_plan fa_plan; /* opaque: layout -> device tile table */

typedef struct fa_plan_info {
  int64_t f32_numel;      /* bucket length covered by the plan             */
  int64_t i64_numel;
  int32_t ntiles;         /* total work tiles (one workgroup each)          */
  int32_t ntiles_cascade; /* vectorised cascade tiles                       */
  int32_t ntiles_tail;    /* ILP-4 tail / M==1 / int64 tiles                */
  int32_t tile_elems;     /* fp32 elements per cascade tile                 */
  int64_t cascade_elems;  /* elements summed by the vectorised cascade      */
  int64_t tail_elems;     /* elements summed in the scalar orders           */
} fa_plan_info;

const char *fa_version(void);
const char *fa_last_error(void);

/* Build a plan for a bucket layout.  seg32 / seg64 describe the fp32 and
 * int64 keys (either may be empty).  tile_elems: fp32 elements per
 * vectorised tile (0 = default).  Allocates + uploads the tile table (sync). */
int fa_plan_create(const fa_seg *seg32, int nseg32, int64_t f32_numel,
                   const fa_seg *seg64, int nseg64, int64_t i64_numel,
                   int tile_elems, unsigned flags, fa_plan **out);
int fa_plan_destroy(fa_plan *plan);

/* Host-only tile table of a layout (no device, no allocation): for tests and
 * inspection.  kind: 0 fp32 cascade (16-B vectors), 1 fp32 cascade (scalar),
 * 2 fp32 ILP-4 tail, 3 fp32 M==1, 4/5/6 int64 cascade/ILP-4/M==1.  With
 * tiles==NULL only info is filled. */
typedef struct fa_tile_desc {
  int64_t start;
  int32_t count;
  int32_t kind;
} fa_tile_desc;
int fa_plan_build_host(const fa_seg *seg32, int nseg32, int64_t f32_numel,
                       const fa_seg *seg64, int nseg64, int64_t i64_numel,
                       int tile_elems, unsigned flags, fa_tile_desc *tiles,
                       int cap, fa_plan_info *info);
int fa_plan_get_info(const fa_plan *plan, fa_plan_info *info);

/* A plan over an explicit subset of a layout's tiles (as returned by
 * fa_plan_build_host): the unit of column-striped work — a GPU's stripe in the
 * exact multi-GPU mode, a chunk of the host-ingress pipeline.  Every tile keeps
 * the order its column needs, so any tile subset reduces bit-exactly. */
int fa_plan_create_from_tiles(const fa_tile_desc *tiles, int ntiles,
                              int64_t f32_numel, int64_t i64_numel,
                              int tile_elems, unsigned flags, fa_plan **out);

/* ---- launch shape by round count (r03) -------------------------------------
 * One workgroup per tile: T tiles over `slots` resident workgroups run
 * ceil(T / slots) rounds, and while a launch is one or two rounds long a
 * part-filled round costs nearly a whole one.  A plain fa_reduce call of
 * N >= 16 clients therefore (a) runs a table whose vector tiles are re-cut
 * to fill the round when its plain table part-fills ONE round of the
 * 16-client kernel (below 97 %), (b) runs the 8-client kernel when that
 * turns two rounds of the 16-client kernel into one, (c) runs the plain
 * table otherwise (re-cutting a longer launch measured slower).  N < 16
 * always runs plain.  Slot counts are queried from the runtime.  Any cut
 * reduces bit-identically: the order is per column.
 * fa_plan_balance_host: the re-cut of (a) on the host — `vec` are vector
 * tiles (kind 0, at most tile_elems each), `nscalar` the packed scalar tiles
 * that lead the launch; writes the new vector tiles to `out` (cap entries)
 * and returns their count, 0 when the plain cut is kept (the round is
 * >= 97 % full or the launch needs more than one round), < 0 on error.
 * fa_plan_launch_shape: the tiles and resident-workgroup slots a plain
 * fa_reduce call with n clients (weighted or not) launches with.
 * fa_plan_launch_form: the kernel that call runs — its vector tile width
 * (floats), clients per load batch, and whether its full tiles take the
 * client loop (pipe = 1: the next client's loads before the current
 * client's adds; 2: the same loop reading the device pointer
 * table, unweighted calls of 256 clients and more, r06) or the batches (0).
 * Torch-GPU-order plans report zeros. */
int fa_plan_balance_host(const fa_tile_desc *vec, int nvec, int tile_elems,
                         int nscalar, int slots, fa_tile_desc *out, int cap);
int fa_plan_launch_shape(const fa_plan *plan, int n, int weighted, int *ntiles,
                         int *slots);
int fa_plan_launch_form(const fa_plan *plan, int n, int weighted, int *tile_elems,
                        int *batch, int *pipe);

/* ---- summation order ------------------------------------------------------
 * FA_ORDER_TORCH_CPU (every plan's default): torch's CPU stack(...).mean(0),
 *   the order above — the reference's BASELINE config 1 and the
 *   device-independent definition.
 * FA_ORDER_TORCH_GPU (opt-in): torch-ROCm's own GPU stack(...).mean(0)
 *   (ATen/native/hip/Reduce.cuh + MeanOps as built into this torch): what the
 *   reference's original runs computed with their models on the GPU
 *   (train_fedavg.py:244-250).  Per tensor of M elements: the N rows split
 *   S ways, 4 round-robin accumulators, block_y tree, times the factor
 *   float(M)/float(N*M); M == 1 keys: lane split + the intra-wave shuffle
 *   tree.  The cut depends on N, so the plan is made for one client count;
 *   unweighted only.  fa_torch_gpu_config() says whether (N, M) is inside
 *   the restated configurations (no cross-block split: ceil(N/S) < 256,
 *   S <= 16; M == 1 needs N < 128) and gives S. */
#define FA_ORDER_TORCH_CPU 0
#define FA_ORDER_TORCH_GPU 1
int fa_torch_gpu_config(int n, int64_t m, int *stride);
int fa_plan_create_order(const fa_seg *seg32, int nseg32, int64_t f32_numel,
                         const fa_seg *seg64, int nseg64, int64_t i64_numel,
                         int n, int order, unsigned flags, fa_plan **out);

/* The hot path: every key of N client buckets -> global bucket, one launch
 * (FA_F_BCAST: plus one broadcast launch — over the same tiles, or the flat
 * bucket copy when the plan covers the whole bucket, see FA_F_BCAST).
 *   c32[i] / c64[i]  : client i's fp32 / int64 bucket (slot order 0..n-1)
 *   weights          : NULL -> mean (sum / n);  else fp32 w[i], result =
 *                      ordered sum of fp32(x_i * w_i) (no division)
 *   out32 / out64    : global buckets (may alias a client bucket)
 *   flags            : FA_F_BCAST | FA_F_SUM_ONLY, or FA_F_BCAST_ONLY
 * int64 keys always take the mean + truncation path (weights ignored). */
int fa_reduce(const fa_plan *plan, const float *const *c32,
              const int64_t *const *c64, int n, const float *weights,
              float *out32, int64_t *out64, unsigned flags, void *stream);

/* fa_reduce with a caller-owned device pointer table: above
 * FA_INLINE_CLIENTS clients the client pointers (and weights) travel in a
 * device table; fa_reduce takes it from a library pool and uploads it with a
 * host memcpy, fa_reduce_tab writes it into `table` (fa_table_bytes(n)
 * bytes of device memory, 8-B aligned) with kernels launched on `stream` —
 * no allocation and no host copy, so the call can be captured into a HIP
 * graph (hipStreamBeginCapture) and replayed.  `table` must stay allocated
 * and untouched while any launch or graph replay that uses it can run.
 * table may be NULL when n <= FA_INLINE_CLIENTS. */
size_t fa_table_bytes(int n);
int fa_reduce_tab(const fa_plan *plan, const float *const *c32,
                  const int64_t *const *c64, int n, const float *weights,
                  void *table, float *out32, int64_t *out64, unsigned flags,
                  void *stream);

/* ---- chained segments: client shards reduced in the exact order ----------
 * The cascade walks the N clients in slot order with four
 * level accumulators; its state after rows 0..k-1 is those accumulators.
 * fa_reduce_chain reduces rows row0..row0+n-1 of an n_total-row reduction:
 * it starts from state_in (the state after rows 0..row0-1) and either writes
 * the state after its last row to state_out, or — for the last segment —
 * finishes into out32 (sum, then /n_total unless weighted or FA_F_SUM_ONLY).
 * Segments chained in slot order reproduce fa_reduce over all n_total
 * clients bit for bit, whatever the cut points (the state-carrying exact
 * form of the client-sharded multi-GPU round, fedagg_comm.h).
 *   state planes : level l lives at state + l*plane (element e at [e]);
 *                  only the levels fa_chain_levels() reports are read or
 *                  written — the others are +0 at that point of the order.
 *                  state_in may equal state_out (in place).
 *   plan         : vector (cascade) tiles only; the ILP-4 tail, M==1 and
 *                  int64 columns of a layout are reduced by fa_reduce over
 *                  all clients' raw values (they are a few hundred bytes).
 * Equal weights as in fa_reduce (per local client, fp32). */
typedef struct fa_chain {
  int row0;              /* slot index of c32[0] in the whole reduction      */
  int n_total;           /* clients in the whole reduction                   */
  const float *state_in; /* state after rows 0..row0-1 (NULL when row0 == 0) */
  float *state_out;      /* NULL: this is the last segment, finish to out32  */
  int64_t plane;         /* floats per state plane (>= the plan's f32_numel) */
} fa_chain;
/* Bit l set: state plane l may be nonzero after `rows` of n_total rows. */
unsigned fa_chain_levels(int rows, int n_total);
int fa_reduce_chain(const fa_plan *plan, const float *const *c32, int n,
                    const float *weights, const fa_chain *chain, float *out32,
                    unsigned flags, void *stream);

/* Stateless fp32 mean over segments (plan cached internally by layout). */
int fa_mean_f32(const float *const *clients, int n, int64_t numel, float *out,
                const fa_seg *segs, int nseg, void *stream);
/* Stateless weighted sum: out = sum_i fp32(x_i * w_i) in torch order. */
int fa_weighted_f32(const float *const *clients, const float *w, int n,
                    int64_t numel, float *out, const fa_seg *segs, int nseg,
                    void *stream);
/* int64 keys, each segment its own tensor; numel elements total. */
int fa_mean_i64_trunc(const int64_t *const *clients, int n, int64_t numel,
                      int64_t *out, const fa_seg *segs, int nseg,
                      void *stream);

/* Elementwise out[j] = x[j] / d (IEEE true division), fp32; and the int64
 * finish of a cross-GPU partial sum: out64[j] = trunc(x[j] / d). */
int fa_div_f32(const float *x, float d, float *out, int64_t numel,
               void *stream);
int fa_div_trunc_i64(const float *x, float d, int64_t *out, int64_t numel,
                     void *stream);
/* Copy a bucket into n destinations (the standalone broadcast). */
int fa_broadcast_f32(const float *src, float *const *dst, int n,
                     int64_t numel, void *stream);

/* Synthetic client state (feddct_amd/synth.py restated bit-exactly). */
int fa_synth_fill_f32(float *dst, int64_t numel, int key_index, int client,
                      float mu, float sigma, int mode, void *stream);
int fa_synth_fill_i64(int64_t *dst, int64_t numel, int key_index, int client,
                      int mode, void *stream);

/* ---- FedProx proximal term (train_fedprox.py:113-116), SURVEY.md §8 f3 ----
 * sum_k ||a_k - b_k||_2 over the tensors (segments) of two flat buckets —
 * the client's and the global's parameters — and its gradient.  A norm plan
 * owns a small device scratch: use one plan from one stream at a time.
 * Segments start on 16-B boundaries (offset % 4 == 0, as every arena layout
 * places them) and all bucket pointers are 16-B aligned (else FA_E_ALIGN). */
typedef struct fa_norm_plan fa_norm_plan;
int fa_norm_plan_create(const fa_seg *segs, int nseg, int64_t numel,
                        fa_norm_plan **out);
int fa_norm_plan_destroy(fa_norm_plan *plan);
/* norms[k] = ||a_k - b_k||_2 (device, nseg floats); *total = sum_k norms[k] */
int fa_prox_norms(const fa_norm_plan *plan, const float *a, const float *b,
                  float *norms, float *total, void *stream);
/* grad_a[e] = (*gout) * alpha * (a[e]-b[e]) / norms[k]  (0 where norms[k]==0);
 * grad_b (nullable) = -grad_a.  Only elements inside segments are written. */
int fa_prox_grad(const fa_norm_plan *plan, const float *a, const float *b,
                 const float *norms, const float *gout, float alpha,
                 float *grad_a, float *grad_b, void *stream);
/* FA_PROX_ACCUMULATE: grad_a += (...), grad_b -= (...) instead (autograd's
 * in-place gradient accumulation, for .grad tensors that are bucket views). */
#define FA_PROX_ACCUMULATE 1u
/* ... for one side only (the other is overwritten): a training step whose
 * optimizer zeroed one model's .grad (set_to_none) and not the other's */
#define FA_PROX_ACCUMULATE_A 2u
#define FA_PROX_ACCUMULATE_B 4u
int fa_prox_grad_ex(const fa_norm_plan *plan, const float *a, const float *b,
                    const float *norms, const float *gout, float alpha,
                    float *grad_a, float *grad_b, unsigned flags, void *stream);

/* Streaming copy (bandwidth ceiling calibration for the roofline). */
int fa_copy_f32(const float *src, float *dst, int64_t numel, void *stream);
/* Tuning (experiments only; calling thread): the proximal-term gradient
 * stores' policy — 0 nt (default), 1 sc1.  Returns the previous one. */
int fa_tune_prox_store(int policy);
/* Tuning (experiments only; calling thread): chunks of 4096 floats per
 * workgroup of fa_prox_norms' partial-sum launch, 1..4 (0: the default, 1);
 * the result bits do not depend on it.  Returns the previous setting. */
int fa_tune_prox_cpw(int cpw);
/* Write-only streaming probe (write-bandwidth ceiling, r04): the round
 * broadcast's launch shape — one workgroup per (1024-float part, group of
 * <= 24 destinations), sc1 nt stores — storing non-zero hashed values (a function of the
 * element index and `seed`) into n <= 256 destination buckets of numel
 * floats (the last numel % 4 are not written); nothing is read. */
int fa_write_probe_f32(float *const *dst, int n, int64_t numel, unsigned seed,
                       void *stream);
/* Read-only streaming probe (read-bandwidth ceiling): grid > 0 — a
 * grid-stride loop, out[grid] partial sums (accumulated: zero out first);
 * grid == 0 — one 2048-float tile per workgroup, the reduce's own load shape,
 * nothing stored (out: >= 256 floats of scratch, never read; the last numel %
 * 4 floats are not read). */
int fa_read_probe_f32(const float *src, int64_t numel, float *out, int grid,
                      void *stream);

#ifdef __cplusplus
}
#endif
#endif /* FEDAGG_H */
