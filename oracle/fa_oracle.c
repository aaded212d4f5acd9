/*
 * ORACLE — test infrastructure only (never linked into or called by the
 * product path).  A second, independent CPU restatement of the reference's
 * aggregation arithmetic, in plain C, over the same flat buckets the HIP
 * engine uses:
 *
 *   torch.stack([client_models[i].state_dict()[k].float() for i], 0).mean(0)
 *       train_fedavg.py:145-146 (== train_fedprox.py:150-151,
 *       train_feddct.py:43-44/48-49)
 *   + load_state_dict copy_ (fp32 -> int64 truncation)  train_fedavg.py:147
 *
 * Order (ATen SumKernel cascade_sum, single-thread; see oracle/torch_order.py
 * for the numpy twin and DESIGN.md §2):
 *   M >= 8      columns < (M/32)*32 : multi_row_sum cascade, rest ILP-4
 *   2 <= M < 8  columns < (M/4)*4   : cascade, rest ILP-4
 *   M == 1      N < 8 : ILP-4 ; else 8-lane inner order
 * then out = (+0 + sum) / N, IEEE fp32, no FMA (build with -ffp-contract=off).
 *
 * Build: oracle/Makefile -> oracle/build/liboracle.so (ctypes:
 * oracle/c_oracle.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  int64_t offset;
  int64_t numel;
} oseg;

/* value of row i at element e: x = rows[i][e] (optionally * w[i]) */
typedef struct {
  const float *const *rows;
  const int64_t *const *irows;
  const float *w;
} src_t;

static inline float val(const src_t *s, int i, int64_t e) {
  if (s->irows) return (float)s->irows[i][e];
  float x = s->rows[i][e];
  return s->w ? x * s->w[i] : x;
}

static int ceil_log2(int64_t n) {
  int r = 0;
  if (n <= 1) return 0;
  uint64_t v = (uint64_t)(n - 1);
  while (v) { ++r; v >>= 1; }
  return r;
}

static int level_power(int64_t n) {
  int c = ceil_log2(n) / 4;
  return c > 4 ? c : 4;
}

/* ATen multi_row_sum, one column, rows first + k*stride (k < count) */
static float cascade(const src_t *s, int64_t e, int first, int stride, int count) {
  const int lp = level_power(count);
  const int64_t step = (int64_t)1 << lp, mask = step - 1;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  int64_t i = 0;
  while (i + step <= count) {
    for (int64_t j = 0; j < step; ++j, ++i) acc[0] += val(s, first + (int)i * stride, e);
    for (int j = 1; j < 4; ++j) {
      acc[j] += acc[j - 1];
      acc[j - 1] = 0.f;
      if (i & (mask << (j * lp))) break;
    }
  }
  for (; i < count; ++i) acc[0] += val(s, first + (int)i * stride, e);
  for (int j = 1; j < 4; ++j) acc[0] += acc[j];
  return acc[0];
}

/* ATen row_sum (ILP-4) */
static float ilp4(const src_t *s, int64_t e, int first, int stride, int count) {
  const int q = count / 4;
  float p[4];
  for (int k = 0; k < 4; ++k) p[k] = cascade(s, e, first + k * stride, 4 * stride, q);
  for (int i = 4 * q; i < count; ++i) p[0] += val(s, first + i * stride, e);
  for (int k = 1; k < 4; ++k) p[0] += p[k];
  return p[0];
}

/* ATen vectorized_inner_sum (M == 1) */
static float inner(const src_t *s, int64_t e, int n) {
  if (n < 8) return ilp4(s, e, 0, 1, n);
  const int nv = n / 8;
  float fin = 0.f;
  for (int k = 8 * nv; k < n; ++k) fin += val(s, k, e);
  for (int l = 0; l < 8; ++l) fin += ilp4(s, e, l, 8, nv);
  return fin;
}

static int64_t body_len(int64_t M) {
  if (M >= 8) return (M / 32) * 32;
  if (M >= 2) return (M / 4) * 4;
  return 0;
}

static float seg_sum(const src_t *s, int n, int64_t off, int64_t M, int64_t col) {
  if (M == 1) return inner(s, off, n);
  return col < body_len(M) ? cascade(s, off + col, 0, 1, n) : ilp4(s, off + col, 0, 1, n);
}

/* fp32 bucket: out[e] for every element of every segment.
 * mode 0: mean (sum / n); 1: sum only; weights != NULL: weighted sum. */
int fao_reduce_f32(const float *const *clients, int n, const oseg *segs, int nseg,
                   const float *weights, int mode, float *out) {
  if (n < 1 || !clients || !out || (nseg > 0 && !segs)) return -1;
  src_t s = {clients, NULL, weights};
  for (int k = 0; k < nseg; ++k) {
    const int64_t o = segs[k].offset, M = segs[k].numel;
    for (int64_t c = 0; c < M; ++c) {
      float r = 0.f + seg_sum(&s, n, o, M, c);
      if (!weights && mode == 0) r = r / (float)n;
      out[o + c] = r;
    }
  }
  return 0;
}

/* int64 bucket: .float() -> mean -> truncation toward zero */
int fao_reduce_i64(const int64_t *const *clients, int n, const oseg *segs, int nseg,
                   int64_t *out) {
  if (n < 1 || !clients || !out || (nseg > 0 && !segs)) return -1;
  src_t s = {NULL, clients, NULL};
  for (int k = 0; k < nseg; ++k) {
    const int64_t o = segs[k].offset, M = segs[k].numel;
    for (int64_t c = 0; c < M; ++c) {
      float r = (0.f + seg_sum(&s, n, o, M, c)) / (float)n;
      out[o + c] = (int64_t)r;
    }
  }
  return 0;
}
