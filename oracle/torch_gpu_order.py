"""ORACLE — test infrastructure only (never imported by the product path).

numpy restatement of torch-ROCm's GPU ``torch.stack(list, 0).mean(0)`` for
fp32 — the order the reference's original runs used, since their models sit
on the GPU (train_fedavg.py:244-250) when ``server_aggregate`` runs
(train_fedavg.py:145-146).  Restated from the ROCm build's own headers,
ATen/native/hip/Reduce.cuh (setReduceConfig, thread_reduce_impl,
block_x_reduce / block_y_reduce) and SharedReduceOps.h (MeanOps), with the
mean kernel's factor (ReduceMomentKernel: factor = float(num_outputs) /
numel, ``project(acc) = acc * factor``).

For a contiguous [N, M] stack reduced over dim 0:

* M >= 2 ("vectorize along output"): output_vec_size ovs = 4/2/1 (largest
  dividing M); dim0 = M / ovs, dim1 = N; block width bw and height bh from
  set_block_dimension (max 512/ovs threads, warp 64).  If N >= min(16*bh,
  256) the N rows are split across the bh warps of a block (warp y takes
  rows y, y+bh, ...) and combined by block_y_reduce's halving tree; else one
  thread walks all N rows.  A thread's rows go round-robin into 4
  accumulators (vt0 = 4: its p-th row into acc[p % 4]), combined
  ((a0 + a1) + a2) + a3.
* M == 1 (a 0-d key stacked to [N]), N < 128: the N values are split over bw =
  last_pow2(N) lanes (lane x: rows x, x+bw, ...; 4 accumulators), then
  block_x_reduce's intra-warp tree with offsets 1, 2, 4, ... (ROCm order).
* M == 1 with N >= 128: torch vectorises along the input (dim0 = N // 4 >=
  32): bw = last_pow2(N // 4) threads (at most 512); thread x adds the
  4-vectors x, x+bw, ... component-wise into 4 accumulators, then row
  N - N%4 + x (if any) into accumulator 0, and combines ((v0+v1)+v2)+v3
  (input_vectorized_thread_reduce_impl); block_x_reduce then halves through
  shared memory for offsets bw/2 .. 64 and finishes with the intra-warp tree
  (offsets 1, 2, 4, ...).
* out = acc * factor, factor = fl(fl(M) / fl(N*M)) — a multiply, not /N.

Scope: N >= 2 and no cross-block ("global") split.  setReduceConfig splits
a reduction across blocks only when the rows are split across warps, the
values per thread reach 256 and the output grid is small against the target
grid (MI355X: 256 CUs; ROCm caps threads per CU at 256 for a 2-D iterator
unless the grid is one block) by a factor of 16 or more; ``supported``
reports it.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32
WARP = 64
NUM_CU = 256             # MI355X multiProcessorCount
MAX_THREADS_PER_CU = 2048  # MI355X maxThreadsPerMultiProcessor


def last_pow2(n: int) -> int:
    return 1 << (int(n).bit_length() - 1) if n > 0 else 0


def _div_up(a: int, b: int) -> int:
    return -(-a // b)


def config(n: int, m: int):
    """Launch shape torch-ROCm picks for a [n, m] stack reduced over dim 0:
    kind 'inner' (m == 1: bw lanes, ``vec`` = input-vectorised) or 'outer'
    (bh = the row split S when ``split``; ``global`` = a cross-block split)."""
    if m == 1:
        if n < 128:
            return {"kind": "inner", "bw": last_pow2(n), "vec": False,
                    "global": False}
        d0 = n // 4
        bw = last_pow2(d0) if d0 < 512 else 512
        return {"kind": "inner", "bw": bw, "vec": True, "global": _div_up(n, bw) >= 256}
    ovs = 4 if m % 4 == 0 else (2 if m % 2 == 0 else 1)
    mnt = 512 // ovs
    dim0, dim1 = m // ovs, n
    d0 = last_pow2(dim0) if dim0 < mnt else mnt
    d1 = last_pow2(dim1) if dim1 < mnt else mnt
    bw = min(d0, WARP)
    bh = min(d1, mnt // bw)
    bw = min(d0, mnt // bh)
    split = n >= min(bh * 16, 256)
    glob = False
    vpt = _div_up(n, bh) if split else n
    if split and vpt >= 256:
        grid = _div_up(dim0, bw)
        tpm = MAX_THREADS_PER_CU if grid == 1 else 256
        target = NUM_CU * (tpm // (bw * bh))
        if grid <= target:
            c = max(min(_div_up(target, grid), _div_up(vpt, 16)), _div_up(vpt, 256))
            if c > NUM_CU:
                c = NUM_CU
            elif c > _div_up(NUM_CU, 2):
                c = _div_up(NUM_CU, 2)
            elif c < 16:
                c = 1
            glob = c > 1
    return {"kind": "outer", "bh": bh if split else 1, "bw": bw, "split": split,
            "global": glob}


def supported(n: int, m: int) -> bool:
    return n >= 2 and not config(n, m)["global"]


def _thread(rows):
    """thread_reduce_impl: rows (in the thread's order) round-robin into 4
    accumulators from +0, combined in order."""
    shape = np.shape(rows[0])
    acc = [np.zeros(shape, F32) for _ in range(4)]
    for p, r in enumerate(rows):
        acc[p % 4] = (acc[p % 4] + r).astype(F32)
    out = acc[0]
    for i in range(1, 4):
        out = (out + acc[i]).astype(F32)
    return out


def factor(n: int, m: int) -> F32:
    return F32(F32(m) / F32(n * m))


def gpu_sum0(x: np.ndarray) -> np.ndarray:
    """The pre-factor accumulator of torch-ROCm's reduction over dim 0."""
    x = np.ascontiguousarray(x, F32)
    n = x.shape[0]
    m = int(np.prod(x.shape[1:])) if x.ndim > 1 else 1
    x2 = x.reshape(n, m)
    assert supported(n, m), (n, m)
    c = config(n, m)
    if c["kind"] == "inner" and c["vec"]:
        return _inner_vec(x2[:, 0], c["bw"]).reshape(x.shape[1:])
    if c["kind"] == "inner":
        bw = c["bw"]
        lanes = [_thread([x2[r] for r in range(ln, n, bw)]) for ln in range(bw)]
        off = 1
        while off < bw:   # lane i += lane i+off (shfl_down), offsets increasing
            lanes = [(lanes[i] + lanes[i + off]).astype(F32) if i + off < bw else lanes[i]
                     for i in range(bw)]
            off <<= 1
        return lanes[0].reshape(x.shape[1:])
    bh = c["bh"]
    vals = [_thread([x2[r] for r in range(y, n, bh)]) for y in range(bh)]
    off = bh // 2
    while off > 0:        # block_y_reduce: shared[y] += shared[y + off]
        vals = [(vals[y] + vals[y + off]).astype(F32) if y < off else vals[y]
                for y in range(bh)]
        off //= 2
    return vals[0].reshape(x.shape[1:])


def _inner_vec(col: np.ndarray, bw: int) -> F32:
    """M == 1, N >= 128: the input-vectorised thread order + block_x_reduce."""
    n = col.shape[0]
    tail = n - n % 4
    vals = []
    for t in range(bw):
        v = [F32(0)] * 4
        q = t
        while 4 * q + 3 < n:
            for i in range(4):
                v[i] = F32(v[i] + col[4 * q + i])
            q += bw
        if tail + t < n:
            v[0] = F32(v[0] + col[tail + t])
        vals.append(F32(F32(F32(v[0] + v[1]) + v[2]) + v[3]))
    dim_x = bw
    if bw > WARP:           # shared-memory halving down to one warp
        off = bw // 2
        while off >= WARP:
            vals = [F32(vals[i] + vals[i + off]) if i < off else vals[i] for i in range(bw)]
            off //= 2
        dim_x = WARP
    off = 1
    while off < dim_x:      # intra-warp tree, increasing offsets (ROCm)
        vals = [F32(vals[i] + vals[i + off]) if i + off < dim_x else vals[i]
                for i in range(dim_x)]
        off <<= 1
    return np.asarray(vals[0], F32)


def gpu_mean0(x: np.ndarray) -> np.ndarray:
    n = x.shape[0]
    m = int(np.prod(x.shape[1:])) if x.ndim > 1 else 1
    return (gpu_sum0(x) * factor(n, m)).astype(F32)


def gpu_mean_i64_trunc(x: np.ndarray) -> np.ndarray:
    """int64 keys on the GPU path: .float(), the GPU mean, copy_ -> int64."""
    return np.trunc(gpu_mean0(np.asarray(x).astype(F32))).astype(np.int64)
