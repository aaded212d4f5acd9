"""ORACLE — test infrastructure only (never imported by the product path).

CPU restatement, in numpy float32, of the arithmetic the reference's hot path
performs:

    global_dict[k] = torch.stack([client_models[i].state_dict()[k].float()
                                  for i in range(N)], 0).mean(0)
    (train_fedavg.py:143-147, train_fedprox.py:148-152, train_feddct.py:42-50,
     train_splitfed.py:42-50)

followed by ``global_model.load_state_dict(global_dict)`` (train_fedavg.py:147)
which copies the fp32 mean into the parameter's own dtype (int64 buffers:
truncation toward zero).

Torch's CPU ``sum`` over dim 0 of a contiguous ``[N, M]`` stack does NOT add
the N rows sequentially.  It uses ATen's SumKernel (``cascade_sum``) whose
order depends on the column's position inside the tensor:

* ``cascade(x_0..x_{n-1})`` = ATen ``multi_row_sum``: 4 accumulator levels,
  level step 2**max(4, ceil_log2(n)//4) (=16 for n < 2**20).
* ``ilp4(x)`` = ATen ``row_sum``: 4 interleaved cascades + remainder.
* ``inner8(x)`` = ATen ``vectorized_inner_sum`` for M == 1, n >= 8.

Column rule (V = 8 floats, the width torch's fp32 sum kernel runs at):
  M >= 8      : columns j <  (M//32)*32 -> cascade, the rest -> ilp4
  2 <= M < 8  : columns j <  (M//4)*4   -> cascade, the rest -> ilp4
  M == 1      : n < 8 -> ilp4, else inner8

then ``out = (+0 + sum) / N`` with IEEE true division (``mean`` = ``sum_out``
then ``div_(N)``).  numpy float32 ``+`` and ``/`` are correctly rounded and
never contracted, so this restatement is bit-exact by construction; it is
pinned against torch itself and the reference's own ``server_aggregate``
outputs by tests/test_oracle.py and tests/golden/.

This file is the checker for the HIP kernels in feddct_amd/csrc/fedagg.hip.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


def ceil_log2(n: int) -> int:
    """c10::utils::CeilLog2 (n <= 1 -> 0)."""
    if n <= 1:
        return 0
    return int(n - 1).bit_length()


def level_power(n: int) -> int:
    return max(4, ceil_log2(n) // 4)


def cascade(rows) -> np.ndarray:
    """ATen multi_row_sum over a sequence of equal-shape float32 rows.

    ``rows`` is an indexable of length n (rows[i] is an array); the result is
    the per-column cascade sum with accumulators starting at +0.
    """
    n = len(rows)
    shape = np.shape(rows[0]) if n else ()
    lp = level_power(n)
    step = 1 << lp
    mask = step - 1
    acc = [np.zeros(shape, F32) for _ in range(4)]
    i = 0
    while i + step <= n:
        for _ in range(step):
            acc[0] = (acc[0] + rows[i]).astype(F32)
            i += 1
        for j in range(1, 4):
            acc[j] = (acc[j] + acc[j - 1]).astype(F32)
            acc[j - 1] = np.zeros(shape, F32)
            if i & (mask << (j * lp)):
                break
    while i < n:
        acc[0] = (acc[0] + rows[i]).astype(F32)
        i += 1
    for j in range(1, 4):
        acc[0] = (acc[0] + acc[j]).astype(F32)
    return acc[0]


def cascade_state(rows, row0: int, n_total: int, acc=None):
    """The cascade's four level accumulators after rows row0..row0+len-1 of
    an ``n_total``-row ``multi_row_sum`` (``acc``: the state after rows
    0..row0-1; None = the start, all +0).  Promotions happen after every
    ``step``-th row of the WHOLE reduction, so chaining segments in slot order
    and finishing with ``cascade_finish`` is ``cascade`` over all rows — the
    order fa_reduce_chain reproduces (feddct_amd/csrc/fedagg.hip)."""
    lp = level_power(n_total)
    step = 1 << lp
    mask = step - 1
    shape = np.shape(rows[0]) if len(rows) else np.shape(acc[0])
    acc = [np.zeros(shape, F32) for _ in range(4)] if acc is None else [a.copy() for a in acc]
    for j in range(len(rows)):
        i = row0 + j + 1
        acc[0] = (acc[0] + rows[j]).astype(F32)
        if i & mask:
            continue
        for lev in range(1, 4):
            acc[lev] = (acc[lev] + acc[lev - 1]).astype(F32)
            acc[lev - 1] = np.zeros(shape, F32)
            if i & (mask << (lev * lp)):
                break
    return acc


def cascade_finish(acc) -> np.ndarray:
    out = acc[0]
    for j in range(1, 4):
        out = (out + acc[j]).astype(F32)
    return out


def chain_levels(rows: int, n_total: int) -> int:
    """Bit l: level l of ``cascade_state`` may be nonzero after ``rows`` rows
    (restates fa_chain_levels)."""
    if rows <= 0:
        return 0
    lp = level_power(n_total)
    step = 1 << lp
    m = 0
    if rows % step:
        m |= 1
    if (rows >> lp) % step:
        m |= 2
    if n_total >= 256:
        if (rows >> (2 * lp)) % step:
            m |= 4
        if rows >> (3 * lp):
            m |= 8
    return m


def ilp4(rows) -> np.ndarray:
    """ATen row_sum: rows viewed as (-1, 4); 4 interleaved cascades."""
    n = len(rows)
    q = n // 4
    parts = [cascade([rows[4 * r + k] for r in range(q)]) if q else None
             for k in range(4)]
    shape = np.shape(rows[0])
    parts = [p if p is not None else np.zeros(shape, F32) for p in parts]
    for i in range(4 * q, n):
        parts[0] = (parts[0] + rows[i]).astype(F32)
    for k in range(1, 4):
        parts[0] = (parts[0] + parts[k]).astype(F32)
    return parts[0]


def inner8(vals: np.ndarray) -> F32:
    """ATen vectorized_inner_sum for a contiguous 1-D reduction (M == 1).

    Lanes of 8: ``row_sum`` (ilp4) over the n//8 vectors, then scalar tail
    into a fresh +0 accumulator, then lanes 0..7 added in order.
    """
    vals = np.asarray(vals, F32)
    n = vals.shape[0]
    nv = n // 8
    vecs = [vals[8 * v:8 * v + 8] for v in range(nv)]
    lanes = ilp4(vecs) if nv else np.zeros(8, F32)
    fin = F32(0)
    for k in range(8 * nv, n):
        fin = F32(fin + vals[k])
    for k in range(8):
        fin = F32(fin + lanes[k])
    return fin


def body_len(M: int) -> int:
    """Number of leading columns of an M-column tensor torch sums by cascade."""
    if M >= 8:
        return (M // 32) * 32
    if M >= 2:
        return (M // 4) * 4
    return 0


def torch_sum0(x: np.ndarray) -> np.ndarray:
    """Bit-exact restatement of ``torch.sum(x, 0)`` for float32 x of shape
    [N, ...] on CPU (single-thread order; see DESIGN.md for the one
    thread-count-dependent corner of torch itself).  Returns shape x.shape[1:].
    """
    x = np.ascontiguousarray(x, F32)
    n = x.shape[0]
    out_shape = x.shape[1:]
    M = int(np.prod(out_shape)) if out_shape else 1
    x2 = x.reshape(n, M)
    if M == 1:
        col = x2[:, 0]
        s = ilp4([col[i:i + 1] for i in range(n)])[0] if n < 8 else inner8(col)
        res = np.array([F32(F32(0) + F32(s))], F32)
        return res.reshape(out_shape)
    b = body_len(M)
    res = np.empty(M, F32)
    if b:
        res[:b] = cascade([x2[i, :b] for i in range(n)])
    if b < M:
        res[b:] = ilp4([x2[i, b:] for i in range(n)])
    res = (F32(0) + res).astype(F32)
    return res.reshape(out_shape)


def torch_mean0(x: np.ndarray) -> np.ndarray:
    """``torch.stack(list).float().mean(0)`` on CPU: sum then true div by N."""
    n = np.shape(x)[0]
    s = torch_sum0(x)
    return (s / F32(n)).astype(F32)


def weighted_sum0(x: np.ndarray, w: np.ndarray) -> np.ndarray:
    """Weighted extension (not in the reference):
    ``torch.stack([x_i.float() * w_i], 0).sum(0)``, w_i float32 scalars.
    Each product is rounded to fp32, then summed in the torch order."""
    x = np.asarray(x, F32)
    w = np.asarray(w, F32).reshape((-1,) + (1,) * (x.ndim - 1))
    return torch_sum0((x * w).astype(F32))


def weights_from_sizes(sizes) -> np.ndarray:
    """w_i = fp32(n_i / sum(n)) computed in float64 then rounded once."""
    s = np.asarray(sizes, np.float64)
    return (s / s.sum()).astype(F32)


def mean_i64_trunc(x: np.ndarray) -> np.ndarray:
    """int64 keys (num_batches_tracked): ``.float()`` (round-to-nearest),
    fp32 mean as above, then ``copy_`` fp32 -> int64 truncation toward zero
    (train_fedavg.py:146-147)."""
    xf = np.asarray(x).astype(F32)
    m = torch_mean0(xf)
    return np.trunc(m).astype(np.int64)


def aggregate_state(client_states):
    """Reference ``server_aggregate`` on one model (train_fedavg.py:143-147):
    ``client_states`` is a list (slot order) of lists of (key, ndarray) in
    global-state_dict key order.  Returns [(key, ndarray)] with each key in its
    own dtype (float32 mean, or int64 trunc of the fp32 mean)."""
    out = []
    for j, (k, v0) in enumerate(client_states[0]):
        x = np.stack([np.asarray(s[j][1]) for s in client_states], 0)
        if np.asarray(v0).dtype == np.int64:
            out.append((k, mean_i64_trunc(x)))
        else:
            out.append((k, torch_mean0(x.astype(F32))))
    return out


def state_digest(state):
    """SHA-256 over key names + raw bytes (matches tests/golden/make_golden.py)."""
    import hashlib
    h = hashlib.sha256()
    for k, v in state:
        h.update(k.encode())
        h.update(np.ascontiguousarray(v).tobytes())
    return h.hexdigest()
