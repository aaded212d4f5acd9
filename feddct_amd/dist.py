"""Client-sharded aggregation across the GPUs of one node.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).
Rank r holds a contiguous shard of the client slots.  A round is:

1. local partial: the HIP kernel sums the rank's clients for every fp32 key
   in the torch order, without the /N (FA_F_SUM_ONLY);
2. exchange: ``all_reduce(SUM)`` of the partial bucket over RCCL — every rank
   needs the global model afterwards to reload its own client slots, so the
   "final reduce" of the north_star is an all-reduce; the bucket is cut into
   chunks at key boundaries and chunk c's all-reduce (RCCL's own stream) runs
   while the kernel sums chunk c+1;
3. finish: ``/ N_total`` (IEEE division, fa_div_f32).

int64 keys (a few bytes) are exchanged raw — an all-gather of every rank's
int64 buckets — and reduced exactly over all N_total clients by the same
kernel, so they match the single-process reference bit-for-bit.

The fp32 result is the exact torch-order sum within each shard, but the
cross-rank all-reduce re-associates it: it is NOT bit-identical to the
single-process reference (bench.py reports the max ULP distance).  The exact
element-sharded mode (§8 e2) is listed under "next" in DESIGN.md.

The arithmetic backends are pluggable so the orchestration is testable on
CPU with gloo (tests/test_dist_gloo.py injects oracle backends); the product
backend is ``HipBackend``.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

from .layout import BucketLayout


def shard_range(n_total: int, world: int, rank: int):
    """Contiguous client-slot shard of ``rank`` (slot order is preserved)."""
    base, rem = divmod(n_total, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def chunk_segments(layout: BucketLayout, nchunks: int):
    """Split the fp32 segments into <= nchunks consecutive groups of roughly
    equal bytes.  Returns [(segs ndarray, lo, hi)] with [lo, hi) the bucket
    range the group spans (gaps are layout padding)."""
    segs = layout.segs32
    if len(segs) == 0:
        return []
    total = int(segs[:, 1].sum())
    target = max(1, total // max(1, nchunks))
    groups, cur, acc = [], [], 0
    for o, m in segs:
        cur.append((o, m))
        acc += m
        if acc >= target and len(groups) < nchunks - 1:
            groups.append(cur)
            cur, acc = [], 0
    if cur:
        groups.append(cur)
    out = []
    for i, g in enumerate(groups):
        arr = np.array(g, np.int64)
        lo = int(arr[0, 0])
        hi = int(groups[i + 1][0][0]) if i + 1 < len(groups) else layout.f32_numel
        out.append((arr, lo, hi))
    return out


class HipBackend:
    """fa_reduce / fa_div_f32 on the current device and stream."""

    def __init__(self, layout: BucketLayout, chunks, n_local: int, n_total: int):
        from . import _lib
        self._lib = _lib
        self.plans = [_lib.Plan(s, layout.f32_numel) for s, _, _ in chunks]
        self.plan64 = (_lib.Plan(np.zeros((0, 2), np.int64), 0, layout.segs64, layout.i64_numel)
                       if layout.i64_numel else None)

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def partial_sum(self, chunk_index, clients32: Sequence[torch.Tensor], out: torch.Tensor):
        L = self._lib
        a = L.ptr_array([t.data_ptr() for t in clients32])
        L.check(L.lib.fa_reduce(self.plans[chunk_index].handle, a, None, len(clients32), None,
                                out.data_ptr(), None, L.FA_F_SUM_ONLY, self._stream()),
                "fa_reduce(partial)")

    def divide(self, x: torch.Tensor, d: float, out: torch.Tensor):
        L = self._lib
        L.check(L.lib.fa_div_f32(x.data_ptr(), float(d), out.data_ptr(), x.numel(),
                                 self._stream()), "fa_div_f32")

    def reduce_i64(self, clients64: Sequence[torch.Tensor], out: torch.Tensor):
        if self.plan64 is None:
            return
        L = self._lib
        a = L.ptr_array([t.data_ptr() for t in clients64])
        L.check(L.lib.fa_reduce(self.plan64.handle, None, a, len(clients64), None, None,
                                out.data_ptr(), 0, self._stream()), "fa_reduce(i64)")


class ShardedAggregator:
    """The cross-GPU round over pre-bound buckets (bench.py's N>1 step).

    ``final="reduce"`` (default): the north_star's final RCCL reduce — the
    global state lands on ``root`` (the server), like the single-process
    reference where the global model is one module; ``final="allreduce"``:
    every rank gets it (reduce + the cross-GPU half of the broadcast)."""

    def __init__(self, layout: BucketLayout, local32: List[torch.Tensor],
                 local64: List[torch.Tensor], n_total: int, out32: torch.Tensor,
                 out64: torch.Tensor, nchunks: int = 8, backend=None, group=None,
                 final: str = "reduce", root: int = 0):
        if final not in ("reduce", "allreduce"):
            raise ValueError(f"final must be 'reduce' or 'allreduce', not {final!r}")
        self.final = final
        self.root = root
        self.rank = dist.get_rank(group)
        self.layout = layout
        self.local32, self.local64 = local32, local64
        self.n_total = n_total
        self.out32, self.out64 = out32, out64
        self.group = group
        self.world = dist.get_world_size(group)
        self.chunks = chunk_segments(layout, nchunks)
        self.backend = backend or HipBackend(layout, self.chunks, len(local32), n_total)
        self.partial = torch.zeros_like(out32)
        # int64 keys: every rank's buckets gathered raw; shards may be uneven,
        # so each rank sends max-shard rows and only the real ones are used
        nmax = -(-n_total // self.world)
        width = max(1, layout.i64_numel)
        self.gather64 = torch.zeros((self.world * nmax, width), dtype=torch.int64,
                                    device=out64.device)
        self.stack64 = torch.zeros((nmax, width), dtype=torch.int64, device=out64.device)
        rows = []
        for r in range(self.world):
            lo, hi = shard_range(n_total, self.world, r)
            rows += [r * nmax + j for j in range(hi - lo)]
        self.rows64 = rows

    def step(self) -> None:
        works = []
        to_root = self.final == "reduce"
        gdst = self.root if self.group is None else dist.get_global_rank(self.group, self.root)
        for c, (_, lo, hi) in enumerate(self.chunks):
            self.backend.partial_sum(c, self.local32, self.partial)
            if to_root:
                works.append(dist.reduce(self.partial[lo:hi], dst=gdst, op=dist.ReduceOp.SUM,
                                         group=self.group, async_op=True))
            else:
                works.append(dist.all_reduce(self.partial[lo:hi], op=dist.ReduceOp.SUM,
                                             group=self.group, async_op=True))
        w64 = None
        if self.layout.i64_numel:
            for j, t in enumerate(self.local64):
                self.stack64[j].copy_(t)
            w64 = dist.all_gather_into_tensor(self.gather64, self.stack64, group=self.group,
                                              async_op=True)
        has_result = not to_root or self.rank == self.root
        # finish chunk c (/N_total) as soon as its exchange lands, while the
        # exchanges of the later chunks are still on the wire
        for w, (_, lo, hi) in zip(works, self.chunks):
            w.wait()
            if has_result:
                self.backend.divide(self.partial[lo:hi], float(self.n_total),
                                    self.out32[lo:hi])
        if w64 is not None:
            w64.wait()
            if has_result:
                self.backend.reduce_i64([self.gather64[r] for r in self.rows64], self.out64)


# --------------------------------------------------------------------------
# Exact mode: element (column) stripes.
# --------------------------------------------------------------------------
class HipStripeBackend:
    """Stripe reduction with the HIP kernel over a tile-subset plan."""

    def __init__(self, layout: BucketLayout, stripe_tiles, tiles64):
        from . import _lib
        self._lib = _lib
        te = 0
        self.plan = (_lib.Plan(None, layout.f32_numel, None, layout.i64_numel, te,
                               tiles=stripe_tiles) if len(stripe_tiles) else None)
        self.plan64 = (_lib.Plan(None, layout.f32_numel, None, layout.i64_numel, te,
                                 tiles=tiles64) if len(tiles64) else None)

    def reduce_stripe(self, sources, out32: torch.Tensor):
        """``sources[k] = (tensor, base)``: client slot k's element e lives at
        ``tensor[e - base]`` for e in this rank's stripe."""
        if self.plan is None:
            return
        L = self._lib
        ptrs = [t.data_ptr() - 4 * base for t, base in sources]
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        L.check(L.lib.fa_reduce(self.plan.handle, L.ptr_array(ptrs), None, len(ptrs), None,
                                out32.data_ptr(), None, 0, s), "fa_reduce(stripe)")

    def reduce_i64(self, clients64, out64: torch.Tensor):
        if self.plan64 is None:
            return
        L = self._lib
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        L.check(L.lib.fa_reduce(self.plan64.handle, None,
                                L.ptr_array([t.data_ptr() for t in clients64]), len(clients64),
                                None, None, out64.data_ptr(), 0, s), "fa_reduce(i64)")


class StripedAggregator:
    """Bit-exact cross-GPU round: rank r owns the column stripe
    [lo_r, hi_r) of the bucket (cut at vector-tile starts, partition.py), gets
    every client's values for those columns, reduces them in the exact torch
    order and the stripes are exchanged so every rank ends with the full
    global state.  Two ingress forms:

    * ``step_device(local32, local64)`` — client slots device-resident and
      sharded by rank (as in ShardedAggregator): the stripes travel
      rank-to-rank as grouped P2P send/recv over RCCL (n·B·(W-1)/W per rank:
      the price of exactness on device-resident inputs);
    * ``step_host(stripes32, clients64)`` — client updates in host memory:
      each GPU uploads only ITS stripe of every client (no xGMI traffic for
      inputs; ingress bandwidth scales with the GPUs' PCIe links).

    The result is the same bits as the single-GPU reduction (tested).
    """

    def __init__(self, layout: BucketLayout, n_total: int, out32: torch.Tensor,
                 out64: torch.Tensor, group=None, backend=None, final: str = "allreduce",
                 root: int = 0):
        from .partition import i64_tiles, layout_tiles, split_tiles
        if final not in ("reduce", "allreduce"):
            raise ValueError(f"final must be 'reduce' or 'allreduce', not {final!r}")
        self.final, self.root = final, root
        self.layout = layout
        self.n_total = n_total
        self.out32, self.out64 = out32, out64
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        info, tiles = layout_tiles(layout)
        parts = split_tiles(tiles, self.world, layout.f32_numel)
        self.ranges = [(lo, hi) for lo, hi, _ in parts]
        self.lo, self.hi = self.ranges[self.rank]
        self.backend = backend or HipStripeBackend(layout, parts[self.rank][2], i64_tiles(tiles))
        L = self.hi - self.lo
        self.lpad = (L + 3) // 4 * 4
        dev = out32.device
        self.recv = torch.zeros((n_total, max(self.lpad, 4)), dtype=torch.float32, device=dev)
        nmax = -(-n_total // self.world)
        width = max(1, layout.i64_numel)
        self.gather64 = torch.zeros((self.world * nmax, width), dtype=torch.int64, device=dev)
        self.stack64 = torch.zeros((nmax, width), dtype=torch.int64, device=dev)
        self.rows64 = []
        self.shards = [shard_range(n_total, self.world, r) for r in range(self.world)]
        for r, (a, b) in enumerate(self.shards):
            self.rows64 += [r * nmax + j for j in range(b - a)]

    def _peer(self, r):
        return r if self.group is None else dist.get_global_rank(self.group, r)

    def _gather_stripes(self, ops):
        """Finished stripes of out32 to every other rank ("allreduce") or to
        the root only ("reduce"), P2P straight into out32 views."""
        me = self.rank
        for r in range(self.world):
            if r == me:
                continue
            lo, hi = self.ranges[r]
            if self.hi > self.lo and (self.final == "allreduce" or r == self.root):
                ops.append(dist.P2POp(dist.isend, self.out32[self.lo:self.hi], self._peer(r),
                                      self.group))
            if hi > lo and (self.final == "allreduce" or me == self.root):
                ops.append(dist.P2POp(dist.irecv, self.out32[lo:hi], self._peer(r), self.group))

    def _run(self, ops):
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()

    def _i64(self, local64):
        if not self.layout.i64_numel:
            return
        for j, t in enumerate(local64):
            self.stack64[j].copy_(t)
        dist.all_gather_into_tensor(self.gather64, self.stack64, group=self.group)
        self.backend.reduce_i64([self.gather64[r] for r in self.rows64], self.out64)

    def step_device(self, local32: List[torch.Tensor], local64: List[torch.Tensor]) -> None:
        me = self.rank
        a, b = self.shards[me]
        assert len(local32) == b - a
        ops = []
        for r in range(self.world):
            if r == me:
                continue
            lo, hi = self.ranges[r]
            if hi > lo:
                for t in local32:
                    ops.append(dist.P2POp(dist.isend, t[lo:hi], self._peer(r), self.group))
            qa, qb = self.shards[r]
            if self.hi > self.lo:
                for k in range(qa, qb):
                    ops.append(dist.P2POp(dist.irecv, self.recv[k, :self.hi - self.lo],
                                          self._peer(r), self.group))
        self._run(ops)
        sources = []
        for k in range(self.n_total):
            if a <= k < b:
                sources.append((local32[k - a], 0))
            else:
                sources.append((self.recv[k], self.lo))
        self.backend.reduce_stripe(sources, self.out32)
        self._i64(local64)
        ops = []
        self._gather_stripes(ops)
        self._run(ops)

    def step_host(self, stripes32: Sequence[torch.Tensor], clients64: Sequence[torch.Tensor],
                  local64: Optional[List[torch.Tensor]] = None) -> None:
        """``stripes32[k]``: client slot k's values for THIS rank's columns
        [lo, hi) (host, pinned), ``clients64[k]``: its int64 bucket."""
        L = self.hi - self.lo
        for k, t in enumerate(stripes32):
            self.recv[k, :L].copy_(t, non_blocking=True)
        self.backend.reduce_stripe([(self.recv[k], self.lo) for k in range(self.n_total)],
                                   self.out32)
        if self.layout.i64_numel:
            g = torch.stack([t.to(self.out64.device, non_blocking=True) for t in clients64])
            self.backend.reduce_i64(list(g.unbind(0)), self.out64)
        ops = []
        self._gather_stripes(ops)
        self._run(ops)
