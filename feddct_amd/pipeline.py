"""Host-ingress / egress pipeline for one GPU.

Client updates arrive in (pinned) host memory and the global model goes back
out: the round is PCIe-bound, not HBM-bound.  The bucket is cut into column
chunks (partition.range_plans); per chunk

    copy stream A : H2D of the chunk of every client bucket
    compute       : waits for A's event, reduces the chunk (exact order)
    copy stream B : waits for the kernel, D2H of the chunk of the result
                    into the global's host bucket

so chunk c+1's upload, chunk c's reduction and chunk c-1's download overlap
(the kernel is <1 % of the round).  Results are bit-identical to the
one-shot path: each chunk is a tile subset.

Chunks taper (r03 session 3): what follows the last upload — that chunk's
reduce and download — is 1/16 of the bucket, and the round makes 2 (no
broadcast: 15/16 + 1/16) or 5 (broadcast: 1/2, 1/4, 1/8, 1/16, 1/16)
copies per client instead of the 8 of r02's even cut; each copy costs
~20 us of its own.

The broadcast back to the clients' host buckets (``bcast*``) goes one of two
ways: ``fanout="host"`` (default) downloads each chunk of the result once
and copies it into every target on the CPU (ATen's multi-threaded copy)
while the GPU uploads the next chunks; ``fanout="dma"`` downloads it once
per target (N D2H copies per chunk on stream B).
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import torch

from . import _lib, slab
from .layout import BucketLayout
from .partition import range_plans


class HostPipeline:
    # measured (tools/archive/exp_pipeline.py, profiles/r03_exp_pipeline.jsonl):
    # with the broadcast the CPU fan-out of a chunk must overlap the later
    # uploads, so the first chunk stays at half; without it only the copy
    # count and the tail matter
    TAPER = (0.5, 0.25, 0.125, 0.0625, 0.0625)
    TAPER_NO_BCAST = (0.9375, 0.0625)

    def __init__(self, layout: BucketLayout, n: int, device: torch.device, nchunks: int = 0,
                 tile_elems: int = 0, fanout: str = "host", fractions=None):
        """``nchunks`` 0: the tapered cut (``fractions``, default TAPER); > 0:
        that many even chunks."""
        if fanout not in ("host", "dma"):
            raise ValueError(f"fanout must be 'host' or 'dma', not {fanout!r}")
        self.layout = layout
        self.device = device
        self.fanout = fanout
        with torch.cuda.device(device):
            if nchunks > 0:
                self.ranges, self.plan64 = range_plans(layout, nchunks, tile_elems)
                self.ranges_nb = self.ranges
            else:
                fr = tuple(fractions or self.TAPER)
                self.ranges, self.plan64 = range_plans(layout, len(fr), tile_elems,
                                                       fractions=fr)
                fr = tuple(fractions or self.TAPER_NO_BCAST)
                self.ranges_nb = range_plans(layout, len(fr), tile_elems, fractions=fr)[0]
            # the staged client buckets side by side in one slab (slab.py)
            self.dev32 = [slab.carve(max(layout.f32_numel, 64), torch.float32, device)
                          for _ in range(n)]
            self.dev64 = [torch.empty(max(layout.i64_numel, 1), dtype=torch.int64,
                                      device=device) for _ in range(n)]
            self.out32 = slab.carve(self.dev32[0].numel(), torch.float32, device)
            self.out64 = torch.zeros_like(self.dev64[0])
            self.s_in = torch.cuda.Stream(device)
            self.s_out = torch.cuda.Stream(device)
        self.n = n
        self.a32 = _lib.ptr_array([t.data_ptr() for t in self.dev32])
        self.a64 = _lib.ptr_array([t.data_ptr() for t in self.dev64])

    def run(self, host32: Sequence[torch.Tensor], host64: Sequence[torch.Tensor],
            out_host32: torch.Tensor, out_host64: torch.Tensor,
            bcast32: Sequence[torch.Tensor] = (), bcast64: Sequence[torch.Tensor] = (),
            weights=None, fanout: str = None) -> None:
        """One round.  ``host*`` are the clients' host buckets (slot order),
        ``out_host*`` the global's, ``bcast*`` extra host buckets that receive
        the result (the broadcast; they may be the clients' own buckets).
        Returns after the result is in every host bucket."""
        fanout = fanout or self.fanout
        ranges = self.ranges if (bcast32 or bcast64) else self.ranges_nb
        n = len(host32)
        if n != self.n:
            raise ValueError(f"pipeline built for {self.n} clients, got {n}")
        compute = torch.cuda.current_stream(self.device)
        w = None if weights is None else (ctypes.c_float * n)(*map(float, weights))
        # buffers of the previous round are free once its work is done
        self.s_in.wait_stream(compute)
        self.s_in.wait_stream(self.s_out)
        compute.wait_stream(self.s_out)
        ev_in = []
        with torch.cuda.stream(self.s_in):
            if self.plan64 is not None:
                for i in range(n):
                    self.dev64[i].copy_(host64[i], non_blocking=True)
            for lo, hi, _ in ranges:
                if hi > lo:
                    for i in range(n):
                        self.dev32[i][lo:hi].copy_(host32[i][lo:hi], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.s_in)
                ev_in.append(ev)
        stream = ctypes.c_void_p(compute.cuda_stream)
        dma = fanout == "dma"
        ev_out = []
        for c, (lo, hi, plan) in enumerate(ranges):
            compute.wait_event(ev_in[c])
            if plan is not None:
                _lib.check(_lib.lib.fa_reduce(plan.handle, self.a32, self.a64, n, w,
                                              self.out32.data_ptr(), self.out64.data_ptr(), 0,
                                              stream), "fa_reduce(chunk)")
            ev = torch.cuda.Event()
            ev.record(compute)
            self.s_out.wait_event(ev)
            if hi > lo:
                with torch.cuda.stream(self.s_out):
                    out_host32[lo:hi].copy_(self.out32[lo:hi], non_blocking=True)
                    if dma:
                        for t in bcast32:
                            t[lo:hi].copy_(self.out32[lo:hi], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.s_out)
            ev_out.append(ev)
        if self.plan64 is not None:
            _lib.check(_lib.lib.fa_reduce(self.plan64.handle, self.a32, self.a64, n, None,
                                          self.out32.data_ptr(), self.out64.data_ptr(), 0,
                                          stream), "fa_reduce(int64)")
            ev = torch.cuda.Event()
            ev.record(compute)
            self.s_out.wait_event(ev)
            with torch.cuda.stream(self.s_out):
                out_host64.copy_(self.out64, non_blocking=True)
                if dma:
                    for t in bcast64:
                        t.copy_(self.out64, non_blocking=True)
        if not dma and (bcast32 or bcast64):
            # each chunk fans out on the CPU as soon as it is in host memory,
            # while the GPU still uploads and reduces the later chunks
            for (lo, hi, _), ev in zip(ranges, ev_out):
                if hi > lo:
                    ev.synchronize()
                    src = out_host32[lo:hi]
                    for t in bcast32:
                        if t.data_ptr() != out_host32.data_ptr():
                            t[lo:hi].copy_(src)
        self.s_out.synchronize()
        if not dma:
            for t in bcast64:
                if t.data_ptr() != out_host64.data_ptr():
                    t.copy_(out_host64)
