"""Device buckets carved from shared slabs (r03).

Every client state lives in one flat fp32 bucket (arena.py).  Allocated one
by one, 20 wrn16_8 clients are 20 separate 44 MB device allocations, and on
some MI355X boxes the headline reduce over them runs ~8 % slower than over
the same buckets inside ONE allocation: 145.3 us against 134.2-134.8 us on
one box, same process, same bits, whatever the stride between the buckets
(256 B, 2 MiB, 2 MiB + 4 KiB, 2 MiB + 64 KiB + 256 B) —
profiles/r03_exp_alloc.jsonl (tools/archive/exp_alloc.py).  The placement of the
buckets in memory, not their data or their alignment, is what the box-to-box
spread of the headline came from (133 us on some boxes, 143-146 us on
others).

So device buckets are carved from slabs: one zero-filled allocation per
device holding many buckets, each bucket handed out as a tensor over its
OWN storage object (a slice of the slab's storage, which keeps the slab
alive).  A module bound to such a bucket therefore saves (torch.save) only
its own bytes, and the slab is freed when the last bucket carved from it
is.  Buckets are never recycled within a slab: the reference creates its
client models once and keeps them for every round (train_fedavg.py:367-380),
so the carve is append-only.  Set FA_SLAB=0 to allocate every bucket on its
own (the r02 behaviour).

Sizing (r04): a new slab holds as many buckets of the requested
size as the caller says it expects (``expecting(count)``: the engine binds a
round's N clients + the global under ``expecting(N + 1)``), else
SLAB_BUCKETS; always within MIN_SLAB..MAX_SLAB.

Limits of carved buckets: a bucket's storage is a slice of the
slab's, so its data pointer is not one the caching allocator handed out —
``Tensor.record_stream`` on a bucket is a silent no-op (a bucket used on a
side stream must be kept alive by the caller until that stream is done), and
CUDA/HIP IPC sharing of buckets (``torch.multiprocessing``) is not
supported.  Callers that need either set FA_SLAB=0 (plain allocations).
"""
from __future__ import annotations

import os
import threading

import torch

ALIGN = 64 * 1024                 # bucket starts, bytes
MIN_SLAB = 64 << 20               # bytes
MAX_SLAB = 2 << 30                # bytes (a bucket larger than this gets a slab of its own)
SLAB_BUCKETS = 24                 # buckets of the requested size per new slab

_lock = threading.Lock()
_current: dict = {}               # device -> [slab tensor (uint8), bytes handed out]
_expect = threading.local()       # .count: buckets the caller expects to carve


def enabled() -> bool:
    return os.environ.get("FA_SLAB", "1") != "0"


class expecting:
    """Context: the buckets carved inside are ``count`` of a kind, so a new
    slab started there is sized for ``count`` of them (not SLAB_BUCKETS)."""

    def __init__(self, count: int):
        self.count = max(1, int(count))

    def __enter__(self):
        self.prev = getattr(_expect, "count", None)
        _expect.count = self.count
        return self

    def __exit__(self, *exc):
        _expect.count = self.prev


def _slab_bytes(need: int) -> int:
    count = getattr(_expect, "count", None) or SLAB_BUCKETS
    size = min(max(count * need, MIN_SLAB), MAX_SLAB)
    return max(size, need)


def carve(numel: int, dtype: torch.dtype, device, force: bool = False) -> torch.Tensor:
    """A zeroed 1-D tensor of ``numel`` elements of ``dtype`` on ``device``,
    carved from the device's current slab (CUDA devices; ``force`` carves on
    any device, for tests) — or a plain ``torch.zeros`` when slabs are off."""
    device = torch.device(device)
    if not force and (device.type != "cuda" or not enabled()):
        return torch.zeros(numel, dtype=dtype, device=device)
    if device.type == "cuda" and device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    es = torch.empty((), dtype=dtype).element_size()
    nbytes = max(numel, 1) * es
    need = -(-nbytes // ALIGN) * ALIGN
    with _lock:
        cur = _current.get(device)
        if cur is None or cur[1] + need > cur[0].numel():
            cur = _current[device] = [torch.zeros(_slab_bytes(need), dtype=torch.uint8,
                                                  device=device), 0]
        off = cur[1]
        cur[1] += need
        st = cur[0].untyped_storage()[off:off + nbytes]
    return torch.empty(0, dtype=dtype, device=device).set_(st, 0, (numel,))


def release() -> None:
    """Forget the current slabs: the next bucket starts a new one (a slab's
    memory goes when its last bucket does)."""
    with _lock:
        _current.clear()
