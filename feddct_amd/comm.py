"""Native multi-GPU rounds over RCCL (libfedagg_comm.so, include/fedagg_comm.h;
SURVEY.md §8 b, e).

One process per GPU, client slots sharded contiguously in slot order.  The
default entry, ``NativeAggregator`` (fa_multi_plan_create / fa_reduce_multi),
is EXACT: bit-identical to one GPU reducing every slot, i.e. to the
reference's single-process ``stack(...).mean(0)`` (train_feddct.py:42-50) —
the exact form (blocked, chained or striped) and chunk count with the lowest
modelled time (r06: fa_round_model, ``round_model``; ``multi_select`` names
the choice without a GPU; r05 chose blocked-else-chained by geometry).
The re-associated e1 round (partial sums + an RCCL sum) is opt-in
(``exact=False``, or ``NativeShardedAggregator``): measured r04, max 22,938
ULP from the exact result (``E1_ULP_R04``).  torch.distributed only carries
the communicator's 128-byte id from rank 0 to the others; the data path is
the library's own RCCL communicator.

No fallback: loading raises if libfedagg_comm.so is missing.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from .dist import shard_range
from .layout import BucketLayout

COMM_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libfedagg_comm.so")
FA_E_COMM = -6
FA_COMM_UID_BYTES = 128

COMM_EXPORTS = ["fa_comm_unique_id", "fa_comm_init_rank", "fa_comm_init", "fa_comm_destroy",
                "fa_comm_info", "fa_comm_set_graphs", "fa_shard_plan_create", "fa_shard_plan_create_ex",
                "fa_shard_plan_destroy", "fa_reduce_sharded", "fa_mean_f32_multi",
                "fa_stripe_plan_create", "fa_stripe_plan_destroy", "fa_reduce_striped",
                "fa_chain_plan_create", "fa_chain_plan_destroy", "fa_reduce_chained",
                "fa_block_plan_create", "fa_block_plan_destroy", "fa_reduce_blocked",
                "fa_describe_round", "fa_multi_select", "fa_multi_plan_create",
                "fa_multi_plan_mode", "fa_multi_plan_destroy", "fa_reduce_multi",
                "fa_mean_f32_multi_ex", "fa_stripe_plan_create_ex", "fa_multi_select_layout",
                "fa_multi_plan_chunks", "fa_round_model", "fa_comm_set_profile",
                "fa_round_plan_profile", "fa_model_constants"]

FA_XCHG_REDUCE, FA_XCHG_RS_GATHER = 0, 1
FA_MODE_SHARDED, FA_MODE_STRIPED, FA_MODE_CHAINED, FA_MODE_BLOCKED = 0, 1, 2, 3
MODE_NAMES = {FA_MODE_SHARDED: "e1", FA_MODE_STRIPED: "striped", FA_MODE_CHAINED: "chained",
              FA_MODE_BLOCKED: "blocked"}
MODE_IDS = {v: k for k, v in MODE_NAMES.items()}
FA_MULTI_EXACT, FA_MULTI_REASSOCIATE, FA_MULTI_ROOT_ALL = 0, 1, 2
# the cost model's constants (fedagg_comm.h FA_MODEL_*)
MODEL_LINK_GBPS, MODEL_HBM_GBPS, MODEL_GROUP_US, MODEL_KERNEL_US = 64.0, 6500.0, 15.0, 3.0
# The e1 round's distance from the exact result, measured r04 (2 ranks x 20
# wrn16_8 clients, realistic synthetic state; bench.py N>1 'modes', file
# profiles/r04_final_bench_n2_gloo_rehearsal.json): fp32 elements per ULP bin.
E1_ULP_R04 = {"max_ulp": 22938, "histogram": {"0": 7072061, "1": 2990526, "2": 892989,
                                              "3-4": 15239, "5-8": 642, "9-16": 342,
                                              "17+": 355}}
X = dict(SEND=1, RECV=2, REDUCE=3, ALLREDUCE=4, REDUCE_SCATTER=5, GATHER=6, ALLGATHER=7, BCAST=8,
         K_SUM=16, K_ZERO=17, K_DIV=18, K_COPY=19, K_STRIPE=20, K_CHAIN=21, K_STACK=22,
         K_TAILS=23, K_PART=24, K_CONT=25, K_BLOCK=26, K_FOLD=27, K_SCALE=28)
B = dict(NONE=0, CLIENT=1, OUT=2, PARTIAL=4, RECV=5, STRIPE=6, STATE=7, FIN=8, STACK=9, GATHER=10,
         PIN=11, TAILP=12, CONT=13, BSUM=14, BLK=15, RELAY=16, WSTAGE=17)
XNAME = {v: k for k, v in X.items()}
BNAME = {v: k for k, v in B.items()}

_P, _I, _I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64


class FaXfer(ctypes.Structure):
    _fields_ = [("step", ctypes.c_int32), ("op", ctypes.c_int32), ("peer", ctypes.c_int32),
                ("chunk", ctypes.c_int32), ("src", ctypes.c_int32), ("src_index", ctypes.c_int32),
                ("dst", ctypes.c_int32), ("dst_index", ctypes.c_int32), ("offset", ctypes.c_int64),
                ("count", ctypes.c_int64), ("row0", ctypes.c_int32), ("nrows", ctypes.c_int32)]


class FaRoundCost(ctypes.Structure):
    _fields_ = [("model_us", ctypes.c_double), ("link_bytes_max", ctypes.c_double),
                ("hbm_bytes_max", ctypes.c_double), ("groups", ctypes.c_int32),
                ("steps", ctypes.c_int32)]


class FaRoundProfile(ctypes.Structure):
    _fields_ = [("exchange_us", ctypes.c_double), ("comm_kernel_us", ctypes.c_double),
                ("compute_kernel_us", ctypes.c_double), ("wall_us", ctypes.c_double),
                ("groups", ctypes.c_int32), ("kernels", ctypes.c_int32)]


class FaShardIO(ctypes.Structure):
    _fields_ = [("c32", _P), ("c64", _P), ("weights", _P), ("out32", _P), ("out64", _P),
                ("stream", _P)]


def _load():
    if not os.path.exists(COMM_PATH):
        raise ImportError(f"feddct_amd: {COMM_PATH} not built (run __graft_entry__.build()); "
                          "there is no fallback")
    lib = ctypes.CDLL(COMM_PATH)
    sig = {
        "fa_comm_unique_id": [ctypes.c_char_p, _I],
        "fa_comm_init_rank": [_I, _I, ctypes.c_char_p, _I, ctypes.POINTER(_P)],
        "fa_comm_init": [_I, ctypes.POINTER(_I), ctypes.POINTER(_P)],
        "fa_comm_destroy": [_P],
        "fa_comm_info": [_P, ctypes.POINTER(_I), ctypes.POINTER(_I), ctypes.POINTER(_I)],
        "fa_comm_set_graphs": [_P, _I],
        "fa_shard_plan_create": [_P, _P, _I, _I64, _P, _I, _I64, ctypes.POINTER(_I), _I,
                                 ctypes.c_uint, ctypes.POINTER(_P)],
        "fa_shard_plan_destroy": [_P],
        "fa_reduce_sharded": [ctypes.POINTER(_P), _I, ctypes.POINTER(FaShardIO), _I],
        "fa_mean_f32_multi": [_P, _P, ctypes.POINTER(_I), _I64, _P, _P, _I, _I, _P],
        "fa_stripe_plan_create": [_P, _P, _I, _I64, _P, _I, _I64, ctypes.POINTER(_I),
                                  ctypes.c_uint, ctypes.POINTER(_P)],
        "fa_stripe_plan_destroy": [_P],
        "fa_reduce_striped": [ctypes.POINTER(_P), _I, ctypes.POINTER(FaShardIO), _I],
        "fa_shard_plan_create_ex": [_P, _P, _I, _I64, _P, _I, _I64, ctypes.POINTER(_I), _I, _I,
                                    ctypes.c_uint, ctypes.POINTER(_P)],
        "fa_chain_plan_create": [_P, _P, _I, _I64, _P, _I, _I64, ctypes.POINTER(_I), _I,
                                 ctypes.c_uint, ctypes.POINTER(_P)],
        "fa_chain_plan_destroy": [_P],
        "fa_reduce_chained": [ctypes.POINTER(_P), _I, ctypes.POINTER(FaShardIO), _I],
        "fa_block_plan_create": [_P, _P, _I, _I64, _P, _I, _I64, ctypes.POINTER(_I),
                                 ctypes.c_uint, ctypes.POINTER(_P)],
        "fa_block_plan_destroy": [_P],
        "fa_reduce_blocked": [ctypes.POINTER(_P), _I, ctypes.POINTER(FaShardIO), _I],
        "fa_describe_round": [_I, _I, _I, ctypes.POINTER(_I), _P, _I, _I64, _P, _I, _I64, _I, _I,
                              ctypes.c_uint, _I, _I, ctypes.POINTER(FaXfer), _I,
                              ctypes.POINTER(_I)],
        "fa_multi_select": [_I, ctypes.POINTER(_I), ctypes.c_uint, ctypes.POINTER(_I)],
        "fa_multi_plan_create": [_P, _P, _I, _I64, _P, _I, _I64, ctypes.POINTER(_I), _I,
                                 ctypes.c_uint, ctypes.c_uint, ctypes.POINTER(_P)],
        "fa_multi_plan_mode": [_P, ctypes.POINTER(_I)],
        "fa_multi_plan_destroy": [_P],
        "fa_reduce_multi": [ctypes.POINTER(_P), _I, ctypes.POINTER(FaShardIO), _I],
        "fa_mean_f32_multi_ex": [_P, _P, ctypes.POINTER(_I), _I64, _P, _P, _I, _I, ctypes.c_uint,
                                 _P],
        "fa_stripe_plan_create_ex": [_P, _P, _I, _I64, _P, _I, _I64, ctypes.POINTER(_I), _I,
                                     ctypes.c_uint, ctypes.POINTER(_P)],
        "fa_multi_select_layout": [_I, ctypes.POINTER(_I), _P, _I, _I64, _P, _I, _I64,
                                   ctypes.c_uint, ctypes.c_uint, ctypes.POINTER(_I),
                                   ctypes.POINTER(_I), ctypes.POINTER(ctypes.c_double)],
        "fa_multi_plan_chunks": [_P, ctypes.POINTER(_I)],
        "fa_round_model": [_I, _I, ctypes.POINTER(_I), _P, _I, _I64, _P, _I, _I64, _I, _I,
                           ctypes.c_uint, _I, _I, ctypes.POINTER(FaRoundCost)],
        "fa_comm_set_profile": [_P, _I],
        "fa_round_plan_profile": [_P, ctypes.POINTER(FaRoundProfile)],
        "fa_model_constants": [ctypes.POINTER(ctypes.c_double)] * 4,
    }
    for name, args in sig.items():
        fn = getattr(lib, name)
        fn.restype = _I
        fn.argtypes = args
    return lib


_clib = None


def lib():
    global _clib
    if _clib is None:
        _clib = _load()
    return _clib


def _mflags(exact: bool, root_all: bool) -> int:
    return (0 if exact else FA_MULTI_REASSOCIATE) | (FA_MULTI_ROOT_ALL if root_all else 0)


def multi_select(counts: Sequence[int], exact: bool = True, layout: Optional[BucketLayout] = None,
                 root_all: bool = False, detail: bool = False):
    """The round form the default entry takes for these shard counts (host
    only): "blocked", "chained", "striped", or "e1" when ``exact=False`` —
    the exact form with the lowest modelled time (fa_multi_select_layout) on
    ``layout`` (None: fa_multi_select's nominal 2^24-float layout).
    ``root_all``: the result on every rank (FA_MULTI_ROOT_ALL) rather than on
    the last rank holding slots.  ``detail``: (form, nchunks, model_us)."""
    c = (_I * len(counts))(*map(int, counts))
    m, k, us = _I(), _I(), ctypes.c_double()
    if layout is None:
        _lib.check(lib().fa_multi_select(len(counts), c, _mflags(exact, root_all),
                                         ctypes.byref(m)), "fa_multi_select")
        return (MODE_NAMES[m.value], None, None) if detail else MODE_NAMES[m.value]
    a32, n32, a64, n64 = _segs(layout)
    _lib.check(lib().fa_multi_select_layout(len(counts), c, a32, n32, int(layout.f32_numel), a64,
                                            n64, int(layout.i64_numel),
                                            _lib.FA_PLAN_GAPS_ARE_PADDING,
                                            _mflags(exact, root_all), ctypes.byref(m),
                                            ctypes.byref(k), ctypes.byref(us)),
               "fa_multi_select_layout")
    if detail:
        return MODE_NAMES[m.value], k.value, us.value
    return MODE_NAMES[m.value]


def model_constants() -> dict:
    """The cost model's constants in effect in this process (fa_model_constants:
    the fedagg_comm.h defaults unless FA_MODEL_LINK_GBPS / FA_MODEL_HBM_GBPS /
    FA_MODEL_GROUP_US / FA_MODEL_KERNEL_US were set when the model first ran)."""
    v = [ctypes.c_double() for _ in range(4)]
    _lib.check(lib().fa_model_constants(*[ctypes.byref(x) for x in v]), "fa_model_constants")
    return dict(zip(("link_GBps", "hbm_GBps", "group_us", "kernel_us"), (x.value for x in v)))


def round_model(mode: int, layout: BucketLayout, counts: Sequence[int], nchunks: int = 0,
                exchange: int = FA_XCHG_REDUCE, root: int = 0, weighted: bool = False) -> dict:
    """The cost model's view of one round (fa_round_model, host only): the
    modelled time in microseconds, the largest byte count on one link
    direction, the largest per-rank HBM byte count, group and step counts."""
    a32, n32, a64, n64 = _segs(layout)
    c = (_I * len(counts))(*map(int, counts))
    out = FaRoundCost()
    _lib.check(lib().fa_round_model(int(mode), len(counts), c, a32, n32, int(layout.f32_numel),
                                    a64, n64, int(layout.i64_numel), int(nchunks), int(exchange),
                                    _lib.FA_PLAN_GAPS_ARE_PADDING, int(root), int(bool(weighted)),
                                    ctypes.byref(out)), "fa_round_model")
    return {f: getattr(out, f) for f, _ in FaRoundCost._fields_}


def unique_id() -> bytes:
    buf = ctypes.create_string_buffer(FA_COMM_UID_BYTES)
    _lib.check(lib().fa_comm_unique_id(buf, FA_COMM_UID_BYTES), "fa_comm_unique_id")
    return buf.raw


def _segs(layout: BucketLayout):
    a32, n32 = _lib.seg_array(layout.segs32 if len(layout.segs32) else np.zeros((0, 2), np.int64))
    a64, n64 = _lib.seg_array(layout.segs64 if len(layout.segs64) else np.zeros((0, 2), np.int64))
    return a32, n32, a64, n64


def describe(mode: int, layout: BucketLayout, counts: Sequence[int], rank: int,
             nchunks: int = 8, exchange: int = FA_XCHG_REDUCE, root: int = 0,
             weighted: bool = False) -> List[dict]:
    """Rank ``rank``'s schedule of one round (fa_describe_round): the exact
    list of exchanges and kernels the native executor issues, computed on the
    host (no GPU, no communicator)."""
    a32, n32, a64, n64 = _segs(layout)
    c = (_I * len(counts))(*map(int, counts))
    n = _I()
    args = (mode, len(counts), rank, c, a32, n32, int(layout.f32_numel), a64, n64,
            int(layout.i64_numel), int(nchunks), int(exchange), _lib.FA_PLAN_GAPS_ARE_PADDING,
            int(root), int(bool(weighted)))
    _lib.check(lib().fa_describe_round(*args, None, 0, ctypes.byref(n)), "fa_describe_round")
    arr = (FaXfer * max(1, n.value))()
    _lib.check(lib().fa_describe_round(*args, arr, n.value, ctypes.byref(n)), "fa_describe_round")
    out = []
    for i in range(n.value):
        x = arr[i]
        d = {f: getattr(x, f) for f, _ in FaXfer._fields_}
        d["op"] = XNAME.get(d["op"], d["op"])
        d["src"] = BNAME.get(d["src"], d["src"])
        d["dst"] = BNAME.get(d["dst"], d["dst"])
        out.append(d)
    return out


class Comm:
    """An RCCL communicator of the library, on the current device."""

    def __init__(self, nranks: int, rank: int, uid: bytes):
        h = _P()
        _lib.check(lib().fa_comm_init_rank(nranks, rank, uid, len(uid), ctypes.byref(h)),
                   "fa_comm_init_rank")
        self.handle = h
        self.nranks, self.rank = nranks, rank

    @classmethod
    def from_process_group(cls, group=None) -> "Comm":
        """Every rank of ``group`` (torch.distributed) joins one communicator;
        rank 0's id travels over the group."""
        import torch.distributed as dist
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        obj = [None]
        if rank == 0:
            try:
                obj = [unique_id()]
            except _lib.FedaggError as e:  # every rank must leave the broadcast
                obj = [repr(e)]
        src = 0 if group is None else dist.get_global_rank(group, 0)
        dist.broadcast_object_list(obj, src=src, group=group)
        if not isinstance(obj[0], bytes):
            raise _lib.FedaggError(f"fa_comm_unique_id failed on rank 0: {obj[0]}")
        return cls(world, rank, obj[0])

    @classmethod
    def single(cls) -> "Comm":
        """A one-rank communicator (no process group needed)."""
        return cls(1, 0, unique_id())

    def set_graphs(self, enable: bool) -> None:
        """Captured rounds on / off (fedagg_comm.h fa_comm_set_graphs; off by
        default, see there): each round's schedule replayed from a HIP graph."""
        _lib.check(lib().fa_comm_set_graphs(self.handle, int(bool(enable))),
                   "fa_comm_set_graphs")

    def set_profile(self, enable: bool) -> None:
        """Round profiles on / off (fa_comm_set_profile): every round of a plan
        of this communicator records its groups' and kernels' durations."""
        _lib.check(lib().fa_comm_set_profile(self.handle, int(bool(enable))),
                   "fa_comm_set_profile")

    def info(self):
        n, r, d = _I(), _I(), _I()
        _lib.check(lib().fa_comm_info(self.handle, ctypes.byref(n), ctypes.byref(r),
                                      ctypes.byref(d)), "fa_comm_info")
        return n.value, r.value, d.value

    def close(self):
        if getattr(self, "handle", None) is not None and self.handle.value:
            _lib.check(lib().fa_comm_destroy(self.handle), "fa_comm_destroy")
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def plan_profile(plan) -> dict:
    """The last profiled round of a plan (any of this module's plan objects;
    fa_round_plan_profile — waits for the round): exchange time (sum of its
    RCCL groups on the communication stream), kernel time on each stream,
    the round's wall time on the caller's stream, and the counts."""
    out = FaRoundProfile()
    _lib.check(lib().fa_round_plan_profile(plan.handle, ctypes.byref(out)),
               "fa_round_plan_profile")
    return {f: (round(getattr(out, f), 2) if isinstance(getattr(out, f), float)
                else getattr(out, f)) for f, _ in FaRoundProfile._fields_}


class ShardPlan:
    """This rank's shard plan for a layout (chunk subplans + scratch)."""

    def __init__(self, comm: Comm, layout: BucketLayout, counts: Sequence[int],
                 nchunks: int = 8, exchange: int = FA_XCHG_REDUCE):
        a32, n32, a64, n64 = _segs(layout)
        c = (_I * len(counts))(*map(int, counts))
        h = _P()
        _lib.check(lib().fa_shard_plan_create_ex(comm.handle, a32, n32, int(layout.f32_numel),
                                                 a64, n64, int(layout.i64_numel), c, int(nchunks),
                                                 int(exchange), _lib.FA_PLAN_GAPS_ARE_PADDING,
                                                 ctypes.byref(h)), "fa_shard_plan_create")
        self.handle = h
        self.comm = comm  # the plan must not outlive its communicator

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                lib().fa_shard_plan_destroy(h)
            except Exception:
                pass
            self.handle = None


class NativeShardedAggregator:
    """The e1 round of ``dist.ShardedAggregator`` through the C ABI (opt-in:
    RE-ASSOCIATED, not within 1 ULP of the reference — max 22,938 ULP
    measured r04, ``E1_ULP_R04``; the default entry is ``NativeAggregator``):
    ``step()`` is ONE fa_reduce_sharded call (kernels, chunked RCCL exchange,
    /N, int64 gather + exact reduce), stream-ordered on the current stream.

    ``final="reduce"``: the global state lands on ``root`` (out buffers of the
    other ranks are untouched); ``"allreduce"``: on every rank."""

    def __init__(self, layout: BucketLayout, local32: List[torch.Tensor],
                 local64: List[torch.Tensor], n_total: int, out32: torch.Tensor,
                 out64: torch.Tensor, comm: Comm, nchunks: int = 8, final: str = "reduce",
                 root: int = 0, weights: Optional[Sequence[float]] = None,
                 exchange: int = FA_XCHG_REDUCE):
        if final not in ("reduce", "allreduce"):
            raise ValueError(f"final must be 'reduce' or 'allreduce', not {final!r}")
        world, rank, _ = comm.info()
        counts = [b - a for a, b in (shard_range(n_total, world, r) for r in range(world))]
        if len(local32) != counts[rank]:
            raise ValueError(f"rank {rank} holds {len(local32)} clients, shard is {counts[rank]}")
        self.plan = ShardPlan(comm, layout, counts, nchunks, exchange)
        self.root = root if final == "reduce" else -1
        self._a32 = _lib.ptr_array([t.data_ptr() for t in local32])
        self._a64 = _lib.ptr_array([t.data_ptr() for t in local64])
        self._w = (None if weights is None
                   else (ctypes.c_float * max(1, len(weights)))(*map(float, weights)))
        self._plans = (_P * 1)(self.plan.handle.value)
        self.io = FaShardIO()
        self.io.c32 = ctypes.cast(self._a32, _P)
        self.io.c64 = ctypes.cast(self._a64, _P) if layout.i64_numel else None
        self.io.weights = ctypes.cast(self._w, _P) if self._w is not None else None
        self.io.out32 = out32.data_ptr()
        self.io.out64 = out64.data_ptr() if layout.i64_numel else None
        self._keep = (local32, local64, out32, out64)

    def step(self, stream=None) -> None:
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        self.io.stream = s
        _lib.check(lib().fa_reduce_sharded(self._plans, 1, ctypes.byref(self.io), self.root),
                   "fa_reduce_sharded")


class StripePlan:
    """This rank's exact-mode plan for a layout (its stripe's chunk plans, the
    receive rows, int64 gather buffers; nchunks 0 = 4)."""

    def __init__(self, comm: Comm, layout: BucketLayout, counts: Sequence[int],
                 nchunks: int = 0):
        a32, n32, a64, n64 = _segs(layout)
        c = (_I * len(counts))(*map(int, counts))
        h = _P()
        _lib.check(lib().fa_stripe_plan_create_ex(comm.handle, a32, n32, int(layout.f32_numel),
                                                  a64, n64, int(layout.i64_numel), c,
                                                  int(nchunks), _lib.FA_PLAN_GAPS_ARE_PADDING,
                                                  ctypes.byref(h)), "fa_stripe_plan_create")
        self.handle = h
        self.comm = comm

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                lib().fa_stripe_plan_destroy(h)
            except Exception:
                pass
            self.handle = None


class NativeStripedAggregator(NativeShardedAggregator):
    """The exact cross-GPU round (dist.StripedAggregator's device-ingress
    form) through the C ABI: ``step()`` is ONE fa_reduce_striped call; the
    result is bit-identical to one GPU reducing all clients.  r06: every
    peer in one RCCL group per column chunk (``nchunks``, 0 = 4), weighted
    rounds too (``weights``: this rank's fp32 client weights)."""

    def __init__(self, layout: BucketLayout, local32: List[torch.Tensor],
                 local64: List[torch.Tensor], n_total: int, out32: torch.Tensor,
                 out64: torch.Tensor, comm: Comm, final: str = "reduce", root: int = 0,
                 weights: Optional[Sequence[float]] = None,
                 counts: Optional[Sequence[int]] = None, nchunks: int = 0):
        if final not in ("reduce", "allreduce"):
            raise ValueError(f"final must be 'reduce' or 'allreduce', not {final!r}")
        world, rank, _ = comm.info()
        if counts is None:
            counts = [b - a for a, b in (shard_range(n_total, world, r) for r in range(world))]
        if len(local32) != counts[rank] or sum(counts) != n_total:
            raise ValueError(f"rank {rank} holds {len(local32)} clients, shard is {counts[rank]}")
        self.plan = StripePlan(comm, layout, counts, nchunks)
        self.root = root if final == "reduce" else -1
        self._a32 = _lib.ptr_array([t.data_ptr() for t in local32])
        self._a64 = _lib.ptr_array([t.data_ptr() for t in local64])
        self._w = (None if weights is None
                   else (ctypes.c_float * max(1, len(weights)))(*map(float, weights)))
        self._plans = (_P * 1)(self.plan.handle.value)
        self.io = FaShardIO()
        self.io.c32 = ctypes.cast(self._a32, _P)
        self.io.c64 = ctypes.cast(self._a64, _P) if layout.i64_numel else None
        self.io.weights = ctypes.cast(self._w, _P) if self._w is not None else None
        self.io.out32 = out32.data_ptr()
        self.io.out64 = out64.data_ptr() if layout.i64_numel else None
        self._keep = (local32, local64, out32, out64)

    def step(self, stream=None) -> None:
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        self.io.stream = s
        _lib.check(lib().fa_reduce_striped(self._plans, 1, ctypes.byref(self.io), self.root),
                   "fa_reduce_striped")


class ChainPlan:
    """This rank's chained-mode plan (vector-tile chunk plans, the state
    planes, the raw scalar-column gather buffers)."""

    def __init__(self, comm: Comm, layout: BucketLayout, counts: Sequence[int],
                 nchunks: int = 16):
        a32, n32, a64, n64 = _segs(layout)
        c = (_I * len(counts))(*map(int, counts))
        h = _P()
        _lib.check(lib().fa_chain_plan_create(comm.handle, a32, n32, int(layout.f32_numel), a64,
                                              n64, int(layout.i64_numel), c, int(nchunks),
                                              _lib.FA_PLAN_GAPS_ARE_PADDING, ctypes.byref(h)),
                   "fa_chain_plan_create")
        self.handle = h
        self.comm = comm

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                lib().fa_chain_plan_destroy(h)
            except Exception:
                pass
            self.handle = None


class NativeChainedAggregator(NativeShardedAggregator):
    """The exact client-sharded round (fa_reduce_chained): the shards stay
    where they are and the cascade state travels rank to rank in slot order
    (train_feddct.py:42-50's order over all slots).  ``final="reduce"``: the
    result lands on ``root`` (cheapest when root is the last rank holding
    clients); ``"allreduce"``: on every rank."""

    def __init__(self, layout: BucketLayout, local32: List[torch.Tensor],
                 local64: List[torch.Tensor], n_total: int, out32: torch.Tensor,
                 out64: torch.Tensor, comm: Comm, nchunks: int = 16, final: str = "reduce",
                 root: int = 0, weights: Optional[Sequence[float]] = None,
                 counts: Optional[Sequence[int]] = None):
        if final not in ("reduce", "allreduce"):
            raise ValueError(f"final must be 'reduce' or 'allreduce', not {final!r}")
        world, rank, _ = comm.info()
        if counts is None:
            counts = [b - a for a, b in (shard_range(n_total, world, r) for r in range(world))]
        if len(local32) != counts[rank] or sum(counts) != n_total:
            raise ValueError(f"rank {rank} holds {len(local32)} clients, shard is {counts[rank]}")
        self.plan = ChainPlan(comm, layout, counts, nchunks)
        self.root = root if final == "reduce" else -1
        self._a32 = _lib.ptr_array([t.data_ptr() for t in local32])
        self._a64 = _lib.ptr_array([t.data_ptr() for t in local64])
        self._w = (None if weights is None
                   else (ctypes.c_float * max(1, len(weights)))(*map(float, weights)))
        self._plans = (_P * 1)(self.plan.handle.value)
        self.io = FaShardIO()
        self.io.c32 = ctypes.cast(self._a32, _P)
        self.io.c64 = ctypes.cast(self._a64, _P) if layout.i64_numel else None
        self.io.weights = ctypes.cast(self._w, _P) if self._w is not None else None
        self.io.out32 = out32.data_ptr()
        self.io.out64 = out64.data_ptr() if layout.i64_numel else None
        self._keep = (local32, local64, out32, out64)

    def step(self, stream=None) -> None:
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        self.io.stream = s
        _lib.check(lib().fa_reduce_chained(self._plans, 1, ctypes.byref(self.io), self.root),
                   "fa_reduce_chained")


class BlockPlan:
    """This rank's blocked-mode plan (block-sum planes, the stripe it owns,
    relay rows, the raw scalar-column gather buffers)."""

    def __init__(self, comm: Comm, layout: BucketLayout, counts: Sequence[int]):
        a32, n32, a64, n64 = _segs(layout)
        c = (_I * len(counts))(*map(int, counts))
        h = _P()
        _lib.check(lib().fa_block_plan_create(comm.handle, a32, n32, int(layout.f32_numel), a64,
                                              n64, int(layout.i64_numel), c,
                                              _lib.FA_PLAN_GAPS_ARE_PADDING, ctypes.byref(h)),
                   "fa_block_plan_create")
        self.handle = h
        self.comm = comm

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                lib().fa_block_plan_destroy(h)
            except Exception:
                pass
            self.handle = None


class NativeBlockedAggregator(NativeChainedAggregator):
    """The exact client-sharded round (fa_reduce_blocked): every rank sums the
    cascade blocks it holds; a block cut by a shard boundary carries its
    level-0 partial (one plane, relayed through the column-stripe owners) to
    the next rank; the block sums go to the stripe owners, which fold them in
    block order — train_feddct.py:42-50's order over all slots, without the
    chained round's rank-to-rank pipeline.  Same arguments as the chained
    form; requires every 16-slot block to lie on at most two ranks."""

    def __init__(self, layout: BucketLayout, local32: List[torch.Tensor],
                 local64: List[torch.Tensor], n_total: int, out32: torch.Tensor,
                 out64: torch.Tensor, comm: Comm, final: str = "reduce", root: int = 0,
                 weights: Optional[Sequence[float]] = None,
                 counts: Optional[Sequence[int]] = None):
        if final not in ("reduce", "allreduce"):
            raise ValueError(f"final must be 'reduce' or 'allreduce', not {final!r}")
        world, rank, _ = comm.info()
        if counts is None:
            counts = [b - a for a, b in (shard_range(n_total, world, r) for r in range(world))]
        if len(local32) != counts[rank] or sum(counts) != n_total:
            raise ValueError(f"rank {rank} holds {len(local32)} clients, shard is {counts[rank]}")
        self.plan = BlockPlan(comm, layout, counts)
        self.root = root if final == "reduce" else -1
        self._a32 = _lib.ptr_array([t.data_ptr() for t in local32])
        self._a64 = _lib.ptr_array([t.data_ptr() for t in local64])
        self._w = (None if weights is None
                   else (ctypes.c_float * max(1, len(weights)))(*map(float, weights)))
        self._plans = (_P * 1)(self.plan.handle.value)
        self.io = FaShardIO()
        self.io.c32 = ctypes.cast(self._a32, _P)
        self.io.c64 = ctypes.cast(self._a64, _P) if layout.i64_numel else None
        self.io.weights = ctypes.cast(self._w, _P) if self._w is not None else None
        self.io.out32 = out32.data_ptr()
        self.io.out64 = out64.data_ptr() if layout.i64_numel else None
        self._keep = (local32, local64, out32, out64)

    def step(self, stream=None) -> None:
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        self.io.stream = s
        _lib.check(lib().fa_reduce_blocked(self._plans, 1, ctypes.byref(self.io), self.root),
                   "fa_reduce_blocked")


class MultiPlan:
    """This rank's plan of the default round (fa_multi_plan_create): the form
    and chunk count the cost model picks for ``counts`` on ``layout``
    (``mode``, ``nchunks`` name them); ``root_all``: the model's root is
    every rank (FA_MULTI_ROOT_ALL)."""

    def __init__(self, comm: Comm, layout: BucketLayout, counts: Sequence[int],
                 nchunks: int = 0, exact: bool = True, root_all: bool = False):
        a32, n32, a64, n64 = _segs(layout)
        c = (_I * len(counts))(*map(int, counts))
        h = _P()
        _lib.check(lib().fa_multi_plan_create(comm.handle, a32, n32, int(layout.f32_numel), a64,
                                              n64, int(layout.i64_numel), c, int(nchunks),
                                              _lib.FA_PLAN_GAPS_ARE_PADDING,
                                              _mflags(exact, root_all),
                                              ctypes.byref(h)), "fa_multi_plan_create")
        self.handle = h
        self.comm = comm
        m, k = _I(), _I()
        _lib.check(lib().fa_multi_plan_mode(h, ctypes.byref(m)), "fa_multi_plan_mode")
        _lib.check(lib().fa_multi_plan_chunks(h, ctypes.byref(k)), "fa_multi_plan_chunks")
        self.mode = MODE_NAMES[m.value]
        self.nchunks = k.value

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                lib().fa_multi_plan_destroy(h)
            except Exception:
                pass
            self.handle = None


class NativeAggregator(NativeShardedAggregator):
    """THE default multi-GPU round (fa_reduce_multi): exact — bit-identical to
    one GPU reducing all ``n_total`` slots in slot order, i.e. to the
    reference's single-process mean (train_feddct.py:42-50).  The form and
    its chunk count are the cost model's pick for the shard counts on this
    layout (``self.mode``, ``self.nchunks``): "blocked" (only where every
    16-slot cascade block lies on at most two ranks), "chained" or "striped".

    ``exact=False`` opts into the re-associated e1 round (partial sums + an
    RCCL sum, ``self.mode == "e1"``): faster on the wire but NOT within 1 ULP
    of the reference — measured r04 (2 ranks x 20 wrn16_8 clients): max
    22,938 ULP, 64.5 % of elements exact, 27.3 % off by 1 ULP, 8.1 % by 2,
    0.14 % by 3-4, 1,339 elements by 5 or more (``E1_ULP_R04``).

    ``counts``: slots per rank (default: ``shard_range``); ``final="reduce"``
    puts the result on ``root`` (default: the last rank holding slots, where
    the chained round ends), ``"allreduce"`` on every rank; ``weights``: this
    rank's fp32 client weights (weighted rounds are exact too)."""

    def __init__(self, layout: BucketLayout, local32: List[torch.Tensor],
                 local64: List[torch.Tensor], n_total: int, out32: torch.Tensor,
                 out64: torch.Tensor, comm: Comm, final: str = "reduce",
                 root: Optional[int] = None, weights: Optional[Sequence[float]] = None,
                 counts: Optional[Sequence[int]] = None, exact: bool = True, nchunks: int = 0):
        if final not in ("reduce", "allreduce"):
            raise ValueError(f"final must be 'reduce' or 'allreduce', not {final!r}")
        world, rank, _ = comm.info()
        if counts is None:
            counts = [b - a for a, b in (shard_range(n_total, world, r) for r in range(world))]
        if len(counts) != world or len(local32) != counts[rank] or sum(counts) != n_total:
            raise ValueError(f"rank {rank} holds {len(local32)} clients, shard is "
                             f"{counts[rank] if rank < len(counts) else '?'}")
        self.plan = MultiPlan(comm, layout, counts, nchunks, exact, root_all=final != "reduce")
        self.mode = self.plan.mode
        self.nchunks = self.plan.nchunks
        if root is None:
            root = max(r for r in range(world) if counts[r] > 0)
        self.root = root if final == "reduce" else -1
        self._a32 = _lib.ptr_array([t.data_ptr() for t in local32])
        self._a64 = _lib.ptr_array([t.data_ptr() for t in local64])
        self._w = (None if weights is None
                   else (ctypes.c_float * max(1, len(weights)))(*map(float, weights)))
        self._plans = (_P * 1)(self.plan.handle.value)
        self.io = FaShardIO()
        self.io.c32 = ctypes.cast(self._a32, _P)
        self.io.c64 = ctypes.cast(self._a64, _P) if layout.i64_numel else None
        self.io.weights = ctypes.cast(self._w, _P) if self._w is not None else None
        self.io.out32 = out32.data_ptr()
        self.io.out64 = out64.data_ptr() if layout.i64_numel else None
        self._keep = (local32, local64, out32, out64)

    def step(self, stream=None) -> None:
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        self.io.stream = s
        _lib.check(lib().fa_reduce_multi(self._plans, 1, ctypes.byref(self.io), self.root),
                   "fa_reduce_multi")
