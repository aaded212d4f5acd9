"""Drop-in ``server_aggregate`` on the MI355X engine.

Mirrors the reference's aggregation call surface and side effects:

* ``server_aggregate(global_model, client_models)`` —
  train_fedavg.py:138-149 (== train_fedprox.py:143-154): for every key of
  ``global_model.state_dict()`` the mean over ``client_models`` in list (slot)
  order, ``.float()`` first; loaded into ``global_model``; then every client
  reloaded from the global state.
* ``server_aggregate_split(g_a, g_b, models_a, models_b)`` —
  train_feddct.py:34-56 (== train_splitfed.py:34-56): two independent such
  reductions (main-client models, proxy models) and two broadcasts.

Results are bit-identical to the reference's CPU torch arithmetic
(oracle/torch_order.py; tests/test_gpu_parity.py).  Error behaviour follows the
reference: ``KeyError`` for a key a client lacks, ``RuntimeError`` for a shape
mismatch or an empty client list, ``RuntimeError`` from the broadcast for a
client carrying keys the global model lacks (after the global is updated).

Where the work runs: client state is bound once into flat device buckets
(arena.py) and the whole state_dict — every fp32 key, every int64 key — is
reduced by ONE launch of the HIP kernel (csrc/fedagg.hip), and the broadcast
is a second launch over the same tile table (FA_F_BCAST).  Modules living in host memory (the reference's CPU configuration)
are bound to pinned host buckets and staged through device buckets
(host-inclusive path).  There is no CPU arithmetic fallback.
"""
from __future__ import annotations

import ctypes
import warnings
import weakref
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from array import array

from . import _lib, slab
from . import arena as _arena
from .arena import ModuleArena, get_arena
from .layout import BucketLayout

__all__ = ["server_aggregate", "server_aggregate_split", "aggregate_weighted", "client_weights",
           "Engine", "engine", "set_summation_order", "summation_order"]

ORDERS = {"torch_cpu": 0, "torch_gpu": 1}


def _require_gpu():
    if not torch.cuda.is_available():
        raise RuntimeError("feddct_amd: no HIP device visible; the aggregation engine has "
                           "no CPU fallback")


# Up to this many client tensors the bound round checks every one before the
# reduce is launched (r06: ~1 ns each while they stay in cache — cfg2's 2,058
# in 2.3 us); beyond it, before the launch, the use count of each client
# bucket's storage, and the tensors while the GPU reduces (cfg5's 9,800: 16 us
# that would otherwise precede the launch; shim.cpp bound_round).
BOUND_PRECHECK_MAX = 4096


class _RoundBinding:
    """The last device-resident round's bound state (r04 fast path): the
    global and client modules, their arenas, plan, pointer arrays, and ONE
    flattened validity check over every bound tensor.  A repeat call on the
    same modules re-checks only (a) that no module anywhere registered a
    parameter, buffer or submodule, and no arena was (re)bound, since
    (arena._STRUCT_GEN), (b) that the caller passed the very objects bound
    (one C call by identity, _fa_shim.src_match), and (c) in one C call
    (_fa_shim.valid_tagged, or inside _fa_shim.bound_round): every
    parameter/buffer dict's PEP 509 version tag — unchanged tag, unchanged
    slots — and every bound tensor's data pointer (a `.data` swap).
    Anything else takes the full path, which re-binds what changed and
    records a new binding."""

    __slots__ = ("gref", "crefs", "arenas", "gen", "dicts", "tags", "tensors", "ptrs",
                 "written", "packed", "plan", "a32", "a64", "n", "dev", "order", "weighted",
                 "native", "src_ids", "split_ids", "ng", "__weakref__")

    def __init__(self, engine, global_model, client_models, ga, cas, plan, a32, a64, order,
                 weighted):
        from . import _fa_shim
        # modules and arenas held weakly: the binding must not keep a dropped
        # round's modules or buckets alive; when any of them goes, so does
        # the binding (its tensor tuples hold the bound parameters)
        eng, me = weakref.ref(engine), weakref.ref(self)

        def dropped(_r):
            e = eng()
            if e is not None and me() is not None and e._round is me():
                e._round = None
        self.gref = weakref.ref(global_model, dropped)
        self.crefs = tuple(weakref.ref(m, dropped) for m in client_models)
        arenas = (ga, *cas)
        self.arenas = tuple(weakref.ref(a, dropped) for a in arenas)
        self.gen = _arena._STRUCT_GEN[0]
        dicts, seen = [], set()
        tensors, ptrs = [], array("Q")
        ng = None
        for i, a in enumerate(arenas):
            if i == 1:   # the global's own checks are the first ones
                ng = (len(dicts), len(tensors))
            for d, _, t, p in a._checks:
                if id(d) not in seen:
                    seen.add(id(d))
                    dicts.append(d)
                tensors.append(t)
                ptrs.append(p)
            for d, _, _, _ in a._packed:
                if id(d) not in seen:
                    seen.add(id(d))
                    dicts.append(d)
        self.ng = ng if ng is not None else (len(dicts), len(tensors))
        self.dicts = tuple(dicts)
        self.tags = _fa_shim.dict_tags(self.dicts)   # None: no tags (CPython >= 3.12)
        self.tensors = tuple(tensors)
        self.ptrs = ptrs.tobytes()
        self.written = tuple(t for a in arenas for t in a._written)
        self.packed = tuple(i for i, a in enumerate(arenas) if a._packed)
        self.plan, self.a32, self.a64 = plan, a32, a64
        self.n = len(cas)
        self.dev = cas[0].device
        self.order = order
        self.weighted = weighted
        # the objects the caller passed, by id (_fa_shim.src_match): alive as
        # long as this binding (the weakref callbacks above end it first);
        # split_ids: the two-model call's objects (server_aggregate_split)
        self.src_ids = array("Q", [id(global_model)] + [id(m) for m in client_models]).tobytes()
        self.split_ids = None
        # the whole repeat round in one C call (_fa_shim.bound_round) when no
        # arena packs (a packed arena copies in and out around the launches)
        self.native = None
        if not self.packed and self.tags is not None:
            self.native = _fa_shim.round_state(
                ctypes.cast(_lib.lib.fa_reduce, ctypes.c_void_p).value, plan.handle.value,
                ctypes.addressof(a32), ctypes.addressof(a64), self.n, ga.f32.data_ptr(),
                ga.i64.data_ptr(), self.dev.index, self.dicts, self.tags, self.tensors,
                self.ptrs, self.written, self.ng[0], self.ng[1], BOUND_PRECHECK_MAX)

    def current(self, order, weighted) -> bool:
        """Same order and weighting, and no tensor/module registration — and
        no arena (re)binding, which bumps the same counter (arena.get_arena)
        — anywhere since the binding."""
        return (self.tags is not None and self.order == order and self.weighted == weighted
                and _arena._STRUCT_GEN[0] == self.gen)

    def same_modules(self, global_model, client_models, order, weighted) -> bool:
        """The cheap half of the check: current(), and the very modules the
        round was bound with (one C call, by identity)."""
        from . import _fa_shim
        if not self.current(order, weighted):
            return False
        if not isinstance(client_models, (list, tuple)):
            client_models = list(client_models)
        return _fa_shim.src_match(self.src_ids, global_model, client_models)

    def views_intact(self) -> bool:
        """The per-tensor half (one C call): every parameter/buffer dict's
        version tag and every bound tensor's data pointer unchanged."""
        from . import _fa_shim
        return _fa_shim.valid_tagged(self.dicts, self.tags, self.tensors, self.ptrs)

    def global_intact(self) -> bool:
        """The global model's own share of views_intact (checked BEFORE the
        reduce, which writes the global's bound bucket)."""
        from . import _fa_shim
        return _fa_shim.valid_tagged(self.dicts, self.tags, self.tensors, self.ptrs,
                                     0, self.ng[0], 0, self.ng[1])

    def clients_intact(self) -> bool:
        """The clients' share of views_intact (checked while the GPU reduces)."""
        from . import _fa_shim
        return _fa_shim.valid_tagged(self.dicts, self.tags, self.tensors, self.ptrs,
                                     self.ng[0], len(self.dicts), self.ng[1], len(self.tensors))

    def matches(self, global_model, client_models, order, weighted) -> bool:
        return (self.same_modules(global_model, client_models, order, weighted)
                and self.views_intact())


class Engine:
    """Plan/staging caches for one process (one GPU per process)."""

    def __init__(self):
        # the summation order device-resident rounds reproduce: torch's CPU
        # order (default), or torch-ROCm's GPU one (set_summation_order)
        self.order = "torch_cpu"
        self._plans: Dict[tuple, _lib.Plan] = {}
        # torch-GPU-order plans are cut per client count: a small LRU, so a
        # loop whose participation varies does not grow device plans forever
        self._gpu_plans: "OrderedDict[tuple, Optional[_lib.Plan]]" = OrderedDict()
        # rounds the torch-GPU order could not restate, per (layout, N): a
        # warning for each new pair, and a count callers can query
        # (gpu_order_fallbacks) — ADVICE r03: warning once per Engine hid
        # every later layout / N from a caller who set the order for parity
        self.gpu_order_fallbacks: Dict[tuple, int] = {}
        self.strict_gpu_order = False
        self._fallback_round = False
        self._layouts: Dict[tuple, BucketLayout] = {}
        self._pipes: Dict[tuple, object] = {}
        self._round: Optional[_RoundBinding] = None

    # ------------------------------------------------------------ caches --
    GPU_PLAN_CACHE = 8

    def plan(self, layout: BucketLayout, device: torch.device, n: int = 0,
             order: str = "torch_cpu") -> Optional[_lib.Plan]:
        """The layout's plan on ``device``.  For the torch-GPU order, the
        plan cut for ``n`` clients, or None when torch itself would split
        some key across blocks there (outside the restated configurations,
        fa_torch_gpu_config)."""
        if order == "torch_gpu":
            key = (layout.signature, device.index, n)
            if key in self._gpu_plans:
                self._gpu_plans.move_to_end(key)
                return self._gpu_plans[key]
            try:
                with torch.cuda.device(device):
                    p = _lib.Plan(layout.segs32, layout.f32_numel, layout.segs64,
                                  layout.i64_numel, order=_lib.FA_ORDER_TORCH_GPU, n=n)
            except _lib.FedaggError as e:
                if "outside the restated" not in str(e):
                    raise
                p = None
            self._gpu_plans[key] = p
            while len(self._gpu_plans) > self.GPU_PLAN_CACHE:
                self._gpu_plans.popitem(last=False)
            return p
        key = (layout.signature, device.index)
        p = self._plans.get(key)
        if p is None:
            with torch.cuda.device(device):
                p = _lib.Plan(layout.segs32, layout.f32_numel, layout.segs64,
                              layout.i64_numel)
            self._plans[key] = p
        return p

    def layout_of(self, module: torch.nn.Module) -> BucketLayout:
        a = getattr(module, "_fa_arena", None)
        if a is not None and a.valid() and len(a.extra_keys) == 0:
            return a.layout
        lay = BucketLayout.from_state_dict(module.state_dict())
        # share one layout object per signature so plans/staging are reused
        return self._layouts.setdefault(lay.signature, lay)

    # ------------------------------------------------------------- core --
    def try_bound_round(self, global_model: torch.nn.Module,
                        client_models: Sequence[torch.nn.Module],
                        weights: Optional[Sequence[float]] = None) -> bool:
        """The repeat call's fast path (r04): when these exact modules made
        the last device-resident round (_RoundBinding.same_modules), the
        per-tensor check (_RoundBinding.views_intact: every dict's tag, every
        bound tensor's storage) runs, then the reduce and the broadcast are
        launched and the version counters bumped while the GPU works.  A
        failed check has launched nothing: False, and the caller takes the
        full path (re-bind, whole round), which raises where the reference
        raises (a client whose parameter was replaced by one of another
        shape) with the global untouched, as the reference leaves it
        (train_fedavg.py:144-147).  Until r05 the clients' share of the check
        ran while the GPU reduced into the global's bucket, so that raise
        left the global holding the mean of the clients' stale buckets
        (VERDICT r05 next 2).  r06: the native check reads cached TensorImpl
        fields (shim.cpp ViewKey) instead of unpacking every Python tensor."""
        rb = self._round
        if rb is None or not rb.same_modules(global_model, client_models, self.order,
                                             weights is not None):
            return False
        return self._run_bound(rb, weights)

    def _run_bound(self, rb: _RoundBinding, weights=None) -> bool:
        """The bound round, its modules already matched (try_bound_round).
        The global model's own dicts and tensors are checked first (the
        reduce writes the global's bound bucket: r05), then the clients'
        (r06), all before anything is launched."""
        if rb.native is not None:
            from . import _fa_shim
            w = None
            if weights is not None:
                w = np.asarray(weights, np.float32).reshape(-1)
                if w.shape[0] != rb.n:
                    raise ValueError(f"{w.shape[0]} weights for {rb.n} clients")
                w = w.tobytes()
            r = _fa_shim.bound_round(rb.native, w)
            if r == 1:
                return True
            if r in (0, 3):
                self._round = None
            elif r < 0:
                _lib.check(r, "fa_reduce")
            return False
        if torch.cuda.current_device() != rb.dev.index:
            return False
        if not rb.global_intact() or not rb.clients_intact():
            self._round = None
            return False
        arenas = [r() for r in rb.arenas]
        for i in rb.packed:
            arenas[i].pack()
        ga = arenas[0]
        stream = ctypes.c_void_p(torch.cuda.current_stream(rb.dev).cuda_stream)
        o32, o64 = ga.f32.data_ptr(), ga.i64.data_ptr()
        fa_reduce = _lib.lib.fa_reduce
        _lib.check(fa_reduce(rb.plan.handle, rb.a32, rb.a64, rb.n,
                             self._weights_arg(weights, rb.n), o32, o64, 0, stream), "fa_reduce")
        _lib.check(fa_reduce(rb.plan.handle, rb.a32, rb.a64, rb.n, None, o32, o64,
                             _lib.FA_F_BCAST_ONLY, stream), "fa_reduce")
        if rb.packed:
            ga.unpack()
            for c in arenas[1:]:
                c.unpack(ga)
        from . import _fa_shim
        _fa_shim.bump_versions(rb.written)
        return True

    def reduce_modules(self, global_model: torch.nn.Module,
                       client_models: Sequence[torch.nn.Module],
                       weights: Optional[Sequence[float]] = None,
                       broadcast: bool = True) -> None:
        if broadcast and self.try_bound_round(global_model, client_models, weights):
            return
        n = len(client_models)
        if n == 0:
            raise RuntimeError("stack expects a non-empty TensorList")
        _require_gpu()
        layout = self.layout_of(global_model)
        with slab.expecting(n + 1):   # a new slab sized for this round's buckets
            ga = get_arena(global_model, layout)
            cas = [get_arena(c, layout) for c in client_models]
        # torch.stack (train_fedavg.py:145) needs the clients on one device;
        # the global may live elsewhere (load_state_dict at :147 copies across)
        dev = cas[0].device
        for c in cas:
            if c.device != dev:
                raise RuntimeError(
                    "Expected all tensors to be on the same device, but found at least two "
                    f"devices, {dev} and {c.device}!")
        # A client with keys the global lacks makes the reference's broadcast
        # raise (train_fedavg.py:149): reduce, load the global, broadcast in
        # order up to that client, then raise the same way.
        bad = next((i for i, c in enumerate(cas) if c.extra_keys), None)
        fuse_bcast = broadcast and bad is None
        for c in cas:
            c.pack()
        if dev.type == "cuda":
            if ga.device == dev:
                self._fallback_round = False
                plan = self._reduce_device(layout, ga.f32, ga.i64, cas, weights, fuse_bcast)
                # (a round the torch-GPU order could not restate is never bound:
                # each such call takes this path, is counted and can be refused)
                if fuse_bcast and _arena._fa_shim is not None and not self._fallback_round:
                    a32, a64 = self._ptr_arrays(cas)
                    self._round = _RoundBinding(self, global_model, client_models, ga, cas,
                                                plan, a32, a64, self.order, weights is not None)
            else:
                o32, o64 = self._stage(layout, dev)
                self._reduce_device(layout, o32, o64, cas, weights, fuse_bcast)
                ga.f32.copy_(o32)
                ga.i64.copy_(o64)
        else:
            self._reduce_host(layout, ga, cas, weights, fuse_bcast)
        ga.unpack()
        ga.mark_written()
        if broadcast and not fuse_bcast:
            for i, c in enumerate(cas):
                if i == bad:
                    raise RuntimeError(
                        f"Error(s) in loading state_dict for {type(client_models[i]).__name__}:"
                        "\n\tMissing key(s) in state_dict: "
                        + ", ".join(f'"{k}"' for k in c.extra_keys) + ". ")
                c.f32.copy_(ga.f32)
                c.i64.copy_(ga.i64)
                c.unpack(ga)
                c.mark_written()
        elif fuse_bcast:
            for c in cas:
                c.unpack(ga)
                c.mark_written()

    def _weights_arg(self, weights, n):
        if weights is None:
            return None
        w = np.asarray(weights, np.float32).reshape(-1)
        if w.shape[0] != n:
            raise ValueError(f"{w.shape[0]} weights for {n} clients")
        return (ctypes.c_float * n)(*[float(x) for x in w])

    def _launch(self, plan, a32, a64, n, weights, out32, out64, flags, device):
        stream = torch.cuda.current_stream(device).cuda_stream
        if torch.cuda.current_device() == device.index:
            _lib.check(_lib.lib.fa_reduce(plan.handle, a32, a64, n, weights, out32, out64,
                                          flags, ctypes.c_void_p(stream)), "fa_reduce")
            return
        with torch.cuda.device(device):
            _lib.check(_lib.lib.fa_reduce(plan.handle, a32, a64, n, weights, out32, out64,
                                          flags, ctypes.c_void_p(stream)), "fa_reduce")

    def _ptr_arrays(self, cas: List[ModuleArena]):
        """Client bucket pointer arrays, kept for the last client list (the
        round loop passes the same slots every round; arenas never move)."""
        key = tuple(map(id, cas))
        hit = getattr(self, "_last_ptrs", None)
        # weak references: the cache must not keep a dropped round's buckets alive
        if hit is not None and hit[0] == key and all(r() is c for r, c in zip(hit[1], cas)):
            return hit[2], hit[3]
        a32 = _lib.ptr_array([c.ptr32 for c in cas])
        a64 = _lib.ptr_array([c.ptr64 for c in cas])
        self._last_ptrs = (key, tuple(weakref.ref(c) for c in cas), a32, a64)
        return a32, a64

    def _stage(self, layout, device: torch.device):
        """Result buckets on the clients' device for a global model that
        lives on another device (cached per layout and device)."""
        key = ("stage", layout.signature, device.index)
        st = self._pipes.get(key)
        if st is None:
            from .arena import alloc_buckets
            st = self._pipes[key] = alloc_buckets(layout, device)
        return st

    def _reduce_device(self, layout, out32: torch.Tensor, out64: torch.Tensor,
                       cas: List[ModuleArena], weights, fuse):
        n = len(cas)
        dev = cas[0].device
        order = self.order
        if order == "torch_gpu" and (weights is not None or n < 2):
            order = "torch_cpu"   # (the GPU order is torch's unweighted mean, N >= 2)
        plan = self.plan(layout, dev, n, order)
        if plan is None:   # torch would split a key across blocks at this N
            msg = (f"feddct_amd: torch-GPU summation order is not restated for N={n} on "
                   f"this layout (torch splits a key across blocks)")
            if self.strict_gpu_order:
                raise RuntimeError(msg + "; strict mode (set_summation_order(..., strict=True))")
            key = (layout.signature, n)
            seen = self.gpu_order_fallbacks.get(key, 0)
            self.gpu_order_fallbacks[key] = seen + 1
            if seen == 0:
                warnings.warn(msg + "; rounds of this layout at this N use torch's CPU order",
                              RuntimeWarning, stacklevel=3)
            plan = self.plan(layout, dev, n, "torch_cpu")
            self._fallback_round = True
        flags = _lib.FA_F_BCAST if fuse else 0
        a32, a64 = self._ptr_arrays(cas)
        self._launch(plan, a32, a64, n, self._weights_arg(weights, n), out32.data_ptr(),
                     out64.data_ptr(), flags, dev)
        return plan

    def _reduce_host(self, layout, ga: ModuleArena, cas: List[ModuleArena], weights, fuse):
        """Host-resident state (the reference's CPU configuration): the
        chunked H2D / reduce / D2H pipeline (pipeline.py) over the modules'
        pinned arenas; the broadcast fans each downloaded chunk out to the
        clients' host buckets on the CPU while later chunks upload."""
        from .pipeline import HostPipeline
        n = len(cas)
        dev = (ga.device if ga.device.type == "cuda"
               else torch.device("cuda", torch.cuda.current_device()))
        key = (layout.signature, dev.index, n)
        pipe = self._pipes.get(key)
        if pipe is None:
            pipe = self._pipes[key] = HostPipeline(layout, n, dev)
        bc32 = [c.f32 for c in cas] if fuse else []
        bc64 = [c.i64 for c in cas] if fuse else []
        pipe.run([c.f32 for c in cas], [c.i64 for c in cas], ga.f32, ga.i64, bc32, bc64,
                 weights=None if weights is None else np.asarray(weights, np.float32))


_ENGINE: Optional[Engine] = None


def engine() -> Engine:
    global _ENGINE
    if _ENGINE is None:
        _ENGINE = Engine()
    return _ENGINE


def server_aggregate(global_model, client_models):
    """train_fedavg.py:138-149 / train_fedprox.py:143-154, on the MI355X engine."""
    engine().reduce_modules(global_model, list(client_models))


class _Pair(torch.nn.Module):
    """A FedDCT client slot as one module: (main client, proxy) under the
    keys "0." and "1.".  Binding a pair puts both halves' state in ONE bucket,
    so a round is one reduce launch (+ its broadcast launch); the per-key
    arithmetic is unchanged.  Each half's tensors still sit in a storage
    object of their own (arena._part_bases), so saving one model's
    state_dict writes only that model's bytes."""

    _fa_storage_parts = ("0.", "1.")

    def __init__(self, a, b):
        super().__init__()
        self.add_module("0", a)
        self.add_module("1", b)


def _pair(a, b) -> "_Pair":
    """The cached pair wrapper of (a, b), kept on ``a`` (a reference cycle the
    GC collects with the modules, no global registry)."""
    cache = a.__dict__.setdefault("_fa_pairs", {})
    p = cache.get(id(b))
    if p is None or p._modules["1"] is not b:
        p = cache[id(b)] = _Pair(a, b)
    return p


def server_aggregate_split(global_model_a, global_model_b, models_a, models_b):
    """train_feddct.py:34-56 / train_splitfed.py:34-56: main-client and proxy
    (or client and server) halves reduced and broadcast independently.

    When every slot has both halves, each slot's pair is bound to one bucket
    and both reductions run as ONE launch, both broadcasts as one more.  Anything the
    joint path would report differently from the reference (a missing or
    mismatched key, extra keys) takes the two-call path, which reproduces the
    reference's errors and their order exactly."""
    e = engine()
    models_a, models_b = list(models_a), list(models_b)
    # the repeat call's fast path: the very objects of the last joint round
    # (no pair lookups: 25 of them cost cfg5's call ~10 us of host time)
    rb = e._round
    if (rb is not None and rb.split_ids is not None and rb.current(e.order, False)
            and _arena._fa_shim.src_match(rb.split_ids, global_model_a, global_model_b,
                                          models_a, models_b)
            and e._run_bound(rb)):
        return
    if len(models_a) == len(models_b) and len(models_a) > 0:
        try:
            g = _pair(global_model_a, global_model_b)
            pairs = [_pair(a, b) for a, b in zip(models_a, models_b)]
            # a bound round exists only for pairs without extra keys
            if e.try_bound_round(g, pairs):
                return
            layout = e.layout_of(g)
            arenas = [get_arena(p, layout) for p in pairs]
            if not any(a.extra_keys for a in arenas):
                e.reduce_modules(g, pairs)
                rb = e._round
                if rb is not None and rb.gref() is g:
                    rb.split_ids = array("Q", [id(global_model_a), id(global_model_b)]
                                         + [id(m) for m in models_a]
                                         + [id(m) for m in models_b]).tobytes()
                return
        except (KeyError, RuntimeError, TypeError):
            pass  # fall through: the reference's own two-step semantics
    e.reduce_modules(global_model_a, models_a)
    e.reduce_modules(global_model_b, models_b)


def client_weights(sizes) -> np.ndarray:
    """FedAvg client weights w_i = fp32(n_i / Σn) (float64 ratio, one rounding)."""
    s = np.asarray(sizes, np.float64)
    return (s / s.sum()).astype(np.float32)


def aggregate_weighted(global_model, client_models, weights=None, sizes=None,
                       broadcast=True):
    """Client-size-weighted FedAvg (SURVEY.md §8 a9 — an extension: the
    reference is unweighted).  ``weights`` are fp32 w_i, or ``sizes`` n_i give
    w_i = fp32(n_i / Σn).  fp32 keys: Σ_i fp32(x_i·w_i) in the torch order;
    int64 keys keep the reference mean.  Equal weights dispatch to the mean
    path, because x·(1/N) is not bit-equal to x/N."""
    if weights is None and sizes is None:
        raise ValueError("give weights or sizes")
    if weights is None:
        weights = client_weights(sizes)
    w = np.asarray(weights, np.float32)
    if np.all(w == w[0]):
        engine().reduce_modules(global_model, list(client_models), None, broadcast)
    else:
        engine().reduce_modules(global_model, list(client_models), w, broadcast)


def set_summation_order(order: str, strict: bool = False) -> None:
    """Which torch order device-resident rounds reproduce bit for bit:
    ``"torch_cpu"`` (default: torch's CPU stack(...).mean(0), the reference's
    BASELINE config 1 and its device-independent definition) or
    ``"torch_gpu"`` (torch-ROCm's GPU reduction on THIS device: what the
    unchanged reference script computes when its models sit on this MI355X,
    train_fedavg.py:244-250 — restated from the torch-ROCm 2.x headers and
    pinned against torch's own `cuda` mean on this GPU.  It is NOT the order
    of the reference's published runs, which ran torch 1.10/1.11 on NVIDIA
    GPUs with another block configuration; parity with those runs is
    unpinned.  Unweighted rounds of N >= 2 clients; a round torch would
    split across thread blocks takes the CPU order, with a RuntimeWarning
    for each new (layout, N) and a count in ``engine().gpu_order_fallbacks``
    — or, with ``strict=True``, raises instead.  See INTEGRATION.md).
    Host-resident modules always take the CPU order, which is what the
    reference computes for them."""
    if order not in ORDERS:
        raise ValueError(f"order must be one of {sorted(ORDERS)}, not {order!r}")
    engine().order = order
    engine().strict_gpu_order = bool(strict)


def summation_order() -> str:
    return engine().order
