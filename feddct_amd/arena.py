"""Persistent flat parameter storage.

``ModuleArena`` re-points every parameter and persistent buffer of an
``nn.Module`` at a view of one flat fp32 bucket (+ one int64 bucket), laid
out by a ``BucketLayout``.  After binding, ``module.state_dict()`` returns
views into the buckets, so the aggregation kernel reads the clients' live
weights and writes the global (and, fused, the broadcast) in place: no
per-round packing, no ``state_dict()`` rebuilds (the K·N rebuilds are what
dominates the reference's time).

Parameter *objects* are kept (only ``.data`` is swapped), so optimizers that
hold them keep working.  ``valid()`` detects a module whose tensors were
replaced since binding (``model.to(...)``, new ``nn.Parameter``), in which
case the shim re-binds.  This is the MI355X-native analogue of the
reference's (unused) flatten helpers get_flat_params_from /
set_flat_params_to (fedml_api/distributed/fedgkt/utils.py:17-32).
"""
from __future__ import annotations

from typing import Dict, List, Tuple

from array import array

import torch
from torch.autograd.graph import increment_version

from . import slab
from .layout import KIND_I64, KIND_PACKF, BucketLayout

# The per-call checks and version bumps in C (csrc/shim.cpp, built by
# build.py); the Python loops below define the same semantics and run when
# the helper is absent (tests compare the two).
try:
    from . import _fa_shim
except ImportError:  # not built
    _fa_shim = None


# Structure generation: bumped by torch's global registration hooks whenever
# any module registers a parameter, buffer or submodule.  An arena re-checks
# its module's key set only when this moved since it last looked, so the
# per-call validity check stays O(tensors) with no module-tree walk.
_STRUCT_GEN = [0]


def _bump(*_args, **_kw):
    _STRUCT_GEN[0] += 1


torch.nn.modules.module.register_module_parameter_registration_hook(_bump)
torch.nn.modules.module.register_module_buffer_registration_hook(_bump)
torch.nn.modules.module.register_module_module_registration_hook(_bump)


def state_owners(module: torch.nn.Module) -> Dict[str, Tuple[dict, str]]:
    """state_dict key → (the dict holding the tensor, name), in state_dict
    registration order (parameters then persistent buffers per module)."""
    out = {}
    for prefix, m in module.named_modules(remove_duplicate=False):
        pre = prefix + "." if prefix else ""
        for n, p in m._parameters.items():
            if p is not None:
                out[pre + n] = (m._parameters, n)
        for n, b in m._buffers.items():
            if b is not None and n not in m._non_persistent_buffers_set:
                out[pre + n] = (m._buffers, n)
    return out


def alloc_buckets(layout: BucketLayout, device: torch.device, pinned: bool = False):
    """A zeroed (fp32, int64) bucket pair.  On a GPU the fp32 bucket is
    carved from a shared slab (slab.py: one allocation under many buckets
    reads ~8 % faster than as many separate allocations on some boxes); it
    is still a storage of its own, so torch.save of the module writes only
    its bytes."""
    device = torch.device(device)
    if device.type == "cpu":
        kw = dict(pin_memory=True) if pinned and torch.cuda.is_available() else {}
        return (torch.zeros(max(layout.f32_numel, 64), dtype=torch.float32, **kw),
                torch.zeros(max(layout.i64_numel, 1), dtype=torch.int64, **kw))
    f32 = slab.carve(max(layout.f32_numel, 64), torch.float32, device)
    i64 = torch.zeros(max(layout.i64_numel, 1), dtype=torch.int64, device=device)
    return f32, i64


class ModuleArena:
    """A module whose state lives in flat buckets laid out by ``layout``."""

    def __init__(self, module: torch.nn.Module, layout: BucketLayout,
                 pinned: bool = True):
        owners = state_owners(module)
        tensors = {k: owners[k][0][owners[k][1]] for k in owners}
        missing = [k for k in layout.keys if k not in tensors]
        if missing:
            raise KeyError(missing[0])
        devs = {t.device for t in tensors.values()}
        if len(devs) != 1:
            raise RuntimeError(f"module state spans several devices: {sorted(map(str, devs))}")
        self.device = devs.pop()
        self.layout = layout
        for s in layout.slots:
            t = tensors[s.key]
            if tuple(t.shape) != s.shape:
                # what torch.stack raises on the reference path (train_fedavg.py:145)
                raise RuntimeError(
                    f"stack expects each tensor to be equal size, but got {list(s.shape)} "
                    f"(global) and {list(t.shape)} for key {s.key!r}")
            if t.dtype != s.dtype and (t.dtype.is_complex or (
                    s.kind == KIND_I64 and t.dtype.is_floating_point)):
                # a float value in an integer key: .float() keeps its fraction,
                # the int64 bucket cannot (the reference's .float() at
                # train_fedavg.py:145 takes every other dtype, see _packed)
                raise TypeError(
                    f"state_dict key {s.key!r}: module dtype {t.dtype} cannot be staged in "
                    f"the global model's {s.dtype} slot")
            if s.alias_of is not None:
                a = tensors[s.alias_of]
                if (t.data_ptr() != a.data_ptr() or t.stride() != a.stride()
                        or t.dtype != a.dtype):
                    # the layout says this key shares the other's storage (tied
                    # weights in the global model); binding an untied module
                    # to it would silently tie its parameters
                    raise RuntimeError(
                        f"state_dict key {s.key!r} is tied to {s.alias_of!r} in the global "
                        "model but not in this module")
        # keys the module has beyond the layout: the reference's broadcast
        # load_state_dict(strict=True) rejects such a client (train_fedavg.py:149)
        self.extra_keys = [k for k in tensors if k not in layout.by_key]
        self._keyset = list(tensors.keys())
        self._gen = _STRUCT_GEN[0]
        self.f32, self.i64 = alloc_buckets(layout, self.device, pinned)
        bases = _part_bases(layout, self.f32, self.i64,
                            getattr(module, "_fa_storage_parts", None))
        self._checks: List[tuple] = []
        self._packed: List[tuple] = []
        self._packed_keys: List[str] = []
        self._via_global = set()
        with torch.no_grad():
            for s in layout.slots:
                d, name = owners[s.key]
                t = d[name]
                bucket = self.i64 if s.kind == KIND_I64 else self.f32
                if s.kind == KIND_PACKF or t.dtype != s.dtype:
                    # staged per call: the key's own dtype differs from its
                    # bucket's (a packed dtype, or a client whose dtype differs
                    # from the global's — the reference's .float() takes both)
                    self._packed.append((d, name, t, bucket[s.offset:s.offset + s.numel]
                                         .view(s.shape)))
                    self._packed_keys.append(s.key)
                    if s.kind == KIND_PACKF and t.dtype != s.dtype:
                        # the reference broadcasts the global's value in the
                        # global's dtype (train_fedavg.py:148-149): this key
                        # gets C(G(mean)), not C(mean)
                        self._via_global.add(s.key)
                    continue
                view = bucket[s.offset:s.offset + s.numel].view(s.shape)
                part = bases.get((s.kind == KIND_I64, _part_of(s.key, bases)))
                if part is not None:
                    # same memory, seen through the part's own storage object
                    pb, plo = part
                    view = pb[s.offset - plo:s.offset - plo + s.numel].view(s.shape)
                if s.alias_of is None:
                    view.copy_(t)
                t.data = view
                self._checks.append((d, name, t, view.data_ptr()))
        self.module_ref = module
        # tensors the kernel writes behind autograd's back (raw pointers)
        self._written = tuple(t for _, _, t, _ in self._checks)
        self._v_dicts = tuple(d for d, _, _, _ in self._checks)
        self._v_names = tuple(n for _, n, _, _ in self._checks)
        self._v_ptrs = array("Q", [p for _, _, _, p in self._checks]).tobytes()

    def mark_written(self) -> None:
        """Bump the autograd version counter of every bucket-backed tensor,
        as the reference's ``load_state_dict`` (an in-place ``copy_``) does:
        a graph that saved the old values then fails loudly in backward
        instead of using the overwritten ones."""
        if _fa_shim is not None:
            _fa_shim.bump_versions(self._written)
        else:
            increment_version(self._written)

    def valid(self, use_shim: bool = True) -> bool:
        if self._gen != _STRUCT_GEN[0]:
            # something somewhere registered a tensor/module: is it ours?
            m = self.module_ref
            if list(state_owners(m).keys()) != self._keyset:
                return False
            self._gen = _STRUCT_GEN[0]
        if use_shim and _fa_shim is not None:
            if not _fa_shim.valid_views(self._v_dicts, self._v_names, self._written,
                                        self._v_ptrs):
                return False
        else:
            for d, name, t, ptr in self._checks:
                if d.get(name) is not t or t.data_ptr() != ptr:
                    return False
        for d, name, t, _ in self._packed:
            if d.get(name) is not t:
                return False
        return True

    # -- keys stored in another dtype: staged through the f32 bucket -------
    def pack(self) -> None:
        """``.float()`` every staged key into its bucket slot (fp32 slots; an
        integer key into an int64 slot, which is exact)."""
        if not self._packed:
            return
        with torch.no_grad():
            for _, _, t, view in self._packed:
                view.copy_(t)

    def unpack(self, glob: "ModuleArena" = None) -> None:
        """``copy_`` the slot back into the key's own dtype (the
        load_state_dict semantics of train_fedavg.py:147).  ``glob``: the
        global model's arena, already unpacked, for a broadcast target whose
        key dtype differs from the global's packed dtype."""
        if not self._packed:
            return
        with torch.no_grad():
            for key, (_, _, t, view) in zip(self._packed_keys, self._packed):
                if glob is not None and key in self._via_global:
                    t.copy_(glob.staged(key))
                else:
                    t.copy_(view)

    def staged(self, key: str) -> torch.Tensor:
        """The module's own tensor of a staged key."""
        return self._packed[self._packed_keys.index(key)][2]

    @property
    def ptr32(self) -> int:
        return self.f32.data_ptr()

    @property
    def ptr64(self) -> int:
        return self.i64.data_ptr()


def _part_of(key: str, bases) -> str:
    for (_, pre) in bases:
        if key.startswith(pre):
            return pre
    return ""


def _part_bases(layout: BucketLayout, f32: torch.Tensor, i64: torch.Tensor, parts):
    """Per key-prefix views of the buckets through their OWN storage objects
    (slices of the bucket storage, which keep it alive).  A FedDCT slot binds
    its main-client and proxy models as one bucket (one launch per round), but
    each model's tensors must stay in a storage of their own: torch.save
    writes whole storages, and the reference saves the two models to separate
    files (train_feddct.py:455,463 via utils/metric.py:16-32)."""
    out = {}
    if not parts:
        return out
    for pre in parts:
        for is64, bucket in ((False, f32), (True, i64)):
            sl = [s for s in layout.slots if s.key.startswith(pre) and s.alias_of is None
                  and (s.kind == KIND_I64) == is64]
            if not sl:
                continue
            lo = min(s.offset for s in sl)
            hi = max(s.offset + s.numel for s in sl)
            if not is64:
                hi = min(-(-hi // 64) * 64, bucket.numel())
            es = bucket.element_size()
            st = bucket.untyped_storage()[lo * es:hi * es]
            base = torch.empty(0, dtype=bucket.dtype, device=bucket.device).set_(
                st, 0, (hi - lo,))
            out[(is64, pre)] = (base, lo)
    return out


def get_arena(module: torch.nn.Module, layout: BucketLayout) -> ModuleArena:
    """The module's arena for ``layout``, binding (or re-binding) if needed."""
    a = getattr(module, "_fa_arena", None)
    if a is not None and a.layout is layout and a.valid():
        return a
    if a is not None and a.layout == layout and a.valid():
        return a
    a = ModuleArena(module, layout)
    object.__setattr__(module, "_fa_arena", a)
    _bump()   # a (re)bound arena ends any round bound over the old one
    return a
