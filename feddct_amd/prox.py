"""FedProx proximal term on the flat buckets.

Drop-in for the loop of train_fedprox.py:113-115:

    proximal_term = 0.0
    for w, w_t in zip(client_model.parameters(), global_model.parameters()):
        proximal_term += (w - w_t).norm(2)

becomes ``proximal_term = feddct_amd.prox.proximal_term(client_model,
global_model)`` — the same value (to fp32 rounding) and the same gradients
for BOTH models' parameters (the reference's graph also reaches the global
model's parameters), computed by three HIP launches (two forward, one backward) over the two arenas
(csrc/prox.hip) instead of 2·K norm/sub kernels plus their backward.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .arena import get_arena


class _NormPlan:
    def __init__(self, segs: np.ndarray, numel: int):
        arr, n = _lib.seg_array(segs)
        h = ctypes.c_void_p()
        _lib.check(_lib.lib.fa_norm_plan_create(arr, n, int(numel), ctypes.byref(h)),
                   "fa_norm_plan_create")
        self.handle = h
        self.nseg = n
        self.owned = True   # False once the C++ one-node state owns it (ProximalTerm._native)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value and getattr(self, "owned", True):
            try:
                _lib.lib.fa_norm_plan_destroy(h)
            except Exception:
                pass


class _Prox(torch.autograd.Function):
    @staticmethod
    def forward(ctx, term, *params):
        dev = term.ca.f32.device
        norms = torch.empty(max(1, term.plan.nseg), dtype=torch.float32, device=dev)
        total = torch.empty((), dtype=torch.float32, device=dev)
        s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        _lib.check(_lib.lib.fa_prox_norms(term.plan.handle, term.ca.ptr32, term.ga.ptr32,
                                          norms.data_ptr(), total.data_ptr(), s),
                   "fa_prox_norms")
        ctx.term = term
        ctx.save_for_backward(norms)
        return total

    @staticmethod
    def backward(ctx, gout):
        term = ctx.term
        (norms,) = ctx.saved_tensors
        dev = norms.device
        gout = gout.to(dtype=torch.float32).contiguous()
        need_b = any(ctx.needs_input_grad[1 + len(term.slots):])
        ga = torch.empty_like(term.ca.f32)
        gb = torch.empty_like(term.ga.f32) if need_b else None
        s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        _lib.check(_lib.lib.fa_prox_grad(term.plan.handle, term.ca.ptr32, term.ga.ptr32,
                                         norms.data_ptr(), gout.data_ptr(), 1.0,
                                         ga.data_ptr(), None if gb is None else gb.data_ptr(),
                                         s), "fa_prox_grad")
        grads_a = [ga[o:o + m].view(shape) for o, m, shape in term.slots]
        grads_b = ([gb[o:o + m].view(shape) for o, m, shape in term.slots] if need_b
                   else [None] * len(term.slots))
        return (None, *grads_a, *grads_b)


class _ProxFlat(torch.autograd.Function):
    """The one-node form (r03; since r04 the definition behind the C++ node
    csrc/shim.cpp ProxNode, which runs it without Python in the backward):
    the parameters are not inputs of the graph
    node, so a backward is ONE node instead of this node plus an
    AccumulateGrad per parameter (200 for wrn16_8's client + global: ~0.6 ms
    of autograd bookkeeping per training step).  Its backward accumulates the
    gradients straight into flat gradient buckets whose slices are the
    parameters' ``.grad`` — what AccumulateGrad does, in one launch."""

    @staticmethod
    def forward(ctx, term, anchor):
        total = term.norms_forward()
        ctx.term = term
        return total

    @staticmethod
    def backward(ctx, gout):
        if torch.is_grad_enabled():
            raise RuntimeError("feddct_amd.prox: the one-node proximal term has no double "
                               "backward; use proximal_term(..., flat_grads=False)")
        ctx.term.accumulate_grads(gout)
        return None, None


class ProximalTerm:
    """Bound (client, global) pair: plan built once, reused every step."""

    def __init__(self, client_model: torch.nn.Module, global_model: torch.nn.Module):
        from .aggregate import engine
        layout = engine().layout_of(global_model)
        self.client_model, self.global_model = client_model, global_model
        self.layout = layout
        self.ca = get_arena(client_model, layout)
        self.ga = get_arena(global_model, layout)
        if self.ca.device.type != "cuda":
            raise RuntimeError("feddct_amd.prox: models must be on the GPU (no CPU fallback)")
        cn = [n for n, _ in client_model.named_parameters()]
        gn = [n for n, _ in global_model.named_parameters()]
        if len(cn) != len(gn):
            raise RuntimeError("client and global models have different parameter counts")
        slots = []
        for a, b in zip(cn, gn):
            sa, sb = layout.by_key.get(a), layout.by_key.get(b)
            if sa is None or sb is None or sa.kind != "f32" or sb.offset != sa.offset:
                raise NotImplementedError(
                    f"proximal term pairs parameters by position; {a!r} / {b!r} are not the "
                    "same fp32 slot of one layout")
            slots.append((sa.offset, sa.numel, sa.shape))
        self.slots = slots
        # the parameter objects are pinned by the arenas' validity checks:
        # a replaced parameter invalidates the arena and with it this term
        self.params = tuple(client_model.parameters()) + tuple(global_model.parameters())
        segs = np.array([(o, m) for o, m, _ in slots], np.int64).reshape(-1, 2)
        with torch.cuda.device(self.ca.device):
            self.plan = _NormPlan(segs, layout.f32_numel)
        self._flat = None   # gradient buckets of the one-node form, made on first use

    # ------------------------------------------------- the one-node form --
    def _flat_state(self):
        if self._flat is None:
            dev = self.ca.device
            sides = []
            for params, arena in ((list(self.client_model.parameters()), self.ca),
                                  (list(self.global_model.parameters()), self.ga)):
                keep = [(p, sl) for p, sl in zip(params, self.slots) if p.requires_grad]
                buf = torch.zeros_like(arena.f32) if keep else None
                views = tuple(buf[o:o + m].view(shape) for _, (o, m, shape) in keep)
                sides.append((tuple(p for p, _ in keep), views, buf))
            self._flat = (sides, torch.zeros((), device=dev, requires_grad=True),
                          torch.empty(max(1, self.plan.nseg), dtype=torch.float32, device=dev))
        return self._flat

    def _native(self):
        """The C++ one-node form's bound state (csrc/shim.cpp ProxNode, r04):
        the same buckets, views and flags as accumulate_grads, handed to a
        C++ autograd node whose backward runs without Python."""
        cap = getattr(self, "_cap", None)
        if cap is None:
            from . import _fa_shim
            sides, _, norms = self._flat_state()
            (pa, va, ba), (pb, vb, bb) = sides
            addr = lambda f: ctypes.cast(f, ctypes.c_void_p).value  # noqa: E731
            # the capsule owns the plan and holds both buckets:
            # a node whose term was dropped before backward stays runnable;
            # this term keeps using the handle while it holds the capsule
            cap = self._cap = _fa_shim.prox_state(
                addr(_lib.lib.fa_prox_norms), addr(_lib.lib.fa_prox_grad_ex),
                addr(_lib.lib.fa_norm_plan_destroy), self.plan.handle.value,
                self.ca.f32, self.ga.f32, norms,
                self._scratch(self.ca.device) if ba is None else norms, pa, va, ba,
                _lib.FA_PROX_ACCUMULATE_A,
                pb, vb, bb, _lib.FA_PROX_ACCUMULATE_B)
            self.plan.owned = False
        return cap

    def norms_forward(self) -> torch.Tensor:
        _, _, norms = self._flat_state()
        dev = self.ca.device
        total = torch.empty((), dtype=torch.float32, device=dev)
        s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        _lib.check(_lib.lib.fa_prox_norms(self.plan.handle, self.ca.ptr32, self.ga.ptr32,
                                          norms.data_ptr(), total.data_ptr(), s),
                   "fa_prox_norms")
        return total

    def accumulate_grads(self, gout: torch.Tensor) -> None:
        """.grad += d term / d w for both models' parameters, through their
        bound flat gradient buckets (one kernel)."""
        from . import _fa_shim
        sides, _, norms = self._flat_state()
        dev = self.ca.device
        gout = gout.to(device=dev, dtype=torch.float32).contiguous()
        states = []
        for params, views, buf in sides:
            if buf is None:
                states.append(None)
                continue
            st = _fa_shim.grad_state(params, views)
            if st == 2:   # some .grad not bucket views: take them over, once
                with torch.no_grad():
                    for p, v in zip(params, views):
                        if p.grad is None:
                            v.zero_()
                        elif p.grad is not v:
                            v.copy_(p.grad)
                _fa_shim.bind_grads(params, views)
                st = 0
            states.append(st)
        if all(st is None for st in states):
            return
        # per side: accumulate into bound .grad (state 0), overwrite where
        # every .grad was None (state 1) — no memset of that bucket first
        flags = ((_lib.FA_PROX_ACCUMULATE_A if states[0] == 0 else 0)
                 | (_lib.FA_PROX_ACCUMULATE_B if states[1] == 0 else 0))
        (_, _, ba), (_, _, bb) = sides
        s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        _lib.check(_lib.lib.fa_prox_grad_ex(
            self.plan.handle, self.ca.ptr32, self.ga.ptr32, norms.data_ptr(), gout.data_ptr(),
            1.0, ba.data_ptr() if ba is not None else self._scratch(dev).data_ptr(),
            None if bb is None else bb.data_ptr(), flags, s),
            "fa_prox_grad_ex")
        for (params, views, buf), st in zip(sides, states):
            if st == 1:
                _fa_shim.bind_grads(params, views)

    def _scratch(self, dev):
        """A write-only target for the client side when no client parameter
        needs a gradient (the kernel always writes grad_a)."""
        sc = getattr(self, "_sc", None)
        if sc is None:
            sc = self._sc = torch.empty_like(self.ca.f32)
        return sc

    def valid(self) -> bool:
        return (getattr(self.client_model, "_fa_arena", None) is self.ca and self.ca.valid()
                and getattr(self.global_model, "_fa_arena", None) is self.ga and self.ga.valid())

    def __call__(self, flat_grads: bool = False) -> torch.Tensor:
        if flat_grads:
            _, anchor, _ = self._flat_state()
            from . import _fa_shim
            if hasattr(_fa_shim, "prox_apply"):
                dev = self.ca.device
                return _fa_shim.prox_apply(self._native(), anchor,
                                           torch.cuda.current_stream(dev).cuda_stream)
            return _ProxFlat.apply(self, anchor)
        return _Prox.apply(self, *self.params)


def proximal_term(client_model: torch.nn.Module, global_model: torch.nn.Module,
                  flat_grads: bool = False) -> torch.Tensor:
    """Σ_k ||w_k − w_t,k||₂ over zip(client.parameters(), global.parameters()),
    differentiable w.r.t. both (train_fedprox.py:113-115).  The bound term is
    cached on the client module (no global registry).

    ``flat_grads=False`` (default): an ordinary autograd node whose inputs are
    the parameters, so every autograd use works as with the reference's loop —
    ``loss.backward()``, ``torch.autograd.grad(loss, params)``,
    ``backward(inputs=...)``, per-parameter hooks and DDP reducer hooks.

    ``flat_grads=True`` (opt-in, for a plain ``loss.backward()`` training
    step, train_fedprox.py:117-127): ONE graph node whose only input is a
    private anchor tensor; its backward adds the gradients into both models'
    ``.grad``, made views of one flat gradient bucket per model (rebound after
    ``zero_grad(set_to_none=True)``), in one launch — autograd's
    per-parameter AccumulateGrad work skipped.  Because the parameters are
    not inputs of that node, autograd prunes it from
    ``torch.autograd.grad(loss, params)`` and ``backward(inputs=params)``
    (the proximal gradient is then silently missing), parameter hooks never
    see its share of ``.grad``, double backward raises, and with gradient
    accumulation the fp32 sum is (g + prox) + task rather than
    g + (task + prox) (equal to rounding).  Use it only where the step is
    ``loss.backward()`` followed by the optimizer."""
    cache = client_model.__dict__.setdefault("_fa_prox", {})
    t = cache.get(id(global_model))
    if t is None or t.global_model is not global_model or not t.valid():
        t = cache[id(global_model)] = ProximalTerm(client_model, global_model)
    return t(flat_grads)
