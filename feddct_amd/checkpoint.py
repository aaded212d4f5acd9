"""Checkpoint serialization of the aggregated global model.

The reference saves, per round, ``{'round', 'arch', 'state_dict':
global_model.state_dict(), 'best_acc1', 'optimizer'[, 'scaler']}`` with
``torch.save`` (train_fedavg.py:421-442 → utils/metric.py:9-14; FedDCT's
best main/proxy models: utils/metric.py:16-32, train_feddct.py:451-471).

With the state in an arena, ``state_dict()`` is a set of views of ONE flat
buffer, so the checkpoint moves one contiguous block instead of K tensors:

* ``bucket_state_dict(module)`` — a CPU copy of the state made with a single
  device→pinned-host DMA of each bucket; the returned tensors are views of
  that copy (same keys, shapes, dtypes as ``module.state_dict()``);
* ``save_checkpoint(state, is_best, model_dir, filename)`` — the reference's
  signature and files; a ``state_dict`` entry that is a bound module's state
  is written from its bucket (torch.save stores each shared storage once);
* ``load_into(module, state_dict)`` — loads a checkpoint's state straight
  into the module's buckets (one host→device copy per bucket when the file
  was written from a bucket).

Files are ordinary ``torch.save`` pickles of tensors and plain values: the
reference's resume path (``torch.load`` + ``load_state_dict``,
train_fedavg.py:276-310) reads them unchanged, and they load with
``torch.load(..., weights_only=True)``.
"""
from __future__ import annotations

import os
import shutil
from collections import OrderedDict

import torch

from .arena import ModuleArena
from .layout import KIND_I64, KIND_PACKF


def _arena(module) -> ModuleArena:
    a = getattr(module, "_fa_arena", None)
    return a if a is not None and a.valid() else None


def bucket_state_dict(module: torch.nn.Module, _stage: bool = False
                      ) -> "OrderedDict[str, torch.Tensor]":
    """CPU state_dict of ``module`` copied out of its arena in one transfer
    per bucket (falls back to ``module.state_dict()`` when not bound).
    ``_stage``: reuse a pinned staging buffer kept on the arena (the result is
    only valid until the next staged call — save_checkpoint's use)."""
    a = _arena(module)
    if a is None:
        return OrderedDict((k, v.detach().cpu()) for k, v in module.state_dict().items())
    pin = a.f32.device.type == "cuda"
    stage = getattr(a, "_ckpt_stage", None) if _stage else None
    if stage is None:
        h32 = torch.empty(a.f32.shape, dtype=a.f32.dtype, pin_memory=pin)
        h64 = torch.empty(a.i64.shape, dtype=a.i64.dtype, pin_memory=pin)
        if _stage:
            a._ckpt_stage = (h32, h64)
    else:
        h32, h64 = stage
    h32.copy_(a.f32, non_blocking=pin)
    h64.copy_(a.i64, non_blocking=pin)
    if pin:
        torch.cuda.current_stream(a.f32.device).synchronize()
    out = OrderedDict()
    for s in a.layout.slots:
        if s.kind == KIND_PACKF:
            out[s.key] = module.state_dict()[s.key].detach().cpu()
            continue
        src = h64 if s.kind == KIND_I64 else h32
        out[s.key] = src[s.offset:s.offset + s.numel].view(s.shape)
    return out


def save_checkpoint(state: dict, is_best: bool, model_dir: str,
                    filename: str = "checkpoint.pth.tar") -> str:
    """utils/metric.py:9-14 with the state_dict written from the bucket."""
    state = dict(state)
    sd = state.get("state_dict")
    if isinstance(sd, torch.nn.Module):
        state["state_dict"] = bucket_state_dict(sd, _stage=True)  # serialised before return
    path = os.path.join(model_dir, filename)
    torch.save(state, path)
    if is_best:
        shutil.copyfile(path, os.path.join(model_dir, "model_best.pth.tar"))
    return path


def save_checkpoint_main_client(state: dict, is_best: bool, model_dir: str) -> None:
    """utils/metric.py:16-23 (FedDCT: only the best main-client model)."""
    if is_best:
        save_checkpoint(state, False, model_dir, "main_client_best.pth.tar")


def save_checkpoint_proxy_clients(state: dict, is_best: bool, model_dir: str) -> None:
    """utils/metric.py:25-32 (FedDCT: only the best proxy model)."""
    if is_best:
        save_checkpoint(state, False, model_dir, "proxy_clients_best.pth.tar")


def _in_slot(t, s, first32) -> bool:
    return (isinstance(t, torch.Tensor) and t.dtype == torch.float32
            and t.untyped_storage().data_ptr() == first32.untyped_storage().data_ptr()
            and t.storage_offset() == s.offset and tuple(t.shape) == s.shape
            and t.is_contiguous())


def load_into(module: torch.nn.Module, state_dict) -> None:
    """``module.load_state_dict(state_dict)`` (strict); when the module is
    bound and the checkpoint's tensors are views of one bucket-shaped
    storage, the bucket is filled with one copy."""
    a = _arena(module)
    if a is None:
        module.load_state_dict(state_dict)
        return
    keys = list(state_dict.keys())
    if keys != a.layout.keys:
        module.load_state_dict(state_dict)  # raises like the reference would
        return
    first32 = next((state_dict[s.key] for s in a.layout.slots if s.kind == "f32"), None)
    # one copy only when every fp32 tensor sits exactly where the bucket
    # layout puts it (offset, shape, dtype, dense): a file packed any other
    # way with the same total size takes load_state_dict's checked path
    whole = (first32 is not None and first32.untyped_storage().nbytes() == a.f32.numel() * 4
             and all(_in_slot(state_dict[s.key], s, first32)
                     for s in a.layout.slots if s.kind == "f32"))
    if whole:
        src = torch.empty(0, dtype=torch.float32, device=first32.device)
        src.set_(first32.untyped_storage(), 0, a.f32.shape)
        with torch.no_grad():
            a.f32.copy_(src)
            for s in a.layout.slots:
                if s.kind != "f32":
                    dst = module.state_dict()[s.key]
                    dst.copy_(state_dict[s.key])
        a.mark_written()
        return
    module.load_state_dict(state_dict)
