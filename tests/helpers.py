"""Shared test helpers: numpy states <-> flat buckets, reference-shaped modules."""
import numpy as np
import torch

from feddct_amd.layout import KIND_I64, BucketLayout


def states_to_buckets(layout: BucketLayout, states, device, pad_value=0.0):
    out = []
    for st in states:
        f32 = torch.full((max(layout.f32_numel, 64),), pad_value, dtype=torch.float32)
        i64 = torch.zeros(max(layout.i64_numel, 1), dtype=torch.int64)
        for (k, v) in st:
            s = layout.by_key[k]
            if s.alias_of is not None:
                continue
            t = torch.from_numpy(np.array(v, copy=True)).reshape(-1)
            if s.kind == KIND_I64:
                i64[s.offset:s.offset + s.numel] = t
            else:
                f32[s.offset:s.offset + s.numel] = t.float()
        out.append((f32.to(device), i64.to(device)))
    return out


def buckets_to_state(layout: BucketLayout, f32, i64):
    f32 = f32.cpu().numpy()
    i64 = i64.cpu().numpy()
    res = []
    for s in layout.slots:
        src = i64 if s.kind == KIND_I64 else f32
        res.append((s.key, src[s.offset:s.offset + s.numel].reshape(s.shape).copy()))
    return res


class StateModule(torch.nn.Module):
    """A module whose state_dict has exactly a manifest's keys (dots allowed)."""

    def __init__(self, manifest):
        super().__init__()
        for e in manifest["keys"]:
            parts = e["key"].split(".")
            mod = self
            for p in parts[:-1]:
                if p not in mod._modules:
                    mod.add_module(p, torch.nn.Module())
                mod = mod._modules[p]
            t = torch.zeros(e["shape"], dtype=getattr(torch, e["dtype"]))
            if not (t.is_floating_point() or t.is_complex()):
                mod.register_buffer(parts[-1], t)
            else:
                mod.register_parameter(parts[-1], torch.nn.Parameter(t))

    def load_numpy(self, state):
        sd = self.state_dict()
        with torch.no_grad():
            for k, v in state:
                sd[k].copy_(torch.from_numpy(np.array(v, copy=True)))
        return self


def bits_equal(a, b):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    if a.dtype != b.dtype or a.shape != b.shape:
        return False
    if a.dtype == np.float32:
        na, nb = np.isnan(a), np.isnan(b)
        if not np.array_equal(na, nb):
            return False
        return np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))
    return np.array_equal(a, b)
