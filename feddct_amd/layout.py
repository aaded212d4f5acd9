"""Flat bucket layout of a model state_dict (SURVEY.md §7 "design stance").

Every client's state lives in two flat HBM buckets:

* ``f32`` — all floating keys (and, packed, every non-int64 key), each key's
  tensor starting on a 256-B boundary (64 fp32 elements) so every vectorised
  cascade run starts 16-B aligned and the gaps are padding the kernel may
  write;
* ``i64`` — all int64 keys (``num_batches_tracked``), densely packed.

The layout fixes key order = ``global_model.state_dict()`` order, which is the
order the reference iterates (train_fedavg.py:144) — it does not change the
per-element arithmetic, only where each key lives.  The same layout object is
shared by the global model and all client slots, so one tile table (plan)
serves every round.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

ALIGN_F32 = 64  # elements: 256 B

KIND_F32 = "f32"      # float32 key, zero-copy view into the f32 bucket
KIND_I64 = "i64"      # int64 key, zero-copy view into the i64 bucket
KIND_PACKF = "packf"  # any other dtype: .float() into the f32 bucket per call

_DTYPES = {
    "float32": torch.float32, "float64": torch.float64, "float16": torch.float16,
    "bfloat16": torch.bfloat16, "int64": torch.int64, "int32": torch.int32,
    "int16": torch.int16, "int8": torch.int8, "uint8": torch.uint8, "bool": torch.bool,
}


def dtype_of(name) -> torch.dtype:
    if isinstance(name, torch.dtype):
        return name
    return _DTYPES[str(name).replace("torch.", "")]


@dataclass(frozen=True)
class Slot:
    key: str
    shape: Tuple[int, ...]
    dtype: torch.dtype
    kind: str
    offset: int  # element offset inside its bucket
    numel: int
    alias_of: Optional[str] = None  # tied tensor: shares another key's slot


def _round_up(x: int, a: int) -> int:
    return (x + a - 1) // a * a


class BucketLayout:
    """Key → (bucket, offset) map plus the fa_seg tables for the kernel."""

    def __init__(self, entries: Sequence[Tuple[str, Sequence[int], object]],
                 aliases: Optional[Dict[str, str]] = None):
        aliases = dict(aliases or {})
        self.slots: List[Slot] = []
        self.by_key: Dict[str, Slot] = {}
        off32 = 0
        off64 = 0
        for key, shape, dt in entries:
            dt = dtype_of(dt)
            shape = tuple(int(s) for s in shape)
            numel = int(np.prod(shape)) if shape else 1
            if key in aliases:
                base = self.by_key[aliases[key]]
                s = Slot(key, shape, dt, base.kind, base.offset, base.numel, aliases[key])
            elif dt == torch.int64:
                s = Slot(key, shape, dt, KIND_I64, off64, numel)
                off64 += numel
            elif dt.is_complex:
                raise TypeError(f"state_dict key {key!r}: complex dtype {dt} not supported")
            else:
                off32 = _round_up(off32, ALIGN_F32)
                s = Slot(key, shape, dt, KIND_F32 if dt == torch.float32 else KIND_PACKF,
                         off32, numel)
                off32 += numel
            self.slots.append(s)
            self.by_key[key] = s
        self.f32_numel = _round_up(off32, ALIGN_F32)
        self.i64_numel = off64
        own = [s for s in self.slots if s.alias_of is None]
        self.segs32 = np.array([(s.offset, s.numel) for s in own if s.kind != KIND_I64],
                               np.int64).reshape(-1, 2)
        self.segs64 = np.array([(s.offset, s.numel) for s in own if s.kind == KIND_I64],
                               np.int64).reshape(-1, 2)
        self.packed = [s for s in own if s.kind == KIND_PACKF]
        # the alias map is part of the identity: a tied and an untied layout
        # with the same keys bind modules differently (arena.py)
        self.signature = tuple((s.key, s.shape, str(s.dtype), s.alias_of) for s in self.slots)
        self.keys = [s.key for s in self.slots]

    # ---------------------------------------------------------- builders --
    @classmethod
    def from_manifest(cls, manifest) -> "BucketLayout":
        return cls([(e["key"], e["shape"], e["dtype"]) for e in manifest["keys"]])

    @classmethod
    def from_state_dict(cls, sd) -> "BucketLayout":
        entries, aliases, seen = [], {}, {}
        for k, v in sd.items():
            if not isinstance(v, torch.Tensor):
                raise TypeError(f"state_dict key {k!r} is not a tensor")
            ident = (v.device, v.data_ptr(), tuple(v.shape), tuple(v.stride()), v.dtype)
            if v.numel() > 0 and ident in seen:
                aliases[k] = seen[ident]
            else:
                seen[ident] = k
            entries.append((k, tuple(v.shape), v.dtype))
        return cls(entries, aliases)

    # ----------------------------------------------------------- queries --
    @property
    def f32_data_elems(self) -> int:
        return int(self.segs32[:, 1].sum()) if len(self.segs32) else 0

    @property
    def i64_data_elems(self) -> int:
        return int(self.segs64[:, 1].sum()) if len(self.segs64) else 0

    def state_bytes(self) -> int:
        """B: bytes of one client's state (fp32 keys as fp32 + int64 keys)."""
        return 4 * self.f32_data_elems + 8 * self.i64_data_elems

    def algorithmic_bytes(self, n: int) -> int:
        """sum over keys of N*in_bytes + out_bytes."""
        return (n + 1) * self.state_bytes()

    def __eq__(self, other):
        return isinstance(other, BucketLayout) and self.signature == other.signature

    def __hash__(self):
        return hash(self.signature)
