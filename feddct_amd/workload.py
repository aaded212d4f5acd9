"""Synthetic device-resident workloads for the bench and the full-size tests.

Client slot ``c`` of a layout is filled on the GPU by the bit-exact HIP
restatement of feddct_amd/synth.py (fa_synth_fill_*), so the box regenerates
the inputs behind tests/golden/digests.json without shipping them.
"""
from __future__ import annotations

import ctypes
import json
import os
from typing import List, Tuple

import torch

from . import _lib, synth
from .arena import alloc_buckets
from .layout import KIND_I64, BucketLayout

MANIFEST_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "manifests")


def load_manifest(name: str) -> dict:
    with open(os.path.join(MANIFEST_DIR, name + ".json")) as f:
        return json.load(f)


def joint_manifest(manifests, prefixes=("0.", "1.")) -> dict:
    """One layout for several models (FedDCT's main + proxy slot): the keys
    of each under its prefix, in order — the layout of aggregate._Pair."""
    keys = []
    for m, p in zip(manifests, prefixes):
        keys += [dict(e, key=p + e["key"]) for e in m["keys"]]
    return {"name": "+".join(m.get("name", "?") for m in manifests), "keys": keys}


def fill_client(layout: BucketLayout, manifest: dict, f32: torch.Tensor, i64: torch.Tensor,
                client: int, mode: int = synth.MODE_REALISTIC, prefix: str = "") -> None:
    """Client ``client``'s synthetic state for ``manifest``'s keys (key index
    = position in that manifest), written at ``layout``'s slots of
    ``prefix + key``."""
    stream = ctypes.c_void_p(torch.cuda.current_stream(f32.device).cuda_stream)
    for j, e in enumerate(manifest["keys"]):
        s = layout.by_key[prefix + e["key"]]
        if s.alias_of is not None:
            continue
        if s.kind == KIND_I64:
            _lib.check(_lib.lib.fa_synth_fill_i64(i64[s.offset:].data_ptr(), s.numel, j, client,
                                                  mode, stream), "fa_synth_fill_i64")
        else:
            mu, sigma = synth.key_params(e["key"], tuple(e["shape"]), e["dtype"])
            _lib.check(_lib.lib.fa_synth_fill_f32(f32[s.offset:].data_ptr(), s.numel, j, client,
                                                  mu, sigma, mode, stream), "fa_synth_fill_f32")


def make_clients(layout: BucketLayout, manifest, clients, device,
                 mode: int = synth.MODE_REALISTIC) -> List[Tuple[torch.Tensor, torch.Tensor]]:
    """``manifest`` may be a list of (manifest, prefix) for a joint layout."""
    parts = manifest if isinstance(manifest, list) else [(manifest, "")]
    out = []
    for c in clients:
        # the product's own storage: fp32 buckets carved from a shared slab
        # on a GPU (arena.alloc_buckets, slab.py)
        f32, i64 = alloc_buckets(layout, torch.device(device))
        for m, prefix in parts:
            fill_client(layout, m, f32, i64, c, mode, prefix)
        out.append((f32, i64))
    return out


class Reducer:
    """Pre-bound fa_reduce call over fixed buckets (what the bench times):
    pointer arrays are built once, each call is one launch."""

    def __init__(self, layout: BucketLayout, clients, out32, out64, weights=None, flags=0,
                 tile_elems=0, plan=None):
        self.plan = plan or _lib.Plan(layout.segs32, layout.f32_numel, layout.segs64,
                                      layout.i64_numel, tile_elems=tile_elems)
        self.n = len(clients)
        self.a32 = _lib.ptr_array([c[0].data_ptr() for c in clients])
        self.a64 = _lib.ptr_array([c[1].data_ptr() for c in clients])
        self.w = None if weights is None else (ctypes.c_float * self.n)(*map(float, weights))
        self.out32 = out32
        self.out64 = out64
        self.flags = flags
        self._keep = (clients, out32, out64)

    def __call__(self, stream=None):
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        _lib.check(_lib.lib.fa_reduce(self.plan.handle, self.a32, self.a64, self.n, self.w,
                                      self.out32.data_ptr(), self.out64.data_ptr(), self.flags,
                                      ctypes.c_void_p(s)), "fa_reduce")
