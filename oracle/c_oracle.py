"""ORACLE — test infrastructure only.  ctypes wrapper of the C restatement
(oracle/fa_oracle.c, built by oracle/Makefile into oracle/build/)."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")


class _Seg(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_int64), ("numel", ctypes.c_int64)]


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def _lib():
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(
            os.path.join(HERE, "fa_oracle.c")):
        build()
    lib = ctypes.CDLL(LIB)
    P = ctypes.c_void_p
    lib.fao_reduce_f32.argtypes = [P, ctypes.c_int, P, ctypes.c_int, P, ctypes.c_int, P]
    lib.fao_reduce_i64.argtypes = [P, ctypes.c_int, P, ctypes.c_int, P]
    return lib


_L = None


def _segs(segs):
    segs = np.asarray(segs, np.int64).reshape(-1, 2)
    arr = (_Seg * max(1, len(segs)))()
    for i, (o, m) in enumerate(segs):
        arr[i].offset, arr[i].numel = int(o), int(m)
    return arr, len(segs)


def reduce_f32(buckets, segs, weights=None, sum_only=False):
    """buckets: list of float32 1-D arrays (slot order) -> out bucket."""
    global _L
    _L = _L or _lib()
    bs = [np.ascontiguousarray(b, np.float32) for b in buckets]
    ptrs = (ctypes.c_void_p * len(bs))(*[b.ctypes.data for b in bs])
    out = np.zeros_like(bs[0])
    sa, ns = _segs(segs)
    w = None if weights is None else np.ascontiguousarray(weights, np.float32)
    rc = _L.fao_reduce_f32(ptrs, len(bs), sa, ns, None if w is None else w.ctypes.data,
                           1 if sum_only else 0, out.ctypes.data)
    assert rc == 0
    return out


def reduce_i64(buckets, segs):
    global _L
    _L = _L or _lib()
    bs = [np.ascontiguousarray(b, np.int64) for b in buckets]
    ptrs = (ctypes.c_void_p * len(bs))(*[b.ctypes.data for b in bs])
    out = np.zeros_like(bs[0])
    sa, ns = _segs(segs)
    assert _L.fao_reduce_i64(ptrs, len(bs), sa, ns, out.ctypes.data) == 0
    return out
