"""A/B: FedProx proximal-term kernels (fa_prox_norms + fa_prox_grad) of the
in-tree libfedagg.so against other builds of the same ABI, wrn16_8 C100
parameter layout, 4 rotated buffer sets (> the 256 MB MALL), interleaved
rounds in one process, HIP events on the launch stream.
Usage: exp_prox_ab.py OTHER.so[,OTHER2.so...]|- ROUNDS   (- = the in-tree build alone)"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import load_manifest  # noqa: E402

_P, _I, _I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
PROTOS = {"fa_norm_plan_create": (_I, [_P, _I, _I64, ctypes.POINTER(_P)]),
          "fa_prox_norms": (_I, [_P, _P, _P, _P, _P, _P]),
          "fa_prox_grad": (_I, [_P, _P, _P, _P, _P, ctypes.c_float, _P, _P, _P])}


def main():
    others = [] if sys.argv[1] == "-" else sys.argv[1].split(",")
    rounds = int(sys.argv[2])
    steps = 40
    dev = torch.device("cuda", 0)
    lay = BucketLayout.from_manifest(load_manifest("wrn16_8_c100"))
    segs = np.asarray(lay.segs32, np.int64).reshape(-1, 2)
    P = int(segs[:, 1].sum())
    libs = {"intree": _lib.lib}
    for o in others:
        L = ctypes.CDLL(os.path.abspath(o))
        for name, (res, args) in PROTOS.items():
            getattr(L, name).restype, getattr(L, name).argtypes = res, args
        libs[os.path.basename(o)] = L
    arr, n = _lib.seg_array(segs)
    plans = {}
    for k, L in libs.items():
        h = ctypes.c_void_p()
        _lib.check(L.fa_norm_plan_create(arr, n, int(lay.f32_numel), ctypes.byref(h)))
        plans[k] = h
    sets = []
    for _ in range(4):
        b = torch.randn(lay.f32_numel, device=dev)
        sets.append((b + 0.01, b, torch.empty_like(b), torch.empty_like(b)))
    norms = torch.empty(len(segs), device=dev)
    total = torch.empty((), device=dev)
    one = torch.ones((), device=dev)
    st = torch.cuda.current_stream()
    sp = ctypes.c_void_p(st.cuda_stream)

    def fwd(L, h, s):
        _lib.check(L.fa_prox_norms(h, s[0].data_ptr(), s[1].data_ptr(), norms.data_ptr(),
                                   total.data_ptr(), sp))

    def bwd(L, h, s):
        _lib.check(L.fa_prox_grad(h, s[0].data_ptr(), s[1].data_ptr(), norms.data_ptr(),
                                  one.data_ptr(), 1.0, s[2].data_ptr(), s[3].data_ptr(), sp))

    def both(L, h, s):
        fwd(L, h, s)
        bwd(L, h, s)

    def timed(fn, L, h):
        for i in range(8):
            fn(L, h, sets[i % 4])
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for i in range(steps):
            fn(L, h, sets[i % 4])
        e1.record(st)
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3 / steps

    res = {k: {"fwd": [], "bwd": [], "both": []} for k in libs}
    for r in range(rounds):
        for k, L in libs.items():
            for name, fn in (("fwd", fwd), ("bwd", bwd), ("both", both)):
                res[k][name].append(timed(fn, L, plans[k]))
        print(f"round {r} done", file=sys.stderr, flush=True)
    for k in libs:
        med = {name: float(np.median(x)) for name, x in res[k].items()}
        print(json.dumps({"exp": "prox_ab", "build": k, "params": P,
                          "fwd_us": round(med["fwd"], 2), "bwd_us": round(med["bwd"], 2),
                          "both_us": round(med["both"], 2),
                          "both_GBps": round(24 * P / med["both"] / 1e3, 1),
                          "both_frac": round(24 * P / med["both"] / 1e3 / 8000.0, 4)}))


if __name__ == "__main__":
    main()
