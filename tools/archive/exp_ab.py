"""A/B: the in-tree libfedagg.so against another build of the same ABI
(e.g. the previous commit's, tools/libfedagg_ab.so) on the same workload,
interleaved rounds in one process.  Usage: exp_ab.py OTHER.so[,OTHER2.so...] LAYOUT N ROUNDS"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import load_manifest, make_clients  # noqa: E402


def main():
    other, lay_name, n, rounds = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    dev = torch.device("cuda", 0)
    man = load_manifest(lay_name)
    lay = BucketLayout.from_manifest(man)
    clients = make_clients(lay, man, range(n), dev)
    nbytes = lay.algorithmic_bytes(n)
    a32 = _lib.ptr_array([c[0].data_ptr() for c in clients])
    a64 = _lib.ptr_array([c[1].data_ptr() for c in clients])
    libs = {"intree": _lib.lib}
    for o in other.split(","):
        libs[os.path.basename(o)] = ctypes.CDLL(os.path.abspath(o))
    runs = {}
    for name, L in libs.items():
        L.fa_plan_create.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64,
                                     ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int,
                                     ctypes.c_uint, ctypes.POINTER(ctypes.c_void_p)]
        L.fa_reduce.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_void_p] * 3 + [ctypes.c_uint,
                                                                               ctypes.c_void_p]
        L.fa_reduce.argtypes[3] = ctypes.c_int
        s32, n32 = _lib.seg_array(lay.segs32)
        s64, n64 = _lib.seg_array(lay.segs64)
        h = ctypes.c_void_p()
        assert L.fa_plan_create(s32, n32, lay.f32_numel, s64, n64, lay.i64_numel, 0,
                                _lib.FA_PLAN_GAPS_ARE_PADDING, ctypes.byref(h)) == 0
        o32, o64 = torch.zeros_like(clients[0][0]), torch.zeros_like(clients[0][1])

        def fn(L=L, h=h, o32=o32, o64=o64):
            st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
            assert L.fa_reduce(h, a32, a64, n, None, o32.data_ptr(), o64.data_ptr(), 0, st) == 0
        runs[name] = (fn, o32, o64, [])
    for _ in range(rounds):
        for name, (fn, _, _, ts) in runs.items():
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 20 * 1e3)
    ref = runs["intree"]
    for name, (_, o32, o64, ts) in runs.items():
        ts = sorted(ts)
        print(json.dumps({"lib": name, "layout": lay_name, "n": n,
                          "us_median": round(ts[len(ts) // 2], 2), "us_min": round(ts[0], 2),
                          "GBps_median": round(nbytes / (ts[len(ts) // 2] * 1e-6) / 1e9, 1),
                          "same": bool(torch.equal(o32, ref[1]) and torch.equal(o64, ref[2]))}))


if __name__ == "__main__":
    main()
