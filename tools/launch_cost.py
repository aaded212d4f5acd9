"""Host cost of one launch call (r04, VERDICT r03 next 4: the drop-in's host
share): each call below is timed on the host while the GPU is kept busy by
a long spin kernel queued first, so the time is the submit path alone (no
wait for the GPU).  Per call the median over REPS calls in microseconds:

  ctypes_noop         a ctypes call into libfedagg that does no HIP work
  torch_add           a 1-element torch kernel (torch's own launch path)
  write_probe_small   fa_write_probe_f32 over 1024 floats (our smallest launch)
  reduce_<shape>      ctypes fa_reduce, the bound round's reduce (flags 0)
  bcast_<shape>       ctypes fa_reduce, FA_F_BCAST_ONLY
  engine_<shape>      the engine's _launch wrapper around the same reduce

Usage: launch_cost.py [REPS]"""
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd import aggregate as A  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import joint_manifest, load_manifest, make_clients  # noqa: E402

SHAPES = {"cfg2": (("wrn16_8_c10",), 20), "cfg3": (("wrnsl16_8_sf4_c10_main",
                                                     "wrnsl16_8_sf4_c10_proxy"), 5),
          "cfg5": (("wrnsl16_8_sf4_c100_main", "wrnsl16_8_sf4_c100_proxy"), 24)}


def busy(ms):
    try:
        torch.cuda._sleep(int(ms * 2.4e6))   # ~2.4 GHz shader clock: ms of spin
    except Exception:
        x = torch.empty(1 << 28, device="cuda")
        for _ in range(int(ms)):
            x.add_(1.0)


def host_time(fn, reps):
    torch.cuda.synchronize()
    busy(40 + reps * 0.5)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e6)
    torch.cuda.synchronize()
    ts.sort()
    return round(ts[len(ts) // 2], 2)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = _lib.lib
    out = {"exp": "launch_cost", "reps": reps}
    out["ctypes_noop"] = host_time(lambda: lib.fa_table_bytes(24), reps)
    t = torch.zeros(1, device=dev)
    out["torch_add"] = host_time(lambda: t.add_(1.0), reps)
    buf = torch.empty(1024, device=dev)
    arr = _lib.ptr_array([buf.data_ptr()])
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    out["write_probe_small"] = host_time(lambda: lib.fa_write_probe_f32(arr, 1, 1024, 1, s), reps)
    e = A.engine()
    for tag, (names, n) in SHAPES.items():
        mans = [load_manifest(x) for x in names]
        prefixes = ("0.", "1.") if len(names) > 1 else ("",)
        man = joint_manifest(mans, prefixes) if len(names) > 1 else mans[0]
        lay = BucketLayout.from_manifest(man)
        cl = make_clients(lay, list(zip(mans, prefixes)), range(n), dev)
        o32, o64 = torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1])
        plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                         flags=_lib.FA_PLAN_GAPS_ARE_PADDING)
        a32 = _lib.ptr_array([c[0].data_ptr() for c in cl])
        a64 = _lib.ptr_array([c[1].data_ptr() for c in cl])
        p32, p64 = o32.data_ptr(), o64.data_ptr()

        def red(fl=0):
            return lib.fa_reduce(plan.handle, a32, a64, n, None, p32, p64, fl, s)
        assert red() == 0
        out[f"reduce_{tag}"] = host_time(red, reps)
        out[f"bcast_{tag}"] = host_time(lambda: red(_lib.FA_F_BCAST_ONLY), reps)
        out[f"engine_{tag}"] = host_time(
            lambda: e._launch(plan, a32, a64, n, None, p32, p64, 0, dev), reps)
        del cl
        torch.cuda.synchronize()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
