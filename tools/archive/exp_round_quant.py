"""Experiment (r03 session 4): is cfg4's ~6 % gap to cfg2 (weighted, same
20 clients) the part-filled last round of its plain tile table?  cfg2's
layout plus one extra fp32 key of k x 2048 floats (k whole vector tiles),
weighted as bench's cfg4, one process, interleaved.  cfg2 alone is 5,358
vector tiles; 768 resident workgroups x 7 rounds = 5,376.  If the time per
step jumps between k = 16 and k = 20 by more than the extra bytes, the
quantization is the cause.  Each k runs the default plan (its tail split,
fedagg.hip split_tail) and the plain table (FA_PLAN_TUNE_NO_BALANCE).

    python tools/archive/exp_round_quant.py [ROUNDS]
"""
import copy
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd.aggregate import client_weights  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, load_manifest, make_clients  # noqa: E402

N = 20
SIZES = [2500 + 97 * ((7 * i) % 11) for i in range(N)]
KS = [0, 8, 16, 17, 18, 20, 25, 40, 60, 100, 112, 150, 200, 250, 300, 350, 400]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    base = load_manifest("wrn16_8_c10")
    reds = {}
    for k in KS:
        man = copy.deepcopy(base)
        if k:
            man["keys"].append({"key": "pad.weight", "shape": [k, 2048], "dtype": "float32"})
        lay = BucketLayout.from_manifest(man)
        cl = make_clients(lay, man, range(N), dev)
        for v, fl in (("default", 0), ("plain", _lib.FA_PLAN_TUNE_NO_BALANCE)):
            plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                             flags=_lib.FA_PLAN_GAPS_ARE_PADDING | fl)
            r = Reducer(lay, cl, torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1]),
                        weights=client_weights(SIZES), plan=plan)
            nt, sl = ctypes.c_int(0), ctypes.c_int(0)
            _lib.check(_lib.lib.fa_plan_launch_shape(r.plan.handle, N, 1, ctypes.byref(nt),
                                                     ctypes.byref(sl)), "fa_plan_launch_shape")
            reds[(k, v)] = (r, lay.algorithmic_bytes(N), nt.value, sl.value)
        torch.cuda.synchronize()
    times = {k: [] for k in reds}
    for _ in range(rounds):
        for k, (fn, _, _, _) in reds.items():
            for _ in range(5):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                fn()
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) / 50 * 1e3)
        print("round", file=sys.stderr, flush=True)
    for k, ts in times.items():
        ts = sorted(ts)
        med = ts[len(ts) // 2]
        _, nb, nt, sl = reds[k]
        print(json.dumps({"exp": "round_quant", "extra_tiles": k[0], "table": k[1],
                          "launch_tiles": nt, "slots": sl,
                          "rounds": round(nt / sl, 3) if sl else None,
                          "us_median": round(med, 2), "us_min": round(ts[0], 2),
                          "GBps": round(nb / med / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
