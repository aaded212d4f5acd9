"""Experiment (r03 session 3): where the torch-GPU-order kernel's ~6 % to the
default reduce goes (cfg2: 141.8 vs 134-135 us).  The same 20 clients'
bytes as cfg2's layout (82 fp32 keys incl. BN vectors, 16 int64) and as one
5376 x 2048 tensor (only the 2048-element wide body), each in both orders,
one process, interleaved, slab buckets.

    python tools/archive/exp_tgpu_gap.py [ROUNDS]
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, load_manifest, make_clients  # noqa: E402

N = 20


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    G = _lib.FA_PLAN_GAPS_ARE_PADDING
    cases = {"cfg2": load_manifest("wrn16_8_c10"),
             "one_tensor": {"name": "t5376", "keys": [{"key": "w", "shape": [5376, 2048],
                                                       "dtype": "float32"}]}}
    reds, nbytes = {}, {}
    for cname, man in cases.items():
        lay = BucketLayout.from_manifest(man)
        cl = make_clients(lay, man, range(N), dev)
        for oname, order in (("cpu", _lib.FA_ORDER_TORCH_CPU), ("tgpu", _lib.FA_ORDER_TORCH_GPU)):
            plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel, flags=G,
                             order=order, n=N)
            k = f"{cname}_{oname}"
            reds[k] = Reducer(lay, cl, torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1]),
                              plan=plan)
            nbytes[k] = lay.algorithmic_bytes(N)
    times = {k: [] for k in reds}
    for _ in range(rounds):
        for k, fn in reds.items():
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
        print(json.dumps({"exp": "tgpu_gap", "variant": k, "us_median": round(med, 2),
                          "us_min": round(ts[0], 2), "GBps": round(nbytes[k] / med / 1e3, 1),
                          "ntiles": reds[k].plan.info.get("ntiles")}), flush=True)


if __name__ == "__main__":
    main()
