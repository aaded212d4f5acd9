"""Experiment (r03): does the 256 MB MALL (Infinity Cache) serve part of the
headline's 922 MB per launch when the same 20 client buckets are reduced
back to back?  cfg2 (wrn16_8 C10, N = 20) with 1, 2 and 3 rotated client
sets (footprint 0.92 / 1.84 / 2.77 GB), and the same bytes as one synthetic
tensor of 5376 x 2048 floats, interleaved in one process, bits compared.

    python tools/archive/exp_mall.py [ROUNDS]
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
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    G = _lib.FA_PLAN_GAPS_ARE_PADDING
    cases = {
        "cfg2": load_manifest("wrn16_8_c10"),
        "one_tensor": {"name": "t5376", "keys": [{"key": "w", "shape": [5376 * 2048],
                                                  "dtype": "float32"}]},
    }
    variants = {}
    nbytes = {}
    for cname, man in cases.items():
        lay = BucketLayout.from_manifest(man)
        nbytes[cname] = lay.algorithmic_bytes(N)
        plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel, flags=G)
        sets = []
        for _ in range(3):
            cl = make_clients(lay, man, range(N), dev)
            sets.append(Reducer(lay, cl, torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1]),
                                plan=plan))
        for rot in (1, 2, 3):
            variants[f"{cname}_rot{rot}"] = (cname, sets[:rot])
    times = {k: [] for k in variants}
    for _ in range(rounds):
        for k, (cname, reds) in variants.items():
            rot = len(reds)
            for i in range(3 * rot):
                reds[i % rot]()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(60):
                reds[i % rot]()
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) / 60 * 1e3)
        print("round", file=sys.stderr, flush=True)
    for k, ts in times.items():
        ts = sorted(ts)
        med = ts[len(ts) // 2]
        nb = nbytes[variants[k][0]]
        print(json.dumps({"exp": "mall", "variant": k, "us_median": round(med, 2),
                          "us_min": round(ts[0], 2), "GBps": round(nb / med / 1e3, 1),
                          "frac": round(nb / med / 1e3 / 8000, 4)}), flush=True)


if __name__ == "__main__":
    main()
