"""Experiment (r03 session 4): does the tail split (fedagg.hip split_tail,
16-client kernels only) pay on the 8-client kernel too (N < 16, e.g. cfg3's
N = 5 at 4.2 rounds of 1,280 slots)?  One fp32 tensor of T x 2048 floats,
plain tile table vs the split table, both as explicit tile tables
(fa_plan_create_from_tiles), one process, interleaved.

    python tools/archive/exp_tail_small_n.py [ROUNDS]
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, make_clients  # noqa: E402

CASES = [(5, 5120 + 20), (5, 5120 + 100), (5, 5120 + 260), (5, 3840 + 50), (5, 5120 + 640),
         (8, 5120 + 60), (12, 5120 + 60)]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    reds = {}
    for n, t in CASES:
        man = {"name": f"t{t}", "keys": [{"key": "w", "shape": [t * 2048], "dtype": "float32"}]}
        lay = BucketLayout.from_manifest(man)
        cl = make_clients(lay, man, range(n), dev)
        probe = _lib.Plan(lay.segs32, lay.f32_numel)
        _, slots = probe.launch_shape(n, False)
        plain = np.array([(c, min(2048, t * 2048 - c), 0) for c in range(0, t * 2048, 2048)],
                         np.int64)
        split = _lib.balance_host(plain, 2048, 0, slots)
        for v, tiles in (("plain", plain), ("split", split)):
            if tiles is None:
                continue
            plan = _lib.Plan(lay.segs32, lay.f32_numel, tiles=tiles, tile_elems=2048)
            reds[(n, t, v)] = (Reducer(lay, cl, torch.zeros_like(cl[0][0]),
                                       torch.zeros_like(cl[0][1]), plan=plan),
                               lay.algorithmic_bytes(n), len(tiles), slots)
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
        print(json.dumps({"exp": "tail_small_n", "n": k[0], "tiles_plain": k[1], "table": k[2],
                          "launch_tiles": nt, "slots": sl, "us_median": round(med, 2),
                          "us_min": round(ts[0], 2), "GBps": round(nb / med / 1e3, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
