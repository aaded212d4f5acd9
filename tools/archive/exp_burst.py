"""Experiment (r03): per-launch time of the headline reduce (cfg2) against
its position in a back-to-back burst, after an idle gap — does a short
burst run faster than a long one (clock / power state), and how much of
the spread between measurement scripts (20 vs 60 vs 200 launches) is
that?  Each launch bracketed by its own pair of events.

    python tools/archive/exp_burst.py [BURST] [GAPS_MS,...]
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, load_manifest, make_clients  # noqa: E402


def main():
    burst = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    gaps = [float(g) for g in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 50, 500]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    man = load_manifest("wrn16_8_c10")
    lay = BucketLayout.from_manifest(man)
    cl = make_clients(lay, man, range(20), dev)
    red = Reducer(lay, cl, torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1]),
                  plan=_lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                                 flags=_lib.FA_PLAN_GAPS_ARE_PADDING))
    nb = lay.algorithmic_bytes(20)
    for _ in range(20):
        red()
    torch.cuda.synchronize()
    for gap in gaps:
        for rep in range(3):
            time.sleep(gap / 1e3)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(burst + 1)]
            ev[0].record()
            for i in range(burst):
                red()
                ev[i + 1].record()
            ev[-1].synchronize()
            ts = [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(burst)]
            tot = ev[0].elapsed_time(ev[-1]) * 1e3
            windows = {}
            for a, b in ((0, 5), (5, 25), (25, 65), (65, 105), (105, 205), (205, 400),
                         (400, 1000)):
                if b <= burst:
                    w = sorted(ts[a:b])
                    windows[f"{a}-{b}"] = round(sum(w) / len(w), 2)
            print(json.dumps({"exp": "burst", "gap_ms": gap, "rep": rep, "burst": burst,
                              "mean_us": round(tot / burst, 2),
                              "frac": round(nb / (tot / burst) / 1e3 / 8000, 4),
                              "window_mean_us": windows}), flush=True)


if __name__ == "__main__":
    main()
