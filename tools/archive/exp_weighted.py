"""Weighted vs unweighted reduce launch (r04), same process, alternating, on
the cfg2 (wrn16_8 C10) and cfg4 (wrn16_8 C100) layouts at N = 20: what the
client weights cost the kernel (one fp32 product per element per client, the
weights read once per batch).  One JSON line per (layout, form).

    python tools/exp_weighted.py [ROUNDS]
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, load_manifest, make_clients  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = 20
    for name in ("wrn16_8_c10", "wrn16_8_c100"):
        man = load_manifest(name)
        lay = BucketLayout.from_manifest(man)
        cl = make_clients(lay, man, range(n), dev)
        o32, o64 = torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1])
        plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                         flags=_lib.FA_PLAN_GAPS_ARE_PADDING)
        w = (np.arange(1, n + 1) / np.arange(1, n + 1).sum()).astype(np.float32)
        fns = {"mean": Reducer(lay, cl, o32, o64, plan=plan),
               "weighted": Reducer(lay, cl, o32, o64, weights=list(w), plan=plan)}
        times = {k: [] for k in fns}
        for _ in range(rounds):
            for k, fn in fns.items():
                for _ in range(5):
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(50):
                    fn()
                e1.record()
                e1.synchronize()
                times[k].append(e0.elapsed_time(e1) / 50 * 1e3)
        nb = lay.algorithmic_bytes(n)
        for k, ts in times.items():
            ts = sorted(ts)
            med = ts[len(ts) // 2]
            print(json.dumps({"exp": "weighted", "layout": name, "form": k,
                              "us_median": round(med, 2),
                              "frac": round(nb / (med * 1e-6) / 8e12, 4)}), flush=True)
        del cl, fns
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
