"""Does the 256 MiB Infinity Cache (MALL) help the headline?  The cfg2
reduction timed on one buffer set (as bench.py) and rotating over 2 and 3
independent sets (each 922 MB), interleaved rounds, one process."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, load_manifest, make_clients  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    man = load_manifest("wrn16_8_c10")
    lay = BucketLayout.from_manifest(man)
    sets = []
    for k in range(3):
        cl = make_clients(lay, man, range(20 * k, 20 * k + 20), dev)
        o32, o64 = torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1])
        sets.append(Reducer(lay, cl, o32, o64))
    nbytes = lay.algorithmic_bytes(20)
    res = {1: [], 2: [], 3: []}
    for _ in range(9):
        for rot in (1, 2, 3):
            for i in range(6):
                sets[i % rot]()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(60):
                sets[i % rot]()
            e1.record()
            torch.cuda.synchronize()
            res[rot].append(e0.elapsed_time(e1) / 60 * 1e3)
    for rot, ts in res.items():
        ts.sort()
        print(json.dumps({"rotated_sets": rot, "us_median": round(ts[len(ts) // 2], 2),
                          "GBps": round(nbytes / (ts[len(ts) // 2] * 1e-6) / 1e9, 1)}))


if __name__ == "__main__":
    main()
