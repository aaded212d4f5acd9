"""Experiment (r03 session 4): why bench's cfg4 line (FedProx C100, 20
clients, weighted) reads ~8 % slower than the weighted headline (cfg2 C10,
same 20 clients' worth of bytes).  bench.other_configs builds cfg4 right
after cfg3's two rotated client sets, so cfg4's buckets start in the middle
of cfg3's slab and spill into a new one (two allocations under one round).
Variants, one process, interleaved:
  cfg4_after_cfg3  - as the bench builds it today
  cfg4_fresh_slab  - slab.release() first: all 20 buckets in one slab
  cfg2w_fresh_slab - the weighted headline's layout, fresh slab

    python tools/archive/exp_cfg4_slab.py [ROUNDS]
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from feddct_amd import slab  # noqa: E402
from feddct_amd.aggregate import client_weights  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, joint_manifest, load_manifest, make_clients  # noqa: E402

N = 20
SIZES = [2500 + 97 * ((7 * i) % 11) for i in range(N)]   # bench.other_configs' cfg4 shards


def reducer(name, dev):
    man = load_manifest(name)
    lay = BucketLayout.from_manifest(man)
    cl = make_clients(lay, man, range(N), dev)
    return Reducer(lay, cl, torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1]),
                   weights=client_weights(SIZES)), lay.algorithmic_bytes(N), cl


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    reds = {}
    # cfg3's two rotated sets first, as bench.other_configs does
    mm, pm = load_manifest("wrnsl16_8_sf4_c10_main"), load_manifest("wrnsl16_8_sf4_c10_proxy")
    lay3 = BucketLayout.from_manifest(joint_manifest([mm, pm], ("0.", "1.")))
    keep = [make_clients(lay3, [(mm, "0."), (pm, "1.")], range(5), dev) for _ in range(2)]
    reds["cfg4_after_cfg3"] = reducer("wrn16_8_c100", dev)
    slab.release()
    reds["cfg4_fresh_slab"] = reducer("wrn16_8_c100", dev)
    slab.release()
    reds["cfg2w_fresh_slab"] = reducer("wrn16_8_c10", dev)
    for k, (_, _, cl) in reds.items():
        p = sorted(c[0].data_ptr() for c in cl)
        gaps = sorted(set(b - a for a, b in zip(p, p[1:])))
        print(json.dumps({"variant": k, "distinct_strides": len(gaps), "max_stride": gaps[-1]}),
              file=sys.stderr, flush=True)
    times = {k: [] for k in reds}
    for _ in range(rounds):
        for k, (fn, _, _) in reds.items():
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
    del keep
    for k, ts in times.items():
        ts = sorted(ts)
        med = ts[len(ts) // 2]
        print(json.dumps({"exp": "cfg4_slab", "variant": k, "us_median": round(med, 2),
                          "us_min": round(ts[0], 2),
                          "GBps": round(reds[k][1] / med / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
