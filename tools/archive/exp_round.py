"""Experiment: the cfg2 round (reduce + broadcast,
train_fedavg.py:145-149) against its two kernels alone, in ONE process,
interleaved, HIP events:

  reduce          fa_reduce, no broadcast
  bcast[_xcd]     FA_F_BCAST_ONLY: the broadcast launch alone (consecutive
                  client groups, the default / XCD-paired groups)
  round[_xcd]   FA_F_BCAST: reduce + broadcast launch
  round_st_plain  the reduce's result stores temporal (the broadcast's source
                  may stay in the MALL)

Prints one JSON line per variant (median / min µs over R rounds of 20
launches) and a summary line: round / (reduce + bcast).
Usage: exp_round.py [ROUNDS]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, load_manifest, make_clients  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    man = load_manifest("wrn16_8_c10")
    lay = BucketLayout.from_manifest(man)
    n = 20
    cl = make_clients(lay, man, range(n), dev)
    o32, o64 = torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1])

    def plan(fl=0):
        return _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                         flags=_lib.FA_PLAN_GAPS_ARE_PADDING | fl)

    XC = _lib.FA_PLAN_TUNE_BCAST_XCD
    B, BO = _lib.FA_F_BCAST, _lib.FA_F_BCAST_ONLY
    p0, pnx, pst = plan(), plan(XC), plan(_lib.FA_PLAN_TUNE_ST_PLAIN)
    v = {
        "reduce": Reducer(lay, cl, o32, o64, plan=p0),
        "bcast": Reducer(lay, cl, o32, o64, flags=BO, plan=p0),
        "bcast_xcd": Reducer(lay, cl, o32, o64, flags=BO, plan=pnx),
        "round": Reducer(lay, cl, o32, o64, flags=B, plan=p0),
        "round_xcd": Reducer(lay, cl, o32, o64, flags=B, plan=pnx),
        "round_st_plain": Reducer(lay, cl, o32, o64, flags=B, plan=pst),
    }
    times = {k: [] for k in v}
    for r in range(rounds):
        for k, fn in v.items():
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) / 20 * 1e3)
        print(f"round {r}", file=sys.stderr, flush=True)
    med = {}
    for k, ts in times.items():
        ts = sorted(ts)
        med[k] = ts[len(ts) // 2]
        print(json.dumps({"exp": "round", "variant": k, "us_median": round(med[k], 2),
                          "us_min": round(ts[0], 2)}), flush=True)
    print(json.dumps({"exp": "round_summary",
                      "round_over_sum": round(med["round"] / (med["reduce"] + med["bcast"]), 4),
                      "xcd_round_over_sum": round(med["round_xcd"] /
                                                    (med["reduce"] + med["bcast_xcd"]), 4)}),
          flush=True)


if __name__ == "__main__":
    main()
