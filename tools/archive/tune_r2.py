"""Round-2 sweep: the weighted cfg2 launch and the cfg3
FedDCT launch (N=5, main + proxy joint bucket, 2 rotated sets > the MALL)
over tile width U (1024*U floats) x client batch B, interleaved rounds in one
process.  One JSON line per (workload, variant) with median / min µs and
GB/s; the launch policy in fedagg.hip's launch_reduce is set from these."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, joint_manifest, load_manifest, make_clients  # noqa: E402

BATCH = {1: _lib.FA_PLAN_TUNE_BATCH1, 4: _lib.FA_PLAN_TUNE_BATCH4, 8: _lib.FA_PLAN_TUNE_BATCH8,
         16: _lib.FA_PLAN_TUNE_BATCH16}


def variants(lay, sets, w, us, bs):
    out = []
    for u in us:
        for b in bs:
            if u == 4 and b == 16:
                continue
            fl = _lib.FA_PLAN_GAPS_ARE_PADDING | BATCH[b]
            plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                             tile_elems=1024 * u, flags=fl)
            reds = [Reducer(lay, cl, torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1]),
                            plan=plan, weights=w) for cl in sets]
            out.append((f"U{u}_B{b}", reds))
    for b in (4, 8):   # the batch's loads issued back to back (FA_PLAN_TUNE_ISSUE_ALL)
        fl = _lib.FA_PLAN_GAPS_ARE_PADDING | BATCH[b] | _lib.FA_PLAN_TUNE_ISSUE_ALL
        plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                         tile_elems=2048, flags=fl)
        out.append((f"U2_B{b}_issue_all", [Reducer(lay, cl, torch.zeros_like(cl[0][0]),
                                                    torch.zeros_like(cl[0][1]), plan=plan,
                                                    weights=w) for cl in sets]))
    auto = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel)
    out.append(("auto", [Reducer(lay, cl, torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1]),
                                 plan=auto, weights=w) for cl in sets]))
    return out


def sweep(name, lay, sets, w, nbytes, rounds, us, bs, extra=None):
    vs = variants(lay, sets, w, us, bs)
    if extra:
        vs += extra
    times = {v[0]: [] for v in vs}
    for _ in range(rounds):
        for vname, reds in vs:
            k = [0]

            def step():
                reds[k[0] % len(reds)]()
                k[0] += 1
            for _ in range(4):
                step()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(40):
                step()
            e1.record()
            torch.cuda.synchronize()
            times[vname].append(e0.elapsed_time(e1) / 40 * 1e3)
    for vname, ts in times.items():
        ts.sort()
        print(json.dumps({"workload": name, "variant": vname, "median_us": round(ts[len(ts) // 2], 2),
                          "min_us": round(ts[0], 2),
                          "GBps_median": round(nbytes / (ts[len(ts) // 2] * 1e-6) / 1e9, 1)}),
              flush=True)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    # cfg2 shape, weighted (sizes 1..20) vs unweighted
    man = load_manifest("wrn16_8_c10")
    lay = BucketLayout.from_manifest(man)
    cl = make_clients(lay, man, range(20), dev)
    s = np.arange(1, 21, dtype=np.float64)
    w = (s / s.sum()).astype(np.float32)
    nb = lay.algorithmic_bytes(20)
    unw = [("unweighted_auto", [Reducer(lay, cl, torch.zeros_like(cl[0][0]),
                                        torch.zeros_like(cl[0][1]))])]
    sweep("cfg2_weighted", lay, [cl], w, nb, rounds, (1, 2, 4), (4, 8, 16), unw)
    del cl
    torch.cuda.empty_cache()
    # cfg3: FedDCT sf4 C10, 5 slots, joint bucket, 2 rotated sets
    mm, pm = load_manifest("wrnsl16_8_sf4_c10_main"), load_manifest("wrnsl16_8_sf4_c10_proxy")
    lay = BucketLayout.from_manifest(joint_manifest([mm, pm]))
    sets = [make_clients(lay, [(mm, "0."), (pm, "1.")], range(5), dev) for _ in range(2)]
    sweep("cfg3_n5", lay, sets, None, lay.algorithmic_bytes(5), rounds, (1, 2, 4), (1, 4, 8))


if __name__ == "__main__":
    main()
