"""Reduce launch time by tile width (vector floats per lane per client: U = 1,
2, 4 -> 1024 / 2048 / 4096-float tiles) on the small FedDCT sweep layouts
and cfg2, same process, alternating (r04): whether the launches that fill
about one round of resident workgroups gain from more bytes in flight per
wave.  One JSON line per (layout, tile width): median us over ROUNDS passes.

    python tools/exp_tile_width.py [ROUNDS] [LAYOUT ...]
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, joint_manifest, load_manifest, make_clients  # noqa: E402

LAYOUTS = {
    "cfg2": (("wrn16_8_c10",), 20, 1),
    "cfg3": (("wrnsl16_8_sf4_c10_main", "wrnsl16_8_sf4_c10_proxy"), 5, 2),
    "sf32": (("wrnsl16_8_sf32_c100_main", "wrnsl16_8_sf32_c100_proxy"), 3, 6),
    "r110": (("resnet110sl_sf4_c100_main", "resnet110sl_sf4_c100_proxy"), 25, 4),
}


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    tags = sys.argv[2:] or list(LAYOUTS)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for tag in tags:
        names, n, rot = LAYOUTS[tag]
        mans = [load_manifest(x) for x in names]
        prefixes = ("0.", "1.") if len(names) > 1 else ("",)
        man = joint_manifest(mans, prefixes) if len(names) > 1 else mans[0]
        lay = BucketLayout.from_manifest(man)
        sets = []
        for _ in range(rot):
            cl = make_clients(lay, list(zip(mans, prefixes)), range(n), dev)
            sets.append((cl, torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1])))
        fns, info = {}, {}
        for te in (1024, 2048, 4096):
            plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                             tile_elems=te, flags=_lib.FA_PLAN_GAPS_ARE_PADDING)
            info[te] = plan.info["ntiles"]
            fns[te] = [Reducer(lay, cl, o32, o64, plan=plan) for cl, o32, o64 in sets]
        times = {te: [] for te in fns}
        reps = 40
        for _ in range(rounds):
            for te, rs in fns.items():
                for i in range(3):
                    rs[i % len(rs)]()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(reps):
                    rs[i % len(rs)]()
                e1.record()
                e1.synchronize()
                times[te].append(e0.elapsed_time(e1) / reps * 1e3)
        nb = lay.algorithmic_bytes(n)
        for te, ts in times.items():
            ts = sorted(ts)
            med = ts[len(ts) // 2]
            print(json.dumps({"exp": "tile_width", "layout": tag, "n": n, "tile_elems": te,
                              "ntiles": info[te], "us_median": round(med, 2),
                              "frac": round(nb / (med * 1e-6) / 8e12, 4)}), flush=True)
        del sets, fns
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
