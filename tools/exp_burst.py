"""Tail-burst experiment (r05): the tiles of the last k rounds of resident
workgroups read the kernarg pointer array directly, so a batch's loads issue
back to back (shorter drain?) while the earlier tiles keep the product's
shape.  FA_EXP_BURST=k, read per launch; k = 0 is the product.  Same
process, same buffers, settings alternated; output bits compared.

    python tools/exp_burst.py [ROUNDS] [LAYOUT ...]
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, joint_manifest, load_manifest, make_clients  # noqa: E402

LAYOUTS = {
    "cfg2": (("wrn16_8_c10",), 20, 1),
    "cfg3": (("wrnsl16_8_sf4_c10_main", "wrnsl16_8_sf4_c10_proxy"), 5, 2),
    "sf32": (("wrnsl16_8_sf32_c100_main", "wrnsl16_8_sf32_c100_proxy"), 3, 6),
    "sf16": (("wrnsl16_8_sf16_c100_main", "wrnsl16_8_sf16_c100_proxy"), 3, 6),
    "r110": (("resnet110sl_sf4_c100_main", "resnet110sl_sf4_c100_proxy"), 25, 4),
}
KS = ("0", "1", "2")


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
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
        rs = [Reducer(lay, cl, o32, o64) for cl, o32, o64 in sets]
        times = {k: [] for k in KS}
        outs = {}
        reps = 40 if n > 10 else 100
        for _ in range(rounds):
            for k in KS:
                os.environ["FA_EXP_BURST"] = k
                for i in range(3):
                    rs[i % rot]()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(reps):
                    rs[i % rot]()
                e1.record()
                e1.synchronize()
                times[k].append(e0.elapsed_time(e1) / reps * 1e3)
                outs[k] = sets[0][1].clone()
        os.environ.pop("FA_EXP_BURST", None)
        nb = lay.algorithmic_bytes(n)
        for k, ts in times.items():
            ts = sorted(ts)
            med = ts[len(ts) // 2]
            print(json.dumps({"exp": "tail_burst", "layout": tag, "n": n, "burst_rounds": int(k),
                              "us_median": round(med, 2), "us_min": round(ts[0], 2),
                              "frac": round(nb / (med * 1e-6) / 8e12, 4),
                              "same_bits": bool(torch.equal(outs[k].view(torch.int32),
                                                            outs["0"].view(torch.int32)))}),
                  flush=True)
        del sets, rs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
