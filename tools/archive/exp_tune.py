"""Experiment (r03): launch shapes for the latency-bound layouts — rows in
flight per batch (BATCH4/8/16: fewer VGPRs -> more resident workgroups),
a persistent grid (PERSIST k = k*256 workgroups looping over tiles) and
workgroups per CU caps — on the FedDCT sweep layouts and cfg3, rotated past
the MALL, interleaved in one process.  Every variant's output is checked
against the default's bits.

    python tools/archive/exp_tune.py [ROUNDS] [LAYOUT,...]
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import (MANIFEST_DIR, Reducer, joint_manifest, load_manifest,  # noqa: E402
                                 make_clients)

LAYOUTS = {   # name -> (manifest stem, N, rotated sets[, weighted]); a stem without
    # _main/_proxy manifests is one model (cfg2 / cfg4)
    "cfg2": ("wrn16_8_c10", 20, 1),
    "cfg4w": ("wrn16_8_c100", 20, 1, True),
    "resnet110sl": ("resnet110sl_sf4_c100", 25, 4),
    "sf32": ("wrnsl16_8_sf32_c100", 3, 6),
    "cfg3": ("wrnsl16_8_sf4_c10", 5, 2),
    "cfg5": ("wrnsl16_8_sf4_c100", 24, 1),
    "sf2": ("wrnsl16_8_sf2_c100", 48, 1),
}

G = _lib.FA_PLAN_GAPS_ARE_PADDING
VARIANTS = {
    "default": (0, 0),
    "plain": (0, _lib.FA_PLAN_TUNE_NO_BALANCE),
    "batch8_plain": (0, _lib.FA_PLAN_TUNE_BATCH8 | _lib.FA_PLAN_TUNE_NO_BALANCE),
    "batch16": (0, _lib.FA_PLAN_TUNE_BATCH16),
    "batch8": (0, _lib.FA_PLAN_TUNE_BATCH8),
    "batch4": (0, _lib.FA_PLAN_TUNE_BATCH4),
    "u4": (4096, 0),
    "u4_batch4": (4096, _lib.FA_PLAN_TUNE_BATCH4),
    "u1": (1024, 0),
}


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    which = sys.argv[2].split(",") if len(sys.argv) > 2 else list(LAYOUTS)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for lname in which:
        stem, n, rot = LAYOUTS[lname][:3]
        weighted = len(LAYOUTS[lname]) > 3
        if os.path.exists(os.path.join(MANIFEST_DIR, stem + "_main.json")):
            mans = [load_manifest(stem + "_main"), load_manifest(stem + "_proxy")]
            lay = BucketLayout.from_manifest(joint_manifest(mans))
            parts = list(zip(mans, ("0.", "1.")))
        else:
            man = load_manifest(stem)
            lay = BucketLayout.from_manifest(man)
            parts = man
        wts = [float(1000 + 37 * c) for c in range(n)] if weighted else None
        sets = []
        for _ in range(rot):
            cl = make_clients(lay, parts, range(n), dev)
            sets.append((cl, torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1])))
        variants = {}
        for k, (te, fl) in VARIANTS.items():
            plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                             tile_elems=te, flags=G | fl)
            variants[k] = [Reducer(lay, cl, o32, o64, weights=wts, plan=plan)
                           for cl, o32, o64 in sets]
        ref = None
        times = {k: [] for k in variants}
        for r in range(rounds):
            for k, reds in variants.items():
                for red in reds:
                    red()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(20 * rot):
                    reds[i % rot]()
                e1.record()
                e1.synchronize()
                times[k].append(e0.elapsed_time(e1) / (20 * rot) * 1e3)
                o32, o64 = sets[0][1], sets[0][2]
                got = (o32.clone(), o64.clone())
                if ref is None:
                    ref = got
                assert torch.equal(got[0].view(torch.int32), ref[0].view(torch.int32)), k
                assert torch.equal(got[1], ref[1]), k
        nb = lay.algorithmic_bytes(n)
        for k, ts in times.items():
            ts = sorted(ts)
            med = ts[len(ts) // 2]
            nt, sl = variants[k][0].plan.launch_shape(n, weighted)
            print(json.dumps({"exp": "tune", "layout": stem, "n": n, "weighted": weighted,
                              "variant": k,
                              "launch_tiles": nt, "slots": sl,
                              "us_median": round(med, 2), "us_min": round(ts[0], 2),
                              "GBps": round(nb / med / 1e3, 1),
                              "frac": round(nb / med / 1e3 / 8000, 4)}), flush=True)


if __name__ == "__main__":
    main()
