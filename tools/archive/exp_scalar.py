"""Experiment (r03): the packed scalar tiles (K_SCALAR_PACKED) of the
reference's BN-heavy FedDCT layouts — pack size 64 / 32 / 16 / 8 columns per
tile (r03: placing them after the vector tiles measured no better), vector
tiles of 2048 (default), 4096 and 1024 floats — on the joint
main + proxy bucket, rotated past the MALL, interleaved in one process.
Every variant's output is checked against the default's bits.

    python tools/archive/exp_scalar.py [ROUNDS]
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, joint_manifest, load_manifest, make_clients  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for name, n, rot in (("resnet110sl_sf4_c100", 25, 4), ("wrnsl16_8_sf32_c100", 3, 6)):
        mans = [load_manifest(name + "_main"), load_manifest(name + "_proxy")]
        lay = BucketLayout.from_manifest(joint_manifest(mans))
        sets = []
        for _ in range(rot):
            cl = make_clients(lay, list(zip(mans, ("0.", "1."))), range(n), dev)
            sets.append((cl, torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1])))
        G = _lib.FA_PLAN_GAPS_ARE_PADDING
        variants = {}
        for te in (2048, 4096, 1024):
            for c, cols in enumerate((64, 32, 16, 8)):
                if te != 2048 and cols not in (64, 16):
                    continue
                fl = G | _lib.FA_PLAN_TUNE_PACK(c)
                plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                                 tile_elems=te, flags=fl)
                variants[f"tile{te}_pack{cols}"] = [Reducer(lay, cl, o32, o64, plan=plan)
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
            print(json.dumps({"exp": "scalar_pack", "layout": name, "n": n, "variant": k,
                              "us_median": round(med, 2), "us_min": round(ts[0], 2),
                              "GBps": round(nb / med / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
