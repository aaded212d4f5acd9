"""Experiment (r03): where the small FedDCT sweep layouts lose their time
(a named cause for every layout below 0.70).  For each
layout: the product reduce; the same fp32 bytes as ONE flat tensor (no
per-tensor tiles, no scalar columns) at the same N; that flat tensor at 1/2,
2 and 4 times the size (the fixed per-launch intercept of a linear fit); and
a float4 copy of the same bytes.  Buffers rotated past the MALL, every
variant interleaved in one process.

    python tools/archive/exp_small.py [ROUNDS] [LAYOUT,...]
"""
import json
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import (Reducer, joint_manifest, load_manifest,  # noqa: E402
                                 make_clients)

LAYOUTS = {"sf32": ("wrnsl16_8_sf32_c100", 3), "resnet110sl": ("resnet110sl_sf4_c100", 25),
           "cfg3": ("wrnsl16_8_sf4_c10", 5)}
G = _lib.FA_PLAN_GAPS_ARE_PADDING


def timed(fns, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for f in fns:
        f()
    e0.record()
    for i in range(reps):
        fns[i % len(fns)]()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def reducers(lay, parts, n, dev, rot):
    plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel, flags=G)
    out = []
    for _ in range(rot):
        cl = make_clients(lay, parts, range(n), dev)
        out.append(Reducer(lay, cl, torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1]),
                           plan=plan))
    return out


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    which = sys.argv[2].split(",") if len(sys.argv) > 2 else list(LAYOUTS)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for name in which:
        stem, n = LAYOUTS[name]
        mans = [load_manifest(stem + "_main"), load_manifest(stem + "_proxy")]
        lay = BucketLayout.from_manifest(joint_manifest(mans))
        nb = lay.algorithmic_bytes(n)
        rot = max(2, math.ceil(1.2e9 / nb))
        f32 = int(sum(int(m) for _, m in np.asarray(lay.segs32).reshape(-1, 2)))
        variants = {"product": (reducers(lay, list(zip(mans, ("0.", "1."))), n, dev, rot), nb)}
        for scale in (0.5, 1, 2, 4):
            numel = int(f32 * scale) // 2048 * 2048
            man = {"name": "flat", "keys": [{"key": "w", "shape": [numel], "dtype": "float32"}]}
            fl = BucketLayout.from_manifest(man)
            r = max(2, math.ceil(1.2e9 / fl.algorithmic_bytes(n)))
            variants[f"flat_x{scale}"] = (reducers(fl, man, n, dev, r), fl.algorithmic_bytes(n))
        # a float4 copy moving the product's bytes (read + write)
        cn = nb // 8 // 4 * 4
        bufs = [(torch.empty(cn, device=dev).uniform_(-1, 1), torch.empty(cn, device=dev))
                for _ in range(rot)]

        def mk(src, dst):
            return lambda: _lib.check(_lib.lib.fa_copy_f32(
                src.data_ptr(), dst.data_ptr(), cn, torch.cuda.current_stream().cuda_stream))
        variants["copy_same_bytes"] = ([mk(s, d) for s, d in bufs], 8 * cn)
        times = {k: [] for k in variants}
        for _ in range(rounds):
            for k, (fns, _) in variants.items():
                times[k].append(timed(fns, 40 * len(fns)))
        rec = {"exp": "small", "layout": stem, "n": n, "rot": rot, "algorithmic_bytes": nb,
               "keys": len(lay.by_key)}
        xs, ys = [], []
        for k, (fns, b) in variants.items():
            med = sorted(times[k])[len(times[k]) // 2]
            rec[k] = {"us": round(med, 2), "bytes": b, "TBps": round(b / med / 1e6, 3)}
            if k.startswith("flat_x"):
                xs.append(b)
                ys.append(med)
        slope, icpt = np.polyfit(np.array(xs, float), np.array(ys, float), 1)
        rec["flat_fit"] = {"intercept_us": round(float(icpt), 2),
                           "marginal_TBps": round(1.0 / float(slope) / 1e6, 3)}
        print(json.dumps(rec), flush=True)
        del variants, bufs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
