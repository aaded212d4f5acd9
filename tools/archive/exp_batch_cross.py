"""Experiment (r03): tile count against resident workgroups — 8-row load
batches (96 VGPRs) against 16-row batches (160 VGPRs, 3 workgroups per CU),
each with the plain tile table (FA_PLAN_TUNE_NO_BALANCE) and the balanced
one (vector tiles re-cut to fill whole rounds) — on one fp32 tensor of
T x 2048 elements, N clients, buffers rotated past the MALL, all variants
interleaved in one process, bits compared.

    python tools/archive/exp_batch_cross.py [ROUNDS]
"""
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, make_clients  # noqa: E402

TILES = (384, 768, 1024, 1280, 1536, 2048, 2560, 3072, 4096, 5376, 5380)
NS = (5, 20, 25)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    G = _lib.FA_PLAN_GAPS_ARE_PADDING
    for n in NS:
        for t in TILES:
            man = {"name": f"t{t}", "keys": [{"key": "w", "shape": [t * 2048],
                                              "dtype": "float32"}]}
            lay = BucketLayout.from_manifest(man)
            nb = lay.algorithmic_bytes(n)
            rot = max(2, math.ceil(1.2e9 / nb))
            if nb * rot > 12e9:
                continue
            sets = []
            for _ in range(rot):
                cl = make_clients(lay, man, range(n), dev)
                sets.append((cl, torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1])))
            variants = {}
            NB = _lib.FA_PLAN_TUNE_NO_BALANCE
            for k, fl in (("b16", _lib.FA_PLAN_TUNE_BATCH16 | NB), ("b8", _lib.FA_PLAN_TUNE_BATCH8 | NB),
                          ("b16_bal", _lib.FA_PLAN_TUNE_BATCH16),
                          ("b8_bal", _lib.FA_PLAN_TUNE_BATCH8)):
                plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                                 flags=G | fl)
                variants[k] = [Reducer(lay, cl, o32, o64, plan=plan) for cl, o32, o64 in sets]
            times = {k: [] for k in variants}
            ref = None
            reps = max(20, min(200, int(2e-3 / (nb / 6.5e12))))
            for _ in range(rounds):
                for k, reds in variants.items():
                    for red in reds:
                        red()
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for i in range(reps):
                        reds[i % rot]()
                    e1.record()
                    e1.synchronize()
                    times[k].append(e0.elapsed_time(e1) / reps * 1e3)
                    got = sets[(reps - 1) % rot][1].clone()
                    if ref is None:
                        ref = got
                    assert torch.equal(got.view(torch.int32), ref.view(torch.int32)), k
            med = {k: sorted(v)[len(v) // 2] for k, v in times.items()}
            rec = {"exp": "batch_cross", "n": n, "tiles": t, "rot": rot}
            for k in variants:
                nt, sl = variants[k][0].plan.launch_shape(n)
                rec[k] = {"us": round(med[k], 2), "frac": round(nb / med[k] / 1e3 / 8000, 4),
                          "launch_tiles": nt, "slots": sl}
            print(json.dumps(rec), flush=True)
            del sets, variants
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
