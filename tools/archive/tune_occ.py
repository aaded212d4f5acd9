"""Occupancy cap and XCD tile-range knobs on the cfg2 reduction (interleaved
rounds in one process).  One JSON line per variant."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, load_manifest, make_clients  # noqa: E402


def main():
    lay_name = sys.argv[1] if len(sys.argv) > 1 else "wrn16_8_c10"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 7
    dev = torch.device("cuda", 0)
    man = load_manifest(lay_name)
    lay = BucketLayout.from_manifest(man)
    clients = make_clients(lay, man, range(n), dev)
    nbytes = lay.algorithmic_bytes(n)
    base = _lib.FA_PLAN_GAPS_ARE_PADDING | _lib.FA_PLAN_TUNE_BATCH16
    variants = []
    for tile in (2048, 4096):
        for xcd in (False, True):  # here: wave-contiguous mapping
            for cap in (0,):
                fl = base | (_lib.FA_PLAN_TUNE_WAVE_CONTIG if xcd else 0)
                plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                                 tile_elems=tile, flags=fl)
                o32, o64 = torch.zeros_like(clients[0][0]), torch.zeros_like(clients[0][1])
                variants.append((f"T{tile}_{'wavecontig' if xcd else 'strided'}",
                                 Reducer(lay, clients, o32, o64, plan=plan), o32, o64))
    times = {v[0]: [] for v in variants}
    for _ in range(rounds):
        for name, red, _, _ in variants:
            for _ in range(3):
                red()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                red()
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / 20 * 1e3)
    r32, r64 = variants[0][2], variants[0][3]
    for name, _, o32, o64 in variants:
        ts = sorted(times[name])
        print(json.dumps({"variant": name, "n": n, "us_median": round(ts[len(ts) // 2], 2),
                          "GBps_median": round(nbytes / (ts[len(ts) // 2] * 1e-6) / 1e9, 1),
                          "same": bool(torch.equal(o32, r32) and torch.equal(o64, r64))}))


if __name__ == "__main__":
    main()
