"""Kernel variant sweep on the bench workload (interleaved rounds, one
process: MI355X guide §5.4 rule 24).  Prints one JSON line per variant."""
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
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    weighted = len(sys.argv) > 4 and sys.argv[4] == "w"
    probe = len(sys.argv) > 5 and sys.argv[5] == "probe"
    dev = torch.device("cuda", 0)
    man = load_manifest(lay_name)
    lay = BucketLayout.from_manifest(man)
    clients = make_clients(lay, man, range(n), dev)
    nbytes = lay.algorithmic_bytes(n)
    variants = []
    auto_plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel)
    o32a, o64a = torch.zeros_like(clients[0][0]), torch.zeros_like(clients[0][1])
    wa = [1.0 / (i + 2) for i in range(n)] if weighted else None
    variants.append(("auto", Reducer(lay, clients, o32a, o64a, plan=auto_plan, weights=wa),
                     o32a, o64a))
    for u in (1, 2, 4):
        for nt in (True, False):
            for b16 in ((False, True) if u < 4 else (False,)):
                fl = _lib.FA_PLAN_GAPS_ARE_PADDING | (0 if nt else _lib.FA_PLAN_TUNE_NO_NT) | \
                    (_lib.FA_PLAN_TUNE_BATCH16 if b16 else _lib.FA_PLAN_TUNE_BATCH8)
                plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                                 tile_elems=1024 * u, flags=fl)
                out32 = torch.zeros_like(clients[0][0])
                out64 = torch.zeros_like(clients[0][1])
                if not nt:
                    continue
                w = [1.0 / (i + 2) for i in range(n)] if weighted else None
                variants.append((f"U{u}_{'nt' if nt else 'plain'}_B{16 if b16 else 8}",
                                 Reducer(lay, clients, out32, out64, plan=plan, weights=w),
                                 out32, out64))
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
    # read-only and copy ceilings on a 2 GiB buffer (beyond the 256 MiB MALL)
    big = torch.empty(512 * 1024 * 1024 if probe else 1024, dtype=torch.float32, device=dev)
    big.uniform_()
    for grid in ((1024, 2048, 4096, 8192) if probe else ()):
        part = torch.zeros(grid, device=dev)
        fn = lambda: _lib.check(_lib.lib.fa_read_probe_f32(  # noqa: E731
            big.data_ptr(), big.numel(), part.data_ptr(), grid,
            torch.cuda.current_stream().cuda_stream))
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 10 * 1e-3
        print(json.dumps({"probe": "read_only", "grid": grid, "GBps": round(big.numel() * 4 / t / 1e9, 1)}))
    del big
    ref32, ref64 = variants[0][2], variants[0][3]
    for name, _, o32, o64 in variants:
        ts = sorted(times[name])
        print(json.dumps({"variant": name, "layout": lay_name, "n": n, "weighted": weighted,
                          "us_median": round(ts[len(ts) // 2], 2), "us_min": round(ts[0], 2),
                          "GBps_median": round(nbytes / (ts[len(ts) // 2] * 1e-6) / 1e9, 1),
                          "same_as_first": bool(torch.equal(o32, ref32) and torch.equal(o64, ref64))}))


if __name__ == "__main__":
    main()
