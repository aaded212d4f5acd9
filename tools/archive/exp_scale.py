"""Experiment: fixed (per-launch) cost of the reduce kernel.  Times N=20
reductions over k concatenated copies of the wrn16_8 layout (k = 1, 2, 4):
T(k) = k*t_stream + t_fixed.  Also sweeps the 1024/2048/4096-float tile
tables at every k.  One JSON line per (k, tile)."""
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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    ks = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "1,2,4").split(",")]
    dev = torch.device("cuda", 0)
    base = load_manifest("wrn16_8_c10")
    for k in ks:
        prefixes = [f"{i}." for i in range(k)]
        man = joint_manifest([base] * k, prefixes) if k > 1 else base
        lay = BucketLayout.from_manifest(man)
        parts = [(base, p) for p in prefixes] if k > 1 else base
        clients = make_clients(lay, parts, range(n), dev)
        nbytes = lay.algorithmic_bytes(n)
        variants = []
        for te in (0, 1024, 2048, 4096):
            fl = 0 if te == 0 else (_lib.FA_PLAN_GAPS_ARE_PADDING | _lib.FA_PLAN_TUNE_BATCH16
                                    if te < 4096 else _lib.FA_PLAN_GAPS_ARE_PADDING
                                    | _lib.FA_PLAN_TUNE_BATCH8)
            plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                             tile_elems=te, flags=fl)
            o32, o64 = torch.zeros_like(clients[0][0]), torch.zeros_like(clients[0][1])
            variants.append((te, plan, Reducer(lay, clients, o32, o64, plan=plan), o32, o64))
        times = {v[0]: [] for v in variants}
        for _ in range(rounds):
            for te, _, red, _, _ in variants:
                for _ in range(3):
                    red()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    red()
                e1.record()
                torch.cuda.synchronize()
                times[te].append(e0.elapsed_time(e1) / 20 * 1e3)
        ref = variants[0]
        for te, plan, _, o32, o64 in variants:
            ts = sorted(times[te])
            print(json.dumps({"k": k, "tile": te or "auto", "ntiles": plan.info["ntiles"],
                              "us_median": round(ts[len(ts) // 2], 2),
                              "GBps_median": round(nbytes / (ts[len(ts) // 2] * 1e-6) / 1e9, 1),
                              "same": bool(torch.equal(o32, ref[3]) and torch.equal(o64, ref[4]))}),
                  flush=True)
        del clients, variants
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
