"""Experiment: time plan-flag variants of the reduce on one workload
(interleaved rounds in one process).  Usage:
  exp_flags.py LAYOUT N ROUNDS [w] -- NAME=TILE:FLAGS ...
FLAGS is a '|'-joined list of _lib constant suffixes (e.g. ST_PLAIN|BATCH16)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, load_manifest, make_clients  # noqa: E402


def parse_flags(s):
    f = _lib.FA_PLAN_GAPS_ARE_PADDING
    for part in filter(None, s.split("|")):
        f |= getattr(_lib, "FA_PLAN_TUNE_" + part) if not part.isdigit() else int(part)
    return f


def main():
    argv = sys.argv[1:]
    sep = argv.index("--")
    head, specs = argv[:sep], argv[sep + 1:]
    lay_name, n, rounds = head[0], int(head[1]), int(head[2])
    weighted = len(head) > 3 and head[3] == "w"
    dev = torch.device("cuda", 0)
    man = load_manifest(lay_name)
    lay = BucketLayout.from_manifest(man)
    clients = make_clients(lay, man, range(n), dev)
    nbytes = lay.algorithmic_bytes(n)
    w = [1.0 / (i + 2) for i in range(n)] if weighted else None
    variants = []
    for spec in specs:
        name, rest = spec.split("=")
        te, fl = rest.split(":") if ":" in rest else (rest, "")
        plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                         tile_elems=int(te), flags=parse_flags(fl))
        o32, o64 = torch.zeros_like(clients[0][0]), torch.zeros_like(clients[0][1])
        variants.append((name, Reducer(lay, clients, o32, o64, plan=plan, weights=w), o32, o64))
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
    ref = variants[0]
    for name, _, o32, o64 in variants:
        ts = sorted(times[name])
        print(json.dumps({"variant": name, "layout": lay_name, "n": n, "weighted": weighted,
                          "us_median": round(ts[len(ts) // 2], 2), "us_min": round(ts[0], 2),
                          "GBps_median": round(nbytes / (ts[len(ts) // 2] * 1e-6) / 1e9, 1),
                          "same": bool(torch.equal(o32, ref[2]) and torch.equal(o64, ref[3]))}),
              flush=True)


if __name__ == "__main__":
    main()
