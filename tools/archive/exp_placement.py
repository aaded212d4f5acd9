"""Experiment: does where the client buckets sit in HBM change the reduce
kernel's bandwidth?  Same cfg2 workload (20 x wrn16_8 C10), clients placed
(a) as separate torch allocations, (b) packed in one allocation at various
strides/skews.  Interleaved rounds in one process; one JSON line per variant."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, fill_client, load_manifest, make_clients  # noqa: E402


def main():
    lay_name = sys.argv[1] if len(sys.argv) > 1 else "wrn16_8_c10"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    dev = torch.device("cuda", 0)
    man = load_manifest(lay_name)
    lay = BucketLayout.from_manifest(man)
    nbytes = lay.algorithmic_bytes(n)
    numel = lay.f32_numel
    plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel)
    variants = []
    sep = make_clients(lay, man, range(n), dev)
    print(json.dumps({"separate_addrs_mod_2M": [c[0].data_ptr() % (2 << 20) for c in sep],
                      "separate_deltas": [sep[i + 1][0].data_ptr() - sep[i][0].data_ptr()
                                          for i in range(n - 1)]}))
    o32, o64 = torch.zeros_like(sep[0][0]), torch.zeros_like(sep[0][1])
    variants.append(("separate", Reducer(lay, sep, o32, o64, plan=plan), o32, o64))
    MB2 = (2 << 20) // 4
    rnd = lambda x, a: (x + a - 1) // a * a  # noqa: E731
    specs = [("packed256B", rnd(numel, 64), 0), ("packed2M", rnd(numel, MB2), 0),
             ("2M+skew4K", rnd(numel, MB2), 1024), ("2M+skew64K", rnd(numel, MB2), 16384),
             ("2M+skew1M", rnd(numel, MB2), MB2 // 2), ("pow2_64M", 16 << 20, 0),
             ("pow2_64M+skew4K", 16 << 20, 1024), ("2M+skew256B", rnd(numel, MB2), 64)]
    bigs = []
    for name, stride, skew in specs:
        total = n * stride + n * skew + 64
        big = torch.zeros(total, dtype=torch.float32, device=dev)
        bigs.append(big)
        cl = []
        for i in range(n):
            f32 = big[i * stride + i * skew:i * stride + i * skew + numel]
            i64 = torch.zeros(max(lay.i64_numel, 1), dtype=torch.int64, device=dev)
            fill_client(lay, man, f32, i64, i)
            cl.append((f32, i64))
        a32, a64 = torch.zeros_like(o32), torch.zeros_like(o64)
        variants.append((name, Reducer(lay, cl, a32, a64, plan=plan), a32, a64))
    torch.cuda.synchronize()
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
    for name, _, a32, a64 in variants:
        ts = sorted(times[name])
        print(json.dumps({"variant": name, "n": n, "us_median": round(ts[len(ts) // 2], 2),
                          "us_min": round(ts[0], 2),
                          "GBps_median": round(nbytes / (ts[len(ts) // 2] * 1e-6) / 1e9, 1),
                          "same": bool(torch.equal(a32, o32) and torch.equal(a64, o64))}))


if __name__ == "__main__":
    main()
