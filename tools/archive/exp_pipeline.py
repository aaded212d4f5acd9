"""Experiment (r03 session 3): the host-ingress pipeline's chunk cut.  Each
chunk costs one H2D copy per client (~20 us each measured), and the round's
tail after the last upload is the last chunk's reduce + download (+ its CPU
fan-out with the broadcast).  cfg2 (20 wrn16_8 clients in pinned host
memory), one process, interleaved; the serial round for reference.

    python tools/archive/exp_pipeline.py [REPS]
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.pipeline import HostPipeline  # noqa: E402
from feddct_amd.workload import Reducer, load_manifest, make_clients  # noqa: E402

CUTS = {
    "taper5": (0.5, 0.25, 0.125, 0.0625, 0.0625),
    "taper4_75": (0.75, 0.125, 0.0625, 0.0625),
    "taper4_625": (0.625, 0.25, 0.0625, 0.0625),
    "taper3_875": (0.875, 0.0625, 0.0625),
    "taper2": (0.9375, 0.0625),
    "taper3_even_tail": (0.8, 0.1, 0.1),
}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    man = load_manifest("wrn16_8_c10")
    lay = BucketLayout.from_manifest(man)
    n = 20
    cl = make_clients(lay, man, range(n), dev)
    o32, o64 = torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1])
    red = Reducer(lay, cl, o32, o64)
    host = [(c[0].cpu().pin_memory(), c[1].cpu().pin_memory()) for c in cl]
    h32 = [h[0] for h in host]
    h64 = [h[1] for h in host]
    oh32 = torch.empty_like(o32, device="cpu").pin_memory()
    oh64 = torch.empty_like(o64, device="cpu").pin_memory()
    nb = lay.algorithmic_bytes(n)

    def serial():
        for (a, b), (d32, d64) in zip(host, cl):
            d32.copy_(a, non_blocking=True)
            d64.copy_(b, non_blocking=True)
        red()
        oh32.copy_(o32, non_blocking=True)
        oh64.copy_(o64, non_blocking=True)
        torch.cuda.synchronize()

    fns = {"serial": serial}
    pipes = {}
    for name, fr in CUTS.items():
        p = pipes[name] = HostPipeline(lay, n, dev, fractions=fr)
        fns[name] = (lambda p: lambda: p.run(h32, h64, oh32, oh64))(p)
        # the broadcast into other host buckets than the inputs (same traffic)
        fns[name + "_bcast"] = (lambda p: lambda: p.run(h32, h64, oh32, oh64, bc32, bc64))(p)
    bc32 = [t.clone().pin_memory() for t in h32]
    bc64 = [t.clone().pin_memory() for t in h64]
    times = {k: [] for k in fns}
    for _ in range(3):
        for k, fn in fns.items():
            fn()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            times[k].append((time.perf_counter() - t0) / reps)
        print("round", file=sys.stderr, flush=True)
    red()
    torch.cuda.synchronize()
    for k, ts in times.items():
        t = sorted(ts)[1]
        rec = {"exp": "pipeline", "variant": k, "ms": round(t * 1e3, 3),
               "GBps": round(nb / t / 1e9, 2)}
        print(json.dumps(rec), flush=True)
    print(json.dumps({"exp": "pipeline", "bit_exact": bool(torch.equal(oh32, o32.cpu())),
                      "bcast_bit_exact": bool(all(torch.equal(b, oh32) for b in bc32)),
                      "torch_threads": torch.get_num_threads()}), flush=True)


if __name__ == "__main__":
    main()
