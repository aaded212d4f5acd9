"""Where the drop-in server_aggregate's wall time goes (cfg2 shape: 20
wrn16_8 client modules on the GPU).  Prints one JSON line of per-phase
medians in microseconds."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from feddct_amd import aggregate as A  # noqa: E402
from feddct_amd.arena import get_arena  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import load_manifest  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    man = load_manifest("wrn16_8_c10")
    lay = BucketLayout.from_manifest(man)
    H = bench._holder_class(lay)
    mods = [H().to(dev) for _ in range(20)]
    g = H().to(dev)
    A.server_aggregate(g, mods)
    torch.cuda.synchronize()
    e = A.engine()
    ph = {k: [] for k in ("layout_of", "get_arenas", "pack", "launch", "unpack_mark", "sync",
                          "total")}
    for _ in range(30):
        t0 = time.perf_counter()
        layout = e.layout_of(g)
        t1 = time.perf_counter()
        ga = get_arena(g, layout)
        cas = [get_arena(c, layout) for c in mods]
        t2 = time.perf_counter()
        for c in cas:
            c.pack()
        t3 = time.perf_counter()
        e._reduce_device(layout, ga, cas, None, True)
        t4 = time.perf_counter()
        ga.unpack()
        ga.mark_written()
        for c in cas:
            c.unpack()
            c.mark_written()
        t5 = time.perf_counter()
        torch.cuda.synchronize()
        t6 = time.perf_counter()
        for k, a, b in (("layout_of", t0, t1), ("get_arenas", t1, t2), ("pack", t2, t3),
                        ("launch", t3, t4), ("unpack_mark", t4, t5), ("sync", t5, t6),
                        ("total", t0, t6)):
            ph[k].append((b - a) * 1e6)
    t = []
    for _ in range(30):
        t0 = time.perf_counter()
        A.server_aggregate(g, mods)
        torch.cuda.synchronize()
        t.append((time.perf_counter() - t0) * 1e6)
    out = {k: round(sorted(v)[len(v) // 2], 1) for k, v in ph.items()}
    out["server_aggregate_us"] = round(sorted(t)[len(t) // 2], 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
