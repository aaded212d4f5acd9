"""Per-kernel time and HBM traffic from rocprofv3 runs of tools/round_prof.py
(kernel trace + separate FETCH_SIZE / WRITE_SIZE passes):

    python tools/round_pmc_summary.py <trace_dir> <fetch_dir> <write_dir> <out.json> [ALGO]

(ALGO: the launch's algorithmic bytes for another layout than cfg2, e.g. a
FedDCT sweep layout from round_prof.py's sweep modes.)

Counters are KiB per dispatch (median over dispatches); FETCH_SIZE is also
given x2, the MI355X_MICROARCH.md §HBM correction for wide coalesced
streaming reads on gfx950 (which applies to the reduce's non-temporal
client streams; the broadcast's source reads are plain loads, partly served
beyond L2, so both numbers are listed).  Algorithmic bytes for the cfg2
shape (20 x wrn16_8 C10, B = 43,888,744): reduce N*B + B, broadcast
B + N*B."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_kernels import per_kernel, rows  # noqa: E402

B, N = 43888744, 20
ALGO = {"reduce_kernel": N * B + B, "tgpu_kernel": N * B + B, "bcast_group_kernel": B + N * B,
        "bcast_flat_kernel": B + N * B, "bcast_flat2_kernel": B + N * B,
        "bcast_group2_kernel": B + N * B}


def main():
    trace_dir, fetch_dir, write_dir, out = sys.argv[1:5]
    if len(sys.argv) > 5:
        for t in ALGO:
            ALGO[t] = int(sys.argv[5])
    fetch = per_kernel(fetch_dir, "FETCH_SIZE")
    write = per_kernel(write_dir, "WRITE_SIZE")
    res = []
    for r in rows(trace_dir, "*kernel_stats.csv"):
        name = r["Name"]
        tag = next((t for t in ALGO if t in name), None)
        if tag is None:
            continue
        f, w = fetch.get(name), write.get(name)
        avg = float(r["AverageNs"]) / 1e3
        e = {"kernel": name, "calls": int(r["Calls"]), "avg_us": round(avg, 2),
             "min_us": round(float(r["MinNs"]) / 1e3, 2), "algorithmic_bytes": ALGO[tag],
             "GBps_avg": round(ALGO[tag] / (avg * 1e-6) / 1e9, 1),
             "fetch_bytes_raw": None if f is None else f * 1024,
             "fetch_bytes_x2": None if f is None else 2 * f * 1024,
             "write_bytes": None if w is None else w * 1024}
        res.append(e)
    with open(out, "w") as fo:
        json.dump({"counters": "KiB per dispatch, median", "kernels": res}, fo, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
