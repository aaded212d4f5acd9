"""Summarise rocprofv3 output for the reduce kernel into profiles/.

    python tools/pmc_summary.py <kernel_trace_dir> <fetch_dir> <write_dir> <out.json> [bench_log]
    env FA_PMC_KERNEL / FA_PMC_WORKLOAD / FA_PMC_ALG_BYTES / FA_PMC_COMMAND:
    another kernel or workload than the headline (e.g. cfg3 from
    tools/cfg3_prof.sh, the proximal term's kernels from tools/prox_prof.sh)

FETCH_SIZE / WRITE_SIZE come from separate --pmc passes (they do not fit in
one pass on gfx950).  Corrections per MI355X_MICROARCH.md §HBM: both are in
KiB; FETCH_SIZE reports exactly half the bytes of a wide (16 B/lane)
coalesced streaming read on gfx950, so it is doubled; WRITE_SIZE is exact for
16-B-per-lane streaming stores.
"""
import csv
import glob
import json
import os
import sys
import time

KERNEL = os.environ.get("FA_PMC_KERNEL", "reduce_kernel")


def rows(d, pattern):
    out = []
    for p in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def counter_per_dispatch(d, counter):
    vals = {}
    for r in rows(d, "*counter_collection.csv"):
        if KERNEL not in r.get("Kernel_Name", "") or r.get("Counter_Name") != counter:
            continue
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    trace_dir, fetch_dir, write_dir, out = sys.argv[1:5]
    bench_line = None
    if len(sys.argv) > 5 and os.path.exists(sys.argv[5]):
        for line in open(sys.argv[5]):
            if line.startswith("{"):
                bench_line = json.loads(line)
    stats = [r for r in rows(trace_dir, "*kernel_stats.csv") if KERNEL in r["Name"]]
    fetch = counter_per_dispatch(fetch_dir, "FETCH_SIZE")
    write = counter_per_dispatch(write_dir, "WRITE_SIZE")
    med = lambda v: sorted(v)[len(v) // 2] if v else None  # noqa: E731
    fk, wk = med(fetch), med(write)
    res = {
        "workload": os.environ.get("FA_PMC_WORKLOAD", "wrn16_8_c10/n20"),
        "kernel": stats[0]["Name"] if stats else None,
        "calls": int(stats[0]["Calls"]) if stats else None,
        "avg_ns": float(stats[0]["AverageNs"]) if stats else None,
        "min_ns": float(stats[0]["MinNs"]) if stats else None,
        "FETCH_SIZE_KiB_raw": fk, "WRITE_SIZE_KiB": wk,
        "fetch_bytes_corrected": None if fk is None else 2 * fk * 1024,
        "write_bytes": None if wk is None else wk * 1024,
        "hbm_bytes_per_launch": None if fk is None or wk is None else 2 * fk * 1024 + wk * 1024,
        "algorithmic_bytes_per_launch": int(os.environ.get("FA_PMC_ALG_BYTES",
                                                            20 * 43888744 + 43888744)),
        "correction": "FETCH_SIZE x2 (gfx950 wide-stream half count), KiB x1024",
        # the HIP-event launch time bench.py measured inside the profiled run
        "bench_kernel_us_same_run": (bench_line or {}).get("roofline", {}).get("kernel_us"),
        "command": os.environ.get("FA_PMC_COMMAND",
                                  "rocprofv3 --kernel-trace --stats -- python3 bench.py "
                                  "--kernel-only --no-cpu-baseline --steps 100 --warmup 100"),
        # where and when the counters were taken (the bench line cites them)
        "date_utc": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()),
        "host": os.uname().nodename,
        "gpu": (bench_line or {}).get("gpu"),
        # the commit of the profiled tree (FA_PROFILE_TREE, set by the caller:
        # the GPU box has no .git)
        "tree": os.environ.get("FA_PROFILE_TREE"),
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
