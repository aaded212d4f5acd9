"""Per-kernel summary of rocprofv3 runs (kernel trace + separate FETCH_SIZE
and WRITE_SIZE passes), for every reduce_kernel instantiation found:

    python tools/pmc_kernels.py <trace_dir> <fetch_dir> <write_dir> <out.json> [map.json]

Corrections per MI355X_MICROARCH.md §HBM: counters in KiB; FETCH_SIZE
reports half the bytes of a wide coalesced streaming read on gfx950 (x2);
WRITE_SIZE exact for 16-B stores.  ``map.json``: {label: algorithmic bytes}
with labels matched to template arguments below."""
import csv
import glob
import json
import os
import sys

LABELS = {"<2, 16, false, false, 3, false>": "cfg2",
          "<2, 8, false, true, 3, false>": "cfg2w",
          "<2, 16, false, true, 3, false>": "cfg2w",
          "<1, 8, false, true, 3, false>": "cfg2w",
          "<1, 4, false, true, 3, false>": "cfg2w",
          "<2, 8, false, false, 3, false>": "cfg3",
          "<4, 8, false, false, 3, false>": "cfg3",
          "<4, 4, false, false, 3, false>": "cfg3",
          "<2, 4, false, false, 3, false>": "cfg3",
          "<1, 4, false, false, 3, false>": "cfg3",
          "<4, 1, false, false, 3, false>": "cfg3"}


def rows(d, pattern):
    out = []
    for p in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def per_kernel(d, counter):
    vals = {}
    for r in rows(d, "*counter_collection.csv"):
        if r.get("Counter_Name") != counter:
            continue
        key = (r.get("Kernel_Name", ""), r.get("Dispatch_Id") or r.get("Correlation_Id"))
        vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    by = {}
    for (name, _), v in vals.items():
        by.setdefault(name, []).append(v)
    return {k: sorted(v)[len(v) // 2] for k, v in by.items()}


def main():
    trace_dir, fetch_dir, write_dir, out = sys.argv[1:5]
    algo = json.load(open(sys.argv[5])) if len(sys.argv) > 5 else {}
    fetch = per_kernel(fetch_dir, "FETCH_SIZE")
    write = per_kernel(write_dir, "WRITE_SIZE")
    res = []
    for r in rows(trace_dir, "*kernel_stats.csv"):
        name = r["Name"]
        if "reduce_kernel" not in name:
            continue
        label = next((v for k, v in LABELS.items() if k in name), None)
        f = next((v for k, v in fetch.items() if k == name), None)
        w = next((v for k, v in write.items() if k == name), None)
        e = {"kernel": name, "label": label, "calls": int(r["Calls"]),
             "avg_us": float(r["AverageNs"]) / 1e3, "min_us": float(r["MinNs"]) / 1e3,
             "hbm_bytes_per_launch": None if f is None or w is None else 2 * f * 1024 + w * 1024}
        if label in algo:
            e["algorithmic_bytes"] = algo[label]
            e["GBps_avg"] = round(algo[label] / (e["avg_us"] * 1e-6) / 1e9, 1)
            if e["hbm_bytes_per_launch"]:
                e["traffic_over_algorithmic"] = round(e["hbm_bytes_per_launch"] / algo[label], 4)
        res.append(e)
    with open(out, "w") as fo:
        json.dump({"correction": "FETCH_SIZE x2 (gfx950), KiB x1024", "kernels": res}, fo,
                  indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
