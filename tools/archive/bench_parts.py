"""bench.py's secondary lines alone (quick GPU iterations): the other
BASELINE configs + the FedDCT sweep layouts (other_configs) and/or the §8 f3 /
f4 rows (next_rows), one JSON line each.

    python tools/bench_parts.py [other] [next]
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    parts = [p for a in sys.argv[1:] for p in a.split(":")] or ["other", "next"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if "other" in parts:
        print(json.dumps({"other_configs": bench.other_configs(dev)}), flush=True)
    if "next" in parts:
        print(json.dumps({"next_rows": bench.next_rows(dev)}), flush=True)


if __name__ == "__main__":
    main()
