"""Does the reduce kernel speed up as the device warms?  Ten consecutive
50-launch windows right after workload generation, then the six variants."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, load_manifest, make_clients  # noqa: E402

dev = torch.device("cuda", 0)
man = load_manifest("wrn16_8_c10")
lay = BucketLayout.from_manifest(man)
cl = make_clients(lay, man, range(20), dev)
o32, o64 = torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1])
red = Reducer(lay, cl, o32, o64)
torch.cuda.synchronize()
t0 = time.perf_counter()
for w in range(12):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        red()
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"window": w, "t_s": round(time.perf_counter() - t0, 3),
                      "us": round(e0.elapsed_time(e1) / 50 * 1e3, 2)}), flush=True)
