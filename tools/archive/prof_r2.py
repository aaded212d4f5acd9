"""Profiling driver: the cfg2 mean, the cfg2
client-size-weighted launch and the cfg3 FedDCT launch (N=5, joint bucket,
2 rotated sets), K launches each, under rocprofv3 (kernel trace, or one PMC
counter per run).  Each workload runs a distinct reduce_kernel
instantiation, so the per-kernel summaries separate them:
  cfg2   reduce_kernel<2, 16, false, false, 3, false>
  cfg2w  reduce_kernel<2, 8,  false, true,  3, false>  (policy at the time)
  cfg3   reduce_kernel<2, 8,  false, false, 3, false>
Writes gpurun_out/prof_r2_workloads.json (algorithmic bytes per launch)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, joint_manifest, load_manifest, make_clients  # noqa: E402


def run(red, k):
    for _ in range(5):
        red()
    torch.cuda.synchronize()
    for _ in range(k):
        red()
    torch.cuda.synchronize()


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    dev = torch.device("cuda", 0)
    info = {}
    man = load_manifest("wrn16_8_c10")
    lay = BucketLayout.from_manifest(man)
    cl = make_clients(lay, man, range(20), dev)
    o32, o64 = torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1])
    run(Reducer(lay, cl, o32, o64), k)
    info["cfg2"] = lay.algorithmic_bytes(20)
    s = np.arange(1, 21, dtype=np.float64)
    run(Reducer(lay, cl, o32, o64, weights=(s / s.sum()).astype(np.float32)), k)
    info["cfg2w"] = lay.algorithmic_bytes(20)
    del cl
    mm, pm = load_manifest("wrnsl16_8_sf4_c10_main"), load_manifest("wrnsl16_8_sf4_c10_proxy")
    lay = BucketLayout.from_manifest(joint_manifest([mm, pm]))
    sets = [make_clients(lay, [(mm, "0."), (pm, "1.")], range(5), dev) for _ in range(2)]
    reds = [Reducer(lay, c, torch.zeros_like(c[0][0]), torch.zeros_like(c[0][1])) for c in sets]
    j = [0]

    def rot():
        reds[j[0] % 2]()
        j[0] += 1
    run(rot, k)
    info["cfg3"] = lay.algorithmic_bytes(5)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "prof_r2_workloads.json"), "w") as f:
        json.dump(info, f)
    print(json.dumps(info))


if __name__ == "__main__":
    main()
