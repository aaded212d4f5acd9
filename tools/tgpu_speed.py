"""Launch time of the torch-GPU-order plan (FA_ORDER_TORCH_GPU) on the cfg2,
cfg3 and cfg5 one-GPU workloads, with bit-exactness against torch's own
cuda stack(...).mean(0) of every key (bench.torch_gpu_order_mode)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import joint_manifest, load_manifest, make_clients  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    man = load_manifest("wrn16_8_c10")
    lay = BucketLayout.from_manifest(man)
    cl = make_clients(lay, man, range(20), dev)
    print(json.dumps({"workload": "cfg2", **bench.torch_gpu_order_mode(lay, cl)}), flush=True)
    del cl
    for name, n in (("c10", 5), ("c100", 24)):
        mm = load_manifest(f"wrnsl16_8_sf4_{name}_main")
        pm = load_manifest(f"wrnsl16_8_sf4_{name}_proxy")
        lay = BucketLayout.from_manifest(joint_manifest([mm, pm]))
        cl = make_clients(lay, [(mm, "0."), (pm, "1.")], range(n), dev)
        print(json.dumps({"workload": f"feddct_{name}_n{n}", **bench.torch_gpu_order_mode(lay, cl)}),
              flush=True)
        del cl
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
