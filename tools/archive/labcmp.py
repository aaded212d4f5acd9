"""The product kernel on the lab's shapes (tools/reducelab.hip), same box:
cfg3 (N=5 joint FedDCT bucket) with 1 set and with 2 rotated sets, and the
cfg2 headline, so the lab's numbers and the product's can be compared."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from feddct_amd import _lib  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import joint_manifest, load_manifest, make_clients  # noqa: E402
from tune_r2 import sweep  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    mm, pm = load_manifest("wrnsl16_8_sf4_c10_main"), load_manifest("wrnsl16_8_sf4_c10_proxy")
    lay = BucketLayout.from_manifest(joint_manifest([mm, pm]))
    sets = [make_clients(lay, [(mm, "0."), (pm, "1.")], range(5), dev) for _ in range(2)]
    nb = lay.algorithmic_bytes(5)
    sweep("cfg3_n5_rot2", lay, sets, None, nb, 3, (1, 2), (1, 8))
    sweep("cfg3_n5_one_set", lay, sets[:1], None, nb, 3, (1, 2), (1, 8))
    del sets
    torch.cuda.empty_cache()
    man = load_manifest("wrn16_8_c10")
    lay = BucketLayout.from_manifest(man)
    cl = make_clients(lay, man, range(20), dev)
    sweep("cfg2_one_set", lay, [cl], None, lay.algorithmic_bytes(20), 3, (1, 2), (8, 16))


if __name__ == "__main__":
    main()
