"""Rehearse the exact column-striped round (feddct_amd.dist.StripedAggregator,
SURVEY §8 e2) on ONE GPU with 2 gloo ranks, with a stack dump if it stalls
(debug aid).  Run under torch.distributed.run --nproc-per-node 2."""
import faulthandler
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from feddct_amd.dist import StripedAggregator, shard_range  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, load_manifest, make_clients  # noqa: E402


def main():
    faulthandler.dump_traceback_later(float(os.environ.get("PROBE_TIMEOUT", "60")), exit=True)
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    name = os.environ.get("PROBE_LAYOUT", "wrnsl16_8_sf4_c10_main")
    n_total = int(os.environ.get("PROBE_N", "6"))
    man = load_manifest(name)
    lay = BucketLayout.from_manifest(man)
    lo, hi = shard_range(n_total, world, rank)
    cl = make_clients(lay, man, range(lo, hi), dev)
    out32 = torch.zeros_like(cl[0][0])
    out64 = torch.zeros_like(cl[0][1])
    agg = StripedAggregator(lay, n_total, out32, out64, final="reduce")
    print(rank, "step_device", flush=True)
    agg.step_device([c[0] for c in cl], [c[1] for c in cl])
    torch.cuda.synchronize()
    print(rank, "done", flush=True)
    if rank == 0:
        allc = make_clients(lay, man, range(n_total), dev)
        e32, e64 = torch.zeros_like(out32), torch.zeros_like(out64)
        Reducer(lay, allc, e32, e64)()
        torch.cuda.synchronize()
        print("bit-exact", bool(torch.equal(out32, e32) and torch.equal(out64, e64)), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    faulthandler.cancel_dump_traceback_later()


if __name__ == "__main__":
    main()
