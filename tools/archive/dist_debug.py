"""Rehearse feddct_amd.dist on ONE GPU with 2 gloo ranks (debug aid)."""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from feddct_amd.dist import ShardedAggregator, shard_range  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, load_manifest, make_clients  # noqa: E402


def main():
    sync = os.environ.get("SYNC", "0") == "1"
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    man = load_manifest("wrnsl16_8_sf4_c10_main")
    lay = BucketLayout.from_manifest(man)
    n_total = 6
    lo, hi = shard_range(n_total, world, rank)
    cl = make_clients(lay, man, range(lo, hi), dev)
    out32 = torch.zeros_like(cl[0][0])
    out64 = torch.zeros_like(cl[0][1])
    agg = ShardedAggregator(lay, [c[0] for c in cl], [c[1] for c in cl], n_total, out32, out64,
                            nchunks=2)
    if sync:
        orig = agg.backend.partial_sum

        def ps(*a):
            orig(*a)
            torch.cuda.synchronize()
        agg.backend.partial_sum = ps
    agg.step()
    torch.cuda.synchronize()
    allc = make_clients(lay, man, range(n_total), dev)
    e32 = torch.zeros_like(out32)
    e64 = torch.zeros_like(out64)
    Reducer(lay, allc, e32, e64)()
    torch.cuda.synchronize()
    # local partial for reference
    p = torch.zeros_like(out32)
    Reducer(lay, cl, p, torch.zeros_like(out64), flags=2)()
    torch.cuda.synchronize()
    print(rank, "sync", sync, "max|out-exact|", float((out32 - e32).abs().max()),
          "i64 eq", bool(torch.equal(out64, e64)), out64[:4].tolist(), e64[:4].tolist(),
          "partial[:3]", p[:3].tolist(), "out[:3]", out32[:3].tolist(), "exact[:3]", e32[:3].tolist(),
          flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
