"""Cost of each native multi-GPU round form on ONE rank (Comm.single(): every
exchange is empty), against the plain single-GPU reduce of the same 20
wrn16_8 clients: what the round's own kernels, chunking and host issue add
before any xGMI traffic — the local floor of bench N>1.  One JSON line per
form: GPU time per step (HIP events over K steps) and host issue time per
step (wall time of the K step() calls, no sync inside).

    python tools/native_round_cost.py [K] [--no-graphs] [--only=form,form]
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd import comm as C  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, load_manifest, make_clients  # noqa: E402


def timed(fn, k, w=10):
    for _ in range(w):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(k):
        fn()
    host = time.perf_counter() - t0
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / k, host * 1e6 / k


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 50
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    man = load_manifest("wrn16_8_c10")
    lay = BucketLayout.from_manifest(man)
    n = 20
    cl = make_clients(lay, man, range(n), dev)
    l32, l64 = [c[0] for c in cl], [c[1] for c in cl]
    ref32, ref64 = torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1])
    red = Reducer(lay, cl, ref32, ref64)
    graphs = "--no-graphs" not in sys.argv   # r03: rounds replayed from captured graphs
    comm = C.Comm.single()
    comm.set_graphs(graphs)
    forms = {"plain_reduce": lambda o32, o64: Reducer(lay, cl, o32, o64, plan=red.plan)}
    forms["blocked"] = lambda o32, o64: C.NativeBlockedAggregator(
        lay, l32, l64, n, o32, o64, comm, final="reduce", root=0).step
    for ch in (1, 4, 16):
        forms[f"chained_{ch}"] = (lambda ch: lambda o32, o64: C.NativeChainedAggregator(
            lay, l32, l64, n, o32, o64, comm, nchunks=ch, final="reduce", root=0).step)(ch)
    forms["sharded_8_reduce"] = lambda o32, o64: C.NativeShardedAggregator(
        lay, l32, l64, n, o32, o64, comm, nchunks=8, final="reduce").step
    forms["sharded_8_rs_gather"] = lambda o32, o64: C.NativeShardedAggregator(
        lay, l32, l64, n, o32, o64, comm, nchunks=8, final="reduce",
        exchange=C.FA_XCHG_RS_GATHER).step
    forms["striped"] = lambda o32, o64: C.NativeStripedAggregator(
        lay, l32, l64, n, o32, o64, comm, final="reduce").step
    nb = lay.algorithmic_bytes(n)
    red()
    torch.cuda.synchronize()
    mask = torch.zeros(lay.f32_numel, dtype=torch.bool, device=dev)
    for o, m in lay.segs32:
        mask[int(o):int(o + m)] = True
    only = [a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--only=")]
    for name, make in forms.items():
        if only and name not in only[0].split(","):
            continue
        o32 = torch.full_like(ref32, float("nan"))
        o64 = torch.zeros_like(ref64)
        fn = make(o32, o64)
        us, host = timed(fn, k)
        exact = bool(torch.equal(o32[mask].view(torch.int32), ref32[mask].view(torch.int32))
                     and torch.equal(o64, ref64))
        print(json.dumps({"form": name, "graphs": graphs, "gpu_us": round(us, 1),
                          "host_issue_us": round(host, 1),
                          "GBps": round(nb / us / 1e3, 1), "bit_exact": exact}), flush=True)
    comm.close()


if __name__ == "__main__":
    main()
