"""Where BASELINE config 3's reduce time goes (r05).

cfg3 = FedDCT sf4 C10, 5 slots x (main + proxy) in one joint bucket (11.0 M
floats, 264.4 MB algorithmic per launch).  Same process, HIP events, each
timing the median of 5 passes of K launches, client sets rotated past the
256 MiB MALL where the working set fits it:

  cfg3            the product reduce (fa_reduce, the shipped launch shape)
  cfg3_vec_only   its vector tiles alone (the packed scalar tiles left out)
  cfg3_scalar_only  its packed scalar tiles alone
  flat_N5_<MB>    one flat fp32 tensor, N = 5 clients, sizes 1/4 .. 4 x
                  cfg3's bucket: the linear fit time = a + bytes / rate
                  separates the per-launch fixed cost (ramp + drain) from
                  the streaming rate
  read_probe_<MB> fa_read_probe_f32 over the same bytes in the reduce's tile
                  shape (nothing computed or stored): the read ceiling at
                  that size

  python tools/cfg3_anatomy.py [K]        -> JSON lines
  python tools/cfg3_anatomy.py prof K     -> only the cfg3 reduce, K launches
                                            (for rocprofv3 kernel trace / PMC)
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, joint_manifest, load_manifest, make_clients  # noqa: E402

N = 5


def timed(fns, k, passes=5):
    ts = []
    c = 0
    for _ in range(passes):
        for _ in range(3):
            fns[c % len(fns)]()
            c += 1
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(k):
            fns[c % len(fns)]()
            c += 1
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / k * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def cfg3(dev):
    mans = [load_manifest("wrnsl16_8_sf4_c10_main"), load_manifest("wrnsl16_8_sf4_c10_proxy")]
    lay = BucketLayout.from_manifest(joint_manifest(mans))
    sets = [make_clients(lay, list(zip(mans, ("0.", "1."))), range(N), dev) for _ in range(2)]
    return lay, sets


def line(**kw):
    print(json.dumps({"exp": "cfg3_anatomy", **kw}), flush=True)


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if len(sys.argv) > 1 and sys.argv[1] == "prof":
        k = int(sys.argv[2])
        lay, sets = cfg3(dev)
        reds = [Reducer(lay, cl, torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1]))
                for cl in sets]
        for i in range(k):
            reds[i % 2]()
        torch.cuda.synchronize()
        print(f"cfg3 reduce: {k} launches, {lay.algorithmic_bytes(N)} algorithmic bytes each")
        return
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    lay, sets = cfg3(dev)
    nb = lay.algorithmic_bytes(N)
    reds = [Reducer(lay, cl, torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1])) for cl in sets]
    plan = reds[0].plan
    info, tiles = _lib.build_tiles_host(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel)
    ntiles, slots = plan.launch_shape(N)
    us = timed(reds, k)
    line(case="cfg3", us=round(us, 2), bytes=nb, frac=round(nb / us / 8e6, 4),
         launch_tiles=ntiles, slots=slots, rounds=round(ntiles / max(1, slots), 3),
         vector_tiles=int(info["ntiles_cascade"]), scalar_tiles=int(info["ntiles_tail"]),
         scalar_columns=int(tiles[tiles[:, 2] != 0][:, 1].sum()))
    for part, sel in (("cfg3_vec_only", tiles[:, 2] == 0), ("cfg3_scalar_only", tiles[:, 2] != 0)):
        p = _lib.Plan(None, lay.f32_numel, None, lay.i64_numel, 0, tiles=tiles[sel])
        rs = [Reducer(lay, cl, torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1]), plan=p)
              for cl in sets]
        line(case=part, us=round(timed(rs, k), 2), tiles=int(sel.sum()))
    del sets, reds
    torch.cuda.empty_cache()
    # flat N = 5 tensors from 1/4 to 4 x cfg3's bucket; the read probe beside
    base = lay.f32_numel // 2048 * 2048
    xs, ys = [], []
    for mult in (0.25, 0.5, 1, 2, 4):
        m = int(base * mult) // 2048 * 2048
        rot = max(1, int(np.ceil(600e6 / (4 * m * (N + 1)))))
        flay = BucketLayout([("x", (m,), "float32")])
        fsets = []
        for r in range(rot):
            cl = [(torch.empty(m, device=dev).uniform_(-1, 1), torch.zeros(1, dtype=torch.int64,
                                                                           device=dev))
                  for _ in range(N)]
            fsets.append(Reducer(flay, cl, torch.zeros(m, device=dev),
                                 torch.zeros(1, dtype=torch.int64, device=dev)))
        fb = flay.algorithmic_bytes(N)
        t = timed(fsets, k)
        xs.append(fb)
        ys.append(t)
        line(case=f"flat_N5_{fb / 1e6:.0f}MB", us=round(t, 2), bytes=fb,
             frac=round(fb / t / 8e6, 4), rotated_sets=rot)
        # the probe rotated over as many buffers (past the MALL) as the reduce
        bigs = [torch.empty(fb // 4, device=dev).uniform_(-1, 1) for _ in range(rot)]
        sink = torch.zeros(256, device=dev)
        probes = [lambda big=big: _lib.check(_lib.lib.fa_read_probe_f32(
            big.data_ptr(), big.numel(), sink.data_ptr(), 0,
            torch.cuda.current_stream().cuda_stream)) for big in bigs]
        tp = timed(probes, k)
        line(case=f"read_probe_{fb / 1e6:.0f}MB", us=round(tp, 2), bytes=fb,
             TBps=round(fb / tp / 1e6, 3))
        del fsets, bigs, probes
        torch.cuda.empty_cache()
    a, b = np.polyfit(np.array(xs, float), np.array(ys, float), 1)
    line(case="flat_N5_linear_fit", us_fixed=round(float(b), 2),
         marginal_TBps=round(1.0 / float(a) / 1e6, 3),
         note="time = us_fixed + bytes / marginal rate, over the five flat sizes")


if __name__ == "__main__":
    main()
