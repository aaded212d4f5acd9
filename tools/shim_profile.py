"""Where the drop-in server_aggregate's wall time goes (r04): the bound-round
fast path (aggregate.Engine.try_bound_round) on the cfg2 shape (20 wrn16_8
client modules), the cfg3 shape (FedDCT, 5 slots of wrnsl16_8 sf4 C10
main + proxy) and the cfg5 shape (24 slots, C100).  Per shape one JSON line
of per-phase medians in microseconds: the binding's cheap check
(same_modules: module and arena identities), the reduce launch call (ctypes
fa_reduce), the per-tensor check that runs while the GPU reduces
(views_intact: dict tags + data pointers in one C call), the broadcast
launch call, the version bumps (these five: the r04 Python form of the fast
path), native_call (the same sequence as one _fa_shim.bound_round call, the
drop-in's form), the wall of a whole drop-in call with its sync, and the GPU
time of the round alone (its two launches back to back).  r06: check_tags /
check_keys / check_all — the native pre-launch check alone (_fa_shim.round_check:
the dicts' version tags, the tensors' cached TensorImpl storage fields, both).
Usage: shim_profile.py [REPS]"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from feddct_amd import _fa_shim, _lib  # noqa: E402
from feddct_amd import aggregate as A  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import load_manifest  # noqa: E402


def phases(call, reps):
    e = A.engine()
    call()
    torch.cuda.synchronize()
    rb = e._round
    assert rb is not None
    ga = rb.arenas[0]()
    g = rb.gref()
    cms = [r() for r in rb.crefs]
    ph = {k: [] for k in ("same_modules", "launch_reduce", "views_intact", "launch_bcast",
                          "bump", "wall")}
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ok = rb.same_modules(g, cms, e.order, False)
        t1 = time.perf_counter()
        e._launch(rb.plan, rb.a32, rb.a64, rb.n, None, ga.f32.data_ptr(), ga.i64.data_ptr(),
                  0, rb.dev)
        t2 = time.perf_counter()
        ok &= rb.views_intact()
        t3 = time.perf_counter()
        e._launch(rb.plan, rb.a32, rb.a64, rb.n, None, ga.f32.data_ptr(), ga.i64.data_ptr(),
                  _lib.FA_F_BCAST_ONLY, rb.dev)
        t4 = time.perf_counter()
        _fa_shim.bump_versions(rb.written)
        t5 = time.perf_counter()
        torch.cuda.synchronize()
        assert ok
        for k, a, b in (("same_modules", t0, t1), ("launch_reduce", t1, t2),
                        ("views_intact", t2, t3), ("launch_bcast", t3, t4), ("bump", t4, t5)):
            ph[k].append((b - a) * 1e6)
    # r06: bound_round's pre-launch check alone (dict tags / tensor ViewKeys / both)
    for what, key in ((0, "check_tags"), (1, "check_keys"), (2, "check_all")):
        ph[key] = []
        for _ in range(reps if rb.native is not None else 0):
            t0 = time.perf_counter()
            assert _fa_shim.round_check(rb.native, what)
            ph[key].append((time.perf_counter() - t0) * 1e6)
    # the same round as one C call (the drop-in's path since r04 session 3)
    ph["native_call"] = []
    for _ in range(reps if rb.native is not None else 0):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        assert _fa_shim.bound_round(rb.native, None) == 1
        ph["native_call"].append((time.perf_counter() - t0) * 1e6)
        torch.cuda.synchronize()
    for _ in range(reps):
        t0 = time.perf_counter()
        call()
        torch.cuda.synchronize()
        ph["wall"].append((time.perf_counter() - t0) * 1e6)
    out = {k: round(sorted(v)[len(v) // 2], 1) for k, v in ph.items() if v}
    gpu = bench._bound_round_gpu(out["wall"] * 1e-6)
    out.update(gpu)
    out["bound_tensors"] = len(rb.tensors)
    out["bound_dicts"] = len(rb.dicts)
    return out


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lay = BucketLayout.from_manifest(load_manifest("wrn16_8_c10"))
    H = bench._holder_class(lay)
    mods = [H().to(dev) for _ in range(20)]
    g = H().to(dev)
    print(json.dumps({"shape": "cfg2_fedavg_n20", **phases(lambda: A.server_aggregate(g, mods),
                                                           reps)}), flush=True)
    del mods, g
    for n, cls in ((5, 10), (24, 100)):
        (_, _, gm, mains), (_, _, gp, proxies) = bench._feddct_modules(dev, n=n, classes=cls)
        print(json.dumps({"shape": f"feddct_c{cls}_n{n}", **phases(
            lambda: A.server_aggregate_split(gm, gp, mains, proxies), reps)}), flush=True)
        del mains, proxies, gm, gp


if __name__ == "__main__":
    main()
