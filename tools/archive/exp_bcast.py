"""Experiment: the round's broadcast (train_fedavg.py:148-149) — the default
FA_F_BCAST (reduce launch + a flat broadcast launch over client groups),
the same groups through the tile table, one workgroup per tile (r01), the
fused form
(FA_PLAN_TUNE_FUSED_BCAST, under several plan tuning flags) and the reduce
followed by the standalone whole-bucket broadcast kernel (fa_broadcast_f32; the int64
keys, 128 B, are left out of that variant), cfg2 shape, interleaved rounds
in one process, HIP events.  Usage: exp_bcast.py ROUNDS"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, load_manifest, make_clients  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    dev = torch.device("cuda", 0)
    man = load_manifest("wrn16_8_c10")
    lay = BucketLayout.from_manifest(man)
    n = 20
    clients = make_clients(lay, man, range(n), dev)
    o32, o64 = torch.zeros_like(clients[0][0]), torch.zeros_like(clients[0][1])
    moved = (n * lay.f32_numel * 4 + n * max(lay.i64_numel, 0) * 8) + (n + 1) * (
        lay.f32_numel * 4 + lay.i64_numel * 8)
    B = _lib.FA_F_BCAST

    def plan(te=0, fl=0):
        return _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel, tile_elems=te,
                         flags=_lib.FA_PLAN_GAPS_ARE_PADDING | fl)

    F = _lib.FA_PLAN_TUNE_FUSED_BCAST
    variants = {
        "default": Reducer(lay, clients, o32, o64, flags=B, plan=plan()),
        "tiles_r01": Reducer(lay, clients, o32, o64, flags=B,
                             plan=plan(0, _lib.FA_PLAN_TUNE_BCAST_TILES)),
        "table": Reducer(lay, clients, o32, o64, flags=B,
                         plan=plan(0, _lib.FA_PLAN_TUNE_BCAST_TABLE)),
        # the reduce's result stores temporal / sc1, so the broadcast that
        # follows may find its source in the caches
        "st_plain": Reducer(lay, clients, o32, o64, flags=B,
                            plan=plan(0, _lib.FA_PLAN_TUNE_ST_PLAIN)),
        "st_sc1": Reducer(lay, clients, o32, o64, flags=B,
                          plan=plan(0, _lib.FA_PLAN_TUNE_ST_SC1)),
        "fused": Reducer(lay, clients, o32, o64, flags=B, plan=plan(0, F)),
        "fused_tile1024": Reducer(lay, clients, o32, o64, flags=B, plan=plan(1024, F)),
        "fused_tile2048": Reducer(lay, clients, o32, o64, flags=B, plan=plan(2048, F)),
        "fused_st_plain": Reducer(lay, clients, o32, o64, flags=B,
                                  plan=plan(0, F | _lib.FA_PLAN_TUNE_ST_PLAIN)),
        "fused_batch8": Reducer(lay, clients, o32, o64, flags=B,
                                plan=plan(0, F | _lib.FA_PLAN_TUNE_BATCH8)),
        "fused_batch4": Reducer(lay, clients, o32, o64, flags=B,
                                plan=plan(0, F | _lib.FA_PLAN_TUNE_BATCH4)),
    }
    red = Reducer(lay, clients, o32, o64)
    dst = _lib.ptr_array([c[0].data_ptr() for c in clients])

    def bcast_only():
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        _lib.check(_lib.lib.fa_broadcast_f32(o32.data_ptr(), dst, n, lay.f32_numel, s))

    def separate():
        red()
        bcast_only()
    variants["reduce_then_bcast_kernel"] = separate
    variants["bcast_kernel_alone"] = bcast_only
    variants["reduce_alone"] = red
    times = {k: [] for k in variants}
    for r in range(rounds):
        for k, fn in variants.items():
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) / 20 * 1e3)
        print(f"round {r}", file=sys.stderr, flush=True)
    for k, ts in times.items():
        ts = sorted(ts)
        med = ts[len(ts) // 2]
        print(json.dumps({"exp": "bcast", "variant": k, "us_median": round(med, 2),
                          "us_min": round(ts[0], 2),
                          "round_GBps": round(moved / med / 1e3, 1)
                          if k not in ("bcast_kernel_alone", "reduce_alone") else None}),
              flush=True)


if __name__ == "__main__":
    main()
