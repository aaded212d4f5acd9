"""Experiment (r04): the whole server_aggregate
round (train_fedavg.py:145-149 / train_feddct.py:42-56: mean, global load,
broadcast into every client slot) on the product's launches, broadcast forms
A/B'd in ONE process, interleaved, HIP events, per layout:

  reduce        fa_reduce alone
  bcast         FA_F_BCAST_ONLY: the r04 broadcast alone
  round         FA_F_BCAST: reduce + r04 broadcast (scalar pointer loads,
                groups of <= 10 clients, 1024-float parts) — the default
  round_u2 / round_g24 / round_u2g24 / round_xcd   r04 kernel, tuning flags
  round_r03     the r02/r03 broadcast kernels (FA_PLAN_TUNE_BCAST_R03)
  reduce_stnt / round_stnt / round_stnt_r03   the reduce's result stores nt
                (FA_PLAN_TUNE_ST_NT: r01-r03) instead of sc1 (r04 default)
  round_fused   FA_F_BCAST inside the reduce (FA_PLAN_TUNE_FUSED_BCAST):
                one launch

Small layouts rotate over enough client sets that every step misses the
256 MiB MALL (as bench other_configs).  Algorithmic bytes of a round:
reduce N*B read + B written, broadcast B read + N*B written.
Usage: exp_round2.py [ROUNDS] [LAYOUT ...]  (cfg2 cfg3 cfg5 sf32 r110)"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from feddct_amd import _lib, slab  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, joint_manifest, load_manifest, make_clients  # noqa: E402

LAYOUTS = {
    "cfg2": (("wrn16_8_c10",), 20, 1),
    "cfg3": (("wrnsl16_8_sf4_c10_main", "wrnsl16_8_sf4_c10_proxy"), 5, 2),
    "cfg5": (("wrnsl16_8_sf4_c100_main", "wrnsl16_8_sf4_c100_proxy"), 24, 1),
    "sf32": (("wrnsl16_8_sf32_c100_main", "wrnsl16_8_sf32_c100_proxy"), 3, 6),
    "r110": (("resnet110sl_sf4_c100_main", "resnet110sl_sf4_c100_proxy"), 25, 4),
}
P = _lib.FA_PLAN_GAPS_ARE_PADDING
DEFAULT_STORE = 2   # the broadcast's default destination stores: sc1 nt
VARIANTS = {
    "reduce": (0, 0),
    "bcast": (_lib.FA_F_BCAST_ONLY, 0),
    "round": (_lib.FA_F_BCAST, 0),
    "round_u2": (_lib.FA_F_BCAST, _lib.FA_PLAN_TUNE_BCAST_U2),
    "round_g10": (_lib.FA_F_BCAST, _lib.FA_PLAN_TUNE_BCAST_G10),
    "round_u2g10": (_lib.FA_F_BCAST, _lib.FA_PLAN_TUNE_BCAST_U2 | _lib.FA_PLAN_TUNE_BCAST_G10),
    "round_xcd": (_lib.FA_F_BCAST, _lib.FA_PLAN_TUNE_BCAST_XCD),
    "round_r03": (_lib.FA_F_BCAST, _lib.FA_PLAN_TUNE_BCAST_R03),
    "round_fused": (_lib.FA_F_BCAST, _lib.FA_PLAN_TUNE_FUSED_BCAST),
    # the broadcast's store policy (fa_tune_bcast_store; default 2 = sc1 nt):
    # sc1 stores leave no dirty lines in the XCDs' L2 at the launch's end
    "round_g10_bnt": (_lib.FA_F_BCAST, _lib.FA_PLAN_TUNE_BCAST_G10, 0),
    "round_bnt": (_lib.FA_F_BCAST, 0, 0),
    "round_bsc1": (_lib.FA_F_BCAST, 0, 1),
    "round_bsc0sc1": (_lib.FA_F_BCAST, 0, 3),
    "round_bplain": (_lib.FA_F_BCAST, 0, 4),
    # clients per load batch forced (the default: 16 from N = 16, else 8)
    "reduce_b1": (0, _lib.FA_PLAN_TUNE_BATCH1),
    "reduce_b4": (0, _lib.FA_PLAN_TUNE_BATCH4),
    "reduce_b8": (0, _lib.FA_PLAN_TUNE_BATCH8),
    "reduce_b16": (0, _lib.FA_PLAN_TUNE_BATCH16),
    # the whole batch's loads back to back (FA_PLAN_TUNE_ISSUE_ALL) instead
    # of each client's behind the previous one's
    "reduce_issue_all": (0, _lib.FA_PLAN_TUNE_ISSUE_ALL),
    "round_issue_all": (_lib.FA_F_BCAST, _lib.FA_PLAN_TUNE_ISSUE_ALL),
    # r04: the reduce's result stores sc1 by default; _stnt: nt (r01-r03)
    "reduce_stnt": (0, _lib.FA_PLAN_TUNE_ST_NT),
    "round_stnt": (_lib.FA_F_BCAST, _lib.FA_PLAN_TUNE_ST_NT),
    "round_stnt_r03": (_lib.FA_F_BCAST, _lib.FA_PLAN_TUNE_ST_NT | _lib.FA_PLAN_TUNE_BCAST_R03),
}


def run_layout(tag, rounds, dev):
    # "TAG:slab": the global's bucket (the broadcast's source) carved from the
    # clients' slab, as the drop-in's arenas place it; default a separate
    # allocation
    tag, _, where = tag.partition(":")
    names, n, rot = LAYOUTS[tag]
    mans = [load_manifest(x) for x in names]
    prefixes = ("0.", "1.") if len(names) > 1 else ("",)
    man = joint_manifest(mans, prefixes) if len(names) > 1 else mans[0]
    lay = BucketLayout.from_manifest(man)
    sets = []
    for _ in range(rot):
        cl = make_clients(lay, list(zip(mans, prefixes)), range(n), dev)
        o32 = (slab.carve(cl[0][0].numel(), torch.float32, dev) if where == "slab"
               else torch.zeros_like(cl[0][0]))
        sets.append((cl, o32, torch.zeros_like(cl[0][1])))
    if where:
        tag = tag + ":" + where
    plans = {}
    fns = {}
    sel = [x for x in os.environ.get("VARIANTS", "").split(",") if x]
    for k, v in VARIANTS.items():
        if sel and k not in sel:
            continue
        fl, pfl, sp = (v + (DEFAULT_STORE,))[:3]
        if pfl not in plans:
            plans[pfl] = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                                   flags=P | pfl)
        reds = [Reducer(lay, cl, o32, o64, flags=fl, plan=plans[pfl]) for cl, o32, o64 in sets]
        ctr = [0]

        def step(reds=reds, ctr=ctr, sp=sp):
            _lib.lib.fa_tune_bcast_store(sp)
            reds[ctr[0] % len(reds)]()
            ctr[0] += 1
        fns[k] = step
    times = {k: [] for k in fns}
    reps = 40 if rot > 1 else 20
    for r in range(rounds):
        for k, fn in fns.items():
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) / reps * 1e3)
    B = lay.state_bytes()
    red_bytes = lay.algorithmic_bytes(n)
    bc_bytes = (n + 1) * B
    med = {}
    _lib.lib.fa_tune_bcast_store(DEFAULT_STORE)
    for k, ts in times.items():
        ts = sorted(ts)
        med[k] = ts[len(ts) // 2]
        nb = (red_bytes if k.startswith("reduce") else bc_bytes if k == "bcast"
              else red_bytes + bc_bytes)
        print(json.dumps({"exp": "round2", "layout": tag, "n": n, "variant": k,
                          "us_median": round(med[k], 2), "us_min": round(ts[0], 2),
                          "bytes": nb, "frac": round(nb / (med[k] * 1e-6) / 8e12, 4)}),
              flush=True)
    if all(k in med for k in ("round", "reduce", "bcast", "round_fused")):
        print(json.dumps({"exp": "round2_summary", "layout": tag,
                          "round_over_sum": round(med["round"] / (med["reduce"] + med["bcast"]),
                                                  4),
                          "fused_over_round": round(med["round_fused"] / med["round"], 4)}),
              flush=True)
    if sel:
        return
    # each kernel's time inside the round: the round as two calls (reduce,
    # then the broadcast alone) with events between them, per broadcast form
    for pfl, nm in ((0, "r04"), (_lib.FA_PLAN_TUNE_BCAST_R03, "r03"),
                    (_lib.FA_PLAN_TUNE_ST_NT, "stnt"),
                    (_lib.FA_PLAN_TUNE_ST_NT | _lib.FA_PLAN_TUNE_BCAST_R03, "stnt_r03"),
                    (_lib.FA_PLAN_TUNE_BCAST_G10, "g10"), (_lib.FA_PLAN_TUNE_BCAST_U2, "u2")):
        if pfl not in plans:
            continue
        rr = [Reducer(lay, cl, o32, o64, plan=plans[pfl]) for cl, o32, o64 in sets]
        bb = [Reducer(lay, cl, o32, o64, flags=_lib.FA_F_BCAST_ONLY, plan=plans[pfl])
              for cl, o32, o64 in sets]
        for i in range(3 * len(rr)):
            rr[i % len(rr)]()
            bb[i % len(rr)]()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps + 1)]
        ev[0].record()
        for i in range(reps):
            rr[i % len(rr)]()
            ev[2 * i + 1].record()
            bb[i % len(rr)]()
            ev[2 * i + 2].record()
        ev[-1].synchronize()
        tr = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) * 1e3 for i in range(reps))
        tb = sorted(ev[2 * i + 1].elapsed_time(ev[2 * i + 2]) * 1e3 for i in range(reps))
        print(json.dumps({"exp": "round2_split", "layout": tag, "bcast_form": nm,
                          "reduce_in_round_us": round(tr[reps // 2], 2),
                          "bcast_in_round_us": round(tb[reps // 2], 2),
                          "round_us": round(ev[0].elapsed_time(ev[-1]) * 1e3 / reps, 2)}),
              flush=True)
    # bits: every round form leaves every client = the global (last set used)
    for k in ("round",):
        cl, o32, o64 = sets[0]
        Reducer(lay, cl, o32, o64, flags=_lib.FA_F_BCAST, plan=plans[0])()
        torch.cuda.synchronize()
        ok = all(torch.equal(c[0], o32) and torch.equal(c[1], o64) for c in cl)
        print(json.dumps({"exp": "round2_bits", "layout": tag, "clients_equal_global": ok}),
              flush=True)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    tags = sys.argv[2:] or list(LAYOUTS)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for t in tags:
        run_layout(t, rounds, dev)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
