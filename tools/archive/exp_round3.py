"""Experiment (r05): the product's round (fa_reduce with
FA_F_BCAST: the mean, the global's load and the broadcast into every client,
train_fedavg.py:145-149 / train_feddct.py:42-56) as ONE launch
(reduce_impl.h round_kernel) against the reduce + broadcast launches, per
layout.  The library picks the form by the client count; FA_EXP_ROUND=two /
one forces it for a whole process (read once), so the A/B is one process per
form, the forms alternated by tools/exp_round3.sh on one box.

Small layouts rotate over enough client sets that every step misses the
256 MiB MALL (as bench.py other_configs).  Bits: after the timed rounds every
client bucket equals the global's, and the global equals the reference's
digest (the layouts whose digests tests/golden holds).
Usage: exp_round3.py TAG [LAYOUT ...]   (cfg2 cfg3 cfg5 sf32 sf16 sf8 r110)"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, joint_manifest, load_manifest, make_clients  # noqa: E402

LAYOUTS = {
    "cfg2": (("wrn16_8_c10",), 20, 1, "fedavg/wrn16_8_c10/n20"),
    "cfg3": (("wrnsl16_8_sf4_c10_main", "wrnsl16_8_sf4_c10_proxy"), 5, 2, "feddct/wrnsl16_8_sf4_c10_{}/n5"),
    "cfg5": (("wrnsl16_8_sf4_c100_main", "wrnsl16_8_sf4_c100_proxy"), 24, 1,
             "feddct/wrnsl16_8_sf4_c100_{}/n24"),
    "sf32": (("wrnsl16_8_sf32_c100_main", "wrnsl16_8_sf32_c100_proxy"), 3, 6,
             "feddct/wrnsl16_8_sf32_c100_{}/n3"),
    "sf16": (("wrnsl16_8_sf16_c100_main", "wrnsl16_8_sf16_c100_proxy"), 6, 4,
             "feddct/wrnsl16_8_sf16_c100_{}/n6"),
    "sf8": (("wrnsl16_8_sf8_c100_main", "wrnsl16_8_sf8_c100_proxy"), 12, 2,
            "feddct/wrnsl16_8_sf8_c100_{}/n12"),
    "r110": (("resnet110sl_sf4_c100_main", "resnet110sl_sf4_c100_proxy"), 25, 4,
             "feddct/resnet110sl_sf4_c100_{}/n25"),
}


def digest(lay, o32, o64, prefix):
    import hashlib
    f, i = o32.cpu().numpy(), o64.cpu().numpy()
    h = hashlib.sha256()
    for s in lay.slots:
        if s.key.startswith(prefix):
            h.update(s.key[len(prefix):].encode())
            h.update((i if s.kind == "i64" else f)[s.offset:s.offset + s.numel].tobytes())
    return h.hexdigest()


def run(tag, form, dev, reps=40, passes=5):
    names, n, rot, dname = LAYOUTS[tag]
    mans = [load_manifest(x) for x in names]
    prefixes = ("0.", "1.") if len(names) > 1 else ("",)
    man = joint_manifest(mans, prefixes) if len(names) > 1 else mans[0]
    lay = BucketLayout.from_manifest(man)
    plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                     flags=_lib.FA_PLAN_GAPS_ARE_PADDING)
    sets = []
    for _ in range(rot):
        cl = make_clients(lay, list(zip(mans, prefixes)), range(n), dev)
        o32, o64 = torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1])
        sets.append((cl, o32, o64, Reducer(lay, cl, o32, o64, flags=_lib.FA_F_BCAST, plan=plan)))
    # bits first (the clients are overwritten by the broadcast afterwards)
    cl, o32, o64, red = sets[0]
    red()
    torch.cuda.synchronize()
    with open(os.path.join(ROOT, "tests", "golden", "digests.json")) as f:
        dig = json.load(f)
    if len(names) > 1:
        ok = all(digest(lay, o32, o64, p) == dig[dname.format(h)]
                 for p, h in zip(prefixes, ("main", "proxy")))
    else:
        ok = digest(lay, o32, o64, "") == dig[dname]
    segs_ok = all(torch.equal(c[0][int(o):int(o + m)], o32[int(o):int(o + m)])
                  for c in cl for o, m in lay.segs32) and all(torch.equal(c[1], o64) for c in cl)
    ts = []
    k = 0
    for _ in range(passes):
        for _ in range(3):
            sets[k % rot][3]()
            k += 1
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            sets[k % rot][3]()
            k += 1
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / reps * 1e3)
    ts.sort()
    nb = 2 * (n + 1) * lay.state_bytes()
    us = ts[len(ts) // 2]
    print(json.dumps({"exp": "round3", "form": form, "layout": tag, "n": n,
                      "us_median": round(us, 2), "us_min": round(ts[0], 2), "bytes": nb,
                      "frac": round(nb / (us * 1e-6) / 8e12, 4),
                      "bit_exact_vs_reference_digest": ok, "clients_equal_global": segs_ok}),
          flush=True)


def main():
    form = sys.argv[1]
    tags = sys.argv[2:] or list(LAYOUTS)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for t in tags:
        run(t, form, dev)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
