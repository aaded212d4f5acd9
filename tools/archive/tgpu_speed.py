"""Launch time of the torch-GPU-order plan (FA_ORDER_TORCH_GPU) on the cfg2,
cfg3 and cfg5 one-GPU workloads, with bit-exactness against torch's own
cuda stack(...).mean(0) of every key (bench.torch_gpu_order_mode).  Each
workload is timed with the default tiles, without the S = 1 group's tail
split (FA_PLAN_TUNE_NO_BALANCE, r04) and with FA_PLAN_TUNE_TGPU_NARROW (the
r02 1024-element form), alternating, ``reps`` times each.

    python tools/tgpu_speed.py [reps]
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from feddct_amd import _lib  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import joint_manifest, load_manifest, make_clients  # noqa: E402

FORMS = {"wide": _lib.FA_PLAN_GAPS_ARE_PADDING,
         "wide_b8": _lib.FA_PLAN_GAPS_ARE_PADDING,
         "wide_b16": _lib.FA_PLAN_GAPS_ARE_PADDING,
         "wide_no_tail_split": _lib.FA_PLAN_GAPS_ARE_PADDING | _lib.FA_PLAN_TUNE_NO_BALANCE,
         "narrow": _lib.FA_PLAN_GAPS_ARE_PADDING | _lib.FA_PLAN_TUNE_TGPU_NARROW}


def measure(name, lay, cl, reps):
    res = {k: [] for k in FORMS}
    exact = {k: True for k in FORMS}
    for _ in range(reps):
        for k, fl in FORMS.items():
            _lib.lib.fa_tune_tgpu_batch({"wide_b8": 8, "wide_b16": 16}.get(k, 0))
            r = bench.torch_gpu_order_mode(lay, cl, steps=100, warmup=20, plan_flags=fl)
            _lib.lib.fa_tune_tgpu_batch(0)
            res[k].append(r["us"])
            exact[k] &= r["bit_exact_vs_torch_cuda_mean"]
    nb = lay.algorithmic_bytes(len(cl))
    for k in FORMS:
        best = min(res[k])
        p = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                      order=_lib.FA_ORDER_TORCH_GPU, n=len(cl), flags=FORMS[k])
        print(json.dumps({"workload": name, "form": k, "ntiles": p.info["ntiles"],
                          "us": res[k], "best_us": best,
                          "GBps": round(nb / best / 1e3, 1),
                          "bit_exact_vs_torch_cuda_mean": exact[k]}), flush=True)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    man = load_manifest("wrn16_8_c10")
    lay = BucketLayout.from_manifest(man)
    cl = make_clients(lay, man, range(20), dev)
    measure("cfg2", lay, cl, reps)
    del cl
    for name, n in (("c10", 5), ("c100", 24)):
        mm = load_manifest(f"wrnsl16_8_sf4_{name}_main")
        pm = load_manifest(f"wrnsl16_8_sf4_{name}_proxy")
        lay = BucketLayout.from_manifest(joint_manifest([mm, pm]))
        cl = make_clients(lay, [(mm, "0."), (pm, "1.")], range(n), dev)
        measure(f"feddct_{name}_n{n}", lay, cl, reps)
        del cl
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
