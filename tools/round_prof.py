"""The cfg2 round's kernels alone, for rocprofv3 (kernel trace and the
separate FETCH_SIZE / WRITE_SIZE passes of tools/gpu_round_pmc.sh):

    python tools/round_prof.py round K        # reduce + broadcast launch (FA_F_BCAST)
    python tools/round_prof.py bcast K        # the broadcast launch alone (FA_F_BCAST_ONLY)
    python tools/round_prof.py tgpu K         # the torch-GPU-order reduce (tgpu_kernel<0>)
    python tools/round_prof.py tgpu32 K       # ... at N = 32 (the S = 2 launch, riders in it)
    python tools/round_prof.py cpu32 K        # the default order at N = 32 (same clients)
    python tools/round_prof.py sf32 K         # FedDCT sweep layouts' reduce alone (joint
    python tools/round_prof.py resnet110sl K  #   main + proxy bucket, rotated past the MALL)
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, load_manifest, make_clients  # noqa: E402


SWEEP = {"sf32": ("wrnsl16_8_sf32_c100", 3, 13), "resnet110sl": ("resnet110sl_sf4_c100", 25, 10)}


def sweep(mode, k, dev):
    from feddct_amd.workload import joint_manifest
    stem, n, rot = SWEEP[mode]
    mans = [load_manifest(stem + "_main"), load_manifest(stem + "_proxy")]
    lay = BucketLayout.from_manifest(joint_manifest(mans))
    plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                     flags=_lib.FA_PLAN_GAPS_ARE_PADDING)
    # one client filled (one synth launch per key), the rest clones of it:
    # a PMC pass crashed in the host runtime (SIGSEGV inside a synth launch,
    # no GPU fault) after ~100K per-key fill launches for 13 x 3 clients
    (c32, c64), = make_clients(lay, list(zip(mans, ("0.", "1."))), range(1), dev)
    reds = []
    for _ in range(rot):
        cl = [(c32.clone(), c64.clone()) for _ in range(n)]
        reds.append(Reducer(lay, cl, torch.zeros_like(c32), torch.zeros_like(c64), plan=plan))
    for i in range(k):
        reds[i % rot]()
    torch.cuda.synchronize()
    print(f"{mode}: {k} launches over {rot} rotated sets, algorithmic bytes "
          f"{lay.algorithmic_bytes(n)}, n = {n}")


def main():
    mode, k = sys.argv[1], int(sys.argv[2])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if mode in SWEEP:
        return sweep(mode, k, dev)
    man = load_manifest("wrn16_8_c10")
    lay = BucketLayout.from_manifest(man)
    n = 32 if mode in ("tgpu32", "cpu32") else 20
    cl = make_clients(lay, man, range(n), dev)
    o32, o64 = torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1])
    if mode in ("round", "bcast"):
        plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                         flags=_lib.FA_PLAN_GAPS_ARE_PADDING)
        red = Reducer(lay, cl, o32, o64, plan=plan,
                      flags=_lib.FA_F_BCAST if mode.startswith("round") else _lib.FA_F_BCAST_ONLY)
    elif mode in ("tgpu", "tgpu32"):
        plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                         order=_lib.FA_ORDER_TORCH_GPU, n=n)
        red = Reducer(lay, cl, o32, o64, plan=plan)
    elif mode == "cpu32":
        plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                         flags=_lib.FA_PLAN_GAPS_ARE_PADDING)
        red = Reducer(lay, cl, o32, o64, plan=plan)
    else:
        raise SystemExit(f"unknown mode {mode!r}")
    for _ in range(k):
        red()
    torch.cuda.synchronize()
    print(f"{mode}: {k} launches, B = {lay.state_bytes()} bytes per client, n = {n}, "
          f"algorithmic bytes {lay.algorithmic_bytes(n)}")


if __name__ == "__main__":
    main()
