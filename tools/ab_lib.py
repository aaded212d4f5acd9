"""A/B of two libfedagg.so builds in ONE process on the same buffers (r03):
the headline cfg2 reduce (wrn16_8 C10, N = 20) and other layouts, each
library's default plan, launches interleaved library by library over
several rounds, output bits compared between the builds.  Used to tell a
code change from box-to-box variance.  Only the C ABI both builds share
is called (fa_plan_create, fa_reduce, fa_synth_fill_*).

    python tools/ab_lib.py LIB_A LIB_B [ROUNDS] [CASES]
    AB_SLAB=1: each client set carved from one slab (feddct_amd/slab.py), as
    the product places them; AB_FLAGS=1: whole rounds (FA_F_BCAST);
    AB_PFLAGS_B=<int>: plan flags ORed into LIB_B's plans (e.g. 8 =
    FA_PLAN_TUNE_BATCH16), so one library can be A/B'd against itself
"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from feddct_amd import synth  # noqa: E402
from feddct_amd.layout import KIND_I64, BucketLayout  # noqa: E402
from feddct_amd.workload import joint_manifest, load_manifest  # noqa: E402

_P, _I, _I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
CASES = [("cfg2", "wrn16_8_c10", 20, 1), ("cfg4w", "wrn16_8_c100", 20, 1),
         ("cfg3", "wrnsl16_8_sf4_c10", 5, 2), ("resnet110sl", "resnet110sl_sf4_c100", 25, 4),
         # torch-ROCm's GPU order (fa_plan_create_order, FA_ORDER_TORCH_GPU)
         ("cfg2_tgpu", "wrn16_8_c10", 20, 1), ("cfg3_tgpu", "wrnsl16_8_sf4_c10", 5, 2),
         # r05: the client-loop rule's range (17..63 unweighted, plain table)
         ("c10_n17", "wrn16_8_c10", 17, 1), ("c10_n32", "wrn16_8_c10", 32, 1),
         ("c10_n48", "wrn16_8_c10", 48, 1), ("c100_n20", "wrn16_8_c100", 20, 1),
         ("cfg5", "wrnsl16_8_sf4_c100", 24, 1), ("c10_n2", "wrn16_8_c10", 2, 1),
         ("c10_n8", "wrn16_8_c10", 8, 1), ("c10_n12", "wrn16_8_c10", 12, 1),
         ("sf32", "wrnsl16_8_sf32_c100", 3, 6), ("sf16", "wrnsl16_8_sf16_c100", 6, 4),
         ("cfg2w", "wrn16_8_c10", 20, 1), ("cfg5w", "wrnsl16_8_sf4_c100", 24, 1),
         ("cfg3w", "wrnsl16_8_sf4_c10", 5, 2), ("c10_n10", "wrn16_8_c10", 10, 1),
         ("c10_n16", "wrn16_8_c10", 16, 1), ("c10_n12w", "wrn16_8_c10", 12, 1),
         ("c10_n64", "wrn16_8_c10", 64, 1), ("c10_n100", "wrn16_8_c10", 100, 1),
         ("c10_n80w", "wrn16_8_c10", 80, 1), ("c10_n128w", "wrn16_8_c10", 128, 1),
         # r05: the client loop in the torch-GPU-order kernel
         ("c10_n2_tgpu", "wrn16_8_c10", 2, 2), ("c10_n10_tgpu", "wrn16_8_c10", 10, 1),
         ("c10_n32_tgpu", "wrn16_8_c10", 32, 1), ("c10_n64_tgpu", "wrn16_8_c10", 64, 1),
         ("cfg5_tgpu", "wrnsl16_8_sf4_c100", 24, 1), ("sf32_tgpu", "wrnsl16_8_sf32_c100", 3, 6),
         ("c10_n5_tgpu", "wrn16_8_c10", 5, 2), ("c10_n12_tgpu", "wrn16_8_c10", 12, 1),
         ("c10_n16_tgpu", "wrn16_8_c10", 16, 1), ("c10_n17_tgpu", "wrn16_8_c10", 17, 1),
         ("c10_n28_tgpu", "wrn16_8_c10", 28, 1), ("c100_n20_tgpu", "wrn16_8_c100", 20, 1),
         ("c10_n48_tgpu", "wrn16_8_c10", 48, 1), ("c10_n100_tgpu", "wrn16_8_c10", 100, 1),
         ("c10_n127_tgpu", "wrn16_8_c10", 127, 1), ("c100_n64_tgpu", "wrn16_8_c100", 64, 1),
         ("c100_n128_tgpu", "wrn16_8_c100", 128, 1),
         # r05: the N <= 3 table (every column in the vector runs)
         ("sf32w", "wrnsl16_8_sf32_c100", 3, 6), ("c10_n3", "wrn16_8_c10", 3, 2),
         ("r110_n2", "resnet110sl_sf4_c100", 2, 6), ("r110_n3", "resnet110sl_sf4_c100", 3, 6),
         ("sf16_n3", "wrnsl16_8_sf16_c100", 3, 6),
         # r06: the default order from 64 clients (the 1024-float table)
         ("c10_n128", "wrn16_8_c10", 128, 1), ("c100_n64", "wrn16_8_c100", 64, 1),
         ("c100_n100", "wrn16_8_c100", 100, 1), ("c10_n200", "wrn16_8_c10", 200, 1),
         ("c10_n256", "wrn16_8_c10", 256, 1),
         # r06: the torch-GPU order's row batch below 16 clients
         ("c10_n8_tgpu", "wrn16_8_c10", 8, 1), ("c10_n9_tgpu", "wrn16_8_c10", 9, 1),
         ("c10_n14_tgpu", "wrn16_8_c10", 14, 1), ("c10_n14", "wrn16_8_c10", 14, 1),
         ("c100_n12w", "wrn16_8_c100", 12, 1), ("c10_n11", "wrn16_8_c10", 11, 1),
         ("c10_n13", "wrn16_8_c10", 13, 1), ("c10_n16w", "wrn16_8_c10", 16, 1),
         ("c10_n150", "wrn16_8_c10", 150, 1), ("c10_n300", "wrn16_8_c10", 300, 1),
         ("c10_n64w", "wrn16_8_c10", 64, 1), ("c10_n100w", "wrn16_8_c10", 100, 1),
         ("c100_n64w", "wrn16_8_c100", 64, 1)]


def load(path):
    lib = ctypes.CDLL(path)
    lib.fa_plan_create.argtypes = [_P, _I, _I64, _P, _I, _I64, _I, ctypes.c_uint,
                                   ctypes.POINTER(_P)]
    lib.fa_reduce.argtypes = [_P, _P, _P, _I, _P, _P, _P, ctypes.c_uint, _P]
    lib.fa_plan_create_order.argtypes = [_P, _I, _I64, _P, _I, _I64, _I, _I, ctypes.c_uint,
                                         ctypes.POINTER(_P)]
    lib.fa_synth_fill_f32.argtypes = [_P, _I64, _I, _I, ctypes.c_float, ctypes.c_float, _I, _P]
    lib.fa_synth_fill_i64.argtypes = [_P, _I64, _I, _I, _I, _P]
    lib.fa_last_error.restype = ctypes.c_char_p
    return lib


def ok(lib, rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: {lib.fa_last_error().decode()}")


def segs(arr):
    a = (_I64 * max(2, 2 * len(arr)))()
    for i, (o, m) in enumerate(arr):
        a[2 * i], a[2 * i + 1] = int(o), int(m)
    return a, len(arr)


def layout_of(stem):
    if os.path.exists(os.path.join(ROOT, "feddct_amd", "manifests", stem + "_main.json")):
        mans = [load_manifest(stem + "_main"), load_manifest(stem + "_proxy")]
        return BucketLayout.from_manifest(joint_manifest(mans)), list(zip(mans, ("0.", "1.")))
    m = load_manifest(stem)
    return BucketLayout.from_manifest(m), [(m, "")]


SLAB = os.environ.get("AB_SLAB", "0") == "1"   # clients carved from one slab (slab.py)
FLAGS = int(os.environ.get("AB_FLAGS", "0"))   # fa_reduce flags (1: FA_F_BCAST, the round)
PFLAGS_B = int(os.environ.get("AB_PFLAGS_B", "0"))   # extra plan flags for LIB_B


def fill(lib, lay, parts, c, dev):
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    if SLAB:
        from feddct_amd import slab
        f32 = slab.carve(max(lay.f32_numel, 64), torch.float32, dev)
    else:
        f32 = torch.zeros(max(lay.f32_numel, 64), dtype=torch.float32, device=dev)
    i64 = torch.zeros(max(lay.i64_numel, 1), dtype=torch.int64, device=dev)
    for man, pre in parts:
        for j, e in enumerate(man["keys"]):
            s = lay.by_key[pre + e["key"]]
            if s.alias_of is not None:
                continue
            if s.kind == KIND_I64:
                ok(lib, lib.fa_synth_fill_i64(i64[s.offset:].data_ptr(), s.numel, j, c, 0, st),
                   "fill")
            else:
                mu, sg = synth.key_params(e["key"], tuple(e["shape"]), e["dtype"])
                ok(lib, lib.fa_synth_fill_f32(f32[s.offset:].data_ptr(), s.numel, j, c, mu, sg, 0,
                                              st), "fill")
    return f32, i64


def parse_case(name):
    """A case not in CASES named like c10_n40, c100_n24w, c10_n40_tgpu: the
    wrn16_8 layout of that class count, that many clients (one set)."""
    import re
    m = re.fullmatch(r"c(10|100)_n(\d+)(w?)(_tgpu)?", name)
    return (name, f"wrn16_8_c{m.group(1)}", int(m.group(2)), 1) if m else None


def main():
    paths = sys.argv[1:3]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 7
    which = sys.argv[4].split(",") if len(sys.argv) > 4 else [c[0] for c in CASES]
    known = {c[0] for c in CASES}
    extra = [parse_case(w) for w in which if w not in known]
    if None in extra:
        raise SystemExit(f"unknown case in {which}")
    CASES.extend(extra)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    libs = [load(p) for p in paths]
    G = 0x1   # FA_PLAN_GAPS_ARE_PADDING
    for name, stem, n, rot in CASES:
        if name not in which:
            continue
        lay, parts = layout_of(stem)
        weighted = name.endswith("w")
        wts = (ctypes.c_float * n)(*[(1000.0 + 37 * c) / 1e5 for c in range(n)]) if weighted \
            else None
        sets = []
        for _ in range(rot):
            if SLAB:
                from feddct_amd import slab
                slab.release()
                ctx = slab.expecting(n + 1)
                ctx.__enter__()
            cl = [fill(libs[0], lay, parts, c, dev) for c in range(n)]
            if SLAB:
                ctx.__exit__(None, None, None)
            sets.append((cl, torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1])))
        plans = []
        for k, lib in enumerate(libs):
            g = G | (PFLAGS_B if k == 1 else 0)
            a32, n32 = segs(lay.segs32)
            a64, n64 = segs(lay.segs64)
            h = _P()
            if name.endswith("_tgpu"):
                ok(lib, lib.fa_plan_create_order(a32, n32, lay.f32_numel, a64, n64, lay.i64_numel,
                                                 n, 1, g, ctypes.byref(h)), "plan")
            else:
                ok(lib, lib.fa_plan_create(a32, n32, lay.f32_numel, a64, n64, lay.i64_numel, 0,
                                           g, ctypes.byref(h)), "plan")
            plans.append(h)
        ptrs = [((_P * n)(*[c[0].data_ptr() for c in cl]), (_P * n)(*[c[1].data_ptr() for c in cl]),
                 o32, o64) for cl, o32, o64 in sets]
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

        def call(k, i):
            p32, p64, o32, o64 = ptrs[i % rot]
            ok(libs[k], libs[k].fa_reduce(plans[k], p32, p64, n, wts, o32.data_ptr(),
                                          o64.data_ptr(), FLAGS, st), "reduce")
        times = [[], []]
        outs = [None, None]
        reps = 60 * rot if n > 10 else 200 * rot
        for _ in range(rounds):
            for k in (0, 1):
                for i in range(3 * rot):
                    call(k, i)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(reps):
                    call(k, i)
                e1.record()
                e1.synchronize()
                times[k].append(e0.elapsed_time(e1) / reps * 1e3)
                outs[k] = (sets[0][1].clone(), sets[0][2].clone())
        same = (torch.equal(outs[0][0].view(torch.int32), outs[1][0].view(torch.int32))
                and torch.equal(outs[0][1], outs[1][1]))
        nb = lay.algorithmic_bytes(n)
        rec = {"exp": "ab_lib", "case": name, "n": n, "rot": rot, "same_bits": bool(same)}
        for k, tag in ((0, "a"), (1, "b")):
            ts = sorted(times[k])
            rec[tag] = {"lib": paths[k], "us_median": round(ts[len(ts) // 2], 2),
                        "us_min": round(ts[0], 2),
                        "frac": round(nb / ts[len(ts) // 2] / 1e3 / 8000, 4)}
        print(json.dumps(rec), flush=True)
        del sets, ptrs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
