"""Experiment (r03 session 3): does the placement of the 20 client buckets in
device memory decide the headline's box-to-box spread (133 us on some boxes,
143-146 us on others, with the same copy ceiling)?  cfg2 (wrn16_8 C10,
N = 20), one process, interleaved rounds, bits compared:

* sep        - 20 separate torch allocations (what bench.py and the shim do)
* arena_256  - one allocation, client i at i * (B rounded up to 256 B)
* arena_2m   - one allocation, stride rounded up to 2 MiB (every client base
               congruent modulo 2 MiB)
* arena_2m_4k - stride 2 MiB-rounded + 4 KiB (bases staggered by 4 KiB steps)
* arena_2m_odd - stride 2 MiB-rounded + 64 KiB + 256 B

plus this box's read-only rate over the same 20 x B bytes (read probe over
the arena_256 allocation) and a copy of one bucket's worth x 20.

    python tools/archive/exp_alloc.py [ROUNDS] [one_tensor]  |  python tools/archive/exp_alloc.py order
"""
import json
import sys
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, load_manifest, make_clients  # noqa: E402

N = 20
MIB2 = 2 << 20


def order_mode(rounds):
    """Separate vs one allocation, alternating in allocation order (sep1,
    one1, sep2, one2, sep3, one3): does a set's speed follow its form or
    the order (memory state) it was allocated in?"""
    dev = torch.device("cuda", 0)
    man = load_manifest("wrn16_8_c10")
    lay = BucketLayout.from_manifest(man)
    nb = lay.algorithmic_bytes(N)
    plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                     flags=_lib.FA_PLAN_GAPS_ARE_PADDING)
    src = make_clients(lay, man, range(N), dev)
    n32 = src[0][0].numel()
    s = (n32 * 4 + 255) // 256 * 256 // 4
    reds, keep = {}, []
    for i in range(1, 4):
        sep = [(c32.clone(), c64) for c32, c64 in src]
        reds[f"sep{i}"] = Reducer(lay, sep, torch.zeros_like(src[0][0]),
                                  torch.zeros_like(src[0][1]), plan=plan)
        a = torch.empty(N * s, dtype=torch.float32, device=dev)
        keep.append(a)
        one = []
        for j in range(N):
            v = a[j * s:j * s + n32]
            v.copy_(src[j][0])
            one.append((v, src[j][1]))
        reds[f"one{i}"] = Reducer(lay, one, torch.zeros_like(src[0][0]),
                                  torch.zeros_like(src[0][1]), plan=plan)
    del src
    times = {k: [] for k in reds}
    for _ in range(rounds):
        for k, fn in reds.items():
            for _ in range(5):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                fn()
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) / 50 * 1e3)
        print("round", file=sys.stderr, flush=True)
    ref = reds["sep1"].out32.view(torch.int32)
    for k, ts in times.items():
        ts = sorted(ts)
        med = ts[len(ts) // 2]
        print(json.dumps({"exp": "alloc_order", "variant": k, "us_median": round(med, 2),
                          "us_min": round(ts[0], 2), "GBps": round(nb / med / 1e3, 1),
                          "frac": round(nb / med / 1e3 / 8000, 4),
                          "bit_equal": bool(torch.equal(reds[k].out32.view(torch.int32), ref))}),
              flush=True)


def main():
    if "order" in sys.argv[1:]:
        return order_mode(5)
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 7
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if "one_tensor" in sys.argv[1:]:   # the same bytes as one 5376 x 2048 tensor
        man = {"name": "t5376", "keys": [{"key": "w", "shape": [5376, 2048],
                                          "dtype": "float32"}]}
    else:
        man = load_manifest("wrn16_8_c10")
    lay = BucketLayout.from_manifest(man)
    nb = lay.algorithmic_bytes(N)
    plan = _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                     flags=_lib.FA_PLAN_GAPS_ARE_PADDING)
    os.environ["FA_SLAB"] = "0"        # "sep": one allocation per bucket
    sep = make_clients(lay, man, range(N), dev)
    os.environ["FA_SLAB"] = "1"
    n32 = sep[0][0].numel()
    b32 = n32 * 4

    def arena(stride_bytes):
        assert stride_bytes % 256 == 0 and stride_bytes >= b32
        s = stride_bytes // 4
        a = torch.empty(N * s, dtype=torch.float32, device=dev)
        cl = []
        for i in range(N):
            v = a[i * s:i * s + n32]
            v.copy_(sep[i][0])
            cl.append((v, sep[i][1]))
        return a, cl

    r256 = (b32 + 255) // 256 * 256
    r2m = (b32 + MIB2 - 1) // MIB2 * MIB2
    strides = {"arena_256": r256, "arena_2m": r2m, "arena_2m_4k": r2m + 4096,
               "arena_2m_odd": r2m + 65536 + 256, "arena_256_plus_1m": r256 + (1 << 20),
               "arena_256_plus_24k": r256 + 24576}
    variants = {"sep": Reducer(lay, sep, torch.zeros_like(sep[0][0]),
                               torch.zeros_like(sep[0][1]), plan=plan)}
    keep = {}
    for k, st in strides.items():
        a, cl = arena(st)
        keep[k] = a
        variants[k] = Reducer(lay, cl, torch.zeros_like(sep[0][0]), torch.zeros_like(sep[0][1]),
                              plan=plan)
    # read probe over the same bytes as 20 buckets, and a copy of the same bytes
    probe_src = keep["arena_256"]
    probe_out = torch.zeros(4096, dtype=torch.float32, device=dev)
    copy_dst = torch.empty_like(probe_src)
    s = torch.cuda.current_stream().cuda_stream

    def probe():
        _lib.check(_lib.lib.fa_read_probe_f32(probe_src.data_ptr(), probe_src.numel(),
                                              probe_out.data_ptr(), 0, s), "probe")

    def copy():
        _lib.check(_lib.lib.fa_copy_f32(probe_src.data_ptr(), copy_dst.data_ptr(),
                                        probe_src.numel(), s), "copy")

    def probe_gs():
        _lib.check(_lib.lib.fa_read_probe_f32(probe_src.data_ptr(), probe_src.numel(),
                                              probe_out.data_ptr(), 4096, s), "probe_gs")

    fns = dict(variants)
    fns["read_probe"] = probe
    fns["read_probe_gridstride"] = probe_gs
    fns["copy"] = copy
    times = {k: [] for k in fns}
    for _ in range(rounds):
        for k, fn in fns.items():
            for _ in range(5):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                fn()
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) / 50 * 1e3)
        print("round", file=sys.stderr, flush=True)
    ref = variants["sep"].out32
    for k, ts in times.items():
        ts = sorted(ts)
        med = ts[len(ts) // 2]
        if k.startswith("read_probe"):
            byts = probe_src.numel() * 4
        elif k == "copy":
            byts = probe_src.numel() * 8
        else:
            byts = nb
        rec = {"exp": "alloc", "variant": k, "us_median": round(med, 2), "us_min": round(ts[0], 2),
               "GBps": round(byts / med / 1e3, 1), "frac": round(byts / med / 1e3 / 8000, 4)}
        if k in variants:
            rec["bit_equal_sep"] = bool(torch.equal(variants[k].out32.view(torch.int32),
                                                    ref.view(torch.int32)))
            bases = [c[0].data_ptr() for c in variants[k]._keep[0]]
            rec["base_mod_2m"] = sorted({b % MIB2 for b in bases})[:4]
        print(json.dumps(rec), flush=True)
    print(json.dumps({"exp": "alloc", "device": torch.cuda.get_device_name(0),
                      "host": os.uname().nodename}), flush=True)


if __name__ == "__main__":
    main()
