"""Experiment (r04): does the physical placement of the client buckets set
the round's speed?  The cfg2 round (reduce + broadcast, train_fedavg.py:
145-149) over client buckets carved from (a) the product's torch slab and
(b) ONE physically contiguous allocation (hipExtMallocWithFlags with
hipDeviceMallocContiguous, wrapped as a torch tensor through
__cuda_array_interface__), interleaved in one process, plus (c) a second
torch slab made after allocation churn.  Prints one JSON line per
(placement, variant).  Usage: exp_contig.py [ROUNDS]"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from feddct_amd import _lib, slab  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, fill_client, load_manifest  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t,
                                      ctypes.c_uint]
hip.hipFree.argtypes = [ctypes.c_void_p]
CONTIG = 0x4


class _Raw:
    """Owner of a hipExtMallocWithFlags allocation, exposed to torch."""

    def __init__(self, nbytes, flags):
        p = ctypes.c_void_p()
        rc = hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, flags)
        if rc != 0:
            raise RuntimeError(f"hipExtMallocWithFlags rc={rc}")
        self.ptr, self.nbytes = p.value, nbytes
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1",
                                         "data": (self.ptr, False), "version": 2}

    def __del__(self):
        hip.hipFree(self.ptr)


def buckets_from(base: torch.Tensor, lay, n):
    """n + 1 fp32 buckets (clients, then the global) at 64 KiB steps."""
    nb = lay.f32_numel * 4
    step = -(-nb // 65536) * 65536
    out = []
    for i in range(n + 1):
        out.append(base[i * step:i * step + nb].view(torch.float32))
    return out


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    man = load_manifest("wrn16_8_c10")
    lay = BucketLayout.from_manifest(man)
    n = 20
    step = -(-lay.f32_numel * 4 // 65536) * 65536
    total = step * (n + 1)
    sets = {}
    keep = []
    # (a) the product's slab, first allocation of the process
    base_a = torch.zeros(total, dtype=torch.uint8, device=dev)
    # (b) one physically contiguous allocation
    raw = _Raw(total, CONTIG)
    keep.append(raw)
    base_b = torch.as_tensor(raw, device=dev)
    # (c) a torch allocation after churn
    churn = [torch.empty(6 << 20, dtype=torch.uint8, device=dev) for _ in range(300)]
    del churn[::2]
    base_c = torch.zeros(total, dtype=torch.uint8, device=dev)
    for tag, base in (("slab_first", base_a), ("contiguous", base_b), ("after_churn", base_c)):
        bk = buckets_from(base, lay, n)
        cl = []
        for c in range(n):
            i64 = torch.zeros(max(1, lay.i64_numel), dtype=torch.int64, device=dev)
            fill_client(lay, man, bk[c], i64, c)
            cl.append((bk[c], i64))
        sets[tag] = (cl, bk[n], torch.zeros_like(cl[0][1]))
    torch.cuda.synchronize()
    plans = {pf: _lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                           flags=_lib.FA_PLAN_GAPS_ARE_PADDING | pf)
             for pf in (0, _lib.FA_PLAN_TUNE_BCAST_G10, _lib.FA_PLAN_TUNE_BCAST_R03)}
    fns = {}
    for tag, (cl, o32, o64) in sets.items():
        fns[(tag, "reduce")] = Reducer(lay, cl, o32, o64, plan=plans[0])
        fns[(tag, "bcast")] = Reducer(lay, cl, o32, o64, flags=_lib.FA_F_BCAST_ONLY, plan=plans[0])
        fns[(tag, "round")] = Reducer(lay, cl, o32, o64, flags=_lib.FA_F_BCAST, plan=plans[0])
        fns[(tag, "round_g10")] = Reducer(lay, cl, o32, o64, flags=_lib.FA_F_BCAST,
                                          plan=plans[_lib.FA_PLAN_TUNE_BCAST_G10])
        fns[(tag, "round_r03")] = Reducer(lay, cl, o32, o64, flags=_lib.FA_F_BCAST,
                                          plan=plans[_lib.FA_PLAN_TUNE_BCAST_R03])
    times = {k: [] for k in fns}
    for r in range(rounds):
        for k, fn in fns.items():
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) / 20 * 1e3)
    B = lay.state_bytes()
    for (tag, v), ts in times.items():
        ts = sorted(ts)
        nb = (lay.algorithmic_bytes(n) if v == "reduce" else (n + 1) * B if v == "bcast"
              else lay.algorithmic_bytes(n) + (n + 1) * B)
        print(json.dumps({"exp": "contig", "placement": tag, "variant": v,
                          "us_median": round(ts[len(ts) // 2], 2), "us_min": round(ts[0], 2),
                          "frac": round(nb / (ts[len(ts) // 2] * 1e-6) / 8e12, 4)}), flush=True)
    del keep


if __name__ == "__main__":
    main()
