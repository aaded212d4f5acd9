"""pipe2 experiment (r05, profiles/r05_exp_pipe2_n.jsonl): the batch form vs
the two-deep client pipeline on plain tables, over client counts on the
wrn16_8 C10 and C100 layouts, mean and weighted; same process, alternated;
bits compared.  It ran against an experiment build that read the knobs
FA_EXP_PIPE2 / FA_EXP_PIPE2_RULE per launch; the product now decides by
fedagg.hip pipe_rule, so on the shipped library both columns are the
product (kept as the record of how the rule was measured; tools/ab_lib.py
with AB_SLAB=1 compares two library builds)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from feddct_amd.aggregate import client_weights  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import Reducer, load_manifest, make_clients  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    ns = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else \
        [2, 3, 5, 8, 12, 16, 20, 24, 32, 48, 64, 100]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    os.environ["FA_EXP_PIPE2_RULE"] = "1"
    for name in ("wrn16_8_c10", "wrn16_8_c100"):
        man = load_manifest(name)
        lay = BucketLayout.from_manifest(man)
        allc = make_clients(lay, [(man, "")], range(max(ns)), dev)
        for n in ns:
            cl = allc[:n]
            o32, o64 = torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1])
            for wname, w in (("mean", None), ("weighted", client_weights(
                    [2500 + 97 * ((7 * i) % 11) for i in range(n)]))):
                red = Reducer(lay, cl, o32, o64, weights=w)
                times = {k: [] for k in ("0", "1")}
                outs = {}
                reps = max(5, min(40, 4000 // n))
                for _ in range(rounds):
                    for k in times:
                        os.environ["FA_EXP_PIPE2"] = k
                        for _ in range(2):
                            red()
                        e0, e1 = (torch.cuda.Event(enable_timing=True),
                                  torch.cuda.Event(enable_timing=True))
                        e0.record()
                        for _ in range(reps):
                            red()
                        e1.record()
                        e1.synchronize()
                        times[k].append(e0.elapsed_time(e1) / reps * 1e3)
                        outs[k] = o32.clone()
                same = bool(torch.equal(outs["0"].view(torch.int32), outs["1"].view(torch.int32)))
                med = {k: sorted(v)[len(v) // 2] for k, v in times.items()}
                ntiles, slots = red.plan.launch_shape(n, weighted=w is not None)
                print(json.dumps({"exp": "pipe2_n", "layout": name, "n": n, "form": wname,
                                  "tiles": ntiles, "slots": slots,
                                  "product_us": round(med["0"], 2), "pipe2_us": round(med["1"], 2),
                                  "ratio": round(med["1"] / med["0"], 4), "same_bits": same}),
                      flush=True)
                del red
        del allc
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
