"""Digests of the client-size-WEIGHTED reduction at full size (SURVEY.md
§8 a9: an extension — the reference has no weights, so its parity is pinned
by the build's own definition: sum_i fp32(x_i * w_i) in the torch order,
int64 keys the unweighted mean + truncation).

Computed here on the CPU by the C restatement (oracle/fa_oracle.c) over
buckets filled by the portable PRNG (feddct_amd/synth.py, the same inputs
the GPU regenerates), and cross-checked against the numpy oracle on a
sample of keys.  Output: tests/golden/weighted_digests.json.

    python tests/golden/make_weighted_digests.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

from feddct_amd import synth  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from oracle import c_oracle  # noqa: E402
from oracle import torch_order as O  # noqa: E402

# name -> (layout, clients, client sizes); weights w_i = fp32(n_i / sum n)
CASES = {
    # bench.py's weighted cfg2 line: sizes 1..20
    "weighted/wrn16_8_c10/n20/sizes_1_20": ("wrn16_8_c10", 20, list(range(1, 21))),
    # BASELINE config 4 (FedProx C100, quantity-skewed shards; bench other_configs)
    "weighted/wrn16_8_c100/n20/cfg4_sizes": ("wrn16_8_c100", 20,
                                             [2500 + 97 * ((7 * i) % 11) for i in range(20)]),
}


def buckets(layout, man, n):
    f32s, i64s = [], []
    for c in range(n):
        f = np.zeros(layout.f32_numel, np.float32)
        i = np.zeros(max(1, layout.i64_numel), np.int64)
        for k, v in synth.gen_state(man, c):
            s = layout.by_key[k]
            (i if s.kind == "i64" else f)[s.offset:s.offset + s.numel] = np.asarray(v).reshape(-1)
        f32s.append(f)
        i64s.append(i)
    return f32s, i64s


def main():
    out = {}
    for name, (lay, n, sizes) in CASES.items():
        with open(os.path.join(REPO, "feddct_amd", "manifests", lay + ".json")) as f:
            man = json.load(f)
        layout = BucketLayout.from_manifest(man)
        w = O.weights_from_sizes(sizes)
        f32s, i64s = buckets(layout, man, n)
        r32 = c_oracle.reduce_f32(f32s, layout.segs32, weights=w)
        r64 = c_oracle.reduce_i64(i64s, layout.segs64)
        state = []
        for s in layout.slots:
            src = r64 if s.kind == "i64" else r32
            state.append((s.key, src[s.offset:s.offset + s.numel].reshape(s.shape)))
        # cross-check a few keys (smallest + a tail-bearing one) with numpy
        for s in [x for x in layout.slots if x.kind != "i64"][-3:]:
            x = np.stack([b[s.offset:s.offset + s.numel] for b in f32s])
            assert O.weighted_sum0(x, w).tobytes() == r32[s.offset:s.offset + s.numel].tobytes()
        out[name] = {"digest": O.state_digest(state), "weights": [float(v) for v in w],
                     "sizes": sizes}
        print(name, out[name]["digest"])
    with open(os.path.join(REPO, "tests", "golden", "weighted_digests.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
