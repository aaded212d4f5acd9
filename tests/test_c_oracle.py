"""The C restatement (oracle/fa_oracle.c) agrees bit-for-bit with the numpy
oracle and with the reference's goldens: two independent restatements."""
import numpy as np
import pytest

from conftest import load_manifest
from feddct_amd import synth
from feddct_amd.layout import BucketLayout
from oracle import c_oracle
from oracle import torch_order as O


def _buckets(layout, states):
    out32, out64 = [], []
    for st in states:
        f = np.zeros(layout.f32_numel, np.float32)
        i = np.zeros(max(1, layout.i64_numel), np.int64)
        for k, v in st:
            s = layout.by_key[k]
            (i if s.kind == "i64" else f)[s.offset:s.offset + s.numel] = np.asarray(v).reshape(-1)
        out32.append(f)
        out64.append(i)
    return out32, out64


@pytest.mark.parametrize("n", [1, 2, 5, 8, 9, 16, 17, 20, 33, 64, 257])
def test_c_oracle_equals_numpy_oracle(n):
    sizes = [1, 2, 3, 4, 5, 7, 8, 9, 31, 32, 33, 100, 1000]
    man = {"keys": [{"key": f"k{j}", "shape": [m], "dtype": "float32"} for j, m in enumerate(sizes)]
           + [{"key": "nbt", "shape": [], "dtype": "int64"}]}
    layout = BucketLayout.from_manifest(man)
    states = [synth.gen_state(man, i, synth.MODE_ADVERSARIAL) for i in range(n)]
    b32, b64 = _buckets(layout, states)
    got32 = c_oracle.reduce_f32(b32, layout.segs32)
    got64 = c_oracle.reduce_i64(b64, layout.segs64)
    for k, want in O.aggregate_state(states):
        s = layout.by_key[k]
        src = got64 if s.kind == "i64" else got32
        got = src[s.offset:s.offset + s.numel].reshape(s.shape)
        assert got.tobytes() == np.asarray(want).tobytes(), (n, k)
    w = O.weights_from_sizes(np.arange(1, n + 1))
    gw = c_oracle.reduce_f32(b32, layout.segs32, weights=w)
    for j, e in enumerate(man["keys"][:-1]):
        s = layout.by_key[e["key"]]
        x = np.stack([st[j][1] for st in states]).astype(np.float32)
        assert gw[s.offset:s.offset + s.numel].tobytes() == O.weighted_sum0(x, w).reshape(-1).tobytes()


def test_c_oracle_full_size_digest(golden):
    man = load_manifest("wrn16_8_c10")
    layout = BucketLayout.from_manifest(man)
    states = [synth.gen_state(man, i) for i in range(20)]
    b32, b64 = _buckets(layout, states)
    o32 = c_oracle.reduce_f32(b32, layout.segs32)
    o64 = c_oracle.reduce_i64(b64, layout.segs64)
    res = []
    for s in layout.slots:
        src = o64 if s.kind == "i64" else o32
        res.append((s.key, src[s.offset:s.offset + s.numel].reshape(s.shape)))
    assert O.state_digest(res) == golden["digests"]["fedavg/wrn16_8_c10/n20"]
