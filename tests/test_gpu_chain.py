"""GPU: chained segments of the cascade (fa_reduce_chain) — the exact form
of the client-sharded round.  Client groups reduced by
separate launches, each continuing the previous group's accumulator state in
slot order, give the single launch's bits; the layout's scalar columns
(ILP-4 tails, M==1, int64) are reduced over all clients' raw values, as the
multi-GPU round gathers them.  Reference order: train_feddct.py:42-50 /
train_fedavg.py:145-146 over the slots in list order."""
import ctypes

import numpy as np
import pytest
import torch

from conftest import load_manifest
from feddct_amd import synth
from feddct_amd.layout import BucketLayout
from helpers import bits_equal, buckets_to_state, states_to_buckets
from oracle import torch_order as O

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def lib():
    from feddct_amd import _lib
    torch.cuda.set_device(DEV)
    return _lib


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _plans(lib, layout):
    from feddct_amd.partition import layout_tiles
    _, tiles = layout_tiles(layout)
    vec, rest = tiles[tiles[:, 2] == 0], tiles[tiles[:, 2] != 0]
    mk = (lambda t: lib.Plan(None, layout.f32_numel, None, layout.i64_numel, 0, tiles=t)
          if len(t) else None)
    return mk(vec), mk(rest)


def chained(lib, layout, buckets, bounds, weights=None, inplace=True):
    """Reduce ``buckets`` as the chained groups [bounds[g], bounds[g+1])."""
    vec, rest = _plans(lib, layout)
    n = len(buckets)
    plane = layout.f32_numel
    out32 = torch.full_like(buckets[0][0], np.nan)
    out64 = torch.full_like(buckets[0][1], -7)
    st = [torch.full((4 * plane,), np.nan, device=DEV) for _ in range(1 if inplace else 2)]
    w = None if weights is None else np.asarray(weights, np.float32)
    prev = None
    for g, (a, b) in enumerate(zip(bounds, bounds[1:])):
        last = b == n
        dst = None if last else st[g % len(st)]
        ch = lib.FaChain(a, n, prev.data_ptr() if prev is not None else None,
                         dst.data_ptr() if dst is not None else None, plane)
        wa = None if w is None else (ctypes.c_float * (b - a))(*map(float, w[a:b]))
        if vec is not None:
            lib.check(lib.lib.fa_reduce_chain(
                vec.handle, lib.ptr_array([x[0].data_ptr() for x in buckets[a:b]]), b - a, wa,
                ctypes.byref(ch), out32.data_ptr() if last else None, 0, _stream()),
                "fa_reduce_chain")
        prev = dst
    if rest is not None:
        wall = None if w is None else (ctypes.c_float * n)(*map(float, w))
        lib.check(lib.lib.fa_reduce(rest.handle, lib.ptr_array([x[0].data_ptr() for x in buckets]),
                                    lib.ptr_array([x[1].data_ptr() for x in buckets]), n, wall,
                                    out32.data_ptr(), out64.data_ptr(), 0, _stream()), "tails")
    torch.cuda.synchronize()
    return out32, out64


def single(lib, layout, buckets, weights=None):
    plan = lib.Plan(layout.segs32, layout.f32_numel, layout.segs64, layout.i64_numel)
    n = len(buckets)
    out32 = torch.full_like(buckets[0][0], np.nan)
    out64 = torch.full_like(buckets[0][1], -7)
    w = None if weights is None else (ctypes.c_float * n)(*map(float, weights))
    lib.check(lib.lib.fa_reduce(plan.handle, lib.ptr_array([x[0].data_ptr() for x in buckets]),
                                lib.ptr_array([x[1].data_ptr() for x in buckets]), n, w,
                                out32.data_ptr(), out64.data_ptr(), 0, _stream()), "fa_reduce")
    torch.cuda.synchronize()
    return out32, out64


MAN = {"keys": [{"key": f"k{j}", "shape": [m] if m else [], "dtype": "float32"}
                for j, m in enumerate([100, 4096, 33, 2048 + 8, 7, 0, 5000, 64, 1])]
       + [{"key": "nbt", "shape": [], "dtype": "int64"}]}


def _cuts(rng, n, groups):
    if groups >= n:
        return list(range(n + 1))
    c = sorted(rng.choice(np.arange(1, n), size=groups - 1, replace=False).tolist())
    return [0] + c + [n]


@pytest.mark.parametrize("n", [2, 5, 16, 20, 24, 33, 64, 100, 257, 300])
@pytest.mark.parametrize("groups", [2, 3, 8])
def test_chain_equals_one_launch(lib, n, groups):
    layout = BucketLayout.from_manifest(MAN)
    states = [synth.gen_state(MAN, i, synth.MODE_ADVERSARIAL) for i in range(n)]
    bk = states_to_buckets(layout, states, DEV)
    r32, r64 = single(lib, layout, bk)
    rng = np.random.default_rng(n * 10 + groups)
    for bounds in (_cuts(rng, n, groups), [0] + [b for b in (16, 32, 256) if b < n] + [n]):
        for inplace in (True, False):
            o32, o64 = chained(lib, layout, bk, bounds, inplace=inplace)
            for (k, a), (_, b) in zip(buckets_to_state(layout, o32, o64),
                                      buckets_to_state(layout, r32, r64)):
                assert bits_equal(a, b), (n, bounds, k)
    want = dict(O.aggregate_state(states))
    for k, v in buckets_to_state(layout, o32, o64):
        assert bits_equal(v, want[k]), k


def test_chain_weighted(lib):
    n = 20
    layout = BucketLayout.from_manifest(MAN)
    states = [synth.gen_state(MAN, i, synth.MODE_ADVERSARIAL) for i in range(n)]
    bk = states_to_buckets(layout, states, DEV)
    w = O.weights_from_sizes(np.arange(1, n + 1) * 7 + 3)
    r32, _ = single(lib, layout, bk, weights=w)
    o32, _ = chained(lib, layout, bk, [0, 7, 13, 20], weights=w)
    assert bits_equal(o32.cpu().numpy(), r32.cpu().numpy())


@pytest.mark.parametrize("groups", [8, 3])
def test_chain_full_size_feddct_c100_digests(lib, golden, groups):
    """BASELINE config 5: 24 FedDCT slots (main + proxy in one bucket) as 8
    shards of 3 (the 8-GPU split) or 3 of 8, chained: both reference digests."""
    from feddct_amd.workload import joint_manifest, make_clients
    mm = load_manifest("wrnsl16_8_sf4_c100_main")
    pm = load_manifest("wrnsl16_8_sf4_c100_proxy")
    layout = BucketLayout.from_manifest(joint_manifest([mm, pm]))
    n = 24
    cl = make_clients(layout, [(mm, "0."), (pm, "1.")], range(n), DEV)
    bounds = list(range(0, n + 1, n // groups))
    o32, o64 = chained(lib, layout, cl, bounds)
    state = buckets_to_state(layout, o32, o64)
    for pf, lay in (("0.", "main"), ("1.", "proxy")):
        part = [(k[2:], v) for k, v in state if k.startswith(pf)]
        assert O.state_digest(part) == golden["digests"][f"feddct/wrnsl16_8_sf4_c100_{lay}/n{n}"]


def test_chain_full_size_fedavg_digest(lib, golden):
    """BASELINE config 2 as 2 ranks x 10 clients: the wrn16_8 N=20 digest."""
    from feddct_amd.workload import make_clients
    man = load_manifest("wrn16_8_c10")
    layout = BucketLayout.from_manifest(man)
    cl = make_clients(layout, man, range(20), DEV)
    o32, o64 = chained(lib, layout, cl, [0, 10, 20])
    assert (O.state_digest(buckets_to_state(layout, o32, o64))
            == golden["digests"]["fedavg/wrn16_8_c10/n20"])


def test_chain_errors(lib):
    layout = BucketLayout.from_manifest(MAN)
    full = lib.Plan(layout.segs32, layout.f32_numel, layout.segs64, layout.i64_numel)
    vec, _ = _plans(lib, layout)
    b = torch.zeros(4 * layout.f32_numel, device=DEV)
    ptrs = lib.ptr_array([b.data_ptr()] * 4)
    L = lib.lib

    def call(plan, n, ch, out=b.data_ptr()):
        return L.fa_reduce_chain(plan.handle, ptrs, n, None, ctypes.byref(ch), out, 0, None)
    P = layout.f32_numel
    assert call(full, 2, lib.FaChain(0, 4, None, b.data_ptr(), P)) == lib.FA_E_INVAL
    assert b"scalar tiles" in L.fa_last_error()
    assert call(vec, 2, lib.FaChain(2, 4, None, None, P)) == lib.FA_E_INVAL   # state_in missing
    assert call(vec, 2, lib.FaChain(0, 4, None, None, P)) == lib.FA_E_INVAL   # finish too early
    assert call(vec, 3, lib.FaChain(2, 4, b.data_ptr(), None, P)) == lib.FA_E_INVAL  # > n_total
    assert call(vec, 2, lib.FaChain(0, 4, None, b.data_ptr(), 10)) == lib.FA_E_INVAL  # plane
    assert call(vec, 1, lib.FaChain(0, lib.FA_MAX_CLIENTS + 1, None, b.data_ptr(), P)) == lib.FA_E_RANGE
