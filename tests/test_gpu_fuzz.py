"""GPU fuzz: random bucket layouts straight through the C ABI — unaligned
segment offsets, gaps that are or are not padding, every column rule, 1–140
clients (inline and table pointer paths), three tile sizes, weighted and
unweighted, FA_F_SUM_ONLY and FA_F_BCAST — against the oracle, bit for bit,
and elements outside the segments must stay untouched unless the plan says
they are padding."""
import ctypes

import numpy as np
import pytest
import torch

from helpers import bits_equal
from oracle import torch_order as O

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)
SIZES = [0, 1, 2, 3, 4, 5, 7, 8, 9, 31, 32, 33, 63, 64, 65, 100, 257, 1023, 2049, 4100]


def _case(seed):
    rng = np.random.default_rng(seed)
    nseg = int(rng.integers(1, 10))
    segs, off = [], int(rng.integers(0, 5)) * 4
    for _ in range(nseg):
        m = int(rng.choice(SIZES)) if rng.random() < 0.8 else int(rng.integers(1, 6000))
        segs.append((off, m))
        gap = int(rng.integers(0, 70))
        if rng.random() < 0.5:
            gap = (gap + 3) // 4 * 4  # often keep 16-B alignment
        off += m + gap
    numel = off + 64
    n = int(rng.choice([1, 2, 3, 5, 8, 15, 16, 17, 20, 33, 40, 129, 140]))
    segs64, o64 = [], 0
    for _ in range(int(rng.integers(0, 4))):  # int64 keys: scalars and longer ones
        m = int(rng.choice([1, 1, 2, 5, 33, 100]))
        segs64.append((o64, m))
        o64 += m
    return dict(segs=np.array(segs, np.int64).reshape(-1, 2), numel=numel, n=n,
                segs64=np.array(segs64, np.int64).reshape(-1, 2), numel64=max(1, o64),
                tile=int(rng.choice([1024, 2048, 4096])),
                gaps_pad=bool(rng.random() < 0.5), weighted=bool(rng.random() < 0.3),
                flags=int(rng.choice([0, 0, 1, 2])), rng=rng)


@pytest.mark.parametrize("seed", range(200))
def test_random_layouts_bit_exact(seed):
    from feddct_amd import _lib
    torch.cuda.set_device(DEV)
    c = _case(seed)
    rng, n, numel = c["rng"], c["n"], c["numel"]
    flags = _lib.FA_PLAN_GAPS_ARE_PADDING if c["gaps_pad"] else 0
    # the broadcast (FA_F_BCAST cases) is a flat copy in client groups on
    # gap-padded plans, client groups per tile on the others; launch shapes
    # rotate over the balanced tables (default) and the plain one
    flags |= (0, _lib.FA_PLAN_TUNE_NO_BALANCE)[seed % 2]
    plan = _lib.Plan(c["segs"], numel, c["segs64"], c["numel64"], tile_elems=c["tile"],
                     flags=flags)
    # adversarial-range values, exact small integers for the int64 keys
    x32 = (rng.standard_normal((n, numel)) * np.exp2(rng.integers(-20, 20, (n, numel)))
           ).astype(np.float32)
    x64 = rng.integers(-2 ** 20, 2 ** 20, (n, c["numel64"]), dtype=np.int64)
    b32 = [torch.from_numpy(x32[i].copy()).to(DEV) for i in range(n)]
    b64 = [torch.from_numpy(x64[i].copy()).to(DEV) for i in range(n)]
    out32 = torch.full((numel,), 7.25, dtype=torch.float32, device=DEV)
    out64 = torch.full((c["numel64"],), -3, dtype=torch.int64, device=DEV)
    w = None
    if c["weighted"]:
        wv = O.weights_from_sizes(rng.integers(1, 1000, n))
        w = (ctypes.c_float * n)(*[float(v) for v in wv])
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(_lib.lib.fa_reduce(plan.handle, _lib.ptr_array([t.data_ptr() for t in b32]),
                                  _lib.ptr_array([t.data_ptr() for t in b64]), n, w,
                                  out32.data_ptr(), out64.data_ptr(), c["flags"], st),
               "fa_reduce")
    torch.cuda.synchronize()
    got32 = out32.cpu().numpy()
    got64 = out64.cpu().numpy()
    inside = np.zeros(numel, bool)
    for o, m in c["segs"]:
        inside[o:o + m] = True
        if m == 0:
            continue
        cols = x32[:, o:o + m]
        if c["weighted"]:
            want = O.weighted_sum0(cols, np.asarray(wv, np.float32))
        elif c["flags"] & _lib.FA_F_SUM_ONLY:
            want = O.torch_sum0(cols)
        else:
            want = O.torch_mean0(cols)
        assert bits_equal(got32[o:o + m], want), (seed, o, m)
    for o, m in c["segs64"]:
        assert np.array_equal(got64[o:o + m], O.mean_i64_trunc(x64[:, o:o + m])), (seed, o)
    if not c["gaps_pad"]:
        assert (got32[~inside] == np.float32(7.25)).all(), "wrote outside the segments"
    if c["flags"] & _lib.FA_F_BCAST:
        for i, t in enumerate(b32):
            assert bits_equal(t.cpu().numpy()[inside], got32[inside]), "broadcast"
            if not c["gaps_pad"]:
                assert bits_equal(t.cpu().numpy()[~inside], x32[i][~inside]), "broadcast gaps"
