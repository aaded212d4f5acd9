"""FedProx proximal-term kernels (csrc/prox.hip) through the
C ABI over the full wrn16_8 C100 parameter layout (2,690 chunks), against
torch's own per-tensor norms (train_fedprox.py:113-115) and gradients;
repeated launches identical; ragged tails, empty segments, one workgroup."""
import ctypes

import numpy as np
import pytest
import torch

from conftest import load_manifest
from feddct_amd.layout import BucketLayout

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _run(segs, numel, a, b, gout_val=0.7, reps=1):
    from feddct_amd import _lib
    from feddct_amd.prox import _NormPlan
    with torch.cuda.device(DEV):
        plan = _NormPlan(segs, numel)
    n = len(segs)
    norms = torch.full((max(1, n),), -1.0, device=DEV)
    total = torch.full((), -1.0, device=DEV)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    outs = []
    for _ in range(reps):
        _lib.check(_lib.lib.fa_prox_norms(plan.handle, a.data_ptr(), b.data_ptr(),
                                          norms.data_ptr(), total.data_ptr(), st))
        outs.append((norms.clone(), total.clone()))
    gout = torch.tensor(gout_val, device=DEV)
    ga = torch.full_like(a, 7.0)
    gb = torch.full_like(a, 7.0)
    _lib.check(_lib.lib.fa_prox_grad(plan.handle, a.data_ptr(), b.data_ptr(), norms.data_ptr(),
                                     gout.data_ptr(), 1.0, ga.data_ptr(), gb.data_ptr(), st))
    torch.cuda.synchronize()
    return outs, ga, gb


@pytest.fixture(scope="module")
def big():
    layout = BucketLayout.from_manifest(load_manifest("wrn16_8_c100"))
    segs = np.asarray(layout.segs32, np.int64).reshape(-1, 2)
    g = torch.Generator(device=DEV).manual_seed(5)
    b = torch.randn(layout.f32_numel, device=DEV, generator=g)
    a = b + 0.01 * torch.randn(layout.f32_numel, device=DEV, generator=g)
    a[segs[3, 0]:segs[3, 0] + segs[3, 1]] = b[segs[3, 0]:segs[3, 0] + segs[3, 1]]  # a zero norm
    return segs, layout.f32_numel, a, b


def test_prox_full_layout_matches_torch(big):
    segs, numel, a, b = big
    want = torch.stack([(a[o:o + m] - b[o:o + m]).norm(2) for o, m in segs])
    outs, ga, gb = _run(segs, numel, a, b, reps=3)
    norms, total = outs[0]
    torch.testing.assert_close(norms[:len(segs)], want, rtol=1e-5, atol=0)
    torch.testing.assert_close(total, want.sum(), rtol=1e-5, atol=0)
    for n2, t2 in outs[1:]:  # fixed reduction order: repeated launches identical
        assert torch.equal(n2, norms) and torch.equal(t2, total)
    # gradient: 0.7 * (a-b)/||a-b|| per tensor, 0 where the norm is 0
    for k, (o, m) in enumerate(segs):
        d = a[o:o + m] - b[o:o + m]
        exp = torch.zeros_like(d) if float(want[k]) == 0 else 0.7 * d / norms[k]
        torch.testing.assert_close(ga[o:o + m], exp, rtol=1e-6, atol=1e-9)
        assert torch.equal(gb[o:o + m], -ga[o:o + m])


def test_prox_tiny_and_ragged():
    """A handful of workgroups, ragged tails and an empty segment."""
    segs = np.array([(0, 3), (4, 0), (8, 1), (12, 1029), (1044, 5)], np.int64)
    numel = 1052
    g = torch.Generator(device=DEV).manual_seed(9)
    a = torch.randn(numel, device=DEV, generator=g)
    b = torch.randn(numel, device=DEV, generator=g)
    want = torch.stack([(a[o:o + m] - b[o:o + m]).norm(2) for o, m in segs])
    (norms, total), = _run(segs, numel, a, b)[0]
    torch.testing.assert_close(norms, want, rtol=1e-6, atol=0)
    torch.testing.assert_close(total, want.sum(), rtol=1e-6, atol=0)


def test_interleaved_plans():
    """Two norm plans launched alternately on one stream (each with its own
    partials buffer): results match torch and are identical launch after
    launch."""
    from feddct_amd import _lib
    from feddct_amd.prox import _NormPlan
    g = torch.Generator(device=DEV).manual_seed(11)
    res = []
    plans = []
    for numel, nseg in ((300_000, 7), (1_000_000, 40)):
        cut = np.linspace(0, numel, nseg + 1).astype(np.int64) // 64 * 64
        segs = np.stack([cut[:-1], cut[1:] - cut[:-1]], 1)
        a = torch.randn(numel, device=DEV, generator=g)
        b = torch.randn(numel, device=DEV, generator=g)
        with torch.cuda.device(DEV):
            plans.append((_NormPlan(segs, numel), segs, a, b))
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    outs = [[], []]
    for _ in range(4):
        for k, (plan, segs, a, b) in enumerate(plans):
            norms = torch.empty(len(segs), device=DEV)
            total = torch.empty((), device=DEV)
            _lib.check(_lib.lib.fa_prox_norms(plan.handle, a.data_ptr(), b.data_ptr(),
                                              norms.data_ptr(), total.data_ptr(), st))
            outs[k].append((norms, total))
    torch.cuda.synchronize()
    for k, (plan, segs, a, b) in enumerate(plans):
        want = torch.stack([(a[o:o + m] - b[o:o + m]).norm(2) for o, m in segs])
        n0, t0 = outs[k][0]
        torch.testing.assert_close(n0, want, rtol=1e-5, atol=0)
        for n, t in outs[k][1:]:
            assert torch.equal(n, n0) and torch.equal(t, t0)


@pytest.mark.parametrize("cpw", [2, 3, 4])
def test_prox_chunks_per_workgroup_same_bits(big, cpw):
    """r04: the forward's chunks-per-workgroup setting (default 1) changes
    the launch shape, not the partials: norms and total are the same bits,
    launch after launch."""
    from feddct_amd import _lib
    segs, numel, a, b = big
    ref, _, _ = _run(segs, numel, a, b)
    old = _lib.lib.fa_tune_prox_cpw(cpw)
    try:
        outs, _, _ = _run(segs, numel, a, b, reps=2)
    finally:
        _lib.lib.fa_tune_prox_cpw(old)
    for n, t in outs:
        assert torch.equal(n, ref[0][0]) and torch.equal(t, ref[0][1])


def test_prox_many_chunks():
    """4,200 chunks (more partials than the finish stages in one load batch):
    still torch's norms, repeated launches identical."""
    numel = 4200 * 4096
    cut = np.linspace(0, numel, 9).astype(np.int64) // 64 * 64
    segs = np.stack([cut[:-1], cut[1:] - cut[:-1]], 1)
    g = torch.Generator(device=DEV).manual_seed(13)
    a = torch.randn(numel, device=DEV, generator=g)
    b = torch.randn(numel, device=DEV, generator=g)
    want = torch.stack([(a[o:o + m] - b[o:o + m]).norm(2) for o, m in segs])
    outs, _, _ = _run(segs, numel, a, b, reps=2)
    torch.testing.assert_close(outs[0][0], want, rtol=1e-5, atol=0)
    assert torch.equal(outs[1][0], outs[0][0])
