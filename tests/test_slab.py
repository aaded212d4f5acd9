"""Slab-carved buckets (feddct_amd/slab.py): each bucket a storage of its
own inside one shared allocation.  The carve is device-independent, so it is
exercised here on CPU (force=True); the GPU tests and the bench use it on
the device through arena.alloc_buckets / workload.make_clients."""
import gc
import io

import pytest
import torch

from feddct_amd import slab


@pytest.fixture(autouse=True)
def _fresh():
    slab.release()
    yield
    slab.release()


def test_carve_zeroed_aligned_and_disjoint():
    a = slab.carve(1000, torch.float32, "cpu", force=True)
    b = slab.carve(10, torch.int64, "cpu", force=True)
    c = slab.carve(70000, torch.float32, "cpu", force=True)
    for t, n in ((a, 1000), (b, 10), (c, 70000)):
        assert t.numel() == n and t.storage_offset() == 0
        assert t.untyped_storage().nbytes() == n * t.element_size()
        assert (t.data_ptr() - a.data_ptr()) % slab.ALIGN == 0   # from the slab's base
        assert not t.any()
    # one slab, buckets in carve order at ALIGN-rounded steps
    assert b.data_ptr() - a.data_ptr() == slab.ALIGN
    assert c.data_ptr() - b.data_ptr() == slab.ALIGN
    a.fill_(1.0)
    b.fill_(-1)
    c.fill_(2.0)
    assert a.sum().item() == 1000 and b.sum().item() == -10 and c.sum().item() == 140000


def test_new_slab_when_full_and_buckets_outlive_release():
    big = (slab.MIN_SLAB // 2)
    a = slab.carve(big // 4, torch.float32, "cpu", force=True)
    b = slab.carve(big // 4, torch.float32, "cpu", force=True)
    c = slab.carve(big // 4, torch.float32, "cpu", force=True)   # MIN_SLAB would overflow
    assert b.data_ptr() - a.data_ptr() == big
    a.fill_(3.0)
    c.fill_(4.0)
    slab.release()
    gc.collect()
    # the storages keep their slab alive
    assert a[:5].tolist() == [3.0] * 5 and c[-5:].tolist() == [4.0] * 5


def test_save_writes_only_the_bucket():
    a = slab.carve(1024, torch.float32, "cpu", force=True)
    slab.carve(1 << 20, torch.float32, "cpu", force=True)
    a.copy_(torch.arange(1024, dtype=torch.float32))
    buf = io.BytesIO()
    torch.save({"w": a[:512].view(16, 32), "b": a[512:]}, buf)
    assert len(buf.getvalue()) < 1024 * 4 + 4096
    back = torch.load(io.BytesIO(buf.getvalue()), weights_only=True)
    assert torch.equal(back["w"].flatten(), torch.arange(512, dtype=torch.float32))
    assert back["w"].untyped_storage().nbytes() == 1024 * 4


def test_slabs_off_and_cpu_default(monkeypatch):
    t = slab.carve(100, torch.float32, "cpu")       # no force: plain allocation
    assert t.untyped_storage().nbytes() == 400 and not t.any()
    monkeypatch.setenv("FA_SLAB", "0")
    assert not slab.enabled()
    monkeypatch.setenv("FA_SLAB", "1")
    assert slab.enabled()


def test_slab_size_rule():
    assert slab._slab_bytes(1) == slab.MIN_SLAB
    n = 44 << 20
    assert slab._slab_bytes(n) == slab.SLAB_BUCKETS * n
    assert slab._slab_bytes(1 << 30) == slab.MAX_SLAB
    assert slab._slab_bytes(3 << 30) == 3 << 30


def test_slab_sized_for_the_expected_bucket_count():
    """a slab started inside expecting(k) holds k buckets of the
    requested size (within MIN_SLAB..MAX_SLAB), not SLAB_BUCKETS."""
    n = 44 << 20
    with slab.expecting(21):
        assert slab._slab_bytes(n) == 21 * n
        with slab.expecting(3):
            assert slab._slab_bytes(n) == 3 * n
            assert slab._slab_bytes(1) == slab.MIN_SLAB
        assert slab._slab_bytes(n) == 21 * n
        assert slab._slab_bytes(1 << 30) == slab.MAX_SLAB
    assert slab._slab_bytes(n) == slab.SLAB_BUCKETS * n
    slab.release()
    with slab.expecting(4):
        a = slab.carve((20 << 20) // 4, torch.float32, "cpu", force=True)
    base = a.untyped_storage()
    assert a.numel() == 5 << 20
    slab.release()
