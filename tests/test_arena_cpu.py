"""Arena binding and the shim's host-side checks (no GPU needed)."""
import pytest
import torch

from feddct_amd.arena import ModuleArena, get_arena, state_owners
from feddct_amd.layout import BucketLayout


def net():
    return torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.BatchNorm2d(8),
                               torch.nn.Linear(5, 2))


def test_binding_keeps_values_and_parameter_objects():
    m = net()
    before = {k: v.clone() for k, v in m.state_dict().items()}
    params = list(m.parameters())
    opt = torch.optim.SGD(m.parameters(), lr=0.1)
    L = BucketLayout.from_state_dict(m.state_dict())
    a = ModuleArena(m, L)
    assert a.valid()
    assert [id(p) for p in m.parameters()] == [id(p) for p in params]
    for k, v in m.state_dict().items():
        assert torch.equal(v, before[k])
        s = L.by_key[k]
        bucket = a.i64 if s.kind == "i64" else a.f32
        assert v.data_ptr() == bucket[s.offset:].data_ptr()
    # training writes land in the bucket
    loss = m[2](torch.randn(4, 5)).sum()
    loss.backward()
    opt.step()
    s = L.by_key["2.weight"]
    assert torch.equal(a.f32[s.offset:s.offset + s.numel].view(s.shape), m[2].weight.detach())


def test_rebind_detection():
    m = net()
    L = BucketLayout.from_state_dict(m.state_dict())
    a = get_arena(m, L)
    assert get_arena(m, L) is a
    m[0].weight = torch.nn.Parameter(torch.zeros_like(m[0].weight))
    assert not a.valid()
    b = get_arena(m, L)
    assert b is not a and b.valid()
    assert torch.equal(m[0].weight.detach(), torch.zeros_like(m[0].weight))


def test_arena_errors_like_reference():
    m = net()
    L = BucketLayout.from_state_dict(m.state_dict())
    other = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3))
    with pytest.raises(KeyError):
        ModuleArena(other, L)
    wrong = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 5), torch.nn.BatchNorm2d(8),
                                torch.nn.Linear(5, 2))
    w0 = wrong[0].weight.data_ptr()
    with pytest.raises(RuntimeError, match="equal size"):
        ModuleArena(wrong, L)
    assert wrong[0].weight.data_ptr() == w0, "a failed bind must not touch the module"
    # a client whose key dtype differs from the global's is staged like the
    # reference's .float() (train_fedavg.py:145) instead of refused ...
    half = net().half()
    ha = ModuleArena(half, L)
    assert len(ha._packed) == 8   # every float key; the int64 one binds in place
    ha.pack()
    s = L.by_key["0.weight"]
    assert torch.equal(ha.f32[s.offset:s.offset + s.numel].view(s.shape), half[0].weight.float())
    # ... except a fractional value in an int64 key, which the int64 bucket
    # cannot hold
    fl = net()
    fl[1].num_batches_tracked = torch.tensor(2.5)
    with pytest.raises(TypeError, match="cannot be staged"):
        ModuleArena(fl, L)
    bigger = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.BatchNorm2d(8),
                                 torch.nn.Linear(5, 2), torch.nn.Linear(2, 2))
    a = ModuleArena(bigger, L)
    assert a.extra_keys == ["3.weight", "3.bias"]


def test_state_owners_order_matches_state_dict():
    m = net()
    assert list(state_owners(m).keys()) == list(m.state_dict().keys())


def test_pack_unpack_roundtrip_dtypes():
    m = torch.nn.Module()
    m.register_buffer("h", torch.tensor([1.5, -2.25], dtype=torch.float16))
    m.register_buffer("b", torch.tensor([True, False]))
    m.register_buffer("i", torch.tensor([7, -3], dtype=torch.int32))
    L = BucketLayout.from_state_dict(m.state_dict())
    a = ModuleArena(m, L)
    a.pack()
    for k in ("h", "b", "i"):
        s = L.by_key[k]
        assert torch.equal(a.f32[s.offset:s.offset + s.numel], m.state_dict()[k].float())
    s = L.by_key["i"]
    a.f32[s.offset:s.offset + s.numel] = torch.tensor([2.9, -2.9])
    a.unpack()
    assert m.i.tolist() == [2, -2]  # copy_ float -> int truncates


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU behaviour")
def test_no_cpu_fallback():
    from feddct_amd.aggregate import server_aggregate
    with pytest.raises(RuntimeError, match="no CPU fallback|no HIP device"):
        server_aggregate(net(), [net(), net()])


def test_empty_client_list_like_torch_stack():
    from feddct_amd.aggregate import server_aggregate
    with pytest.raises(RuntimeError, match="non-empty"):
        server_aggregate(net(), [])


def test_structure_change_after_binding_is_seen():
    """A buffer registered after binding changes the key set: the arena turns
    invalid and the engine's layout picks the new key up (the reference's
    per-call state_dict() would see it)."""
    from feddct_amd.aggregate import Engine
    m = net()
    e = Engine()
    L = e.layout_of(m)
    a = get_arena(m, L)
    assert a.valid() and e.layout_of(m) is L
    other = torch.nn.Linear(2, 2)  # registering elsewhere bumps the generation only
    assert a.valid()
    m[1].register_buffer("extra_stat", torch.ones(3))
    assert not a.valid()
    L2 = e.layout_of(m)
    assert "1.extra_stat" in L2.keys and L2 is not L
    del other


def test_kernel_writes_bump_autograd_versions():
    """The kernel overwrites bucket memory through raw pointers; like the
    reference's load_state_dict (an in-place copy_), the shim then bumps every
    bound tensor's version, so a graph that saved the old values fails loudly
    in backward instead of silently using the new ones."""
    m = net()
    a = ModuleArena(m, BucketLayout.from_state_dict(m.state_dict()))
    w = m[2].weight
    y = (w * w).sum()  # saves w for backward
    v0 = w._version
    a.mark_written()
    assert w._version > v0
    with pytest.raises(RuntimeError, match="modified by an inplace operation"):
        y.backward()
    # a graph built after the write is fine
    (w * w).sum().backward()


def test_c_helper_matches_python_checks():
    """csrc/shim.cpp (valid_views / bump_versions) against the Python loops
    that define them, on intact and tampered modules."""
    from feddct_amd import arena as A
    if A._fa_shim is None:
        pytest.skip("_fa_shim not built")
    m = net()
    a = ModuleArena(m, BucketLayout.from_state_dict(m.state_dict()))
    assert a.valid(use_shim=True) and a.valid(use_shim=False)
    w = m[0].weight
    old = w.data
    w.data = torch.zeros_like(old)  # a .data swap (what model.to() does)
    assert not a.valid(use_shim=True) and not a.valid(use_shim=False)
    w.data = old
    assert a.valid(use_shim=True)
    m[1]._parameters["bias"] = torch.nn.Parameter(m[1].bias.detach().clone())  # replaced
    assert not a.valid(use_shim=True) and not a.valid(use_shim=False)
    v = [t._version for t in a._written]
    A._fa_shim.bump_versions(a._written)
    assert all(t._version > x for t, x in zip(a._written, v))
    with pytest.raises(TypeError):
        A._fa_shim.bump_versions((1,))


def test_tied_layout_refuses_untied_client():
    """the alias map is part of a layout's identity, and a client
    whose tensors are not tied where the global's are is refused instead of
    being silently tied."""
    def tied():
        m = torch.nn.Sequential(torch.nn.Linear(4, 4), torch.nn.Linear(4, 4))
        m[1].weight = m[0].weight
        return m
    untied = torch.nn.Sequential(torch.nn.Linear(4, 4), torch.nn.Linear(4, 4))
    Lt = BucketLayout.from_state_dict(tied().state_dict())
    Lu = BucketLayout.from_state_dict(untied.state_dict())
    assert Lt.by_key["1.weight"].alias_of == "0.weight"
    assert Lt != Lu and Lt.signature != Lu.signature
    w1 = untied[1].weight.detach().clone()
    with pytest.raises(RuntimeError, match="tied"):
        ModuleArena(untied, Lt)
    assert torch.equal(untied[1].weight.detach(), w1)
    t = tied()
    a = ModuleArena(t, Lt)
    assert t[0].weight is t[1].weight and a.valid()


def test_pair_halves_keep_their_own_storage(tmp_path):
    """a FedDCT slot (main + proxy) shares one bucket for the
    launch, but each model's tensors sit in a storage of its own, so saving
    one model's state_dict (train_feddct.py:455,463) writes only its bytes."""
    import io
    from feddct_amd.aggregate import _Pair
    main = torch.nn.Sequential(torch.nn.Conv2d(3, 4, 3), torch.nn.BatchNorm2d(4))
    proxy = torch.nn.Sequential(torch.nn.Linear(300, 200), torch.nn.BatchNorm1d(200))
    ref_main = {k: v.clone() for k, v in main.state_dict().items()}
    pair = _Pair(main, proxy)
    L = BucketLayout.from_state_dict(pair.state_dict())
    a = ModuleArena(pair, L)
    for m, pre in ((main, "0."), (proxy, "1.")):
        own = BucketLayout.from_state_dict(m.state_dict())
        stores = {(t.untyped_storage().data_ptr(), t.untyped_storage().nbytes())
                  for t in m.state_dict().values()}
        assert len(stores) == 2          # one fp32 + one int64 storage
        assert sum(nb for _, nb in stores) <= 4 * own.f32_numel + 8 * own.i64_numel
        for k, v in m.state_dict().items():   # still the pair bucket's memory
            s = L.by_key[pre + k]
            b = a.i64 if s.kind == "i64" else a.f32
            assert v.data_ptr() == b[s.offset:].data_ptr()
    for k, v in main.state_dict().items():
        assert torch.equal(v, ref_main[k])
    bm, bp = io.BytesIO(), io.BytesIO()
    torch.save(main.state_dict(), bm)
    torch.save(proxy.state_dict(), bp)
    assert len(bm.getvalue()) < 8192 < len(bp.getvalue())
    # writes through the pair bucket are seen by the halves
    a.f32.fill_(1.5)
    assert float(main[0].weight.detach().view(-1)[0]) == 1.5
