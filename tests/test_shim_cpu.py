"""CPU: the _fa_shim gradient-binding helpers behind the one-node proximal
term (feddct_amd/prox.py, r03): .grad made views of a flat bucket, the state
check, and autograd's in-place accumulation landing in the bucket."""
import pytest
import torch

_fa_shim = pytest.importorskip("feddct_amd._fa_shim")


def _params():
    ps = tuple(torch.nn.Parameter(torch.randn(3, 4)) for _ in range(3))
    buf = torch.zeros(40)
    views = tuple(buf[i * 12:(i + 1) * 12].view(3, 4) for i in range(3))
    return ps, buf, views


def test_grad_state_and_binding():
    ps, buf, views = _params()
    assert _fa_shim.grad_state(ps, views) == 1          # all None
    _fa_shim.bind_grads(ps, views)
    assert _fa_shim.grad_state(ps, views) == 0          # all bound
    assert all(p.grad.data_ptr() == v.data_ptr() for p, v in zip(ps, views))
    ps[0].grad = None
    assert _fa_shim.grad_state(ps, views) == 2          # mixed
    ps[0].grad = torch.zeros(3, 4)
    assert _fa_shim.grad_state(ps, views) == 2          # a grad that is not the view


def test_autograd_accumulates_into_the_bucket():
    ps, buf, views = _params()
    _fa_shim.bind_grads(ps, views)
    (ps[1] * 2).sum().backward()
    (ps[1] * 3).sum().backward()
    assert torch.equal(buf[12:24], torch.full((12,), 5.0))
    assert _fa_shim.grad_state(ps, views) == 0


def test_bind_grads_refuses_mismatched_views():
    ps, buf, _ = _params()
    with pytest.raises(ValueError):
        _fa_shim.bind_grads(ps, tuple(buf[:12] for _ in ps))


def test_src_match_is_an_identity_check():
    """_fa_shim.src_match (the bound round's module check, r04): the objects
    passed — single objects, or lists / tuples taken item by item — are
    exactly the ones whose ids were recorded, in order and in number."""
    from array import array
    from feddct_amd import _fa_shim
    g, a, b, c = object(), object(), object(), object()
    ids = array("Q", [id(g), id(a), id(b)]).tobytes()
    assert _fa_shim.src_match(ids, g, [a, b])
    assert _fa_shim.src_match(ids, g, (a, b))
    assert _fa_shim.src_match(ids, g, a, b)
    assert not _fa_shim.src_match(ids, g, [b, a])        # order
    assert not _fa_shim.src_match(ids, g, [a, b, c])     # one more
    assert not _fa_shim.src_match(ids, g, [a])           # one fewer
    assert not _fa_shim.src_match(ids, c, [a, b])        # another object
    assert _fa_shim.src_match(array("Q").tobytes())      # nothing recorded, nothing passed
    with pytest.raises(TypeError):
        _fa_shim.src_match("not bytes", g)


def test_prox_state_takes_the_plan_only_on_success():
    """prox_state (the one-node proximal term's capsule):
    the norm plan's ownership passes to the capsule only once nothing can
    fail — a rejected call leaves the plan with the caller (no destroy, so
    the caller's own release is the only one), and a made capsule destroys it
    exactly once, when the capsule goes (no autograd node holds it here)."""
    import ctypes
    import gc
    import torch
    freed = []
    DESTROY = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)
    cb = DESTROY(lambda p: freed.append(p) or 0)
    addr = ctypes.cast(cb, ctypes.c_void_p).value
    plan = 0x1234500
    f = torch.zeros(64)
    norms, scratch = torch.zeros(2), torch.zeros(64)
    ps = (torch.nn.Parameter(torch.zeros(4)),)
    vs = (torch.zeros(4),)
    # the caller's fault after the tensors were checked: a params tuple of non-tensors
    with pytest.raises(TypeError):
        _fa_shim.prox_state(addr, addr, addr, plan, f, f, norms, scratch, (1, 2), vs, None, 1,
                            ps, vs, None, 2)
    gc.collect()
    assert freed == []
    cap = _fa_shim.prox_state(addr, addr, addr, plan, f, f, norms, scratch, ps, vs, None, 1,
                              ps, vs, None, 2)
    assert freed == []
    del cap
    gc.collect()
    assert freed == [plan]
