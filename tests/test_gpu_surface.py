"""GPU: the reference's call surface beyond same-dtype, same-device slots
(VERDICT r1 "what's missing" 3).  ``train_fedavg.py:145-147`` takes clients
whose key dtype differs from the global's (``.float()`` before the stack)
and a global model on another device than its clients (``load_state_dict``
copies across); the broadcast (``:148-149``) then writes the global's values
back in each client's own dtype.  Every case is compared bit for bit with
the reference loop restated on CPU torch (oracle/torch_mirror.py)."""
import copy

import pytest
import torch

from helpers import StateModule
from oracle.torch_mirror import reference_loop

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)

BASE = [("w", [100], "float32"), ("h", [70], "float16"), ("c", [3, 33], "float32"),
        ("n", [], "int64"), ("s", [], "float32")]


def _man(overrides=None):
    o = overrides or {}
    return {"keys": [{"key": k, "shape": sh, "dtype": o.get(k, dt)} for k, sh, dt in BASE]}


def _filled(man, seed):
    m = StateModule(man)
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for k, v in m.state_dict().items():
            if v.dtype.is_floating_point:
                v.copy_(torch.randn(v.shape, generator=g) * 3)
            else:
                v.copy_(torch.randint(0, 1000, v.shape, generator=g))
    return m


def _check(ours, ref):
    for k, v in ref.state_dict().items():
        o = ours.state_dict()[k]
        assert o.dtype == v.dtype, k
        assert torch.equal(o.detach().cpu(), v.detach()), k


@pytest.mark.parametrize("n", [3, 9, 20])
def test_client_dtypes_differing_from_the_global(n):
    from feddct_amd.fedavg import server_aggregate
    variants = [{}, {"w": "float16", "h": "float32", "n": "int32"},
                {"w": "float64", "h": "bfloat16", "c": "float16"},
                {"s": "float64", "n": "int16", "h": "float64"}]
    g_ref = _filled(_man(), 1000)
    c_ref = [_filled(_man(variants[i % len(variants)]), i) for i in range(n)]
    g, clients = copy.deepcopy(g_ref).to(DEV), [copy.deepcopy(c).to(DEV) for c in c_ref]
    reference_loop(g_ref, c_ref)
    server_aggregate(g, clients)
    torch.cuda.synchronize()
    _check(g, g_ref)
    for c, r in zip(clients, c_ref):
        _check(c, r)
    # second round on the same (already bound) modules
    # (local training stand-in: new values made on CPU, written in place into
    # both copies, so the inputs are identical bit for bit)
    with torch.no_grad():
        for i, (c, r) in enumerate(zip(clients, c_ref)):
            for (k, v), (_, w) in zip(c.state_dict().items(), r.state_dict().items()):
                if w.dtype.is_floating_point:
                    w.mul_(1.0 + i / 7)
                    v.copy_(w)
    reference_loop(g_ref, c_ref)
    server_aggregate(g, clients)
    torch.cuda.synchronize()
    _check(g, g_ref)
    _check(clients[-1], c_ref[-1])


def test_float_value_in_an_int64_key_is_refused():
    from feddct_amd.fedavg import server_aggregate
    g = _filled(_man(), 0).to(DEV)
    clients = [_filled(_man(), 1).to(DEV), _filled(_man({"n": "float32"}), 2).to(DEV)]
    with pytest.raises(TypeError, match="cannot be staged"):
        server_aggregate(g, clients)


@pytest.mark.parametrize("where", ["global_cpu", "clients_cpu"])
def test_global_on_another_device_than_the_clients(where):
    from feddct_amd.fedavg import server_aggregate
    n = 6
    g_ref = _filled(_man(), 50)
    c_ref = [_filled(_man(), 60 + i) for i in range(n)]
    g = copy.deepcopy(g_ref)
    clients = [copy.deepcopy(c) for c in c_ref]
    if where == "global_cpu":
        clients = [c.to(DEV) for c in clients]
    else:
        g = g.to(DEV)
    reference_loop(g_ref, c_ref)
    server_aggregate(g, clients)
    torch.cuda.synchronize()
    assert next(g.parameters()).device.type == ("cpu" if where == "global_cpu" else "cuda")
    _check(g, g_ref)
    for c, r in zip(clients, c_ref):
        _check(c, r)


def test_clients_on_different_devices_raise_like_torch_stack():
    from feddct_amd.fedavg import server_aggregate
    g = _filled(_man(), 0).to(DEV)
    clients = [_filled(_man(), 1).to(DEV), _filled(_man(), 2)]
    with pytest.raises(RuntimeError, match="same device"):
        server_aggregate(g, clients)


def test_feddct_checkpoint_of_one_half_holds_only_its_bytes(tmp_path):
    """after the joint FedDCT round (both halves in one bucket),
    torch.save of one model's state_dict (train_feddct.py:455,463) writes that
    model's bytes only and loads back into a plain module."""
    import os
    from feddct_amd.feddct import server_aggregate
    from feddct_amd.layout import BucketLayout
    mm = {"keys": [{"key": "a", "shape": [16, 3], "dtype": "float32"},
                   {"key": "nb", "shape": [], "dtype": "int64"}]}
    pm = {"keys": [{"key": "b", "shape": [200, 300], "dtype": "float32"},
                   {"key": "nb", "shape": [], "dtype": "int64"}]}
    n = 5
    ms = [_filled(mm, i).to(DEV) for i in range(n)]
    ps = [_filled(pm, 10 + i).to(DEV) for i in range(n)]
    gm, gp = _filled(mm, 99).to(DEV), _filled(pm, 98).to(DEV)
    server_aggregate(gm, gp, ms, ps)
    torch.cuda.synchronize()
    assert gm._fa_pairs[id(gp)]._fa_arena.f32.numel() > 60000   # one joint bucket
    torch.save({"state_dict": gm.state_dict()}, tmp_path / "main_client_best.pth.tar")
    torch.save({"state_dict": gp.state_dict()}, tmp_path / "proxy_clients_best.pth.tar")
    sm = os.path.getsize(tmp_path / "main_client_best.pth.tar")
    sp = os.path.getsize(tmp_path / "proxy_clients_best.pth.tar")
    own_main = BucketLayout.from_manifest(mm)
    assert sm < 4 * own_main.f32_numel + 8 + 4096, sm
    assert sp > 200 * 300 * 4
    back = StateModule(mm)
    back.load_state_dict(torch.load(tmp_path / "main_client_best.pth.tar",
                                    weights_only=True)["state_dict"])
    for k, v in gm.state_dict().items():
        assert torch.equal(back.state_dict()[k], v.cpu())


def test_bound_clients_share_a_slab_and_save_only_their_bytes(tmp_path):
    """slab.py: after a FedAvg round the clients' fp32 buckets sit side by side
    in one device allocation (the ~8 % faster placement), each still a
    storage of its own: torch.save of one client writes its bytes only, and
    the round is the reference's."""
    import os
    from feddct_amd import slab
    from feddct_amd.fedavg import server_aggregate
    from feddct_amd.layout import BucketLayout
    slab.release()
    man = _man()
    n = 6
    g = _filled(man, 0).to(DEV)
    clients = [_filled(man, 1 + i).to(DEV) for i in range(n)]
    ref_g = copy.deepcopy(g).cpu()
    ref_c = [copy.deepcopy(c).cpu() for c in clients]
    reference_loop(ref_g, ref_c)
    server_aggregate(g, clients)
    torch.cuda.synchronize()
    _check(g, ref_g)
    ptrs = sorted(c._fa_arena.f32.data_ptr() for c in clients)
    step = -(-clients[0]._fa_arena.f32.untyped_storage().nbytes() // slab.ALIGN) * slab.ALIGN
    # consecutive carves of one slab (the global's bucket may sit among them)
    assert all((b - a) % step == 0 and b > a for a, b in zip(ptrs, ptrs[1:]))
    assert ptrs[-1] - ptrs[0] <= n * step
    torch.save({"state_dict": clients[3].state_dict()}, tmp_path / "c3.pth")
    own = BucketLayout.from_manifest(man)
    assert os.path.getsize(tmp_path / "c3.pth") < 4 * own.f32_numel + 8 * own.i64_numel + 8192
    back = StateModule(man)
    back.load_state_dict(torch.load(tmp_path / "c3.pth", weights_only=True)["state_dict"])
    for k, v in clients[3].state_dict().items():
        assert torch.equal(back.state_dict()[k], v.cpu())
