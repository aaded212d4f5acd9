"""GPU: the reference's other FedDCT sweep layouts (VERDICT r02 missing 1).

``train_feddct.py:34-56`` runs with more layouts than split_factor 4: the
wide_resnetsl16_8 CIFAR-100 scripts at split_factor 2 / 8 / 16 / 32 with 48 /
12 / 6 / 3 cluster slots (script/feddct_wrn168_split{2,8,16,32}_cifar100_
96clients_96choose_650rounds.sh:27) and resnet110sl at split_factor 4 with 25
and 20 slots (script/feddct_resnet110_split4_cifar100_{100,80}clients_...sh;
model/resnet_sl.py:520).  Their manifests and the reference's own
``server_aggregate`` digests come from tests/golden/make_golden.py --sweep;
here every one is reproduced by ONE launch over the joint main + proxy
bucket, and through the drop-in on nn.Modules."""
import ctypes

import pytest
import torch

from conftest import load_manifest
from feddct_amd import synth
from feddct_amd.layout import BucketLayout
from helpers import StateModule, buckets_to_state
from oracle import torch_order as O

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)

SWEEP = [("wrnsl16_8_sf2_c100", 48), ("wrnsl16_8_sf8_c100", 12), ("wrnsl16_8_sf16_c100", 6),
         ("wrnsl16_8_sf32_c100", 3), ("resnet110sl_sf4_c100", 25), ("resnet110sl_sf4_c100", 20)]


@pytest.fixture(scope="module")
def lib():
    from feddct_amd import _lib
    torch.cuda.set_device(DEV)
    return _lib


def _joint(name):
    from feddct_amd.workload import joint_manifest
    mm, pm = load_manifest(name + "_main"), load_manifest(name + "_proxy")
    return mm, pm, BucketLayout.from_manifest(joint_manifest([mm, pm]))


@pytest.mark.parametrize("name,n", SWEEP)
def test_sweep_joint_digest(lib, golden, name, n):
    """Main + proxy of every slot in one bucket, one reduce launch: both of
    the reference's digests, bit for bit."""
    from feddct_amd.workload import make_clients
    mm, pm, layout = _joint(name)
    cl = make_clients(layout, [(mm, "0."), (pm, "1.")], range(n), DEV)
    out32 = torch.full_like(cl[0][0], float("nan"))
    out64 = torch.full_like(cl[0][1], -7)
    plan = lib.Plan(layout.segs32, layout.f32_numel, layout.segs64, layout.i64_numel)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    lib.check(lib.lib.fa_reduce(plan.handle, lib.ptr_array([c[0].data_ptr() for c in cl]),
                                lib.ptr_array([c[1].data_ptr() for c in cl]), n, None,
                                out32.data_ptr(), out64.data_ptr(), 0, s), "fa_reduce")
    torch.cuda.synchronize()
    state = buckets_to_state(layout, out32, out64)
    for pf, half in (("0.", "main"), ("1.", "proxy")):
        part = [(k[2:], v) for k, v in state if k.startswith(pf)]
        assert O.state_digest(part) == golden["digests"][f"feddct/{name}_{half}/n{n}"], half


def _fill_module(lib, module, manifest, client):
    """Client ``client``'s synthetic state written straight into a device
    module's tensors by the HIP restatement of the PRNG."""
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    sd = module.state_dict()
    for j, e in enumerate(manifest["keys"]):
        t = sd[e["key"]]
        if t.dtype == torch.int64:
            lib.check(lib.lib.fa_synth_fill_i64(t.data_ptr(), t.numel(), j, client, 0, s))
        else:
            mu, sigma = synth.key_params(e["key"], tuple(e["shape"]), e["dtype"])
            lib.check(lib.lib.fa_synth_fill_f32(t.data_ptr(), t.numel(), j, client, mu, sigma,
                                                0, s))


@pytest.mark.parametrize("name,n", [("wrnsl16_8_sf32_c100", 3), ("resnet110sl_sf4_c100", 25),
                                    ("wrnsl16_8_sf2_c100", 48)])
def test_sweep_dropin_feddct(lib, golden, name, n):
    """feddct.server_aggregate(g_main, g_proxy, mains, proxies) — the
    reference's call (train_feddct.py:436) — on device modules of the
    layout: global halves equal the reference digests, every client got the
    global state back."""
    from feddct_amd.feddct import server_aggregate
    mm, pm = load_manifest(name + "_main"), load_manifest(name + "_proxy")
    gm, gp = StateModule(mm).to(DEV), StateModule(pm).to(DEV)
    ms = [StateModule(mm).to(DEV) for _ in range(n)]
    ps = [StateModule(pm).to(DEV) for _ in range(n)]
    for i in range(n):
        _fill_module(lib, ms[i], mm, i)
        _fill_module(lib, ps[i], pm, i)
    server_aggregate(gm, gp, ms, ps)
    torch.cuda.synchronize()
    for g, half in ((gm, "main"), (gp, "proxy")):
        st = [(k, v.detach().cpu().numpy()) for k, v in g.state_dict().items()]
        assert O.state_digest(st) == golden["digests"][f"feddct/{name}_{half}/n{n}"], half
    for c, g in ((ms[-1], gm), (ps[0], gp)):
        for k, v in g.state_dict().items():
            assert torch.equal(c.state_dict()[k], v), k
