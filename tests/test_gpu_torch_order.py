"""GPU: torch-ROCm's own GPU order for the reference's averaging (VERDICT r1
missing 1).  The reference's runs put the models on the GPU
(train_fedavg.py:244-250), so ``torch.stack(...).mean(0)`` (:145-146) ran
torch-ROCm's reduction there, not the CPU cascade.  The opt-in plan order
FA_ORDER_TORCH_GPU reproduces it; these tests compare it bit for bit with
torch's own cuda mean on the box — first the numpy restatement
(oracle/torch_gpu_order.py) over many shapes, then the kernel at the
BASELINE config 2, 3 and 5 sizes."""
import ctypes

import numpy as np
import pytest
import torch

from conftest import load_manifest
from feddct_amd import synth
from feddct_amd.layout import BucketLayout
from helpers import bits_equal, buckets_to_state, states_to_buckets
from oracle import torch_gpu_order as G

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def lib():
    from feddct_amd import _lib
    torch.cuda.set_device(DEV)
    return _lib


def _torch_gpu_mean(rows):
    """The reference's expression on device tensors (train_fedavg.py:145-146)."""
    return torch.stack([r.float() for r in rows], 0).mean(0)


SHAPES = [(n, m) for n in (2, 3, 5, 8, 9, 16, 17, 20, 24, 31, 32, 33, 64, 100, 127, 200)
          for m in (1, 2, 3, 5, 10, 16, 17, 100, 432, 1000, 4096, 2 ** 16 + 4)]


@pytest.mark.parametrize("n,m", [s for s in SHAPES if G.supported(*s)])
def test_restatement_matches_torch_gpu(n, m):
    rng = np.random.default_rng(n * 7919 + m)
    x = (rng.standard_normal((n, m)) * 10.0 ** rng.integers(-3, 4, (n, m))).astype(np.float32)
    got = _torch_gpu_mean([torch.from_numpy(x[i]).to(DEV) for i in range(n)]).cpu().numpy()
    assert bits_equal(got, G.gpu_mean0(x)), (n, m, G.config(n, m))


def _gpu_order_reduce(lib, layout, buckets):
    n = len(buckets)
    plan = lib.Plan(layout.segs32, layout.f32_numel, layout.segs64, layout.i64_numel,
                    order=lib.FA_ORDER_TORCH_GPU, n=n)
    out32 = torch.full_like(buckets[0][0], np.nan)
    out64 = torch.full_like(buckets[0][1], -7)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    lib.check(lib.lib.fa_reduce(plan.handle, lib.ptr_array([b[0].data_ptr() for b in buckets]),
                                lib.ptr_array([b[1].data_ptr() for b in buckets]), n, None,
                                out32.data_ptr(), out64.data_ptr(), 0, s), "fa_reduce(gpu order)")
    torch.cuda.synchronize()
    return out32, out64


def _vs_torch(layout, buckets, out32, out64):
    bad = []
    for s in layout.slots:
        src = 1 if s.kind == "i64" else 0
        rows = [b[src][s.offset:s.offset + s.numel].view(s.shape) for b in buckets]
        ref = _torch_gpu_mean(rows)
        if s.kind == "i64":
            want = torch.zeros(s.shape, dtype=torch.int64, device=DEV)
            want.copy_(ref)          # load_state_dict's copy_: fp32 -> int64 truncation
            got = out64[s.offset:s.offset + s.numel].view(s.shape)
            ok = torch.equal(got, want)
        else:
            got = out32[s.offset:s.offset + s.numel].view(s.shape)
            ok = bits_equal(got.cpu().numpy(), ref.cpu().numpy())
        if not ok:
            bad.append(s.key)
    return bad


@pytest.mark.parametrize("case", ["cfg2", "cfg3", "cfg5", "small_adversarial"])
def test_kernel_matches_torch_gpu_mean(lib, case):
    from feddct_amd.workload import joint_manifest, make_clients
    if case == "cfg2":
        man = load_manifest("wrn16_8_c10")
        layout = BucketLayout.from_manifest(man)
        cl = make_clients(layout, man, range(20), DEV)
    elif case in ("cfg3", "cfg5"):
        tag, n = ("c10", 5) if case == "cfg3" else ("c100", 24)
        mm = load_manifest(f"wrnsl16_8_sf4_{tag}_main")
        pm = load_manifest(f"wrnsl16_8_sf4_{tag}_proxy")
        layout = BucketLayout.from_manifest(joint_manifest([mm, pm]))
        cl = make_clients(layout, [(mm, "0."), (pm, "1.")], range(n), DEV)
    else:
        man = {"keys": [{"key": f"k{j}", "shape": [m] if m else [], "dtype": "float32"}
                        for j, m in enumerate([0, 1, 3, 10, 33, 100, 4097])]
               + [{"key": "nbt", "shape": [], "dtype": "int64"}]}
        layout = BucketLayout.from_manifest(man)
        states = [synth.gen_state(man, i, synth.MODE_ADVERSARIAL) for i in range(33)]
        cl = states_to_buckets(layout, states, DEV)
    out32, out64 = _gpu_order_reduce(lib, layout, cl)
    assert _vs_torch(layout, cl, out32, out64) == []


def test_gpu_order_broadcast_and_errors(lib):
    man = load_manifest("wrnsl16_8_sf4_c10_main")
    layout = BucketLayout.from_manifest(man)
    from feddct_amd.workload import make_clients
    cl = make_clients(layout, man, range(5), DEV)
    plan = lib.Plan(layout.segs32, layout.f32_numel, layout.segs64, layout.i64_numel,
                    order=lib.FA_ORDER_TORCH_GPU, n=5)
    o32, o64 = torch.zeros_like(cl[0][0]), torch.zeros_like(cl[0][1])
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    a32 = lib.ptr_array([b[0].data_ptr() for b in cl])
    a64 = lib.ptr_array([b[1].data_ptr() for b in cl])
    w = (ctypes.c_float * 5)(*[0.2] * 5)
    assert lib.lib.fa_reduce(plan.handle, a32, a64, 5, w, o32.data_ptr(), o64.data_ptr(), 0,
                             s) == lib.FA_E_INVAL
    assert lib.lib.fa_reduce(plan.handle, a32, a64, 4, None, o32.data_ptr(), o64.data_ptr(), 0,
                             s) == lib.FA_E_INVAL
    lib.check(lib.lib.fa_reduce(plan.handle, a32, a64, 5, None, o32.data_ptr(), o64.data_ptr(),
                                lib.FA_F_BCAST, s))
    torch.cuda.synchronize()
    for b in cl:   # the broadcast wrote every client's segments
        for sl in layout.slots:
            src, res = (b[1], o64) if sl.kind == "i64" else (b[0], o32)
            assert torch.equal(src[sl.offset:sl.offset + sl.numel],
                               res[sl.offset:sl.offset + sl.numel])
    with pytest.raises(lib.FedaggError, match="outside the restated"):
        lib.Plan(np.array([[0, 64]]), 64, order=lib.FA_ORDER_TORCH_GPU, n=4000)


@pytest.mark.parametrize("n", [2, 5, 20, 24])
def test_dropin_with_gpu_order_matches_reference_loop_on_gpu(n):
    """set_summation_order("torch_gpu"): the drop-in server_aggregate on GPU
    modules against the reference's own loop (train_fedavg.py:143-149,
    restated in oracle/torch_mirror.py) run on GPU modules — global and every
    client, bit for bit, int64 keys included."""
    import copy
    import feddct_amd
    from feddct_amd.fedavg import server_aggregate
    from helpers import StateModule
    from oracle.torch_mirror import reference_loop
    man = {"keys": [{"key": "conv.weight", "shape": [16, 3, 3, 3], "dtype": "float32"},
                    {"key": "bn.weight", "shape": [16], "dtype": "float32"},
                    {"key": "bn.num_batches_tracked", "shape": [], "dtype": "int64"},
                    {"key": "fc.weight", "shape": [10, 100], "dtype": "float32"},
                    {"key": "fc.bias", "shape": [10], "dtype": "float32"},
                    {"key": "odd", "shape": [3, 11], "dtype": "float32"},
                    {"key": "scale", "shape": [], "dtype": "float32"}]}
    states = [synth.gen_state(man, i, synth.MODE_ADVERSARIAL) for i in range(n)]
    mods = [StateModule(man).load_numpy(s).to(DEV) for s in states]
    ref_g, ref_c = StateModule(man).to(DEV), [copy.deepcopy(m) for m in mods]
    reference_loop(ref_g, ref_c)
    feddct_amd.set_summation_order("torch_gpu")
    try:
        g = StateModule(man).to(DEV)
        server_aggregate(g, mods)
        torch.cuda.synchronize()
    finally:
        feddct_amd.set_summation_order("torch_cpu")
    for k, v in ref_g.state_dict().items():
        assert torch.equal(g.state_dict()[k].view(torch.int32) if v.dtype == torch.float32
                           else g.state_dict()[k],
                           v.view(torch.int32) if v.dtype == torch.float32 else v), k
        assert torch.equal(mods[-1].state_dict()[k], ref_c[-1].state_dict()[k]), k
