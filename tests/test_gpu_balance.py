"""GPU: balanced tile tables (r03).  A plan keeps, per slot count of the
reduce kernels a call may run, a table whose vector tiles are re-cut to fill
whole rounds of resident workgroups (fedagg.hip balance_vec).  Each call
here runs once through the plan's choice and once through the plain table
(FA_PLAN_TUNE_NO_BALANCE): the results must be the same bits, and the
launch shape must be the re-cut one where the plain cut leaves its last
round part-filled.  The layouts' reference digests go through the balanced
tables in test_gpu_sweep / test_gpu_parity as well."""
import ctypes

import pytest
import torch

from conftest import load_manifest
from feddct_amd.layout import BucketLayout

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def lib():
    from feddct_amd import _lib
    torch.cuda.set_device(DEV)
    return _lib


def _layout(name):
    from feddct_amd.workload import joint_manifest
    if name.startswith("one_tensor_"):
        t = int(name.split("_")[-1])
        man = {"name": name, "keys": [{"key": "w", "shape": [t * 2048], "dtype": "float32"}]}
        return man, BucketLayout.from_manifest(man)
    if name.endswith("_joint"):
        stem = name[:-len("_joint")]
        mans = [load_manifest(stem + "_main"), load_manifest(stem + "_proxy")]
        return list(zip(mans, ("0.", "1."))), BucketLayout.from_manifest(joint_manifest(mans))
    man = load_manifest(name)
    return man, BucketLayout.from_manifest(man)


def _run(lib, plan, cl, n, weights):
    out32 = torch.full_like(cl[0][0], float("nan"))
    out64 = torch.full_like(cl[0][1], -7)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    w = None if weights is None else (ctypes.c_float * n)(*map(float, weights))  # host array
    lib.check(lib.lib.fa_reduce(plan.handle, lib.ptr_array([c[0].data_ptr() for c in cl]),
                                lib.ptr_array([c[1].data_ptr() for c in cl]), n, w,
                                out32.data_ptr(), out64.data_ptr(), 0, s), "fa_reduce")
    torch.cuda.synchronize()
    return out32, out64


CASES = [("one_tensor_1024", 20, False), ("one_tensor_1280", 16, False),
         ("one_tensor_1280", 5, False), ("one_tensor_300", 300, False),
         ("wrn16_8_c100", 20, False), ("wrn16_8_c100", 20, True), ("wrn16_8_c10", 20, False),
         ("wrnsl16_8_sf4_c10_joint", 5, False), ("resnet110sl_sf4_c100_joint", 25, False),
         ("wrnsl16_8_sf32_c100_joint", 3, False), ("wrnsl16_8_sf2_c100_joint", 48, True)]


@pytest.mark.parametrize("name,n,weighted", CASES)
def test_balanced_table_same_bits(lib, name, n, weighted):
    from feddct_amd.workload import make_clients
    man, lay = _layout(name)
    cl = make_clients(lay, man, range(n), DEV)
    weights = None
    if weighted:
        g = torch.Generator().manual_seed(n)
        w = torch.rand(n, generator=g) + 0.5
        weights = (w / w.sum()).tolist()
    G = lib.FA_PLAN_GAPS_ARE_PADDING
    pb = lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel, flags=G)
    pp = lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel,
                  flags=G | lib.FA_PLAN_TUNE_NO_BALANCE)
    a32, a64 = _run(lib, pb, cl, n, weights)
    b32, b64 = _run(lib, pp, cl, n, weights)
    assert torch.equal(a32.view(torch.int32), b32.view(torch.int32))
    assert torch.equal(a64, b64)
    assert not torch.isnan(a32[lay.segs32[0][0]:lay.segs32[0][0] + lay.segs32[0][1]]).any()
    nt_b, slots = pb.launch_shape(n, weighted)
    nt_p, slots_p = pp.launch_shape(n, weighted)
    assert slots > 0 and slots == slots_p and slots % 256 == 0
    k = -(-nt_p // slots)
    if nt_p >= 0.97 * k * slots:
        assert nt_b == nt_p          # the plain cut already fills its last round
    else:
        assert nt_p < nt_b <= k * slots


def test_occupancy_of_the_default_kernels(lib):
    """The slot counts the tables are cut for: 16-client batches 3 workgroups
    per CU (VGPR-bound), 8-client batches more (the 16 KB scalar stage no
    longer caps them at 4)."""
    man, lay = _layout("one_tensor_1024")
    p = lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel)
    cus = torch.cuda.get_device_properties(DEV).multi_processor_count
    _, s16 = p.launch_shape(20)
    _, s8 = p.launch_shape(5)
    print(f"slots: 16-client {s16} ({s16 // cus}/CU), 8-client {s8} ({s8 // cus}/CU)")
    assert s16 == 3 * cus
    assert s8 >= 4 * cus
