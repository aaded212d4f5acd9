"""GPU: launch shapes by round count (r03).  A call of N >= 16 clients whose
plain tile table part-fills one round of the 16-client kernel's resident
workgroups runs a table re-cut to fill it; one that needs two rounds of the
16-client kernel but one of the 8-client kernel runs the 8-client kernel;
one that spills r <= 0.44 slots tiles past its last full round has its last
slots - r tiles split in halves (session 4, split_tail; at N < 16 too, on
the 8-client kernels' slots); everything else
runs the plain table (fedagg.hip balance_vec / round_batch).
Each call here runs once through the plan's choice and once through the
plain table with the default batch (FA_PLAN_TUNE_NO_BALANCE): the results
must be the same bits, and the launch shape must be the one the rule names.
The layouts' reference digests go through the same choice in test_gpu_sweep
/ test_gpu_parity as well."""
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
         ("one_tensor_384", 20, False), ("one_tensor_384", 20, True), ("one_tensor_600", 5, False),
         ("one_tensor_3000", 17, False), ("one_tensor_5380", 20, False),
         ("one_tensor_5380", 20, True), ("one_tensor_1700", 20, False),
         ("one_tensor_1700", 300, False), ("one_tensor_5380", 5, False),
         ("one_tensor_5380", 12, True), ("one_tensor_5760", 5, False),
         ("wrn16_8_c100", 20, False), ("wrn16_8_c100", 20, True), ("wrn16_8_c10", 20, False),
         ("wrnsl16_8_sf4_c10_joint", 5, False), ("resnet110sl_sf4_c100_joint", 25, False),
         ("wrnsl16_8_sf32_c100_joint", 3, False), ("wrnsl16_8_sf2_c100_joint", 48, True)]


B16 = 12


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
    nt_p, slots_p = pp.launch_shape(n, weighted)   # the default batch's slots
    assert slots > 0 and slots_p > 0 and slots % 256 == 0
    # the 16-client kernels from B16 clients (r06: 12; fedagg.hip pick_batch)
    s8 = pp.launch_shape(5, weighted)[1] if n >= B16 else slots_p
    k = -(-nt_p // slots_p)
    r = nt_p - (k - 1) * slots_p
    if k > 1 and 100 * r <= 44 * slots_p and (n < B16 or nt_p > s8):
        assert (nt_b, slots) == (k * slots_p, slots_p)   # tail split: exactly k rounds
    elif n < B16 or nt_p > s8 or (nt_p <= slots_p and nt_p >= 0.97 * slots_p):
        assert (nt_b, slots) == (nt_p, slots_p)    # plain table, default batch
    elif nt_p <= slots_p:
        assert nt_p < nt_b <= slots_p and slots == slots_p   # one round, re-cut to fill it
    else:
        assert (nt_b, slots) == (nt_p, s8)         # two rounds of 16 -> one of 8


def test_occupancy_of_the_default_kernels(lib):
    """The slot counts the tables are cut for: 16-client batches 3 workgroups
    per CU (VGPR-bound), 8-client batches more (the 16 KB scalar stage no
    longer caps them at 4)."""
    man, lay = _layout("one_tensor_5380")
    p = lib.Plan(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel)
    cus = torch.cuda.get_device_properties(DEV).multi_processor_count
    _, s16 = p.launch_shape(20)
    _, s8 = p.launch_shape(5)
    print(f"slots: 16-client {s16} ({s16 // cus}/CU), 8-client {s8} ({s8 // cus}/CU)")
    assert s16 == 3 * cus
    assert s8 >= 4 * cus
