"""Bucket layouts of the reference's models (manifests committed from the
reference's own model code by tests/golden/make_golden.py)."""
import pytest
import torch

from conftest import load_manifest
from feddct_amd.layout import ALIGN_F32, KIND_I64, BucketLayout

# SURVEY.md §8 notation (measured from the reference models)
EXPECT = {
    "wrn16_8_c10": (98, 43_888_744),
    "wrn16_8_c100": (98, 44_073_424),
    "wrnsl16_8_sf4_c10_main": (24, 7_968),
    "wrnsl16_8_sf4_c100_main": (24, 7_968),
    "wrnsl16_8_sf4_c10_proxy": (368, 44_061_312),
    "wrnsl16_8_sf4_c100_proxy": (368, 44_431_392),
}


@pytest.mark.parametrize("name", sorted(EXPECT))
def test_manifest_sizes_match_survey(name):
    L = BucketLayout.from_manifest(load_manifest(name))
    k, b = EXPECT[name]
    assert len(L.slots) == k
    assert L.state_bytes() == b


def test_algorithmic_bytes_cfg2():
    L = BucketLayout.from_manifest(load_manifest("wrn16_8_c10"))
    assert L.algorithmic_bytes(20) == 921_663_624


@pytest.mark.parametrize("name", sorted(EXPECT))
def test_offsets_aligned_and_disjoint(name):
    L = BucketLayout.from_manifest(load_manifest(name))
    end = 0
    for o, m in L.segs32:
        assert o % ALIGN_F32 == 0 and o >= end
        end = o + m
    assert L.f32_numel % ALIGN_F32 == 0 and L.f32_numel >= end
    assert all(s.kind == KIND_I64 for s in L.slots if s.dtype == torch.int64)
    assert L.keys == [e["key"] for e in load_manifest(name)["keys"]]


def test_from_state_dict_matches_manifest_and_handles_ties():
    m = torch.nn.Sequential(torch.nn.Linear(4, 3), torch.nn.BatchNorm1d(3),
                            torch.nn.Linear(3, 4))
    L = BucketLayout.from_state_dict(m.state_dict())
    assert L.keys == list(m.state_dict().keys())
    m[2].weight = torch.nn.Parameter(m[0].weight.detach().t().contiguous())
    tied = torch.nn.Module()
    tied.a = torch.nn.Linear(5, 5)
    tied.b = torch.nn.Linear(5, 5)
    tied.b.weight = tied.a.weight
    L2 = BucketLayout.from_state_dict(tied.state_dict())
    assert L2.by_key["b.weight"].alias_of == "a.weight"
    assert L2.by_key["b.weight"].offset == L2.by_key["a.weight"].offset
    assert len(L2.segs32) == 3


def test_packed_dtypes_go_to_f32_bucket():
    L = BucketLayout([("h", (7,), torch.float16), ("i", (3,), torch.int32),
                      ("n", (), torch.int64), ("f", (9,), torch.float32)])
    assert [s.kind for s in L.slots] == ["packf", "packf", "i64", "f32"]
    assert len(L.packed) == 2
    with pytest.raises(TypeError):
        BucketLayout([("c", (2,), torch.complex64)])
