"""C-ABI library: loads, exports every symbol include/fedagg.h declares, and
the host-side paths (argument checks, tile planning) behave without a GPU."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT, load_manifest
from feddct_amd import _lib
from feddct_amd.layout import BucketLayout


def header_functions():
    src = open(os.path.join(ROOT, "include", "fedagg.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fa_[a-z0-9_]+)\s*\(", src)))


def test_every_declared_symbol_is_exported():
    fns = header_functions()
    assert len(fns) >= 15
    so = ctypes.CDLL(_lib.LIB_PATH)
    for f in fns:
        assert hasattr(so, f), f"{f} declared in include/fedagg.h but not exported"
    assert set(fns) == set(_lib.EXPORTS), "python binding table out of sync with the header"


def test_version_and_error_paths():
    assert "gfx950" in _lib.version()
    L = _lib.lib
    assert L.fa_plan_create(None, 0, 0, None, 0, 0, 0, 0, None) == _lib.FA_E_INVAL
    assert b"NULL" in L.fa_last_error()
    segs, n = _lib.seg_array(np.array([[0, 10], [5, 10]], np.int64))
    h = ctypes.c_void_p()
    assert L.fa_plan_create(segs, n, 20, None, 0, 0, 0, 0, ctypes.byref(h)) == _lib.FA_E_INVAL
    assert b"overlap" in L.fa_last_error()
    segs, n = _lib.seg_array(np.array([[0, 30]], np.int64))
    assert L.fa_plan_create(segs, n, 20, None, 0, 0, 0, 0, ctypes.byref(h)) == _lib.FA_E_INVAL
    assert L.fa_plan_create(segs, n, 64, None, 0, 0, 3000, 0, ctypes.byref(h)) == _lib.FA_E_INVAL
    assert L.fa_reduce(None, None, None, 1, None, None, None, 0, None) == _lib.FA_E_INVAL
    assert L.fa_div_f32(None, 2.0, None, 0, None) == _lib.FA_OK
    assert L.fa_div_f32(None, 2.0, None, 5, None) == _lib.FA_E_INVAL
    assert L.fa_broadcast_f32(None, None, _lib.FA_MAX_CLIENTS + 1, 10, None) == _lib.FA_E_RANGE
    with pytest.raises(_lib.FedaggError, match="overlap"):
        _lib.build_tiles_host(np.array([[0, 10], [5, 10]]), 20)


def _expected_kind(M, col):
    """Which torch order an element uses (oracle column rule)."""
    if M == 1:
        return "inner"
    b = (M // 32) * 32 if M >= 8 else (M // 4) * 4
    return "cascade" if col < b else "ilp4"


KIND_NAME = {0: "cascade", 1: "cascade", 2: "ilp4", 3: "inner", 4: "cascade", 5: "ilp4", 6: "inner"}


@pytest.mark.parametrize("lay", ["wrn16_8_c10", "wrnsl16_8_sf4_c100_main",
                                 "wrnsl16_8_sf4_c100_proxy"])
@pytest.mark.parametrize("tile", [1024, 2048, 4096])
def test_tiles_partition_every_key_with_the_right_order(lay, tile):
    L = BucketLayout.from_manifest(load_manifest(lay))
    info, tiles = _lib.build_tiles_host(L.segs32, L.f32_numel, L.segs64, L.i64_numel, tile)
    assert info["ntiles"] == len(tiles)
    cover32 = np.full(L.f32_numel, "", dtype=object)
    cover64 = np.full(max(1, L.i64_numel), "", dtype=object)
    for start, count, kind in tiles:
        assert 1 <= count <= (tile if kind == 0 else 256)
        tgt = cover64 if kind >= 4 else cover32
        assert (tgt[start:start + count] == "").all(), "tiles overlap"
        tgt[start:start + count] = KIND_NAME[kind]
        if kind == 0:
            assert start % 4 == 0 and count % 4 == 0
    for o, M in L.segs32:
        for col in range(M):
            assert cover32[o + col] == _expected_kind(M, col), (lay, o, M, col)
    for o, M in L.segs64:
        for col in range(M):
            assert cover64[o + col] == _expected_kind(M, col)


def test_stateless_plans_never_cover_gaps():
    segs = np.array([[0, 100], [128, 64], [200, 33]], np.int64)
    info, tiles = _lib.build_tiles_host(segs, 256, flags=0)
    covered = np.zeros(256, bool)
    for s, c, k in tiles:
        covered[s:s + c] = True
    want = np.zeros(256, bool)
    for o, m in segs:
        want[o:o + m] = True
    assert np.array_equal(covered, want)


def test_unit_tensor_between_vector_runs_is_covered_once():
    """A 1-element fp32 key between two aligned keys (a scalar nn.Parameter,
    PReLU's weight): with padding-gaps planning the vector run must stop
    before it, or the element gets both the cascade and the inner order."""
    lay = BucketLayout([("w", (64,), "float32"), ("s", (), "float32"),
                        ("w2", (64,), "float32"), ("t", (37,), "float32"),
                        ("u", (1,), "float32"), ("w3", (4, 32), "float32")])
    info, tiles = _lib.build_tiles_host(lay.segs32, lay.f32_numel)
    cover = np.zeros(lay.f32_numel, np.int64)
    for s, c, k in tiles:
        cover[s:s + c] += 1
    assert cover.max() == 1
    for o, M in lay.segs32:
        assert (cover[o:o + M] == 1).all()
    s_off = lay.by_key["s"].offset
    kinds = [k for s, c, k in tiles if s <= s_off < s + c]
    assert kinds == [3]


def test_overlapping_tile_subsets_are_refused():
    L = _lib.lib
    arr = (_lib.FaTileDesc * 2)()
    arr[0].start, arr[0].count, arr[0].kind = 0, 64, 0
    arr[1].start, arr[1].count, arr[1].kind = 60, 1, 3
    h = ctypes.c_void_p()
    assert L.fa_plan_create_from_tiles(arr, 2, 128, 0, 0, 1, ctypes.byref(h)) == _lib.FA_E_INVAL
    assert b"overlap" in L.fa_last_error()


def test_norm_plan_host_errors():
    L = _lib.lib
    h = ctypes.c_void_p()
    assert L.fa_norm_plan_create(None, 0, 0, None) == _lib.FA_E_INVAL
    segs, n = _lib.seg_array(np.array([[0, 100]], np.int64))
    assert L.fa_norm_plan_create(segs, n, 50, ctypes.byref(h)) == _lib.FA_E_INVAL
    assert L.fa_prox_norms(None, None, None, None, None, None) == _lib.FA_E_INVAL


def test_comm_library_exports_every_declared_symbol():
    """libfedagg_comm.so (the RCCL exchange) exports include/fedagg_comm.h."""
    from feddct_amd import comm
    src = open(os.path.join(ROOT, "include", "fedagg_comm.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    fns = sorted(set(re.findall(r"\b(fa_[a-z0-9_]+)\s*\(", src)))
    so = comm.lib()
    for f in fns:
        assert hasattr(so, f), f"{f} declared in include/fedagg_comm.h but not exported"
    assert set(fns) == set(comm.COMM_EXPORTS)
    # host-side argument checks (no GPU, no communicator needed)
    h = ctypes.c_void_p()
    assert so.fa_comm_init_rank(0, 0, b"x" * 128, 128, ctypes.byref(h)) == _lib.FA_E_INVAL
    assert so.fa_comm_unique_id(None, 0) == _lib.FA_E_INVAL
    assert so.fa_reduce_sharded(None, 0, None, 0) == _lib.FA_E_INVAL
    assert so.fa_shard_plan_create(None, None, 0, 0, None, 0, 0, None, 0, 1,
                                   ctypes.byref(h)) == _lib.FA_E_INVAL
    assert b"NULL" in _lib.lib.fa_last_error()  # one error channel for both libraries


def test_header_constants_match_binding():
    """Every plain FA_* integer macro of include/fedagg.h that the Python
    binding also names has the same value there."""
    src = open(os.path.join(ROOT, "include", "fedagg.h")).read()
    macros = dict(re.findall(r"#define\s+(FA_[A-Z0-9_]+)\s+\(?(-?(?:0x[0-9a-fA-F]+|\d+))u?\)?",
                             src))
    checked = 0
    for name, val in macros.items():
        if hasattr(_lib, name) and isinstance(getattr(_lib, name), int):
            assert getattr(_lib, name) == int(val, 0), name
            checked += 1
    assert checked >= 10
    assert _lib.FA_PLAN_FLAGS_KNOWN == 0x1000000D


@pytest.mark.parametrize("bit", [2, 16, 32, 64, 0x10000, 0x80000, 0x400000, 0x800000, 0x1000000,
                                 0x20000000, 0x80000000, 3 << 26, 3 << 8, 5 << 12])
def test_removed_tuning_flags_are_refused(bit):
    """r05: the r01-r04 tuning flags are gone
    from the library, and a caller still passing one (e.g. 0x1000000, which
    named two different r03 / r04 flags) gets FA_E_INVAL, not a silently
    different kernel.  fa_plan_build_host is host-only: no GPU needed."""
    import ctypes
    import numpy as np
    segs, n = _lib.seg_array(np.array([[0, 4096]], np.int64))
    info = _lib.FaPlanInfo()
    rc = _lib.lib.fa_plan_build_host(segs, n, 4096, None, 0, 0, 0,
                                     _lib.FA_PLAN_GAPS_ARE_PADDING | bit, None, 0,
                                     ctypes.byref(info))
    assert rc == _lib.FA_E_INVAL, (hex(bit), rc)
    assert b"unknown flag bits" in _lib.lib.fa_last_error()
    rc = _lib.lib.fa_plan_build_host(segs, n, 4096, None, 0, 0, 0,
                                     _lib.FA_PLAN_FLAGS_KNOWN, None, 0, ctypes.byref(info))
    assert rc == 0
