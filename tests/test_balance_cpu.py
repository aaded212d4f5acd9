"""Balanced tile tables (fa_plan_balance_host, r03) on the host: the re-cut
vector tiles cover exactly the plain tiles' elements (so any reduction over
them is the same per-column order), stay within the kernel's tile width, sit
on 64-element lines, and with the packed scalar tiles fill the one round of
the slot count they part-fill — or the plain cut is kept when that round is
>= 97 % full or the launch needs more than one round (measured: re-cutting a
multi-round launch is slower, fedagg.hip balance_vec), except that a
multi-round launch spilling 0 < r <= 0.44 slots tiles past its last full
round (the measured range, r04) has its last slots - r tiles split in halves
(split_tail, r03 session 4).
No GPU."""
import numpy as np
import pytest

from conftest import load_manifest
from feddct_amd import _lib
from feddct_amd.layout import BucketLayout

VEC = 0


def _vec_tiles(runs, width=2048):
    out = []
    for s, e in runs:
        for c in range(s, e, width):
            out.append((c, min(width, e - c), VEC))
    return np.array(out, np.int64).reshape(-1, 3)


def _elements(tiles):
    return np.concatenate([np.arange(s, s + c) for s, c, _ in tiles])


def _check(plain, cut, width, nscalar, slots):
    assert cut is not None
    assert (cut[:, 2] == VEC).all()
    assert (cut[:, 1] > 0).all() and (cut[:, 1] % 4 == 0).all() and (cut[:, 1] <= width).all()
    a, b = np.sort(_elements(plain)), np.sort(_elements(cut))
    assert np.array_equal(a, b), "re-cut tiles must cover exactly the plain tiles' elements"
    k = -(-(len(plain) + nscalar) // slots)
    assert len(plain) < len(cut) <= k * slots - nscalar
    # every boundary inside a run is on a 64-element line
    ends = set((plain[:, 0] + plain[:, 1]).tolist())
    for s, c, _ in cut:
        if int(s + c) not in ends:
            assert (s + c) % 64 == 0


@pytest.mark.parametrize("t,slots", [(384, 768), (700, 768), (1000, 1280), (200, 1024),
                                     (1100, 1280)])
def test_one_run_fills_whole_rounds(t, slots):
    plain = _vec_tiles([(0, t * 2048)])
    cut = _lib.balance_host(plain, 2048, 0, slots)
    _check(plain, cut, 2048, 0, slots)
    k = -(-t // slots)
    assert len(cut) == k * slots     # one long run: every slot of every round
    sizes = cut[:, 1]
    assert sizes.max() - sizes.min() <= 64


@pytest.mark.parametrize("t,ns,slots", [(768, 0, 768), (5358, 2, 768), (3070, 0, 1024),
                                        (750, 5, 768), (1280, 0, 768),
                                        (5120 + 700, 0, 1280), (5376 + 385, 0, 768),
                                        (5376, 0, 768), (5376 + 384, 0, 768),
                                        (5376 + 338, 0, 768)])
def test_full_or_multi_round_keeps_plain_cut(t, ns, slots):
    assert _lib.balance_host(_vec_tiles([(0, t * 2048)]), 2048, ns, slots) is None


@pytest.mark.parametrize("t,ns,slots", [(5377, 0, 768), (5380, 0, 768), (5376 + 337, 0, 768),
                                        (5370, 10, 768), (2 * 1280 + 7, 3, 1280), (2560, 0, 768), (1024, 0, 768),
                                        (4096, 0, 1280)])
def test_multi_round_tail_split(t, ns, slots):
    """A few tiles past the last full round: the last slots - r tiles are
    split in halves, every earlier tile untouched, exactly k rounds."""
    plain = _vec_tiles([(0, t * 2048)])
    cut = _lib.balance_host(plain, 2048, ns, slots)
    _check(plain, cut, 2048, ns, slots)
    k = -(-(t + ns) // slots)
    r = t + ns - (k - 1) * slots
    assert len(cut) == k * slots - ns
    keep = t - (slots - r)
    assert np.array_equal(cut[:keep], plain[:keep])
    assert (cut[keep:, 1] == 1024).all()


def test_tail_split_leaves_tiles_too_small_to_halve():
    """the tail split halves only tiles of >= kMinTile (256)
    elements; ragged run ends below that stay whole (so the table is a few
    tiles short of exactly k rounds), every other tile of the last
    slots - r is halved, and the elements are still covered exactly once."""
    slots, t = 768, 4610
    small = [(t * 2048 + 1024 * i, t * 2048 + 1024 * i + 128) for i in range(3)]
    plain = np.concatenate([_vec_tiles([(0, t * 2048)]), _vec_tiles(small)])
    k = -(-len(plain) // slots)         # 4,613 tiles: 7 rounds, r = 5
    r = len(plain) - (k - 1) * slots
    cut = _lib.balance_host(plain, 2048, 0, slots)
    assert cut is not None
    a, b = np.sort(_elements(plain)), np.sort(_elements(cut))
    assert np.array_equal(a, b)
    m = slots - r                       # tiles the split wanted to halve
    keep = len(plain) - m
    assert np.array_equal(cut[:keep], plain[:keep])
    assert len(cut) == len(plain) + m - 3 == k * slots - 3
    assert np.array_equal(cut[-3:], plain[-3:])        # the 128-element tiles, whole
    assert (cut[keep:-3, 1] == 1024).all()


def test_runs_with_gaps_and_ragged_ends():
    runs = [(0, 96_000), (96_064, 100_032), (200_000, 200_032), (204_800, 3_000_000),
            (3_000_064, 3_001_024)]
    plain = _vec_tiles(runs)
    cut = _lib.balance_host(plain, 2048, 155, 2048)
    _check(plain, cut, 2048, 155, 2048)
    for s, c, _ in cut:   # no tile crosses a gap
        assert any(rs <= s and s + c <= re for rs, re in runs)


def test_small_layout_floor():
    # 100 tiles on 768 slots: split down to 256-element tiles, not below
    plain = _vec_tiles([(0, 100 * 2048)])
    cut = _lib.balance_host(plain, 2048, 0, 768)
    _check(plain, cut, 2048, 0, 768)
    assert cut[:, 1].min() >= 192     # 64-line rounding of >= 256-element cuts


@pytest.mark.parametrize("width", [1024, 4096])
def test_other_tile_widths(width):
    plain = _vec_tiles([(0, 1000 * width)], width)
    cut = _lib.balance_host(plain, width, 3, 1280)
    _check(plain, cut, width, 3, 1280)


@pytest.mark.parametrize("name,slots", [("wrn16_8_c100", 768), ("wrn16_8_c10", 1280),
                                        ("resnet110sl_sf4_c100_proxy", 768)])
def test_reference_layouts(name, slots):
    lay = BucketLayout.from_manifest(load_manifest(name))
    info, tiles = _lib.build_tiles_host(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel)
    vec = tiles[tiles[:, 2] == VEC]
    ns = -(-int((tiles[tiles[:, 2] != VEC][:, 1]).sum()) // 64)   # packed 64 columns a tile
    cut = _lib.balance_host(vec, 2048, ns, slots)
    if cut is None:
        k = -(-(len(vec) + ns) // slots)
        r = len(vec) + ns - (k - 1) * slots
        assert (k > 1 and 100 * r > 44 * slots) or (k == 1 and len(vec) + ns >= 0.97 * k * slots)
    else:
        _check(vec, cut, 2048, ns, slots)


def test_rejects_non_vector_tiles():
    bad = np.array([[0, 16, 2]], np.int64)
    with pytest.raises(_lib.FedaggError):
        _lib.balance_host(bad, 2048, 0, 768)
    with pytest.raises(_lib.FedaggError):
        _lib.balance_host(np.array([[0, 4096, VEC]], np.int64), 2048, 0, 768)
