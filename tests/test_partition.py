import pytest

from conftest import load_manifest
from feddct_amd.layout import BucketLayout
from feddct_amd.partition import i64_tiles, layout_tiles, split_tiles


@pytest.mark.parametrize("lay", ["wrn16_8_c10", "wrnsl16_8_sf4_c100_proxy", "wrnsl16_8_sf4_c10_main"])
@pytest.mark.parametrize("parts", [1, 2, 3, 8, 100])
def test_split_covers_every_tile_once(lay, parts):
    L = BucketLayout.from_manifest(load_manifest(lay))
    info, tiles = layout_tiles(L)
    sp = split_tiles(tiles, parts, L.f32_numel)
    assert len(sp) == parts
    assert sp[0][0] == 0 and sp[-1][1] == L.f32_numel
    n = 0
    for (lo, hi, sel), nxt in zip(sp, sp[1:] + [(L.f32_numel, None, None)]):
        assert hi == nxt[0] and lo <= hi and lo % 4 == 0
        if len(sel):
            assert (sel[:, 0] >= lo).all() and ((sel[:, 0] + sel[:, 1]) <= hi).all()
        n += len(sel)
    assert n + len(i64_tiles(tiles)) == len(tiles)
    if parts <= 8 and lay != "wrnsl16_8_sf4_c10_main":
        sizes = [int(sel[:, 1].sum()) if len(sel) else 0 for _, _, sel in sp]
        assert max(sizes) < 2.5 * (sum(sizes) / parts) + 4096


@pytest.mark.parametrize("lay", ["wrn16_8_c10", "wrnsl16_8_sf4_c100_proxy"])
def test_split_by_fractions_tapers(lay):
    """pipeline.HostPipeline's tapered cut: every tile once, each range near
    its fraction of the elements (cuts fall on tile starts)."""
    fr = (0.5, 0.25, 0.125, 0.0625, 0.0625)
    L = BucketLayout.from_manifest(load_manifest(lay))
    info, tiles = layout_tiles(L)
    sp = split_tiles(tiles, len(fr), L.f32_numel, fr)
    assert sp[0][0] == 0 and sp[-1][1] == L.f32_numel
    assert sum(len(sel) for _, _, sel in sp) + len(i64_tiles(tiles)) == len(tiles)
    sizes = [int(sel[:, 1].sum()) for _, _, sel in sp]
    total = sum(sizes)
    for got, want in zip(sizes, fr):
        assert abs(got / total - want) < 0.03, (sizes, fr)
    with pytest.raises(ValueError):
        split_tiles(tiles, 3, L.f32_numel, fr)
