"""Column partitions of a layout's tile table.

Every tile of a plan carries the summation order its columns need (cascade /
ILP-4 / inner), so ANY subset of tiles reduces bit-exactly on its own.  This
module cuts the table into contiguous column ranges — the stripes of the
exact multi-GPU mode (dist.StripedAggregator) and the chunks of the
host-ingress pipeline (pipeline.HostPipeline) — always at vector-tile starts,
so every range starts 16-B aligned and no tile straddles a cut.
"""
from __future__ import annotations

from functools import lru_cache
from typing import List, Tuple

import numpy as np

from . import _lib
from .layout import BucketLayout

K_I64_MIN = 4  # tile kinds >= 4 are int64 tiles


@lru_cache(maxsize=32)
def _tiles_cached(signature, segs32_b, f32_numel, segs64_b, i64_numel, tile_elems):
    segs32 = np.frombuffer(segs32_b, np.int64).reshape(-1, 2)
    segs64 = np.frombuffer(segs64_b, np.int64).reshape(-1, 2)
    return _lib.build_tiles_host(segs32, f32_numel, segs64, i64_numel, tile_elems)


def layout_tiles(layout: BucketLayout, tile_elems: int = 0):
    """(info, tiles[start, count, kind]) of the layout's full plan."""
    return _tiles_cached(layout.signature, layout.segs32.tobytes(), layout.f32_numel,
                         layout.segs64.tobytes(), layout.i64_numel, tile_elems)


def split_tiles(tiles: np.ndarray, parts: int, f32_numel: int
                ) -> List[Tuple[int, int, np.ndarray]]:
    """Cut the fp32 tiles into ``parts`` contiguous ranges of about equal
    element count.  Returns [(lo, hi, tiles_in_range)], covering
    [0, f32_numel) exactly (some ranges may be empty)."""
    t32 = tiles[tiles[:, 2] < K_I64_MIN]
    t32 = t32[np.argsort(t32[:, 0], kind="stable")]
    total = int(t32[:, 1].sum()) if len(t32) else 0
    cuts = [0]
    acc = 0
    k = 1
    for s, c, kind in t32:
        if k < parts and kind == 0 and acc >= total * k / parts and s > cuts[-1]:
            cuts.append(int(s))
            k += 1
        acc += int(c)
    while len(cuts) < parts:
        cuts.append(f32_numel)
    cuts.append(f32_numel)
    out = []
    for i in range(parts):
        lo, hi = cuts[i], cuts[i + 1]
        sel = t32[(t32[:, 0] >= lo) & (t32[:, 0] < hi)]
        out.append((lo, hi, sel))
    return out


def i64_tiles(tiles: np.ndarray) -> np.ndarray:
    return tiles[tiles[:, 2] >= K_I64_MIN]


def range_plans(layout: BucketLayout, parts: int, tile_elems: int = 0, flags=None):
    """[(lo, hi, Plan or None)] for each fp32 range, plus the int64 Plan."""
    if flags is None:
        flags = _lib.FA_PLAN_GAPS_ARE_PADDING
    info, tiles = layout_tiles(layout, tile_elems)
    te = info["tile_elems"]
    out = []
    for lo, hi, sel in split_tiles(tiles, parts, layout.f32_numel):
        p = (_lib.Plan(None, layout.f32_numel, None, layout.i64_numel, te, flags, tiles=sel)
             if len(sel) else None)
        out.append((lo, hi, p))
    t64 = i64_tiles(tiles)
    p64 = (_lib.Plan(None, layout.f32_numel, None, layout.i64_numel, te, flags, tiles=t64)
           if len(t64) else None)
    return out, p64
