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


def cut_index(t: np.ndarray, parts: int, fractions=None) -> List[int]:
    """Group boundaries (tile indices, len parts+1) of the sorted tiles ``t``
    into ``parts`` runs of about equal element count (or of the given
    ``fractions`` of it, which sum to 1), cut only before a vector tile on a
    256-B boundary — fedcomm.hip's cut_tiles, the same rule the native
    schedules use."""
    total = int(t[:, 1].sum()) if len(t) else 0
    if fractions is None:
        goal = [total * k // parts for k in range(parts)]
    else:
        if len(fractions) != parts:
            raise ValueError("one fraction per part")
        cum = np.concatenate([[0.0], np.cumsum(fractions)])
        goal = [int(total * cum[k]) for k in range(parts)]
    cut = [0]
    acc = 0
    for i, (s, c, kind) in enumerate(t):
        k = len(cut)
        if k < parts and i > 0 and acc >= goal[k] and kind == 0 and s % 64 == 0:
            cut.append(i)
        acc += int(c)
    while len(cut) < parts + 1:
        cut.append(len(t))
    return cut


def split_tiles(tiles: np.ndarray, parts: int, f32_numel: int, fractions=None
                ) -> List[Tuple[int, int, np.ndarray]]:
    """Cut the fp32 tiles into ``parts`` contiguous ranges of about equal
    element count (or ``fractions`` of it).  Returns [(lo, hi,
    tiles_in_range)], covering [0, f32_numel) exactly (some ranges may be
    empty)."""
    t32 = tiles[tiles[:, 2] < K_I64_MIN]
    t32 = t32[np.argsort(t32[:, 0], kind="stable")]
    ci = cut_index(t32, parts, fractions)
    cuts = [0] + [int(t32[ci[g], 0]) if ci[g] < len(t32) else f32_numel
                  for g in range(1, parts)]
    cuts.append(f32_numel)
    out = []
    for i in range(parts):
        lo, hi = cuts[i], cuts[i + 1]
        sel = t32[(t32[:, 0] >= lo) & (t32[:, 0] < hi)]
        out.append((lo, hi, sel))
    return out


def stripe_chunks(tiles: np.ndarray, parts: int, f32_numel: int, nchunks: int):
    """The striped round's cut (fedcomm.hip build_round, r06): ``parts``
    stripes (split_tiles), each cut into ``nchunks`` column chunks by the
    same rule.  Returns, per stripe, [(lo, hi, tiles)] of its chunks, in
    order, covering the stripe exactly (trailing chunks may be empty)."""
    out = []
    for lo, hi, sub in split_tiles(tiles, parts, f32_numel):
        ci = cut_index(sub, nchunks)
        b = [lo] + [int(sub[ci[c], 0]) if ci[c] < len(sub) else hi
                    for c in range(1, nchunks)] + [hi]
        out.append([(b[c], b[c + 1], sub[ci[c]:ci[c + 1]]) for c in range(nchunks)])
    return out


def i64_tiles(tiles: np.ndarray) -> np.ndarray:
    return tiles[tiles[:, 2] >= K_I64_MIN]


def range_plans(layout: BucketLayout, parts: int, tile_elems: int = 0, flags=None,
                fractions=None):
    """[(lo, hi, Plan or None)] for each fp32 range, plus the int64 Plan."""
    if flags is None:
        flags = _lib.FA_PLAN_GAPS_ARE_PADDING
    info, tiles = layout_tiles(layout, tile_elems)
    te = info["tile_elems"]
    out = []
    for lo, hi, sel in split_tiles(tiles, parts, layout.f32_numel, fractions):
        p = (_lib.Plan(None, layout.f32_numel, None, layout.i64_numel, te, flags, tiles=sel)
             if len(sel) else None)
        out.append((lo, hi, p))
    t64 = i64_tiles(tiles)
    p64 = (_lib.Plan(None, layout.f32_numel, None, layout.i64_numel, te, flags, tiles=t64)
           if len(t64) else None)
    return out, p64


def chain_cut(layout: BucketLayout, nchunks: int):
    """The chained round's cut (fedcomm.hip chain_geo): the vector (cascade)
    tiles in ``nchunks`` column chunks [(lo, hi, tiles)], empty ones dropped;
    the scalar fp32 tiles re-based to compact columns (tiles, and the bucket
    index of each compact column); the int64 tiles."""
    _, tiles = layout_tiles(layout)
    t32 = tiles[tiles[:, 2] < K_I64_MIN]
    t32 = t32[np.argsort(t32[:, 0], kind="stable")]
    vec = t32[t32[:, 2] == 0]
    sc = t32[t32[:, 2] != 0]
    ci = cut_index(vec, nchunks)
    chunks = []
    for g in range(nchunks):
        if ci[g] == ci[g + 1]:
            continue
        sel = vec[ci[g]:ci[g + 1]]
        chunks.append((int(sel[0, 0]), int(sel[-1, 0] + sel[-1, 1]), sel))
    tidx = (np.concatenate([np.arange(s, s + c) for s, c, _ in sc]) if len(sc)
            else np.zeros(0, np.int64))
    starts = np.concatenate([[0], np.cumsum(sc[:, 1])[:-1]]) if len(sc) else np.zeros(0, np.int64)
    compact = np.stack([starts, sc[:, 1], sc[:, 2]], 1) if len(sc) else np.zeros((0, 3), np.int64)
    return chunks, compact, tidx, i64_tiles(tiles)
