"""The default multi-GPU entry is exact, on a CPU:

* the form it takes (native fa_multi_select) agrees with the Python rule
  (dist.exact_form) and with the blocked round's own refusal (block_geo:
  fa_describe_round of the blocked mode fails exactly where the rule says
  "chained");
* the schedule of the selected form, replayed for all ranks at once
  (tests/schedsim.py, the oracle as arithmetic), gives the single-process
  reference's bits — including BASELINE config 5's 8 x 3 shape;
* the opt-in e1 form is what ``exact=False`` selects and nothing else does;
* the Python default (dist.Aggregator) over gloo, world 2 and 3, with the
  oracle backends: the reference's bits on every result rank.
"""
import os
import random
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from feddct_amd import comm as C
from feddct_amd import synth
from feddct_amd.dist import exact_form
from feddct_amd.layout import BucketLayout
from feddct_amd.partition import layout_tiles
from oracle import torch_order as O
from schedsim import Sim
from test_schedule import MAN, _buckets, _expected, _result_ranks

MODES = {"blocked": C.FA_MODE_BLOCKED, "chained": C.FA_MODE_CHAINED, "e1": C.FA_MODE_SHARDED}


def _random_counts(rng, n):
    out = []
    for _ in range(n):
        W = rng.randint(1, 8)
        c = [rng.choice([0, 0, 1, 2, 3, 5, 7, 8, 10, 15, 16, 17, 20, 33]) for _ in range(W)]
        if sum(c):
            out.append(c)
    return out


def test_select_matches_python_rule_and_block_geo():
    rng = random.Random(5)
    layout = BucketLayout.from_manifest(MAN)
    seen = set()
    for counts in _random_counts(rng, 400) + [[3] * 8, [20] * 8, [24], [1, 23], [16, 16, 1]]:
        form = C.multi_select(counts)
        assert form == exact_form(counts), counts
        assert C.multi_select(counts, exact=False) == "e1"
        seen.add(form)
        # the blocked round refuses exactly the counts the rule sends to the chain
        for r in range(len(counts)):
            try:
                C.describe(C.FA_MODE_BLOCKED, layout, counts, r)
                ok = True
            except Exception as e:  # noqa: BLE001
                assert "more than two" in str(e), e
                ok = False
            assert ok == (form == "blocked") or len(counts) == 1, (counts, r)
    assert seen == {"blocked", "chained"}


def test_select_named_shapes():
    assert C.multi_select([3] * 8) == "chained"        # cfg5: a block spans 6 ranks
    assert C.multi_select([20] * 8) == "blocked"       # the bench's N>1 shape
    assert C.multi_select([10, 10]) == "blocked"
    assert C.multi_select([7, 0, 13]) == "blocked"     # an empty rank between two
    assert C.multi_select([1, 1, 1, 17]) == "chained"
    with pytest.raises(Exception):
        C.multi_select([0, 0])


@pytest.mark.parametrize("counts", [[10, 10], [7, 0, 13], [3, 3, 3, 3, 3, 3, 3, 3],
                                    [1, 1, 1, 17], [16, 16, 1], [2, 30, 2, 0, 0, 1, 3, 2]])
@pytest.mark.parametrize("root", [0, -1, "last"])
@pytest.mark.parametrize("weighted", [False, True])
def test_default_form_schedule_is_exact(counts, root, weighted):
    W = len(counts)
    root = W - 1 if root == "last" else root
    mode = MODES[C.multi_select(counts)]
    layout = BucketLayout.from_manifest(MAN)
    n = sum(counts)
    states = [synth.gen_state(MAN, c, synth.MODE_ADVERSARIAL) for c in range(n)]
    c32, c64 = _buckets(layout, states)
    w = O.weights_from_sizes(np.arange(1, n + 1) * 5 + 1) if weighted else None
    _, tiles = layout_tiles(layout)
    nchunks = 16 if mode == C.FA_MODE_CHAINED else 1
    scheds = [C.describe(mode, layout, counts, r, nchunks=nchunks, root=root, weighted=weighted)
              for r in range(W)]
    bufs = Sim(layout, tiles, counts, c32, c64, w, root).run(scheds)
    want = _expected(states, w)
    for r in _result_ranks(W, root):
        for s in layout.slots:
            src = bufs[r]["OUT64"] if s.kind == "i64" else bufs[r]["OUT"]
            got = src[s.offset:s.offset + s.numel].reshape(s.shape)
            assert got.tobytes() == np.asarray(want[s.key]).tobytes(), (r, s.key)


# ------------------------------------------------ the Python default, gloo --
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, counts, final, weighted, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from feddct_amd.dist import Aggregator
    from feddct_amd.partition import chain_cut
    from test_dist_gloo import MAN as GMAN
    from test_dist_gloo import OracleChainBackend, _bucket
    layout = BucketLayout.from_manifest(GMAN)
    n = sum(counts)
    a = sum(counts[:rank])
    bk = [_bucket(layout, synth.gen_state(GMAN, c, synth.MODE_ADVERSARIAL))
          for c in range(a, a + counts[rank])]
    out32 = torch.full((layout.f32_numel,), float("nan"))
    out64 = torch.full((max(1, layout.i64_numel),), -7, dtype=torch.int64)
    chunks, compact, _, _ = chain_cut(layout, 3)
    w = O.weights_from_sizes(np.arange(1, n + 1) * 3 + 2) if weighted else None
    agg = Aggregator(layout, [x[0] for x in bk], [x[1] for x in bk], n, out32, out64,
                     final=final, counts=counts, nchunks=3,
                     weights=None if w is None else w[a:a + counts[rank]],
                     backend=OracleChainBackend(layout, chunks, compact))
    agg.step()
    q.put((rank, agg.form, agg._agg.root, out32.numpy().copy(), out64.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("counts,final,weighted", [([10, 10], "reduce", False),
                                                   ([3, 4, 2], "allreduce", False),
                                                   ([0, 6, 3], "reduce", True)])
def test_default_aggregator_is_exact_gloo(counts, final, weighted):
    """dist.Aggregator() with no form named: world 2 and 3 over gloo, the
    reference's bits on every result rank (the root defaults to the last
    rank holding slots)."""
    from test_dist_gloo import MAN as GMAN
    world = len(counts)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, counts, final, weighted, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    layout = BucketLayout.from_manifest(GMAN)
    n = sum(counts)
    states = [synth.gen_state(GMAN, c, synth.MODE_ADVERSARIAL) for c in range(n)]
    w = O.weights_from_sizes(np.arange(1, n + 1) * 3 + 2) if weighted else None
    want = _expected(states, w)
    last = max(r for r in range(world) if counts[r] > 0)
    checked = 0
    for rk, form, root, o32, o64 in res:
        assert form == "chained/torch.distributed"
        assert root == (last if final == "reduce" else -1)
        if final == "reduce" and rk != last:
            continue
        checked += 1
        for s in layout.slots:
            src = o64 if s.kind == "i64" else o32
            got = src[s.offset:s.offset + s.numel].reshape(s.shape)
            assert got.tobytes() == np.asarray(want[s.key]).tobytes(), (rk, s.key)
    assert checked == (1 if final == "reduce" else world)
