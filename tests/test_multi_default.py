"""The default multi-GPU entry is exact and picks its
form by a cost model (r06), on a CPU:

* the native model (fa_round_model) equals its Python restatement
  (tests/roundmodel.py) on every form and shard shape tried, and the native
  choice (fa_multi_select_layout) is the argmin of the restated model over
  the candidate forms and chunk counts; the blocked form is chosen only
  where its precondition holds (dist.blocked_allowed = block_geo's own
  refusal), and the Python rule (dist.exact_form) names the same form;
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
import roundmodel as RM
from feddct_amd.dist import blocked_allowed, exact_form
from feddct_amd.layout import BucketLayout
from feddct_amd.partition import layout_tiles
from oracle import torch_order as O
from schedsim import Sim
from test_schedule import MAN, _buckets, _expected, _result_ranks

MODES = {"blocked": C.FA_MODE_BLOCKED, "chained": C.FA_MODE_CHAINED, "e1": C.FA_MODE_SHARDED,
         "striped": C.FA_MODE_STRIPED}
CANDIDATES = [("blocked", 1)] + [("chained", k) for k in (4, 8, 16, 32)] + \
    [("striped", k) for k in (1, 2, 4, 8)]


def _random_counts(rng, n):
    out = []
    for _ in range(n):
        W = rng.randint(1, 8)
        c = [rng.choice([0, 0, 1, 2, 3, 5, 7, 8, 10, 15, 16, 17, 20, 33]) for _ in range(W)]
        if sum(c):
            out.append(c)
    return out


def test_blocked_precondition_matches_block_geo():
    """dist.blocked_allowed is exactly where the blocked round's own geometry
    (block_geo) accepts the counts."""
    rng = random.Random(5)
    layout = BucketLayout.from_manifest(MAN)
    seen = set()
    for counts in _random_counts(rng, 300) + [[3] * 8, [20] * 8, [24], [1, 23], [16, 16, 1]]:
        allowed = blocked_allowed(counts)
        seen.add(allowed)
        for r in range(len(counts)):
            try:
                C.describe(C.FA_MODE_BLOCKED, layout, counts, r)
                ok = True
            except Exception as e:  # noqa: BLE001
                assert "more than two" in str(e), e
                ok = False
            assert ok == allowed or len(counts) == 1, (counts, r)
    assert seen == {True, False}


def _restated(layout, counts, mode, nchunks, root, weighted=False):
    _, tiles = layout_tiles(layout)
    V = int(tiles[tiles[:, 2] == 0][:, 1].sum())
    scheds = [C.describe(MODES[mode], layout, counts, r, nchunks=nchunks, root=root,
                         weighted=weighted) for r in range(len(counts))]
    return RM.model(scheds, sum(counts), V)


@pytest.mark.parametrize("counts", [[10, 10], [7, 0, 13], [3] * 8, [1, 1, 1, 17], [20] * 4,
                                    [2, 30, 2, 0, 0, 1, 3, 2], [5, 6]])
@pytest.mark.parametrize("root", [-1, "last"])
def test_native_model_equals_its_restatement(counts, root):
    """fa_round_model == tests/roundmodel.py on every candidate form, and
    the native default's choice is the restated model's argmin (blocked only
    where allowed; ties keep the earlier candidate)."""
    W = len(counts)
    root = max(r for r in range(W) if counts[r]) if root == "last" else root
    layout = BucketLayout.from_manifest(MAN)
    best = None
    for mode, k in CANDIDATES + [("striped", 3)]:
        if mode == "blocked" and not blocked_allowed(counts):
            continue
        nat = C.round_model(MODES[mode], layout, counts, nchunks=k, root=root)
        py = _restated(layout, counts, mode, k, root)
        for f in ("model_us", "link_bytes_max", "hbm_bytes_max"):
            assert nat[f] == pytest.approx(py[f], rel=1e-9, abs=1e-9), (mode, k, f, nat, py)
        assert (nat["groups"], nat["steps"]) == (py["groups"], py["steps"]), (mode, k)
        if (mode, k) in CANDIDATES and (best is None or py["model_us"] < best[2]):
            best = (mode, k, py["model_us"])
    form, k, us = C.multi_select(counts, layout=layout, root_all=root < 0, detail=True)
    assert (form, k) == best[:2], (form, k, best)
    assert us == pytest.approx(best[2], rel=1e-9)
    assert exact_form(counts, layout, root_all=root < 0) == form


def test_weighted_striped_model_pays_the_staging():
    """A weighted striped round stages the clients it sends (K_SCALE): more
    HBM bytes than the unweighted round, same link bytes."""
    layout = BucketLayout.from_manifest(MAN)
    u = C.round_model(C.FA_MODE_STRIPED, layout, [3] * 4, nchunks=2, root=-1)
    w = C.round_model(C.FA_MODE_STRIPED, layout, [3] * 4, nchunks=2, root=-1, weighted=True)
    assert w["link_bytes_max"] == u["link_bytes_max"]
    assert w["hbm_bytes_max"] > u["hbm_bytes_max"]
    assert w == pytest.approx(_restated(layout, [3] * 4, "striped", 2, -1, weighted=True))


def test_select_named_shapes():
    """BASELINE config 5's shape (8 ranks x 3 FedDCT slots) takes the striped
    round: one group per chunk over all 7 links against the chained round's
    one hop at a time; the bench's N>1 shape (8 x 20 wrn16_8 slots) the
    blocked round.  r05 chose chained for cfg5 by geometry alone."""
    from feddct_amd.workload import joint_manifest, load_manifest
    cfg5 = BucketLayout.from_manifest(joint_manifest(
        [load_manifest("wrnsl16_8_sf4_c100_main"), load_manifest("wrnsl16_8_sf4_c100_proxy")]))
    wrn = BucketLayout.from_manifest(load_manifest("wrn16_8_c10"))
    form, k, us = C.multi_select([3] * 8, layout=cfg5, detail=True)
    assert form == "striped", (form, k, us)
    ch = min(C.round_model(C.FA_MODE_CHAINED, cfg5, [3] * 8, nchunks=c, root=7)["model_us"]
             for c in (4, 8, 16, 32))
    assert us < ch / 2
    assert C.multi_select([20] * 8, layout=wrn) == "blocked"
    assert C.multi_select([3] * 8) == "striped"        # the nominal layout
    assert C.multi_select([20] * 8) == "blocked"
    assert C.multi_select([3] * 8, exact=False) == "e1"
    for counts in ([10, 10], [7, 0, 13], [1, 1, 1, 17]):
        assert C.multi_select(counts) in ("blocked", "chained", "striped")
        if not blocked_allowed(counts):
            assert C.multi_select(counts) != "blocked"
    with pytest.raises(Exception):
        C.multi_select([0, 0])


def test_cfg5_striped_per_link_bytes():
    """VERDICT r05 next 1 'done': on cfg5's 8 x 3 shape the striped round's
    largest per-step byte count on one link is about 1/7 of what the r05
    pairwise form put on one link per step (all of a peer's share in one
    group per chunk vs every peer in turn)."""
    from feddct_amd.workload import joint_manifest, load_manifest
    cfg5 = BucketLayout.from_manifest(joint_manifest(
        [load_manifest("wrnsl16_8_sf4_c100_main"), load_manifest("wrnsl16_8_sf4_c100_proxy")]))
    W, counts = 8, [3] * 8
    worst_link = worst_total = 0.0
    for r in range(W):
        steps = RM.per_step(C.describe(C.FA_MODE_STRIPED, cfg5, counts, r, nchunks=1, root=7), W)
        for _, link, _ in steps:
            worst_link = max(worst_link, link)
        # what the same rank moves over all its links in its busiest step
        by = {}
        for x in C.describe(C.FA_MODE_STRIPED, cfg5, counts, r, nchunks=1, root=7):
            if x["op"] in ("SEND", "RECV") and x["dst"] != "OUT" and x["src"] != "OUT":
                by[(x["step"], x["op"])] = by.get((x["step"], x["op"]), 0) + 4 * x["count"]
        worst_total = max([worst_total] + list(by.values()))
    # one peer's share of a rank's exchange: 1/7 of its whole per-step volume
    assert worst_link == pytest.approx(worst_total / 7, rel=0.02), (worst_link, worst_total)


@pytest.mark.parametrize("counts", [[10, 10], [7, 0, 13], [3, 3, 3, 3, 3, 3, 3, 3],
                                    [1, 1, 1, 17], [16, 16, 1], [2, 30, 2, 0, 0, 1, 3, 2]])
@pytest.mark.parametrize("root", [0, -1, "last"])
@pytest.mark.parametrize("weighted", [False, True])
def test_default_form_schedule_is_exact(counts, root, weighted):
    W = len(counts)
    root = W - 1 if root == "last" else root
    layout = BucketLayout.from_manifest(MAN)
    form, nchunks, _ = C.multi_select(counts, layout=layout, root_all=root < 0, detail=True)
    mode = MODES[form]
    n = sum(counts)
    states = [synth.gen_state(MAN, c, synth.MODE_ADVERSARIAL) for c in range(n)]
    c32, c64 = _buckets(layout, states)
    w = O.weights_from_sizes(np.arange(1, n + 1) * 5 + 1) if weighted else None
    _, tiles = layout_tiles(layout)
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
    from test_dist_gloo import OracleChainBackend, OracleStripeBackend, _bucket
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
                     backend=OracleChainBackend(layout, chunks, compact),
                     stripe_backend=OracleStripeBackend(layout))
    agg.step()
    q.put((rank, agg.form, agg._agg.root, out32.numpy().copy(), out64.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("counts,final,weighted", [([10, 10], "reduce", False),
                                                   ([3, 4, 2], "allreduce", False),
                                                   ([0, 6, 3], "reduce", True),
                                                   ([2, 2, 3], "reduce", True)])
def test_default_aggregator_is_exact_gloo(counts, final, weighted):
    """dist.Aggregator() with no form named: world 2 and 3 over gloo, the
    form the cost model picks (chained or striped; the blocked round is
    native only), the reference's bits on every result rank (the root
    defaults to the last rank holding slots)."""
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
    want_form = exact_form(counts, layout, root_all=final != "reduce")
    want_form = "striped" if want_form == "striped" else "chained"
    for rk, form, root, o32, o64 in res:
        assert form == f"{want_form}/torch.distributed"
        assert root == (last if final == "reduce" else -1)
        if final == "reduce" and rk != last:
            continue
        checked += 1
        for s in layout.slots:
            src = o64 if s.kind == "i64" else o32
            got = src[s.offset:s.offset + s.numel].reshape(s.shape)
            assert got.tobytes() == np.asarray(want[s.key]).tobytes(), (rk, s.key)
    assert checked == (1 if final == "reduce" else world)


def test_one_rank_model_is_the_plain_reduction():
    """With one rank every form is the single-GPU reduction (make_round): the
    model prices exactly that kernel, whatever form is named."""
    layout = BucketLayout.from_manifest(MAN)
    want = RM.KERNEL_US + 21 * (4.0 * layout.f32_numel + 8.0 * layout.i64_numel) / (
        RM.HBM_GBPS * 1e3)
    for mode in ("blocked", "chained", "striped"):
        m = C.round_model(MODES[mode], layout, [20], nchunks=4, root=0)
        assert m["model_us"] == pytest.approx(want) and m["groups"] == 0
    # the one-rank choice carries that same time (the bench's default_choice)
    form, k, us = C.multi_select([20], layout=layout, detail=True)
    assert form == "blocked" and k == 1 and us == pytest.approx(want)


def test_model_constants_from_the_environment():
    """The cost model's constants can be overridden per process
    (FA_MODEL_LINK_GBPS ...; fa_model_constants reports them), so rates
    measured on a multi-GPU node re-rank the forms without a rebuild: a
    faster link makes cfg5's exchange cheaper, a slower one dearer.  Run in
    child processes: the library reads the environment once."""
    import json
    import subprocess
    import sys
    code = ("import json, sys; sys.path.insert(0, %r); from feddct_amd import comm as C; "
            "from feddct_amd.layout import BucketLayout; from feddct_amd.workload import "
            "load_manifest, joint_manifest; "
            "m = [load_manifest('wrnsl16_8_sf4_c100_main'), load_manifest('wrnsl16_8_sf4_c100_proxy')]; "
            "lay = BucketLayout.from_manifest(joint_manifest(m)); "
            "print(json.dumps([C.model_constants(), C.multi_select([3] * 8, layout=lay, detail=True)]))"
            % os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    out = {}
    for tag, env in (("default", {}), ("fast", {"FA_MODEL_LINK_GBPS": "200"}),
                     ("slow", {"FA_MODEL_LINK_GBPS": "20", "FA_MODEL_GROUP_US": "0"}),
                     ("bad", {"FA_MODEL_LINK_GBPS": "-3"})):
        e = {k: v for k, v in os.environ.items() if not k.startswith("FA_MODEL_")}
        e.update(env)
        r = subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        out[tag] = json.loads(r.stdout.strip().splitlines()[-1])
    d, f, s, b = (out[k] for k in ("default", "fast", "slow", "bad"))
    assert d[0] == {"link_GBps": C.MODEL_LINK_GBPS, "hbm_GBps": C.MODEL_HBM_GBPS,
                    "group_us": C.MODEL_GROUP_US, "kernel_us": C.MODEL_KERNEL_US}
    assert f[0]["link_GBps"] == 200.0 and s[0]["link_GBps"] == 20.0 and s[0]["group_us"] == 0.0
    assert b[0] == d[0]          # a non-positive rate is ignored
    assert f[1][2] < d[1][2] < s[1][2]
