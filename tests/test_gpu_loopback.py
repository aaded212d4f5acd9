"""GPU: the native multi-rank rounds of libfedagg_comm (fedcomm.hip, unchanged)
with W = 2..8 ranks on the one GPU of the box, over an in-process loopback of
the RCCL calls it makes (tests/loopback/loopccl.hip; RCCL itself refuses two
ranks on one device).  The C++ driver (tests/loopback/loop_round.cpp) builds
the clients with the portable synthetic state, runs one round per case and
compares every result rank with one GPU's fa_reduce over all clients:
chained, striped and blocked bit for bit, sharded (e1) within the forward error bound
of two N-term sums; int64 keys bit for bit everywhere.

Both process models of fedcomm run: one thread + communicator per rank
(fa_comm_init_rank — the product's one-process-per-GPU model, ranks progress
independently) for every mode, and one thread driving every rank
(fa_comm_init) for the sharded and blocked rounds.  The chained and striped schedules
pair a send in one step with its receive in a later step of another rank;
RCCL matches those on the device, a host-side loopback driven by one thread
cannot (the receive would wait for a send the same thread has not issued),
so their single-thread form is left to tests/schedsim.py.  Cases cover
uneven counts, a rank without clients, every root (first, middle, last, all),
weighted rounds, 1..13 column chunks, N >= 256 (the deep cascade's four state
planes) and the layouts of BASELINE configs 3 and 5."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import load_manifest
from feddct_amd.layout import BucketLayout
from feddct_amd.workload import joint_manifest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "tests", "loopback", "loop_round")


def _write_layout(layout, path, params=None):
    """``params``: {offset: (key_index, mu, sigma)} per fp32 segment and
    {offset: key_index} per int64 one — the digest generator's inputs."""
    with open(path, "w") as f:
        f.write(f"{layout.f32_numel} {layout.i64_numel} {len(layout.segs32)} "
                f"{len(layout.segs64)}{' P' if params else ''}\n")
        for o, m in layout.segs32:
            extra = ""
            if params:
                k, mu, sg = params[0][int(o)]
                extra = f" {k} {float(np.float32(mu)):.9g} {float(np.float32(sg)):.9g}"
            f.write(f"{int(o)} {int(m)}{extra}\n")
        for o, m in layout.segs64:
            extra = f" {params[1][int(o)]}" if params else ""
            f.write(f"{int(o)} {int(m)}{extra}\n")


def _digest_params(layout, parts):
    """Per-segment generator parameters of a (joint) layout: key index = the
    key's position in its own manifest (feddct_amd/workload.py fill_client)."""
    from feddct_amd import synth
    p32, p64 = {}, {}
    for man, prefix in parts:
        for j, e in enumerate(man["keys"]):
            s = layout.by_key[prefix + e["key"]]
            if s.kind == "i64":
                p64[s.offset] = j
            else:
                mu, sg = synth.key_params(e["key"], tuple(e["shape"]), e["dtype"])
                p32[s.offset] = (j, mu, sg)
    return p32, p64


def _run(layout, cases, tmp_path, timeout=240, params=None, dump=None, profile=False):
    assert os.path.exists(DRIVER), "tests/loopback/loop_round is not built (run build())"
    lf = str(tmp_path / "layout.txt")
    _write_layout(layout, lf, params)
    env = dict(os.environ, FA_LOOP_TIMEOUT_S="30")
    if profile:
        env["FA_LOOP_PROFILE"] = "1"
    if dump:
        env["FA_LOOP_DUMP"] = dump
    p = subprocess.run([DRIVER, lf, *cases], capture_output=True, text=True, timeout=timeout,
                       env=env)
    rows = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    for r in rows:
        print(json.dumps(r))
    assert len(rows) == len(cases), (p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    bad = [r for r in rows if not r["ok"]]
    assert not bad, (bad, p.stderr[-2000:])
    assert p.returncode == 0, p.stderr[-2000:]
    return rows


def _small_layout():
    """Every column class the schedules treat separately: vector runs, ILP-4
    tails, 0-d fp32 keys between vector keys, unaligned sizes, int64 keys."""
    return BucketLayout([("a", (37, 3), "float32"), ("s", (), "float32"),
                         ("b", (4101,), "float32"), ("t", (), "float32"),
                         ("c", (70000,), "float32"), ("d", (3,), "float32"),
                         ("e", (193,), "float32"), ("n1", (), "int64"),
                         ("f", (65, 65), "float32"), ("n2", (), "int64")])


@pytest.fixture(scope="module")
def cfg3_layout():
    mm, pm = load_manifest("wrnsl16_8_sf4_c10_main"), load_manifest("wrnsl16_8_sf4_c10_proxy")
    return BucketLayout.from_manifest(joint_manifest([mm, pm]))


def test_loopback_small_layout_all_modes(tmp_path):
    cases = [
        "chained:2:3,2:-1:threads:0:1",
        "chained:3:2,0,3:0:threads:0:4",
        "chained:3:4,5,3:1:threads:1:3",
        "chained:5:4,4,4,4,4:4:threads:1:13",
        "chained:8:1,2,1,3,1,1,2,9:-1:threads:0:8",
        "chained:4:65,65,65,65:3:threads:0:4",          # N=260: four state planes
        "striped:2:3,2:0:threads:0:0",
        "striped:3:2,0,3:-1:threads:0:0",
        "striped:8:1,2,1,3,1,1,2,9:5:threads:0:0",
        "striped:4:65,65,65,65:-1:threads:0:0",          # N=260: device pointer tables
        # r06: every peer in one group per chunk; chunk counts; weighted
        "striped:8:3,3,3,3,3,3,3,3:7:threads:0:1",
        "striped:8:3,3,3,3,3,3,3,3:-1:threads:1:3",
        "striped:5:4,0,2,1,6:2:threads:1:8",
        "striped:3:2,5,1:-1:threads:1:2",
        "striped:4:65,65,65,65:0:threads:1:4",           # weighted, N=260
        "sharded:4:65,65,65,65:0:threads:1:4",
        "sharded:2:3,2:0:threads:0:8",
        "sharded:4:5,0,2,1:-1:threads:1:4",
        "sharded:3:4,5,3:2:single:0:1",
        "sharded_rs:2:3,2:0:threads:0:8",
        "sharded_rs:4:5,1,2,1:-1:threads:1:4",
        "sharded_rs:8:1,2,1,3,1,1,2,9:7:threads:0:13",
        "sharded_rs:3:4,5,3:-1:single:0:2",
        "blocked:1:20:0:threads:0:0",
        "blocked:2:10,10:1:threads:0:0",
        "blocked:3:7,0,13:-1:threads:1:0",
        "blocked:3:16,16,1:0:single:0:0",
        "blocked:8:20,20,20,20,20,20,20,20:0:threads:0:0",
        "blocked:8:20,20,20,20,20,20,20,20:-1:single:1:0",
        "blocked:6:12,9,30,0,14,8:4:threads:0:0",
        "blocked:3:100,156,44:-1:threads:0:0",            # N=300: the fold's level 2
        # r05: the default entry picks the exact form from the counts
        "multi:8:1,2,1,3,1,1,2,9:-1:threads:0:0",
        "multi:3:7,0,13:-1:threads:1:0",
        "multi:4:65,65,65,65:3:threads:1:0",               # N=260
        "multi_e1:4:5,0,2,1:-1:threads:1:4",               # opt-in e1: error bound
        "mean_multi:3:4,5,3:2:threads:0:0",                # stateless fp32 form
        "mean_multi:8:3,3,3,3,3,3,3,3:-1:threads:0:0",
    ]
    _run(_small_layout(), cases, tmp_path)


def test_loopback_cfg3_layout(cfg3_layout, tmp_path):
    """BASELINE config 3's joint FedDCT bucket (main + proxy, 11.0 M floats),
    5 client slots over 2..5 ranks."""
    cases = [
        "chained:2:3,2:-1:threads:0:8",
        "chained:5:1,1,1,1,1:4:threads:0:8",
        "chained:3:2,1,2:0:threads:1:4",
        "striped:2:3,2:1:threads:0:0",
        "striped:4:2,1,1,1:-1:threads:0:0",
        "striped:5:1,1,1,1,1:4:threads:0:4",
        "striped:5:1,1,1,1,1:-1:threads:1:2",
        "sharded:2:3,2:0:threads:0:8",
        "sharded_rs:4:2,1,1,1:-1:threads:1:8",
        "blocked:2:3,2:0:threads:0:0",
        "blocked:2:20,20:-1:threads:1:0",
    ]
    _run(cfg3_layout, cases, tmp_path)


def test_loopback_cfg5_sharded_chain(tmp_path):
    """BASELINE config 5's shape: 24 FedDCT slots (wrnsl16_8 sf4 C100) over
    8 ranks of 3 slots, chained to the last rank and to every rank, and
    striped (r06: every peer in one group per chunk) in 1 and 4 chunks,
    weighted too."""
    mm, pm = load_manifest("wrnsl16_8_sf4_c100_main"), load_manifest("wrnsl16_8_sf4_c100_proxy")
    lay = BucketLayout.from_manifest(joint_manifest([mm, pm]))
    cases = ["chained:8:3,3,3,3,3,3,3,3:7:threads:0:8",
             "chained:8:3,3,3,3,3,3,3,3:-1:threads:0:8",
             "striped:8:3,3,3,3,3,3,3,3:-1:threads:0:4",
             "striped:8:3,3,3,3,3,3,3,3:7:threads:1:1"]
    _run(lay, cases, tmp_path, timeout=300)


def test_loopback_blocked_bench_shape(tmp_path):
    """The bench's N>1 shape: 20 wrn16_8 clients per rank, 4 and 8 ranks
    (160 slots: 10 blocks, six of them cut by a shard boundary), the
    result on rank 0 and on every rank."""
    lay = BucketLayout.from_manifest(load_manifest("wrn16_8_c10"))
    cases = ["blocked:4:20,20,20,20:0:threads:0:0",
             "blocked:8:20,20,20,20,20,20,20,20:0:threads:0:0",
             "blocked:8:20,20,20,20,20,20,20,20:-1:threads:0:0"]
    _run(lay, cases, tmp_path, timeout=300)


def test_loopback_cfg5_default_entry_matches_reference_digest(tmp_path):
    """the DEFAULT multi-GPU entry (fa_multi_plan_create /
    fa_reduce_multi — no form named by the caller) on BASELINE config 5's
    shape, 24 FedDCT slots (wrnsl16_8 sf4 C100, main + proxy in one bucket)
    over 8 ranks of 3 slots, with the digest generator's inputs: the result
    rank's main and proxy halves hash to the digests the REFERENCE's own
    server_aggregate produced (tests/golden/digests.json, n24), and equal one
    GPU's reduction bit for bit.  With 3 slots per rank a 16-slot cascade
    block spans 6 ranks (no blocked round); r06: the cost model takes the
    link-parallel striped round (r05: chained)."""
    from feddct_amd import dist
    mm, pm = load_manifest("wrnsl16_8_sf4_c100_main"), load_manifest("wrnsl16_8_sf4_c100_proxy")
    lay = BucketLayout.from_manifest(joint_manifest([mm, pm]))
    assert dist.exact_form([3] * 8, lay) == "striped"
    params = _digest_params(lay, [(mm, "0."), (pm, "1.")])
    dump = str(tmp_path / "out.bin")
    rows = _run(lay, ["multi:8:3,3,3,3,3,3,3,3:7:threads:0:0"], tmp_path, timeout=300,
                params=params, dump=dump)
    assert rows[0]["check"] == "bit-exact"
    raw = open(dump, "rb").read()
    f32 = np.frombuffer(raw[:4 * lay.f32_numel], np.float32)
    i64 = np.frombuffer(raw[4 * lay.f32_numel:], np.int64)
    with open(os.path.join(ROOT, "tests", "golden", "digests.json")) as f:
        want = json.load(f)
    for prefix, name in (("0.", "main"), ("1.", "proxy")):
        h = hashlib.sha256()
        for s in lay.slots:
            if not s.key.startswith(prefix):
                continue
            src = i64 if s.kind == "i64" else f32
            h.update(s.key[len(prefix):].encode())
            h.update(np.ascontiguousarray(src[s.offset:s.offset + s.numel]).tobytes())
        assert h.hexdigest() == want[f"feddct/wrnsl16_8_sf4_c100_{name}/n24"], name


def test_loopback_default_entry_random_shards(tmp_path):
    """The default entry over seeded random shard shapes (W = 2..8, 0..40
    slots per rank, empty ranks, every root, weighted and not): whatever form
    and chunk count the cost model picks, the result equals one GPU's
    reduction of all the slots bit for bit."""
    from feddct_amd import dist
    rng = np.random.default_rng(20260518)
    cases, forms = [], set()
    while len(cases) < 14:
        w = int(rng.integers(2, 9))
        counts = [int(c) for c in rng.integers(0, 41, size=w)]
        counts = [c if rng.random() > 0.15 else 0 for c in counts]
        if sum(counts) == 0:
            continue
        holders = [r for r, c in enumerate(counts) if c]
        root = int(rng.choice(holders + [-1]))
        forms.add(dist.exact_form(counts, _small_layout(), root_all=root < 0))
        cases.append(f"multi:{w}:{','.join(map(str, counts))}:{root}:threads:"
                     f"{int(rng.random() < 0.5)}:0")
    print("forms", sorted(forms))
    _run(_small_layout(), cases, tmp_path, timeout=300)


def test_loopback_default_entry_each_form(tmp_path):
    """The default entry's three exact forms each run at least once on the
    loopback: shapes the model sends to blocked, to chained and to striped
    (on a layout where a long chain of small hops loses to the stripes and
    the blocks win for many slots per rank)."""
    from feddct_amd import dist
    lay = BucketLayout([("a", (300000,), "float32"), ("s", (), "float32"),
                        ("b", (4101,), "float32"), ("n1", (), "int64")])
    shapes = {"striped": [3] * 8, "blocked": [20] * 4, "chained": [60, 60]}
    for form, counts in shapes.items():
        assert dist.exact_form(counts, lay) == form, (form, dist.exact_form(counts, lay))
    cases = [f"multi:{len(c)}:{','.join(map(str, c))}:{len(c) - 1}:threads:{i % 2}:0"
             for i, c in enumerate(shapes.values())]
    _run(lay, cases, tmp_path, timeout=300)


def test_loopback_round_profiles(tmp_path):
    """fa_comm_set_profile / fa_round_plan_profile (r06):
    a profiled round of each exact form reports its RCCL groups, its kernels
    and its wall time (rank 0 of the loopback), and stays bit-exact."""
    cases = ["striped:4:3,3,3,3:-1:threads:0:2", "chained:4:3,3,3,3:3:threads:0:4",
             "blocked:2:10,10:0:threads:1:0", "multi:8:3,3,3,3,3,3,3,3:7:threads:0:0"]
    rows = _run(_small_layout(), cases, tmp_path, profile=True)
    for r in rows:
        p = r["profile"]
        assert p is not None, r
        assert p["groups"] > 0 and p["kernels"] > 0 and p["wall_us"] > 0, r
        assert p["exchange_us"] > 0, r
