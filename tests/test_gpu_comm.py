"""GPU: the native RCCL round (libfedagg_comm.so) on a one-rank communicator
(the box has one GPU; RCCL refuses two ranks on one device).  With one rank
the exchange is the identity, so the result must equal the single-GPU
reduction bit for bit — which checks the chunking (every column summed once,
padding-spanning exchanges), the /N finish on the comm stream, the int64
gather + exact reduce and the stream joins.  The multi-rank orchestration is
covered on CPU with gloo (tests/test_dist_gloo.py) and by bench.py --gpus N."""
import ctypes

import numpy as np
import pytest
import torch

from conftest import load_manifest
from feddct_amd import synth
from feddct_amd.layout import BucketLayout
from feddct_amd.workload import make_clients

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def comm():
    torch.cuda.set_device(DEV)
    from feddct_amd import comm as C
    c = C.Comm.single()
    yield c
    c.close()


def _single_gpu(layout, clients, weights=None):
    from feddct_amd import _lib
    from feddct_amd.workload import Reducer
    o32, o64 = torch.zeros_like(clients[0][0]), torch.zeros_like(clients[0][1])
    Reducer(layout, clients, o32, o64, weights=weights)()
    torch.cuda.synchronize()
    return o32, o64


def _layout_pad_mask(layout):
    m = np.zeros(layout.f32_numel, bool)
    for o, n in layout.segs32:
        m[o:o + n] = True
    return torch.from_numpy(m).to(DEV)


@pytest.mark.parametrize("lay", ["wrn16_8_c10", "wrnsl16_8_sf4_c10_proxy"])
@pytest.mark.parametrize("final", ["reduce", "allreduce"])
@pytest.mark.parametrize("nchunks", [1, 8, 13])
def test_native_round_one_rank_is_bit_exact(comm, lay, final, nchunks):
    from feddct_amd.comm import NativeShardedAggregator
    man = load_manifest(lay)
    layout = BucketLayout.from_manifest(man)
    n = 20
    clients = make_clients(layout, man, range(n), DEV, mode=synth.MODE_ADVERSARIAL)
    want32, want64 = _single_gpu(layout, clients)
    out32 = torch.full_like(clients[0][0], float("nan"))
    out64 = torch.full_like(clients[0][1], -7)
    agg = NativeShardedAggregator(layout, [c[0] for c in clients], [c[1] for c in clients], n,
                                  out32, out64, comm, nchunks=nchunks, final=final)
    for _ in range(2):  # the second round reuses the plan's scratch and events
        agg.step()
    torch.cuda.synchronize()
    mask = _layout_pad_mask(layout)
    a, b = out32[mask].view(torch.int32), want32[mask].view(torch.int32)
    nan = torch.isnan(want32[mask])
    assert torch.equal(torch.isnan(out32[mask]), nan)
    assert torch.equal(a[~nan], b[~nan])
    assert torch.equal(out64, want64)


def test_native_round_weighted(comm):
    from feddct_amd.comm import NativeShardedAggregator
    man = load_manifest("wrn16_8_c100")
    layout = BucketLayout.from_manifest(man)
    n = 7
    clients = make_clients(layout, man, range(n), DEV)
    w = [float(np.float32(k / 28.0)) for k in range(1, n + 1)]
    want32, want64 = _single_gpu(layout, clients, weights=w)
    out32, out64 = torch.zeros_like(want32), torch.zeros_like(want64)
    NativeShardedAggregator(layout, [c[0] for c in clients], [c[1] for c in clients], n, out32,
                            out64, comm, weights=w).step()
    torch.cuda.synchronize()
    mask = _layout_pad_mask(layout)
    assert torch.equal(out32[mask], want32[mask])
    assert torch.equal(out64, want64)


def test_single_process_multi_device_form():
    """fa_comm_init(ndev, devs) + fa_reduce_sharded over an array of local
    plans (here ndev = 1: the one GPU of the box)."""
    from feddct_amd import _lib
    from feddct_amd import comm as C
    torch.cuda.set_device(DEV)
    man = load_manifest("wrnsl16_8_sf4_c10_main")
    layout = BucketLayout.from_manifest(man)
    n = 5
    clients = make_clients(layout, man, range(n), DEV)
    want32, want64 = _single_gpu(layout, clients)
    devs = (ctypes.c_int * 1)(0)
    hs = (ctypes.c_void_p * 1)()
    _lib.check(C.lib().fa_comm_init(1, devs, hs), "fa_comm_init")
    comm = C.Comm.__new__(C.Comm)
    comm.handle, comm.nranks, comm.rank = ctypes.c_void_p(hs[0]), 1, 0
    assert comm.info() == (1, 0, 0)
    out32, out64 = torch.zeros_like(want32), torch.zeros_like(want64)
    agg = C.NativeShardedAggregator(layout, [c[0] for c in clients], [c[1] for c in clients], n,
                                    out32, out64, comm, final="allreduce")
    agg.step()
    torch.cuda.synchronize()
    mask = _layout_pad_mask(layout)
    assert torch.equal(out32[mask], want32[mask])
    assert torch.equal(out64, want64)
    del agg
    comm.close()


def test_native_errors(comm):
    from feddct_amd import _lib
    from feddct_amd.comm import NativeShardedAggregator, ShardPlan
    man = load_manifest("wrnsl16_8_sf4_c10_main")
    layout = BucketLayout.from_manifest(man)
    clients = make_clients(layout, man, range(3), DEV)
    o32, o64 = torch.zeros_like(clients[0][0]), torch.zeros_like(clients[0][1])
    with pytest.raises(ValueError, match="shard"):
        NativeShardedAggregator(layout, [c[0] for c in clients], [c[1] for c in clients], 4,
                                o32, o64, comm)
    agg = NativeShardedAggregator(layout, [c[0] for c in clients], [c[1] for c in clients], 3,
                                  o32, o64, comm)
    agg.root = 5
    with pytest.raises(_lib.FedaggError, match="root"):
        agg.step()
    with pytest.raises(_lib.FedaggError, match="clients in total"):
        ShardPlan(comm, layout, [0])


@pytest.mark.parametrize("lay", ["wrn16_8_c10", "wrnsl16_8_sf4_c10_proxy",
                                 "wrnsl16_8_sf4_c10_main"])
@pytest.mark.parametrize("final", ["reduce", "allreduce"])
def test_native_striped_one_rank_is_bit_exact(comm, lay, final):
    """The exact mode (fa_reduce_striped): with one rank the stripe is the
    whole bucket and the exchanges are empty — the tile subset, the receive
    pointer arithmetic for local clients, the stripe gather copy and the
    int64 path must reproduce the single-GPU result bit for bit."""
    from feddct_amd.comm import NativeStripedAggregator
    man = load_manifest(lay)
    layout = BucketLayout.from_manifest(man)
    n = 20
    clients = make_clients(layout, man, range(n), DEV, mode=synth.MODE_ADVERSARIAL)
    want32, want64 = _single_gpu(layout, clients)
    out32 = torch.full_like(clients[0][0], float("nan"))
    out64 = torch.full_like(clients[0][1], -7)
    agg = NativeStripedAggregator(layout, [c[0] for c in clients], [c[1] for c in clients], n,
                                  out32, out64, comm, final=final)
    for _ in range(2):
        agg.step()
    torch.cuda.synchronize()
    mask = _layout_pad_mask(layout)
    nan = torch.isnan(want32[mask])
    assert torch.equal(torch.isnan(out32[mask]), nan)
    assert torch.equal(out32[mask].view(torch.int32)[~nan], want32[mask].view(torch.int32)[~nan])
    assert torch.equal(out64, want64)


def test_native_striped_weighted_one_rank(comm):
    """r06: the striped round takes weights (VERDICT r05 next 1 — it became
    a candidate of the default entry); with one rank it is the single-GPU
    weighted reduction, bit for bit (the multi-rank weighted rounds: the
    loopback and schedule-replay tests)."""
    from feddct_amd.comm import NativeStripedAggregator
    man = load_manifest("wrnsl16_8_sf4_c10_main")
    layout = BucketLayout.from_manifest(man)
    clients = make_clients(layout, man, range(3), DEV, mode=synth.MODE_ADVERSARIAL)
    w = [0.25, 0.5, 0.125]
    want32, want64 = _single_gpu(layout, clients, weights=w)
    o32 = torch.full_like(clients[0][0], float("nan"))
    o64 = torch.full_like(clients[0][1], -7)
    agg = NativeStripedAggregator(layout, [c[0] for c in clients], [c[1] for c in clients], 3,
                                  o32, o64, comm, weights=w)
    agg.step()
    torch.cuda.synchronize()
    mask = _layout_pad_mask(layout)
    assert torch.equal(o32[mask].view(torch.int32), want32[mask].view(torch.int32))
    assert torch.equal(o64, want64)


def test_stateless_mean_f32_multi():
    """fa_mean_f32_multi (SURVEY.md §8 b's stateless form) on a one-rank
    communicator: the fp32 mean equals the single-GPU fa_mean_f32; its cached
    plan goes away with the communicator."""
    from feddct_amd import _lib
    from feddct_amd import comm as C
    torch.cuda.set_device(DEV)
    c = C.Comm.single()
    man = load_manifest("wrn16_8_c10")
    layout = BucketLayout.from_manifest(man)
    clients = make_clients(layout, man, range(6), DEV, mode=synth.MODE_ADVERSARIAL)
    ptrs = _lib.ptr_array([x[0].data_ptr() for x in clients])
    segs, nseg = _lib.seg_array(layout.segs32)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    want = torch.zeros_like(clients[0][0])
    _lib.check(_lib.lib.fa_mean_f32(ptrs, 6, layout.f32_numel, want.data_ptr(), segs, nseg, st))
    got = torch.zeros_like(want)
    counts = (ctypes.c_int * 1)(6)
    for _ in range(2):  # the second call takes the cached plan
        _lib.check(C.lib().fa_mean_f32_multi(c.handle, ptrs, counts, layout.f32_numel,
                                             got.data_ptr(), segs, nseg, 0, st),
                   "fa_mean_f32_multi")
    torch.cuda.synchronize()
    mask = _layout_pad_mask(layout)
    assert torch.equal(got[mask], want[mask])
    c.close()


@pytest.mark.parametrize("lay", ["wrn16_8_c10", "wrnsl16_8_sf4_c10_proxy", "wrnsl16_8_sf4_c10_main"])
@pytest.mark.parametrize("final", ["reduce", "allreduce"])
@pytest.mark.parametrize("nchunks", [1, 16])
def test_native_chained_one_rank_is_bit_exact(comm, lay, final, nchunks):
    """fa_reduce_chained with one rank: the rank is its own finisher, so the
    vector chunks finish from the first segment and the scalar columns go
    through the raw stack/gather/compact-reduce/scatter path — all of which
    must reproduce the single-GPU reduction bit for bit (the multi-rank
    hops are replayed on CPU: tests/test_schedule.py)."""
    from feddct_amd.comm import NativeChainedAggregator
    man = load_manifest(lay)
    layout = BucketLayout.from_manifest(man)
    n = 20
    clients = make_clients(layout, man, range(n), DEV, mode=synth.MODE_ADVERSARIAL)
    want32, want64 = _single_gpu(layout, clients)
    out32 = torch.full_like(clients[0][0], float("nan"))
    out64 = torch.full_like(clients[0][1], -7)
    agg = NativeChainedAggregator(layout, [c[0] for c in clients], [c[1] for c in clients], n,
                                  out32, out64, comm, nchunks=nchunks, final=final)
    for _ in range(2):
        agg.step()
    torch.cuda.synchronize()
    mask = _layout_pad_mask(layout)
    nan = torch.isnan(want32[mask])
    assert torch.equal(torch.isnan(out32[mask]), nan)
    assert torch.equal(out32[mask].view(torch.int32)[~nan], want32[mask].view(torch.int32)[~nan])
    assert torch.equal(out64, want64)


def test_native_chained_weighted(comm):
    from feddct_amd.comm import NativeChainedAggregator
    man = load_manifest("wrn16_8_c100")
    layout = BucketLayout.from_manifest(man)
    n = 7
    clients = make_clients(layout, man, range(n), DEV, mode=synth.MODE_ADVERSARIAL)
    w = [float(np.float32(k / 28.0)) for k in range(1, n + 1)]
    want32, want64 = _single_gpu(layout, clients, weights=w)
    out32, out64 = torch.zeros_like(want32), torch.zeros_like(want64)
    NativeChainedAggregator(layout, [c[0] for c in clients], [c[1] for c in clients], n, out32,
                            out64, comm, weights=w).step()
    torch.cuda.synchronize()
    mask = _layout_pad_mask(layout)
    assert torch.equal(out32[mask].view(torch.int32), want32[mask].view(torch.int32))
    assert torch.equal(out64, want64)


@pytest.mark.parametrize("lay", ["wrn16_8_c10", "wrnsl16_8_sf4_c10_proxy"])
@pytest.mark.parametrize("final", ["reduce", "allreduce"])
@pytest.mark.parametrize("n,weighted", [(20, False), (5, False), (300, False), (33, True)])
def test_native_blocked_one_rank_is_bit_exact(comm, lay, final, n, weighted):
    """fa_reduce_blocked on a real RCCL communicator with one rank: every
    block is local (fa_reduce per 16 slots), the rank owns the one stripe and
    folds the block sums with the cascade's promotions (n=300: level 2) —
    the single-GPU reduction bit for bit.  Multi-rank: tests/test_schedule.py
    (CPU replay) and tests/test_gpu_loopback.py (2..8 ranks on this GPU)."""
    from feddct_amd.comm import NativeBlockedAggregator
    man = load_manifest(lay)
    layout = BucketLayout.from_manifest(man)
    clients = make_clients(layout, man, range(n), DEV, mode=synth.MODE_ADVERSARIAL)
    w = [float(np.float32(k / (n * (n + 1) / 2))) for k in range(1, n + 1)] if weighted else None
    want32, want64 = _single_gpu(layout, clients, weights=w)
    out32 = torch.full_like(clients[0][0], float("nan"))
    out64 = torch.full_like(clients[0][1], -7)
    agg = NativeBlockedAggregator(layout, [c[0] for c in clients], [c[1] for c in clients], n,
                                  out32, out64, comm, final=final, weights=w)
    for _ in range(2):
        agg.step()
    torch.cuda.synchronize()
    mask = _layout_pad_mask(layout)
    nan = torch.isnan(want32[mask])
    assert torch.equal(torch.isnan(out32[mask]), nan)
    assert torch.equal(out32[mask].view(torch.int32)[~nan], want32[mask].view(torch.int32)[~nan])
    assert torch.equal(out64, want64)


@pytest.mark.parametrize("final", ["reduce", "allreduce"])
def test_native_rs_gather_exchange_one_rank(comm, final):
    """e1 with the reduce-scatter + gather exchange (FA_XCHG_RS_GATHER): one
    rank's reduce-scatter / gather are the identity, so the round equals the
    single-GPU reduction (the remainder path included: chunk lengths are not
    multiples of anything in particular)."""
    from feddct_amd.comm import FA_XCHG_RS_GATHER, NativeShardedAggregator
    man = load_manifest("wrn16_8_c10")
    layout = BucketLayout.from_manifest(man)
    n = 20
    clients = make_clients(layout, man, range(n), DEV, mode=synth.MODE_ADVERSARIAL)
    want32, want64 = _single_gpu(layout, clients)
    out32 = torch.full_like(clients[0][0], float("nan"))
    out64 = torch.full_like(clients[0][1], -7)
    agg = NativeShardedAggregator(layout, [c[0] for c in clients], [c[1] for c in clients], n,
                                  out32, out64, comm, nchunks=13, final=final,
                                  exchange=FA_XCHG_RS_GATHER)
    for _ in range(2):
        agg.step()
    torch.cuda.synchronize()
    mask = _layout_pad_mask(layout)
    nan = torch.isnan(want32[mask])
    assert torch.equal(out32[mask].view(torch.int32)[~nan], want32[mask].view(torch.int32)[~nan])
    assert torch.equal(out64, want64)


def test_python_chain_aggregator_one_rank_nccl():
    """dist.ChainAggregator (torch.distributed orchestration, HIP backend) in
    a one-rank RCCL group: bit-exact with the single-GPU reduction, also for
    the full FedDCT config-5 layout (24 slots)."""
    import os
    import socket
    import torch.distributed as dist
    from feddct_amd.dist import ChainAggregator
    from feddct_amd.workload import joint_manifest
    torch.cuda.set_device(DEV)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=DEV)
    try:
        mm = load_manifest("wrnsl16_8_sf4_c100_main")
        pm = load_manifest("wrnsl16_8_sf4_c100_proxy")
        layout = BucketLayout.from_manifest(joint_manifest([mm, pm]))
        n = 24
        clients = make_clients(layout, [(mm, "0."), (pm, "1.")], range(n), DEV)
        want32, want64 = _single_gpu(layout, clients)
        out32 = torch.full_like(clients[0][0], float("nan"))
        out64 = torch.full_like(clients[0][1], -7)
        agg = ChainAggregator(layout, n, out32, out64, final="reduce", root=0, nchunks=8)
        agg.step([c[0] for c in clients], [c[1] for c in clients])
        torch.cuda.synchronize()
        mask = _layout_pad_mask(layout)
        assert torch.equal(out32[mask].view(torch.int32), want32[mask].view(torch.int32))
        assert torch.equal(out64, want64)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("form", ["chained16", "blocked", "sharded", "rs_gather", "striped"])
@pytest.mark.parametrize("n", [20, 300])
def test_captured_rounds_replay_bit_exact(form, n):
    """a native round's schedule is captured into a HIP
    graph on its first step and replayed by one launch afterwards
    (fa_comm_set_graphs).  The replays follow in-place changes of the client
    buckets (the graph holds pointers, not values), a new output buffer is a
    new capture, and every result equals the uncaptured executor's and one
    GPU's reduce, bit for bit — at 300 slots too, where the tails and the
    stripe take the graph's own device pointer tables."""
    from feddct_amd import comm as C
    torch.cuda.set_device(DEV)
    man = load_manifest("wrnsl16_8_sf4_c10_main" if n > 20 else "wrn16_8_c10")
    layout = BucketLayout.from_manifest(man)
    clients = make_clients(layout, man, range(n), DEV, mode=synth.MODE_ADVERSARIAL)
    l32, l64 = [c[0] for c in clients], [c[1] for c in clients]
    mask = _layout_pad_mask(layout)

    def make(comm, o32, o64):
        kw = dict(final="reduce", root=0)
        if form == "chained16":
            return C.NativeChainedAggregator(layout, l32, l64, n, o32, o64, comm, nchunks=16, **kw)
        if form == "blocked":
            return C.NativeBlockedAggregator(layout, l32, l64, n, o32, o64, comm, **kw)
        if form == "striped":
            return C.NativeStripedAggregator(layout, l32, l64, n, o32, o64, comm, **kw)
        ex = C.FA_XCHG_RS_GATHER if form == "rs_gather" else C.FA_XCHG_REDUCE
        return C.NativeShardedAggregator(layout, l32, l64, n, o32, o64, comm, nchunks=8,
                                         exchange=ex, **kw)

    results = {}
    for graphs in (False, True):
        comm = C.Comm.single()
        comm.set_graphs(graphs)
        o32 = torch.full_like(clients[0][0], float("nan"))
        o64 = torch.full_like(clients[0][1], -7)
        agg = make(comm, o32, o64)
        got = []
        for step in range(3):
            if step == 2:          # the clients change in place between rounds
                for c in clients:
                    c[0].mul_(-0.5)
                    c[1].add_(3)
            agg.step()
            torch.cuda.synchronize()
            got.append((o32[mask].clone(), o64.clone()))
        if step == 2:
            for c in clients:       # restore for the other executor
                c[0].mul_(-2.0)
                c[1].sub_(3)
        # a new output buffer: another capture, same bits
        p32 = torch.full_like(o32, float("nan"))
        p64 = torch.full_like(o64, -7)
        make(comm, p32, p64).step()
        torch.cuda.synchronize()
        got.append((p32[mask].clone(), p64.clone()))
        results[graphs] = got
        comm.close()
    want32, want64 = _single_gpu(layout, clients)
    for graphs, got in results.items():
        for i, (g32, g64) in enumerate(got):
            if i == 2:
                continue
            assert torch.equal(g32.view(torch.int32), want32[mask].view(torch.int32)), (graphs, i)
            assert torch.equal(g64, want64), (graphs, i)
    for a, b in zip(results[False], results[True]):
        assert torch.equal(a[0].view(torch.int32), b[0].view(torch.int32))
        assert torch.equal(a[1], b[1])
    assert not torch.equal(results[True][2][0], results[True][1][0])  # step 2 saw the change
