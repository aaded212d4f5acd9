"""Multi-GPU orchestration (feddct_amd/dist.py) rehearsed on CPU with gloo,
world_size 2 and 3: the arithmetic backends are the oracle, the exchange is
real torch.distributed.  Checks chunking at key boundaries, the cross-rank
sum, the /N_total finish and the exact int64 path."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from feddct_amd import synth
from feddct_amd.dist import ShardedAggregator, chunk_segments, shard_range
from feddct_amd.layout import BucketLayout
from oracle import torch_order as O

MAN = {"keys": [{"key": f"k{j}", "shape": [m], "dtype": "float32"}
                for j, m in enumerate([100, 4096, 33, 2048, 7, 1, 5000])]
       + [{"key": "nbt", "shape": [], "dtype": "int64"},
          {"key": "nbt2", "shape": [], "dtype": "int64"}]}


class OracleBackend:
    def __init__(self, layout, chunks):
        self.layout, self.chunks = layout, chunks

    def partial_sum(self, c, clients32, out):
        segs, _, _ = self.chunks[c]
        for o, m in segs:
            x = np.stack([t[o:o + m].numpy() for t in clients32])
            out[o:o + m] = torch.from_numpy(O.torch_sum0(x))

    def divide(self, x, d, out):
        out.copy_(torch.from_numpy((x.numpy() / np.float32(d)).astype(np.float32)))

    def reduce_i64(self, clients64, out):
        for o, m in self.layout.segs64:
            x = np.stack([t[o:o + m].numpy() for t in clients64])
            out[o:o + m] = torch.from_numpy(O.mean_i64_trunc(x))


def _bucket(layout, state):
    f32 = torch.zeros(layout.f32_numel)
    i64 = torch.zeros(max(1, layout.i64_numel), dtype=torch.int64)
    for k, v in state:
        s = layout.by_key[k]
        tgt = i64 if s.kind == "i64" else f32
        tgt[s.offset:s.offset + s.numel] = torch.from_numpy(np.array(v, copy=True)).reshape(-1)
    return f32, i64


def _worker(rank, world, port, n_total, q, final="allreduce", exchange="reduce"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    layout = BucketLayout.from_manifest(MAN)
    lo, hi = shard_range(n_total, world, rank)
    bk = [_bucket(layout, synth.gen_state(MAN, c, synth.MODE_ADVERSARIAL)) for c in range(lo, hi)]
    out32 = torch.zeros(layout.f32_numel)
    out64 = torch.zeros(max(1, layout.i64_numel), dtype=torch.int64)
    chunks = chunk_segments(layout, 3)
    agg = ShardedAggregator(layout, [b[0] for b in bk], [b[1] for b in bk], n_total, out32,
                            out64, nchunks=3, backend=OracleBackend(layout, chunks), final=final,
                            exchange=exchange)
    agg.step()
    # what each rank contributed, to rebuild the expected cross-rank sum
    part = torch.zeros(layout.f32_numel)
    for c in range(len(chunks)):
        OracleBackend(layout, chunks).partial_sum(c, [b[0] for b in bk], part)
    parts = [torch.zeros_like(part) for _ in range(world)]
    dist.all_gather(parts, part)
    if rank == 0:
        q.put((out32.numpy().copy(), out64.numpy().copy(), [p.numpy() for p in parts]))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,n_total,final,exchange", [
    (2, 20, "allreduce", "reduce"), (3, 7, "allreduce", "reduce"), (2, 20, "reduce", "reduce"),
    (3, 7, "reduce", "reduce"), (2, 20, "reduce", "rs_gather"), (3, 7, "allreduce", "rs_gather"),
    (3, 7, "reduce", "rs_gather")])
def test_sharded_round_gloo(world, n_total, final, exchange):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q, final, exchange))
             for r in range(world)]
    for p in procs:
        p.start()
    out32, out64, parts = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    layout = BucketLayout.from_manifest(MAN)
    states = [synth.gen_state(MAN, c, synth.MODE_ADVERSARIAL) for c in range(n_total)]
    exact = dict(O.aggregate_state(states))
    # int64 keys: raw all-gather + exact reduction == single-process reference
    for k in ("nbt", "nbt2"):
        s = layout.by_key[k]
        assert out64[s.offset] == exact[k][()]
    # fp32: exact within shards, summed across ranks, then /N_total
    tot = parts[0].copy()
    for p in parts[1:]:
        tot = (tot + p).astype(np.float32)
    want = (tot / np.float32(n_total)).astype(np.float32)
    for o, m in layout.segs32:
        if world == 2:  # a two-term sum is order-free: the exchange is exactly p0 + p1
            assert np.array_equal(out32[o:o + m].view(np.uint32), want[o:o + m].view(np.uint32))
        # and within the re-association error bound of the exact order:
        # |err| <= 2 N eps mean|x_i| (N-term fp32 summation, both orders)
        key = layout.slots[[s.offset for s in layout.slots].index(o)].key
        mag = np.mean(np.abs(np.stack([dict(st)[key].reshape(-1) for st in states])), 0)
        err = np.abs(out32[o:o + m].astype(np.float64) - exact[key].reshape(-1))
        assert (err <= 2 * n_total * 2.0 ** -24 * mag + 1e-38).all()


def test_shard_range_and_chunks():
    assert [shard_range(20, 8, r) for r in range(8)] == [(0, 3), (3, 6), (6, 9), (9, 12),
                                                          (12, 14), (14, 16), (16, 18), (18, 20)]
    layout = BucketLayout.from_manifest(MAN)
    ch = chunk_segments(layout, 3)
    assert 1 <= len(ch) <= 3
    assert ch[0][1] == 0 and ch[-1][2] == layout.f32_numel
    for (a, _, hi), (b, lo, _) in zip(ch, ch[1:]):
        assert hi == lo
    assert sum(len(c[0]) for c in ch) == len(layout.segs32)


# ------------------------------------------------ exact striped mode (e2) --
class OracleStripeBackend:
    """Per-column oracle over whatever columns a stripe chunk holds: the
    order a column needs depends only on its position inside its tensor.
    Weighted (n_total weights): the weighted order, no division."""

    def __init__(self, layout, lo=None, hi=None):
        self.layout = layout

    def reduce_chunk(self, c, lo, hi, sources, out32, weights=None):
        n = len(sources)
        for o, M in self.layout.segs32:
            a, b = max(o, lo), min(o + M, hi)
            if a >= b:
                continue
            x = np.stack([t[a - base:b - base].numpy() for t, base in sources])
            if weights is not None:
                x = (x * np.asarray(weights, np.float32)[:, None]).astype(np.float32)
            body = O.body_len(M)
            res = np.empty(b - a, np.float32)
            for j, e in enumerate(range(a, b)):
                col = [x[i, j:j + 1] for i in range(n)]
                if M == 1:
                    s = O.ilp4(col)[0] if n < 8 else O.inner8(x[:, j])
                elif e - o < body:
                    s = O.cascade(col)[0]
                else:
                    s = O.ilp4(col)[0]
                s = np.float32(np.float32(0) + np.float32(s))
                res[j] = s if weights is not None else s / np.float32(n)
            out32[a:b] = torch.from_numpy(res)

    def reduce_i64(self, clients64, out):
        for o, m in self.layout.segs64:
            x = np.stack([t[o:o + m].numpy() for t in clients64])
            out[o:o + m] = torch.from_numpy(O.mean_i64_trunc(x))


def _striped_worker(rank, world, port, n_total, host, q, final="allreduce", weighted=False,
                    nchunks=4):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from feddct_amd.dist import StripedAggregator
    layout = BucketLayout.from_manifest(MAN)
    out32 = torch.full((layout.f32_numel,), float("nan"))
    out64 = torch.zeros(max(1, layout.i64_numel), dtype=torch.int64)
    agg = StripedAggregator(layout, n_total, out32, out64, backend=OracleStripeBackend(layout),
                            final=final, nchunks=nchunks)
    if host:
        lo, hi = agg.lo, agg.hi
        allb = [_bucket(layout, synth.gen_state(MAN, c, synth.MODE_ADVERSARIAL))
                for c in range(n_total)]
        agg.step_host([b[0][lo:hi].clone() for b in allb], [b[1] for b in allb])
    else:
        a, b = shard_range(n_total, world, rank)
        bk = [_bucket(layout, synth.gen_state(MAN, c, synth.MODE_ADVERSARIAL)) for c in range(a, b)]
        w = O.weights_from_sizes(np.arange(1, n_total + 1) * 3 + 2) if weighted else None
        agg.step_device([x[0] for x in bk], [x[1] for x in bk],
                        None if w is None else w[a:b])
    q.put((rank, out32.numpy().copy(), out64.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_total,host,final,weighted,nchunks", [
    (2, 20, False, "allreduce", False, 4), (3, 7, False, "allreduce", False, 2),
    (2, 9, True, "allreduce", False, 4), (3, 7, False, "reduce", False, 1),
    (3, 8, False, "reduce", True, 3), (2, 5, False, "allreduce", True, 4)])
def test_striped_round_is_exact_gloo(world, n_total, host, final, weighted, nchunks):
    """The Python StripedAggregator over real torch.distributed (gloo), r06:
    per column chunk one batch with every peer (the native schedule), weighted
    rounds too — every result rank ends with the single-process bits."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_striped_worker, args=(r, world, port, n_total, host, q, final,
                                                       weighted, nchunks))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    layout = BucketLayout.from_manifest(MAN)
    states = [synth.gen_state(MAN, c, synth.MODE_ADVERSARIAL) for c in range(n_total)]
    if weighted:
        w = O.weights_from_sizes(np.arange(1, n_total + 1) * 3 + 2)
        exact = {}
        for j, (k, v0) in enumerate(states[0]):
            x = np.stack([np.asarray(st[j][1]) for st in states])
            exact[k] = O.mean_i64_trunc(x) if x.dtype == np.int64 else O.weighted_sum0(x, w)
    else:
        exact = dict(O.aggregate_state(states))
    for rk, o32, o64 in res:  # every rank (or the root) holds the full, exact state
        if final == "reduce" and rk != 0:
            continue
        for s in layout.slots:
            src = o64 if s.kind == "i64" else o32
            got = src[s.offset:s.offset + s.numel].reshape(s.shape)
            want = exact[s.key]
            assert got.tobytes() == np.asarray(want).tobytes(), s.key


# ------------------------------------------- exact client shards (chained) --
class OracleChainBackend:
    """The chained kernels restated with the oracle (cascade_state)."""

    def __init__(self, layout, chunks, compact):
        self.layout, self.chunks, self.compact = layout, chunks, compact

    def chain(self, c, clients32, row0, n_total, state, state_in, out, plane, weights=None):
        lev_in = O.chain_levels(row0, n_total)
        lev_out = O.chain_levels(row0 + len(clients32), n_total)
        for st, cnt, _ in self.chunks[c][2]:
            rows = []
            for j, t in enumerate(clients32):
                v = t[st:st + cnt].numpy()
                if weights is not None:
                    v = (v * np.float32(weights[j])).astype(np.float32)
                rows.append(v)
            acc = None
            if state_in:
                acc = [state[l * plane + st:l * plane + st + cnt].numpy().copy()
                       if lev_in & (1 << l) else np.zeros(cnt, np.float32) for l in range(4)]
            acc = O.cascade_state(rows, row0, n_total, acc)
            if out is None:
                for l in range(4):
                    if lev_out & (1 << l):
                        state[l * plane + st:l * plane + st + cnt] = torch.from_numpy(acc[l])
            else:
                s = O.cascade_finish(acc)
                if weights is None:
                    s = (s / np.float32(n_total)).astype(np.float32)
                out[st:st + cnt] = torch.from_numpy(s)

    def tails(self, rows32, tidx, out32, weighted):
        from schedsim import _column_sum
        n = len(rows32)
        for cs, cnt, kind in self.compact:
            res = _column_sum(kind, [r[cs:cs + cnt].numpy() for r in rows32])
            res = (np.float32(0) + res).astype(np.float32)
            if not weighted:
                res = (res / np.float32(n)).astype(np.float32)
            out32[tidx[cs:cs + cnt]] = torch.from_numpy(res)

    def reduce_i64(self, clients64, out):
        for o, m in self.layout.segs64:
            x = np.stack([t[o:o + m].numpy() for t in clients64])
            out[o:o + m] = torch.from_numpy(O.mean_i64_trunc(x))


def _chain_worker(rank, world, port, counts, final, weighted, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from feddct_amd.dist import ChainAggregator
    from feddct_amd.partition import chain_cut
    layout = BucketLayout.from_manifest(MAN)
    n_total = sum(counts)
    a = sum(counts[:rank])
    bk = [_bucket(layout, synth.gen_state(MAN, c, synth.MODE_ADVERSARIAL))
          for c in range(a, a + counts[rank])]
    out32 = torch.full((layout.f32_numel,), float("nan"))
    out64 = torch.full((max(1, layout.i64_numel),), -7, dtype=torch.int64)
    chunks, compact, tidx, _ = chain_cut(layout, 3)
    w = O.weights_from_sizes(np.arange(1, n_total + 1) * 3 + 2) if weighted else None
    agg = ChainAggregator(layout, n_total, out32, out64, backend=OracleChainBackend(
        layout, chunks, compact), final=final, nchunks=3, counts=counts)
    agg.step([x[0] for x in bk], [x[1] for x in bk],
             None if w is None else w[a:a + counts[rank]])
    q.put((rank, out32.numpy().copy(), out64.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("counts,final,weighted", [([10, 10], "reduce", False),
                                                   ([3, 4, 2], "allreduce", False),
                                                   ([0, 6, 3], "reduce", False),
                                                   ([5, 17], "allreduce", True),
                                                   ([9, 0, 8], "reduce", True)])
def test_chained_round_is_exact_gloo(counts, final, weighted):
    """The Python ChainAggregator over real torch.distributed (gloo): client
    shards stay put, the cascade state hops rank to rank; every result rank
    ends with the single-process reference's bits."""
    world = len(counts)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_chain_worker, args=(r, world, port, counts, final, weighted, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    layout = BucketLayout.from_manifest(MAN)
    n = sum(counts)
    states = [synth.gen_state(MAN, c, synth.MODE_ADVERSARIAL) for c in range(n)]
    if weighted:
        w = O.weights_from_sizes(np.arange(1, n + 1) * 3 + 2)
        exact = {}
        for j, (k, v0) in enumerate(states[0]):
            x = np.stack([np.asarray(s[j][1]) for s in states])
            exact[k] = O.mean_i64_trunc(x) if x.dtype == np.int64 else O.weighted_sum0(x, w)
    else:
        exact = dict(O.aggregate_state(states))
    for rk, o32, o64 in res:
        if final == "reduce" and rk != 0:
            continue
        for s in layout.slots:
            src = o64 if s.kind == "i64" else o32
            got = src[s.offset:s.offset + s.numel].reshape(s.shape)
            assert got.tobytes() == np.asarray(exact[s.key]).tobytes(), (rk, s.key)
