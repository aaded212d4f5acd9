"""Replay of the native multi-GPU schedules on a CPU (test infrastructure).

``feddct_amd.comm.describe`` returns, per rank, the exact list of exchanges
and kernels libfedagg_comm.so issues for a round (fa_describe_round).  This
module runs ALL ranks' lists together with numpy buffers:

* exchanges follow RCCL's semantics: a step's exchanges are one group that
  completes when every send has met its receive (in posting order per
  sender/receiver pair) and every collective has been posted by every rank;
  a rank blocks on its current group.  No progress = a deadlock, reported;
* kernels are the oracle's restatement of what each kernel computes
  (oracle/torch_order.py: the column orders, the chained cascade state, the
  int64 truncation).

So the multi-rank logic of the native library — cut points, peers, offsets,
receive rows, state planes, roots — is exercised at any world size without
RCCL or a GPU.  Only the arithmetic of the kernels is substituted, and that
is pinned by the GPU tests.

r06: the executor's stream rules are checked too.  A compute-stream kernel
that reads exchanged data (the striped round's chunk reduce, fedcomm.hip
reads_exchanged) runs concurrently with its own step's group: it must not
read what that group receives, nor write what that group sends or receives;
and a step's sends must not read what the same step's kernels write (they
run after the group).  A violation raises Hazard.
"""
from __future__ import annotations

from collections import defaultdict

import numpy as np

from oracle import torch_order as O

F32 = np.float32
COMM = {"SEND", "RECV", "REDUCE", "ALLREDUCE", "REDUCE_SCATTER", "GATHER", "ALLGATHER", "BCAST"}


class Deadlock(AssertionError):
    pass


class Hazard(AssertionError):
    pass


# kernels the executor runs on the caller's (compute) stream
USER_KERNELS = {"K_SUM", "K_ZERO", "K_STACK", "K_PART", "K_BLOCK", "K_SCALE", "K_STRIPE"}


def _column_sum(kind, rows):
    """Per-column order of a tile kind (fedagg.hip TileKind) over rows (list
    of equal 1-D arrays)."""
    if kind in (0, 1):
        return O.cascade(rows)
    if kind == 2:
        return O.ilp4(rows)
    # M == 1 (one column)
    col = np.array([r[0] for r in rows], F32)
    n = len(rows)
    s = O.ilp4([col[i:i + 1] for i in range(n)])[0] if n < 8 else O.inner8(col)
    return np.array([s], F32)


class Sim:
    def __init__(self, layout, tiles, counts, clients32, clients64, weights=None, root=0):
        """``tiles``: the layout's tile table (partition.layout_tiles);
        ``clients32[s]`` / ``clients64[s]``: slot s's buckets (numpy);
        ``weights``: per slot fp32 or None."""
        self.layout = layout
        self.tiles = tiles
        self.counts = list(counts)
        self.W = len(counts)
        self.first = [int(sum(counts[:r])) for r in range(self.W)]
        self.n = int(sum(counts))
        self.nmax = max(counts)
        self.c32 = clients32
        self.c64 = clients64
        self.w = None if weights is None else np.asarray(weights, F32)
        self.t32 = tiles[tiles[:, 2] < 4]
        self.t32 = self.t32[np.argsort(self.t32[:, 0], kind="stable")]
        self.t64 = tiles[tiles[:, 2] >= 4]
        self.tail = self.t32[self.t32[:, 2] != 0]           # compact order = sorted by start
        self.tidx = np.concatenate([np.arange(s, s + c) for s, c, _ in self.tail]) \
            if len(self.tail) else np.zeros(0, np.int64)
        T = len(self.tidx)
        self.trow = (T + 63) // 64 * 64
        N32, N64 = layout.f32_numel, max(1, layout.i64_numel)
        self.t32_gathered = False
        self.buf = []
        for r in range(self.W):
            b = {"OUT": np.full(N32, np.nan, F32), "OUT64": np.full(N64, -7, np.int64),
                 "PARTIAL": np.zeros(N32, F32), "STRIPE": np.full(N32, np.nan, F32),
                 "FIN": np.full(N32, np.nan, F32), "RECV": defaultdict(
                     lambda: np.full(N32, np.nan, F32)),
                 "STATE": [np.full(N32, np.nan, F32) for _ in range(4)],
                 "STACK": [np.full(self.nmax * self.trow, np.nan, F32),
                           np.zeros(self.nmax * max(1, layout.i64_numel), np.int64)],
                 "GATHER": [np.full(self.W * self.nmax * self.trow, np.nan, F32),
                            np.zeros(self.W * self.nmax * max(1, layout.i64_numel), np.int64)],
                 # blocked mode (bucket offsets everywhere, stripes included)
                 "PIN": [np.zeros(N32, F32) for _ in range(4)],
                 "TAILP": [np.full(N32, np.nan, F32) for _ in range(4)],
                 "CONT": [np.full(N32, np.nan, F32) for _ in range(4)],
                 "BSUM": defaultdict(lambda: np.full(N32, np.nan, F32)),
                 "BLK": defaultdict(lambda: np.full(N32, np.nan, F32)),
                 "RELAY": defaultdict(lambda: np.full(N32, np.nan, F32)),
                 # striped, weighted: pre-multiplied local clients
                 "WSTAGE": defaultdict(lambda: np.full(N32, np.nan, F32))}
            self.buf.append(b)

    # ------------------------------------------------------------ buffers --
    def _view(self, r, name, index, off, cnt):
        b = self.buf[r]
        if name == "CLIENT":
            return self.c32[self.first[r] + index][off:off + cnt]
        if name in ("OUT", "PARTIAL", "STRIPE", "FIN"):
            return b[name][off:off + cnt]
        if name == "RECV":
            return b["RECV"][index][off:off + cnt]
        if name in ("STATE", "PIN", "TAILP", "CONT", "BSUM", "BLK", "RELAY", "WSTAGE"):
            return b[name][index][off:off + cnt]
        if name in ("STACK", "GATHER"):
            return b[name][index][off:off + cnt]
        raise KeyError(name)

    def _tiles_in(self, off, cnt, vec_only=False):
        t = self.t32
        sel = t[(t[:, 0] >= off) & (t[:, 0] < off + cnt)]
        return sel[sel[:, 2] == 0] if vec_only else sel

    def _rows(self, slots, getter):
        return [getter(s) for s in slots]

    # ------------------------------------------------------------ kernels --
    def _kernel(self, r, x):
        op = x["op"]
        b = self.buf[r]
        n_loc = self.counts[r]
        slots = range(self.first[r], self.first[r] + n_loc)
        wt = self.w

        def val(s, st, cnt):
            v = self.c32[s][st:st + cnt]
            return (v * wt[s]).astype(F32) if wt is not None else v

        if op == "K_SUM":
            for st, cnt, kind in self._tiles_in(x["offset"], x["count"]):
                b["PARTIAL"][st:st + cnt] = _column_sum(kind, [val(s, st, cnt) for s in slots])
        elif op == "K_ZERO":
            b["PARTIAL"][x["offset"]:x["offset"] + x["count"]] = 0
        elif op == "K_DIV":
            v = b["OUT"][x["offset"]:x["offset"] + x["count"]]
            v[:] = (v / F32(self.n)).astype(F32)
        elif op == "K_COPY":
            self._view(r, x["dst"], x["dst_index"], x["offset"], x["count"])[:] = \
                self._view(r, x["src"], x["src_index"], x["offset"], x["count"])
        elif op == "K_STRIPE":
            # local clients from their buckets (times their weights), the
            # others from their receive rows (pre-multiplied when weighted)
            for st, cnt, kind in self._tiles_in(x["offset"], x["count"]):
                rows = []
                for s in range(self.n):
                    if self.first[r] <= s < self.first[r] + n_loc:
                        rows.append(val(s, st, cnt))
                    else:
                        rows.append(b["RECV"][s][st:st + cnt])
                res = (F32(0) + _column_sum(kind, rows)).astype(F32)
                b[x["dst"]][st:st + cnt] = res if wt is not None else res / F32(self.n)
        elif op == "K_SCALE":
            off, cnt = x["offset"], x["count"]
            for j in range(x["nrows"]):
                s = self.first[r] + j
                b["WSTAGE"][j][off:off + cnt] = (self.c32[s][off:off + cnt] * wt[s]).astype(F32)
        elif op == "K_CHAIN":
            row0, nr = x["row0"], x["nrows"]
            lin = O.chain_levels(row0, self.n)
            lout = O.chain_levels(row0 + nr, self.n)
            for st, cnt, kind in self._tiles_in(x["offset"], x["count"], vec_only=True):
                acc = None
                if x["src"] == "STATE":
                    acc = [b["STATE"][l][st:st + cnt].copy() if lin & (1 << l)
                           else np.zeros(cnt, F32) for l in range(4)]
                elif lin:
                    raise AssertionError(f"rank {r}: chain kernel at row {row0} without state")
                acc = O.cascade_state([val(s, st, cnt) for s in range(row0, row0 + nr)], row0,
                                      self.n, acc)
                if x["dst"] == "STATE":
                    for l in range(4):
                        if lout & (1 << l):
                            b["STATE"][l][st:st + cnt] = acc[l]
                else:
                    s = O.cascade_finish(acc)
                    res = s if wt is not None else (s / F32(self.n)).astype(F32)
                    b[x["dst"]][st:st + cnt] = res
        elif op in ("K_PART", "K_CONT"):
            # fa_reduce_chain: PIN (plane 0 = the incoming partial, 1-3 zero) in
            row0, nr = x["row0"], x["nrows"]
            lin = O.chain_levels(row0, self.n)
            lout = O.chain_levels(row0 + nr, self.n)
            finishes = row0 + nr == self.n
            assert op == "K_CONT" or not finishes
            for st, cnt, kind in self.t32[self.t32[:, 2] == 0]:
                acc = [b["PIN"][l][st:st + cnt].copy() if lin & (1 << l) else np.zeros(cnt, F32)
                       for l in range(4)]
                acc = O.cascade_state([val(s, st, cnt) for s in range(row0, row0 + nr)], row0,
                                      self.n, acc)
                if finishes:   # sum only, into CONT plane 0
                    b["CONT"][0][st:st + cnt] = O.cascade_finish(acc)
                else:
                    dst = b["TAILP" if op == "K_PART" else "CONT"]
                    for l in range(4):
                        if lout & (1 << l):
                            dst[l][st:st + cnt] = acc[l]
        elif op == "K_BLOCK":
            row0, nr = x["row0"], x["nrows"]
            for st, cnt, kind in self.t32[self.t32[:, 2] == 0]:
                b["BSUM"][x["dst_index"]][st:st + cnt] = O.cascade(
                    [val(s, st, cnt) for s in range(row0, row0 + nr)])
        elif op == "K_FOLD":
            off, cnt, P = x["offset"], x["count"], x["nrows"]
            lp = O.level_power(self.n)
            Q, mask = 1 << lp, (1 << lp) - 1
            K = self.n // Q
            l1 = np.zeros(cnt, F32)
            l2 = np.zeros(cnt, F32)
            l3 = np.zeros(cnt, F32)
            for k in range(K):
                l1 = (l1 + b["BLK"][k][off:off + cnt]).astype(F32)
                i = (k + 1) << lp
                if i & (mask << lp):
                    continue
                l2, l1 = (l2 + l1).astype(F32), np.zeros(cnt, F32)
                if i & (mask << (2 * lp)):
                    continue
                l3, l2 = (l3 + l2).astype(F32), np.zeros(cnt, F32)
            l0 = b["BLK"][K][off:off + cnt] if P > K else np.zeros(cnt, F32)
            res = (((l0 + l1).astype(F32) + l2).astype(F32) + l3).astype(F32)
            if wt is None:
                res = (res / F32(self.n)).astype(F32)
            b[x["dst"]][off:off + cnt] = res
        elif op == "K_STACK":
            for j, s in enumerate(slots):
                if len(self.tidx):
                    v = self.c32[s][self.tidx]
                    if wt is not None:
                        v = (v * wt[s]).astype(F32)
                    b["STACK"][0][j * self.trow:j * self.trow + len(self.tidx)] = v
                if self.layout.i64_numel:
                    w64 = self.layout.i64_numel
                    b["STACK"][1][j * w64:(j + 1) * w64] = self.c64[s]
        elif op == "K_TAILS":
            rows = [(rr, j) for rr in range(self.W) for j in range(self.counts[rr])]
            if len(self.tidx) and self.t32_gathered:   # (chained mode only)
                g = b["GATHER"][0]
                comp = {int(e): k for k, e in enumerate(self.tidx)}
                for st, cnt, kind in self.tail:
                    ks = [comp[int(e)] for e in range(st, st + cnt)]
                    data = [g[(rr * self.nmax + j) * self.trow:][ks] for rr, j in rows]
                    res = _column_sum(kind, data)
                    res = (F32(0) + res).astype(F32)
                    b["OUT"][st:st + cnt] = res if wt is not None else (res / F32(self.n))
            if self.layout.i64_numel:
                w64 = self.layout.i64_numel
                g = b["GATHER"][1]
                data = np.stack([g[(rr * self.nmax + j) * w64:(rr * self.nmax + j + 1) * w64]
                                 for rr, j in rows])
                for o, m in self.layout.segs64:
                    b["OUT64"][o:o + m] = O.mean_i64_trunc(data[:, o:o + m])
        else:
            raise AssertionError(f"unknown kernel {op}")

    # ---------------------------------------------------------- exchanges --
    def _collective(self, xs):
        """xs[r] = rank r's op for one collective."""
        x0 = xs[0]
        op = x0["op"]
        for x in xs:
            assert x["op"] == op and x["count"] == x0["count"] and x["peer"] == x0["peer"], xs
        W = self.W
        off, cnt = x0["offset"], x0["count"]
        if op in ("REDUCE", "ALLREDUCE"):
            tot = self._view(0, xs[0]["src"], xs[0]["src_index"], off, cnt).copy()
            for r in range(1, W):
                tot = (tot + self._view(r, xs[r]["src"], xs[r]["src_index"], off, cnt)).astype(F32)
            for r in range(W):
                if op == "ALLREDUCE" or r == x0["peer"]:
                    self._view(r, xs[r]["dst"], xs[r]["dst_index"], off, cnt)[:] = tot
        elif op == "REDUCE_SCATTER":
            q = cnt // W
            parts = []
            for r in range(W):
                tot = self._view(0, xs[0]["src"], -1, off + r * q, q).copy()
                for rr in range(1, W):
                    tot = (tot + self._view(rr, xs[rr]["src"], -1, off + r * q, q)).astype(F32)
                parts.append(tot)
            for r in range(W):
                self._view(r, xs[r]["dst"], -1, off + r * q, q)[:] = parts[r]
        elif op in ("GATHER", "ALLGATHER") and xs[0]["src"] == "PARTIAL":
            q = cnt // W
            shares = [self._view(r, "PARTIAL", -1, off + r * q, q).copy() for r in range(W)]
            for r in range(W):
                if op == "ALLGATHER" or r == x0["peer"]:
                    for rr in range(W):
                        self._view(r, xs[r]["dst"], -1, off + rr * q, q)[:] = shares[rr]
        elif op == "ALLGATHER":
            idx = x0["src_index"]
            self.t32_gathered |= idx == 0
            rows = [self._view(r, "STACK", idx, 0, cnt).copy() for r in range(W)]
            for r in range(W):
                g = self.buf[r]["GATHER"][idx]
                for rr in range(W):
                    g[rr * cnt:(rr + 1) * cnt] = rows[rr]
        elif op == "BCAST":
            root = x0["peer"]
            data = self._view(root, xs[root]["dst"], -1, off, cnt).copy()
            for r in range(W):
                self._view(r, xs[r]["dst"], -1, off, cnt)[:] = data
        else:
            raise AssertionError(op)

    # ------------------------------------------------------------ hazards --
    def _regions_read(self, x):
        """(buffer, index, lo, hi) a kernel reads, as far as the hazard check
        needs (exchanged buffers only)."""
        if x["op"] == "K_STRIPE":
            return [("RECV", s, x["offset"], x["offset"] + x["count"]) for s in range(self.n)]
        return []

    def _regions_written(self, x):
        if x["op"] in COMM or x["dst"] in ("NONE",):
            return []
        if x["count"] <= 0:
            return [(x["dst"], None, 0, 1 << 62)]
        return [(x["dst"], x["dst_index"] if x["dst"] not in ("OUT", "STRIPE", "FIN", "PARTIAL")
                 else None, x["offset"], x["offset"] + x["count"])]

    @staticmethod
    def _overlap(a, b):
        return a[0] == b[0] and (a[1] is None or b[1] is None or a[1] == b[1]) and \
            a[2] < b[3] and b[2] < a[3]

    def _hazards(self, r, grp):
        recv_w = [(x["dst"], x["dst_index"] if x["dst"] not in ("OUT", "STRIPE", "FIN") else None,
                   x["offset"], x["offset"] + x["count"]) for x in grp if x["op"] == "RECV"]
        send_r = [(x["src"], x["src_index"] if x["src"] not in ("OUT", "STRIPE", "FIN") else None,
                   x["offset"], x["offset"] + x["count"]) for x in grp if x["op"] == "SEND"]
        for x in grp:
            if x["op"] in COMM:
                continue
            wr = self._regions_written(x)
            for a in wr:            # the step's sends ran before this kernel
                for b in send_r:
                    if self._overlap(a, b):
                        raise Hazard(f"rank {r} step {x['step']}: {x['op']} writes {a} "
                                     f"which the same step's send {b} reads")
            if x["op"] in USER_KERNELS:   # concurrent with the step's group
                for a in self._regions_read(x) + wr:
                    for b in recv_w:
                        if self._overlap(a, b):
                            raise Hazard(f"rank {r} step {x['step']}: {x['op']} touches {a} "
                                         f"while the same step's group receives {b}")

    def run(self, scheds):
        """``scheds[r]``: rank r's op list (comm.describe).  Runs to the end
        or raises Deadlock."""
        W = self.W
        pos = [0] * W
        posted = [None] * W          # ops of the current group, once posted
        sends = defaultdict(list)    # (src, dst) -> [(rank, op, matched flag holder)]
        recvs = defaultdict(list)
        coll = defaultdict(dict)     # seq -> {rank: op}
        coll_seq = [0] * W
        done_coll = set()
        matched = set()              # id of matched p2p entries

        def group_of(r):
            o = scheds[r]
            if pos[r] >= len(o):
                return None
            st = o[pos[r]]["step"]
            j = pos[r]
            while j < len(o) and o[j]["step"] == st:
                j += 1
            return o[pos[r]:j]

        while True:
            progress = False
            if all(pos[r] >= len(scheds[r]) for r in range(W)):
                break
            for r in range(W):
                grp = group_of(r)
                if grp is None:
                    continue
                if posted[r] is None:
                    entries = []
                    for x in grp:
                        if x["op"] == "SEND":
                            e = [r, x]
                            sends[(r, x["peer"])].append(e)
                            entries.append(("p2p", e))
                        elif x["op"] == "RECV":
                            e = [r, x]
                            recvs[(x["peer"], r)].append(e)
                            entries.append(("p2p", e))
                        elif x["op"] in COMM:
                            seq = coll_seq[r]
                            coll_seq[r] += 1
                            coll[seq][r] = x
                            entries.append(("coll", seq))
                    posted[r] = entries
                    progress = True
                # match p2p in posting order per channel
                for key in list(sends):
                    ss, rs = sends[key], recvs[key]
                    for k in range(min(len(ss), len(rs))):
                        if id(ss[k]) in matched:
                            continue
                        xs_, xr = ss[k][1], rs[k][1]
                        assert xs_["count"] == xr["count"], (key, xs_, xr)
                        src = self._view(ss[k][0], xs_["src"], xs_["src_index"], xs_["offset"],
                                         xs_["count"])
                        self._view(rs[k][0], xr["dst"], xr["dst_index"], xr["offset"],
                                   xr["count"])[:] = src
                        matched.add(id(ss[k]))
                        matched.add(id(rs[k]))
                        progress = True
                for seq, d in coll.items():
                    if seq not in done_coll and len(d) == W:
                        self._collective([d[rr] for rr in range(W)])
                        done_coll.add(seq)
                        progress = True
                ok = all((id(e) in matched) if kind == "p2p" else (e in done_coll)
                         for kind, e in posted[r])
                if ok:
                    self._hazards(r, grp)
                    for x in grp:
                        if x["op"] not in COMM:
                            self._kernel(r, x)
                    pos[r] += len(grp)
                    posted[r] = None
                    progress = True
            if not progress:
                stuck = {r: (group_of(r) or [{}])[0] for r in range(W)
                         if pos[r] < len(scheds[r])}
                raise Deadlock(f"no rank can progress: {stuck}")
        return self.buf
