"""The round cost model restated in Python (test infrastructure; r06).

fedcomm.hip's fa_round_model times every rank's schedule (fa_describe_round)
in virtual time under the executor's stream rules; this module replays the
same schedules (``feddct_amd.comm.describe``) by the rules written out again
from the header (include/fedagg_comm.h, "the round cost model"), so a test
can hold the native model to its own definition:

* per rank two clocks: the communication stream ``tc`` and the caller's
  (compute) stream ``tu``;
* a step's exchanges are one group, posted on ``tc`` — after ``tu`` when one
  of them reads compute-stream output — and complete when every peer has
  posted the matching operations (p2p: the k-th send of a pair meets its
  k-th receive; collectives: the k-th of every rank), then take
  GROUP_US + max(the largest byte count on one link direction / LINK,
  the group's HBM bytes / HBM);
* kernels: KERNEL_US + HBM bytes / HBM, on the stream the executor uses; a
  compute-stream kernel reading exchanged data waits for ``tc`` as it was
  before its own step's group.

Nothing here is shipped; ``tools/round_bytes.py`` prints the same per-step
quantities for a layout.
"""
from __future__ import annotations

from collections import defaultdict

from oracle import torch_order as O

LINK_GBPS, HBM_GBPS, GROUP_US, KERNEL_US = 64.0, 6500.0, 15.0, 3.0
COMM = {"SEND", "RECV", "REDUCE", "ALLREDUCE", "REDUCE_SCATTER", "GATHER", "ALLGATHER", "BCAST"}
USER_WRITTEN = {"PARTIAL", "STACK", "TAILP", "BSUM", "STATE", "OUT", "FIN", "STRIPE", "WSTAGE"}


def us_link(b):
    return b / (LINK_GBPS * 1e3)


def us_hbm(b):
    return b / (HBM_GBPS * 1e3)


def on_comm_stream(x):
    if x["op"] in COMM:
        return True
    if x["op"] in ("K_SUM", "K_ZERO", "K_STACK", "K_PART", "K_BLOCK", "K_SCALE", "K_STRIPE"):
        return False
    if x["op"] == "K_CHAIN":
        return x["src"] == "STATE"
    return True


def reads_exchanged(x):
    return x["op"] == "K_STRIPE"


def needs_compute(x):
    return x["src"] in USER_WRITTEN


def kernel_bytes(x, n_total, V):
    b = 4.0 * (x["count"] if x["count"] > 0 else V)
    op = x["op"]
    if op in ("K_SUM", "K_STRIPE", "K_FOLD", "K_PART", "K_BLOCK"):
        return (x["nrows"] + 1) * b
    if op == "K_CONT":
        return (x["nrows"] + 2) * b
    if op == "K_CHAIN":
        lin = bin(O.chain_levels(x["row0"], n_total)).count("1") if x["src"] == "STATE" else 0
        lout = (bin(O.chain_levels(x["row0"] + x["nrows"], n_total)).count("1")
                if x["dst"] == "STATE" else 1)
        return (x["nrows"] + lin + max(lout, 1)) * b
    if op == "K_COPY":
        return 0.0 if x["dst"] == "BLK" else 2 * b
    if op == "K_DIV":
        return 2 * b
    if op == "K_ZERO":
        return b
    if op == "K_SCALE":
        return 2.0 * x["nrows"] * b
    return 0.0


def elem_bytes(x):
    buf, idx = (x["dst"], x["dst_index"]) if x["op"] == "RECV" else (x["src"], x["src_index"])
    return 8.0 if buf in ("STACK", "GATHER") and idx == 1 else 4.0


def coll_link_bytes(x, W):
    n = x["count"] * elem_bytes(x)
    if x["op"] == "ALLGATHER":
        return n * (W - 1) / W if x["src"] == "PARTIAL" else n * (W - 1)
    if x["op"] == "BCAST":
        return n
    if x["op"] == "ALLREDUCE":
        return 2.0 * n * (W - 1) / W
    return n * (W - 1) / W


def model(scheds, n_total, V):
    """``scheds[r]``: rank r's op list (comm.describe).  Returns the dict
    fa_round_model returns."""
    W = len(scheds)
    pos = [0] * W
    posted = [False] * W
    tc, tu, post, ev3 = [0.0] * W, [0.0] * W, [0.0] * W, [0.0] * W
    hbm = [0.0] * W
    lout = [[0.0] * W for _ in range(W)]
    lin = [[0.0] * W for _ in range(W)]
    groups = [0] * W
    sendt, recvt = defaultdict(list), defaultdict(list)
    collt = {}
    cseq = [0] * W
    pend = [None] * W
    steps = 0
    while True:
        progress, done = False, True
        for r in range(W):
            o = scheds[r]
            if pos[r] >= len(o):
                continue
            done = False
            step = o[pos[r]]["step"]
            e = pos[r]
            while e < len(o) and o[e]["step"] == step:
                e += 1
            steps = max(steps, step + 1)
            grp = o[pos[r]:e]
            if not posted[r]:
                ev3[r] = tc[r]
                comm = any(x["op"] in COMM for x in grp)
                if any(x["op"] in COMM and needs_compute(x) for x in grp):
                    tc[r] = max(tc[r], tu[r])
                post[r] = tc[r]
                p2p, colls = [], []
                for x in grp:
                    if x["op"] == "SEND":
                        v = sendt[(r, x["peer"])]
                        p2p.append((x, len(v)))
                        v.append(post[r])
                    elif x["op"] == "RECV":
                        v = recvt[(x["peer"], r)]
                        p2p.append((x, len(v)))
                        v.append(post[r])
                    elif x["op"] in COMM:
                        q = cseq[r]
                        cseq[r] += 1
                        collt.setdefault(q, [-1.0] * W)[r] = post[r]
                        colls.append(q)
                pend[r] = (p2p, colls)
                groups[r] += 1 if comm else 0
                posted[r] = True
                progress = True
            start, ok = post[r], True
            for x, k in pend[r][0]:
                v = recvt[(r, x["peer"])] if x["op"] == "SEND" else sendt[(x["peer"], r)]
                if len(v) <= k:
                    ok = False
                    break
                start = max(start, v[k])
            if ok:
                for q in pend[r][1]:
                    if min(collt[q]) < 0:
                        ok = False
                        break
                    start = max(start, max(collt[q]))
            if not ok:
                continue
            go, gi = [0.0] * W, [0.0] * W
            ghbm = gcoll = 0.0
            comm = False
            for x in grp:
                if x["op"] not in COMM:
                    continue
                comm = True
                if x["op"] in ("SEND", "RECV"):
                    b = x["count"] * elem_bytes(x)
                    (go if x["op"] == "SEND" else gi)[x["peer"]] += b
                    (lout if x["op"] == "SEND" else lin)[r][x["peer"]] += b
                    ghbm += b
                else:
                    b = coll_link_bytes(x, W)
                    gcoll += b
                    ghbm += 2.0 * b
            if comm:
                link = max([gcoll] + [max(go[q], gi[q]) for q in range(W)])
                tc[r] = start + GROUP_US + max(us_link(link), us_hbm(ghbm))
                hbm[r] += ghbm
            for x in grp:
                if x["op"] in COMM:
                    continue
                kb = kernel_bytes(x, n_total, V)
                dur = KERNEL_US + us_hbm(kb)
                hbm[r] += kb
                if on_comm_stream(x):
                    if needs_compute(x):
                        tc[r] = max(tc[r], tu[r])
                    tc[r] += dur
                else:
                    if reads_exchanged(x):
                        tu[r] = max(tu[r], ev3[r])
                    tu[r] += dur
            pos[r] = e
            posted[r] = False
            progress = True
        if done:
            break
        if not progress:
            raise AssertionError("the schedules deadlock")
    return {"model_us": max(max(tc[r], tu[r]) for r in range(W)),
            "link_bytes_max": max(max(lout[r][q], lin[r][q]) for r in range(W) for q in range(W)),
            "hbm_bytes_max": max(hbm), "groups": max(groups), "steps": steps}


def per_step(ops, W):
    """One rank's schedule per step: (step, the largest byte count on one
    link direction, the DMA's HBM bytes) — what tools/round_bytes.py prints."""
    out = {}
    for x in ops:
        if x["op"] not in COMM:
            continue
        st = out.setdefault(x["step"], {"link": defaultdict(float), "coll": 0.0, "hbm": 0.0})
        if x["op"] in ("SEND", "RECV"):
            b = x["count"] * elem_bytes(x)
            st["link"][(x["op"], x["peer"])] += b
            st["hbm"] += b
        else:
            b = coll_link_bytes(x, W)
            st["coll"] += b
            st["hbm"] += 2 * b
    return [(k, max([v["coll"]] + list(v["link"].values())), v["hbm"]) for k, v in sorted(out.items())]
