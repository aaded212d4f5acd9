"""Algorithmic bytes of each native multi-GPU round form, per rank (r04,
VERDICT r03 next 2): what every rank's own kernels read and write in HBM,
what its DMA engines move for the exchanges, and what crosses each xGMI link
— from the schedule the executor issues (fa_describe_round, host only, no
GPU), against the plain single-GPU reduce of the rank's own clients
((n_local + 1) * F * 4 bytes).  These are the per-rank local floors of the
weak-scaling curve that one GPU cannot measure.

Byte model per op (fp32 elements of the rank's bucket, F = f32_numel,
V = elements in vector tiles, the cascade region):
  K_SUM / K_PART / K_BLOCK   nrows rows of the op's range read, one plane written
  K_CONT                     + the incoming partial plane read
  K_CHAIN                    + the state planes read and written (fa_chain_levels)
  K_FOLD                     nrows stripe pieces read, one stripe written
  K_STRIPE                   n_total receive rows read, one stripe written
  K_COPY into BLK            0 (the executor binds the fold's piece in place)
  K_COPY otherwise           read + write; K_DIV read + write; K_ZERO write
  SEND / RECV                the range over the link to/from `peer`, read /
                             written in HBM by the DMA
  collectives                ring traffic: (W-1)/W of the range per link
                             direction (x2 for all-reduce), in and out of HBM
Scalar columns (ILP-4 tails, M == 1, int64: < 0.1 % of the bytes) are left
out.  Usage: round_bytes.py [LAYOUT] [SLOTS_PER_RANK] [W ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd import comm as C  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.workload import joint_manifest, load_manifest  # noqa: E402


def layout_of(name):
    if name.endswith("_pair"):
        stem = name[:-5]
        return BucketLayout.from_manifest(joint_manifest(
            [load_manifest(stem + "_main"), load_manifest(stem + "_proxy")]))
    return BucketLayout.from_manifest(load_manifest(name))


def rank_bytes(ops, F, V, n_total, W):
    hbm = link_out = link_in = 0
    per_peer = {}
    for o in ops:
        op, cnt = o["op"], o["count"]
        rng = cnt if cnt > 0 else V
        b = 4 * rng
        if op in ("K_SUM", "K_PART", "K_BLOCK"):
            hbm += o["nrows"] * b + b
        elif op == "K_CONT":
            hbm += o["nrows"] * b + 2 * b
        elif op == "K_CHAIN":
            lv_in = bin(_lib.lib.fa_chain_levels(o["row0"], n_total)).count("1")
            lv_out = bin(_lib.lib.fa_chain_levels(o["row0"] + o["nrows"], n_total)).count("1")
            hbm += o["nrows"] * b + (lv_in + max(lv_out, 1)) * b
        elif op == "K_FOLD":
            hbm += o["nrows"] * b + b
        elif op == "K_STRIPE":
            hbm += n_total * b + b
        elif op == "K_COPY":
            hbm += 0 if o["dst"] == "BLK" else 2 * b
        elif op == "K_DIV":
            hbm += 2 * b
        elif op == "K_ZERO":
            hbm += b
        elif op == "SEND":
            hbm += b
            link_out += b
            per_peer[o["peer"]] = per_peer.get(o["peer"], 0) + b
        elif op == "RECV":
            hbm += b
            link_in += b
        elif op in ("REDUCE", "REDUCE_SCATTER", "GATHER", "BCAST", "ALLGATHER"):
            if o["src"] in ("STACK",) or o["dst"] in ("GATHER",):
                continue   # scalar columns: negligible
            t = b * (W - 1) / W
            hbm += 2 * t
            link_out += t
            link_in += t
        elif op == "ALLREDUCE":
            t = 2 * b * (W - 1) / W
            hbm += 2 * t
            link_out += t
            link_in += t
    return hbm, link_out, link_in, max(per_peer.values()) if per_peer else 0


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "wrn16_8_c10"
    spr = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    ws = [int(x) for x in sys.argv[3:]] or [2, 4, 8]
    lay = layout_of(name)
    info, tiles = _lib.build_tiles_host(lay.segs32, lay.f32_numel, lay.segs64, lay.i64_numel)
    F, V = int(lay.f32_numel), int(info["cascade_elems"])
    forms = [("blocked", C.FA_MODE_BLOCKED, {}), ("chained_1", C.FA_MODE_CHAINED, {"nchunks": 1}),
             ("chained_16", C.FA_MODE_CHAINED, {"nchunks": 16}),
             ("striped", C.FA_MODE_STRIPED, {}),
             ("sharded_reduce", C.FA_MODE_SHARDED, {"nchunks": 8}),
             ("sharded_rs_gather", C.FA_MODE_SHARDED,
              {"nchunks": 8, "exchange": C.FA_XCHG_RS_GATHER})]
    for W in ws:
        counts = [spr] * W
        n_total = spr * W
        plain = (spr + 1) * F * 4
        for fname, mode, kw in forms:
            root = W - 1 if mode == C.FA_MODE_CHAINED else 0
            try:
                per = [rank_bytes(C.describe(mode, lay, counts, r, root=root, **kw), F, V,
                                  n_total, W) for r in range(W)]
            except _lib.FedaggError as e:
                print(json.dumps({"layout": name, "W": W, "form": fname, "error": str(e)}))
                continue
            hb = max(p[0] for p in per)
            print(json.dumps({
                "layout": name, "W": W, "slots_per_rank": spr, "form": fname,
                "max_rank_hbm_bytes": int(hb), "over_plain_reduce": round(hb / plain, 3),
                "max_rank_link_out_bytes": int(max(p[1] for p in per)),
                "max_rank_link_in_bytes": int(max(p[2] for p in per)),
                "max_bytes_to_one_peer": int(max(p[3] for p in per)),
                "bucket_bytes": F * 4}), flush=True)


if __name__ == "__main__":
    main()
