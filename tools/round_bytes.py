"""Bytes and modelled time of each native multi-GPU round form, per rank
(r04; r06: per step, and the cost model) — from the schedule the executor
issues (fa_describe_round, host only, no GPU).

Per form and world size one JSON line:
  * max_rank_hbm_bytes / over_plain_reduce: what the busiest rank's kernels
    and DMA read and write in HBM, against the plain single-GPU reduce of the
    rank's own clients ((n_local + 1) * F * 4 bytes);
  * max_link_bytes: the largest byte count on one link direction over the
    round (any rank, any peer) — what one xGMI link carries;
  * max_step_link_bytes: the largest byte count on one link direction in ONE
    step (one RCCL group) of any rank;
  * serialized_link_bytes: per rank the sum over its steps of the step's
    largest per-link byte count (the link-bound time of the round x the link
    rate), max over ranks; pairwise_serialized_link_bytes: the same had every
    peer been exchanged with in a step of its own, one link at a time (r02-r05's
    striped round) — the sum over peers of max(bytes out, bytes in);
  * groups: RCCL groups on the busiest rank;
  * model_us: fa_round_model's time (include/fedagg_comm.h: link rate
    FA_MODEL_LINK_GBPS per direction, HBM FA_MODEL_HBM_GBPS, a fixed cost per
    group and per kernel; the stream rules of the executor);
  * chosen: the (form, chunks) the default entry takes for this shape.
The byte model per op is tests/roundmodel.py's (kernel_bytes,
coll_link_bytes), the same as the native model's.
Usage: round_bytes.py [LAYOUT] [SLOTS_PER_RANK] [W ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import roundmodel as RM  # noqa: E402
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


FORMS = [("blocked", C.FA_MODE_BLOCKED, {}),
         ("chained_4", C.FA_MODE_CHAINED, {"nchunks": 4}),
         ("chained_16", C.FA_MODE_CHAINED, {"nchunks": 16}),
         ("striped_1", C.FA_MODE_STRIPED, {"nchunks": 1}),
         ("striped_4", C.FA_MODE_STRIPED, {"nchunks": 4}),
         ("sharded_reduce", C.FA_MODE_SHARDED, {"nchunks": 8}),
         ("sharded_rs_gather", C.FA_MODE_SHARDED,
          {"nchunks": 8, "exchange": C.FA_XCHG_RS_GATHER})]


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "wrn16_8_c10"
    spr = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    ws = [int(x) for x in sys.argv[3:]] or [2, 4, 8]
    lay = layout_of(name)
    F = int(lay.f32_numel)
    for W in ws:
        counts = [spr] * W
        plain = (spr + 1) * F * 4
        root = W - 1
        chosen = C.multi_select(counts, layout=lay, detail=True)
        for fname, mode, kw in FORMS:
            try:
                m = C.round_model(mode, lay, counts, root=root, **kw)
                scheds = [C.describe(mode, lay, counts, r, root=root, **kw) for r in range(W)]
                steps = [RM.per_step(o, W) for o in scheds]
                step_link = max(link for st in steps for _, link, _ in st)
                serial = max(sum(link for _, link, _ in st) for st in steps)
                pair = max(pairwise(o, W) for o in scheds)
            except _lib.FedaggError as e:
                print(json.dumps({"layout": name, "W": W, "form": fname, "error": str(e)}))
                continue
            print(json.dumps({
                "layout": name, "W": W, "slots_per_rank": spr, "form": fname, "root": root,
                "max_rank_hbm_bytes": int(m["hbm_bytes_max"]),
                "over_plain_reduce": round(m["hbm_bytes_max"] / plain, 3),
                "max_link_bytes": int(m["link_bytes_max"]),
                "max_step_link_bytes": int(step_link), "serialized_link_bytes": int(serial),
                "pairwise_serialized_link_bytes": int(pair),
                "groups": m["groups"], "model_us": round(m["model_us"], 1),
                "chosen": list(chosen[:2]), "bucket_bytes": F * 4}), flush=True)


def pairwise(ops, W):
    """Bytes one rank would serialize exchanging with one peer at a time."""
    out, inn = [0.0] * W, [0.0] * W
    for x in ops:
        if x["op"] in ("SEND", "RECV"):
            (out if x["op"] == "SEND" else inn)[x["peer"]] += x["count"] * RM.elem_bytes(x)
    return sum(max(a, b) for a, b in zip(out, inn))


if __name__ == "__main__":
    main()
