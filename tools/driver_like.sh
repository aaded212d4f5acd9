#!/bin/bash
# The driver's own N=1 bench command (20 steps after 5 warm-up), summarised.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/driver_like_${1:-x}.json
timeout -k 10 420 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out 2> ${out%.json}.err || exit $?
python3 - "$out" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["value"], d["roofline"]["frac"], d["copy_ceiling_GBps"], d.get("read_ceiling_GBps"), d.get("headline_vs_box_ceilings"), d["round_with_broadcast_us"],
      d["dropin"], d["torch_gpu_order_mode"], d["headline_launch"])
PY
