#!/bin/bash
# The driver's multi-GPU bench command with ONE rank over RCCL (nccl backend,
# native communicator, every round form, the parity phase, config 5): what
# bench.py --gpus N runs on an 8-GPU node, minus the cross-GPU traffic.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
FA_BENCH_STACK_DUMP_S=200 timeout -k 10 400 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --multi-rehearsal --steps 20 --warmup 5 > gpurun_out/multi_rehearsal.json 2> gpurun_out/multi_rehearsal.err || exit $?
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/multi_rehearsal.json").read().strip().splitlines()[-1])
print(d["value"], d["selected_mode"], d["config"]["parallelism"])
for k, v in d["modes"].items():
    print(" ", k, v.get("ms_per_step"), v.get("bit_exact"), v.get("error", ""))
print(json.dumps(d.get("cfg5_feddct_c100_n24_sharded"))[:800])
print("native_comm_error", d.get("native_comm_error"))
PY
