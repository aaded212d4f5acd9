#!/bin/bash
# The driver's own bench command twice (short run: 20 steps after 5 warm-up),
# then the N>1 phase deadline forced on a two-rank gloo rehearsal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/driver_like_1.json 2> gpurun_out/driver_like_1.err \
&& timeout -k 10 420 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/driver_like_2.json 2> gpurun_out/driver_like_2.err \
&& FA_BENCH_PHASE_DEADLINE_S=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --same-device --steps 20 --warmup 2 > gpurun_out/deadline_rehearsal.json 2> gpurun_out/deadline_rehearsal.err
rc=$?
echo "exit=$rc"
for f in gpurun_out/driver_like_1.json gpurun_out/driver_like_2.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d.get('headline_launch'), d.get('torch_gpu_order_mode'), d['other_configs']['cfg3_feddct_c10_n5']['us_per_step'])"; done
head -c 300 gpurun_out/deadline_rehearsal.json; echo
grep -a "exceeded" gpurun_out/deadline_rehearsal.err
exit $rc
