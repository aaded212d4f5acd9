#!/bin/bash
# r02 session 2: torch-GPU-order parity + wide/narrow A/B; the N>1 bench's
# phase deadline exercised on a two-rank gloo rehearsal (short deadline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_torch_order.py -x -v --timeout 120 --timeout-method thread > gpurun_out/tgpu_tests.log 2>&1 \
&& timeout -k 10 300 python3 tools/tgpu_speed.py 3 > gpurun_out/tgpu_speed.jsonl 2> gpurun_out/tgpu_speed.err \
&& FA_BENCH_PHASE_DEADLINE_S=3 timeout -k 10 300 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --same-device --steps 60 --warmup 2 > gpurun_out/deadline_rehearsal.json 2> gpurun_out/deadline_rehearsal.err
rc=$?
echo "exit=$rc"
tail -2 gpurun_out/tgpu_tests.log
cat gpurun_out/tgpu_speed.jsonl
head -c 600 gpurun_out/deadline_rehearsal.json
grep -a "exceeded" gpurun_out/deadline_rehearsal.err
exit $rc
