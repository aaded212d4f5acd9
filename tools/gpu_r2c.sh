#!/bin/bash
# GPU-order vector tiles + the reduce lab.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_torch_order.py tests/test_gpu_parity.py -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/pytest_tgpu.log 2>&1 \
&& timeout -k 10 120 ./tools/reducelab > gpurun_out/reducelab.jsonl 2>&1 \
&& timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/bench_c.json 2> gpurun_out/bench_c.err
rc=$?
echo "exit=$rc"; tail -3 gpurun_out/pytest_tgpu.log
exit $rc
