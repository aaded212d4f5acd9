#!/bin/bash
# Broadcast forms: parity (fuzz over the four broadcast forms, shim/e2e
# broadcast tests, broadcast_f32, torch-GPU order with its broadcast) and
# the A/B of every form in one process.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_gpu_e2e.py tests/test_gpu_surface.py tests/test_gpu_torch_order.py -x -q --timeout 150 --timeout-method thread > gpurun_out/bcast_tests.log 2>&1 \
&& timeout -k 10 300 python3 tools/exp_bcast.py 5 > gpurun_out/exp_bcast.jsonl 2> gpurun_out/exp_bcast.err
rc=$?
echo "exit=$rc"
tail -3 gpurun_out/bcast_tests.log
cat gpurun_out/exp_bcast.jsonl
exit $rc
