#!/bin/bash
# Weighted-path change check: weighted parity tests, the sweep, the bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -x -v -m gpu -k "weighted or tuning or special or many or reduce_matches" --timeout 150 --timeout-method thread > gpurun_out/pytest_w.log 2>&1 \
&& timeout -k 10 300 python3 tools/tune_r2.py 5 > gpurun_out/tune_r2b.jsonl 2> gpurun_out/tune_r2b.err \
&& timeout -k 10 420 python3 bench.py --no-cpu-baseline > gpurun_out/bench_n1b.json 2> gpurun_out/bench_n1b.err
rc=$?
echo "exit=$rc"
tail -3 gpurun_out/pytest_w.log
cat gpurun_out/tune_r2b.jsonl
exit $rc
