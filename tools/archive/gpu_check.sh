#!/bin/bash
# One GPU-box session: smoke, parity tests, bench, kernel-trace profile.
# Every GPU step has its own time limit; steps are chained with && so the
# first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
&& timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
&& timeout -k 10 400 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof -o run -- python3 bench.py --kernel-only --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/prof.log 2>&1
rc=$?
echo "exit=$rc"
tail -3 gpurun_out/pytest_gpu.log 2>/dev/null
cat gpurun_out/bench.json 2>/dev/null
exit $rc
