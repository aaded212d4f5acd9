#!/bin/bash
# Sweep + counters for the weighted cfg2 and cfg3 launches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/tune_r2.py 5 > gpurun_out/tune_r2.jsonl 2> gpurun_out/tune_r2.err \
&& timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/p2_trace -o run -- python3 tools/prof_r2.py 50 > gpurun_out/p2_trace.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d gpurun_out/p2_fetch -o run -- python3 tools/prof_r2.py 10 > gpurun_out/p2_fetch.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d gpurun_out/p2_write -o run -- python3 tools/prof_r2.py 10 > gpurun_out/p2_write.log 2>&1 \
&& python3 tools/pmc_kernels.py gpurun_out/p2_trace gpurun_out/p2_fetch gpurun_out/p2_write gpurun_out/p2_pmc.json gpurun_out/prof_r2_workloads.json > gpurun_out/p2_pmc.log 2>&1
rc=$?
echo "exit=$rc"
cat gpurun_out/tune_r2.jsonl
cat gpurun_out/p2_pmc.log | head -80
exit $rc
