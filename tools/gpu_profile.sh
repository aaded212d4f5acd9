#!/bin/bash
# Kernel-trace + PMC (FETCH_SIZE, WRITE_SIZE in separate passes) of the bench
# workload; summaries are copied into profiles/ by the caller.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="bench.py --kernel-only --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof -o run -- python3 $B --steps 100 --warmup 100 > gpurun_out/prof_bench.json 2> gpurun_out/prof.log \
&& timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d gpurun_out/pmc_fetch -o run -- python3 $B --steps 10 --warmup 2 > gpurun_out/pmc_fetch.log 2>&1 \
&& timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d gpurun_out/pmc_write -o run -- python3 $B --steps 10 --warmup 2 > gpurun_out/pmc_write.log 2>&1 \
&& python3 tools/pmc_summary.py gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/reduce_pmc.json gpurun_out/prof_bench.json
