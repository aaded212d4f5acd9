#!/bin/bash
# cfg3's reduce (tools/cfg3_anatomy.py prof): kernel trace + FETCH_SIZE /
# WRITE_SIZE passes, each its own run; the anatomy lines -> gpurun_out/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/cfg3_anatomy.py 50 > gpurun_out/cfg3_anatomy.jsonl 2> gpurun_out/cfg3_anatomy.err \
&& timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/cfg3_trace -o run -- python3 tools/cfg3_anatomy.py prof 100 > gpurun_out/cfg3_prof.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d gpurun_out/cfg3_fetch -o run -- python3 tools/cfg3_anatomy.py prof 10 >> gpurun_out/cfg3_prof.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d gpurun_out/cfg3_write -o run -- python3 tools/cfg3_anatomy.py prof 10 >> gpurun_out/cfg3_prof.log 2>&1
