#!/bin/bash
# The FedProx term's kernels (tools/prox_profile.py prof, wrn16_8 C100,
# 11.0 M params): kernel trace + FETCH_SIZE / WRITE_SIZE passes, each its own
# run; then proxlab's same-shape read probe beside the product's partials
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prox_trace -o run -- python3 tools/prox_profile.py prof 200 > gpurun_out/prox_prof.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d gpurun_out/prox_fetch -o run -- python3 tools/prox_profile.py prof 10 >> gpurun_out/prox_prof.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d gpurun_out/prox_write -o run -- python3 tools/prox_profile.py prof 10 >> gpurun_out/prox_prof.log 2>&1 \
&& timeout -k 10 120 ./tools/proxlab tools/proxlab_wrn16_8_c100.txt 50 > gpurun_out/proxlab_probe.jsonl 2>> gpurun_out/prox_prof.log
