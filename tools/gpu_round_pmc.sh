#!/bin/bash
# Kernel trace + FETCH_SIZE / WRITE_SIZE passes (separate runs) of the cfg2
# round (reduce + broadcast) and of the torch-GPU-order reduce (MODES: any
# tools/round_prof.py modes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in ${MODES:-round tgpu}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/rp_${m}_trace -o run -- python3 tools/round_prof.py $m 50 > gpurun_out/rp_${m}.log 2>&1 \
  && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d gpurun_out/rp_${m}_fetch -o run -- python3 tools/round_prof.py $m 10 >> gpurun_out/rp_${m}.log 2>&1 \
  && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d gpurun_out/rp_${m}_write -o run -- python3 tools/round_prof.py $m 10 >> gpurun_out/rp_${m}.log 2>&1 \
  && python3 tools/round_pmc_summary.py gpurun_out/rp_${m}_trace gpurun_out/rp_${m}_fetch gpurun_out/rp_${m}_write gpurun_out/round_pmc_${m}.json $(grep -o 'algorithmic bytes [0-9]*' gpurun_out/rp_${m}.log | head -1 | grep -o '[0-9]*$') || exit 1
done
