#!/bin/bash
# Where the opt-in torch-GPU order loses to the default order at N = 32
# (VERDICT r05 next 5): both orders' reduce over the same 32 wrn16_8 C10
# clients (tools/round_prof.py tgpu32 / cpu32), each as a kernel trace, the
# FETCH_SIZE and WRITE_SIZE passes, and one pass of wave-occupancy counters
# (SQ_WAVES: waves launched; SQ_WAVE_CYCLES: wave-resident cycles summed over
# waves; SQ_BUSY_CYCLES: cycles the SQs were busy; GRBM_GUI_ACTIVE: the GPU's
# busy cycles) — separate runs, as the PMC rules require.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in tgpu32 cpu32; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/rp_${m}_trace -o run -- python3 tools/round_prof.py $m 50 > gpurun_out/rp_${m}.log 2>&1 \
  && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d gpurun_out/rp_${m}_fetch -o run -- python3 tools/round_prof.py $m 10 >> gpurun_out/rp_${m}.log 2>&1 \
  && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d gpurun_out/rp_${m}_write -o run -- python3 tools/round_prof.py $m 10 >> gpurun_out/rp_${m}.log 2>&1 \
  && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d gpurun_out/rp_${m}_occ -o run -- python3 tools/round_prof.py $m 10 >> gpurun_out/rp_${m}.log 2>&1 \
  && python3 tools/round_pmc_summary.py gpurun_out/rp_${m}_trace gpurun_out/rp_${m}_fetch gpurun_out/rp_${m}_write gpurun_out/round_pmc_${m}.json $(grep -o 'algorithmic bytes [0-9]*' gpurun_out/rp_${m}.log | head -1 | grep -o '[0-9]*$') || exit 1
done
python3 - <<'PY'
import json, sys
sys.path.insert(0, "tools")
from pmc_kernels import per_kernel
out = {}
for m in ("tgpu32", "cpu32"):
    d = f"gpurun_out/rp_{m}_occ"
    out[m] = {c: per_kernel(d, c) for c in ("SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
                                             "GRBM_GUI_ACTIVE")}
json.dump(out, open("gpurun_out/round_occ_n32.json", "w"), indent=1)
print(json.dumps(out)[:3000])
PY
