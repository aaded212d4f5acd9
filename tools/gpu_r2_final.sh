#!/bin/bash
# Round-2 closing session: smoke, -m gpu, the distance print, bench N=1, the
# headline's kernel trace + PMC passes, kernel stats of the round's
# broadcast and the torch-GPU-order mode, the N>1 path over RCCL with one
# rank, a two-rank gloo rehearsal of N>1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
&& timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
&& timeout -k 10 200 python3 -u -m pytest tests/test_gpu_parity.py -k distance -s -q --timeout 150 --timeout-method thread > gpurun_out/distance.log 2>&1 \
&& timeout -k 10 420 python3 bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err \
&& bash tools/gpu_profile.sh > gpurun_out/profile.log 2>&1 \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_bcast -o run -- python3 tools/exp_bcast.py 1 > gpurun_out/prof_bcast.jsonl 2> gpurun_out/prof_bcast.err \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_tgpu -o run -- python3 tools/tgpu_speed.py 1 > gpurun_out/prof_tgpu.jsonl 2> gpurun_out/prof_tgpu.err \
&& bash tools/multi_rehearsal.sh > gpurun_out/multi_rehearsal.log 2>&1 \
&& FA_BENCH_STACK_DUMP_S=150 timeout -k 10 500 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --same-device --steps 3 --warmup 1 > gpurun_out/bench_n2_rehearsal.json 2> gpurun_out/bench_n2_rehearsal.err
rc=$?
echo "exit=$rc"
tail -2 gpurun_out/smoke.log
tail -2 gpurun_out/pytest_gpu.log
grep "vs torch GPU" gpurun_out/distance.log
head -c 400 gpurun_out/bench_n1.json
exit $rc
