#!/bin/bash
# Round-2 GPU session: smoke, the whole -m gpu suite, the N=1 bench line, and
# a two-rank gloo rehearsal of the N>1 bench path on the box's one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
&& timeout -k 10 120 ./tools/copylab > gpurun_out/copylab.jsonl 2>&1 \
&& timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
&& timeout -k 10 420 python3 bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err \
&& FA_BENCH_STACK_DUMP_S=150 timeout -k 10 400 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --same-device --steps 3 --warmup 1 > gpurun_out/bench_n2_rehearsal.json 2> gpurun_out/bench_n2_rehearsal.err
rc=$?
echo "exit=$rc"
tail -3 gpurun_out/smoke.log
sort gpurun_out/copylab.jsonl | tail -12
tail -3 gpurun_out/pytest_gpu.log
head -c 600 gpurun_out/bench_n1.json
exit $rc
