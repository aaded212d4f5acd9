#!/bin/bash
# One GPU-box session made of named steps, run in the order given:
#
#   bash tools/gpu_session.sh smoke tests bench profile ...
#
# Steps (each GPU step has its own time limit; the first failure ends the
# call, and nothing else touches the GPU after it):
#   smoke             __graft_entry__.smoke()
#   tests             pytest -m gpu over tests/ (the driver's round-end tier)
#   tests=<args>      pytest -m gpu with <args> (commas -> spaces), e.g.
#                     tests=tests/test_gpu_sweep.py,-k,digest
#   bench             bench.py (N=1 defaults)           -> gpurun_out/bench_n1.json
#   driver=<tag>      the driver's N=1 command           -> gpurun_out/driver_like_<tag>.json
#   profile           kernel trace + FETCH/WRITE passes of the headline (gpu_profile.sh)
#   round_pmc         the same for the round and the torch-GPU-order reduce
#   prof=<tool>[:arg] kernel trace of python3 tools/<tool>.py <arg>
#   run=<tool>[:args] python3 tools/<tool>.py <args> (commas -> spaces) -> gpurun_out/<tool>.jsonl
#   multi             bench.py's N>1 path over RCCL with one rank (multi_rehearsal.sh)
#   n2                two-rank gloo rehearsal of bench.py --gpus 2 on one GPU
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"

step() {
  local s="$1" arg="${1#*=}"
  case "$s" in
    smoke) timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" \
             > gpurun_out/smoke.log 2>&1 ;;
    tests) timeout -k 10 1500 $PYT tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 ;;
    tests=*) timeout -k 10 900 $PYT -m gpu ${arg//,/ } > gpurun_out/pytest_part.log 2>&1 ;;
    bench) timeout -k 10 420 python3 bench.py > gpurun_out/bench_n1.json \
             2> gpurun_out/bench_n1.err ;;
    driver=*) bash tools/driver_like.sh "$arg" ;;
    profile) bash tools/gpu_profile.sh > gpurun_out/profile.log 2>&1 ;;
    round_pmc) bash tools/gpu_round_pmc.sh > gpurun_out/round_pmc.log 2>&1 ;;
    prof=*) local t="${arg%%:*}" a=""; [[ "$arg" == *:* ]] && a="${arg#*:}"
            timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "gpurun_out/prof_$t" \
              -o run -- python3 "tools/$t.py" $a > "gpurun_out/prof_$t.jsonl" \
              2> "gpurun_out/prof_$t.err" ;;
    run=*) local t="${arg%%:*}" a=""; [[ "$arg" == *:* ]] && a="${arg#*:}"
           timeout -k 10 600 python3 "tools/$t.py" ${a//,/ } > "gpurun_out/$t.jsonl" \
             2> "gpurun_out/$t.err" ;;
    multi) bash tools/multi_rehearsal.sh > gpurun_out/multi_rehearsal.log 2>&1 ;;
    n2) FA_BENCH_STACK_DUMP_S=150 timeout -k 10 500 python3 -m torch.distributed.run \
          --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py \
          --gpus 2 --dist-backend gloo --same-device --steps 3 --warmup 1 \
          > gpurun_out/bench_n2_rehearsal.json 2> gpurun_out/bench_n2_rehearsal.err ;;
    *) echo "unknown step $s" >&2; return 2 ;;
  esac
}

rc=0
for s in "$@"; do
  echo "== $s ($(date +%T))"
  step "$s" || { rc=$?; echo "step $s failed: exit $rc"; break; }
done
echo "exit=$rc"
for f in smoke.log pytest_gpu.log pytest_part.log; do
  [ -f "gpurun_out/$f" ] && { echo "-- $f"; tail -3 "gpurun_out/$f"; }
done
[ -f gpurun_out/bench_n1.json ] && head -c 600 gpurun_out/bench_n1.json
exit $rc
