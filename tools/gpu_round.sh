set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_prox.py tests/test_gpu_parity.py -k prox -x -v --timeout 120 --timeout-method thread > gpurun_out/prox_tests.log 2>&1 \
&& timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/proxprof -o run -- python3 tools/exp_prox_ab.py - 5 > gpurun_out/proxprof.jsonl 2> gpurun_out/proxprof.err \
&& bash tools/gpu_check.sh
rc=$?; tail -3 gpurun_out/prox_tests.log; cat gpurun_out/proxprof.jsonl; exit $rc
