set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_chain.py tests/test_gpu_surface.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_chain.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_chain.log
if [ $rc -eq 0 ]; then timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench2.json 2> gpurun_out/bench2.err; rc=$?; cat gpurun_out/bench2.json | head -c 1500; fi
exit $rc
