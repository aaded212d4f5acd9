set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats -f csv -d gpurun_out/nrc -o run -- python3 tools/native_round_cost.py 20 --no-graphs --only=plain_reduce,chained_16,blocked > gpurun_out/nrc.jsonl 2> gpurun_out/nrc.err
rc=$?; find gpurun_out/nrc -name "*stats*" | head; exit $rc
