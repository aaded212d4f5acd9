#!/bin/bash
# The one-launch round A/B (tools/exp_round3.py): one process per form, the
# forms alternated twice on one box -> gpurun_out/exp_round3.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/exp_round3.jsonl
: > $out
for pass in 1 2; do
  FA_EXP_ROUND=two timeout -k 10 240 python3 tools/exp_round3.py two "$@" >> $out || exit 1
  timeout -k 10 240 python3 tools/exp_round3.py default "$@" >> $out || exit 1
  FA_EXP_ROUND=one timeout -k 10 240 python3 tools/exp_round3.py one "$@" >> $out || exit 1
  FA_EXP_ROUND=one FA_EXP_ROUND_NBC=split timeout -k 10 240 python3 tools/exp_round3.py one_split "$@" >> $out || exit 1
done
