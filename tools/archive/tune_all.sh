#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for args in "wrn16_8_c10 20 7" "wrn16_8_c10 20 7 w" "wrnsl16_8_sf4_c10_proxy 5 7" "wrn16_8_c10 2 7" "wrnsl16_8_sf4_c100_proxy 24 5" "wrn16_8_c10 100 3"; do
  timeout -k 10 300 python3 tools/tune.py $args >> gpurun_out/tune_all.jsonl 2>> gpurun_out/tune_all.err || exit 1
done
