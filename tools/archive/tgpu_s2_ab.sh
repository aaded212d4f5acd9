#!/bin/bash
# Experiment record (r06): the torch-GPU order's S = 2
# launch (N >= 32) against another libfedagg.so build, same process, bits
# compared, the default order at the same N beside it.  Variants were built by
# tools/lib_variant.sh (depth 2 / 3: -DFA_TGPU_LOOP_DEPTH; nobal: the S = 2
# tail halving off) or kept from the r05 planner (base); the variants are not
# kept.  Results: profiles/r06_ab_lib_tgpu_runs.jsonl.
#   bash tools/archive/tgpu_s2_ab.sh base [nobal ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
C=c10_n32_tgpu,c10_n48_tgpu,c10_n64_tgpu,c100_n64_tgpu,c10_n100_tgpu,c100_n128_tgpu,cfg2_tgpu,cfg5_tgpu,c10_n32,c10_n48,c10_n64,c10_n100
out=gpurun_out/tgpu_s2_ab.jsonl
: > $out
for v in "$@"; do
  AB_SLAB=1 timeout -k 10 400 python3 -u tools/ab_lib.py feddct_amd/libfedagg.so tools/libfedagg_$v.so 5 $C \
    | sed "s/^{/{\"variant\": \"$v\", /" >> $out || exit 1
done
cat $out
