#!/bin/bash
# Experiment record (r06): the default order from 64 clients — the 1024-float
# table (r02's tools/tune.py rule, unweighted N >= 64) against the 2048-float
# table with the client loop (the shipped rule for 64..128), and past the
# inline pointers (N > 128) the 1024-float table against the 2048-float one
# (altoff: -DFA_ALT_MIN_N=1000000).  base = the r06 build before the change;
# variants by tools/lib_variant.sh, not kept.  Same process, bits compared.
#   bash tools/archive/n64_ab.sh CASES VARIANT...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
C=$1; shift
out=gpurun_out/n64_ab.jsonl
for v in "$@"; do
  AB_SLAB=1 timeout -k 10 500 python3 -u tools/ab_lib.py feddct_amd/libfedagg.so tools/libfedagg_$v.so 5 $C \
    | sed "s/^{/{\"variant\": \"$v\", /" >> $out || exit 1
done
cat $out
