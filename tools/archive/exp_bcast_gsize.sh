set -o pipefail
# Experiment record (r05): needs an experiment build of libfedagg.so that reads
# FA_EXP_BCAST_GSIZE in launch_bcast (tools/libfedagg_bcast_exp.so, not kept);
# results in profiles/r05_ab_lib_bcast_group_size.jsonl
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for g in 1 2 4 8 24; do
  FA_EXP_BCAST_GSIZE=$g AB_SLAB=1 AB_FLAGS=1 timeout -k 10 200 python -u tools/ab_lib.py feddct_amd/libfedagg.so tools/libfedagg_bcast_exp.so 7 cfg2,cfg3 | sed "s/^{/{\"gmax\": $g, /" >> gpurun_out/ab_bcast_g.jsonl || exit 1
done
