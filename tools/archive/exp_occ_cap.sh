# Experiment record (r05): the 8-client kernels (N < 16) capped at fewer
# resident workgroups per CU by a dynamic LDS reservation (the experiment
# build reads FA_EXP_RED_LDS); results in profiles/r05_ab_lib_occupancy_cap.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
python3 -c "import torch; p=torch.cuda.get_device_properties(0); print({k: getattr(p, k) for k in dir(p) if 'shared' in k or 'multi' in k})" > gpurun_out/occ_dev.txt 2>&1
C=${CASES:-cfg3,sf32,c10_n2,c10_n8,c10_n12,cfg3w,sf16,cfg3_tgpu,sf32_tgpu,c10_n10_tgpu}
run() { tag=$1; shift; env "$@" AB_SLAB=1 timeout -k 10 300 python -u tools/ab_lib.py tools/libfedagg_before_tgpu_w2.so feddct_amd/libfedagg.so 5 $C | sed "s/^{/{\"exp_cfg\": \"$tag\", /" >> gpurun_out/ab_occ.jsonl; }
run none FA_EXP_NONE=1 || exit 1
run lds40k FA_EXP_RED_LDS=40960 || exit 1
run lds48k FA_EXP_RED_LDS=49152 || exit 1
