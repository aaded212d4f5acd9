# Experiment record (r05): the torch-GPU-order S = 2 group (N >= 32) as
# 2048-element client-loop tiles with the small groups riding in its launch,
# against the build before it (tools/libfedagg_before_tgpu_w2.so, not kept);
# r1 = S = 1 riders only (tools/libfedagg_tgpu_r1.so, not kept), r14 = S = 1 and S = 4
# riders (the tree's build); results in profiles/r05_ab_lib_tgpu_s2.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
C=c10_n32_tgpu,c10_n48_tgpu,c10_n64_tgpu,c10_n100_tgpu,c10_n127_tgpu,c100_n64_tgpu,c100_n128_tgpu,cfg2_tgpu,cfg3_tgpu,cfg5_tgpu
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_torch_order.py > gpurun_out/w2_final_tests.log 2>&1 || exit 1
AB_SLAB=1 timeout -k 10 500 python -u tools/ab_lib.py tools/libfedagg_before_tgpu_w2.so tools/libfedagg_tgpu_r1.so 5 $C | sed 's/^{/{"build": "r1", /' > gpurun_out/ab_w2_final.jsonl || exit 1
AB_SLAB=1 timeout -k 10 500 python -u tools/ab_lib.py tools/libfedagg_before_tgpu_w2.so feddct_amd/libfedagg.so 5 $C | sed 's/^{/{"build": "r14", /' >> gpurun_out/ab_w2_final.jsonl
