mkdir -p gpurun_out
V="def=0: b1=2048:BATCH1 b4=2048:BATCH4 b8=2048:BATCH8 b16=2048:BATCH16 u1b1=1024:BATCH1 u1b4=1024:BATCH4"
timeout -k 10 200 python3 tools/exp_flags.py wrn16_8_c10 20 11 -- $V > gpurun_out/exp_b_20.jsonl 2>&1 && \
timeout -k 10 200 python3 tools/exp_ab.py tools/libfedagg_D.so wrn16_8_c10 20 15 > gpurun_out/exp_b_ab.jsonl 2>&1 && \
timeout -k 10 200 python3 tools/exp_flags.py wrnsl16_8_sf4_c10_proxy 5 11 -- $V > gpurun_out/exp_b_5.jsonl 2>&1 && \
timeout -k 10 200 python3 tools/exp_flags.py wrn16_8_c10 20 7 w -- $V > gpurun_out/exp_b_20w.jsonl 2>&1
rc=$?; cat gpurun_out/exp_b_*.jsonl | grep -E "variant|lib"; exit $rc
