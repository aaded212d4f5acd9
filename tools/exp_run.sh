mkdir -p gpurun_out
V="def=0: b16=2048:BATCH16 b8=2048:BATCH8 u1b16=1024:BATCH16 def2=0:"
timeout -k 10 200 python3 tools/exp_flags.py wrn16_8_c10 20 11 w -- $V > gpurun_out/exp_w_20.jsonl 2>&1 && \
timeout -k 10 200 python3 tools/exp_flags.py wrn16_8_c100 20 11 w -- $V > gpurun_out/exp_w_c100.jsonl 2>&1 && \
timeout -k 10 200 python3 tools/exp_flags.py wrnsl16_8_sf4_c10_proxy 5 11 -- $V > gpurun_out/exp_w_5.jsonl 2>&1 && \
timeout -k 10 200 python3 tools/exp_flags.py wrnsl16_8_sf4_c10_proxy 5 11 w -- $V > gpurun_out/exp_w_5w.jsonl 2>&1
rc=$?; cat gpurun_out/exp_w_*.jsonl | grep variant; exit $rc
