mkdir -p gpurun_out
V="def=0: st_nt=2048:BATCH16 st_sc1nt=2048:BATCH16|ST_SC1 st_sc1=2048:BATCH16|ST_SC1|ST_PLAIN st_nt_b=2048:BATCH16 st_sc1_b=2048:BATCH16|ST_SC1|ST_PLAIN"
timeout -k 10 200 python3 tools/exp_flags.py wrn16_8_c10 20 9 -- $V > gpurun_out/exp_sc1_20.jsonl 2>&1 && \
timeout -k 10 200 python3 tools/exp_flags.py wrnsl16_8_sf4_c10_proxy 5 9 -- $V > gpurun_out/exp_sc1_5.jsonl 2>&1
rc=$?; cat gpurun_out/exp_sc1_*.jsonl; exit $rc
