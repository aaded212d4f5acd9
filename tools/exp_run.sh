mkdir -p gpurun_out
V="def=0: park8=2048:PARK|BATCH8 park16=2048:PARK|BATCH16 def2=0: park8b=2048:PARK|BATCH8"
timeout -k 10 200 python3 tools/exp_flags.py wrn16_8_c10 20 9 -- $V > gpurun_out/exp_park_20.jsonl 2>&1 && \
timeout -k 10 200 python3 tools/exp_flags.py wrnsl16_8_sf4_c10_proxy 5 9 -- $V > gpurun_out/exp_park_5.jsonl 2>&1
rc=$?; cat gpurun_out/exp_park_*.jsonl | grep variant; exit $rc
