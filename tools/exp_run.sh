mkdir -p gpurun_out
V="def=0: u2b1=2048:BATCH1 u2b4=2048:BATCH4 u2b16=2048:BATCH16 u4b1=4096:BATCH1 u4b4=4096:BATCH4 u4b8=4096:BATCH8 u1b1=1024:BATCH1 u1b4=1024:BATCH4 u1b16=1024:BATCH16"
timeout -k 10 250 python3 tools/exp_flags.py wrn16_8_c10 20 11 -- $V > gpurun_out/exp_u_20.jsonl 2>&1
rc=$?; cat gpurun_out/exp_u_*.jsonl | grep variant; exit $rc
