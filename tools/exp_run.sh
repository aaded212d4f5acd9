mkdir -p gpurun_out
V="def=0: ntnt=2048:BATCH16 stplain=2048:BATCH16|ST_PLAIN ldplain=2048:BATCH16|LD_PLAIN plain=2048:BATCH16|NO_NT u1st=1024:BATCH16|ST_PLAIN u4st=4096:BATCH8|ST_PLAIN"
timeout -k 10 200 python3 tools/exp_flags.py wrn16_8_c10 20 7 -- $V > gpurun_out/exp_pol20.jsonl 2>&1 && \
timeout -k 10 200 python3 tools/exp_flags.py wrn16_8_c10 100 5 -- $V > gpurun_out/exp_pol100.jsonl 2>&1 && \
timeout -k 10 200 python3 tools/exp_flags.py wrn16_8_c10 5 7 -- $V > gpurun_out/exp_pol5.jsonl 2>&1
rc=$?; cat gpurun_out/exp_pol*.jsonl; exit $rc
