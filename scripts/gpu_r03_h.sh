mkdir -p gpurun_out
QAB_STEPS=40 timeout -k 10 300 python3 -u scripts/diag/queue_ab.py queue,256,3,2,40 queue,256,3,2,51020 queue,256,3,2,18472 queue,256,3,2,51020 queue,256,3,2,40 > gpurun_out/qab_r03h.jsonl 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/diag/trace_phases.py 51030 > gpurun_out/trace_r03h.jsonl 2>&1
