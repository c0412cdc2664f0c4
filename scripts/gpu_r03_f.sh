mkdir -p gpurun_out
timeout -k 10 300 python3 -u scripts/diag/trace_phases.py 51010 51014 51012 > gpurun_out/trace_r03f.jsonl 2>&1 || exit 1
QAB_STEPS=40 timeout -k 10 300 python3 -u scripts/diag/queue_ab.py queue,256,3,2,40 queue,256,3,2,51002 queue,256,3,2,51006 > gpurun_out/qab_r03f.jsonl 2>&1
