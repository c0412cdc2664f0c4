mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_runtime.py -k "single_launch" > gpurun_out/pytest_r03e.log 2>&1 || { echo "queue tests failed"; exit 1; }
QAB_STEPS=40 timeout -k 10 400 python3 -u scripts/diag/queue_ab.py queue,256,3,2,18472 queue,256,3,2,40 queue,256,3,2,51001 queue,256,3,2,51000 queue,256,3,2,50004 queue,256,3,2,50772 queue,256,3,2,40 queue,256,3,2,18472 > gpurun_out/qab_r03e.jsonl 2>&1
