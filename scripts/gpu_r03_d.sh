mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_runtime.py -k "single_launch" > gpurun_out/pytest_r03b.log 2>&1 || { echo "queue tests failed"; exit 1; }
QAB_STEPS=40 timeout -k 10 300 python3 -u scripts/diag/queue_ab.py queue,256,3,2,18472 queue,256,3,2,40 queue,256,3,2,50002 queue,256,3,2,50004 queue,256,3,2,50768 queue,256,3,2,50772 > gpurun_out/qab_r03b.jsonl 2>&1 || exit 2
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_runtime.py tests/test_gpu_eds.py tests/test_gpu_nmt.py > gpurun_out/pytest_r03c.log 2>&1
