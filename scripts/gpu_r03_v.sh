# round 3 (v): c2 at the power cap -- does a smaller persistent grid (fewer active CUs,
# each at a higher clock) change the time per square?  grid 256 / 224 / 192 / 160 / 128,
# then the GPU runtime tests (grid caps 1 / 7 / 224 reach the queue launch now)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
QAB_STEPS=60 timeout -k 10 400 python3 -u scripts/diag/queue_ab.py queue,256,3,2,40,0 queue,256,3,2,40,224 queue,256,3,2,40,192 queue,256,3,2,40,160 queue,256,3,2,40,128 queue,256,3,2,40,0 queue,256,3,2,40,192 > gpurun_out/qab_r03v.jsonl 2>&1 || exit 3
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_runtime.py -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_r03v.log 2>&1 || exit 2
