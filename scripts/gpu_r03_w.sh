# round 3 (w): single square -- the one-launch form with replicated done flags and wave
# priorities (rows / Q1 columns high, Q0 columns low) against the two launches; c2 with
# one stream at grid 256 / 224 / 192 (fewer active CUs under the power cap)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u scripts/diag/single_ab.py > gpurun_out/single_r03w.jsonl 2>&1 || exit 2
QAB_STEPS=60 timeout -k 10 400 python3 -u scripts/diag/queue_ab.py queue,256,1,2,40,0 queue,256,1,2,40,224 queue,256,1,2,40,192 queue,256,1,2,40,0 queue,256,1,2,40,192 > gpurun_out/qab_r03w.jsonl 2>&1 || exit 3
