# round 3 (u): phase blocks hold only the SGPR masks they use; queue parity at non-dividing
# share sizes (general per-lane offsets); A/B and headline bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_r03u.log 2>&1 || exit 2
QAB_STEPS=60 timeout -k 10 300 python3 -u scripts/diag/queue_ab.py queue,256,3,2,40 queue,256,3,2,54000 queue,256,3,2,40 queue,256,3,2,54000 > gpurun_out/qab_r03u.jsonl 2>&1 || exit 3
timeout -k 10 300 python3 bench.py --headline-only --steps 100 --warmup 10 > gpurun_out/bench_head_r03u.log 2>&1 || exit 4
