# round 3 (t): fixed per-lane set offsets (GEO) in the production c2 kernel -- GPU parity
# (all GPU tests), same-box A/B against the divided form (diag 54000), headline bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_r03t.log 2>&1 || exit 2
QAB_STEPS=60 timeout -k 10 300 python3 -u scripts/diag/queue_ab.py queue,256,3,2,40 queue,256,3,2,54000 queue,256,3,2,40 queue,256,3,2,54000 queue,256,3,2,40 > gpurun_out/qab_r03t.jsonl 2>&1 || exit 3
timeout -k 10 300 python3 bench.py --headline-only --steps 100 --warmup 10 > gpurun_out/bench_head_r03t.log 2>&1 || exit 4
