# round 3 (r): rotate-and-select transposes in the production c2 kernel -- GPU parity
# (all GPU tests, incl. the bench-scale queue test), same-box A/B against the shift form
# (diag 53000), default bench, power probe
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r03r.log 2>&1 || exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_r03r.log 2>&1 || exit 2
QAB_STEPS=40 timeout -k 10 300 python3 -u scripts/diag/queue_ab.py queue,256,3,2,40 queue,256,3,2,53000 queue,256,3,2,40 queue,256,3,2,53000 > gpurun_out/qab_r03r.jsonl 2>&1 || exit 3
timeout -k 10 600 python3 bench.py > gpurun_out/bench_r03r.log 2>&1 || exit 4
timeout -k 10 300 python3 -u scripts/diag/power_probe.py 3000 > gpurun_out/power_r03r.jsonl 2>&1 || exit 5
