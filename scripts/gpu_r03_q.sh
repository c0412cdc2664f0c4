# round 3 (q): re-entry validation of HEAD: smoke, GPU parity tests, default bench, power probe
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=smoke,pytest,bench bash scripts/gpu_round.sh || exit $?
timeout -k 10 300 python3 -u scripts/diag/power_probe.py 3000 > gpurun_out/power_r03q.jsonl 2>&1 || exit 9
