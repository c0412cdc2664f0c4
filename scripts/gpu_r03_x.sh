# round 3 (x): validation of the round's tree -- smoke, all GPU tests, the default bench
# (every sub-line), rocprofv3 kernel stats of the default bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=smoke,pytest,bench,prof bash scripts/gpu_round.sh || exit $?
