# round 3 (final): validation of the round's tree -- smoke, all GPU tests, the default
# bench (every sub-line), rocprofv3 kernel stats of the default bench, headline PMC
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=smoke,pytest,bench,prof,pmc BENCH_ARGS="" bash scripts/gpu_round.sh || exit $?
