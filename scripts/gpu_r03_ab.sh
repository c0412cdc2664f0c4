# round 3 (ab): bench with the NMT-roots sub-line (extension + Celestia NMT roots)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py --steps 50 --warmup 5 > gpurun_out/bench_r03ab.log 2>&1 || exit 4
