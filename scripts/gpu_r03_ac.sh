# round 3 (ac): batched device NMT roots -- NMT / roots / EDS GPU tests and the bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_nmt.py tests/test_gpu_roots.py tests/test_gpu_eds.py -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_r03ac.log 2>&1 || exit 2
timeout -k 10 600 python3 bench.py --steps 50 --warmup 5 > gpurun_out/bench_r03ac.log 2>&1 || exit 4
