# round 3 (y): zero-copy Codec Encode / Decode (k = 65..128) -- codec tests and the codec
# / fraud-proof bench lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_codec.py tests/test_gpu_runtime.py tests/test_gpu_eds.py -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_r03y.log 2>&1 || exit 2
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_r03y.log 2>&1 || exit 4
