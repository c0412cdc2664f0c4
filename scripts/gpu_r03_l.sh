# round 3 (l): fused single-square launch, decoder table staging
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_codec.py tests/test_gpu_eds.py tests/test_gpu_runtime.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_r03l.log 2>&1 || exit 1
timeout -k 10 120 python3 -u scripts/diag/trace_decode.py > gpurun_out/trace_dec_r03l.jsonl 2>&1 || exit 2
timeout -k 10 300 python3 -u scripts/diag/single_ab.py > gpurun_out/single_r03l.jsonl 2>&1 || exit 3
timeout -k 10 600 python3 bench.py > gpurun_out/bench_r03l.log 2>&1 || exit 4
