# round 3 (k): decoder presence-first loads (trace), latency-form A/B and batch crossover
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_codec.py tests/test_gpu_eds.py tests/test_gpu_runtime.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_r03k.log 2>&1 || exit 1
timeout -k 10 120 python3 -u scripts/diag/trace_decode.py > gpurun_out/trace_dec_r03k.jsonl 2>&1 || exit 2
timeout -k 10 300 python3 -u scripts/diag/single_ab.py > gpurun_out/single_r03k.jsonl 2>&1 || exit 3
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_single" -o run --output-format csv -- python3 scripts/diag/single_ab.py > /dev/null 2>&1 || exit 4
