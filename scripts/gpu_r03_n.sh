# round 3 (n): decoder FWHT on DPP / swizzle / permlane, per-wave table reads
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_codec.py tests/test_gpu_eds.py tests/test_gpu_runtime.py tests/test_gpu_gf16.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_r03n.log 2>&1 || exit 1
timeout -k 10 120 python3 -u scripts/diag/trace_decode.py > gpurun_out/trace_dec_r03n.jsonl 2>&1 || exit 2
timeout -k 10 600 python3 bench.py --no-cpu-baseline > gpurun_out/bench_r03n.log 2>&1 || exit 3
