# round 3 (p): GF16 merged pair for m = 256 only; bench with the gate ahead of the warmup
set -u
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_gf16.py tests/test_gpu_gf16_large.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_r03p.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_r03p.log 2>&1 || exit 2
timeout -k 10 200 python3 -u scripts/diag/power_probe.py 3000 > gpurun_out/power_r03p.jsonl 2>&1 || exit 3
