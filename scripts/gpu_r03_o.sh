# round 3 (o): GF16 merged middle pair; headline-only kernel trace + PMC for profiles/
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_gf16.py tests/test_gpu_gf16_large.py tests/test_gpu_eds.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_r03o.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_head" -o run --output-format csv -- python3 bench.py --headline-only --steps 50 --warmup 5 > gpurun_out/bench_head_r03o.log 2>&1 || exit 2
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d "$PWD/gpurun_out/pmc_head_f" -o run --output-format csv -- python3 bench.py --headline-only --steps 3 --warmup 1 > /dev/null 2>&1 || exit 3
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d "$PWD/gpurun_out/pmc_head_w" -o run --output-format csv -- python3 bench.py --headline-only --steps 3 --warmup 1 > /dev/null 2>&1 || exit 4
timeout -k 10 600 python3 bench.py --steps 100 > gpurun_out/bench_r03o.log 2>&1 || exit 5
