# round 3 (s): power/energy decomposition of the c2 kernel (production, no arithmetic,
# no global memory, no LDS exchange, arithmetic only, memory only), headline kernel trace
# and PMC of the new arithmetic
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u scripts/diag/power_probe.py 5000 40:5000 50002:7000 50004:7000 50768:5000 50772:7000 50770:7000 40:5000 > gpurun_out/power_r03s.jsonl 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_head_s" -o run --output-format csv -- python3 bench.py --headline-only --steps 50 --warmup 5 > gpurun_out/bench_head_r03s.log 2>&1 || exit 2
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d "$PWD/gpurun_out/pmc_head_f_s" -o run --output-format csv -- python3 bench.py --headline-only --steps 3 --warmup 1 > /dev/null 2>&1 || exit 3
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d "$PWD/gpurun_out/pmc_head_w_s" -o run --output-format csv -- python3 bench.py --headline-only --steps 3 --warmup 1 > /dev/null 2>&1 || exit 4
