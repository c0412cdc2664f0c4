#!/bin/bash
# final tree: headline kernel trace + PMC of the production queue kernel (<16777216>)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_head_fin" -o run --output-format csv -- python3 bench.py --headline-only --steps 50 --warmup 5 > gpurun_out/bench_head_fin.log 2>&1 || exit 2
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d "$PWD/gpurun_out/pmc_head_f_fin" -o run --output-format csv -- python3 bench.py --headline-only --steps 3 --warmup 1 > /dev/null 2>&1 || exit 3
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d "$PWD/gpurun_out/pmc_head_w_fin" -o run --output-format csv -- python3 bench.py --headline-only --steps 3 --warmup 1 > /dev/null 2>&1 || exit 4
