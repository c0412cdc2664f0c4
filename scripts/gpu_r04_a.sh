#!/bin/bash
# r04 a: cross-lane issue costs (permlane swaps, DPP) + L2 hit rate of the production c2 launch
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04a; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/diag/xlaneprobe 2048 > $OUT/xlane.jsonl 2>&1 || exit 3
cat $OUT/xlane.jsonl
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$PWD/$OUT/pmc_tcc" -o run --output-format csv -- \
    python3 bench.py --headline-only --steps 3 --warmup 1 > $OUT/pmc_tcc.log 2>&1 || exit 4
tail -2 $OUT/pmc_tcc.log
