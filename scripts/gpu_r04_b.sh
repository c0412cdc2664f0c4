#!/bin/bash
# r04 b: cross-lane issue costs; GF(2^16) m=256 prefetch A/B; GPU tests touched this round
# (multi-GPU C ABI incl. the pinned in-place form, GF(2^16) encode); L2 hit rate of c2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04b; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n" >> $OUT/steps.log; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc" >> $OUT/steps.log; tail -n 4 $OUT/$n.log; return $rc; }
step xlane 120 ./scripts/diag/xlaneprobe 2048 || exit 3
step gf16_pf 300 python3 scripts/diag/gf16_pf_ab.py || exit 4
step tests 600 python3 -u -m pytest tests/test_gpu_runtime.py tests/test_gpu_gf16.py -x -q --timeout 300 --timeout-method thread || exit 5
step pmc_tcc 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$PWD/$OUT/pmc_tcc" -o run --output-format csv -- python3 bench.py --headline-only --steps 3 --warmup 1 || exit 6
