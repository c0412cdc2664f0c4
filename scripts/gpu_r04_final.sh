#!/bin/bash
# r04 final: A) smoke + every GPU test; B) headline PMC passes, the default bench, the
# headline kernel trace/stats.  PART=A|B picks the half (one gpurun call each).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN:-r04final}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n" >> $OUT/steps.log; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc" >> $OUT/steps.log; tail -n 3 $OUT/$n.log; return $rc; }
if [ "${PART:-A}" = A ]; then
  step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 3
  step pytest_gpu 900 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread || exit 4
else
  step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$PWD/$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py --headline-only --steps 3 --warmup 1 || exit 5
  step pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d "$PWD/$OUT/pmc_write" -o run --output-format csv -- python3 bench.py --headline-only --steps 3 --warmup 1 || exit 6
  python3 scripts/pmc_summary.py $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_latest.json > $OUT/pmc_summary.log 2>&1
  timeout -k 10 700 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -c 3000 $OUT/bench.err; exit 7; }
  step prof 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/prof" -o run --output-format csv -- python3 bench.py --headline-only --steps 50 || exit 8
fi
