#!/bin/bash
# r05 GPU runner: STEPS picks what runs (space-separated):
#   smoke      __graft_entry__.smoke()
#   large      tests/test_gpu_large.py (the 2 GiB+ squares and the wide forms)
#   tests      every -m gpu test
#   bench      the default bench.py line
#   headline   rocprofv3 stats of the headline launch
#   pmc        FETCH_SIZE / WRITE_SIZE passes of the headline launch
# RUN names the output directory under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN:-r05}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n" >> $OUT/steps.log; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc" >> $OUT/steps.log; tail -n 4 $OUT/$n.log; return $rc; }
for s in ${STEPS:-smoke tests}; do
  case $s in
    smoke) step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 3 ;;
    large) step large 900 python3 -u -m pytest tests/test_gpu_large.py -m gpu -v -x --timeout 300 --timeout-method thread || exit 4 ;;
    tests) step pytest_gpu 1000 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread || exit 5 ;;
    bench) step bench 700 python3 bench.py || exit 6 ;;
    headline) step prof 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/prof" -o run --output-format csv -- python3 bench.py --headline-only --steps 50 || exit 7 ;;
    pmc) step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$PWD/$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py --headline-only --steps 3 --warmup 1 || exit 8
         step pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d "$PWD/$OUT/pmc_write" -o run --output-format csv -- python3 bench.py --headline-only --steps 3 --warmup 1 || exit 9
         python3 scripts/pmc_summary.py $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_latest.json > $OUT/pmc_summary.log 2>&1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
