#!/bin/bash
# One gpurun session: smoke -> GPU parity tests -> bench -> rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/abort/timeout (rc > 1) ends the
# script immediately (no further GPU work in this call).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
STEPS=${STEPS:-smoke,pytest,bench,prof}
run() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" >> $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> $OUT/steps.log
  tail -n 3 "$OUT/$name.log"
  return $rc
}
ok() { [ "$1" -le 1 ]; }
if [[ $STEPS == *smoke* ]]; then run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"; ok $? || exit 3; fi
if [[ $STEPS == *pytest* ]]; then run pytest_gpu 1200 python3 -u -m pytest tests -m gpu -q --maxfail=30 --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}; ok $? || exit 4; fi
if [[ $STEPS == *bench* ]]; then run bench 600 python3 bench.py ${BENCH_ARGS:-}; ok $? || exit 5; fi
if [[ $STEPS == *prof* ]]; then
  export TMPDIR=/tmp
  run rocprof 600 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/prof" -o run --output-format csv -- \
      python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ${PROF_ARGS:-} ${BENCH_ARGS:-}; ok $? || exit 6
fi
if [[ $STEPS == *pmc* ]]; then
  export TMPDIR=/tmp
  run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$PWD/$OUT/pmc_fetch" -o run --output-format csv -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-}; ok $? || exit 7
  run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d "$PWD/$OUT/pmc_write" -o run --output-format csv -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-}; ok $? || exit 8
fi
exit 0
