#!/bin/bash
# r04 e: kernel trace of the GF(2^16) decode A/B; every GPU test; smoke
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04e; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n" >> $OUT/steps.log; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc" >> $OUT/steps.log; tail -n 6 $OUT/$n.log; return $rc; }
step dectrace 240 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/dectrace" -o run --output-format csv -- python3 scripts/diag/dec_ab.py || exit 3
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 4
step pytest 1100 python3 -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread || exit 5
