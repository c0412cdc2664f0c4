#!/bin/bash
# r04 y: phase timeline of the m = 512 half-wave GF(2^16) decoder
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN:-r04y}; mkdir -p $OUT
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n" >> $OUT/steps.log; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc" >> $OUT/steps.log; tail -n 12 $OUT/$n.log; return $rc; }
step trace 200 python3 scripts/diag/trace_dec16.py || exit 3
