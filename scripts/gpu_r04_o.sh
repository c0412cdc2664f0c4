#!/bin/bash
# r04 o: GF(2^8) split decoder, staggered point loads (diagnostic delay sweep)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04o; mkdir -p $OUT
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n" >> $OUT/steps.log; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc" >> $OUT/steps.log; tail -n 20 $OUT/$n.log; return $rc; }
DECAB_KS=128 DECAB_DELAYS=0,100,200,300,400,600 step dec 240 python3 scripts/diag/dec_ab.py || exit 3
