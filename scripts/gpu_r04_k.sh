#!/bin/bash
# r04 k: GF(2^16) encoder forms (c5 m=512 and c4 m=256 16-wave form)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04k; mkdir -p $OUT
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n" >> $OUT/steps.log; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc" >> $OUT/steps.log; tail -n 14 $OUT/$n.log; return $rc; }
step enc 240 python3 scripts/diag/gf16_ab.py || exit 3
