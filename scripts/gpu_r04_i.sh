#!/bin/bash
# r04 i: which piece of the HX encoder form breaks parity (0 = HX full, 2 = round-3 form, 3 = half exchange only, 4 = + LDS tables)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04i; mkdir -p $OUT
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n" >> $OUT/steps.log; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc" >> $OUT/steps.log; tail -n 12 $OUT/$n.log; return $rc; }
step enc 180 python3 scripts/diag/gf16_ab.py || exit 3
