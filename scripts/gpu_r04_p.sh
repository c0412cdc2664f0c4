#!/bin/bash
# r04 p: c4 encoder, two workgroups per CU (forms 10-13) against the production 16-wave form
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN:-r04p}; mkdir -p $OUT
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n" >> $OUT/steps.log; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc" >> $OUT/steps.log; tail -n 20 $OUT/$n.log; return $rc; }
GF16AB_FORMS=${FORMS:-0} GF16AB_REPS=${REPS:-1} GF16AB_C4FORMS=${C4F:-0,14,15} step enc 240 python3 scripts/diag/gf16_ab.py || exit 3
