#!/bin/bash
# r04 o: decode sweep A/B (scripts/diag/dec_ab.py; KS picks k)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN:-r04o}; mkdir -p $OUT
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n" >> $OUT/steps.log; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc" >> $OUT/steps.log; tail -n 20 $OUT/$n.log; return $rc; }
DECAB_KS=${KS:-512} step dec 300 python3 scripts/diag/dec_ab.py || exit 3
