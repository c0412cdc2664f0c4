#!/bin/bash
# r04 t: kernel stats of the GF(2^16) decode sweeps (k = 512 / 256, both forms)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04t; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n" >> $OUT/steps.log; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc" >> $OUT/steps.log; tail -n 12 $OUT/$n.log; return $rc; }
DECAB_KS=512,256 step prof 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o dec --output-format csv -- python3 scripts/diag/dec_ab.py || exit 3
