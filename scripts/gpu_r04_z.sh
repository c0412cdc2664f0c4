#!/bin/bash
# r04 z: GF(2^16) decoder parity + decode sweep A/B + phase trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN:-r04z}; mkdir -p $OUT
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n" >> $OUT/steps.log; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc" >> $OUT/steps.log; tail -n 12 $OUT/$n.log; return $rc; }
step tests 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gf16.py tests/test_gpu_gf16_large.py tests/test_gpu_eds.py || exit 3
DECAB_KS=512,256 step dec 300 python3 scripts/diag/dec_ab.py || exit 3
step trace 200 python3 scripts/diag/trace_dec16.py || exit 3
