#!/bin/bash
# r04 j: GF(2^16) m=512 forms after the parity-split half exchange: encoder A/B, decoder A/B, GF(2^16) tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04j; mkdir -p $OUT
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n" >> $OUT/steps.log; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc" >> $OUT/steps.log; tail -n 12 $OUT/$n.log; return $rc; }
step enc 180 python3 scripts/diag/gf16_ab.py || exit 3
step dec 180 python3 scripts/diag/dec_ab.py || exit 4
step tests 600 python3 -u -m pytest tests/test_gpu_gf16.py tests/test_gpu_gf16_large.py tests/test_gpu_eds.py tests/test_gpu_runtime.py tests/test_gpu_codec.py -x -q --timeout 300 --timeout-method thread || exit 5
