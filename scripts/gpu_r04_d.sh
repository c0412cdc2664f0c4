#!/bin/bash
# r04 d: single-pass GF(2^16) decoder A/B + GF(2^16) tests; per-use symbol offsets (40) vs hoisted (56000); XCD-affine queue variant of the c2 launch (diagnostic 55000: per-XCD queues, Q1 stored
# with the default policy) against production (40): every square checked, timing, memory-only
# (no arithmetic) forms, socket power, L2 hit rate
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04d; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n" >> $OUT/steps.log; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc" >> $OUT/steps.log; tail -n 12 $OUT/$n.log; return $rc; }
step dec 240 python3 scripts/diag/dec_ab.py || exit 7
step dectests 600 python3 -u -m pytest tests/test_gpu_gf16.py tests/test_gpu_gf16_large.py tests/test_gpu_eds.py tests/test_gpu_codec.py -x -q --timeout 300 --timeout-method thread || exit 8
QAB_CHECK_ALL=1 QAB_STEPS=60 step qab 300 python3 scripts/diag/queue_ab.py queue,256,3,2,40 queue,256,3,2,56000 queue,256,3,2,55000 queue,256,3,2,40 queue,256,3,2,56000 queue,256,3,2,55000 queue,256,3,0,55000 queue,256,3,0,40 queue,256,3,2,55002 queue,256,3,2,50002 queue,512,3,2,40 queue,256,3,2,40 queue,512,2,2,40 || exit 3
step power 500 python3 scripts/diag/power_probe.py 3000 40:3000:2 56000:3000:2 55000:3000:2 55002:4000:2 50002:4000:2 || exit 4
QAB_STEPS=3 step pmc40 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$PWD/$OUT/pmc40" -o run --output-format csv -- python3 scripts/diag/queue_ab.py queue,256,3,2,40 || exit 5
QAB_STEPS=3 step pmc55 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$PWD/$OUT/pmc55" -o run --output-format csv -- python3 scripts/diag/queue_ab.py queue,256,3,2,55000 || exit 6
