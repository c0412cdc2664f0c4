#!/bin/bash
# r04 v: SQ counters of the single-pass GF(2^16) decoders (k = 512 half-wave, k = 256)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04v; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n" >> $OUT/steps.log; timeout -s KILL $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc" >> $OUT/steps.log; tail -n 3 $OUT/$n.log; return $rc; }
P1=SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_WAIT_INST_LDS
P2=SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_SMEM,SQ_ACTIVE_INST_LDS,SQ_INSTS_SALU,SQ_WAVES,SQ_INSTS_VMEM
export DECAB_KS=512,256
step p1 120 rocprofv3 --pmc $P1 -d $OUT/p1 -o pmc --output-format csv -- python3 scripts/diag/dec_ab.py || exit 3
step p2 120 rocprofv3 --pmc $P2 -d $OUT/p2 -o pmc --output-format csv -- python3 scripts/diag/dec_ab.py || exit 3
