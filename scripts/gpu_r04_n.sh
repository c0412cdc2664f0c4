#!/bin/bash
# r04 n: SQ counters of the m = 512 GF(2^16) encoder forms 0 (production, spills) and 5 (JIT tables, no scratch)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04n; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n" >> $OUT/steps.log; timeout -s KILL $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc" >> $OUT/steps.log; tail -n 6 $OUT/$n.log; return $rc; }
P1=SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_WAIT_INST_LDS
P2=SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_SMEM,SQ_ACTIVE_INST_LDS,SQ_INSTS_SALU,SQ_WAVES,SQ_ACTIVE_INST_SCA
for f in 0 5; do
  export GF16AB_FORMS=$f GF16AB_REPS=1 GF16AB_C4=0
  step f${f}_p1 90 rocprofv3 --pmc $P1 -d $OUT/f${f}_p1 -o pmc --output-format csv -- python3 scripts/diag/gf16_ab.py || exit 3
  step f${f}_p2 90 rocprofv3 --pmc $P2 -d $OUT/f${f}_p2 -o pmc --output-format csv -- python3 scripts/diag/gf16_ab.py || exit 3
done
