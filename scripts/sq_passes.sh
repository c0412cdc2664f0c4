#!/bin/bash
# SQ counter passes over scripts/run_extend.py (column pass, batch 16), one rocprofv3 run each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
PH=${PHASE:-2}
timeout -k 10 120 python3 scripts/run_extend.py 20 16 $PH > $OUT/plain.log 2>&1 || exit 3
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU" \
         "SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA" \
         "${EXTRA_PMC:-SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d "$PWD/$OUT/pmc_sq$i" -o run --output-format csv -- python3 scripts/run_extend.py 5 16 $PH > $OUT/pmc_sq$i.log 2>&1 || exit 4
done
exit 0
