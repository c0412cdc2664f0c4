#!/bin/bash
# A/B of the M = 128 encode kernel: correctness of both passes vs the oracle, then
# row / column / whole-step timing, for RSM_BS_MODE (0 production, 2 no
# arithmetic, 4 no global memory -- diagnostics, wrong output; 8 production) x RSM_BS_REV.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
# CONFIGS: MODE_REV tokens
for cfg in ${CONFIGS:-8_1 0_1 2_1 4_1}; do
  m=${cfg%_*}; r=${cfg#*_}
  if [ "$m" = 0 ] || [ "$m" = 8 ]; then
    RSM_BS_MODE=$m RSM_BS_REV=$r CHECK=1 timeout -k 10 60 python3 scripts/run_extend.py 20 16 3 > /tmp/o.txt 2>&1 || { cat /tmp/o.txt; exit 3; }
    echo "mode=$m rev=$r $(cat /tmp/o.txt)"
  fi
  for ph in 1 2 3; do
    for b in ${BATCHES:-16 64}; do
      RSM_BS_MODE=$m RSM_BS_REV=$r timeout -k 10 60 python3 scripts/run_extend.py 30 $b $ph > /tmp/o.txt 2>&1 || { cat /tmp/o.txt; exit 3; }
      echo "mode=$m rev=$r $(cat /tmp/o.txt)"
    done
  done
done
