#!/bin/bash
# A/B of encode kernel variants (RSM_BS_VARIANT): correctness (phase 0, CHECK) + row/col timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-0 10}; do
  RSM_BS_VARIANT=$v CHECK=1 timeout -k 10 60 python3 scripts/run_extend.py 20 16 3 > /tmp/o.txt 2>&1 || { cat /tmp/o.txt; exit 3; }
  echo "v=$v $(cat /tmp/o.txt)"
  for ph in 1 2; do
    for b in ${BATCHES:-16 64}; do
      RSM_BS_VARIANT=$v timeout -k 10 60 python3 scripts/run_extend.py 30 $b $ph > /tmp/o.txt 2>&1 || { cat /tmp/o.txt; exit 3; }
      echo "v=$v $(cat /tmp/o.txt)"
    done
  done
done
