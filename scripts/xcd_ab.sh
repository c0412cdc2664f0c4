#!/bin/bash
# A/B of the XCD-grouped set order (RSM_BS_XCD: bit 0 row pass, bit 1 column pass)
# for the production mode and the no-arithmetic diagnostic mode.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
RSM_BS_XCD=3 CHECK=1 timeout -k 10 60 python3 scripts/run_extend.py 20 16 3 > /tmp/o.txt 2>&1 || { cat /tmp/o.txt; exit 3; }
echo "xcd=3 check: $(cat /tmp/o.txt)"
for m in ${MODES:-40 2}; do
  for x in 0 3; do
    for ph in 1 2 3; do
      RSM_BS_MODE=$m RSM_BS_XCD=$x timeout -k 10 60 python3 scripts/run_extend.py 40 16 $ph > /tmp/o.txt 2>&1 || { cat /tmp/o.txt; exit 3; }
      echo "mode=$m xcd=$x $(cat /tmp/o.txt)"
    done
  done
done
