#!/bin/bash
# Narrow a GPU parity failure of the M = 128 kernel: the same tests under kernel
# switches (table kernel / column-order) plus whole-square checks at several batches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for e in RSM_GF8_KERNEL=table RSM_BS_REV=0 RSM_BS_REV=1; do
  i=$((i+1))
  env $e timeout -k 10 120 python3 -m pytest tests/test_gpu_codec.py -q -k "partial_chunks or extend_square_matches or batched or bitsliced" --timeout 60 > gpurun_out/bisect_$i.log 2>&1
  echo "$e pytest rc=$? $(tail -1 gpurun_out/bisect_$i.log)"
done
for r in 0 1; do
  for b in 1 3 16; do
    RSM_BS_REV=$r CHECK=1 timeout -k 10 60 python3 scripts/run_extend.py 3 $b 3 2>&1 | tail -1 | sed "s/^/rev=$r /"
  done
done
