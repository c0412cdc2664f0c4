#!/bin/bash
# r04 c: the default bench (all sub-lines: c_abi multi-GPU at world 1, GF(2^16) k=256 x 512 B, affinity CPU baseline)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04c; mkdir -p $OUT
timeout -k 10 900 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?
tail -c 3000 $OUT/bench.err; exit $rc
