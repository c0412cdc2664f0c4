#!/bin/bash
# Group-size A/B of the production two-launch schedule: smaller batches per step (row
# pass then column pass of the same few squares, so the column pass can re-read Q0/Q1
# from the Infinity Cache), rotating over >= 1 GiB of EDS buffers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r02b
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline --no-c3 --no-c5 --no-roots --steps 60 --warmup 5"
run() { echo "== $*" >> $OUT/grp.log; timeout -k 10 120 $B "$@" >> $OUT/grp.log 2>&1 || exit 3; }
run --batch 16 --buffers 2
run --batch 8 --buffers 4
run --batch 8 --buffers 4 --row-grid 0
run --batch 4 --buffers 8
run --batch 4 --buffers 8 --row-grid 0
run --batch 4 --buffers 8 --streams 3 --row-grid 0
run --batch 4 --buffers 8 --streams 4 --row-grid 0
run --batch 2 --buffers 16 --streams 4 --row-grid 0
run --batch 8 --buffers 4 --streams 3 --row-grid 0
run --batch 16 --buffers 2 --one-stream
run --batch 4 --buffers 8 --one-stream
exit 0
