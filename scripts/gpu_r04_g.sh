#!/bin/bash
# r04 g: c2 wave-priority A/B (57000) and batch A/B; the N>1 bench path rehearsed at world 1
# (torch.distributed + RCCL initialised, the C-ABI clique beside it)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04g; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n" >> $OUT/steps.log; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc" >> $OUT/steps.log; tail -n 8 $OUT/$n.log; return $rc; }
QAB_STEPS=60 step qab 300 python3 scripts/diag/queue_ab.py queue,512,3,2,40 queue,512,3,2,57000 queue,512,3,2,40 queue,512,3,2,57000 queue,768,3,2,40 queue,512,4,2,40 || exit 3
step dist1 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --dist --steps 20 --warmup 3 || exit 4
