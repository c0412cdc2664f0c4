#!/bin/bash
# Profiling session: GF16 batch-cap sweep (c4, c5), new roots test, rocprofv3 kernel
# stats of the default bench, PMC FETCH/WRITE passes, one SQ pass on the column
# kernel, and the kernel-mode A/B.  Every GPU step has its own limit; a crash or
# timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
ok() { [ "$1" -le 1 ]; }
timeout -k 10 120 python3 -m pytest tests/test_gpu_roots.py -q --timeout 60 > $O/roots_test.log 2>&1; ok $? || exit 3
for mb in 1024 256 64; do
  RSM_GF16_BATCH_MB=$mb timeout -k 10 300 python3 bench.py --workload c4 --steps 5 --warmup 1 --no-c3 --no-roots --no-cpu-baseline > $O/c4_$mb.json 2>&1; ok $? || exit 4
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-c3 > $O/rocprof.log 2>&1; ok $? || exit 5
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$PWD/$O/pmc_fetch" -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-c3 --no-c5 --no-roots > $O/pmc_fetch.log 2>&1; ok $? || exit 6
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$PWD/$O/pmc_write" -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-c3 --no-c5 --no-roots > $O/pmc_write.log 2>&1; ok $? || exit 7
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU -d "$PWD/$O/pmc_sq1" -o run --output-format csv -- python3 scripts/run_extend.py 5 16 3 > $O/pmc_sq1.log 2>&1; ok $? || exit 8
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_IFETCH -d "$PWD/$O/pmc_sq2" -o run --output-format csv -- python3 scripts/run_extend.py 5 16 3 > $O/pmc_sq2.log 2>&1; ok $? || exit 9
CONFIGS="0_1 0_0 2_1 4_1" BATCHES=16 bash scripts/ab.sh > $O/ab.txt 2>&1 || exit 10
exit 0
