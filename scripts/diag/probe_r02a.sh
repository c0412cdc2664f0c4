#!/bin/bash
# Round-2 diagnostics: (1) HBM rate of the extension's access patterns with no
# arithmetic (memprobe), (2) instruction-cache counters of the production column pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r02a
mkdir -p $OUT
export TMPDIR=/tmp
P=scripts/diag/memprobe
M=16777216
run() { timeout -k 5 60 "$@" >> $OUT/memprobe.jsonl 2>>$OUT/memprobe.err; local rc=$?; [ $rc -le 2 ] || exit 3; }
for J in 16 8; do
for mode in 0 2 6 1 3 8 10 16 20; do
  for wg in 1 2; do
    [ $J = 16 ] && [ $wg = 2 ] && [ $mode -lt 16 ] && continue
    run $P copy   2048 2048   0      262144 64 $M 1024 0 $mode $wg 32 $J
    run $P col    2048 131072 0      2048   64 $M 1024 0 $mode $wg 32 $J
    run $P row    512  512    131072 524288 32 65536 1024 0 $mode $wg 32 $J
  done
done
done
run $P col_o1   2048 131072 0      2048   64 $M 1024 1 2 1
run $P colpad2k 2048 133120 0      2048   64 17825792 1024 0 2 1 36
run $P colpad256 2048 131328 0     2048   64 17825792 1024 0 2 1 36
run $P colbase36 2048 131072 0     2048   64 17825792 1024 0 2 1 36
echo memprobe done
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
grep -i -E "ICACHE|IFETCH|SQC_" $OUT/counters.txt | head -80 > $OUT/counters_sqc.txt || true
timeout -k 10 120 python3 scripts/run_extend.py 10 16 2 > $OUT/plain.log 2>&1 || exit 4
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -d "$PWD/$OUT/pmc_ic" -o run --output-format csv -- python3 scripts/run_extend.py 5 16 2 > $OUT/pmc_ic.log 2>&1 || echo "icache pmc failed rc=$?"
exit 0
