# round 3 (z): instruction-cache behaviour of the c2 kernel -- list the gfx950 counters,
# then one PMC pass with the SQC instruction-cache counters over a short headline bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_r03z.txt 2>&1 || true
grep -i -E "icache|SQC_|INST_LEVEL|WAIT_INST|IFETCH" gpurun_out/counters_r03z.txt | head -60 > gpurun_out/counters_icache_r03z.txt || true
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -d "$PWD/gpurun_out/pmc_ic" -o run --output-format csv -- python3 bench.py --headline-only --steps 3 --warmup 1 > gpurun_out/pmc_ic_r03z.log 2>&1 || exit 3
