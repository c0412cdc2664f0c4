#!/bin/bash
# icache counters of the small-batch kernels (per-wave twiddle variants)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -d "$PWD/gpurun_out/pmc_ic_small" -o run --output-format csv -- python3 scripts/diag/icache_small.py > gpurun_out/pmc_ic_small_r03ae.log 2>&1 || exit 3
