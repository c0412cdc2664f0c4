#!/bin/bash
# GF(2^16) decoder: N-point error locator (folded LogWalsh) -- parity + repair_gf16 timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gf16.py tests/test_gpu_gf16_large.py tests/test_gpu_eds.py > gpurun_out/pytest_r03ag.log 2>&1 || exit 3
timeout -k 10 200 python3 -c "
import sys; sys.path.insert(0,'.')
import bench, rsmt2d_amd as R, json
L=R.library()
for kk in (256, 512): print(json.dumps(bench.bench_c3(0, L, R, repeats=3, k=kk)), flush=True)
" > gpurun_out/gf16rep_r03ag.jsonl 2>&1 || exit 5
