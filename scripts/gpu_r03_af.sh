#!/bin/bash
# decoder: per-point multiply tables resolved by wave 0 (ptab) -- parity + c3 sweep + phases
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_codec.py tests/test_gpu_eds.py tests/test_gpu_runtime.py > gpurun_out/pytest_r03af.log 2>&1 || exit 3
timeout -k 10 120 python3 scripts/diag/trace_decode.py > gpurun_out/trace_decode_r03af.jsonl 2>&1 || exit 4
timeout -k 10 200 python3 -c "
import sys; sys.path.insert(0,'.')
import bench, rsmt2d_amd as R, json
L=R.library()
for i in range(3): print(json.dumps(bench.bench_c3(0, L, R, repeats=3)), flush=True)
" > gpurun_out/c3_r03af.jsonl 2>&1 || exit 5
