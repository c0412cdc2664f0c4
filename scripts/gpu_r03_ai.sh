#!/bin/bash
# GF(2^16) Codec zero-copy: parity + latency
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_codec.py tests/test_gpu_gf16.py tests/test_gpu_gf16_large.py > gpurun_out/pytest_r03ai.log 2>&1 || exit 3
timeout -k 10 180 python3 scripts/diag/codec16_latency.py > gpurun_out/codec16_r03ai.jsonl 2>&1 || exit 4
