#!/bin/bash
# GF(2^16) Codec per-codeword latency after the n-point error locator
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 180 python3 scripts/diag/codec16_latency.py > gpurun_out/codec16_r03ah.jsonl 2>&1 || exit 3
