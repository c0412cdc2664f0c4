#!/bin/bash
# end-of-round validation after the GF(2^8) decoder table and GF(2^16) error-locator changes: smoke, all GPU tests, default bench
STEPS=smoke,pytest,bench BENCH_ARGS="" bash scripts/gpu_round.sh
