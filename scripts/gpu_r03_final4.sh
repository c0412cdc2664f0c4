#!/bin/bash
# end-of-round validation final tree of round 3 (GF16 Codec zero-copy included): smoke, all GPU tests, default bench
STEPS=smoke,pytest,bench BENCH_ARGS="" bash scripts/gpu_round.sh
