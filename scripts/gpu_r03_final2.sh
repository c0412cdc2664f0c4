#!/bin/bash
# end-of-round validation after the decoder table change: smoke, all GPU tests, default bench
STEPS=smoke,pytest,bench BENCH_ARGS="" bash scripts/gpu_round.sh
