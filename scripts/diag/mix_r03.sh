#!/bin/bash
# algorithmic-traffic ceiling sweep (scripts/diag/mixprobe.hip); one JSON line each
set -u
B=scripts/diag/mixprobe
for cfg in "256 1 0 512" "256 2 0 512" "256 4 0 256" "256 2 2 512" "256 2 3 512" "256 2 4 512" "256 4 2 256" "256 8 2 256" "256 2 1 512" "256 4 3 256" "256 2 8 512" "256 2 16 512" "256 2 18 512" "256 2 20 512" "256 4 5 256"; do
  timeout -k 5 60 $B $cfg || exit $?
done
