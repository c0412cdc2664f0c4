#!/bin/bash
# A/B of the fused extension launch: queue lag sweep and the two-launch form.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline --no-roots --no-c3 --no-c5 ${BENCH_ARGS:-}"
for lag in ${LAGS:-4 6 8 12}; do
  RSM_FUSED=1 RSM_FUSED_LAG=$lag timeout -k 10 200 $B > $OUT/ab_lag$lag.json 2> $OUT/ab_lag$lag.err || exit 3
  echo "lag $lag: $(python3 -c "import json;d=json.load(open('$OUT/ab_lag$lag.json'));print(d['value'], d['roofline']['avg_launch_us'], d['step_roofline']['frac'])")"
done
RSM_FUSED=0 timeout -k 10 200 $B > $OUT/ab_twolaunch.json 2> $OUT/ab_twolaunch.err || exit 4
echo "two-launch: $(python3 -c "import json;d=json.load(open('$OUT/ab_twolaunch.json'));print(d['value'], d['step_roofline'])")"
