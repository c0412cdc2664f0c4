#!/bin/bash
# bench.py (c2, alternating batches) under kernel variants: stream pipelining and
# cache policies (RSM_BS_MODE 8 default, 24 nt stores, 40 nt loads, 56 both).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() { local tag=$1; shift; timeout -k 10 180 "$@" python3 bench.py --steps 30 --no-c3 --no-c5 --no-roots --no-cpu-baseline ${EXTRA:-} > gpurun_out/bab_$tag.json 2>&1 || return 1;
  python3 -c "import json;d=json.loads(open('gpurun_out/bab_$tag.json').read().strip().splitlines()[-1]);print('$tag', d['value'], d['ms_per_step'], d['step_roofline']['row_pass_us'], d['step_roofline']['col_pass_us'])"; }
EXTRA=--one-stream run one_stream_m8 env RSM_BS_MODE=8 || exit 3
for m in 8 24 40 56; do run m$m env RSM_BS_MODE=$m || exit 3; done
for m in 24 40 56; do
  RSM_BS_MODE=$m timeout -k 10 120 python3 -m pytest tests/test_gpu_codec.py -q -k "extend or bitsliced or partial" --timeout 60 2>&1 | tail -1 | sed "s/^/mode $m tests: /"
done
