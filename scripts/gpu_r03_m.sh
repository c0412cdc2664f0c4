# round 3 (m): split encoder merged middle layer, wave-count A/B
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_runtime.py -q -x --timeout 120 --timeout-method thread -k "split or single" > gpurun_out/pytest_r03m.log 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/diag/single_ab.py > gpurun_out/single_r03m.jsonl 2>&1 || exit 3
