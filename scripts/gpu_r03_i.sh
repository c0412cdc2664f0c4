# round 3 (i): plane-pair exchange layout -- parity, same-box A/B, GF16 counter
# calibration, then the full round script
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_runtime.py -q -x --timeout 120 --timeout-method thread -k "single_launch or queue or bench_scale" > gpurun_out/pytest_r03i.log 2>&1 || exit 1
QAB_STEPS=40 timeout -k 10 300 python3 -u scripts/diag/queue_ab.py queue,256,3,2,40 queue,256,3,2,51020 queue,256,3,2,18472 queue,256,3,2,40 queue,256,3,2,51020 queue,256,3,2,50004 queue,256,3,2,52040 queue,256,3,2,40 > gpurun_out/qab_r03i.jsonl 2>&1 || exit 2
( cd scripts/diag && timeout -k 10 60 ./calib16 0 1024 5 && timeout -k 10 60 ./calib16 1 1024 5 ) > gpurun_out/calib16_r03i.jsonl 2>&1 || exit 3
for sh in 0 1; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d "$PWD/gpurun_out/cal_f$sh" -o run --output-format csv -- scripts/diag/calib16 $sh 1024 2 > /dev/null 2>&1 || exit 4
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d "$PWD/gpurun_out/cal_w$sh" -o run --output-format csv -- scripts/diag/calib16 $sh 1024 2 > /dev/null 2>&1 || exit 5
done
STEPS=smoke,pytest,bench,prof bash scripts/gpu_round.sh
