# round 3 (j): latency form for single squares, direct-load production kernel
set -u
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_runtime.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_r03j.log 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r03j.log 2>&1 || exit 2
QAB_STEPS=40 timeout -k 10 300 python3 -u scripts/diag/queue_ab.py queue,256,3,2,40 queue,256,3,2,51021 queue,256,3,2,40 queue,256,3,2,51021 > gpurun_out/qab_r03j.jsonl 2>&1 || exit 3
timeout -k 10 600 python3 bench.py > gpurun_out/bench_r03j.log 2>&1 || exit 4
timeout -k 10 120 python3 -u scripts/diag/trace_decode.py > gpurun_out/trace_dec_r03j.jsonl 2>&1 || exit 5
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$PWD/gpurun_out/g16_f" -o run --output-format csv -- python3 scripts/diag/run_gf16.py 3 > /dev/null 2>&1 || exit 6
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$PWD/gpurun_out/g16_w" -o run --output-format csv -- python3 scripts/diag/run_gf16.py 3 > /dev/null 2>&1 || exit 7
