# round 3 (ad): GF(2^16) m = 512 encoder as 8 waves x 64 elements -- GF16 parity tests and
# the A/B against the 16-wave form
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_gf16.py tests/test_gpu_gf16_large.py -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_r03ad.log 2>&1 || exit 2
timeout -k 10 300 python3 -u scripts/diag/gf16_ab.py > gpurun_out/gf16ab_r03ad.jsonl 2>&1 || exit 3
