# round 3 (aa): energy of pure algorithmic streaming (mixprobe: read Q0 rows, write Q1/Q2/Q3
# rows, 4k^2 S per square, no re-reads, no arithmetic) against the c2 kernel's memory-only
# and production modes, same box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd scripts/diag
for m in 2 0 4; do
  timeout -k 10 120 python3 -u power_cmd.py 3 ./mixprobe 256 2 $m 512 6000 >> ../../gpurun_out/power_mix_r03aa.jsonl 2>&1 || exit 2
done
cd ../..
timeout -k 10 300 python3 -u scripts/diag/power_probe.py 5000 40:5000 50770:7000 > gpurun_out/power_q_r03aa.jsonl 2>&1 || exit 3
