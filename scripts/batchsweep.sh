set -e
for b in 4 8 16 32 64; do
  timeout -k 10 120 python3 bench.py --batch $b --steps 20 --no-c3 --no-c5 --no-roots --no-cpu-baseline > gpurun_out/b$b.json
done
