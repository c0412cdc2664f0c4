"""Small-batch kernels under a PMC pass (diagnostic): the latency-form split encoder
(single square), the M = 128 split decoder (c3 sweep + Repair) and the Codec path,
for SQC instruction-cache counters.  usage: python3 scripts/diag/icache_small.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import rsmt2d_amd as R  # noqa: E402


def main():
    L = R.library()
    print("single", bench.bench_single_square(0, L, R), flush=True)
    print("c3", bench.bench_c3(0, L, R, repeats=1), flush=True)


if __name__ == "__main__":
    main()
