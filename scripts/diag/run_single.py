"""A short single-square workload for counter passes (the shape one cgo
ComputeExtendedDataSquare call sees, extendeddatasquare.go:50-77): N device-resident
extensions of ONE k = 128, S = 512 square (rsm_extend_squares_dev with count = 1: the
latency form, two launches of encode_gf8_split_kernel<8>).
usage: python3 scripts/diag/run_single.py [N]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import rsmt2d_amd as R  # noqa: E402


def main(n):
    L = R.library()
    ctx = R.device_context(0)
    k, S = 128, 512
    W = 2 * k
    buf = R.DeviceBuffer(W * W * S)
    buf.fill_random(k)
    for _ in range(n):
        R._check(L.rsm_extend_squares_dev(ctx, buf.ptr, k, S, 1, None))
    R._check(L.rsm_sync(ctx))
    buf.free()
    print("ok")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
