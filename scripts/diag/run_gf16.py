"""A short GF(2^16) workload for counter passes: N device-resident extensions of one
c4 square (k = 256, S = 2048) and one c5 square (k = 512, S = 512), each launch pair
(row pass, column pass) of enc16_kernel<256 / 512>.  Algorithmic bytes per square:
4 k^2 S = 512 MiB (row pass: 2 k^2 S, column pass: 4 k^2 S... see DESIGN.md §7).
usage: python3 scripts/diag/run_gf16.py [N]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import rsmt2d_amd as R  # noqa: E402


def main(n):
    L = R.library()
    ctx = R.device_context(0)
    for k, S in ((256, 2048), (512, 512)):
        W = 2 * k
        buf = R.DeviceBuffer(W * W * S)
        buf.fill_random(k)
        for _ in range(n):
            R._check(L.rsm_extend_squares_dev(ctx, buf.ptr, k, S, 1, None))
        R._check(L.rsm_sync(ctx))
        buf.free()
    print("ok")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
