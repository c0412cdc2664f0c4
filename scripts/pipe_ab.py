"""Timing: two-launch steps vs software-pipelined steps (rsm_extend_pipeline_dev),
B squares of k=128/S=512 per step over two alternating buffers; event-free wall
clock over N steps after warm-up (device-resident)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rsmt2d_amd as R  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 40
B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
k, S, W = 128, 512, 256
L = R.library()
ctx = R.device_context(0)
bufs = [R.DeviceBuffer(B * W * W * S) for _ in range(2)]
for i, b in enumerate(bufs):
    b.fill_random(9 + i)


def two_launch(n):
    for i in range(n):
        R._check(L.rsm_extend_squares_dev(ctx, bufs[i & 1].ptr, k, S, B, None))


def pipelined(n):
    R._check(L.rsm_extend_pipeline_dev(ctx, bufs[0].ptr, None, k, S, B, None))
    for i in range(n):
        rows = bufs[(i + 1) & 1].ptr if i + 1 < n else None
        R._check(L.rsm_extend_pipeline_dev(ctx, rows, bufs[i & 1].ptr, k, S, B, None))


for name, fn in [("two-launch", two_launch), ("pipelined", pipelined), ("two-launch", two_launch),
                 ("pipelined", pipelined)]:
    fn(4)
    R._check(L.rsm_sync(ctx))
    t0 = time.perf_counter()
    fn(N)
    R._check(L.rsm_sync(ctx))
    dt = (time.perf_counter() - t0) / N
    print("%-10s B=%d: %.1f us/step, %.1f GiB/s ODS" % (name, B, dt * 1e6, B * k * k * S / dt / 2**30))
