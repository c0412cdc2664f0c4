"""Minimal driver for profiling: B squares of k=128/S=512 extended N times on the device.
usage: python3 scripts/run_extend.py [reps] [batch] [phase]   (3 = both, 1 = rows, 2 = cols)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rsmt2d_amd as R

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
phase = int(sys.argv[3]) if len(sys.argv) > 3 else 3
k, S = 128, 512
W = 2 * k
L = R.library()
ctx = R.device_context(0)
buf = R.DeviceBuffer(B * W * W * S, 0)
buf.fill_random(7)
for _ in range(3):
    R._check(L.rsm_extend_squares_phase_dev(ctx, buf.ptr, k, S, B, phase, None))
R._check(L.rsm_sync(ctx))
t0 = time.perf_counter()
for _ in range(reps):
    R._check(L.rsm_extend_squares_phase_dev(ctx, buf.ptr, k, S, B, phase, None))
R._check(L.rsm_sync(ctx))
dt = (time.perf_counter() - t0) / reps
msg = ""
if os.environ.get("CHECK") and phase == 3:
    import numpy as np
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "diag"))
    from refcheck import matches_two_launch
    buf.fill_random(11)
    R._check(L.rsm_extend_squares_phase_dev(ctx, buf.ptr, k, S, B, 3, None))
    R._check(L.rsm_sync(ctx))
    allb = buf.download(B * W * W * S).reshape(B, W, W, S)
    bad = 0
    for i in sorted({0, B // 2, B - 1}):
        bad += int(not matches_two_launch(L, ctx, allb[i].copy(), k))
    msg = " CHECK " + ("ok" if bad == 0 else f"FAILED ({bad} squares differ)")
print(f"B={B} phase={phase}: {dt*1e6:.1f} us/step, {B*k*k*S/dt/2**30:.1f} GiB/s ODS{msg}")
buf.free()
