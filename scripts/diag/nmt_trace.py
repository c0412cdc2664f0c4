"""NMT roots of a batch of k = 128, S = 512 squares (bench `with_nmt_roots` shape:
rsm_nmt_roots_squares_dev, namespace 29 B) for a kernel trace: leaf vs tree launch times,
beside the DefaultTree batch and a 28-byte-namespace batch (the generic leaf kernel).
usage: rocprofv3 --kernel-trace ... -- python3 scripts/diag/nmt_trace.py [squares] [reps]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import rsmt2d_amd as R  # noqa: E402

squares = int(sys.argv[1]) if len(sys.argv) > 1 else 32
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
k, S, ns = 128, 512, 29
W = 2 * k
L = R.library()
ctx = R.device_context(0)
buf = R.DeviceBuffer(squares * W * W * S)
buf.fill_random(0x4E)
R._check(L.rsm_extend_squares_dev(ctx, buf.ptr, k, S, squares, None))
roots = R.DeviceBuffer(squares * 2 * W * (2 * ns + 32))
status = R.DeviceBuffer(squares * 2 * W * 4)
p = R.NmtParams(ns, 1, k)
for _ in range(reps):  # random namespaces: push-order statuses are set, the hashing is the same
    R._check(L.rsm_nmt_roots_squares_dev(ctx, buf.ptr, W, S, squares, ctypes.byref(p), roots.ptr, status.ptr, None))
    R._check(L.rsm_default_roots_squares_dev(ctx, buf.ptr, W, S, squares, roots.ptr, None)
             if hasattr(L, "rsm_default_roots_squares_dev") else
             L.rsm_roots_squares_dev(ctx, buf.ptr, W, S, squares, roots.ptr, None))
p28 = R.NmtParams(28, 1, k)  # 28-byte namespaces: the generic leaf kernel on the same 9 blocks per cell
for _ in range(reps):
    R._check(L.rsm_nmt_roots_squares_dev(ctx, buf.ptr, W, S, squares, ctypes.byref(p28), roots.ptr, status.ptr, None))
R._check(L.rsm_sync(ctx))
print("ok", flush=True)
