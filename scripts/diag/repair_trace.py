"""Repair (config 3) under a copy + kernel trace: k=128, S=512, 128 of 256 cells of
every row erased (BenchmarkRepair), repaired `reps` times.  (The split-transport trace of
DESIGN.md §5 was taken with a diagnostic Repair mode since removed.)
usage: repair_trace.py [reps]"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

import rsmt2d_amd as R  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
k, S = 128, 512
W = 2 * k
L = R.library()
LR = L
ctx = R.device_context(0)
buf = R.DeviceBuffer(W * W * S)
buf.fill_random(0xC3)
R._check(L.rsm_extend_squares_dev(ctx, buf.ptr, k, S, 1, None))
R._check(L.rsm_sync(ctx))
full = buf.download(W * W * S).reshape(W, W, S)
rng = np.random.default_rng(0xC3)
present = np.ones((W, W), np.uint8)
for r in range(W):
    present[r, rng.choice(W, size=k, replace=False)] = 0
base = full.ctypes.data
ptrs = (ctypes.c_void_p * (W * W))(*[base + i * S for i in range(W * W)])
lens = (ctypes.c_uint32 * (W * W))(*([S] * (W * W)))
h = ctypes.c_void_p()
R._check(L.rsm_eds_import(None, ptrs, lens, W * W, ctypes.byref(h)))
roots = {}
for axis in (0, 1):
    out = ctypes.create_string_buffer(W * 32)
    rl = ctypes.c_uint32()
    R._check(L.rsm_eds_roots(h, axis, None, None, out, 32, ctypes.byref(rl)))
    roots[axis] = out.raw
L.rsm_eds_free(h)
fp = (ctypes.c_void_p * (W * W))(*[base + i * S if present.flat[i] else None for i in range(W * W)])
fl = (ctypes.c_uint32 * (W * W))(*[S if present.flat[i] else 0 for i in range(W * W)])
ctx_r = ctx
for i in range(reps):
    h = ctypes.c_void_p()
    R._check_with(LR, LR.rsm_eds_import(None, fp, fl, W * W, ctypes.byref(h)))
    R._check_with(LR, LR.rsm_eds_set_context(h, ctx_r))
    byz = R._Byz()
    t0 = time.perf_counter()
    m0 = time.monotonic_ns()
    R._check_with(LR, LR.rsm_eds_repair(h, roots[0], roots[1], 32, None, None, ctypes.byref(byz)))
    m1 = time.monotonic_ns()
    print(f"repair {i}: {(time.perf_counter() - t0) * 1e3:.3f} ms monotonic_ns {m0} {m1}", flush=True)
    LR.rsm_eds_free(h)
