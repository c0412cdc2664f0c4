"""Locates wrong cells of the single-launch queue extension (diagnostic library).

For a few (count, delay) shapes: extends with the two-launch form and with
rsm_diag_extend_fused twice on the same queue words, and prints, per quadrant, the
rows/columns that differ and whether the differing cells still hold the untouched
source bytes (a set never processed) or something else (a set processed from stale
inputs).  Written while finding the round-2g dropped-claim bug.
usage: python3 scripts/diag/qdbg.py   (on a GPU box)
"""
import ctypes, sys, os
sys.path.insert(0, os.getcwd())
import numpy as np
import rsmt2d_amd as R
D = R.diag_library()
chk = lambda rc: R._check_with(D, rc)
ctx = ctypes.c_void_p(); chk(D.rsm_ctx_create(0, ctypes.byref(ctx))); ctx = ctx.value
k, S = 128, 512
W = 2 * k
for count, delay in ((1, 0), (1, 1), (3, 2)):
    n = W * W * S * count
    bufs = []
    for _ in range(3):
        p = ctypes.c_void_p(); chk(D.rsm_dev_alloc(ctx, n, ctypes.byref(p))); bufs.append(p.value)
    src, a, b = bufs
    chk(D.rsm_dev_fill_random(ctx, src, n, 5)); chk(D.rsm_sync(ctx))
    chk(D.rsm_memcpy(ctx, a, src, n, 2)); chk(D.rsm_extend_squares_dev(ctx, a, k, S, count, None))
    chk(D.rsm_sync(ctx))
    ga = np.empty(n, np.uint8); chk(D.rsm_memcpy(ctx, ga.ctypes.data, a, n, 1))
    for it in range(2):
        chk(D.rsm_memcpy(ctx, b, src, n, 2)); chk(D.rsm_sync(ctx))
        chk(D.rsm_diag_extend_fused(ctx, b, k, S, count, delay, None))
        rc = D.rsm_diag_queue_check(ctx, None)
        chk(D.rsm_sync(ctx))
        gb = np.empty(n, np.uint8); chk(D.rsm_memcpy(ctx, gb.ctypes.data, b, n, 1))
        d = (ga.reshape(count, W, W, S) != gb.reshape(count, W, W, S)).any(axis=3)
        print("count", count, "delay", delay, "launch", it, "rc", rc, "bad cells", int(d.sum()), flush=True)
        if d.any():
            for s in range(count):
                for (r0, c0, name) in ((0, k, "Q1"), (k, 0, "Q2"), (k, k, "Q3")):
                    q = d[s, r0:r0 + k, c0:c0 + k]
                    if q.any():
                        rows = np.nonzero(q.any(axis=1))[0]; cols = np.nonzero(q.any(axis=0))[0]
                        print("  sq", s, name, "bad", int(q.sum()), "rows", rows[:8], "..", len(rows), "cols", cols[:16], "..", len(cols))
                        gs = np.empty(n, np.uint8); chk(D.rsm_memcpy(ctx, gs.ctypes.data, src, n, 1))
                        gs = gs.reshape(count, W, W, S); gbb = gb.reshape(count, W, W, S)
                        cc = cols + c0
                        untouched = (gbb[s, r0:r0 + k][:, cc] == gs[s, r0:r0 + k][:, cc]).all(axis=2)
                        print("    cells equal to the untouched source:", int(untouched.sum()), "of", untouched.size)
    for p in bufs: chk(D.rsm_dev_free(ctx, p))
