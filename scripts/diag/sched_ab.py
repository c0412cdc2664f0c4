"""Schedule / cache-policy A/B for the c2 extension (diagnostic library only).

Each configuration times `steps` steps of B squares (k=128, S=512) rotating over
`buffers` batches and `streams` streams (a step's two passes stay ordered on its
stream), with the bit-sliced kernel variant of each pass chosen through the
diagnostic switches (row_mode / col_mode: 40 production, 8 plain loads, 56 NT
loads + NT stores, 24 plain loads + NT stores), and checks one square of the last
step against the two-launch form (refcheck.py).  Prints one JSON line per configuration.
usage: python3 scripts/diag/sched_ab.py "row,col,B,streams,buffers,grid[,rev[,col_grid]]" ...
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import rsmt2d_amd as R  # noqa: E402

D = R.diag_library()
chk = lambda rc: R._check_with(D, rc)
k, S = 128, 512
W = 2 * k
SQ = W * W * S
ctx = ctypes.c_void_p()
chk(D.rsm_ctx_create(0, ctypes.byref(ctx)))
ctx = ctx.value


def run(cfg, steps=60, warmup=6):
    f = [int(x) for x in cfg.split(",")]
    rmode, cmode, B, ns, nb, grid = f[:6]
    rev = f[6] if len(f) > 6 else 1
    cgrid = f[7] if len(f) > 7 else 0
    chk(D.rsm_diag_set_bs_row_mode(rmode))
    chk(D.rsm_diag_set_bs_mode(cmode, rev, 0))
    chk(D.rsm_ctx_set_pass_grid(ctx, 0, grid, None))
    chk(D.rsm_ctx_set_pass_grid(ctx, 1, cgrid, None))
    bufs = []
    for i in range(nb):
        p = ctypes.c_void_p()
        chk(D.rsm_dev_alloc(ctx, B * SQ, ctypes.byref(p)))
        chk(D.rsm_dev_fill_random(ctx, p.value, B * SQ, 1234 + i))
        bufs.append(p.value)
    streams = [None]
    for _ in range(ns - 1):
        s = ctypes.c_void_p()
        chk(D.rsm_stream_create(ctx, ctypes.byref(s)))
        streams.append(s.value)

    def sync():
        chk(D.rsm_sync(ctx))
        for s in streams[1:]:
            chk(D.rsm_stream_sync(s))

    n = [0]

    def step():
        i = n[0]
        n[0] += 1
        chk(D.rsm_extend_squares_dev(ctx, bufs[i % nb], k, S, B, streams[i % ns]))

    for _ in range(warmup):
        step()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    dt = (time.perf_counter() - t0) / steps
    # correctness: the first square of the last step's batch
    last = bufs[(n[0] - 1) % nb]
    got = np.empty(SQ, np.uint8)
    chk(D.rsm_memcpy(ctx, got.ctypes.data, last, SQ, 1))
    got = got.reshape(W, W, S)
    from refcheck import matches_two_launch
    ok = matches_two_launch(D, ctx, got, k)
    for b in bufs:
        chk(D.rsm_dev_free(ctx, b))
    for s in streams[1:]:
        chk(D.rsm_stream_destroy(ctx, s))
    chk(D.rsm_ctx_set_pass_grid(ctx, 0, 0, None))
    chk(D.rsm_ctx_set_pass_grid(ctx, 1, 0, None))
    out = {"cfg": cfg, "row_mode": rmode, "col_mode": cmode, "batch": B, "streams": ns, "buffers": nb, "row_grid": grid, "col_grid": cgrid,
           "rev": rev, "us_per_step": round(dt * 1e6, 2), "us_per_square": round(dt * 1e6 / B, 3),
           "step_frac": round(4 * k * k * S / (dt / B) / 8e12, 4), "ok": ok}
    print(json.dumps(out), flush=True)


for c in sys.argv[1:]:
    run(c)
