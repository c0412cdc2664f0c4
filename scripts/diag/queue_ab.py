"""Single-launch queue schedule vs the production two-launch schedule, c2 (k=128, S=512).

Configurations "kind,B,streams,delay": kind "two" = the round-1 two-launch schedule
(rsm_extend_squares_phase_dev row pass + column pass), kind "queue" = rsm_diag_extend_fused (extend_gf8_bs128q_kernel,
diagnostic library).  Steps of B squares rotate over 2 buffers and `streams` streams;
the first and last square of the last step are checked against the two-launch form (refcheck.py), and the
queue's stuck-wait word is checked.  One JSON line per configuration.
usage: python3 scripts/diag/queue_ab.py two,32,2,0 queue,32,1,2 queue,256,3,2,40,192 ...
(fields: kind, squares per step, streams, delay[, mode[, grid]])
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
STEPS = int(os.environ.get("QAB_STEPS", "100"))
EVENTS = os.environ.get("QAB_EVENTS", "0") == "1"  # a HIP event either side of every timed launch (as bench.py)


def run(cfg, steps=STEPS, warmup=6):
    f = cfg.split(",")
    kind, B, ns, delay = f[0], int(f[1]), int(f[2]), int(f[3])
    # optional 5th field: diagnostic kernel mode (2 = no arithmetic, 4 = no global
    # memory; both give wrong output by design) -- two-launch: "row/col" modes
    mode = f[4] if len(f) > 4 else "40"
    if kind == "two":
        rm, cm = mode.split("/") if "/" in mode else (mode, mode)
        chk(D.rsm_diag_set_bs_row_mode(int(rm)))
        chk(D.rsm_diag_set_bs_mode(int(cm), 1, 0))
    else:
        chk(D.rsm_diag_set_bs_mode(int(mode), 1, 0))
    grid = 224 if (kind == "two" and ns > 1) else 0
    if len(f) > 5:  # optional 6th field: persistent grid (workgroups) of the queue launch
        grid = int(f[5])
    chk(D.rsm_ctx_set_pass_grid(ctx, 0, grid, None))
    bufs = []
    nb = max(2, ns)  # a buffer per concurrently running step
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
    evs = []

    def step(timed=False):
        i = n[0]
        n[0] += 1
        st = streams[i % ns]
        if timed and EVENTS:
            e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
            chk(D.rsm_event_create(ctx, ctypes.byref(e0)))
            chk(D.rsm_event_create(ctx, ctypes.byref(e1)))
            evs.append((e0, e1))
            chk(D.rsm_event_record(ctx, e0, st))
        if kind == "two":  # the two launches explicitly (rsm_extend_squares_dev takes the queue path)
            chk(D.rsm_extend_squares_phase_dev(ctx, bufs[i % nb], k, S, B, 1, st))
            chk(D.rsm_extend_squares_phase_dev(ctx, bufs[i % nb], k, S, B, 2, st))
        else:
            chk(D.rsm_diag_extend_fused(ctx, bufs[i % nb], k, S, B, delay, st))
        if timed and EVENTS:
            chk(D.rsm_event_record(ctx, evs[-1][1], st))

    for _ in range(warmup):
        step()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(True)
    sync()
    dt = (time.perf_counter() - t0) / steps
    ok = True
    # diagnostic modes whose output is wrong by design (no arithmetic / memory / exchange)
    WRONG = {"2", "4", "32768", "65536", "131072", "98304", "32772", "50002", "50004", "50768", "50772",
             "51004", "51006", "51012", "51014", "50770", "55002", "55004"}
    if mode in WRONG or (kind == "two" and mode != "40"):
        ok = None  # diagnostic mode: output wrong by design, not checked
    elif kind == "queue":
        for st in streams:
            ok &= D.rsm_diag_queue_check(ctx, st) == 0
    last = bufs[(n[0] - 1) % nb]
    if ok is not None and os.environ.get("QAB_CHECK_ALL", "0") == "1":
        # every square of the last step against the product's two-launch form of the
        # same Q0, compared on the device (an XCD-affine launch leaves an XCD's squares
        # undone if that XCD got fewer workgroups than gridDim / 8)
        ref = ctypes.c_void_p()
        chk(D.rsm_dev_alloc(ctx, B * SQ, ctypes.byref(ref)))
        chk(D.rsm_memcpy(ctx, ref.value, last, B * SQ, 2))
        chk(D.rsm_extend_squares_phase_dev(ctx, ref.value, k, S, B, 1, None))
        chk(D.rsm_extend_squares_phase_dev(ctx, ref.value, k, S, B, 2, None))
        chk(D.rsm_sync(ctx))
        eq = ctypes.c_int(0)
        chk(D.rsm_dev_equal(ctx, ref.value, last, B * SQ, None, ctypes.byref(eq)))
        ok &= bool(eq.value)
        chk(D.rsm_dev_free(ctx, ref.value))
    from refcheck import matches_two_launch
    for j in ((0, B - 1) if ok is not None else ()):
        got = np.empty(SQ, np.uint8)
        chk(D.rsm_memcpy(ctx, got.ctypes.data, last + j * SQ, SQ, 1))
        got = got.reshape(W, W, S)
        ok &= matches_two_launch(D, ctx, got, k)
    for e0, e1 in evs:
        D.rsm_event_destroy(e0)
        D.rsm_event_destroy(e1)
    for s in streams[1:]:
        chk(D.rsm_stream_destroy(ctx, s))
    for p in bufs:
        chk(D.rsm_dev_free(ctx, p))
    us_sq = dt / B * 1e6
    algo = 4 * k * k * S
    return {"cfg": cfg, "events": EVENTS, "us_per_step": round(dt * 1e6, 2), "us_per_square": round(us_sq, 3),
            "step_frac": round(algo / (us_sq * 1e-6) / 8e12, 4), "ok": ok}


if __name__ == "__main__":
    for c in sys.argv[1:]:
        print(json.dumps(run(c)), flush=True)
