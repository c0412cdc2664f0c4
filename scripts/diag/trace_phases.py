"""Phase timeline of the half-split queue kernel (diagnostic library, trace modes).

Runs the c2 production shape (256 squares per launch, launches on 3 streams over 3
buffers), records one launch's per-set phase boundaries (thread 0, 100 MHz clock)
and prints the mean duration of every phase in us, per set kind.
usage: python3 scripts/diag/trace_phases.py [mode ...]   (51030 production + trace,
       51010 LDS-DMA form + trace, 51014 no global memory + trace, 51012 no arithmetic
       + trace)
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import rsmt2d_amd as R  # noqa: E402

D = R.diag_library()
chk = lambda rc: R._check_with(D, rc)
k, S, B = 128, 512, 256
W = 2 * k
SQ = W * W * S
NAMES = ["top+T0+IFFTs h0", "P1 issue (w0||T1+IFFTs h1)", "P1 LDS drain+bar", "read h0+bar",
         "P2 (w1||IFFTl h0)+sync+read h1", "IFFTl h1+mid+FFTl h0", "publish+claim", "P3 (w0||FFTl h1)+sync+read",
         "P4 (w1||FFTs+T h0+st h0)+sync+read h1+loads", "FFTs h1+T+st h1"]


def main(modes):
    ctx = ctypes.c_void_p()
    chk(D.rsm_ctx_create(0, ctypes.byref(ctx)))
    ctx = ctx.value
    bufs = []
    for i in range(3):
        p = ctypes.c_void_p()
        chk(D.rsm_dev_alloc(ctx, B * SQ, ctypes.byref(p)))
        chk(D.rsm_dev_fill_random(ctx, p.value, B * SQ, 4321 + i))
        bufs.append(p.value)
    streams = [None]
    for _ in range(2):
        s = ctypes.c_void_p()
        chk(D.rsm_stream_create(ctx, ctypes.byref(s)))
        streams.append(s.value)
    nwords = 256 * 256 * 14
    tr = ctypes.c_void_p()
    chk(D.rsm_dev_alloc(ctx, nwords * 4, ctypes.byref(tr)))
    for mode in modes:
        chk(D.rsm_diag_set_bs_mode(int(mode), 1, 0))
        chk(D.rsm_diag_set_trace(None))
        for i in range(9):  # warm, 3 concurrent streams
            chk(D.rsm_diag_extend_fused(ctx, bufs[i % 3], k, S, B, 2, streams[i % 3]))
        chk(D.rsm_sync(ctx))
        zero = np.zeros(nwords, np.uint32)
        chk(D.rsm_memcpy(ctx, tr.value, zero.ctypes.data, nwords * 4, 0))
        # traced launch on stream 0 between two untraced ones (the production overlap)
        chk(D.rsm_diag_extend_fused(ctx, bufs[1], k, S, B, 2, streams[1]))
        chk(D.rsm_diag_set_trace(tr))
        chk(D.rsm_diag_extend_fused(ctx, bufs[0], k, S, B, 2, streams[0]))
        chk(D.rsm_diag_set_trace(None))
        chk(D.rsm_diag_extend_fused(ctx, bufs[2], k, S, B, 2, streams[2]))
        chk(D.rsm_sync(ctx))
        for s in streams[1:]:
            chk(D.rsm_stream_sync(s))
        t = np.empty(nwords, np.uint32)
        chk(D.rsm_memcpy(ctx, t.ctypes.data, tr.value, nwords * 4, 1))
        t = t.reshape(256, 256, 14).astype(np.int64)
        ok = t[:, :, 0] != 0
        ok[:, 0] = False  # skip each workgroup's first set
        rows = t[ok]
        d = np.diff(rows[:, :11], axis=1) * 0.01  # us
        nxt = np.zeros(len(rows))  # set-to-set gap: next set's stamp 0 - this set's stamp 10
        out = {"mode": mode, "sets": int(ok.sum()), "set_us_mean": round(float((rows[:, 10] - rows[:, 0]).mean() * 0.01), 3)}
        # shader clock over the large layers (no memory ops there): cycles / real time
        cyc = (rows[:, 13] - rows[:, 12]) % (1 << 32)
        out["clock_GHz_large_layers"] = round(float(np.median(cyc / np.maximum(rows[:, 6] - rows[:, 5], 1) / 10.0)), 3)
        for kind, msk in (("all", np.ones(len(rows), bool)), ("row", (rows[:, 11] & 3) == 1),
                          ("q0col", (rows[:, 11] & 3) == 0), ("q1col", (rows[:, 11] & 2) == 2)):
            if msk.sum():
                out[kind] = {NAMES[i]: round(float(d[msk, i].mean()), 3) for i in range(10)}
                out[kind]["n"] = int(msk.sum())
        # gap between consecutive sets of a workgroup (loop back-edge)
        g = []
        for wg in range(256):
            r = t[wg][t[wg][:, 0] != 0]
            if len(r) > 2:
                g.extend(((r[1:, 0] - r[:-1, 10]) * 0.01).tolist())
        out["backedge_us_mean"] = round(float(np.mean(g)), 3) if g else None
        print(json.dumps(out), flush=True)
    chk(D.rsm_diag_set_trace(None))


if __name__ == "__main__":
    main(sys.argv[1:] or ["51030", "51014", "51012"])
