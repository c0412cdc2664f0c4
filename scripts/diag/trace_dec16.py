"""Phase timeline of the GF(2^16) m = 512 half-wave decoder (dec16h_kernel; diagnostic
library, decode trace): the BenchmarkRepair decode sweep k = 512, S = 512 (every row of
the EDS with k of its 2k cells erased; 2048 workgroups).  Thread 0 of every workgroup
stamps the 100 MHz clock at 13 points (kernels_gf16.hip d16_stamp); prints the mean
phase durations, the mean task time and the launch span in us, for each A/B mode of
TRACE_MODES (rsm_diag_set_dec16_mode bits; 0 = production, the only one whose output
is checked).
usage: python3 scripts/diag/trace_dec16.py"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import rsmt2d_amd as R  # noqa: E402

D = R.diag_library()
NAMES = ["presence", "loads+scale tables", "scale+twiddle staging", "group IFFT", "to residue+restage",
         "residue IFFT", "derivative", "residue FFT", "to group", "group FFT", "reveal tables", "reveal+stores"]
WORDS = 16


def chk(rc):
    R._check_with(D, rc)


def main():
    k, S = 512, 512
    W = 2 * k
    n = W * W * S
    ctx = ctypes.c_void_p()
    chk(D.rsm_ctx_create(0, ctypes.byref(ctx)))
    buf, ref = ctypes.c_void_p(), ctypes.c_void_p()
    chk(D.rsm_dev_alloc(ctx, n, ctypes.byref(buf)))
    chk(D.rsm_dev_alloc(ctx, n, ctypes.byref(ref)))
    chk(D.rsm_dev_fill_random(ctx, ref.value, n, 0xD16 + k))
    chk(D.rsm_extend_squares_dev(ctx, ref.value, k, S, 1, None))
    chk(D.rsm_sync(ctx))
    full = np.empty(n, np.uint8)
    chk(D.rsm_memcpy(ctx, full.ctypes.data, ref.value, n, 1))
    rng = np.random.default_rng(k)
    present = np.ones((W, W), np.uint8)
    for r in range(W):
        present[r, rng.choice(W, size=k, replace=False)] = 0
    damaged = (full.reshape(W, W, S) * present[:, :, None]).reshape(-1)
    pres, idx = ctypes.c_void_p(), ctypes.c_void_p()
    chk(D.rsm_dev_alloc(ctx, W * W, ctypes.byref(pres)))
    chk(D.rsm_dev_alloc(ctx, 4 * W, ctypes.byref(idx)))
    chk(D.rsm_memcpy(ctx, pres.value, present.ctypes.data, W * W, 0))
    ids = np.arange(W, dtype=np.uint32)
    chk(D.rsm_memcpy(ctx, idx.value, ids.ctypes.data, 4 * W, 0))
    tasks = W * ((S + 255) // 256)
    tr = ctypes.c_void_p()
    chk(D.rsm_dev_alloc(ctx, tasks * WORDS * 4, ctypes.byref(tr)))
    for mode in [int(x) for x in os.environ.get("TRACE_MODES", "0").split(",")]:
        chk(D.rsm_diag_set_dec16_mode(mode))
        for rep in range(3):
            chk(D.rsm_memcpy(ctx, buf.value, damaged.ctypes.data, n, 0))
            chk(D.rsm_diag_set_dec_trace(tr.value if rep == 2 else None))
            chk(D.rsm_decode_vectors_dev(ctx, buf.value, pres.value, k, S, 0, idx.value, W, None))
            chk(D.rsm_sync(ctx))
        chk(D.rsm_diag_set_dec_trace(None))
        chk(D.rsm_diag_set_dec16_mode(0))
        report(D, ctx, buf, ref, tr, n, tasks, k, S, mode)
    for b in (buf, ref, pres, idx, tr):
        chk(D.rsm_dev_free(ctx, b))


def report(D, ctx, buf, ref, tr, n, tasks, k, S, mode):
    eq = ctypes.c_int(0)
    chk(D.rsm_dev_equal(ctx, buf.value, ref.value, n, None, ctypes.byref(eq)))
    raw = np.empty(tasks * WORDS, np.uint32)
    chk(D.rsm_memcpy(ctx, raw.ctypes.data, tr.value, tasks * WORDS * 4, 1))
    st = raw.reshape(tasks, WORDS)[:, :13].astype(np.int64)
    st -= st[:, :1].min()
    d = np.diff(st, axis=1) * 0.01
    out = {"k": k, "S": S, "mode": mode, "rebuilt_equal": bool(eq.value),
           "phases_us_mean": {nm: round(float(d[:, i].mean()), 3) for i, nm in enumerate(NAMES)},
           "task_us_mean": round(float((st[:, 12] - st[:, 0]).mean() * 0.01), 3),
           "start_spread_us": round(float((st[:, 0].max() - st[:, 0].min()) * 0.01), 3),
           "launch_span_us": round(float((st[:, 12].max() - st[:, 0].min()) * 0.01), 3)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
