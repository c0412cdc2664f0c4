"""Codec Decode latency A/B (diagnostic library): rsm_decode of one k = 128, S = 512
codeword with 64 of its 256 shares nil (BenchmarkDecoding's shape, codec_test.go:45-80),
the split decoder's error locator computed by wave 0 and shared through LDS (dec8 mode 0,
production) or by every wave itself (mode 1, the per-wave locator).  One JSON line per
(mode, repetition): p10/p50/p90 of single-thread latency in us.
usage: python3 scripts/diag/codec_dec_ab.py"""
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


def chk(rc):
    R._check_with(D, rc)


def main():
    ctx = ctypes.c_void_p()
    chk(D.rsm_ctx_create(0, ctypes.byref(ctx)))
    k, S = 128, 512
    rng = np.random.default_rng(11)
    data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
    par = [np.empty(S, np.uint8) for _ in range(k)]
    dp = (ctypes.c_void_p * k)(*[d.ctypes.data for d in data])
    pp = (ctypes.c_void_p * k)(*[p.ctypes.data for p in par])
    chk(D.rsm_encode(ctx.value, dp, k, S, pp))
    full = data + [p.copy() for p in par]
    present = np.ones(2 * k, np.uint8)
    present[rng.choice(2 * k, size=64, replace=False)] = 0
    work = [np.empty(S, np.uint8) for _ in range(2 * k)]
    wp = (ctypes.c_void_p * (2 * k))(*[w.ctypes.data for w in work])

    def dec():
        for i in range(2 * k):
            if present[i]:
                work[i][:] = full[i]
        chk(D.rsm_decode(ctx.value, wp, present.ctypes.data, 2 * k, S))

    for rep in range(3):
        for mode in (0, 1):
            chk(D.rsm_diag_set_dec8_mode(mode))
            for _ in range(50):
                dec()
            ok = all(np.array_equal(work[i], full[i]) for i in range(2 * k))
            lat = []
            for _ in range(1000):
                t = time.perf_counter()
                dec()
                lat.append((time.perf_counter() - t) * 1e6)
            q = np.percentile(lat, [10, 50, 90])
            print(json.dumps({"mode": mode, "rep": rep, "p10": round(q[0], 1), "p50": round(q[1], 1),
                              "p90": round(q[2], 1), "ok": ok}), flush=True)
    chk(D.rsm_diag_set_dec8_mode(0))


if __name__ == "__main__":
    main()
