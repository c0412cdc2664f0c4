"""Codec call latency A/B (diagnostic library): rsm_encode / rsm_decode of one k = 128,
S = 512 codeword (BenchmarkEncoding / BenchmarkDecoding shape, codec_test.go:15-80) with
the lane wait blocking at once (spin 0, production) or spinning on hipStreamQuery for up to
N us first (rsm_diag_set_codec_spin).  Prints one JSON line per (op, spin): p10/p50/p90 of
single-thread latency and the 16-thread aggregate rate.
usage: python3 scripts/diag/codec_spin_ab.py"""
import ctypes
import json
import os
import sys
import threading
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
    rng = np.random.default_rng(7)
    data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
    par = [np.empty(S, np.uint8) for _ in range(k)]
    dp = (ctypes.c_void_p * k)(*[d.ctypes.data for d in data])
    pp = (ctypes.c_void_p * k)(*[p.ctypes.data for p in par])
    chk(D.rsm_encode(ctx.value, dp, k, S, pp))
    full = data + [p.copy() for p in par]
    present = np.ones(2 * k, np.uint8)
    present[rng.choice(2 * k, size=k, replace=False)] = 0
    work = [np.empty(S, np.uint8) for _ in range(2 * k)]
    wp = (ctypes.c_void_p * (2 * k))(*[w.ctypes.data for w in work])

    def enc():
        chk(D.rsm_encode(ctx.value, dp, k, S, pp))

    def dec():
        for i in range(2 * k):
            if present[i]:
                work[i][:] = full[i]
        chk(D.rsm_decode(ctx.value, wp, present.ctypes.data, 2 * k, S))

    for spin in (0, 30, 100, 0, 30, 100):
        chk(D.rsm_diag_set_codec_spin(spin))
        for name, fn in (("encode", enc), ("decode", dec)):
            for _ in range(50):
                fn()
            lat = []
            for _ in range(1000):
                t = time.perf_counter()
                fn()
                lat.append((time.perf_counter() - t) * 1e6)
            lat.sort()
            n_thr, dur = 16, 1.0
            counts = [0] * n_thr
            stop = time.perf_counter() + dur

            def worker(j):
                while time.perf_counter() < stop:
                    fn()
                    counts[j] += 1

            ts = [threading.Thread(target=worker, args=(j,)) for j in range(n_thr)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
            print(json.dumps({"op": name, "spin_us": spin, "p10_us": round(lat[100], 1),
                              "p50_us": round(lat[500], 1), "p90_us": round(lat[900], 1),
                              "threads16_calls_per_s": round(sum(counts) / dur)}), flush=True)
    chk(D.rsm_diag_set_codec_spin(0))


if __name__ == "__main__":
    main()
