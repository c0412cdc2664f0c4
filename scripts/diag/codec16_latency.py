"""Codec Decode / Encode latency for one GF(2^16) codeword (k = 256, 512; S = 512; half
of the 2k shares nil), from host memory through rsm_decode / rsm_encode -- the per-
codeword path a Go Codec user with k > 128 takes.  Checked against the original shares.
usage: python3 scripts/diag/codec16_latency.py"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import rsmt2d_amd as R  # noqa: E402


def main():
    L = R.library()
    ctx = R.device_context(0)
    for k in (256, 512):
        S = 512
        rng = np.random.default_rng(k)
        data = rng.integers(0, 256, (k, S), dtype=np.uint8)
        par = np.empty((k, S), np.uint8)
        dp = (ctypes.c_void_p * k)(*[data.ctypes.data + i * S for i in range(k)])
        pp = (ctypes.c_void_p * k)(*[par.ctypes.data + i * S for i in range(k)])
        enc = []
        for i in range(60):
            t0 = time.perf_counter()
            R._check(L.rsm_encode(ctx, dp, k, S, pp))
            enc.append(time.perf_counter() - t0)
        full = np.concatenate([data, par])
        present = np.ones(2 * k, np.uint8)
        present[rng.choice(2 * k, size=k, replace=False)] = 0
        work = np.empty_like(full)
        wp = (ctypes.c_void_p * (2 * k))(*[work.ctypes.data + i * S for i in range(2 * k)])
        dec = []
        for i in range(60):
            work[:] = full * present[:, None]
            t0 = time.perf_counter()
            R._check(L.rsm_decode(ctx, wp, present.ctypes.data, 2 * k, S))
            dec.append(time.perf_counter() - t0)
            if not np.array_equal(work, full):
                raise SystemExit("codec16: decoded codeword differs")
        print(json.dumps({"k": k, "S": S, "encode_us_p50": round(float(np.median(enc[10:])) * 1e6, 1),
                          "decode_us_p50": round(float(np.median(dec[10:])) * 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
