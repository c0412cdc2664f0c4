"""Decode sweep A/B (diagnostic library): the c3 scheme (k of the 2k cells of every row
erased, BenchmarkRepair), S = 512, decoded by rsm_decode_vectors_dev:
  k = 256, 200 (GF(2^16), m = 256): the single-pass decoder (dec16f_kernel,
          production) or the five global passes (rsm_diag_set_dec16_five_pass);
  k = 128 (GF(2^8) split decoder): DECAB_V8 variants -- 0 production, 1 the other
          error-locator form (rsm_diag_set_dec8_mode), 100 + t the upper half of the grid
          delaying its point loads by t ticks of the 100 MHz clock (rsm_diag_set_dec_delay).
DECAB_KS picks the k values (default 256,200); DECAB_V16 the GF(2^16) variants (0 production,
1 the five passes, other values rsm_diag_set_dec16_mode bits).  Every rebuilt square compared with the original EDS.  One JSON line per configuration.
usage: python3 scripts/diag/dec_ab.py"""
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
    for k in [int(x) for x in os.environ.get("DECAB_KS", "256,200").split(",")]:
        S = 512
        W = 2 * k
        n = W * W * S
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
        pres = ctypes.c_void_p()
        idx = ctypes.c_void_p()
        chk(D.rsm_dev_alloc(ctx, W * W, ctypes.byref(pres)))
        chk(D.rsm_dev_alloc(ctx, 4 * W, ctypes.byref(idx)))
        chk(D.rsm_memcpy(ctx, pres.value, present.ctypes.data, W * W, 0))
        ids = np.arange(W, dtype=np.uint32)
        chk(D.rsm_memcpy(ctx, idx.value, ids.ctypes.data, 4 * W, 0))
        def set16(v):  # 0 production, 1 the five passes, other values rsm_diag_set_dec16_mode bits
            chk(D.rsm_diag_set_dec16_five_pass(1 if v == 1 else 0))
            chk(D.rsm_diag_set_dec16_mode(0 if v == 1 else v))
            return 0
        def set8(v):  # DECAB_V8: 0 production, 1 the other locator form, 2 the setup-free floor of a
            # pre-pass design (wrong output: timing only), >= 100: load delay v - 100 ticks
            chk(D.rsm_diag_set_dec8_mode(v if v < 100 else 0))
            return D.rsm_diag_set_dec_delay(v - 100 if v >= 100 else 0)
        setter = set16 if k > 128 else set8
        variants = ([int(x) for x in os.environ.get("DECAB_V16", "0,1").split(",")] if k > 128
                    else [int(x) for x in os.environ.get("DECAB_V8", "0,1").split(",")])
        for rep in range(2):
            for five in variants:
                chk(setter(five))
                chk(D.rsm_memcpy(ctx, buf.value, damaged.ctypes.data, n, 0))
                chk(D.rsm_decode_vectors_dev(ctx, buf.value, pres.value, k, S, 0, idx.value, W, None))
                chk(D.rsm_sync(ctx))
                eq = ctypes.c_int(0)
                chk(D.rsm_dev_equal(ctx, buf.value, ref.value, n, None, ctypes.byref(eq)))
                reps = 50 if k <= 128 else 10
                t0 = time.perf_counter()
                for _ in range(reps):
                    chk(D.rsm_decode_vectors_dev(ctx, buf.value, pres.value, k, S, 0, idx.value, W, None))
                chk(D.rsm_sync(ctx))
                dt = (time.perf_counter() - t0) / reps
                print(json.dumps({"k": k, "S": S, ("variant" if k <= 128 else "five_pass"): five, "rep": rep,
                                  "sweep_ms": round(dt * 1e3, 4),
                                  "frac": round(W * W * S / dt / 8e12, 4), "rebuilt_equal": bool(eq.value)}),
                      flush=True)
        chk(setter(0))
        for b in (buf, ref, pres, idx):
            chk(D.rsm_dev_free(ctx, b))


if __name__ == "__main__":
    main()
