"""GF(2^8) byte-table kernels A/B (diagnostic library; RSM_DIAG_LIB picks the build):
device time of (1) one k = 128, S = 512 square (the latency form, two launches of
encode_gf8_split_kernel<8>), (2) the c3 decode sweep (k = 128, S = 512, k of the 2k cells
of every row erased, decode_gf8_split_kernel<16>), (3) batches of k = 16 / 32 / 64
squares (encode_gf8_kernel<M>).  Each line carries a digest of the output so two builds
can be compared bit for bit.  usage: RSM_DIAG_LIB=... python3 scripts/diag/gf8_ab.py"""
import ctypes
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import rsmt2d_amd as R  # noqa: E402

D = R.diag_library()
LIB = os.path.basename(R.DIAG_LIB_PATH)


def chk(rc):
    R._check_with(D, rc)


def digest(ctx, p, n):
    out = np.empty(n, np.uint8)
    chk(D.rsm_memcpy(ctx, out.ctypes.data, p, n, 1))
    return hashlib.sha256(out.tobytes()).hexdigest()[:16]


def main():
    ctx = ctypes.c_void_p()
    chk(D.rsm_ctx_create(0, ctypes.byref(ctx)))
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    chk(D.rsm_event_create(ctx, ctypes.byref(e0)))
    chk(D.rsm_event_create(ctx, ctypes.byref(e1)))
    ms = ctypes.c_float()

    def timed(fn, n):
        fn()
        chk(D.rsm_event_record(ctx, e0, None))
        for _ in range(n):
            fn()
        chk(D.rsm_event_record(ctx, e1, None))
        chk(D.rsm_sync(ctx))
        chk(D.rsm_event_elapsed_ms(e0, e1, ctypes.byref(ms)))
        return ms.value / n * 1e3

    k, S = 128, 512
    W = 2 * k
    n = W * W * S
    p = ctypes.c_void_p()
    chk(D.rsm_dev_alloc(ctx, n, ctypes.byref(p)))
    chk(D.rsm_dev_fill_random(ctx, p.value, n, 0x5A))
    us = timed(lambda: chk(D.rsm_extend_squares_dev(ctx, p.value, k, S, 1, None)), 200)
    print(json.dumps({"lib": LIB, "what": "single square k=128 S=512", "us": round(us, 2),
                      "digest": digest(ctx, p.value, n)}), flush=True)
    # c3 decode sweep
    full = np.empty(n, np.uint8)
    chk(D.rsm_memcpy(ctx, full.ctypes.data, p.value, n, 1))
    rng = np.random.default_rng(0xC3)
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
    chk(D.rsm_memcpy(ctx, p.value, damaged.ctypes.data, n, 0))
    sweep = lambda: chk(D.rsm_decode_vectors_dev(ctx, p.value, pres.value, k, S, 0, idx.value, W, None))
    sweep()
    chk(D.rsm_sync(ctx))
    out = np.empty(n, np.uint8)
    chk(D.rsm_memcpy(ctx, out.ctypes.data, p.value, n, 1))
    us = timed(sweep, 50)
    print(json.dumps({"lib": LIB, "what": "c3 decode sweep", "us": round(us, 2),
                      "rebuilt_equal": bool(np.array_equal(out, full))}), flush=True)
    for b in (p, pres, idx):
        chk(D.rsm_dev_free(ctx, b))
    # small squares, 256 MiB of EDS per call
    for k in (16, 32, 64):
        W = 2 * k
        cnt = (256 << 20) // (W * W * S)
        n = W * W * S * cnt
        q = ctypes.c_void_p()
        chk(D.rsm_dev_alloc(ctx, n, ctypes.byref(q)))
        chk(D.rsm_dev_fill_random(ctx, q.value, n, k))
        us = timed(lambda: chk(D.rsm_extend_squares_dev(ctx, q.value, k, S, cnt, None)), 10)
        print(json.dumps({"lib": LIB, "what": f"batch of {cnt} squares k={k} S=512", "us_per_square": round(us / cnt, 4),
                          "frac": round(4 * k * k * S / (us / cnt * 1e-6) / 8e12, 4),
                          "digest": digest(ctx, q.value, min(n, 1 << 24))}), flush=True)
        chk(D.rsm_dev_free(ctx, q))


if __name__ == "__main__":
    main()
