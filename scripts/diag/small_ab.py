"""Small-square latency-form A/B (product library): device time of rsm_extend_squares_dev
for k = 32 / 64, S = 512 and 1..12 squares per call, with the split form
(encode_gf8_splitm_kernel, rsm_ctx_set_split_max 12) and with the byte-table passes
(split_max 0).  Each line carries a digest of the first square so the two forms can be
compared bit for bit.  usage: [SMALL_COUNTS=1,2,4] python3 scripts/diag/small_ab.py  (the split form: split_max raised past the count)"""
import ctypes
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import rsmt2d_amd as R  # noqa: E402


def main():
    L = R.library()
    ctx = R.device_context(0)
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    R._check(L.rsm_event_create(ctx, ctypes.byref(e0)))
    R._check(L.rsm_event_create(ctx, ctypes.byref(e1)))
    ms = ctypes.c_float()
    S = 512
    for rep in range(2):
        for k in [int(x) for x in os.environ.get("SMALL_KS", "32,64").split(",")]:
            W = 2 * k
            counts = [int(c) for c in os.environ.get("SMALL_COUNTS", "1,2,4,8,12").split(",")]
            for count in counts:
                buf = R.DeviceBuffer(W * W * S * count)
                for split_max in (1 << 20, 0):
                    buf.fill_random(k + count)
                    R._check(L.rsm_ctx_set_split_max(ctx, split_max, None))
                    R._check(L.rsm_extend_squares_dev(ctx, buf.ptr, k, S, count, None))
                    R._check(L.rsm_sync(ctx))
                    dig = hashlib.sha256(buf.download(W * W * S).tobytes()).hexdigest()[:16]
                    n = max(10, 200 // count)
                    R._check(L.rsm_event_record(ctx, e0, None))
                    for _ in range(n):
                        R._check(L.rsm_extend_squares_dev(ctx, buf.ptr, k, S, count, None))
                    R._check(L.rsm_event_record(ctx, e1, None))
                    R._check(L.rsm_sync(ctx))
                    R._check(L.rsm_event_elapsed_ms(e0, e1, ctypes.byref(ms)))
                    print(json.dumps({"rep": rep, "k": k, "count": count, "form": "split" if split_max else "byte-table",
                                      "us": round(ms.value / n * 1e3, 2), "digest": dig}), flush=True)
                buf.free()
    R._check(L.rsm_ctx_set_split_max(ctx, 12, None))
    L.rsm_event_destroy(e0)
    L.rsm_event_destroy(e1)


if __name__ == "__main__":
    main()
