"""Latency-form A/B (diagnostic library): device time of rsm_extend_squares_dev for
small batches of k = 128, S = 512 squares -- the split encoder's waves per task in
each of its two launches, and the batch size where the queue-driven launch overtakes
it (rsm_ctx_set_split_max).  One JSON line per configuration.
usage: [SINGLE_AB="0,8,8 0,16,16 ..."] python3 scripts/diag/single_ab.py  (fused,waves1,waves2 triples)
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import rsmt2d_amd as R  # noqa: E402
from refcheck import matches_two_launch  # noqa: E402

D = R.diag_library()


def chk(rc):
    R._check_with(D, rc)


def main():
    k, S = 128, 512
    W = 2 * k
    ctx = ctypes.c_void_p()
    chk(D.rsm_ctx_create(0, ctypes.byref(ctx)))
    buf = R.DeviceBuffer(W * W * S * 64)
    buf.fill_random(3)
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    chk(D.rsm_event_create(ctx, ctypes.byref(e0)))
    chk(D.rsm_event_create(ctx, ctypes.byref(e1)))

    def dev_us(count, n):
        chk(D.rsm_extend_squares_dev(ctx, buf.ptr, k, S, count, None))
        chk(D.rsm_event_record(ctx, e0, None))
        for _ in range(n):
            chk(D.rsm_extend_squares_dev(ctx, buf.ptr, k, S, count, None))
        chk(D.rsm_event_record(ctx, e1, None))
        ms = ctypes.c_float()
        chk(D.rsm_event_elapsed_ms(e0, e1, ctypes.byref(ms)))
        return round(ms.value / n * 1e3, 2)

    chk(D.rsm_ctx_set_split_max(ctx, 64, None))
    configs = [tuple(int(x) for x in c.split(",")) for c in os.environ["SINGLE_AB"].split()] \
        if os.environ.get("SINGLE_AB") else [(0, 8, 8), (0, 4, 4), (1, 8, 8), (0, 8, 8)]
    for fused, a, b in configs:
        chk(D.rsm_diag_set_split_fused(fused))
        chk(D.rsm_diag_set_split_waves(a, b))
        got = dev_us(1, 200)
        sq = buf.download(W * W * S).reshape(W, W, S)
        ok = matches_two_launch(D, ctx, sq, k)
        print(json.dumps({"fused": fused, "waves": [a, b], "count": 1, "us": got, "ok": ok}), flush=True)
    chk(D.rsm_diag_set_split_fused(0))
    if os.environ.get("SINGLE_SWEEP"):  # waves per task x batch size (latency form only)
        for a, b in ((8, 8), (16, 16), (8, 8), (16, 16)):
            chk(D.rsm_diag_set_split_waves(a, b))
            for c in (1, 2, 4, 8, 12):
                got = dev_us(c, 100 if c < 8 else 40)
                print(json.dumps({"waves": [a, b], "count": c, "us": got, "us_per_sq": round(got / c, 2)}), flush=True)
        chk(D.rsm_diag_set_split_waves(0, 0))
        return
    chk(D.rsm_diag_set_split_waves(0, 0))
    for c in (1, 2, 4, 8, 16, 24, 32):
        chk(D.rsm_ctx_set_split_max(ctx, 64, None))
        sp = dev_us(c, 30)
        chk(D.rsm_ctx_set_split_max(ctx, 0, None))
        q = dev_us(c, 30)
        print(json.dumps({"count": c, "split_us": sp, "queue_us": q, "split_us_per_sq": round(sp / c, 2),
                          "queue_us_per_sq": round(q / c, 2)}), flush=True)


if __name__ == "__main__":
    main()
