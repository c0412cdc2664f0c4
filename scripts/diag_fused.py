"""Fused-kernel diagnosis: per queue item, does its output match the two-launch
form, and which path (first item / prefetched / synchronous) computed it."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("RSM_FUSED_TRACE", "1")
os.environ.setdefault("RSM_FUSED", "1")
import rsmt2d_amd as R  # noqa: E402


def items(k, S, count, lag):
    rn, cn = k * S // 2048, 2 * k * S // 2048
    out = []
    for s in range(min(lag, count)):
        out += [("r", s * rn + i) for i in range(rn)]
    for b in range(count - lag):
        out += [("r", (lag + b) * rn + i) for i in range(rn)]
        out += [("c", b * cn + i) for i in range(cn)]
    for t in range((count - lag) * cn, count * cn):
        out.append(("c", t))
    return out


def main(S, count, lag=4):
    L = R.library()
    ctx = R.device_context(0)
    k, W = 128, 256
    lag = min(lag, count)
    n = W * W * S * count
    a, b = R.DeviceBuffer(n), R.DeviceBuffer(n)
    a.fill_random(11)
    R._check(L.rsm_sync(ctx))
    R._check(L.rsm_memcpy(ctx, b.ptr, a.ptr, n, 2))
    R._check(L.rsm_extend_squares_phase_dev(ctx, a.ptr, k, S, count, 1, None))
    R._check(L.rsm_extend_squares_phase_dev(ctx, a.ptr, k, S, count, 2, None))
    R._check(L.rsm_extend_squares_dev(ctx, b.ptr, k, S, count, None))
    R._check(L.rsm_sync(ctx))
    ga = a.download().reshape(count, W, W, S)
    gb = b.download().reshape(count, W, W, S)
    it = items(k, S, count, lag)
    tr = (ctypes.c_uint32 * len(it))()
    err = ctypes.c_uint32()
    m = L.rsm_fused_trace(ctx, tr, len(it), ctypes.byref(err))
    per = 2048 // S  # codewords per set (S <= 2048)
    bad_paths, good_paths = {}, {}
    lines = []
    for u, (kind, t) in enumerate(it):
        q0 = t * per
        sq, off = divmod(q0, k if kind == "r" else W)
        if kind == "r":
            d = (ga[sq, off:off + per, k:] != gb[sq, off:off + per, k:]).any()
        else:
            d = (ga[sq, k:, off:off + per] != gb[sq, k:, off:off + per]).any()
        v = tr[u]
        path = v & 3
        (bad_paths if d else good_paths)[path] = (bad_paths if d else good_paths).get(path, 0) + 1
        if d and len(lines) < 40:
            lines.append("item %d %s set %d sq %d: wg %d iter %d path %d" % (u, kind, t, sq, v >> 8, (v >> 2) & 63, path))
    print("S=%d count=%d items=%d traced=%d err=%d" % (S, count, len(it), m, err.value))
    print("bad by path", bad_paths, "good by path", good_paths)
    print("\n".join(lines))


if __name__ == "__main__":
    cases = [(64, 1), (512, 1), (512, 4)]
    if len(sys.argv) > 1:
        cases = [(512, int(sys.argv[1]))]
    for S, c in cases:
        main(S, c, int(os.environ.get("RSM_FUSED_LAG", "4")))
