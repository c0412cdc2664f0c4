"""Phase timeline of the M = 128 split decoder (diagnostic library, decode trace).

The c3 decode-sweep shape of bench.py (k = 128, S = 512, all 256 rows of an EDS with
128 of their 256 cells erased, one rsm_decode_vectors_dev launch = 512 workgroups):
thread 0 of every workgroup stamps the 100 MHz clock at 8 points of
decode_split_task (kernels_gf8.hip dec_stamp); prints the mean phase durations and
the launch span in us.
usage: python3 scripts/diag/trace_decode.py
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
NAMES = ["presence+ballot", "errloc+tables+sync", "scale+IFFT low", "S->L+IFFT high+deriv",
         "FFT high+L->S", "FFT low", "reveal+stores issued"]


def chk(rc):
    R._check_with(D, rc)


def main():
    k, S = 128, 512
    W = 2 * k
    ctx = ctypes.c_void_p()
    chk(D.rsm_ctx_create(0, ctypes.byref(ctx)))
    rng = np.random.default_rng(7)
    buf = R.DeviceBuffer(W * W * S)
    host = np.zeros((W, W, S), np.uint8)
    host[:k, :k] = rng.integers(0, 256, (k, k, S), dtype=np.uint8)
    buf.upload(host.reshape(-1))
    chk(D.rsm_extend_squares_dev(ctx, buf.ptr, k, S, 1, None))
    chk(D.rsm_sync(ctx))
    full = buf.download(W * W * S).reshape(W, W, S)
    present = np.ones((W, W), np.uint8)
    for r in range(W):
        present[r, rng.choice(W, size=k, replace=False)] = 0
    pres_d = R.DeviceBuffer(W * W)
    pres_d.upload(present)
    idx_d = R.DeviceBuffer(4 * W)
    idx_d.upload(np.arange(W, dtype=np.uint32))
    tasks = W * (S // 256)
    tr = R.DeviceBuffer(tasks * 8 * 4)
    out = {}
    for rep in range(3):
        buf.upload((full * present[:, :, None]).reshape(-1))
        chk(D.rsm_sync(ctx))
        chk(D.rsm_diag_set_dec_trace(tr.ptr if rep == 2 else None))
        chk(D.rsm_decode_vectors_dev(ctx, buf.ptr, pres_d.ptr, k, S, 0, idx_d.ptr, W, None))
        chk(D.rsm_sync(ctx))
    chk(D.rsm_diag_set_dec_trace(None))
    assert np.array_equal(buf.download(W * W * S).reshape(W, W, S), full)
    st = tr.download(tasks * 32).view(np.uint32).reshape(tasks, 8).astype(np.int64)
    st -= st[:, :1].min()
    d = np.diff(st, axis=1) * 0.01  # us
    out["phases_us_mean"] = {n: round(float(d[:, i].mean()), 3) for i, n in enumerate(NAMES)}
    out["task_us_mean"] = round(float((st[:, 7] - st[:, 0]).mean() * 0.01), 3)
    out["start_spread_us"] = round(float((st[:, 0].max() - st[:, 0].min()) * 0.01), 3)
    out["launch_span_us"] = round(float((st[:, 7].max() - st[:, 0].min()) * 0.01), 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
