"""Measurement-script correctness check WITHOUT the oracle (only tests/, smoke() and
bench.py's cpu_baseline may use oracle/): a square is re-extended from its Q0 by the
product's two-launch path (rsm_extend_squares_phase_dev, phases 1 then 2 -- the form
tests/ check bit-exact against the oracle) and compared byte for byte."""
import ctypes

import numpy as np

import rsmt2d_amd as R


def matches_two_launch(L, ctx, sq, k):
    """sq: (2k, 2k, S) uint8 host array of an extended square."""
    W, S = sq.shape[0], sq.shape[2]
    ref = np.zeros_like(sq)
    ref[:k, :k] = sq[:k, :k]
    buf = R.DeviceBuffer(ref.nbytes)
    buf.upload(ref.reshape(-1))
    R._check_with(L, L.rsm_extend_squares_phase_dev(ctx, buf.ptr, k, S, 1, 1, None))
    R._check_with(L, L.rsm_extend_squares_phase_dev(ctx, buf.ptr, k, S, 1, 2, None))
    R._check_with(L, L.rsm_sync(ctx))
    want = buf.download(ref.nbytes).reshape(W, W, S)
    buf.free()
    return bool(np.array_equal(sq, want))
