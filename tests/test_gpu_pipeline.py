"""Software-pipelined batches (rsm_extend_pipeline_dev, encode_gf8_bs128p_kernel).

One launch runs the row pass (erasureExtendRow, extendeddatasquare.go:228-233) of
one batch and the column pass (erasureExtendCol, :235-243) of another; a batch is
extended by its row call followed by its column call.  Checked bit-exact against
the two-launch form and, for one square, the oracle.
"""
import numpy as np
import pytest

import oracle
import rsmt2d_amd as R

pytestmark = pytest.mark.gpu


def _bufs(L, ctx, k, S, count, n, seed):
    size = (2 * k) ** 2 * S * count
    out = [R.DeviceBuffer(size) for _ in range(n)]
    for i, b in enumerate(out):
        b.fill_random(seed + i)
    R._check(L.rsm_sync(ctx))
    return out


@pytest.mark.parametrize("k,S,count", [(128, 512, 16), (128, 64, 5), (100, 512, 3), (64, 512, 2)])
def test_pipeline_matches_two_launch(k, S, count):
    L = R.library()
    ctx = R.device_context(0)
    nb = 3
    work = _bufs(L, ctx, k, S, count, nb, 500 + k)
    ref = _bufs(L, ctx, k, S, count, nb, 500 + k)
    for b in ref:
        R._check(L.rsm_extend_squares_phase_dev(ctx, b.ptr, k, S, count, 1, None))
        R._check(L.rsm_extend_squares_phase_dev(ctx, b.ptr, k, S, count, 2, None))
    # call i: rows of batch i, columns of batch i - 1
    for i in range(nb + 1):
        rows = work[i].ptr if i < nb else None
        cols = work[i - 1].ptr if i > 0 else None
        R._check(L.rsm_extend_pipeline_dev(ctx, rows, cols, k, S, count, None))
    R._check(L.rsm_sync(ctx))
    for w, r in zip(work, ref):
        assert (w.download() == r.download()).all()
    for b in work + ref:
        b.free()


def test_pipeline_one_square_matches_oracle():
    L = R.library()
    ctx = R.device_context(0)
    k, S = 128, 512
    rng = np.random.default_rng(3)
    ods = [rng.integers(0, 256, (k, k, S), dtype=np.uint8) for _ in range(2)]
    bufs = []
    for o in ods:
        b = R.DeviceBuffer((2 * k) ** 2 * S)
        sq = np.zeros((2 * k, 2 * k, S), np.uint8)
        sq[:k, :k] = o
        b.upload(sq)
        bufs.append(b)
    R._check(L.rsm_extend_pipeline_dev(ctx, bufs[0].ptr, None, k, S, 1, None))
    R._check(L.rsm_extend_pipeline_dev(ctx, bufs[1].ptr, bufs[0].ptr, k, S, 1, None))
    R._check(L.rsm_extend_pipeline_dev(ctx, None, bufs[1].ptr, k, S, 1, None))
    R._check(L.rsm_sync(ctx))
    for o, b in zip(ods, bufs):
        assert (b.download().reshape(2 * k, 2 * k, S) == oracle.extend_square(o, nthreads=8)).all()
        b.free()


def test_pipeline_rejects_bad_arguments():
    L = R.library()
    ctx = R.device_context(0)
    assert L.rsm_extend_pipeline_dev(ctx, None, None, 128, 512, 1, None) != 0
    b = R.DeviceBuffer(256 * 256 * 64)
    assert L.rsm_extend_pipeline_dev(ctx, b.ptr, None, 128, 100, 1, None) != 0  # S % 64
    b.free()
