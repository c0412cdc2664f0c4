"""Fused two-pass extension kernel (encode_gf8_bs128f_kernel, one launch per batch).

The production k = 128 path of rsm_extend_squares_dev runs the row pass
(erasureExtendRow, extendeddatasquare.go:228-233) and the column pass
(erasureExtendCol, :235-243) in ONE launch whose column sets wait on per-square
counters of completed row sets.  Checked bit-exact against the oracle (one
square) and against the two-launch form (rsm_extend_squares_phase_dev 1 then 2)
over batches, lags and concurrent streams.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle
import rsmt2d_amd as R

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(autouse=True)
def fused_on():
    L = R.library()
    prev = L.rsm_set_fused(1)
    yield
    L.rsm_set_fused(prev)


def _square_bytes(k, S):
    return (2 * k) ** 2 * S


def _quadrant_report(got, want, k):
    bad = got != want
    return {q: int(bad[r0:r0 + k, c0:c0 + k].any(axis=2).sum())
            for q, (r0, c0) in {"Q0": (0, 0), "Q1": (0, k), "Q2": (k, 0), "Q3": (k, k)}.items()}


def _two_launch(L, ctx, buf, k, S, count):
    R._check(L.rsm_extend_squares_phase_dev(ctx, buf.ptr, k, S, count, 1, None))
    R._check(L.rsm_extend_squares_phase_dev(ctx, buf.ptr, k, S, count, 2, None))
    R._check(L.rsm_sync(ctx))


def _fused(L, ctx, buf, k, S, count, stream=None):
    R._check(L.rsm_extend_squares_dev(ctx, buf.ptr, k, S, count, stream))


def test_fused_is_selected():
    L = R.library()
    assert L.rsm_set_fused(0) == 1
    assert L.rsm_extend_fused(128, 512) == 0
    L.rsm_set_fused(1)
    assert L.rsm_extend_fused(128, 512) == 1
    assert L.rsm_extend_fused(128, 64) == 1
    assert L.rsm_extend_fused(64, 512) == 0
    assert L.rsm_extend_fused(100, 512) == 0


@pytest.mark.parametrize("S", [64, 512])
def test_fused_one_square_matches_oracle(S):
    L = R.library()
    ctx = R.device_context(0)
    k = 128
    rng = np.random.default_rng(7 + S)
    ods = rng.integers(0, 256, (k, k, S), dtype=np.uint8)
    buf = R.DeviceBuffer(_square_bytes(k, S))
    buf.fill_random(99)  # garbage in Q1..Q3
    R._check(L.rsm_sync(ctx))  # fill runs on the ctx stream; rsm_memcpy does not order with it
    sq = np.empty((2 * k, 2 * k, S), np.uint8)
    sq[:] = buf.download().reshape(sq.shape)
    sq[:k, :k] = ods
    buf.upload(sq)
    _fused(L, ctx, buf, k, S, 1)
    R._check(L.rsm_sync(ctx))
    got = buf.download().reshape(2 * k, 2 * k, S)
    want = oracle.extend_square(ods, nthreads=8)
    assert (got == want).all(), _quadrant_report(got, want, k)
    buf.free()


@pytest.mark.parametrize("count,S", [(2, 512), (5, 512), (16, 512), (24, 64), (3, 128)])
def test_fused_batch_matches_two_launch(count, S):
    L = R.library()
    ctx = R.device_context(0)
    k = 128
    n = _square_bytes(k, S) * count
    a, b = R.DeviceBuffer(n), R.DeviceBuffer(n)
    a.fill_random(1234 + count)
    R._check(L.rsm_sync(ctx))
    R._check(L.rsm_memcpy(ctx, b.ptr, a.ptr, n, 2))
    R._check(L.rsm_sync(ctx))
    _two_launch(L, ctx, a, k, S, count)
    for _ in range(3):  # repeated launches reuse the self-reset queue
        _fused(L, ctx, b, k, S, count)
    R._check(L.rsm_sync(ctx))
    ga, gb = a.download(), b.download()
    if not (ga == gb).all():
        bad = (ga != gb).reshape(count, 2 * k, 2 * k, S).any(axis=3)
        pytest.fail("mismatching cells per square: %s" % bad.reshape(count, -1).sum(axis=1).tolist())
    a.free()
    b.free()


def test_fused_two_streams_concurrently():
    L = R.library()
    ctx = R.device_context(0)
    k, S, count = 128, 512, 8
    n = _square_bytes(k, S) * count
    bufs = [R.DeviceBuffer(n) for _ in range(3)]
    bufs[0].fill_random(5)
    R._check(L.rsm_sync(ctx))
    for b in bufs[1:]:
        R._check(L.rsm_memcpy(ctx, b.ptr, bufs[0].ptr, n, 2))
    R._check(L.rsm_sync(ctx))
    s2 = ctypes.c_void_p()
    R._check(L.rsm_stream_create(ctx, ctypes.byref(s2)))
    for _ in range(4):
        _fused(L, ctx, bufs[1], k, S, count)
        _fused(L, ctx, bufs[2], k, S, count, s2)
    R._check(L.rsm_stream_sync(s2))
    R._check(L.rsm_sync(ctx))
    _two_launch(L, ctx, bufs[0], k, S, count)
    ref = bufs[0].download()
    assert (bufs[1].download() == ref).all()
    assert (bufs[2].download() == ref).all()
    R._check(L.rsm_stream_destroy(ctx, s2))
    for b in bufs:
        b.free()


@pytest.mark.parametrize("lag", ["1", "2", "16"])
def test_fused_lag_variants(lag):
    # RSM_FUSED_LAG is read once per process: run each lag in a child process
    code = (
        "import numpy as np, rsmt2d_amd as R\n"
        "L=R.library(); ctx=R.device_context(0); k,S,c=128,512,6\n"
        "n=(2*k)**2*S*c; a=R.DeviceBuffer(n); b=R.DeviceBuffer(n); a.fill_random(77); R._check(L.rsm_sync(ctx))\n"
        "R._check(L.rsm_memcpy(ctx,b.ptr,a.ptr,n,2)); R._check(L.rsm_sync(ctx))\n"
        "R._check(L.rsm_extend_squares_phase_dev(ctx,a.ptr,k,S,c,1,None))\n"
        "R._check(L.rsm_extend_squares_phase_dev(ctx,a.ptr,k,S,c,2,None))\n"
        "R._check(L.rsm_extend_squares_dev(ctx,b.ptr,k,S,c,None)); R._check(L.rsm_sync(ctx))\n"
        "assert (a.download()==b.download()).all()\n"
    )
    env = dict(os.environ, RSM_FUSED="1", RSM_FUSED_LAG=lag, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, timeout=100)
    assert r.returncode == 0
