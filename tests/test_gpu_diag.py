"""Diagnostic library (librsmt2d_hip_diag.so, -DRSM_DIAG): the A-B kernels kept for
measurements -- the fused single-launch extension and the software-pipelined dual
launch -- must still match the production two-launch form bit for bit.  The
product library contains neither (tests/test_capi_cpu.py::test_product_has_no_diagnostics).
"""
import ctypes

import numpy as np
import pytest

import oracle
import rsmt2d_amd as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dl():
    return R.diag_library()


def _ctx(dl):
    h = ctypes.c_void_p()
    R._check_with(dl, dl.rsm_ctx_create(0, ctypes.byref(h)))
    return h.value


def _buf(dl, ctx, n):
    p = ctypes.c_void_p()
    R._check_with(dl, dl.rsm_dev_alloc(ctx, n, ctypes.byref(p)))
    return p.value


def _down(dl, ctx, ptr, n):
    out = np.empty(n, np.uint8)
    R._check_with(dl, dl.rsm_memcpy(ctx, out.ctypes.data, ptr, n, 1))
    return out


@pytest.mark.parametrize("count,S,lag", [(1, 512, 0), (1, 512, 1), (3, 512, 2), (4, 64, 4), (9, 512, 2),
                                         (40, 512, 0), (2, 1024, 1), (5, 192, 3)])
def test_fused_matches_two_launch(dl, count, S, lag):
    """Queue-driven single launch (extend_gf8_bs128q_kernel) == the two-launch
    production schedule, bit for bit, twice on the same (self-re-zeroed) queue words."""
    k = 128
    n = (2 * k) ** 2 * S * count
    ctx = _ctx(dl)
    src, a, b = _buf(dl, ctx, n), _buf(dl, ctx, n), _buf(dl, ctx, n)
    R._check_with(dl, dl.rsm_dev_fill_random(ctx, src, n, 91 + count))
    R._check_with(dl, dl.rsm_sync(ctx))
    R._check_with(dl, dl.rsm_memcpy(ctx, a, src, n, 2))
    R._check_with(dl, dl.rsm_extend_squares_dev(ctx, a, k, S, count, None))
    R._check_with(dl, dl.rsm_sync(ctx))
    ga = _down(dl, ctx, a, n)
    sq = ga[: (2 * k) ** 2 * S].reshape(2 * k, 2 * k, S)
    assert np.array_equal(sq, oracle.extend_square(sq[:k, :k].copy(), nthreads=8))
    for _ in range(2):
        R._check_with(dl, dl.rsm_memcpy(ctx, b, src, n, 2))
        R._check_with(dl, dl.rsm_sync(ctx))
        R._check_with(dl, dl.rsm_diag_extend_fused(ctx, b, k, S, count, lag, None))
        R._check_with(dl, dl.rsm_diag_queue_check(ctx, None))
        R._check_with(dl, dl.rsm_sync(ctx))
        assert np.array_equal(ga, _down(dl, ctx, b, n))
    for p in (src, a, b):
        dl.rsm_dev_free(ctx, p)
    dl.rsm_ctx_destroy(ctx)


def test_pipeline_matches_two_launch(dl):
    k, S, count = 128, 512, 2
    n = (2 * k) ** 2 * S * count
    ctx = _ctx(dl)
    ref, x0, x1 = _buf(dl, ctx, n), _buf(dl, ctx, n), _buf(dl, ctx, n)
    R._check_with(dl, dl.rsm_dev_fill_random(ctx, ref, n, 5))
    R._check_with(dl, dl.rsm_sync(ctx))
    for x in (x0, x1):
        R._check_with(dl, dl.rsm_memcpy(ctx, x, ref, n, 2))
    R._check_with(dl, dl.rsm_extend_squares_dev(ctx, ref, k, S, count, None))
    # launch 0: rows of x0; launch 1: rows of x1 + columns of x0; launch 2: columns of x1
    R._check_with(dl, dl.rsm_diag_extend_pipeline_dev(ctx, x0, None, k, S, count, None))
    R._check_with(dl, dl.rsm_diag_extend_pipeline_dev(ctx, x1, x0, k, S, count, None))
    R._check_with(dl, dl.rsm_diag_extend_pipeline_dev(ctx, None, x1, k, S, count, None))
    R._check_with(dl, dl.rsm_sync(ctx))
    want = _down(dl, ctx, ref, n)
    assert np.array_equal(_down(dl, ctx, x0, n), want)
    assert np.array_equal(_down(dl, ctx, x1, n), want)
    for p in (ref, x0, x1):
        dl.rsm_dev_free(ctx, p)
    dl.rsm_ctx_destroy(ctx)


@pytest.mark.parametrize("k,S", [(128, 512), (100, 320)])
def test_split_one_launch_form(dl, k, S):
    """The latency form's one-launch variant (diagnostic: Q1-column workgroups wait on
    64 replicated done flags, wave priorities) == the two-launch latency form and the
    oracle, three times on the same self-re-zeroed words."""
    n = (2 * k) ** 2 * S
    ctx = _ctx(dl)
    src, a, b = _buf(dl, ctx, n), _buf(dl, ctx, n), _buf(dl, ctx, n)
    R._check_with(dl, dl.rsm_dev_fill_random(ctx, src, n, 77))
    R._check_with(dl, dl.rsm_sync(ctx))
    R._check_with(dl, dl.rsm_memcpy(ctx, a, src, n, 2))
    R._check_with(dl, dl.rsm_diag_set_split_fused(0))
    R._check_with(dl, dl.rsm_extend_squares_dev(ctx, a, k, S, 1, None))
    R._check_with(dl, dl.rsm_sync(ctx))
    ga = _down(dl, ctx, a, n)
    sq = ga.reshape(2 * k, 2 * k, S)
    assert np.array_equal(sq, oracle.extend_square(sq[:k, :k].copy(), nthreads=8))
    try:
        R._check_with(dl, dl.rsm_diag_set_split_fused(1))
        for _ in range(3):
            R._check_with(dl, dl.rsm_memcpy(ctx, b, src, n, 2))
            R._check_with(dl, dl.rsm_extend_squares_dev(ctx, b, k, S, 1, None))
            R._check_with(dl, dl.rsm_diag_queue_check(ctx, None))
            R._check_with(dl, dl.rsm_sync(ctx))
            assert np.array_equal(ga, _down(dl, ctx, b, n))
    finally:
        R._check_with(dl, dl.rsm_diag_set_split_fused(0))
    for p in (src, a, b):
        dl.rsm_dev_free(ctx, p)
    dl.rsm_ctx_destroy(ctx)


@pytest.mark.parametrize("G,k,S", [(2, 192, 64), (2, 256, 192), (4, 256, 512), (4, 384, 128), (8, 256, 64),
                                   (8, 512, 128), (8, 512, 512), (2, 512, 256)])
def test_alltoall_without_copies(dl, G, k, S):
    """The copy-free all-to-all of rsm_multi_extend_dev (RSM_SCHED_ALLTOALL) with G ranks
    emulated on one GPU: the row pass's side output into the send blocks and the column
    pass's blocked input from the receive blocks leave every rank's rows of the top half
    and the bottom half of its column slice equal to the single-GPU extension (and the
    oracle).  Every rank's buffer holds garbage outside its own Q0 rows, so a read of
    another rank's rows from the square instead of the received blocks shows up."""
    W = 2 * k
    row = W * S
    n = W * row
    rk, ck = k // G, W // G
    ctx = _ctx(dl)
    src = _buf(dl, ctx, n)
    R._check_with(dl, dl.rsm_dev_fill_random(ctx, src, n, 7 * G + k))
    R._check_with(dl, dl.rsm_sync(ctx))
    ranks = []
    for g in range(G):
        b = _buf(dl, ctx, n)
        R._check_with(dl, dl.rsm_dev_fill_random(ctx, b, n, 1000 + g))
        R._check_with(dl, dl.rsm_sync(ctx))
        R._check_with(dl, dl.rsm_memcpy(ctx, b + g * rk * row, src + g * rk * row, rk * row, 2))
        ranks.append(b)
    R._check_with(dl, dl.rsm_extend_squares_dev(ctx, src, k, S, 1, None))
    arr = (ctypes.c_void_p * G)(*ranks)
    R._check_with(dl, dl.rsm_diag_alltoall_emulated(ctx, arr, G, k, S))
    R._check_with(dl, dl.rsm_sync(ctx))
    want = _down(dl, ctx, src, n).reshape(W, W, S)
    if k * S <= 192 * 64:
        assert np.array_equal(want, oracle.extend_square(want[:k, :k].copy(), nthreads=8))
    for g, b in enumerate(ranks):
        got = _down(dl, ctx, b, n).reshape(W, W, S)
        assert np.array_equal(got[g * rk:(g + 1) * rk], want[g * rk:(g + 1) * rk]), f"rank {g}: top-half rows"
        sl = slice(g * ck, (g + 1) * ck)
        assert np.array_equal(got[k:, sl], want[k:, sl]), f"rank {g}: bottom half of its column slice"
    for p in [src] + ranks:
        dl.rsm_dev_free(ctx, p)
    dl.rsm_ctx_destroy(ctx)


@pytest.mark.parametrize("k,S,count,waves", [(128, 512, 1, (16, 16)), (100, 320, 1, (16, 8)), (128, 512, 3, (8, 16)),
                                              (65, 64, 2, (16, 16))])
def test_split16_latency_form(dl, k, S, count, waves):
    """The 16-wave latency form (three layouts, four exchanges; diagnostic) == the oracle."""
    W = 2 * k
    n = W * W * S * count
    ctx = _ctx(dl)
    a = _buf(dl, ctx, n)
    R._check_with(dl, dl.rsm_dev_fill_random(ctx, a, n, 1600 + k))
    R._check_with(dl, dl.rsm_sync(ctx))
    try:
        R._check_with(dl, dl.rsm_diag_set_split_waves(*waves))
        R._check_with(dl, dl.rsm_extend_squares_dev(ctx, a, k, S, count, None))
        R._check_with(dl, dl.rsm_sync(ctx))
    finally:
        R._check_with(dl, dl.rsm_diag_set_split_waves(0, 0))
    got = _down(dl, ctx, a, n).reshape(count, W, W, S)
    for c in range(count):
        assert np.array_equal(got[c], oracle.extend_square(got[c, :k, :k].copy(), nthreads=8)), c
    dl.rsm_dev_free(ctx, a)
    dl.rsm_ctx_destroy(ctx)
