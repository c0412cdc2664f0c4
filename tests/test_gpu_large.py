"""GPU parity past the single-pass kernels' 32-bit addressing, and at BenchmarkRepair's
k = 512 shape.

The reference extends and repairs any square whose shares are a multiple of 64 bytes
(leopard.go:76-99, extendeddatasquare.go:50-77); its only refusal is 2k > 65536.  The
single-pass kernels address each half of a codeword from its own 64-bit base with
32-bit offsets (rsm_kernels.hpp narrow_fits: squares up to 4 GiB), and the wide forms
(64-bit per-symbol bases; GF(2^16) through the multi-pass kernels, byte-slabbed when a
codeword's work arrays exceed the stream budget) take everything beyond.  The wide
forms are tested at small sizes through rsm_ctx_set_limits on a private context, and
at their real sizes on a 4 GiB square.  Oracle: oracle/leopard_oracle.c (parity
unpinned past k = 2).
"""
import ctypes
import os

import numpy as np
import pytest

import oracle
import rsmt2d_amd as R
from oracle import crossword

pytestmark = pytest.mark.gpu
CPU = min(16, os.cpu_count() or 1)


@pytest.fixture
def pctx(lib):
    """A private context (its limits are lowered; the shared one keeps the defaults)."""
    h = ctypes.c_void_p()
    R._check(lib.rsm_ctx_create(0, ctypes.byref(h)))
    yield h.value
    lib.rsm_ctx_destroy(h.value)


def _square(k, S, seed):
    W = 2 * k
    ods = oracle.splitmix64_bytes(k * k * S, seed=seed).reshape(k, k, S)
    full = np.zeros((W, W, S), np.uint8)
    full[:k, :k] = ods
    return ods, full


def _erase(rng, W, k, axis):
    """every row (axis 0) or column (axis 1) loses between 1 and k cells"""
    pres = np.ones((W, W), np.uint8)
    for v in range(W):
        lost = rng.choice(W, size=int(rng.integers(1, k + 1)), replace=False)
        if axis == 0:
            pres[v, lost] = 0
        else:
            pres[lost, v] = 0
    return pres


def _decode_dev(lib, ctx, dmg, pres, k, S, axis, vecs):
    W = 2 * k
    buf = R.DeviceBuffer(dmg.nbytes)
    buf.upload(dmg)
    pd = R.DeviceBuffer(W * W)
    pd.upload(pres)
    idx = R.DeviceBuffer(4 * len(vecs))
    idx.upload(np.asarray(vecs, dtype=np.uint32))
    R._check(lib.rsm_decode_vectors_dev(ctx, buf.ptr, pd.ptr, k, S, axis, idx.ptr, len(vecs), None))
    R._check(lib.rsm_sync(ctx))
    return buf.download(dmg.nbytes).reshape(dmg.shape)


# ---------------------------------------------------------------------------
# the wide forms at small sizes (forced by a lowered offset limit)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("k,S", [(1, 64), (4, 64), (64, 320), (100, 192), (128, 256),
                                 (129, 576), (300, 192), (512, 128)])
@pytest.mark.parametrize("which", ["all", "columns"])
def test_wide_extension_matches_oracle(lib, pctx, k, S, which):
    """Both passes (or only the column pass: rows stay narrow) on the wide forms; two
    squares per call (the batched layout), both against the oracle."""
    W = 2 * k
    limit = 1 if which == "all" else (k + 1) * S + S
    R._check(lib.rsm_ctx_set_limits(pctx, limit, 0))
    ods0, full0 = _square(k, S, 0x11 + k)
    ods1, full1 = _square(k, S, 0x22 + k)
    both = np.stack([full0, full1])
    buf = R.DeviceBuffer(both.nbytes)
    buf.upload(both)
    R._check(lib.rsm_extend_squares_dev(pctx, buf.ptr, k, S, 2, None))
    R._check(lib.rsm_sync(pctx))
    got = buf.download(both.nbytes).reshape(2, W, W, S)
    assert np.array_equal(got[0], oracle.extend_square(ods0, nthreads=CPU))
    assert np.array_equal(got[1], oracle.extend_square(ods1, nthreads=CPU))


@pytest.mark.parametrize("k,S", [(8, 64), (64, 192), (100, 320), (128, 256), (200, 320), (300, 320), (512, 192)])
@pytest.mark.parametrize("axis", [0, 1])
def test_wide_decode_matches_oracle(lib, pctx, k, S, axis):
    R._check(lib.rsm_ctx_set_limits(pctx, 1, 0))
    rng = np.random.default_rng(k * 11 + axis)
    W = 2 * k
    ods, _ = _square(k, S, 0x33 + k)
    full = oracle.extend_square(ods, nthreads=CPU)
    pres = _erase(rng, W, k, axis)
    got = _decode_dev(lib, pctx, full * pres[:, :, None], pres, k, S, axis, range(W))
    assert np.array_equal(got, full)


@pytest.mark.parametrize("k,S,budget", [(300, 2048, 1 << 18), (512, 704, 1 << 17), (1024, 192, 1 << 18)])
def test_gf16_byte_slabs_match_oracle(lib, pctx, k, S, budget):
    """GF(2^16) codewords whose work arrays exceed the stream budget run as byte slabs
    of their shares (a 64-byte multiple; the last slab ragged): encode and a column
    decode sweep, against the oracle."""
    R._check(lib.rsm_ctx_set_limits(pctx, 1, budget))
    W = 2 * k
    ods, full = _square(k, S, 0x44 + k)
    want = oracle.extend_square(ods, nthreads=CPU)
    buf = R.DeviceBuffer(full.nbytes)
    buf.upload(full)
    R._check(lib.rsm_extend_squares_dev(pctx, buf.ptr, k, S, 1, None))
    R._check(lib.rsm_sync(pctx))
    assert np.array_equal(buf.download(full.nbytes).reshape(W, W, S), want)
    rng = np.random.default_rng(k)
    pres = _erase(rng, W, k, 1)
    cols = sorted(rng.choice(W, size=8, replace=False).tolist())
    got = _decode_dev(lib, pctx, want * pres[:, :, None], pres, k, S, 1, cols)
    assert np.array_equal(got[:, cols], want[:, cols])


# ---------------------------------------------------------------------------
# the m = 512 single-pass decoder over many codewords; BenchmarkRepair at k = 512
# (extendeddatacrossword_test.go:407-471)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("k", [256, 300, 512])
@pytest.mark.parametrize("axis", [0, 1])
def test_gf16_decode_sweep_matches_oracle(lib, k, axis):
    """Every row (or column) of a square, each with its own random erasures, in one
    batched launch of the single-pass decoder (dec16f_kernel<256> / dec16h_kernel<512>);
    S = 320 ends on a partial 256-byte chunk."""
    S = 320
    rng = np.random.default_rng(k * 5 + axis)
    W = 2 * k
    ods, _ = _square(k, S, 0x55 + k + axis)
    full = oracle.extend_square(ods, nthreads=CPU)
    pres = _erase(rng, W, k, axis)
    got = _decode_dev(lib, R.device_context(), full * pres[:, :, None], pres, k, S, axis, range(W))
    assert np.array_equal(got, full)


def _benchmark_repair_flat(rng, original, k):
    """extendeddatacrossword_test.go:443-453: k of the 2k cells of every row erased"""
    flat = original.Flattened()
    w = 2 * k
    for r in range(w):
        for c in rng.choice(w, size=k, replace=False):
            flat[r * w + c] = None
    return flat


def test_gf16_repair_k512_benchmark_scheme(lib, rng):
    k, S = 512, 512
    ods = [bytes(x) for x in oracle.splitmix64_bytes(k * k * S, seed=0x512).reshape(k * k, S)]
    original = R.ComputeExtendedDataSquare(ods, R.NewLeoRSCodec(), R.NewDefaultTree)
    rr, cr = original.RowRoots(), original.ColRoots()
    eds = R.ImportExtendedDataSquare(_benchmark_repair_flat(rng, original, k), R.NewLeoRSCodec(), R.NewDefaultTree)
    eds.Repair(rr, cr)
    assert eds.repair_stats().fast_path == 1
    assert eds.Equals(original)


def test_gf16_repair_k512_byzantine_matches_oracle(lib, rng):
    """BenchmarkRepair's erasures plus one corrupted present share in row 1: the device
    verification rejects the fast path, and the exact solver reports the oracle
    crossword's ErrByzantineData (axis, index and the pre-repair shares)."""
    k, S = 512, 64
    ods = [bytes(x) for x in oracle.splitmix64_bytes(k * k * S, seed=0x1B).reshape(k * k, S)]
    original = R.ComputeExtendedDataSquare(ods, R.NewLeoRSCodec(), R.NewDefaultTree)
    rr, cr = original.RowRoots(), original.ColRoots()
    flat = _benchmark_repair_flat(rng, original, k)
    w = 2 * k
    c = next(c for c in range(w) if flat[w + c] is not None)
    flat[w + c] = bytes(b ^ 0xA5 for b in flat[w + c])
    try:
        crossword.repair(list(flat), rr, cr)
        want = None
    except crossword.Byzantine as b:
        want = (b.axis, b.index, b.shares)
    assert want is not None
    eds = R.ImportExtendedDataSquare(flat, R.NewLeoRSCodec(), R.NewDefaultTree)
    with pytest.raises(R.ErrByzantineData) as ei:
        eds.Repair(rr, cr)
    assert (ei.value.Axis, ei.value.Index, ei.value.Shares) == want
    assert eds.repair_stats().fast_path == 0


@pytest.mark.timeout(180)
@pytest.mark.parametrize("k,S", [(128, 256), (256, 128)])
@pytest.mark.parametrize("limits", ["columns", "all", "budget"])
def test_repair_under_lowered_limits(lib, pctx, k, S, limits):
    """BenchmarkRepair's erasures (extendeddatacrossword_test.go:443-453) repaired on a
    private context whose offset limit sends the columns (or every codeword) to the
    wide forms, or whose GF(2^16) work budget is lowered.  Results never depend on the
    limits (rsm_ctx_set_limits): the repaired square must equal the oracle's EDS.
    The "columns" case is the shape the zero-copy Repair must decline (its column
    verification would take the wide encoder's scratch lock on its own stream)."""
    W = 2 * k
    ods, _ = _square(k, S, 0x7E0 + k)
    want = oracle.extend_square(ods, nthreads=CPU)
    cells = np.ascontiguousarray(want.reshape(W * W, S))
    lens = np.full(W * W, S, np.uint32)
    rr = np.empty(W * 32, np.uint8)
    cr = np.empty(W * 32, np.uint8)
    ln = ctypes.c_uint32(0)
    h = ctypes.c_void_p()
    ptrs = _ptr_array(cells)  # (held: the C call reads it)
    R._check(lib.rsm_eds_import(R.device_context(), ptrs.ctypes.data, lens.ctypes.data, W * W, ctypes.byref(h)))
    try:
        R._check(lib.rsm_eds_roots(h, 0, None, None, rr.ctypes.data, 32, ctypes.byref(ln)))
        R._check(lib.rsm_eds_roots(h, 1, None, None, cr.ctypes.data, 32, ctypes.byref(ln)))
    finally:
        lib.rsm_eds_free(h)
    limit = {"columns": (k + 1) * S + S, "all": 1, "budget": 0}[limits]
    budget = 1 << 16 if limits == "budget" else 0
    R._check(lib.rsm_ctx_set_limits(pctx, limit, budget))
    rng = np.random.default_rng(k + len(limits))
    pres = np.ones((W, W), np.uint8)
    for r in range(W):
        pres[r, rng.choice(W, size=k, replace=False)] = 0
    ptrs = _ptr_array(cells, pres.reshape(-1))
    h = ctypes.c_void_p()
    R._check(lib.rsm_eds_import(pctx, ptrs.ctypes.data, lens.ctypes.data, W * W, ctypes.byref(h)))
    try:
        byz = R._Byz()
        R._check(lib.rsm_eds_repair(h, rr.ctypes.data, cr.ctypes.data, 32, None, None, ctypes.byref(byz)))
        got = np.empty_like(want)
        R._check(lib.rsm_eds_flattened(h, got.ctypes.data, None))
        assert np.array_equal(got, want)
        st = R.RepairStats()
        R._check(lib.rsm_eds_repair_stats(h, ctypes.byref(st)))
        assert (st.fast_path, st.fallback_reason) == (1, 0)
    finally:
        lib.rsm_eds_free(h)


# ---------------------------------------------------------------------------
# squares of 2 GiB and more (the round-4 build refused these with RSM_EUNSUPPORTED)
# ---------------------------------------------------------------------------
def _check_sampled(eds, k, rows, cols):
    """row r: parity half == oracle.encode(data half); column c likewise"""
    for r in rows:
        data = [eds[r, i].tobytes() for i in range(k)]
        assert oracle.encode(data) == [eds[r, k + i].tobytes() for i in range(k)], ("row", r)
    for c in cols:
        data = [eds[i, c].tobytes() for i in range(k)]
        assert oracle.encode(data) == [eds[k + i, c].tobytes() for i in range(k)], ("col", c)


def _ptr_array(arr, present=None):
    n, S = arr.shape[0], arr.shape[1]
    p = np.arange(n, dtype=np.uint64) * np.uint64(S) + np.uint64(arr.ctypes.data)
    if present is not None:
        p[present == 0] = 0
    return p


def test_k512_s2048_square(lib):
    """k = 512, 2 KiB shares (a 2 GiB EDS): device extension (single-pass, rebased halves),
    ComputeExtendedDataSquare through the host path, a row and a column decode sweep
    and the DefaultTree Repair in BenchmarkRepair's scheme."""
    k, S = 512, 2048
    W = 2 * k
    ctx = R.device_context()
    ods, full = _square(k, S, 0x2048)
    buf = R.DeviceBuffer(full.nbytes)
    buf.upload(full)
    R._check(lib.rsm_extend_squares_dev(ctx, buf.ptr, k, S, 1, None))
    R._check(lib.rsm_sync(ctx))
    eds = buf.download(full.nbytes).reshape(W, W, S)
    assert np.array_equal(eds[:k, :k], ods)
    _check_sampled(eds, k, rows=[0, 1, 511, 512, 1023], cols=[0, 510, 511, 512, 1023])
    # rsm_eds_compute (host in, host out): the same square
    cells = np.ascontiguousarray(ods.reshape(k * k, S))
    ptrs = _ptr_array(cells)
    lens = np.full(k * k, S, np.uint32)
    h = ctypes.c_void_p()
    R._check(lib.rsm_eds_compute(ctx, ptrs.ctypes.data, lens.ctypes.data, k * k, ctypes.byref(h)))
    try:
        got = np.empty_like(eds)
        R._check(lib.rsm_eds_flattened(h, got.ctypes.data, None))
        assert np.array_equal(got, eds)
    finally:
        lib.rsm_eds_free(h)
    # decode sweeps: 6 rows and 6 columns with k cells each lost
    rng = np.random.default_rng(0x2048)
    for axis in (0, 1):
        vecs = sorted(rng.choice(W, size=6, replace=False).tolist())
        pres = np.ones((W, W), np.uint8)
        for v in vecs:
            lost = rng.choice(W, size=k, replace=False)
            if axis == 0:
                pres[v, lost] = 0
            else:
                pres[lost, v] = 0
        dmg = eds * pres[:, :, None]
        got = _decode_dev(lib, ctx, dmg, pres, k, S, axis, vecs)
        assert np.array_equal(got, eds), axis
        del dmg, got
    # Repair (DefaultTree, roots on the device): k of every row's 2k cells erased
    cells = eds.reshape(W * W, S)
    lens = np.full(W * W, S, np.uint32)
    h = ctypes.c_void_p()
    ptrs = _ptr_array(cells)  # (held: the C call reads it)
    R._check(lib.rsm_eds_import(ctx, ptrs.ctypes.data, lens.ctypes.data, W * W, ctypes.byref(h)))
    rr = np.empty(W * 32, np.uint8)
    cr = np.empty(W * 32, np.uint8)
    ln = ctypes.c_uint32(0)
    try:
        R._check(lib.rsm_eds_roots(h, 0, None, None, rr.ctypes.data, 32, ctypes.byref(ln)))
        R._check(lib.rsm_eds_roots(h, 1, None, None, cr.ctypes.data, 32, ctypes.byref(ln)))
    finally:
        lib.rsm_eds_free(h)
    pres = np.ones((W, W), np.uint8)
    for r in range(W):
        pres[r, rng.choice(W, size=k, replace=False)] = 0
    h = ctypes.c_void_p()
    ptrs = _ptr_array(cells, pres.reshape(-1))
    R._check(lib.rsm_eds_import(ctx, ptrs.ctypes.data, lens.ctypes.data, W * W, ctypes.byref(h)))
    try:
        byz = R._Byz()
        R._check(lib.rsm_eds_repair(h, rr.ctypes.data, cr.ctypes.data, 32, None, None, ctypes.byref(byz)))
        st = R.RepairStats()
        R._check(lib.rsm_eds_repair_stats(h, ctypes.byref(st)))
        assert st.fast_path == 1
        got = np.empty_like(eds)
        R._check(lib.rsm_eds_flattened(h, got.ctypes.data, None))
        assert np.array_equal(got, eds)
    finally:
        lib.rsm_eds_free(h)


def test_k128_s32768_square(lib):
    """A 2 GiB GF(2^8) square (k = 128, 32 KiB shares): one square takes the latency
    form (split encoder, rebased halves), a batch of two the two-pass byte-table
    launches; the whole square against the oracle."""
    k, S = 128, 32768
    W = 2 * k
    ods, full = _square(k, S, 0x8000)
    want = oracle.extend_square(ods, nthreads=CPU)
    got = np.empty_like(want)
    R._check(lib.rsm_extend_square(R.device_context(), ods.ctypes.data, k, S, got.ctypes.data))
    assert np.array_equal(got, want)
    rng = np.random.default_rng(7)
    pres = _erase(rng, W, k, 1)
    vecs = sorted(rng.choice(W, size=12, replace=False).tolist())
    keep = np.ones((W, W), np.uint8)
    keep[:, vecs] = pres[:, vecs]
    got = _decode_dev(lib, R.device_context(), want * keep[:, :, None], keep, k, S, 1, vecs)
    assert np.array_equal(got, want)


def test_k128_s65536_square_wide(lib):
    """A 4 GiB GF(2^8) square (k = 128, 64 KiB shares): its column halves span 2 GiB, so
    the column pass and column decodes run on the wide forms at their real size."""
    k, S = 128, 65536
    W = 2 * k
    ctx = R.device_context()
    ods, full = _square(k, S, 0x10000)
    buf = R.DeviceBuffer(full.nbytes)
    buf.upload(full)
    del full
    R._check(lib.rsm_extend_squares_dev(ctx, buf.ptr, k, S, 1, None))
    R._check(lib.rsm_sync(ctx))
    want = oracle.extend_square(ods, nthreads=CPU)
    got = buf.download(want.nbytes).reshape(W, W, S)
    assert np.array_equal(got, want)
    del got
    rng = np.random.default_rng(9)
    vecs = [0, 127, 128, 255]
    pres = np.ones((W, W), np.uint8)
    for v in vecs:
        pres[rng.choice(W, size=k, replace=False), v] = 0
    got = _decode_dev(lib, ctx, want * pres[:, :, None], pres, k, S, 1, vecs)
    assert np.array_equal(got, want)
