"""GPU: the runtime around the kernels -- concurrent Codec callers, per-stream
scratch, per-context grid caps, the pinned host-memory path and the multi-GPU C
ABI (rsm_multi_*, RCCL from C++) -- each result checked bit-exact against the
CPU oracle."""
import ctypes
import threading

import numpy as np
import pytest

import oracle
import rsmt2d_amd as R

pytestmark = pytest.mark.gpu


def _encode_args(data, parity):
    k, S = data.shape
    dp = (ctypes.c_void_p * k)(*[data.ctypes.data + i * S for i in range(k)])
    pp = (ctypes.c_void_p * k)(*[parity.ctypes.data + i * S for i in range(k)])
    return dp, pp


def test_concurrent_codec_callers(lib):
    """64 host threads call Encode and Decode at once on ONE context (rsmt2d calls
    the Codec from up to 2k goroutines, extendeddatasquare.go:186-224); every result
    equals the oracle's."""
    ctx = R.device_context(0)
    S = 512
    rng = np.random.default_rng(64)
    jobs = []
    for t in range(64):
        k = [128, 64, 100, 37, 128, 256][t % 6]  # GF(2^8) and GF(2^16) callers mixed
        data = rng.integers(0, 256, (k, S), dtype=np.uint8)
        want = np.frombuffer(b"".join(oracle.encode([bytes(r) for r in data])), np.uint8).reshape(k, S)
        jobs.append((k, data, want))
    errors = []

    def worker(t):
        k, data, want = jobs[t]
        try:
            for it in range(4):
                par = np.zeros((k, S), np.uint8)
                dp, pp = _encode_args(data, par)
                rc = lib.rsm_encode(ctx, dp, k, S, pp)
                if rc or not np.array_equal(par, want):
                    errors.append(("encode", t, it, rc))
                    return
                full = np.concatenate([data, want])
                pres = np.ones(2 * k, np.uint8)
                lost = np.random.default_rng(1000 * t + it).choice(2 * k, size=k, replace=False)
                pres[lost] = 0
                work = full.copy()
                work[lost] = 0
                ptrs = (ctypes.c_void_p * (2 * k))(*[work.ctypes.data + i * S for i in range(2 * k)])
                rc = lib.rsm_decode(ctx, ptrs, pres.ctypes.data, 2 * k, S)
                if rc or not np.array_equal(work, full):
                    errors.append(("decode", t, it, rc))
                    return
        except Exception as e:  # pragma: no cover - reported below
            errors.append(("exception", t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(64)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=100)
    assert not any(x.is_alive() for x in th), "a Codec caller hung"
    assert not errors, errors[:5]


def test_streams_own_their_scratch(lib):
    """Device roots and GF(2^16) extensions queued at once on different streams
    (each with its own leaf / work-array scratch) match the one-stream results."""
    ctx = R.device_context(0)
    k, S, W = 256, 128, 512
    n = W * W * S
    bufs = [R.DeviceBuffer(n) for _ in range(2)]
    for i, b in enumerate(bufs):
        b.fill_random(300 + i)
    R._check(lib.rsm_sync(ctx))
    ods = [b.download(n).reshape(W, W, S)[:k, :k].copy() for b in bufs]
    roots = [R.DeviceBuffer(2 * W * 32) for _ in range(2)]
    st = [ctypes.c_void_p() for _ in range(2)]
    for s in st:
        R._check(lib.rsm_stream_create(ctx, ctypes.byref(s)))
    for i in range(2):
        R._check(lib.rsm_extend_squares_dev(ctx, bufs[i].ptr, k, S, 1, st[i]))
        R._check(lib.rsm_roots_dev(ctx, bufs[i].ptr, W, S, roots[i].ptr, st[i]))
    for s in st:
        R._check(lib.rsm_stream_sync(s))
    for i in range(2):
        got = bufs[i].download(n).reshape(W, W, S)
        assert np.array_equal(got, oracle.extend_square(ods[i], nthreads=8))
        cells = [bytes(got[r, c]) for r in range(W) for c in range(W)]
        e = R.ImportExtendedDataSquare(cells, R.NewLeoRSCodec(), R.NewDefaultTree)
        rr = roots[i].download(2 * W * 32)
        assert bytes(rr[: W * 32]) == b"".join(e.RowRoots())
    for s in st:
        R._check(lib.rsm_stream_destroy(ctx, s))


@pytest.mark.parametrize("cap", [1, 7, 224])
def test_pass_grid_caps_do_not_change_results(lib, cap):
    """rsm_ctx_set_pass_grid only reshapes the persistent grid."""
    ctx = R.device_context(0)
    k, S, B = 128, 512, 2
    n = (2 * k) ** 2 * S * B
    b = R.DeviceBuffer(n)
    b.fill_random(cap)
    R._check(lib.rsm_sync(ctx))
    prev = ctypes.c_int()
    for p in (0, 1):
        R._check(lib.rsm_ctx_set_pass_grid(ctx, p, cap, ctypes.byref(prev) if p == 0 else None))
    try:
        # the two-launch form (row pass, column pass): the single-launch batch path
        # always runs on every CU
        R._check(lib.rsm_extend_squares_phase_dev(ctx, b.ptr, k, S, B, 1, None))
        R._check(lib.rsm_extend_squares_phase_dev(ctx, b.ptr, k, S, B, 2, None))
        R._check(lib.rsm_sync(ctx))
    finally:
        for p in (0, 1):
            R._check(lib.rsm_ctx_set_pass_grid(ctx, p, 0, None))
    got = b.download(n).reshape(B, 2 * k, 2 * k, S)
    for i in range(B):
        assert np.array_equal(got[i], oracle.extend_square(got[i, :k, :k].copy(), nthreads=8))
    assert lib.rsm_ctx_set_pass_grid(ctx, 2, 0, None) == R.RSM_EINVAL


@pytest.mark.parametrize("S,count", [(512, 1), (512, 2), (512, 3), (512, 17), (64, 9), (1024, 4), (512, 70), (64, 1),
                                     (2048, 2), (192, 3), (320, 2), (4096, 1)])
def test_single_launch_batch_matches_two_launch(lib, S, count):
    """Batches of k = 128 squares run as ONE queue-driven launch (row sets, Q0-column
    sets, Q1-column sets from a ready list: extend_gf8_bs128s_kernel); bit-exact with
    the two-launch form, twice on the same (self-re-zeroed) queue words, and the
    first / last square against the oracle.  S dividing the 2 KiB set width takes the
    fixed per-lane offsets (kernel variant 16777216), 192 / 320 / 4096 the general
    per-lane division."""
    ctx = R.device_context(0)
    k = 128
    W = 2 * k
    n = W * W * S * count
    src, a, b = (R.DeviceBuffer(n) for _ in range(3))
    src.fill_random(900 + count)
    R._check(lib.rsm_sync(ctx))
    R._check(lib.rsm_memcpy(ctx, a.ptr, src.ptr, n, 2))
    R._check(lib.rsm_extend_squares_phase_dev(ctx, a.ptr, k, S, count, 1, None))
    R._check(lib.rsm_extend_squares_phase_dev(ctx, a.ptr, k, S, count, 2, None))
    R._check(lib.rsm_sync(ctx))
    want = a.download(n)
    prev = ctypes.c_int(0)
    R._check(lib.rsm_ctx_set_split_max(ctx, 0, ctypes.byref(prev)))  # the queue launch even for 1..4
    try:
        for _ in range(2):
            R._check(lib.rsm_memcpy(ctx, b.ptr, src.ptr, n, 2))
            R._check(lib.rsm_extend_squares_dev(ctx, b.ptr, k, S, count, None))
            R._check(lib.rsm_sync(ctx))
            assert np.array_equal(b.download(n), want)
    finally:
        R._check(lib.rsm_ctx_set_split_max(ctx, prev.value, None))
    sq = want.reshape(count, W, W, S)
    for i in (0, count - 1):
        assert np.array_equal(sq[i], oracle.extend_square(sq[i, :k, :k].copy(), nthreads=8))


@pytest.mark.parametrize("k,S,count", [(128, 512, 1), (128, 512, 4), (65, 64, 2), (100, 1024, 1), (128, 64, 3),
                                       (127, 320, 1)])
def test_split_latency_form(lib, k, S, count):
    """Up to rsm_ctx_set_split_max squares per call (default 12) with 65 <= k <= 128 take
    the latency form (encode_gf8_split_kernel: rows + Q0 columns in one launch, Q1
    columns in a second): every square bit-exact with the oracle and with the
    queue-driven launch of the same batch."""
    ctx = R.device_context(0)
    W = 2 * k
    n = W * W * S * count
    src, a, b = (R.DeviceBuffer(n) for _ in range(3))
    src.fill_random(1300 + k + count)
    R._check(lib.rsm_sync(ctx))
    prev = ctypes.c_int(0)
    R._check(lib.rsm_ctx_set_split_max(ctx, 4, ctypes.byref(prev)))
    try:
        R._check(lib.rsm_memcpy(ctx, a.ptr, src.ptr, n, 2))
        R._check(lib.rsm_extend_squares_dev(ctx, a.ptr, k, S, count, None))  # split form
        R._check(lib.rsm_ctx_set_split_max(ctx, 0, None))
        R._check(lib.rsm_memcpy(ctx, b.ptr, src.ptr, n, 2))
        R._check(lib.rsm_extend_squares_dev(ctx, b.ptr, k, S, count, None))  # queue / two-launch form
        R._check(lib.rsm_sync(ctx))
    finally:
        R._check(lib.rsm_ctx_set_split_max(ctx, prev.value, None))
    got = a.download(n)
    assert np.array_equal(got, b.download(n))
    sq = got.reshape(count, W, W, S)
    for i in range(count):
        assert np.array_equal(sq[i], oracle.extend_square(sq[i, :k, :k].copy(), nthreads=8))
    assert lib.rsm_ctx_set_split_max(ctx, -1, None) == R.RSM_EINVAL


def test_single_launch_batches_on_three_streams(lib):
    """Three streams each run single-launch batches on their own buffer (each stream
    owns its queue words), several rounds; every square equals the two-launch result."""
    ctx = R.device_context(0)
    k, S, B = 128, 512, 6
    W = 2 * k
    n = W * W * S * B
    src = [R.DeviceBuffer(n) for _ in range(3)]
    work = [R.DeviceBuffer(n) for _ in range(3)]
    for i, b in enumerate(src):
        b.fill_random(77 + i)
    R._check(lib.rsm_sync(ctx))
    want = []
    for i in range(3):
        R._check(lib.rsm_memcpy(ctx, work[i].ptr, src[i].ptr, n, 2))
        R._check(lib.rsm_extend_squares_phase_dev(ctx, work[i].ptr, k, S, B, 1, None))
        R._check(lib.rsm_extend_squares_phase_dev(ctx, work[i].ptr, k, S, B, 2, None))
        R._check(lib.rsm_sync(ctx))
        want.append(work[i].download(n))
    st = [ctypes.c_void_p() for _ in range(3)]
    for s in st:
        R._check(lib.rsm_stream_create(ctx, ctypes.byref(s)))
    for _ in range(3):
        for i in range(3):
            R._check(lib.rsm_memcpy(ctx, work[i].ptr, src[i].ptr, n, 2))
        for i in range(3):
            R._check(lib.rsm_extend_squares_dev(ctx, work[i].ptr, k, S, B, st[i]))
        for s in st:
            R._check(lib.rsm_stream_sync(s))
        R._check(lib.rsm_sync(ctx))  # also reports a stuck queue wait on any stream
        for i in range(3):
            assert np.array_equal(work[i].download(n), want[i])
    for s in st:
        R._check(lib.rsm_stream_destroy(ctx, s))


def test_single_launch_at_bench_scale(lib):
    """The bench's exact configuration (bench.py c2: k = 128, S = 512, 512 squares per
    launch, launches on 3 streams over 3 buffers, running concurrently): EVERY square
    of every launch equals the two-launch result, compared on the device
    (rsm_dev_equal), over several rounds.  The parity quadrants are re-poisoned
    before every launch, so a Q1-column set that read a stale or unfinished Q1 (the
    inter-workgroup hand-off of extend_gf8_bs128q_kernel) could not match by
    accident; the two-launch references are themselves oracle-checked, every square
    of every buffer (1,536 squares).  Reference: extendeddatasquare.go:154-227."""
    ctx = R.device_context(0)
    k, S, B, NS = 128, 512, 512, 3
    W = 2 * k
    sq = W * W * S
    n = sq * B
    seeds = [0xBE5C0 + i for i in range(NS)]
    ref = [R.DeviceBuffer(n) for _ in range(NS)]
    work = [R.DeviceBuffer(n) for _ in range(NS)]
    st = [ctypes.c_void_p() for _ in range(NS)]
    try:
        for i in range(NS):
            ref[i].fill_random(seeds[i])
            R._check(lib.rsm_sync(ctx))
            R._check(lib.rsm_extend_squares_phase_dev(ctx, ref[i].ptr, k, S, B, 1, None))
            R._check(lib.rsm_extend_squares_phase_dev(ctx, ref[i].ptr, k, S, B, 2, None))
            R._check(lib.rsm_sync(ctx))
            # every reference square against the oracle (the AVX-512 + GFNI build of the
            # restatement where the host has it -- pinned to the scalar oracle by
            # tests/test_oracle.py -- else the first and last square with the scalar one)
            gfni = oracle.gfni_supported()
            for j in (range(B) if gfni else (0, B - 1)):
                got = ref[i].download(sq, j * sq).reshape(W, W, S)
                ods = got[:k, :k].copy()
                want = oracle.extend_square_gfni(ods, nthreads=16) if gfni else oracle.extend_square(ods, nthreads=8)
                assert np.array_equal(got, want), (i, j)
        for s in st:
            R._check(lib.rsm_stream_create(ctx, ctypes.byref(s)))
        eq = ctypes.c_int()
        for rnd in range(4):
            for i in range(NS):  # Q0 = the reference input, Q1..Q3 = garbage
                work[i].fill_random(seeds[i] if rnd % 2 == 0 else seeds[(i + 1) % NS] ^ 0x55)
                R._check(lib.rsm_sync(ctx))
                if rnd % 2:
                    # restore the ODS quadrant of every square from the reference
                    _restore_ods(lib, ctx, work[i], ref[i], k, S, B)
            for i in range(NS):
                R._check(lib.rsm_extend_squares_dev(ctx, work[i].ptr, k, S, B, st[i]))
            for i in range(NS):
                R._check(lib.rsm_stream_check(ctx, st[i]))  # also reports a stuck queue wait
            for i in range(NS):
                R._check(lib.rsm_dev_equal(ctx, work[i].ptr, ref[i].ptr, n, None, ctypes.byref(eq)))
                assert eq.value == 1, (rnd, i)
    finally:
        for s in st:
            if s.value:
                R._check(lib.rsm_stream_destroy(ctx, s))
        for b in ref + work:
            b.free()


def _restore_ods(lib, ctx, dst, src, k, S, B):
    """Q0 of every square of src into dst (device to device, one copy per ODS row)."""
    W = 2 * k
    for b in range(B):
        for r in range(k):
            off = (b * W + r) * W * S
            R._check(lib.rsm_memcpy(ctx, dst.ptr + off, src.ptr + off, k * S, 2))


@pytest.mark.parametrize("k,S,count", [(128, 512, 5), (16, 64, 3), (256, 128, 2)])
def test_pinned_host_batch(lib, k, S, count):
    """rsm_extend_squares_host over pinned arenas: three lanes overlap H2D,
    extension and D2H; Q0 is filled on the host."""
    ctx = R.device_context(0)
    W = 2 * k
    ob, eb = k * k * S, W * W * S
    ho, he = ctypes.c_void_p(), ctypes.c_void_p()
    R._check(lib.rsm_host_alloc(ctx, ob * count, ctypes.byref(ho)))
    R._check(lib.rsm_host_alloc(ctx, eb * count, ctypes.byref(he)))
    try:
        ods = np.ctypeslib.as_array((ctypes.c_uint8 * (ob * count)).from_address(ho.value))
        ods[:] = np.random.default_rng(k + count).integers(0, 256, ob * count, dtype=np.uint8)
        R._check(lib.rsm_extend_squares_host(ctx, ho, k, S, count, he))
        eds = np.ctypeslib.as_array((ctypes.c_uint8 * (eb * count)).from_address(he.value))
        for i in range(count):
            want = oracle.extend_square(ods[i * ob:(i + 1) * ob].reshape(k, k, S), nthreads=8)
            assert np.array_equal(eds[i * eb:(i + 1) * eb].reshape(W, W, S), want), i
    finally:
        R._check(lib.rsm_host_free(ctx, ho))
        R._check(lib.rsm_host_free(ctx, he))


def test_inplace_host_and_pageable(lib):
    ctx = R.device_context(0)
    k, S = 128, 256
    W = 2 * k
    rng = np.random.default_rng(9)
    ods = rng.integers(0, 256, (k, k, S), dtype=np.uint8)
    want = oracle.extend_square(ods, nthreads=8)
    eds = np.full((W, W, S), 0xAB, np.uint8)
    R._check(lib.rsm_extend_square(ctx, ods.ctypes.data, k, S, eds.ctypes.data))
    assert np.array_equal(eds, want)
    eds2 = np.full((W, W, S), 0xCD, np.uint8)
    eds2[:k, :k] = ods
    R._check(lib.rsm_extend_square_inplace_host(ctx, eds2.ctypes.data, k, S))
    assert np.array_equal(eds2, want)


@pytest.fixture(scope="module")
def multi(lib):
    m = ctypes.c_void_p()
    devs = (ctypes.c_int * 1)(0)
    R._check(lib.rsm_multi_create(devs, 1, ctypes.byref(m)))
    yield m
    lib.rsm_multi_destroy(m)


@pytest.mark.parametrize("sched", [0, 1])
def test_multi_gpu_c_abi_config5_world1(lib, multi, sched):
    """Config 5 through the C ABI (rsm_multi_extend_square: RCCL clique driven from
    C++, all-gather and all-to-all schedules) at k = 512, S = 512 on the one GPU of
    this box, bit-exact against the oracle."""
    k, S = 512, 512
    W = 2 * k
    assert lib.rsm_multi_size(multi) == 1
    ods = oracle.splitmix64_bytes(k * k * S, seed=0xC5 + sched).reshape(k, k, S)
    eds = np.zeros((W, W, S), np.uint8)
    R._check(lib.rsm_multi_extend_square(multi, ods.ctypes.data, k, S, eds.ctypes.data, sched))
    assert np.array_equal(eds, oracle.extend_square(ods, nthreads=8))


@pytest.mark.parametrize("k,S", [(128, 512), (64, 192)])
def test_multi_gpu_dev_world1(lib, multi, k, S):
    W = 2 * k
    ctx = lib.rsm_multi_context(multi, 0)
    p = ctypes.c_void_p()
    R._check(lib.rsm_dev_alloc(ctx, W * W * S, ctypes.byref(p)))
    try:
        ods = np.random.default_rng(k).integers(0, 256, (k, k, S), dtype=np.uint8)
        full = np.zeros((W, W, S), np.uint8)
        full[:k, :k] = ods
        R._check(lib.rsm_memcpy(ctx, p, full.ctypes.data, full.nbytes, 0))
        arr = (ctypes.c_void_p * 1)(p.value)
        R._check(lib.rsm_multi_extend_dev(multi, arr, k, S, 1))
        R._check(lib.rsm_multi_sync(multi))
        out = np.empty_like(full)
        R._check(lib.rsm_memcpy(ctx, out.ctypes.data, p, out.nbytes, 1))
        assert np.array_equal(out, oracle.extend_square(ods, nthreads=8))
    finally:
        lib.rsm_dev_free(ctx, p)


def test_multi_gpu_shape_errors(lib, multi):
    eds = np.zeros(16, np.uint8)
    assert lib.rsm_multi_extend_square(multi, eds.ctypes.data, 4, 100, eds.ctypes.data, 0) == R.RSM_ESHARESIZE
    assert lib.rsm_multi_extend_square(multi, eds.ctypes.data, 4, 64, eds.ctypes.data, 7) == R.RSM_EINVAL


@pytest.mark.parametrize("sched", [0, 1])
def test_multi_gpu_inplace_pinned_world1(lib, multi, sched):
    """The pinned in-place host form (rsm_multi_extend_square_inplace on an
    rsm_multi_host_alloc arena whose Q0 quadrant holds the ODS) at config 5's k = 512,
    S = 512: only Q1..Q3 written, the whole EDS bit-exact against the oracle."""
    k, S = 512, 512
    W = 2 * k
    ods = oracle.splitmix64_bytes(k * k * S, seed=0x5C + sched).reshape(k, k, S)
    p = ctypes.c_void_p()
    R._check(lib.rsm_multi_host_alloc(multi, W * W * S, ctypes.byref(p)))
    try:
        eds = np.ctypeslib.as_array((ctypes.c_uint8 * (W * W * S)).from_address(p.value)).reshape(W, W, S)
        eds[:] = 0x3C
        eds[:k, :k] = ods
        R._check(lib.rsm_multi_extend_square_inplace(multi, p, k, S, sched))
        assert np.array_equal(eds, oracle.extend_square(ods, nthreads=8))
    finally:
        R._check(lib.rsm_multi_host_free(multi, p))


@pytest.mark.parametrize("k,S,count", [(17, 64, 1), (32, 512, 1), (33, 320, 2), (50, 512, 1), (64, 512, 1),
                                       (64, 512, 12), (64, 128, 13), (24, 1024, 5), (32, 128, 64), (64, 64, 65),
                                       (9, 64, 1), (16, 512, 1), (13, 192, 7), (16, 64, 70)])
def test_small_square_latency_form(lib, k, S, count):
    """17 <= k <= 64: up to 64 squares per call take the split latency form
    (encode_gf8_splitm_kernel), larger batches the byte-table passes; both == oracle."""
    W = 2 * k
    n = W * W * S * count
    buf = R.DeviceBuffer(n)
    buf.fill_random(700 + k + count)
    R._check(lib.rsm_extend_squares_dev(buf.ctx, buf.ptr, k, S, count, None))
    R._check(lib.rsm_sync(buf.ctx))
    got = buf.download().reshape(count, W, W, S)
    for c in range(count):
        assert np.array_equal(got[c], oracle.extend_square(got[c, :k, :k].copy(), nthreads=8)), c
    buf.free()
