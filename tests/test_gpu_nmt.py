"""GPU: namespaced-Merkle-tree roots on the device (kernels_nmt.hip) and
ComputeExtendedDataSquareWithBuffer (extendeddatasquare.go:81-92), restating
TestComputeExtendedDataSquareVsWithBuffer (extendeddatasquare_test.go:503-604):
buffered vs plain roots for ODS 32..512 and the uneven 35/67/83/127, with a
pool reused across sizes.  Here both constructors land on the device NMT, so each
case is also checked against the host restatement (rsm_nmt_tree_root, through a
Python tree callback) and, up to k = 128, the Python oracle (oracle/nmt.py).
Parity vs the nmt library itself is unpinned (not vendored)."""
import ctypes

import numpy as np
import pytest

import oracle
import rsmt2d_amd as R
from oracle import nmt

pytestmark = pytest.mark.gpu

SHARE = 512  # shareSize of the reference tests (rsmt2d_test.go)
NS = 29      # defaultNamespaceIDSize (datasquare_test.go:20)


def gen_rand_sorted_ds(width, share_size, ns, seed):
    """genRandSortedDS (extendeddatasquare_test.go:352-362): random shares sorted by
    their first `ns` bytes."""
    rng = np.random.default_rng(seed)
    sh = rng.integers(0, 256, (width * width, share_size), dtype=np.uint8)
    return [bytes(x) for x in sh[np.lexsort(sh[:, :ns][:, ::-1].T)]]


def host_constructor(k, ns=NS):
    """The same tree through the generic Python-callback path: host C++ roots."""
    c = R.ErasuredNamespacedMerkleTreeConstructor(k, ns)
    return lambda axis, idx: c(axis, idx)


SIZES = [32, 64, 83, 127, 128, 256, 512, 35, 67]


@pytest.fixture(scope="module")
def pool():
    return R.newTreePool(32, 4, NS)  # smallest size first: "pool-reallocation"


@pytest.mark.parametrize("k", SIZES)
def test_with_buffer_vs_plain(pool, k):
    codec = R.NewLeoRSCodec()
    data = gen_rand_sorted_ds(k, SHARE, 8, seed=k)
    std = R.ComputeExtendedDataSquare(data, codec, R.newErasuredNamespacedMerkleTreeConstructor(k, NS))
    buf = R.ComputeExtendedDataSquareWithBuffer(data, codec, pool)
    assert buf.parallelOps == 4
    rr, cr = std.RowRoots(), std.ColRoots()
    assert buf.RowRoots() == rr and buf.ColRoots() == cr
    assert len(rr) == 2 * k and all(len(r) == 2 * NS + 32 for r in rr)
    # the device NMT against the host restatement, all 4k trees
    host = R.ImportExtendedDataSquare(std.Flattened(), codec, host_constructor(k))
    assert host.RowRoots() == rr and host.ColRoots() == cr
    if k <= 128:  # and against the Python oracle
        W = 2 * k
        sq = np.frombuffer(b"".join(std.Flattened()), np.uint8).reshape(W, W, SHARE)
        want_r, want_c = nmt.eds_roots(sq, k, NS)
        assert rr == want_r and cr == want_c


def test_with_buffer_error_cases(pool):
    codec = R.NewLeoRSCodec()
    with pytest.raises(R.RSMError):  # shareSize not a multiple of 64
        R.ComputeExtendedDataSquareWithBuffer([b"\x01" * 65], codec, pool)
    with pytest.raises(R.RSMError):  # number of shares not a perfect square
        R.ComputeExtendedDataSquareWithBuffer([bytes([i + 1]) * SHARE for i in range(3)], codec, pool)


@pytest.mark.parametrize("k,ns,S", [(4, 29, 64), (3, 8, 128), (16, 1, 64), (64, 32, 512), (5, 29, 64), (6, 29, 64),
                                    (10, 29, 128), (1, 29, 64)])
def test_nmt_roots_dev_vs_oracle(lib, k, ns, S):
    """rsm_nmt_roots_dev over a device-resident square, bit-exact vs the oracle."""
    ctx = R.device_context(0)
    W = 2 * k
    ods = np.frombuffer(b"".join(gen_rand_sorted_ds(k, S, ns, seed=k * ns)), np.uint8).reshape(k, k, S)
    eds = oracle.extend_square(ods, nthreads=8)
    RL = 2 * ns + 32
    d = R.DeviceBuffer(eds.nbytes)
    roots = R.DeviceBuffer(2 * W * RL)
    status = R.DeviceBuffer(2 * W * 4)
    R._check(lib.rsm_memcpy(ctx, d.ptr, eds.ctypes.data, eds.nbytes, 0))
    p = R.NmtParams(ns, 1, k)
    R._check(lib.rsm_nmt_roots_dev(ctx, d.ptr, W, S, ctypes.byref(p), roots.ptr, status.ptr, None))
    R._check(lib.rsm_sync(ctx))
    got = roots.download(2 * W * RL)
    st = np.frombuffer(status.download(2 * W * 4).tobytes(), np.uint32)
    assert not st.any()
    want_r, want_c = nmt.eds_roots(eds, k, ns)
    assert [bytes(got[i * RL:(i + 1) * RL]) for i in range(W)] == want_r
    assert [bytes(got[(W + i) * RL:(W + i + 1) * RL]) for i in range(W)] == want_c


@pytest.mark.parametrize("k,ns,S,count", [(4, 29, 64, 3), (16, 29, 512, 5), (8, 8, 128, 2), (64, 29, 512, 3),
                                         (128, 29, 512, 2), (6, 29, 64, 3), (10, 29, 576, 2)])
def test_nmt_roots_squares_dev_batched(lib, k, ns, S, count):
    """rsm_nmt_roots_squares_dev over a batch of squares (one launch pair) == the
    oracle's roots of every square; one square with an unordered namespace reports its
    failing trees in its own status words only.  k = 64 / 128 take the wave kernel's
    batch shape (two trees per wave, levels 1-2 in one pass)."""
    ctx = R.device_context(0)
    W = 2 * k
    RL = 2 * ns + 32
    sqs = []
    for q in range(count):
        ods = np.frombuffer(b"".join(gen_rand_sorted_ds(k, S, ns, seed=100 + q)), np.uint8).reshape(k, k, S).copy()
        if q == count - 1:
            ods[0, 1, :ns], ods[0, 0, :ns] = ods[0, 0, :ns].copy(), ods[0, 1, :ns].copy()  # row 0 out of order
        sqs.append(oracle.extend_square(ods, nthreads=8))
    batch = np.stack(sqs)
    d = R.DeviceBuffer(batch.nbytes)
    roots = R.DeviceBuffer(count * 2 * W * RL)
    status = R.DeviceBuffer(count * 2 * W * 4)
    d.upload(batch)
    p = R.NmtParams(ns, 1, k)
    R._check(lib.rsm_nmt_roots_squares_dev(ctx, d.ptr, W, S, count, ctypes.byref(p), roots.ptr, status.ptr, None))
    R._check(lib.rsm_sync(ctx))
    got = roots.download(count * 2 * W * RL).reshape(count, 2 * W, RL)
    st = np.frombuffer(status.download(count * 2 * W * 4).tobytes(), np.uint32).reshape(count, 2 * W)
    for q in range(count - 1):
        assert not st[q].any()
        want_r, want_c = nmt.eds_roots(sqs[q], k, ns)
        assert [bytes(got[q, i]) for i in range(W)] == want_r
        assert [bytes(got[q, W + i]) for i in range(W)] == want_c
    bad = st[count - 1]
    if not np.array_equal(sqs[-1][0, 0, :ns], sqs[-1][0, 1, :ns]):
        assert bad[0] != 0  # row 0's push order
    assert not bad[k:W].any()  # parity rows: parity namespace everywhere past Q0


def test_nmt_push_order_error_device_and_host():
    """Unsorted namespaces: the reference's Push fails, so RowRoots errors (device
    and host paths alike)."""
    codec = R.NewLeoRSCodec()
    k = 8
    data = gen_rand_sorted_ds(k, SHARE, 8, seed=99)[::-1]  # descending namespaces
    eds = R.ComputeExtendedDataSquare(data, codec, R.newErasuredNamespacedMerkleTreeConstructor(k, NS))
    with pytest.raises(R.RSMError):
        eds.RowRoots()
    host = R.ImportExtendedDataSquare(eds.Flattened(), codec, host_constructor(k))
    with pytest.raises(R.RSMError):
        host.RowRoots()


@pytest.mark.parametrize("k", [128, 35])
def test_nmt_repair(k):
    """Repair with NMT roots (the Celestia producer/sampler tree): the zero-copy
    fast path with device NMT verification restores the square; a corrupted share
    surfaces as ErrByzantineData from the exact path."""
    codec = R.NewLeoRSCodec()
    W = 2 * k
    data = gen_rand_sorted_ds(k, SHARE, 8, seed=7 + k)
    ctor = R.newErasuredNamespacedMerkleTreeConstructor(k, NS)
    eds = R.ComputeExtendedDataSquare(data, codec, ctor)
    rr, cr = eds.RowRoots(), eds.ColRoots()
    full = eds.Flattened()
    rng = np.random.default_rng(k)
    present = np.ones((W, W), bool)
    for r in range(W):
        present[r, rng.choice(W, size=k, replace=False)] = False
    holey = [full[i] if present.flat[i] else None for i in range(W * W)]
    h = R.ImportExtendedDataSquare(holey, codec, ctor)
    h.Repair(rr, cr)
    assert h.repair_stats().fast_path == 1
    assert h.Flattened() == full
    # byzantine: one present share of row 1 altered
    c = int(np.flatnonzero(present[1])[0])
    bad = list(holey)
    bad[W + c] = bytes([full[W + c][0] ^ 1]) + full[W + c][1:]
    h2 = R.ImportExtendedDataSquare(bad, codec, ctor)
    with pytest.raises(R.ErrByzantineData):
        h2.Repair(rr, cr)


def _nmt_eds(values, ns=1, share=512):
    """createTestEdsWithNMT (extendeddatacrossword_test.go:788-804): a 2x2 ODS of
    constant shares, erasured NMT with `ns`-byte namespaces."""
    data = [bytes([v]) * share for v in values]
    return R.ComputeExtendedDataSquare(data, R.NewLeoRSCodec(), R.newErasuredNamespacedMerkleTreeConstructor(2, ns))


ONE, TWO, THREE = (bytes([v]) * SHARE for v in (1, 2, 3))
ALL_BUT = lambda keep: [(r, c) for r in range(4) for c in range(4) if (r, c) not in keep]


@pytest.mark.parametrize("name,cells,axis", [
    ("no corruption", {}, None),
    # row 0 = [two, one, parity...] complete, everything else erased: row 0's tree
    # push fails on the namespace order -> ErrByzantineData{Row, 0}
    ("rows with unordered shares", {**{(0, 0): TWO, (0, 1): ONE}, **{rc: None for rc in ALL_BUT(
        {(0, 0), (0, 1), (0, 2), (0, 3)})}}, R.Row),
    # column 0 = [three, one, parity...] complete, the rest erased -> {Col, 0}
    ("columns with unordered shares", {**{(0, 0): THREE, (1, 0): ONE}, **{rc: None for rc in ALL_BUT(
        {(0, 0), (1, 0), (2, 0), (3, 0)})}}, R.Col),
])
def test_corrupted_eds_byzantine_unordered_shares(name, cells, axis):
    """TestCorruptedEdsReturnsErrByzantineData_UnorderedShares
    (extendeddatacrossword_test.go:490-602): the DA header of the ODS {1,2,3,4}
    with 1-byte namespaces; a corrupted copy whose only complete vector has its
    shares out of namespace order must fail Repair with ErrByzantineData on exactly
    that axis, index 0."""
    header = _nmt_eds([1, 2, 3, 4])
    rr, cr = header.RowRoots(), header.ColRoots()
    eds = _nmt_eds([1, 2, 3, 4])
    for (r, c), v in cells.items():
        eds.setCell(r, c, v)
    if axis is None:
        eds.Repair(rr, cr)
        assert eds.Flattened() == header.Flattened()
        return
    with pytest.raises(R.ErrByzantineData) as ei:
        eds.Repair(rr, cr)
    assert ei.value.Axis == axis and ei.value.Index == 0

