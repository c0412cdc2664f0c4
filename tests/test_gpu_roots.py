"""GPU: DefaultTree row/column Merkle roots on the device (kernels_sha.hip,
SURVEY.md §8(f) f1) vs the hashlib restatement (oracle/crossword.merkle_root,
leaf = H(0x00||share), node = H(0x01||l||r), NebulousLabs fold for non-powers of
two) -- bit-exact."""
import numpy as np
import pytest

import oracle
import rsmt2d_amd as R
from oracle import crossword

pytestmark = pytest.mark.gpu


def _device_roots(lib, eds):
    W, _, S = eds.shape
    buf = R.DeviceBuffer(eds.nbytes)
    buf.upload(np.ascontiguousarray(eds))
    out = R.DeviceBuffer(2 * W * 32)
    R._check(lib.rsm_roots_dev(buf.ctx, buf.ptr, W, S, out.ptr, None))
    R._check(lib.rsm_sync(buf.ctx))
    raw = out.download()
    buf.free()
    out.free()
    return [raw[i * 32:(i + 1) * 32].tobytes() for i in range(2 * W)]


@pytest.mark.parametrize("W,S", [(2, 64), (6, 64), (10, 128), (24, 64), (256, 512), (200, 576)])
def test_device_roots_match_hashlib(lib, W, S):
    eds = oracle.splitmix64_bytes(W * W * S, seed=W * 131 + S).reshape(W, W, S)
    got = _device_roots(lib, eds)
    rows = list(range(W)) if W <= 24 else [0, 1, W // 2, W - 1]
    for r in rows:
        assert got[r] == crossword.merkle_root([eds[r, c].tobytes() for c in range(W)]), ("row", r)
        assert got[W + r] == crossword.merkle_root([eds[c, r].tobytes() for c in range(W)]), ("col", r)


def test_device_roots_match_host_tree_all(lib):
    """All 2W roots of a k=128 EDS vs the host DefaultTree (merkle.cpp)."""
    k, S = 128, 512
    ods = oracle.splitmix64_bytes(k * k * S, seed=5).reshape(k, k, S)
    eds = oracle.extend_square(ods, nthreads=8)
    got = _device_roots(lib, eds)
    W = 2 * k
    for r in range(W):
        assert got[r] == R._default_root([eds[r, c].tobytes() for c in range(W)]), r
        assert got[W + r] == R._default_root([eds[c, r].tobytes() for c in range(W)]), r


def test_eds_roots_device_path(lib, rng):
    """ComputeExtendedDataSquare(...).RowRoots()/ColRoots() (context set -> GPU roots)."""
    k, S = 16, 128
    ods = [rng.integers(0, 256, S, dtype=np.uint8).tobytes() for _ in range(k * k)]
    eds = R.ComputeExtendedDataSquare(ods, R.NewLeoRSCodec(), R.NewDefaultTree)
    sq = crossword.Square(eds.Flattened())
    assert eds.RowRoots() == sq.roots(crossword.Row)
    assert eds.ColRoots() == sq.roots(crossword.Col)


@pytest.mark.parametrize("W,S,n", [(24, 64, 3), (2, 64, 5), (6, 64, 3), (10, 128, 2), (200, 64, 3), (256, 64, 3)])
def test_batched_roots_match_per_square(lib, W, S, n):
    """rsm_roots_squares_dev over n squares (the batch form: workgroup-cooperative upper
    levels) == rsm_roots_dev of each (the one-square form, pinned above)."""
    eds = oracle.splitmix64_bytes(n * W * W * S, seed=77 + W).reshape(n, W, W, S)
    buf = R.DeviceBuffer(eds.nbytes)
    buf.upload(np.ascontiguousarray(eds))
    out = R.DeviceBuffer(n * 2 * W * 32)
    R._check(lib.rsm_roots_squares_dev(buf.ctx, buf.ptr, W, S, n, out.ptr, None))
    R._check(lib.rsm_sync(buf.ctx))
    raw = out.download()
    buf.free()
    out.free()
    for i in range(n):
        got = [raw[(2 * W * i + j) * 32:(2 * W * i + j + 1) * 32].tobytes() for j in range(2 * W)]
        assert got == _device_roots(lib, eds[i]), i
