"""GPU parity: the HIP codec and 2D extension vs the CPU oracle (bit-exact)."""
import ctypes

import numpy as np
import pytest

import oracle
import rsmt2d_amd as R
from conftest import rand_shares

pytestmark = pytest.mark.gpu

GF8_K = [1, 2, 3, 4, 5, 7, 8, 16, 31, 32, 35, 64, 67, 83, 100, 127, 128]


@pytest.mark.parametrize("k", GF8_K)
@pytest.mark.parametrize("S", [64, 512])
def test_encode_matches_oracle(lib, rng, k, S):
    data = rand_shares(rng, k, S)
    assert R.NewLeoRSCodec().Encode(data) == oracle.encode(data)


@pytest.mark.parametrize("S", [64, 192, 320, 1024, 2112, 4096])
def test_encode_partial_chunks(lib, rng, S):
    data = rand_shares(rng, 128, S)
    assert R.NewLeoRSCodec().Encode(data) == oracle.encode(data)


@pytest.mark.parametrize("k", GF8_K)
def test_decode_matches_oracle(lib, rng, k):
    S = 128
    data = rand_shares(rng, k, S)
    full = data + oracle.encode(data)
    for trial in range(3):
        n_missing = [k, max(0, k // 2), 1][trial]
        sh = list(full)
        for i in rng.choice(2 * k, size=n_missing, replace=False):
            sh[i] = None
        got = R.NewLeoRSCodec().Decode(list(sh))
        assert got == full, (k, trial)


def test_decode_too_few(lib, rng):
    k = 8
    data = rand_shares(rng, k, 64)
    sh = data + oracle.encode(data)
    for i in range(k + 1):
        sh[i] = None
    with pytest.raises(R.RSMError) as e:
        R.NewLeoRSCodec().Decode(sh)
    assert e.value.code == R.RSM_ETOOFEW


def test_decode_byzantine_matches_oracle_formula(lib, rng):
    """With > k inconsistent shares present the output depends on the exact
    reconstruct formula; GPU must agree with the oracle bit for bit."""
    k, S = 16, 64
    data = rand_shares(rng, k, S)
    sh = data + oracle.encode(data)
    sh[3] = bytes([66]) * S
    for i in (0, 20, 21):
        sh[i] = None
    assert R.NewLeoRSCodec().Decode(list(sh)) == oracle.decode(list(sh))


@pytest.mark.parametrize("k", [1, 2, 4, 8, 35, 64, 127, 128])
def test_extend_square_matches_oracle(lib, rng, k):
    S = 512 if k >= 64 else 64
    ods = rng.integers(0, 256, (k, k, S), dtype=np.uint8)
    want = oracle.extend_square(ods, nthreads=8)
    got = np.empty_like(want)
    ctx = R.device_context()
    R._check(lib.rsm_extend_square(ctx, ods.ctypes.data, k, S, got.ctypes.data))
    assert (got == want).all()


def test_extend_squares_dev_batched(lib):
    """Device-resident in-place batch (the bench path) on 3 squares, k=128, S=512; the
    synthetic input generator must reproduce oracle.splitmix64_bytes."""
    k, S, n = 128, 512, 3
    W = 2 * k
    buf = R.DeviceBuffer(n * W * W * S)
    buf.fill_random(1234)
    ref = oracle.splitmix64_bytes(n * W * W * S, seed=1234).reshape(n, W, W, S)
    assert (buf.download().reshape(n, W, W, S) == ref).all()
    R._check(lib.rsm_extend_squares_dev(buf.ctx, buf.ptr, k, S, n, None))
    R._check(lib.rsm_sync(buf.ctx))
    got = buf.download().reshape(n, W, W, S)
    for i in range(n):
        assert (got[i] == oracle.extend_square(ref[i, :k, :k].copy(), nthreads=8)).all(), i
    buf.free()


@pytest.mark.parametrize("k,S", [(65, 64), (100, 2112), (128, 3072)])
def test_extend_square_bitsliced_shapes(lib, rng, k, S):
    """M = 128 squares whose 2 KiB bit-sliced sets straddle codewords / shares."""
    ods = rng.integers(0, 256, (k, k, S), dtype=np.uint8)
    want = oracle.extend_square(ods, nthreads=8)
    got = np.empty_like(want)
    R._check(lib.rsm_extend_square(R.device_context(), ods.ctypes.data, k, S, got.ctypes.data))
    assert (got == want).all()


def test_affine_digest_k128(lib):
    import hashlib
    import json, os
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "restatement.json")))
    want = [r for r in gold["affine_digests_survey"] if r["k"] == 128][0]["sha256"]
    ods = oracle.affine_pattern(128, 512)
    got = np.empty((256, 256, 512), np.uint8)
    R._check(lib.rsm_extend_square(R.device_context(), ods.ctypes.data, 128, 512, got.ctypes.data))
    assert hashlib.sha256(got.tobytes()).hexdigest() == want


@pytest.mark.parametrize("k", [65, 100, 127, 128])
@pytest.mark.parametrize("axis", [0, 1])
@pytest.mark.parametrize("S", [192, 512, 1024])
def test_decode_sweep_matches_oracle(lib, k, axis, S):
    """Batched device decode of every row (or column) of a square, each with its own
    random erasure pattern (the C3 sweep; split M = 128 decoder), bit-exact."""
    rng = np.random.default_rng(k * 7 + axis * 3 + S)
    W = 2 * k
    ods = rng.integers(0, 256, (k, k, S), dtype=np.uint8)
    full = oracle.extend_square(ods, nthreads=8)
    pres = np.ones((W, W), np.uint8)
    for v in range(W):
        lost = rng.choice(W, size=int(rng.integers(1, k + 1)), replace=False)
        if axis == 0:
            pres[v, lost] = 0
        else:
            pres[lost, v] = 0
    dmg = full * pres[:, :, None]
    buf = R.DeviceBuffer(full.nbytes)
    buf.upload(dmg)
    pd = R.DeviceBuffer(W * W)
    pd.upload(pres)
    idx = R.DeviceBuffer(4 * W)
    idx.upload(np.arange(W, dtype=np.uint32))
    ctx = R.device_context(0)
    R._check(lib.rsm_decode_vectors_dev(ctx, buf.ptr, pd.ptr, k, S, axis, idx.ptr, W, None))
    R._check(lib.rsm_sync(ctx))
    assert np.array_equal(buf.download(full.nbytes).reshape(W, W, S), full)
