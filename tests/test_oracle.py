"""CPU: the oracle itself, pinned against the reference's golden vectors.

Reference-pinned: the 1x1 / 2x2 grids of extendeddatasquare_test.go:39-59 and the
Repair semantics asserted by extendeddatacrossword_test.go / rsmt2d_test.go.
Everything else is a self-consistency property of the restatement.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
from oracle import crossword

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_tables_match_survey_selfcheck():
    e, lg, sk, _ = oracle.tables8()
    assert list(e[:8]) == [1, 104, 92, 100, 114, 240, 86, 18]
    assert list(lg[:8]) == [255, 0, 85, 170, 17, 68, 34, 136]
    assert list(sk[:16]) == [255, 255, 85, 255, 17, 85, 34, 255, 153, 17, 102, 85, 51, 34, 187, 255]
    _, _, sk16, _ = oracle.tables16()
    assert list(sk16[:8]) == [65535, 65535, 21845, 65535, 17476, 21845, 34952, 65535]


@pytest.mark.parametrize("name", ["1x1", "2x2"])
@pytest.mark.parametrize("S", [64, 512])
def test_reference_kat_grids(name, S):
    kat = json.load(open(os.path.join(GOLD, "kat_grids.json")))[name]
    ods = np.array(kat["ods"], dtype=np.uint8)
    k = ods.shape[0]
    eds = oracle.extend_square(np.repeat(ods[:, :, None], S, axis=2))
    assert (eds == np.array(kat["eds"], dtype=np.uint8)[:, :, None]).all()


def test_restatement_digests():
    gold = json.load(open(os.path.join(GOLD, "restatement.json")))
    for row in gold["affine_digests_survey"] + gold["affine_digests_more"]:
        if row["k"] > 130:
            continue  # k=256 digest is re-checked in make_golden.py (seconds of CPU)
        eds = oracle.extend_square(oracle.affine_pattern(row["k"], row["S"]), nthreads=os.cpu_count() or 1)
        assert hashlib.sha256(eds.tobytes()).hexdigest() == row["sha256"], row
        assert oracle.field_bits(row["k"]) == row["field_bits"]


def test_golden_npy():
    for k in (3, 4, 8):
        want = np.load(os.path.join(GOLD, f"eds_k{k}_s64.npy"))
        assert (oracle.extend_square(oracle.affine_pattern(k, 64)) == want).all()


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 8, 35, 64, 100, 128, 129, 200])
def test_roundtrip_decode(rng, k):
    S = 64
    data = [rng.integers(0, 256, S, dtype=np.uint8).tobytes() for _ in range(k)]
    full = data + oracle.encode(data)
    sh = list(full)
    for i in rng.choice(2 * k, size=k, replace=False):
        sh[i] = None
    assert oracle.decode(sh) == full
    with pytest.raises(oracle.TooFewShards):
        sh2 = list(full)
        for i in rng.choice(2 * k, size=k + 1, replace=False):
            sh2[i] = None
        oracle.decode(sh2)


@pytest.mark.parametrize("k", [2, 4, 8, 35, 64])
def test_q3_rows_of_q2_equal_cols_of_q1(rng, k):
    """extendeddatasquare.go:204-207: Q3 from Q2 rows == Q3 from Q1 columns (the device
    schedule uses the latter)."""
    S = 64
    ods = rng.integers(0, 256, (k, k, S), dtype=np.uint8)
    eds = oracle.extend_square(ods)
    q1 = eds[:k, k:]
    for c in range(k):
        parity = oracle.encode([q1[r, c].tobytes() for r in range(k)])
        for r in range(k):
            assert parity[r] == eds[k + r, k + c].tobytes()


# --- the Repair restatement against the reference's own test expectations ---
def _example_flat(S=512):
    ods = np.repeat(np.array([[1, 2], [3, 4]], np.uint8)[:, :, None], S, axis=2)
    eds = oracle.extend_square(ods)
    return [eds[r, c].tobytes() for r in range(4) for c in range(4)]


def _roots(flat):
    sq = crossword.Square(flat)
    return sq.roots(crossword.Row), sq.roots(crossword.Col)


def test_crossword_maximum_erasures():  # extendeddatacrossword_test.go:38-60
    flat = _example_flat()
    rr, cr = _roots(flat)
    f = list(flat)
    for i in (0, 2, 3, 4, 5, 6, 7, 8, 9, 10, 12, 13):
        f[i] = None
    assert crossword.repair(f, rr, cr) == flat


def test_crossword_unrepairable():  # extendeddatacrossword_test.go:63-80
    flat = _example_flat()
    rr, cr = _roots(flat)
    f = list(flat)
    for i in (0, 2, 3, 4, 5, 6, 7, 8, 9, 10, 12, 13, 14):
        f[i] = None
    with pytest.raises(crossword.Unrepairable):
        crossword.repair(f, rr, cr)


def test_crossword_orthogonal_byzantine():  # extendeddatacrossword_test.go:275-359
    flat = _example_flat()
    rr, cr = _roots(flat)
    f = list(flat)
    f[0 * 4 + 2] = None
    f[2 * 4 + 0] = None
    f[2 * 4 + 2] = bytes([66]) * 512
    with pytest.raises(crossword.Byzantine) as ei:
        crossword.repair(f, rr, cr)
    assert (ei.value.axis, ei.value.index) == (crossword.Col, 2)
    assert ei.value.shares[0] is None and bytes([66]) * 512 in ei.value.shares


def test_crossword_row_byzantine_preserves_nils():  # extendeddatacrossword_test.go:368-405
    flat = _example_flat()
    rr, cr = _roots(flat)
    f = list(flat)
    f[0] = bytes([66]) * 512
    f[2] = f[3] = None
    f[12] = None
    with pytest.raises(crossword.Byzantine) as ei:
        crossword.repair(f, rr, cr)
    assert (ei.value.axis, ei.value.index) == (crossword.Row, 0)
    assert ei.value.shares[2] is None and ei.value.shares[3] is None


@pytest.mark.parametrize("k,S", [(2, 64), (8, 128), (33, 64), (128, 512)])
def test_simd_restatement_matches_scalar(k, S):
    """The AVX2 build (cpu_baseline) computes exactly what the scalar oracle does."""
    ods = oracle.splitmix64_bytes(k * k * S, seed=0x51D + k).reshape(k, k, S)
    assert np.array_equal(oracle.extend_square_simd(ods, nthreads=4), oracle.extend_square(ods, nthreads=4))


@pytest.mark.skipif(not oracle.gfni_supported(), reason="host has no GFNI / AVX-512BW")
@pytest.mark.parametrize("k,S", [(1, 64), (2, 64), (4, 512), (16, 128), (128, 512)])
def test_gfni_restatement_matches_scalar(k, S):
    """The cpu_baseline's AVX-512 GFNI build (fused butterflies, GF2P8AFFINEQB
    multiplies) computes exactly the scalar oracle's extension."""
    ods = np.random.default_rng(k * 31 + S).integers(0, 256, (k, k, S), dtype=np.uint8)
    assert np.array_equal(oracle.extend_square_gfni(ods, nthreads=4), oracle.extend_square(ods, nthreads=4))
