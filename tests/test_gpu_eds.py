"""GPU: the reference's own EDS / Repair tests restated over the HIP engine
(extendeddatasquare_test.go, extendeddatacrossword_test.go, rsmt2d_test.go)."""
import json
import os

import numpy as np
import pytest

import oracle
import rsmt2d_amd as R
from oracle import crossword
from conftest import const_share, rand_shares

pytestmark = pytest.mark.gpu
S = 512  # extendeddatacrossword_test.go:17


def example_eds(share_size=S):
    return R.ComputeExtendedDataSquare([const_share(v, share_size) for v in (1, 2, 3, 4)],
                                       R.NewLeoRSCodec(), R.NewDefaultTree)


def test_compute_kat(lib):  # extendeddatasquare_test.go:30-68
    kat = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kat_grids.json")))
    eds = R.ComputeExtendedDataSquare([const_share(1)], R.NewLeoRSCodec(), R.NewDefaultTree)
    assert eds.Flattened() == [const_share(v) for row in kat["1x1"]["eds"] for v in row]
    eds = example_eds()
    assert eds.Flattened() == [const_share(v) for row in kat["2x2"]["eds"] for v in row]
    assert eds.FlattenedODS() == [const_share(v) for v in (1, 2, 3, 4)]
    with pytest.raises(R.RSMError):
        R.ComputeExtendedDataSquare([b"\1" * 65], R.NewLeoRSCodec(), R.NewDefaultTree)


def test_equals_and_json(lib):  # extendeddatasquare_test.go:92-112, 420-470
    a, b = example_eds(), example_eds()
    assert a.Equals(b)
    assert not a.Equals(example_eds(S * 2))
    one = R.ComputeExtendedDataSquare([const_share(1)], R.NewLeoRSCodec(), R.NewDefaultTree)
    assert not a.Equals(one)
    back = R.ExtendedDataSquare.UnmarshalJSON(a.MarshalJSON())
    assert back.Flattened() == a.Flattened()


def test_immutable_rows_and_roots(lib):  # extendeddatasquare_test.go:167-224
    eds = example_eds()
    r = eds.RowRoots()
    r[0] = b"x"
    assert eds.RowRoots()[0] != b"x"
    assert len(eds.Roots()) == 8


def _roots(eds):
    return eds.RowRoots(), eds.ColRoots()


def test_repair_maximum_erasures_and_unrepairable(lib):  # extendeddatacrossword_test.go:27-80
    original = example_eds()
    rr, cr = _roots(original)
    flat = original.Flattened()
    for i in (0, 2, 3, 4, 5, 6, 7, 8, 9, 10, 12, 13):
        flat[i] = None
    eds = R.ImportExtendedDataSquare(flat, R.NewLeoRSCodec(), R.NewDefaultTree)
    eds.Repair(rr, cr)
    assert eds.Equals(original)
    flat[14] = None
    eds = R.ImportExtendedDataSquare(flat, R.NewLeoRSCodec(), R.NewDefaultTree)
    with pytest.raises(type(R.ErrUnrepairableDataSquare)):
        eds.Repair(rr, cr)


def test_repair_random_order(lib, rng):  # extendeddatacrossword_test.go:82-113
    original = example_eds()
    rr, cr = _roots(original)
    w = original.Width()
    for _ in range(20):
        new = R.NewExtendedDataSquare(R.NewLeoRSCodec(), R.NewDefaultTree, w, S)
        while True:
            x, y = int(rng.integers(w)), int(rng.integers(w))
            if new.GetCell(x, y) is not None:
                continue
            new.SetCell(x, y, original.GetCell(x, y))
            try:
                new.Repair(rr, cr)
            except R.RSMError as e:
                if e is R.ErrUnrepairableDataSquare:
                    continue
                raise
            break
        assert new.Equals(original)
        assert _roots(new) == (rr, cr)


def test_repair_twice_and_quarter(lib):  # rsmt2d_test.go:79-196
    original = example_eds()
    rr, cr = _roots(original)
    flat = original.Flattened()
    missing = flat[1]
    for i in (0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 12, 13):
        flat[i] = None
    eds = R.ImportExtendedDataSquare(flat, R.NewLeoRSCodec(), R.NewDefaultTree)
    with pytest.raises(type(R.ErrUnrepairableDataSquare)):
        eds.Repair(rr, cr)
    flat[1] = missing
    eds = R.ImportExtendedDataSquare(flat, R.NewLeoRSCodec(), R.NewDefaultTree)
    eds.Repair(rr, cr)
    assert eds.Equals(original)
    q = R.NewExtendedDataSquare(R.NewLeoRSCodec(), R.NewDefaultTree, 4, S)
    for r, c in ((0, 0), (0, 1), (1, 0), (1, 1)):
        q.SetCell(r, c, original.GetCell(r, c))
    q.Repair(rr, cr)
    assert q.Flattened() == original.Flattened()


CORRUPT = bytes([66]) * S


@pytest.mark.parametrize("coords,values", [
    ([(0, 0)], [CORRUPT]),
    ([(0, 3)], [CORRUPT]),
    ([(0, 0), (0, 1), (0, 2), (0, 3)], [CORRUPT, None, None, None]),
    ([(3, 0), (0, 1), (0, 2), (0, 3)], [CORRUPT, None, None, None]),
    ([(0, 0), (1, 1), (2, 2), (3, 3), (0, 1)], [None, None, None, None, CORRUPT]),
])
def test_corrupted_returns_byzantine(lib, coords, values):  # extendeddatacrossword_test.go:185-261
    eds = example_eds()
    rr, cr = _roots(eds)
    for (r, c), v in zip(coords, values):
        eds.setCell(r, c, v)
    with pytest.raises(R.ErrByzantineData) as ei:
        eds.Repair(rr, cr)
    assert ei.value.Shares and CORRUPT in ei.value.Shares


def test_orthogonal_vector_byzantine(lib):  # extendeddatacrossword_test.go:275-359
    eds = example_eds()
    rr, cr = _roots(eds)
    eds.setCell(0, 2, None)
    eds.setCell(2, 0, None)
    eds.setCell(2, 2, CORRUPT)
    with pytest.raises(R.ErrByzantineData) as ei:
        eds.Repair(rr, cr)
    assert (ei.value.Axis, ei.value.Index) == (R.Col, 2)
    assert len(ei.value.Shares) == 4 and CORRUPT in ei.value.Shares and ei.value.Shares[0] is None


def test_byzantine_preserves_nils(lib):  # extendeddatacrossword_test.go:368-405
    eds = example_eds()
    rr, cr = _roots(eds)
    eds.setCell(0, 0, CORRUPT)
    eds.setCell(0, 2, None)
    eds.setCell(0, 3, None)
    eds.setCell(3, 0, None)
    with pytest.raises(R.ErrByzantineData) as ei:
        eds.Repair(rr, cr)
    assert (ei.value.Axis, ei.value.Index) == (R.Row, 0)
    assert ei.value.Shares[2] is None and ei.value.Shares[3] is None and CORRUPT in ei.value.Shares


def test_valid_fraud_proof(lib):  # extendeddatacrossword_test.go:116-163
    codec = R.NewLeoRSCodec()
    original = example_eds()
    corrupted = original.deepCopy(codec)
    corrupted.setCell(0, 0, CORRUPT)
    rr, cr = _roots(corrupted)
    with pytest.raises(R.ErrByzantineData) as ei:
        corrupted.Repair(rr, cr)
    byz = ei.value
    # PseudoFraudProof{0, byzData.Index, byzData.Shares}, verified exactly as the
    # reference does (:144-162): decode the shares, compare the root of the rebuilt
    # vector with getRowRoot(Index); only if they match must the re-encoded parity
    # differ from the rebuilt parity half.
    rebuilt = codec.Decode(list(byz.Shares))
    assert all(s is not None for s in rebuilt)
    root = R._default_root(rebuilt)           # computeSharesRoot(rebuilt, byzData.Axis, Index)
    row_root = rr[byz.Index]                  # getRowRoot(fraudProof.Index)
    if root == row_root:
        odw = corrupted.originalDataWidth
        parity = codec.Encode(rebuilt[:odw])
        assert b"".join(parity) != b"".join(rebuilt[len(rebuilt) - odw:]), "invalid fraud proof"


def test_random_byzantine_8x8_matches_oracle(lib, rng):
    """extendeddatacrossword_test.go:612-744 style: one random corrupt share in a k=8
    square; the GPU Repair must report the same error as the oracle crossword."""
    k = 8
    for trial in range(6):
        ods = [rng.integers(0, 256, 64, dtype=np.uint8).tobytes() for _ in range(k * k)]
        eds = R.ComputeExtendedDataSquare(ods, R.NewLeoRSCodec(), R.NewDefaultTree)
        rr, cr = _roots(eds)
        flat = eds.Flattened()
        idx = int(rng.integers(len(flat)))
        flat[idx] = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
        for j in rng.choice(len(flat), size=len(flat) // 2, replace=False):
            if j != idx:
                flat[j] = None
        mine = R.ImportExtendedDataSquare(flat, R.NewLeoRSCodec(), R.NewDefaultTree)
        try:
            crossword.repair(list(flat), rr, cr)
            want = None
        except crossword.Byzantine as b:
            want = (b.axis, b.index, b.shares)
        except crossword.Unrepairable:
            want = "unrepairable"
        try:
            mine.Repair(rr, cr)
            got = None
        except R.ErrByzantineData as b:
            got = (b.Axis, b.Index, b.Shares)
        except R.RSMError as e:
            assert e is R.ErrUnrepairableDataSquare
            got = "unrepairable"
        assert got == want, trial


def _oracle_repair_keep(flat, rr, cr):
    """oracle crossword.repair, returning ("ok" | "unrepairable" | (axis, index, shares),
    the square's cells afterwards): the reference leaves the cells it solved in place
    when it gives up (extendeddatacrossword.go:74-122)."""
    sq = crossword.Square(list(flat))
    try:
        crossword.pre_repair_sanity_check(sq, rr, cr)
        while True:
            solved, progress = True, False
            for i in range(sq.w):
                s1, p1 = crossword.solve_vector(sq, crossword.Row, i, rr, cr)
                s2, p2 = crossword.solve_vector(sq, crossword.Col, i, cr, rr)
                solved = solved and s1 and s2
                progress = progress or p1 or p2
            if solved:
                return "ok", sq.flattened()
            if not progress:
                return "unrepairable", sq.flattened()
    except crossword.Byzantine as b:
        return (b.axis, b.index, b.shares), sq.flattened()


def test_err_rand_byzantine_incremental(lib, rng):
    """TestErrRandByzantine's protocol (extendeddatacrossword_test.go:612-744): one
    random share of a k = 8 square replaced (its first 29 bytes kept), set first into an
    empty square, then random cells of the corrupted square one at a time with a Repair
    after each, until Repair reports ErrByzantineData -- whose index must be the
    corrupted cell's row or column (checkErrByzantine).  Every Repair's outcome and the
    cells it leaves behind (solved cells stay when it gives up) are compared with the
    oracle crossword on the same cells."""
    k, W = 8, 16
    for trial in range(12):
        ods = [rng.integers(0, 256, S, dtype=np.uint8).tobytes() for _ in range(k * k)]
        original = R.ComputeExtendedDataSquare(ods, R.NewLeoRSCodec(), R.NewDefaultTree)
        flat = original.Flattened()
        idx = int(rng.integers(len(flat)))
        bad = bytearray(rng.integers(0, 256, S, dtype=np.uint8).tobytes())
        bad[:29] = flat[idx][:29]
        flat[idx] = bytes(bad)
        corrupted = R.ImportExtendedDataSquare(flat, R.NewLeoRSCodec(), R.NewDefaultTree)
        assert not original.Equals(corrupted)
        rr, cr = corrupted.RowRoots(), corrupted.ColRoots()
        square = R.NewExtendedDataSquare(R.NewLeoRSCodec(), R.NewDefaultTree, W, S)
        cx, cy = divmod(idx, W)
        square.SetCell(cx, cy, corrupted.GetCell(cx, cy))
        byz = None
        for step in range(40 * W * W):
            x, y = int(rng.integers(W)), int(rng.integers(W))
            if square.GetCell(x, y) is not None:
                continue
            square.SetCell(x, y, corrupted.GetCell(x, y))
            before = square.Flattened()
            want, after = _oracle_repair_keep(before, rr, cr)
            try:
                square.Repair(rr, cr)
                got = "ok"
            except R.ErrByzantineData as b:
                got = (b.Axis, b.Index, b.Shares)
            except R.RSMError as e:
                assert e is R.ErrUnrepairableDataSquare
                got = "unrepairable"
            assert got == want, (trial, step)
            assert got != "ok", "no byzantine error"  # repairNewFromCorrupted
            if got == "unrepairable":
                assert square.Flattened() == after, (trial, step)
                continue
            byz = got
            break
        assert byz is not None
        axis, index, _ = byz
        assert index == (cx if axis == R.Row else cy)  # checkErrByzantine


@pytest.mark.parametrize("k", [16, 128])
def test_repair_half_of_each_row(lib, rng, k):
    """BenchmarkRepair's erasure scheme (extendeddatacrossword_test.go:443-453):
    exactly k of the 2k cells of every row erased; device fast path must repair it."""
    S_ = 512
    ods = [rng.integers(0, 256, S_, dtype=np.uint8).tobytes() for _ in range(k * k)]
    original = R.ComputeExtendedDataSquare(ods, R.NewLeoRSCodec(), R.NewDefaultTree)
    rr, cr = _roots(original)
    flat = original.Flattened()
    w = 2 * k
    for r in range(w):
        for c in rng.choice(w, size=k, replace=False):
            flat[r * w + c] = None
    eds = R.ImportExtendedDataSquare(flat, R.NewLeoRSCodec(), R.NewDefaultTree)
    eds.Repair(rr, cr)
    assert eds.Equals(original)
    assert eds.repair_stats().fast_path == 1


def test_repair_half_of_each_row_byzantine_k128(lib, rng):
    """The zero-copy row sweep (k = 128, every row decodable) with one corrupted
    present share: the device verification rejects it, the EDS is left as it was
    (rebuilt bytes only ever land in nil cells), and the exact sequential solver
    reports the same ErrByzantineData as the oracle crossword."""
    k, S_ = 128, 64
    ods = [rng.integers(0, 256, S_, dtype=np.uint8).tobytes() for _ in range(k * k)]
    original = R.ComputeExtendedDataSquare(ods, R.NewLeoRSCodec(), R.NewDefaultTree)
    rr, cr = _roots(original)
    flat = original.Flattened()
    w = 2 * k
    for r in range(w):
        for c in rng.choice(w, size=k, replace=False):
            flat[r * w + c] = None
    present = [i for i, s in enumerate(flat) if s is not None]
    bad = present[len(present) // 3]
    flat[bad] = bytes(b ^ 0x5A for b in flat[bad])
    eds = R.ImportExtendedDataSquare(flat, R.NewLeoRSCodec(), R.NewDefaultTree)
    before = eds.Flattened()
    try:
        crossword.repair(list(flat), rr, cr)
        want = None
    except crossword.Byzantine as b:
        want = (b.axis, b.index, b.shares)
    with pytest.raises(R.ErrByzantineData) as ei:
        eds.Repair(rr, cr)
    assert (ei.value.Axis, ei.value.Index, ei.value.Shares) == want
    assert eds.repair_stats().fast_path == 0
    # nil cells stay nil and present cells unchanged up to the exact solver's own
    # progress (it inserts verified rows before meeting the byzantine one)
    after = eds.Flattened()
    assert all(a == b for a, b in zip(before, after) if a is not None)


def test_cannot_repair_square_with_bad_roots(lib):  # extendeddatacrossword_test.go:165-183
    """Roots taken from the original, then one cell of the (complete) square
    replaced: Repair must fail (the pre-repair check finds row 0 / column 0
    inconsistent with its committed root)."""
    original = example_eds()
    rr, cr = _roots(original)
    original.setCell(0, 0, CORRUPT)
    with pytest.raises(R.RSMError):
        original.Repair(rr, cr)
