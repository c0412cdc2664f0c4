"""CPU: the C ABI library loads, exports every symbol include/rsmt2d_hip.h declares,
and its host-only logic (shape/size validation, grid get/set, DefaultTree roots)
matches the reference semantics.  No compute call runs without a GPU."""
import os
import re

import numpy as np
import pytest

import rsmt2d_amd as R
from oracle import crossword
from conftest import const_share, rand_shares

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "rsmt2d_hip.h")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(rsm_[a-z0-9_]+)\s*\(", txt)) - {"rsm_tree_root_fn"})


def test_every_declared_symbol_is_exported(lib):
    syms = declared_symbols()
    assert len(syms) >= 30
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(R.SIGNATURES), set(syms) ^ set(R.SIGNATURES)


def test_codec_surface(lib):
    codec = R.NewLeoRSCodec()
    assert codec.Name() == "Leopard" == R.Leopard                 # codecs.go:11
    assert codec.MaxChunks() == 32768 * 32768                      # leopard.go:76-84
    assert codec.ValidateChunkSize(512) is None                    # leopard.go:92-99
    assert codec.ValidateChunkSize(64) is None
    assert codec.ValidateChunkSize(65).code == R.RSM_ESHARESIZE
    assert lib.rsm_codec_field_bits(128) == 8 and lib.rsm_codec_field_bits(129) == 16


def test_import_flattened_and_cells(lib, rng):
    shares = rand_shares(rng, 16, 64)
    shares[5] = None
    eds = R.ImportExtendedDataSquare(shares, R.NewLeoRSCodec(), R.NewDefaultTree)
    assert eds.Width() == 4 and eds.originalDataWidth == 2 and eds.shareSize == 64
    assert eds.Flattened() == shares
    assert eds.GetCell(1, 1) is None
    assert eds.GetCell(0, 1) == shares[1]
    with pytest.raises(R.RSMError) as e:                            # SetCell on non-nil
        eds.SetCell(0, 1, shares[1])
    assert e.value.code == R.RSM_ECELL
    with pytest.raises(R.RSMError):                                 # wrong size
        eds.SetCell(1, 1, b"\0" * 65)
    eds.SetCell(1, 1, b"\7" * 64)
    assert eds.GetCell(1, 1) == b"\7" * 64
    assert eds.Row(1)[1] == b"\7" * 64 and eds.Col(1)[1] == b"\7" * 64


def test_shape_errors(lib):
    codec = R.NewLeoRSCodec()
    with pytest.raises(R.RSMError) as e:                            # extendeddatasquare_test.go:84-88
        R.ImportExtendedDataSquare([b"\1" * 65], codec, R.NewDefaultTree)
    assert e.value.code == R.RSM_ESHARESIZE
    with pytest.raises(R.RSMError) as e:                            # datasquare_test.go:48-65
        R.ImportExtendedDataSquare([b"\1" * 64] * 3, codec, R.NewDefaultTree)
    assert e.value.code == R.RSM_ESHAPE
    with pytest.raises(R.RSMError) as e:                            # uneven shares
        R.ImportExtendedDataSquare([b"\1" * 64] * 3 + [b"\1" * 128], codec, R.NewDefaultTree)
    assert e.value.code == R.RSM_ESHAPE
    with pytest.raises(R.RSMError) as e:                            # odd EDS width
        R.ImportExtendedDataSquare([b"\1" * 64] * 9, codec, R.NewDefaultTree)
    assert e.value.code == R.RSM_ESHAPE
    with pytest.raises(R.RSMError):                                 # NewExtendedDataSquare odd width
        R.NewExtendedDataSquare(codec, R.NewDefaultTree, 1, 512)
    with pytest.raises(R.RSMError):                                 # ... and bad share size
        R.NewExtendedDataSquare(codec, R.NewDefaultTree, 4, 65)
    eds = R.NewExtendedDataSquare(codec, R.NewDefaultTree, 4, 512)  # extendeddatasquare_test.go:131-146
    assert eds.Width() == 4 and eds.shareSize == 512
    eds.SetCell(0, 0, const_share(1))
    assert eds.GetCell(0, 0) == const_share(1)


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7, 8, 13, 16, 70])
def test_default_tree_matches_restatement(lib, rng, n):
    leaves = rand_shares(rng, n, 64)
    assert R._default_root(leaves) == crossword.merkle_root(leaves)


@pytest.mark.parametrize("n,size", [(9, 1), (17, 55), (33, 56), (256, 512), (257, 119), (100, 575)])
def test_default_tree_batched_hashing(lib, rng, n, size):
    """merkle.cpp hashes leaves and nodes eight messages at a time (multi-buffer
    SHA-NI): ragged batches, odd lengths and every padding boundary (a 1-byte prefix
    plus 55 / 56 payload bytes: the length field in the same block or the next)."""
    leaves = [rng.integers(0, 256, size, dtype=np.uint8).tobytes() for _ in range(n)]
    assert R._default_root(leaves) == crossword.merkle_root(leaves)


def test_roots_of_imported_square(lib, rng):
    shares = rand_shares(rng, 64, 128)
    eds = R.ImportExtendedDataSquare(shares, R.NewLeoRSCodec(), R.NewDefaultTree)
    sq = crossword.Square(shares)
    assert eds.RowRoots() == sq.roots(crossword.Row)
    assert eds.ColRoots() == sq.roots(crossword.Col)
    assert eds.Roots() == sq.roots(crossword.Row) + sq.roots(crossword.Col)
    eds.setCell(0, 0, None)                                         # extendeddatasquare_test.go:250-262
    with pytest.raises(R.RSMError) as e:
        eds.RowRoots()
    assert e.value.code == R.RSM_ETREE


def test_custom_tree_plugin(lib, rng):
    class XorTree(R.Tree):
        def __init__(self):
            self.acc = bytearray(8)

        def Push(self, d):
            for i, b in enumerate(d[:8]):
                self.acc[i] ^= b

        def Root(self):
            return bytes(self.acc)

    shares = rand_shares(rng, 16, 64)
    eds = R.ImportExtendedDataSquare(shares, R.NewLeoRSCodec(), lambda axis, idx: XorTree())
    roots = eds.RowRoots()
    assert len(roots) == 4 and all(len(r) == 8 for r in roots)


def test_json_roundtrip_host_only(lib, rng):
    shares = rand_shares(rng, 16, 64)
    eds = R.ImportExtendedDataSquare(shares, R.NewLeoRSCodec(), R.NewDefaultTree)
    back = R.ExtendedDataSquare.UnmarshalJSON(eds.MarshalJSON())
    assert back.Equals(eds)


def test_no_gpu_fails_loudly(lib):
    if lib.rsm_device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(R.DeviceError):
        R.NewLeoRSCodec().Encode([b"\1" * 64] * 2)


DIAG_HEADER = os.path.join(os.path.dirname(HEADER), "rsmt2d_hip_diag.h")


def test_product_has_no_diagnostics(lib):
    """The shipped library carries only the production kernels and no switch that
    could change results: the A-B / no-arithmetic / no-memory / fused / pipelined
    kernels and every environment knob live in librsmt2d_hip_diag.so only (VERDICT
    round 1, item 7).  getenv needs the variable's name in the binary, so the absence
    of every RSM_* name proves no environment variable can reach the product."""
    blob = open(R.LIB_PATH, "rb").read()
    for name in (b"RSM_BS_MODE", b"RSM_BS_REV", b"RSM_BS_XCD", b"RSM_BS_ROWGRID", b"RSM_BS_COLGRID", b"RSM_FUSED",
                 b"RSM_GF8_KERNEL", b"RSM_GF16_BATCH_MB"):
        assert name not in blob, name
    assert not re.search(rb"RSM_[A-Z0-9_]{3,}\x00", blob), re.search(rb"RSM_[A-Z0-9_]{3,}\x00", blob)
    # kernel symbols embedded in the gfx950 code object: only the production modes
    # of the bit-sliced encode (row pass 104, column pass 184, the single-launch
    # half-split queue extension: 16777216 with fixed per-lane set offsets where S divides
    # the set width, 0 otherwise -- kernels_gf8_bs.hip), no diagnostic mode (bits
    # 2 / 4 / 32768: no arithmetic / no memory / no exchange), no round-2 queue
    # kernel (diag A/B only), no dual (bs128p) kernel
    modes = set(re.findall(rb"encode_gf8_bs128u_kernelILi(\d+)E", blob))
    assert modes == {b"104", b"184"}, modes
    smodes = set(re.findall(rb"extend_gf8_bs128s_kernelILi(\d+)E", blob))
    assert smodes == {b"0", b"16777216"}, smodes
    assert b"extend_gf8_bs128q_kernel" not in blob
    assert not any(int(m) & (6 | 32768) for m in modes | smodes)
    assert b"encode_gf8_bs128p_kernel" not in blob
    txt = re.sub(r"/\*.*?\*/", "", open(DIAG_HEADER).read(), flags=re.S)
    for s in set(re.findall(r"\b(rsm_diag_[a-z0-9_]+)\s*\(", txt)):
        assert not hasattr(lib, s), s
    for s in ("rsm_set_fused", "rsm_fused_trace", "rsm_extend_fused", "rsm_extend_pipeline_dev", "rsm_set_pass_grid"):
        assert not hasattr(lib, s), s


def test_diag_library_is_separate():
    if not os.path.exists(R.DIAG_LIB_PATH):
        pytest.skip("diagnostic library not built")
    blob = open(R.DIAG_LIB_PATH, "rb").read()
    assert set(re.findall(rb"extend_gf8_bs128q_kernelILi(\d+)E", blob)) > {b"18472"}  # round-2 schedule, A-B
    assert set(re.findall(rb"extend_gf8_bs128s_kernelILi(\d+)E", blob)) > {b"0"}  # + diagnostic modes
    dl = R.diag_library()
    for s in R.DIAG_SIGNATURES:
        assert hasattr(dl, s), s
