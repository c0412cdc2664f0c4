"""CPU oracle for the rsmt2d hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package.  The product (``rsmt2d_amd``) never does.

* ``libleopard_oracle.so`` (built from ``leopard_oracle.c`` by ``make``) is a scalar C
  restatement of klauspost/reedsolomon v1.14.1's Leopard codec as configured by
  rsmt2d's ``LeoRSCodec`` (``leopard.go:28-72``).  That Go module is absent from
  ``/root/reference`` and no Go toolchain exists here, so parity is pinned only by
  the reference's own known-answer grids (``extendeddatasquare_test.go:39-59``);
  every larger size is "parity unpinned vs LeoRSCodec" (DESIGN.md).
* ``crossword.py`` restates ``extendeddatacrossword.go`` (Repair) in Python over this
  codec, for small squares.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libleopard_oracle.so")
_lib = None
_lock = threading.Lock()


def build() -> str:
    """Compile the C restatement (make)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(_LIB_PATH):
                build()
            L = ctypes.CDLL(_LIB_PATH)
            P = ctypes.POINTER(ctypes.c_void_p)
            L.leo_field_bits.argtypes = [ctypes.c_uint]
            L.leo_field_bits.restype = ctypes.c_int
            L.leo_encode.argtypes = [ctypes.c_uint, ctypes.c_size_t, P, P]
            L.leo_encode.restype = ctypes.c_int
            L.leo_decode.argtypes = [ctypes.c_uint, ctypes.c_size_t, P, ctypes.c_char_p]
            L.leo_decode.restype = ctypes.c_int
            L.leo_extend_square.argtypes = [ctypes.c_uint, ctypes.c_size_t, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_int]
            L.leo_extend_square.restype = ctypes.c_int
            L.leo_tables8.argtypes = [ctypes.c_void_p] * 4
            L.leo_tables16.argtypes = [ctypes.c_void_p] * 4
            _lib = L
    return _lib


def field_bits(k: int) -> int:
    """8 when the 2k-shard code fits GF(2^8) (2k <= 256), else 16 (codecs.go:6-10)."""
    return lib().leo_field_bits(k)


def _ptr_array(bufs):
    arr = (ctypes.c_void_p * len(bufs))()
    for i, b in enumerate(bufs):
        arr[i] = b.ctypes.data if b is not None else None
    return arr


def encode(data):
    """LeoRSCodec.Encode (leopard.go:28-45): k shares -> k new parity shares."""
    k = len(data)
    shares = [np.ascontiguousarray(np.frombuffer(bytes(d), dtype=np.uint8)) for d in data]
    S = shares[0].size
    parity = [np.zeros(S, dtype=np.uint8) for _ in range(k)]
    rc = lib().leo_encode(k, S, _ptr_array(shares), _ptr_array(parity))
    if rc != 0:
        raise ValueError(f"leo_encode failed rc={rc}")
    return [bytes(p) for p in parity]


class TooFewShards(Exception):
    pass


def decode(shares):
    """LeoRSCodec.Decode (leopard.go:51-59): 2k slots, None = missing; returns a new
    list with the missing slots filled (the reference fills in place)."""
    n = len(shares)
    k = n // 2
    S = next((len(s) for s in shares if s is not None), None)
    if S is None:
        raise TooFewShards("too few shards given")
    bufs = [np.frombuffer(bytes(s), dtype=np.uint8).copy() if s is not None
            else np.zeros(S, dtype=np.uint8) for s in shares]
    present = bytes(1 if s is not None else 0 for s in shares)
    rc = lib().leo_decode(k, S, _ptr_array(bufs), present)
    if rc == -3:
        raise TooFewShards("too few shards given")
    if rc != 0:
        raise ValueError(f"leo_decode failed rc={rc}")
    return [bytes(b) for b in bufs]


def extend_square(ods: np.ndarray, nthreads: int = 1) -> np.ndarray:
    """erasureExtendSquare (extendeddatasquare.go:154-227) on a [k, k, S] uint8 ODS."""
    ods = np.ascontiguousarray(ods, dtype=np.uint8)
    k, k2, S = ods.shape
    assert k == k2
    eds = np.empty((2 * k, 2 * k, S), dtype=np.uint8)
    rc = lib().leo_extend_square(k, S, ods.ctypes.data, eds.ctypes.data, int(nthreads))
    if rc != 0:
        raise ValueError(f"leo_extend_square failed rc={rc}")
    return eds


_simd = None


def simd_lib() -> ctypes.CDLL:
    """libleopard_simd.so: the same restatement with AVX2 pshufb nibble-table rows
    (LEO_SIMD) -- bench.py's cpu_baseline only, checked against the scalar oracle in
    tests/test_oracle.py.  A restatement of klauspost's SIMD technique, not the
    reference itself (which needs Go and the absent klauspost module)."""
    global _simd
    with _lock:
        if _simd is None:
            path = os.path.join(_HERE, "libleopard_simd.so")
            if not os.path.exists(path):
                build()
            L = ctypes.CDLL(path)
            L.leo_extend_square.argtypes = [ctypes.c_uint, ctypes.c_size_t, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_int]
            L.leo_extend_square.restype = ctypes.c_int
            _simd = L
    return _simd


def extend_square_simd(ods: np.ndarray, nthreads: int = 1, out: np.ndarray = None) -> np.ndarray:
    ods = np.ascontiguousarray(ods, dtype=np.uint8)
    k, _, S = ods.shape
    eds = out if out is not None else np.empty((2 * k, 2 * k, S), dtype=np.uint8)
    assert eds.shape == (2 * k, 2 * k, S) and eds.dtype == np.uint8 and eds.flags.c_contiguous
    rc = simd_lib().leo_extend_square(k, S, ods.ctypes.data, eds.ctypes.data, int(nthreads))
    if rc != 0:
        raise ValueError(f"leo_extend_square (simd) failed rc={rc}")
    return eds


_gfni = None


def gfni_supported() -> bool:
    """GFNI + AVX-512BW on this host (the GPU box's EPYC 9575F has both)."""
    try:
        flags = open("/proc/cpuinfo").read()
    except OSError:
        return False
    return " gfni" in flags and " avx512bw" in flags


def gfni_lib() -> ctypes.CDLL:
    """libleopard_gfni.so: the restatement with AVX-512 rows, GF2P8AFFINEQB multiplies
    and fused GF(2^8) butterflies (LEO_GFNI) -- bench.py's cpu_baseline only, checked
    against the scalar oracle in tests/test_oracle.py (klauspost's fastest x86
    leopard8 technique, restated; not the reference)."""
    global _gfni
    with _lock:
        if _gfni is None:
            path = os.path.join(_HERE, "libleopard_gfni.so")
            if not os.path.exists(path):
                build()
            L = ctypes.CDLL(path)
            L.leo_extend_square.argtypes = [ctypes.c_uint, ctypes.c_size_t, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_int]
            L.leo_extend_square.restype = ctypes.c_int
            _gfni = L
    return _gfni


def extend_square_gfni(ods: np.ndarray, nthreads: int = 1, out: np.ndarray = None) -> np.ndarray:
    ods = np.ascontiguousarray(ods, dtype=np.uint8)
    k, _, S = ods.shape
    eds = out if out is not None else np.empty((2 * k, 2 * k, S), dtype=np.uint8)
    assert eds.shape == (2 * k, 2 * k, S) and eds.dtype == np.uint8 and eds.flags.c_contiguous
    rc = gfni_lib().leo_extend_square(k, S, ods.ctypes.data, eds.ctypes.data, int(nthreads))
    if rc != 0:
        raise ValueError(f"leo_extend_square (gfni) failed rc={rc}")
    return eds


def tables8():
    e = np.zeros(256, np.uint8)
    lg = np.zeros(256, np.uint8)
    sk = np.zeros(255, np.uint8)
    lw = np.zeros(256, np.uint8)
    lib().leo_tables8(e.ctypes.data, lg.ctypes.data, sk.ctypes.data, lw.ctypes.data)
    return e, lg, sk, lw


def tables16():
    e = np.zeros(65536, np.uint16)
    lg = np.zeros(65536, np.uint16)
    sk = np.zeros(65535, np.uint16)
    lw = np.zeros(65536, np.uint16)
    lib().leo_tables16(e.ctypes.data, lg.ctypes.data, sk.ctypes.data, lw.ctypes.data)
    return e, lg, sk, lw


def splitmix64_bytes(n: int, seed: int = 0x52534D543244) -> np.ndarray:
    """Seeded uniform bytes (SplitMix64), the BASELINE.md input generator."""
    nwords = (n + 7) // 8
    idx = np.arange(1, nwords + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + idx * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.view(np.uint8)[:n].copy()


def affine_pattern(k: int, S: int) -> np.ndarray:
    """SURVEY Appendix B input: ods[r][c][b] = (r*251 + c*17 + b*3 + 5) mod 256."""
    r = np.arange(k).reshape(k, 1, 1)
    c = np.arange(k).reshape(1, k, 1)
    b = np.arange(S).reshape(1, 1, S)
    return ((r * 251 + c * 17 + b * 3 + 5) % 256).astype(np.uint8)
