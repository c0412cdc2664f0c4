"""rsmt2d_amd -- Python mirror of celestiaorg/rsmt2d's API over the MI355X engine.

The product is ``librsmt2d_hip.so`` (HIP kernels for gfx950 + C++ host runtime,
C ABI in ``include/rsmt2d_hip.h``).  This module is a thin ``ctypes`` binding
that keeps the reference's names and semantics so tests read like the
reference's own:

    codec = NewLeoRSCodec()                                   # leopard.go:101
    eds = ComputeExtendedDataSquare(shares, codec, NewDefaultTree)
    row_roots, col_roots = eds.RowRoots(), eds.ColRoots()
    eds2 = ImportExtendedDataSquare(flattened_with_nones, codec, NewDefaultTree)
    eds2.Repair(row_roots, col_roots)    # raises ErrByzantineData / ErrUnrepairableDataSquare

Every compute entry point runs the HIP path; with no GPU it raises
``DeviceError`` -- there is no CPU fallback.
"""
from __future__ import annotations

import base64
import ctypes
import json
import math
import os
import subprocess
import threading
from typing import Callable, List, Optional, Sequence

__all__ = [
    "Leopard", "Row", "Col", "Axis", "Codec", "LeoRSCodec", "NewLeoRSCodec",
    "ExtendedDataSquare", "ComputeExtendedDataSquare", "ImportExtendedDataSquare",
    "NewExtendedDataSquare", "NewDefaultTree", "Tree", "ErrByzantineData",
    "ComputeExtendedDataSquareWithBuffer", "BufferedTreeConstructor", "NmtParams",
    "ErasuredNamespacedMerkleTreeConstructor", "newErasuredNamespacedMerkleTreeConstructor",
    "TreePool", "newTreePool",
    "ErrUnrepairableDataSquare", "ErrUnevenChunks", "RSMError", "DeviceError",
    "library", "build", "device_context",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "librsmt2d_hip.so")

Leopard = "Leopard"  # codecs.go:11
Row = 0              # extendeddatacrossword.go:15-18
Col = 1
Axis = int

# rsmt2d_hip.h return codes
RSM_OK, RSM_EINVAL, RSM_ESHARESIZE, RSM_ETOOFEW, RSM_ESHAPE, RSM_EDEVICE = 0, -1, -2, -3, -4, -5
RSM_ENOMEM, RSM_EUNSUPPORTED, RSM_EUNREPAIRABLE, RSM_EBYZANTINE, RSM_ECELL, RSM_ETREE = -6, -7, -8, -9, -10, -11


class RSMError(Exception):
    """Error returned by the C ABI (code = RSM_E*)."""

    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


class DeviceError(RSMError):
    """No usable GPU / HIP failure.  The product never falls back to the CPU."""


class _Unrepairable(RSMError):
    pass


#: ErrUnrepairableDataSquare (extendeddatacrossword.go:37) -- a singleton like the Go sentinel.
ErrUnrepairableDataSquare = _Unrepairable(RSM_EUNREPAIRABLE, "failed to solve data square")

#: ErrUnevenChunks (datasquare.go:14)
ErrUnevenChunks = "non-nil shares not all of equal size"


class ErrByzantineData(RSMError):
    """ErrByzantineData (extendeddatacrossword.go:42-58): Axis, Index, Shares (None = missing)."""

    def __init__(self, axis: int, index: int, shares: List[Optional[bytes]]):
        super().__init__(RSM_EBYZANTINE, f"byzantine {'row' if axis == Row else 'col'}: {index}")
        self.Axis = axis
        self.Index = index
        self.Shares = shares


# ---------------------------------------------------------------------------
# library loading
# ---------------------------------------------------------------------------
_lib = None
# re-entrant: a __del__ run by the garbage collector while the lock is held calls library()
_lib_lock = threading.RLock()
_TREE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32,
                            ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32, ctypes.c_uint32,
                            ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_uint32))


class _Byz(ctypes.Structure):
    _fields_ = [("axis", ctypes.c_int32), ("index", ctypes.c_uint32)]


class NmtParams(ctypes.Structure):
    """rsm_nmt_params (include/rsmt2d_hip.h)."""
    _fields_ = [("namespace_size", ctypes.c_uint32), ("ignore_max_namespace", ctypes.c_uint32),
                ("square_size", ctypes.c_uint32)]


class RepairStats(ctypes.Structure):
    _fields_ = [("fast_path", ctypes.c_int32), ("sweeps", ctypes.c_uint32),
                ("decoded_vectors", ctypes.c_uint32), ("fallback_reason", ctypes.c_uint32)]


# (name, restype, argtypes) of every symbol declared in include/rsmt2d_hip.h
_VP, _U8P, _U32, _I32, _I64, _U64 = (ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                     ctypes.c_int, ctypes.c_int64, ctypes.c_uint64)
SIGNATURES = {
    "rsm_ctx_create": (_I32, [_I32, ctypes.POINTER(_VP)]),
    "rsm_ctx_destroy": (None, [_VP]),
    "rsm_ctx_device": (_I32, [_VP]),
    "rsm_ctx_set_pass_grid": (_I32, [_VP, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    "rsm_ctx_set_split_max": (_I32, [_VP, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    "rsm_ctx_set_limits": (_I32, [_VP, _U64, _U64]),
    "rsm_last_error": (ctypes.c_char_p, []),
    "rsm_version": (ctypes.c_char_p, []),
    "rsm_device_count": (_I32, []),
    "rsm_codec_name": (ctypes.c_char_p, []),
    "rsm_codec_max_chunks": (_I64, []),
    "rsm_codec_validate_chunk_size": (_I32, [_I64]),
    "rsm_codec_field_bits": (_I32, [_U32]),
    "rsm_encode": (_I32, [_VP, _VP, _U32, _U32, _VP]),
    "rsm_decode": (_I32, [_VP, _VP, _VP, _U32, _U32]),
    "rsm_extend_square": (_I32, [_VP, _VP, _U32, _U32, _VP]),
    "rsm_extend_square_inplace_host": (_I32, [_VP, _VP, _U32, _U32]),
    "rsm_extend_squares_host": (_I32, [_VP, _VP, _U32, _U32, _U32, _VP]),
    "rsm_host_alloc": (_I32, [_VP, _U64, ctypes.POINTER(_VP)]),
    "rsm_host_free": (_I32, [_VP, _VP]),
    "rsm_multi_create": (_I32, [_VP, ctypes.c_int, ctypes.POINTER(_VP)]),
    "rsm_multi_destroy": (None, [_VP]),
    "rsm_multi_size": (_I32, [_VP]),
    "rsm_multi_context": (_VP, [_VP, ctypes.c_int]),
    "rsm_multi_extend_square": (_I32, [_VP, _VP, _U32, _U32, _VP, ctypes.c_int]),
    "rsm_multi_extend_dev": (_I32, [_VP, _VP, _U32, _U32, ctypes.c_int]),
    "rsm_multi_sync": (_I32, [_VP]),
    "rsm_multi_host_alloc": (_I32, [_VP, _U64, ctypes.POINTER(_VP)]),
    "rsm_multi_host_free": (_I32, [_VP, _VP]),
    "rsm_multi_extend_square_inplace": (_I32, [_VP, _VP, _U32, _U32, ctypes.c_int]),
    "rsm_extend_squares_dev": (_I32, [_VP, _VP, _U32, _U32, _U32, _VP]),
    "rsm_extend_squares_phase_dev": (_I32, [_VP, _VP, _U32, _U32, _U32, _I32, _VP]),
    "rsm_extend_rows_dev": (_I32, [_VP, _VP, _U32, _U32, _U32, _U32, _VP]),
    "rsm_extend_rows_blocks_dev": (_I32, [_VP, _VP, _U32, _U32, _U32, _U32, _VP, _U32, _VP]),
    "rsm_extend_cols_dev": (_I32, [_VP, _VP, _U32, _U32, _U32, _U32, _VP]),
    "rsm_roots_dev": (_I32, [_VP, _VP, _U32, _U32, _VP, _VP]),
    "rsm_roots_squares_dev": (_I32, [_VP, _VP, _U32, _U32, _U32, _VP, _VP]),
    "rsm_encode_batch_dev": (_I32, [_VP, _VP, _VP, _U32, _U32, _U32, _U64, _U64, _VP]),
    "rsm_decode_vectors_dev": (_I32, [_VP, _VP, _VP, _U32, _U32, _I32, _VP, _U32, _VP]),
    "rsm_ctx_stream": (_VP, [_VP]),
    "rsm_dev_alloc": (_I32, [_VP, _U64, ctypes.POINTER(_VP)]),
    "rsm_dev_free": (_I32, [_VP, _VP]),
    "rsm_memcpy": (_I32, [_VP, _VP, _VP, _U64, _I32]),
    "rsm_dev_fill_random": (_I32, [_VP, _VP, _U64, _U64]),
    "rsm_sync": (_I32, [_VP]),
    "rsm_event_create": (_I32, [_VP, ctypes.POINTER(_VP)]),
    "rsm_event_destroy": (_I32, [_VP]),
    "rsm_event_record": (_I32, [_VP, _VP, _VP]),
    "rsm_event_elapsed_ms": (_I32, [_VP, _VP, ctypes.POINTER(ctypes.c_float)]),
    "rsm_stream_create": (_I32, [_VP, ctypes.POINTER(_VP)]),
    "rsm_stream_destroy": (_I32, [_VP, _VP]),
    "rsm_stream_sync": (_I32, [_VP]),
    "rsm_stream_check": (_I32, [_VP, _VP]),
    "rsm_dev_equal": (_I32, [_VP, _VP, _VP, _U64, _VP, ctypes.POINTER(ctypes.c_int)]),
    "rsm_time_extend": (_I32, [_VP, _VP, _U32, _U32, _U32, _U32, ctypes.POINTER(ctypes.c_float),
                               ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]),
    "rsm_default_tree_root": (_I32, [_VP, _I32, _U32, _VP, _U32, _U32, _VP, _VP]),
    "rsm_nmt_tree_root": (_I32, [_VP, _I32, _U32, _VP, _U32, _U32, _VP, _VP]),
    "rsm_nmt_roots_dev": (_I32, [_VP, _VP, _U32, _U32, ctypes.POINTER(NmtParams), _VP, _VP, _VP]),
    "rsm_nmt_roots_squares_dev": (_I32, [_VP, _VP, _U32, _U32, _U32, ctypes.POINTER(NmtParams), _VP, _VP, _VP]),
    "rsm_eds_compute": (_I32, [_VP, _VP, _VP, _U64, ctypes.POINTER(_VP)]),
    "rsm_eds_import": (_I32, [_VP, _VP, _VP, _U64, ctypes.POINTER(_VP)]),
    "rsm_eds_new": (_I32, [_VP, _U32, _U32, ctypes.POINTER(_VP)]),
    "rsm_eds_free": (None, [_VP]),
    "rsm_eds_set_context": (_I32, [_VP, _VP]),
    "rsm_eds_width": (_U32, [_VP]),
    "rsm_eds_original_width": (_U32, [_VP]),
    "rsm_eds_share_size": (_U32, [_VP]),
    "rsm_eds_get_cell": (_I32, [_VP, _U32, _U32, _VP]),
    "rsm_eds_set_cell": (_I32, [_VP, _U32, _U32, _VP, _U32]),
    "rsm_eds_overwrite_cell": (_I32, [_VP, _U32, _U32, _VP, _U32]),
    "rsm_eds_flattened": (_I32, [_VP, _VP, _VP]),
    "rsm_eds_roots": (_I32, [_VP, _I32, _VP, _VP, _VP, _U32, ctypes.POINTER(_U32)]),
    "rsm_eds_repair": (_I32, [_VP, _VP, _VP, _U32, _VP, _VP, ctypes.POINTER(_Byz)]),
    "rsm_eds_byzantine_shares": (_I32, [_VP, _VP, _VP]),
    "rsm_eds_repair_stats": (_I32, [_VP, ctypes.POINTER(RepairStats)]),
}


#: entry points of the diagnostic library only (include/rsmt2d_hip_diag.h)
DIAG_SIGNATURES = {
    "rsm_diag_set_bs_mode": (_I32, [ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "rsm_diag_set_trace": (_I32, [_VP]),
    "rsm_diag_set_dec_trace": (_I32, [_VP]),
    "rsm_diag_set_split_waves": (_I32, [ctypes.c_int, ctypes.c_int]),
    "rsm_diag_set_split_fused": (_I32, [ctypes.c_int]),
    "rsm_diag_set_enc16_e64": (_I32, [ctypes.c_int]),
    "rsm_diag_set_dec16_five_pass": (_I32, [ctypes.c_int]),
    "rsm_diag_set_dec_delay": (_I32, [ctypes.c_uint32]),
    "rsm_diag_set_dec8_mode": (_I32, [ctypes.c_uint32]),
    "rsm_diag_set_codec_spin": (_I32, [ctypes.c_uint32]),
    "rsm_diag_set_repair_mode": (_I32, [ctypes.c_uint32]),
    "rsm_diag_set_dec16_mode": (_I32, [ctypes.c_uint32]),
    "rsm_diag_set_bs_row_mode": (_I32, [ctypes.c_int]),
    "rsm_diag_extend_fused": (_I32, [_VP, _VP, _U32, _U32, _U32, _U32, _VP]),
    "rsm_diag_queue_check": (_I32, [_VP, _VP]),
    "rsm_diag_extend_pipeline_dev": (_I32, [_VP, _VP, _VP, _U32, _U32, _U32, _VP]),
    "rsm_diag_alltoall_emulated": (_I32, [_VP, _VP, ctypes.c_int, _U32, _U32]),
}
# (A/B runs may point the DIAGNOSTIC library at a variant build; the product library
# path is fixed)
DIAG_LIB_PATH = os.environ.get("RSM_DIAG_LIB") or os.path.join(_HERE, "librsmt2d_hip_diag.so")


def build(diag: bool = True) -> str:
    """Compile librsmt2d_hip.so for gfx950 (make in rsmt2d_amd/csrc); with ``diag``
    also the measurement-only librsmt2d_hip_diag.so (-DRSM_DIAG)."""
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(_HERE, "csrc")], check=True)
    if diag:
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(_HERE, "csrc"), "diag"], check=True)
    return LIB_PATH


_diag = None


def diag_library() -> ctypes.CDLL:
    """The DIAGNOSTIC library (A-B / no-arithmetic / fused kernels): measurement
    tooling, never the product.  It carries its own HIP state: do not mix its
    contexts with library()'s."""
    global _diag
    with _lib_lock:
        if _diag is None:
            if not os.path.exists(DIAG_LIB_PATH):
                raise DeviceError(RSM_EDEVICE, f"{DIAG_LIB_PATH} is missing: run rsmt2d_amd.build()")
            L = ctypes.CDLL(DIAG_LIB_PATH)
            for name, (res, args) in list(SIGNATURES.items()) + list(DIAG_SIGNATURES.items()):
                f = getattr(L, name)
                f.restype = res
                f.argtypes = args
            _diag = L
    return _diag


def library() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    with _lib_lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise DeviceError(RSM_EDEVICE, f"{LIB_PATH} is missing: run rsmt2d_amd.build() "
                                               "(the HIP extension is required; there is no CPU path)")
            L = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                f = getattr(L, name)
                f.restype = res
                f.argtypes = args
            _lib = L
    return _lib


def _err(rc: int) -> RSMError:
    msg = (library().rsm_last_error() or b"").decode(errors="replace")
    if rc == RSM_EDEVICE:
        return DeviceError(rc, msg)
    return RSMError(rc, msg)


def _check(rc: int) -> None:
    if rc != RSM_OK:
        raise _err(rc)


def _check_with(L: ctypes.CDLL, rc: int) -> None:
    """_check for a call into another copy of the ABI (the diagnostic library)."""
    if rc != RSM_OK:
        msg = (L.rsm_last_error() or b"").decode(errors="replace")
        raise (DeviceError if rc == RSM_EDEVICE else RSMError)(rc, msg)


_ctx = {}
_ctx_lock = threading.Lock()


def device_context(device: int = 0) -> int:
    """The per-process rsm_ctx for a GPU (created on first use)."""
    with _ctx_lock:
        if device not in _ctx:
            h = ctypes.c_void_p()
            _check(library().rsm_ctx_create(device, ctypes.byref(h)))
            _ctx[device] = h.value
        return _ctx[device]


class DeviceBuffer:
    """Device memory owned by this library's HIP runtime (bench / tests plumbing)."""

    def __init__(self, nbytes: int, device: int = 0):
        self.ctx = device_context(device)
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        _check(library().rsm_dev_alloc(self.ctx, self.nbytes, ctypes.byref(p)))
        self.ptr = p.value

    def fill_random(self, seed: int):
        _check(library().rsm_dev_fill_random(self.ctx, self.ptr, self.nbytes, seed))

    def upload(self, arr, offset: int = 0):
        import numpy as np
        a = np.ascontiguousarray(arr)
        _check(library().rsm_memcpy(self.ctx, self.ptr + offset, a.ctypes.data, a.nbytes, 0))

    def download(self, nbytes: int = None, offset: int = 0):
        import numpy as np
        n = self.nbytes - offset if nbytes is None else nbytes
        out = np.empty(n, np.uint8)
        _check(library().rsm_memcpy(self.ctx, out.ctypes.data, self.ptr + offset, n, 1))
        return out

    def free(self):
        if self.ptr:
            library().rsm_dev_free(self.ctx, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def _bufs(shares: Sequence[Optional[bytes]]):
    """Keeps the bytes objects alive; returns (keepalive, void* array, u32 lens)."""
    n = len(shares)
    ptrs = (ctypes.c_void_p * max(n, 1))()
    lens = (ctypes.c_uint32 * max(n, 1))()
    keep = []
    for i, s in enumerate(shares):
        if s is None:
            ptrs[i] = None
            lens[i] = 0
        else:
            b = ctypes.create_string_buffer(bytes(s), len(s))
            keep.append(b)
            ptrs[i] = ctypes.cast(b, ctypes.c_void_p)
            lens[i] = len(s)
    return keep, ptrs, lens


# ---------------------------------------------------------------------------
# Codec (codecs.go:14-30) and LeoRSCodec (leopard.go)
# ---------------------------------------------------------------------------
class Codec:
    def Encode(self, data):  # pragma: no cover - interface
        raise NotImplementedError

    def Decode(self, data):  # pragma: no cover - interface
        raise NotImplementedError

    def MaxChunks(self) -> int:  # pragma: no cover - interface
        raise NotImplementedError

    def Name(self) -> str:  # pragma: no cover - interface
        raise NotImplementedError

    def ValidateChunkSize(self, chunkSize: int):  # pragma: no cover - interface
        raise NotImplementedError


class LeoRSCodec(Codec):
    """HIP-backed drop-in for rsmt2d.LeoRSCodec (leopard.go:16-103)."""

    def __init__(self, device: int = 0):
        self.device = device

    def Encode(self, data: Sequence[bytes]) -> List[bytes]:
        k = len(data)
        if k == 0:
            raise RSMError(RSM_EINVAL, "no shares")
        S = len(data[0])
        if any(d is None or len(d) != S for d in data):
            raise RSMError(RSM_ESHAPE, "shard sizes do not match")
        keep, ptrs, _ = _bufs(data)
        outs = [ctypes.create_string_buffer(S) for _ in range(k)]
        optr = (ctypes.c_void_p * k)(*[ctypes.cast(o, ctypes.c_void_p) for o in outs])
        _check(library().rsm_encode(device_context(self.device), ptrs, k, S, optr))
        return [o.raw for o in outs]

    def Decode(self, data: List[Optional[bytes]]) -> List[Optional[bytes]]:
        """Fills the None entries of ``data`` in place (as klauspost Reconstruct does)
        and returns the same list; raises RSMError(RSM_ETOOFEW) if < half present."""
        n = len(data)
        S = next((len(d) for d in data if d is not None), 0)
        present = (ctypes.c_uint8 * n)(*[0 if d is None else 1 for d in data])
        bufs = [ctypes.create_string_buffer(bytes(d) if d is not None else S, S) for d in data]
        ptrs = (ctypes.c_void_p * n)(*[ctypes.cast(b, ctypes.c_void_p) for b in bufs])
        _check(library().rsm_decode(device_context(self.device), ptrs, present, n, S))
        for i in range(n):
            if data[i] is None:
                data[i] = bufs[i].raw
        return data

    def MaxChunks(self) -> int:
        return int(library().rsm_codec_max_chunks())

    def Name(self) -> str:
        return library().rsm_codec_name().decode()

    def ValidateChunkSize(self, chunkSize: int):
        rc = library().rsm_codec_validate_chunk_size(int(chunkSize))
        if rc != RSM_OK:
            return _err(rc)
        return None


def NewLeoRSCodec(device: int = 0) -> LeoRSCodec:
    return LeoRSCodec(device)


# codecs registry (codecs.go:32-40), used by JSON unmarshalling
codecs = {Leopard: NewLeoRSCodec()}


# ---------------------------------------------------------------------------
# Tree plugin (tree.go)
# ---------------------------------------------------------------------------
class Tree:
    """Tree interface: Push(data) / Root() -> bytes."""

    def Push(self, data: bytes):  # pragma: no cover - interface
        raise NotImplementedError

    def Root(self) -> bytes:  # pragma: no cover - interface
        raise NotImplementedError


def NewDefaultTree(axis: int = Row, index: int = 0):
    """Marker for the built-in DefaultTree (SHA-256 merkletree, tree.go:38)."""
    return None


class _NmtTree(Tree):
    """Host Tree of the erasured NMT (Push validates and collects, Root hashes via
    rsm_nmt_tree_root).  Push reports the wrapper's errors where the reference does
    (nmtwrapper_test.go:103-108: share or axis index past 2*squareSize, data shorter
    than the namespace) and the NMT's namespace push-order error (celestiaorg/nmt
    v0.24.3 Push: namespaces must not decrease; the parity namespace 0xFF.. is the
    largest)."""

    def __init__(self, params: "NmtParams", axis: int, index: int):
        self._p, self._axis, self._index, self._leaves = params, axis, index, []
        self._last_ns = None

    def Push(self, data: bytes):
        ns, n = self._p.namespace_size, int(self._p.square_size)
        share = len(self._leaves)
        if self._index + 1 > 2 * n or share + 1 > 2 * n:
            raise RSMError(RSM_EINVAL, f"pushed past predetermined square size: boundary at {2 * n} index at "
                                       f"{self._index} {share}")
        data = bytes(data)
        if len(data) < ns:
            raise RSMError(RSM_EINVAL, "data is too short to contain namespace ID")
        nid = data[:ns] if (share < n and self._index < n) else b"\xff" * ns
        if self._last_ns is not None and nid < self._last_ns:
            raise RSMError(RSM_EINVAL, "pushed data has to be lexicographically ordered by namespace IDs")
        self._last_ns = nid
        self._leaves.append(data)

    def Root(self) -> bytes:
        keep, ptrs, _ = _bufs(self._leaves) if self._leaves else ([], None, None)
        cap = 2 * self._p.namespace_size + 32
        out = (ctypes.c_uint8 * cap)()
        ln = ctypes.c_uint32(cap)
        size = len(self._leaves[0]) if self._leaves else 0
        if any(len(x) != size for x in self._leaves):
            raise ValueError("NMT leaves of unequal size")
        rc = library().rsm_nmt_tree_root(ctypes.byref(self._p), self._axis, self._index, ptrs, len(self._leaves),
                                         size, out, ctypes.byref(ln))
        if rc:
            raise _err(rc)
        return bytes(out[:ln.value])


class ErasuredNamespacedMerkleTreeConstructor:
    """TreeConstructorFn of rsmt2d's erasured namespaced Merkle tree
    (nmtwrapper_test.go:75-92: celestiaorg/nmt with the parity namespace 0xFF.. for
    every cell outside quadrant 0, IgnoreMaxNamespace).  Recognised by the EDS
    layer, which computes these roots on the GPU (kernels_nmt.hip) for complete
    squares; calling it returns a host Tree like the reference's NewTree."""

    def __init__(self, squareSize: int, namespaceSize: int = 29, ignoreMaxNamespace: bool = True):
        if squareSize == 0:
            raise ValueError("cannot create a erasuredNamespacedMerkleTree of squareSize == 0")
        self.params = NmtParams(namespaceSize, 1 if ignoreMaxNamespace else 0, squareSize)

    def __call__(self, axis: int = Row, index: int = 0) -> Tree:
        return _NmtTree(self.params, axis, index)


def newErasuredNamespacedMerkleTreeConstructor(squareSize: int, namespaceSize: int = 29,
                                               ignoreMaxNamespace: bool = True):
    return ErasuredNamespacedMerkleTreeConstructor(squareSize, namespaceSize, ignoreMaxNamespace)


class BufferedTreeConstructor:
    """tree.go:13-16: NewConstructor(squareSize) -> TreeConstructorFn; TreeCount()."""

    def NewConstructor(self, squareSize: int):  # pragma: no cover - interface
        raise NotImplementedError

    def TreeCount(self) -> int:  # pragma: no cover - interface
        raise NotImplementedError


class TreePool(BufferedTreeConstructor):
    """The pooled NMT of nmtbuffered_tree_test.go:10-58 (newTreePool): a fixed number
    of trees reused across squares of any size.  Its trees push exactly as the
    erasured wrapper does, so here the pool hands out the device-computed NMT
    constructor; TreeCount bounds the host-side root parallelism as setParallelOps
    does (extendeddatasquare.go:90)."""

    def __init__(self, initSquareSize: int, poolSize: int, namespaceSize: int = 29, ignoreMaxNamespace: bool = True):
        if initSquareSize == 0:
            raise ValueError("cannot create a resizeableBufferTree of maxSquareSize == 0")
        self.poolSize, self.namespaceSize, self.ignoreMaxNamespace = poolSize, namespaceSize, ignoreMaxNamespace

    def NewConstructor(self, squareSize: int):
        return ErasuredNamespacedMerkleTreeConstructor(squareSize, self.namespaceSize, self.ignoreMaxNamespace)

    def TreeCount(self) -> int:
        return self.poolSize


def newTreePool(initSquareSize: int, poolSize: int, namespaceSize: int = 29, ignoreMaxNamespace: bool = True):
    return TreePool(initSquareSize, poolSize, namespaceSize, ignoreMaxNamespace)


def _tree_callback(tree_fn):
    """(keep-alive, tree_fn pointer, user pointer) for the C ABI: NULL for
    NewDefaultTree, the library's rsm_nmt_tree_root for the NMT constructor (so the
    GPU computes it), a ctypes callback for any other Python TreeConstructorFn."""
    if tree_fn is None or tree_fn is NewDefaultTree:
        return None, None, None
    if isinstance(tree_fn, ErasuredNamespacedMerkleTreeConstructor):
        fn = ctypes.cast(library().rsm_nmt_tree_root, ctypes.c_void_p)
        return tree_fn.params, fn, ctypes.cast(ctypes.byref(tree_fn.params), ctypes.c_void_p)

    def cb(user, axis, index, leaves, n, leaf_size, root_out, root_len):
        try:
            t = tree_fn(axis, index)
            for i in range(n):
                t.Push(ctypes.string_at(leaves[i], leaf_size))
            r = t.Root()
            if len(r) > root_len[0]:
                return RSM_EINVAL
            ctypes.memmove(root_out, r, len(r))
            root_len[0] = len(r)
            return 0
        except Exception:  # tree errors are byzantine evidence, as in the reference
            return RSM_ETREE

    c = _TREE_FN(cb)
    return c, ctypes.cast(c, ctypes.c_void_p), None


def _default_root(leaves: Sequence[bytes]) -> bytes:
    keep, ptrs, _ = _bufs(leaves)
    out = (ctypes.c_uint8 * 64)()
    ln = ctypes.c_uint32(64)
    _check(library().rsm_default_tree_root(None, 0, 0, ptrs, len(leaves),
                                           len(leaves[0]) if leaves else 0, out, ctypes.byref(ln)))
    return bytes(out[:ln.value])


# ---------------------------------------------------------------------------
# ExtendedDataSquare (extendeddatasquare.go)
# ---------------------------------------------------------------------------
class ExtendedDataSquare:
    def __init__(self, handle: int, codec: Codec, tree_fn, device: int = 0):
        self._h = ctypes.c_void_p(handle)
        self.codec = codec
        self._tree_fn = tree_fn
        self._device = device

    def __del__(self):
        try:
            if self._h:
                library().rsm_eds_free(self._h)
                self._h = None
        except Exception:
            pass

    # --- geometry ---
    def Width(self) -> int:
        return int(library().rsm_eds_width(self._h))

    @property
    def width(self) -> int:
        return self.Width()

    @property
    def originalDataWidth(self) -> int:
        return int(library().rsm_eds_original_width(self._h))

    @property
    def shareSize(self) -> int:
        return int(library().rsm_eds_share_size(self._h))

    # --- cells ---
    def GetCell(self, rowIdx: int, colIdx: int) -> Optional[bytes]:
        buf = ctypes.create_string_buffer(max(self.shareSize, 1))
        rc = library().rsm_eds_get_cell(self._h, rowIdx, colIdx, buf)
        if rc < 0:
            raise _err(rc)
        return buf.raw[: self.shareSize] if rc == 1 else None

    def SetCell(self, rowIdx: int, colIdx: int, newShare: bytes):
        _check(library().rsm_eds_set_cell(self._h, rowIdx, colIdx, newShare, len(newShare)))

    def setCell(self, rowIdx: int, colIdx: int, newShare: Optional[bytes]):
        """Test hook mirroring the reference's unexported setCell (datasquare_test.go:735)."""
        if newShare is None:
            _check(library().rsm_eds_overwrite_cell(self._h, rowIdx, colIdx, None, 0))
        else:
            _check(library().rsm_eds_overwrite_cell(self._h, rowIdx, colIdx, newShare, len(newShare)))

    def Flattened(self) -> List[Optional[bytes]]:
        w, S = self.Width(), self.shareSize
        out = ctypes.create_string_buffer(max(w * w * S, 1))
        pres = ctypes.create_string_buffer(max(w * w, 1))
        _check(library().rsm_eds_flattened(self._h, out, pres))
        raw, p = out.raw, pres.raw
        return [raw[i * S:(i + 1) * S] if p[i] else None for i in range(w * w)]

    def FlattenedODS(self) -> List[Optional[bytes]]:
        f, w, o = self.Flattened(), self.Width(), self.originalDataWidth
        return [f[r * w + c] for r in range(o) for c in range(o)]

    def Row(self, rowIdx: int) -> List[Optional[bytes]]:
        w = self.Width()
        return [self.GetCell(rowIdx, c) for c in range(w)]

    def Col(self, colIdx: int) -> List[Optional[bytes]]:
        w = self.Width()
        return [self.GetCell(r, colIdx) for r in range(w)]

    # --- roots ---
    def _roots(self, axis: int) -> List[bytes]:
        w = self.Width()
        cap = 256
        out = ctypes.create_string_buffer(max(w * cap, 1))
        ln = ctypes.c_uint32(0)
        keep, fn, user = _tree_callback(self._tree_fn)
        _check(library().rsm_eds_roots(self._h, axis, fn, user, out, cap, ctypes.byref(ln)))
        raw = out.raw
        return [raw[i * cap: i * cap + ln.value] for i in range(w)]

    def RowRoots(self) -> List[bytes]:
        return self._roots(Row)

    def ColRoots(self) -> List[bytes]:
        return self._roots(Col)

    def Roots(self) -> List[bytes]:
        return self.RowRoots() + self.ColRoots()

    # --- Repair (extendeddatacrossword.go:74-84) ---
    def Repair(self, rowRoots: Sequence[bytes], colRoots: Sequence[bytes]) -> None:
        L = library()
        _check(L.rsm_eds_set_context(self._h, device_context(self._device)))
        root_len = len(rowRoots[0]) if rowRoots else 0
        rr = b"".join(bytes(r) for r in rowRoots)
        cr = b"".join(bytes(c) for c in colRoots)
        byz = _Byz()
        keep, fn, user = _tree_callback(self._tree_fn)
        rc = L.rsm_eds_repair(self._h, rr, cr, root_len, fn, user, ctypes.byref(byz))
        if rc == RSM_OK:
            return
        if rc == RSM_EUNREPAIRABLE:
            raise ErrUnrepairableDataSquare
        if rc == RSM_EBYZANTINE:
            w, S = self.Width(), self.shareSize
            out = ctypes.create_string_buffer(max(w * S, 1))
            pres = ctypes.create_string_buffer(max(w, 1))
            _check(L.rsm_eds_byzantine_shares(self._h, out, pres))
            raw, p = out.raw, pres.raw
            raise ErrByzantineData(byz.axis, byz.index, [raw[i * S:(i + 1) * S] if p[i] else None for i in range(w)])
        raise _err(rc)

    def repair_stats(self) -> RepairStats:
        st = RepairStats()
        _check(library().rsm_eds_repair_stats(self._h, ctypes.byref(st)))
        return st

    # --- equality / JSON ---
    def Equals(self, other: "ExtendedDataSquare") -> bool:
        if self.originalDataWidth != other.originalDataWidth:
            return False
        if self.codec.Name() != other.codec.Name():
            return False
        if self.shareSize != other.shareSize or self.Width() != other.Width():
            return False
        return self.Flattened() == other.Flattened()

    def MarshalJSON(self) -> bytes:
        shares = [None if s is None else base64.b64encode(s).decode() for s in self.Flattened()]
        return json.dumps({"data_square": shares, "codec": self.codec.Name()}).encode()

    @staticmethod
    def UnmarshalJSON(b: bytes) -> "ExtendedDataSquare":
        aux = json.loads(b)
        shares = [None if s is None else base64.b64decode(s) for s in aux["data_square"]]
        return ImportExtendedDataSquare(shares, codecs[aux["codec"]], NewDefaultTree)

    def deepCopy(self, codec: Codec) -> "ExtendedDataSquare":
        return ImportExtendedDataSquare(self.Flattened(), codec, self._tree_fn)


def _device_of(codec) -> int:
    return getattr(codec, "device", 0)


def ComputeExtendedDataSquare(data: Sequence[bytes], codec: Codec, treeCreatorFn=NewDefaultTree):
    """extendeddatasquare.go:50-77 on the GPU."""
    keep, ptrs, lens = _bufs(data)
    h = ctypes.c_void_p()
    _check(library().rsm_eds_compute(device_context(_device_of(codec)), ptrs, lens, len(data), ctypes.byref(h)))
    return ExtendedDataSquare(h.value, codec, treeCreatorFn, _device_of(codec))


def ComputeExtendedDataSquareWithBuffer(data: Sequence[bytes], codec: Codec, treeCreator: BufferedTreeConstructor):
    """extendeddatasquare.go:81-92: ComputeExtendedDataSquare with the buffered
    constructor's trees, root parallelism limited to treeCreator.TreeCount()."""
    width = math.isqrt(len(data))
    if width * width < len(data):
        width += 1  # getWidth rounds up (datasquare.go:35-37); the shape check rejects it
    eds = ComputeExtendedDataSquare(data, codec, treeCreator.NewConstructor(width))
    eds.parallelOps = treeCreator.TreeCount()  # setParallelOps
    return eds


def ImportExtendedDataSquare(data: Sequence[Optional[bytes]], codec: Codec, treeCreatorFn=NewDefaultTree):
    """extendeddatasquare.go:95-124 (host-only; no GPU needed until Repair)."""
    keep, ptrs, lens = _bufs(data)
    h = ctypes.c_void_p()
    _check(library().rsm_eds_import(None, ptrs, lens, len(data), ctypes.byref(h)))
    return ExtendedDataSquare(h.value, codec, treeCreatorFn, _device_of(codec))


def NewExtendedDataSquare(codec: Codec, treeCreatorFn, edsWidth: int, shareSize: int):
    """extendeddatasquare.go:129-152 (host-only)."""
    h = ctypes.c_void_p()
    _check(library().rsm_eds_new(None, edsWidth, shareSize, ctypes.byref(h)))
    return ExtendedDataSquare(h.value, codec, treeCreatorFn, _device_of(codec))
