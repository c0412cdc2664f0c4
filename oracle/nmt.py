"""TEST INFRASTRUCTURE ONLY -- pure-Python (hashlib) restatement of the namespaced
Merkle tree rsmt2d's NMT wrappers build, the checker for rsm_nmt_tree_root
(rsmt2d_amd/csrc/merkle.cpp) and the device kernels (kernels_nmt.hip).

The tree itself is celestiaorg/nmt v0.24.3 (/root/reference/go.mod:7), a
dependency that is NOT in /root/reference, so this restates its published
algorithm:
  HashLeaf(ndata)  = ns || ns || SHA256(0x00 || ndata),   ns = ndata[:nsSize]
  HashNode(l, r)   = l.min || max || SHA256(0x01 || l || r)
                     max = l.max if IgnoreMaxNamespace and r.min == 0xFF.. else r.max
                     (error if r.min < l.max: ErrUnorderedSiblings)
  Push(ndata)      : error if ns < previous ns (ErrInvalidPushOrder)
  Root()           : RFC 6962 split at the largest power of two below n;
                     empty tree = zero ns || zero ns || SHA256("")
and the wrapper rule (nmtwrapper_test.go:94-120, nmtbuffered_tree_test.go:118-152):
leaf i of row/column `index` is pushed as ns || share with ns = share[:nsSize] in
quadrant 0 (i < k and index < k), else the parity namespace 0xFF...
Parity vs the nmt library itself is UNPINNED (no nmt golden vectors exist in the
reference); the restatement is cross-checked against the C++ and device forms."""
import hashlib


class NmtError(Exception):
    pass


def hash_leaf(ndata: bytes, ns_size: int) -> bytes:
    if len(ndata) < ns_size:
        raise NmtError("data too short for namespace")
    ns = ndata[:ns_size]
    return ns + ns + hashlib.sha256(b"\x00" + ndata).digest()


def hash_node(left: bytes, right: bytes, ns_size: int, ignore_max: bool = True) -> bytes:
    lmin, lmax = left[:ns_size], left[ns_size:2 * ns_size]
    rmin, rmax = right[:ns_size], right[ns_size:2 * ns_size]
    if rmin < lmax:
        raise NmtError("unordered siblings")
    mx = lmax if (ignore_max and rmin == b"\xff" * ns_size) else rmax
    return lmin + mx + hashlib.sha256(b"\x01" + left + right).digest()


def _root(nodes, ns_size, ignore_max):
    n = len(nodes)
    if n == 1:
        return nodes[0]
    k = 1
    while k * 2 < n:
        k *= 2
    return hash_node(_root(nodes[:k], ns_size, ignore_max), _root(nodes[k:], ns_size, ignore_max), ns_size,
                     ignore_max)


def nmt_root(ndatas, ns_size: int, ignore_max: bool = True) -> bytes:
    """Push every namespaced datum in order, then Root()."""
    prev = None
    leaves = []
    for d in ndatas:
        if len(d) < ns_size:
            raise NmtError("data too short for namespace")
        ns = d[:ns_size]
        if prev is not None and ns < prev:
            raise NmtError("invalid push order")
        prev = ns
        leaves.append(hash_leaf(d, ns_size))
    if not leaves:
        return b"\x00" * (2 * ns_size) + hashlib.sha256(b"").digest()
    return _root(leaves, ns_size, ignore_max)


def erasured_root(shares, axis_index: int, square_size: int, ns_size: int = 29, ignore_max: bool = True) -> bytes:
    """Root of one row/column as erasuredNamespacedMerkleTree computes it."""
    if axis_index + 1 > 2 * square_size or len(shares) > 2 * square_size:
        raise NmtError("pushed past predetermined square size")
    out = []
    for i, sh in enumerate(shares):
        if len(sh) < ns_size:
            raise NmtError("data is too short to contain namespace ID")
        q0 = i < square_size and axis_index < square_size
        ns = bytes(sh[:ns_size]) if q0 else b"\xff" * ns_size
        out.append(ns + bytes(sh))
    return nmt_root(out, ns_size, ignore_max)


def eds_roots(eds, square_size: int, ns_size: int = 29):
    """(row roots, column roots) of a complete [W][W][S] numpy square."""
    W = eds.shape[0]
    rows = [erasured_root([eds[r, c].tobytes() for c in range(W)], r, square_size, ns_size) for r in range(W)]
    cols = [erasured_root([eds[r, c].tobytes() for r in range(W)], c, square_size, ns_size) for c in range(W)]
    return rows, cols
