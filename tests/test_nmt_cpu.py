"""CPU: the namespaced Merkle tree (celestiaorg/nmt v0.24.3 as rsmt2d's erasured
wrappers push it, nmtwrapper_test.go:94-120) -- the host restatement
rsm_nmt_tree_root (merkle.cpp) against the Python oracle (oracle/nmt.py), its
error behaviour, and the Python mirror's buffered-constructor plumbing.
Parity vs the nmt library itself is unpinned (not vendored; no golden vectors in
the reference) -- see oracle/nmt.py."""
import hashlib

import numpy as np
import pytest

import rsmt2d_amd as R
from oracle import nmt


def sorted_shares(rng, n, S, ns):
    sh = rng.integers(0, 256, (n, S), dtype=np.uint8)
    return [bytes(x) for x in sh[np.lexsort(sh[:, :ns][:, ::-1].T)]]


def host_root(leaves, k, idx, ns=29, axis=0):
    t = R.ErasuredNamespacedMerkleTreeConstructor(k, ns)(axis, idx)
    for x in leaves:
        t.Push(x)
    return t.Root()


@pytest.mark.parametrize("ns", [29, 8, 1, 32, 40])
@pytest.mark.parametrize("n,k,idx", [(6, 3, 0), (6, 3, 4), (70, 35, 3), (70, 35, 40), (5, 3, 1), (1, 1, 0),
                                     (256, 128, 7), (256, 128, 200), (2, 1, 0)])
def test_host_nmt_matches_oracle(ns, n, k, idx):
    rng = np.random.default_rng(ns * 1000 + n + idx)
    leaves = sorted_shares(rng, n, 64, ns)
    assert host_root(leaves, k, idx, ns) == nmt.erasured_root(leaves, idx, k, ns)


def test_root_layout_and_parity_namespace():
    """root = minNs || maxNs || digest; with IgnoreMaxNamespace a row of quadrant 0
    (data namespaces, then parity 0xFF..) reports the data namespaces' range."""
    rng = np.random.default_rng(3)
    k, ns = 4, 29
    leaves = sorted_shares(rng, 2 * k, 64, ns)
    r = host_root(leaves, k, 0, ns)
    assert len(r) == 2 * ns + 32
    assert r[:ns] == leaves[0][:ns] and r[ns:2 * ns] == leaves[k - 1][:ns]
    r2 = host_root(leaves, k, k, ns)  # a parity row: every leaf carries the parity namespace
    assert r2[:2 * ns] == b"\xff" * (2 * ns)


def test_leaf_and_node_hash_definitions():
    ns = 8
    d = bytes(range(8)) + b"payload"
    assert nmt.hash_leaf(d, ns) == d[:8] * 2 + hashlib.sha256(b"\x00" + d).digest()
    a, b = nmt.hash_leaf(b"\x01" * 8 + b"x", ns), nmt.hash_leaf(b"\x02" * 8 + b"y", ns)
    assert nmt.hash_node(a, b, ns) == b"\x01" * 8 + b"\x02" * 8 + hashlib.sha256(b"\x01" + a + b).digest()
    assert nmt.nmt_root([], ns) == b"\x00" * 16 + hashlib.sha256(b"").digest()


def test_push_order_and_size_errors():
    rng = np.random.default_rng(5)
    k, ns = 4, 29
    leaves = sorted_shares(rng, 2 * k, 64, ns)
    bad = [leaves[1], leaves[0]] + leaves[2:]
    if bad[0][:ns] != bad[1][:ns]:
        with pytest.raises(R.RSMError):
            host_root(bad, k, 0, ns)
        with pytest.raises(nmt.NmtError):
            nmt.erasured_root(bad, 0, k, ns)
    with pytest.raises(R.RSMError):  # pushed past the predetermined square size
        host_root(leaves, k, 2 * k, ns)
    with pytest.raises(R.RSMError):  # data too short to contain a namespace
        host_root([b"\x00" * 16] * 2, 1, 0, ns)


def test_buffered_constructor_interface():
    pool = R.newTreePool(32, 4)
    assert isinstance(pool, R.BufferedTreeConstructor)
    assert pool.TreeCount() == 4
    c = pool.NewConstructor(67)
    assert isinstance(c, R.ErasuredNamespacedMerkleTreeConstructor)
    assert c.params.square_size == 67 and c.params.namespace_size == 29 and c.params.ignore_max_namespace == 1
    with pytest.raises(ValueError):
        R.newErasuredNamespacedMerkleTreeConstructor(0)


def test_nmt_push_validates_like_the_wrapper():
    """The host tree reports the wrapper's Push errors at Push
    (nmtwrapper_test.go:103-108, nmtwrapper.go Push)."""
    t = R.newErasuredNamespacedMerkleTreeConstructor(2, 1)(R.Row, 0)
    t.Push(bytes([1]) * 8)
    with pytest.raises(R.RSMError, match="lexicographically"):
        t.Push(bytes([0]) * 8)  # namespace 0 after 1 (both in Q0)
    t = R.newErasuredNamespacedMerkleTreeConstructor(2, 29)(R.Row, 0)
    with pytest.raises(R.RSMError, match="too short"):
        t.Push(b"\1" * 28)
    t = R.newErasuredNamespacedMerkleTreeConstructor(2, 1)(R.Row, 4)
    with pytest.raises(R.RSMError, match="past predetermined"):
        t.Push(b"\1" * 8)
    t = R.newErasuredNamespacedMerkleTreeConstructor(1, 1)(R.Row, 0)
    t.Push(b"\1" * 8)
    t.Push(b"\1" * 8)  # parity namespace 0xFF >= 1
    with pytest.raises(R.RSMError, match="past predetermined"):
        t.Push(b"\1" * 8)
