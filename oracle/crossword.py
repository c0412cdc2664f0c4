"""Python restatement of rsmt2d's Repair -- TEST INFRASTRUCTURE ONLY.

Follows extendeddatacrossword.go line by line (file:line cited per function) over
the C oracle codec (oracle.encode / oracle.decode) and a hashlib restatement of
DefaultTree (tree.go:32-59: celestiaorg/merkletree over SHA-256, leaf
H(0x00||d), node H(0x01||l||r)).  Small squares only (pure Python control flow).
preRepairSanityCheck runs its checks in index order (row i root, row i
encoding, col i root, col i encoding); the reference runs them concurrently and
returns whichever failure its errgroup observes first.
"""
from __future__ import annotations

import hashlib
from typing import List, Optional

from . import TooFewShards, decode, encode

Row, Col = 0, 1


class Unrepairable(Exception):
    pass


class Byzantine(Exception):
    def __init__(self, axis, index, shares):
        super().__init__(f"byzantine {'row' if axis == Row else 'col'}: {index}")
        self.axis, self.index, self.shares = axis, index, shares


def merkle_root(leaves: List[bytes]) -> bytes:
    """DefaultTree.Root (tree.go:51-59) restated."""
    stack = []  # (height, digest)
    for leaf in leaves:
        cur = (0, hashlib.sha256(b"\x00" + leaf).digest())
        while stack and stack[-1][0] == cur[0]:
            h, d = stack.pop()
            cur = (h + 1, hashlib.sha256(b"\x01" + d + cur[1]).digest())
        stack.append(cur)
    if not stack:
        return b""
    acc = stack[-1][1]
    for h, d in reversed(stack[:-1]):
        acc = hashlib.sha256(b"\x01" + d + acc).digest()
    return acc


class Square:
    """datasquare.go grid: width x width cells of bytes or None."""

    def __init__(self, flat: List[Optional[bytes]]):
        n = len(flat)
        w = int(round(n ** 0.5))
        assert w * w == n
        self.w = w
        self.cells = [list(flat[r * w:(r + 1) * w]) for r in range(w)]

    def row(self, i):
        return list(self.cells[i])

    def col(self, i):
        return [self.cells[r][i] for r in range(self.w)]

    def vec(self, axis, i):
        return self.row(i) if axis == Row else self.col(i)

    def set(self, r, c, v):
        self.cells[r][c] = v

    def flattened(self):
        return [x for row in self.cells for x in row]

    def roots(self, axis):
        return [merkle_root(self.vec(axis, i)) for i in range(self.w)]


def no_missing(v, skip=-1):  # noMissingData (:431-441)
    return all(x is not None for j, x in enumerate(v) if j != skip)


def verify_encoding(v, idx=-1, share=None):  # verifyEncoding (:480-502)
    v = list(v)
    if share is not None and idx >= 0:
        v[idx] = share
    half = len(v) // 2
    if any(x is None for x in v[:half]):
        return False
    parity = encode(v[:half])
    return all(v[half + i] == parity[i] for i in range(half))


def pre_repair_sanity_check(sq: Square, row_roots, col_roots):  # (:366-429)
    for i in range(sq.w):
        for axis, roots in ((Row, row_roots), (Col, col_roots)):
            v = sq.vec(axis, i)
            if no_missing(v):
                if merkle_root(v) != roots[i] or not verify_encoding(v):
                    raise Byzantine(axis, i, v)


def solve_vector(sq: Square, axis, idx, my_roots, orth_roots):  # solveCrosswordRow/Col (:129-282)
    v = sq.vec(axis, idx)
    if no_missing(v):
        return True, False
    try:
        rebuilt = decode(list(v))
    except TooFewShards:
        return False, False
    if merkle_root(rebuilt) != my_roots[idx]:
        raise Byzantine(axis, idx, v)
    oaxis = Col if axis == Row else Row
    for o in range(sq.w):
        ov = sq.vec(oaxis, o)
        if ov[idx] is not None:
            continue
        if no_missing(ov, idx):
            leaves = list(ov)
            leaves[idx] = rebuilt[o]
            if merkle_root(leaves) != orth_roots[o]:
                raise Byzantine(oaxis, o, ov)
            if not verify_encoding(ov, idx, rebuilt[o]):
                raise Byzantine(oaxis, o, ov)
    for p in range(sq.w):
        r, c = (idx, p) if axis == Row else (p, idx)
        if sq.cells[r][c] is None:
            sq.set(r, c, rebuilt[p])
    return True, True


def repair(flat: List[Optional[bytes]], row_roots, col_roots) -> List[Optional[bytes]]:
    """Repair (:74-84): returns the repaired flattened square or raises
    Unrepairable / Byzantine (the square is modified as in the reference)."""
    sq = Square(flat)
    pre_repair_sanity_check(sq, row_roots, col_roots)
    while True:
        solved, progress = True, False
        for i in range(sq.w):
            s1, p1 = solve_vector(sq, Row, i, row_roots, col_roots)
            s2, p2 = solve_vector(sq, Col, i, col_roots, row_roots)
            solved = solved and s1 and s2
            progress = progress or p1 or p2
        if solved:
            return sq.flattened()
        if not progress:
            raise Unrepairable()
