"""Row-sharded 2D extension of one large square across the GPUs of a node.

BASELINE config 5 / SURVEY.md §8(e): one process per GPU, ``torch.distributed``
(backend "nccl" = RCCL over xGMI).  Rank g of G owns ODS rows [g*k/G, (g+1)*k/G):

  1. row pass: encode its rows -> its row block of the top half [Q0 | Q1]
     (erasureExtendRow, extendeddatasquare.go:229-235);
  2. all-gather of the top-half row blocks (the north_star's exchange step), so
     every rank holds all of [Q0 | Q1];
  3. column pass over its 2k/G columns -> its column slice of the bottom half
     [Q2 | Q3] (Q2 as erasureExtendCol; Q3 = column-encoding of Q1, equal to the
     reference's row-encoding of Q2 by linearity, extendeddatasquare.go:204-207).

Afterwards the top half is replicated and the bottom half is column-sharded.  The
encode steps are pluggable so the exchange logic runs under ``gloo`` on CPU in the
tests; the product binding (`hip_backend`) launches the HIP kernels through the C
ABI on the rank's device, with host-side ordering between this library's HIP
stream and the collective (the collective runs on PyTorch's stream).
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist


def shard(n: int, parts: int, idx: int) -> Tuple[int, int]:
    """Contiguous [start, end) slice of range(n) owned by part idx (n % parts == 0)."""
    if n % parts != 0:
        raise ValueError(f"{n} rows/columns do not split evenly over {parts} ranks")
    step = n // parts
    return idx * step, (idx + 1) * step


class RowShardedExtender:
    """Extends one [2k][2k][S] square (uint8 tensor, Q0 rows of this rank filled) in place."""

    def __init__(self, k: int, share_size: int, encode_rows: Callable, encode_cols: Callable,
                 after_local: Optional[Callable] = None, before_local: Optional[Callable] = None, *,
                 group: Optional[dist.ProcessGroup] = None):
        self.k, self.S = k, share_size
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.rows = shard(k, self.world, self.rank)
        self.cols = shard(2 * k, self.world, self.rank)
        self._enc_rows, self._enc_cols = encode_rows, encode_cols
        self._after_local = after_local or (lambda: None)    # drain the encoder's stream
        self._before_local = before_local or (lambda: None)  # drain the collective's stream

    def extend(self, eds: torch.Tensor) -> None:
        k = self.k
        r0, r1 = self.rows
        c0, c1 = self.cols
        assert eds.shape == (2 * k, 2 * k, self.S) and eds.dtype == torch.uint8 and eds.is_contiguous()
        self._enc_rows(eds, r0, r1 - r0)
        self._after_local()
        top = eds[:k].view(-1)
        mine = eds[r0:r1].reshape(-1)
        if eds.is_cuda:
            dist.all_gather_into_tensor(top, mine, group=self.group)   # in place (RCCL)
        else:
            dist.all_gather_into_tensor(top, mine.clone(), group=self.group)
        self._before_local()
        self._enc_cols(eds, c0, c1 - c0)
        self._after_local()


class TransposeShardedExtender:
    """SURVEY.md §8(e) Option B: the all-gather of the top half replaced by an
    all-to-all transpose, so each rank receives only its own column slice.

    Rank g of G (n = k/G rows, w = 2k/G columns):
      rows   [n][2k][S]  its ODS rows (Q0 part filled); the row pass writes Q1 in place
      top    [k][w][S]   receives columns [g*w, (g+1)*w) of the whole top half [Q0|Q1]
      bottom [k][w][S]   the column pass writes the same columns of [Q2|Q3]
    Bytes received per rank: (G-1)/G * k*w*S  (config 5, G = 8: 28 MiB) instead of the
    all-gather's (G-1)/G * k*2k*S (224 MiB).  The send buffer holds, for every
    destination d, this rank's rows restricted to d's columns: written by the row pass
    itself when `encode_rows` carries `writes_blocks = True` (it is then called as
    encode_rows(rows, send); the HIP backend's rsm_extend_rows_blocks_dev), else packed
    by one strided copy after it.  The received blocks are `top` in row order already,
    so the column pass reads them in place: no unpack either."""

    def __init__(self, k: int, share_size: int, encode_rows: Callable, encode_batch: Callable,
                 after_local: Optional[Callable] = None, before_local: Optional[Callable] = None, *,
                 group: Optional[dist.ProcessGroup] = None):
        self.k, self.S = k, share_size
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.rows = shard(k, self.world, self.rank)
        self.cols = shard(2 * k, self.world, self.rank)
        self._enc_rows, self._enc_batch = encode_rows, encode_batch
        self._after_local = after_local or (lambda: None)
        self._before_local = before_local or (lambda: None)
        self._send = None

    def extend(self, rows: torch.Tensor, top: torch.Tensor, bottom: torch.Tensor) -> None:
        k, S, G = self.k, self.S, self.world
        n, w = k // G, 2 * k // G
        assert rows.shape == (n, 2 * k, S) and top.shape == (k, w, S) and bottom.shape == (k, w, S)
        assert rows.is_contiguous() and top.is_contiguous() and bottom.is_contiguous()
        if getattr(self._enc_rows, "writes_blocks", False):
            send = self._send
            if send is None or send.shape != (G, n, w, S) or send.device != rows.device:
                send = self._send = torch.empty((G, n, w, S), dtype=torch.uint8, device=rows.device)
            self._enc_rows(rows, send)                           # Q0 -> Q1 rows, and their blocks
            self._after_local()
        else:
            self._enc_rows(rows)                                 # Q0 rows -> Q1 rows (in place)
            self._after_local()
            send = rows.view(n, G, w, S).transpose(0, 1).contiguous()  # [G][n][w][S]: block d -> rank d
        dist.all_to_all_single(top.view(-1), send.view(-1), group=self.group)
        self._before_local()
        self._enc_batch(top, bottom)                             # my w columns: [Q0|Q1] -> [Q2|Q3]
        self._after_local()


def hip_backend(device: int = 0):
    """(encode_rows, encode_cols, after_local, before_local) bound to the HIP C ABI."""
    from . import _check, device_context, library

    L = library()
    ctx = device_context(device)

    def rows(eds, r0, n):
        k = eds.shape[1] // 2
        _check(L.rsm_extend_rows_dev(ctx, eds.data_ptr(), k, eds.shape[2], r0, n, None))

    def cols(eds, c0, n):
        k = eds.shape[1] // 2
        _check(L.rsm_extend_cols_dev(ctx, eds.data_ptr(), k, eds.shape[2], c0, n, None))

    def after():
        _check(L.rsm_sync(ctx))

    def before():
        torch.cuda.current_stream().synchronize()

    return rows, cols, after, before


def hip_transpose_backend(device: int = 0):
    """(encode_rows, encode_batch, after_local, before_local) for TransposeShardedExtender."""
    from . import _check, device_context, library

    L = library()
    ctx = device_context(device)

    def rows(r, send):
        n, W, S = r.shape
        assert send.is_contiguous() and send.numel() == r.numel()
        _check(L.rsm_extend_rows_blocks_dev(ctx, r.data_ptr(), W // 2, S, 0, n, send.data_ptr(), send.shape[0], None))

    rows.writes_blocks = True

    def batch(top, bottom):
        k, w, S = top.shape
        _check(L.rsm_encode_batch_dev(ctx, top.data_ptr(), bottom.data_ptr(), k, S, w, S, w * S, None))

    def after():
        _check(L.rsm_sync(ctx))

    def before():
        torch.cuda.current_stream().synchronize()

    return rows, batch, after, before
