"""CPU (gloo, world_size 2 and 4): the row-sharded multi-GPU schedule of config 5
(rsmt2d_amd.distributed) assembles exactly the reference extension.  The per-rank
encode steps are the oracle here (test injection); on GPUs they are the HIP kernels."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_rows(eds, r0, n):
    import oracle
    k = eds.shape[1] // 2
    a = eds.numpy()
    for r in range(r0, r0 + n):
        par = oracle.encode([a[r, c].tobytes() for c in range(k)])
        for i, p in enumerate(par):
            a[r, k + i] = np.frombuffer(p, np.uint8)


def _oracle_cols(eds, c0, n):
    import oracle
    k = eds.shape[1] // 2
    a = eds.numpy()
    for c in range(c0, c0 + n):
        par = oracle.encode([a[r, c].tobytes() for r in range(k)])
        for i, p in enumerate(par):
            a[k + i, c] = np.frombuffer(p, np.uint8)


def _worker(rank, world, port, k, S, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from rsmt2d_amd.distributed import RowShardedExtender
        rng = np.random.default_rng(7)
        ods = rng.integers(0, 256, (k, k, S), dtype=np.uint8)  # same on every rank
        eds = torch.zeros((2 * k, 2 * k, S), dtype=torch.uint8)
        ext = RowShardedExtender(k, S, _oracle_rows, _oracle_cols)
        r0, r1 = ext.rows
        eds[r0:r1, :k] = torch.from_numpy(ods[r0:r1])  # only this rank's ODS rows
        ext.extend(eds)
        c0, c1 = ext.cols
        pieces = [torch.zeros_like(eds[k:, c0:c1]) for _ in range(world)]
        dist.all_gather(pieces, eds[k:, c0:c1].contiguous())
        if rank == 0:
            import oracle
            want = oracle.extend_square(ods)
            got = eds.numpy().copy()
            w = 2 * k // world
            for g, p in enumerate(pieces):
                got[k:, g * w:(g + 1) * w] = p.numpy()
            q.put(bool((got == want).all()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - surfaced through the queue
        q.put(repr(e))


@pytest.mark.parametrize("world", [2, 4])
def test_row_sharded_matches_reference(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 8, 64, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
    assert res is True, res


def test_shard_math():
    from rsmt2d_amd.distributed import shard
    assert [shard(512, 8, g) for g in (0, 7)] == [(0, 64), (448, 512)]
    assert shard(1024, 8, 3) == (384, 512)
    with pytest.raises(ValueError):
        shard(10, 4, 0)


def _oracle_row_block(rows):
    import oracle
    n, W, S = rows.shape
    k = W // 2
    a = rows.numpy()
    for r in range(n):
        par = oracle.encode([a[r, c].tobytes() for c in range(k)])
        for i, p in enumerate(par):
            a[r, k + i] = np.frombuffer(p, np.uint8)


def _oracle_row_blocks(rows, send):
    """The writes_blocks contract (rsm_extend_rows_blocks_dev): the row pass, and the
    extended rows split into send[h] = rows restricted to column block h."""
    _oracle_row_block(rows)
    G = send.shape[0]
    n, W, S = rows.shape
    send.copy_(rows.view(n, G, W // G, S).transpose(0, 1))


_oracle_row_blocks.writes_blocks = True


def _oracle_batch(top, bottom):
    import oracle
    k, w, S = top.shape
    t, b = top.numpy(), bottom.numpy()
    for c in range(w):
        par = oracle.encode([t[r, c].tobytes() for r in range(k)])
        for i, p in enumerate(par):
            b[i, c] = np.frombuffer(p, np.uint8)


def _worker_transpose(rank, world, port, k, S, q, blocks=False):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from rsmt2d_amd.distributed import TransposeShardedExtender
        ods = np.random.default_rng(11).integers(0, 256, (k, k, S), dtype=np.uint8)
        ext = TransposeShardedExtender(k, S, _oracle_row_blocks if blocks else _oracle_row_block, _oracle_batch)
        r0, r1 = ext.rows
        c0, c1 = ext.cols
        rows = torch.zeros((r1 - r0, 2 * k, S), dtype=torch.uint8)
        rows[:, :k] = torch.from_numpy(ods[r0:r1])
        top = torch.zeros((k, c1 - c0, S), dtype=torch.uint8)
        bottom = torch.zeros_like(top)
        ext.extend(rows, top, bottom)
        import oracle
        want = oracle.extend_square(ods)
        ok = bool((top.numpy() == want[:k, c0:c1]).all() and (bottom.numpy() == want[k:, c0:c1]).all()
                  and (rows.numpy() == want[r0:r1]).all())
        flags = [None] * world
        dist.all_gather_object(flags, ok)
        if rank == 0:
            q.put(all(flags))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - surfaced through the queue
        q.put(repr(e))


@pytest.mark.parametrize("world,blocks", [(2, False), (4, False), (4, True)])
def test_transpose_sharded_matches_reference(world, blocks):
    """Option B (all-to-all of column slices): every rank ends with its exact column
    slice of the reference EDS (top and bottom) and its extended rows -- with the send
    blocks packed after the row pass, or written by it (writes_blocks)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_transpose, args=(r, world, port, 8, 64, q, blocks)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
    assert res is True, res
