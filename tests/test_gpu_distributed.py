"""GPU: the per-GPU units of the row-sharded schedule (config 5) and the
RowShardedExtender on RCCL (world_size 1 on the one-GPU test box; N>1 runs in the
driver's multi-GPU bench, the exchange logic is covered by test_distributed_cpu)."""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle
import rsmt2d_amd as R

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("k,S,parts", [(64, 512, 4), (128, 512, 4), (128, 1088, 2), (512, 512, 8)])
def test_row_and_column_slices(lib, k, S, parts):
    """Rows then columns in `parts` slices each == the full extension (what 8 ranks do)."""
    W = 2 * k
    ods = oracle.splitmix64_bytes(k * k * S, seed=99).reshape(k, k, S)
    buf = R.DeviceBuffer(W * W * S)
    full = np.zeros((W, W, S), np.uint8)
    full[:k, :k] = ods
    buf.upload(full)
    for g in range(parts):
        R._check(lib.rsm_extend_rows_dev(buf.ctx, buf.ptr, k, S, g * k // parts, k // parts, None))
    for g in range(parts):
        R._check(lib.rsm_extend_cols_dev(buf.ctx, buf.ptr, k, S, g * W // parts, W // parts, None))
    R._check(lib.rsm_sync(buf.ctx))
    got = buf.download().reshape(W, W, S)
    assert (got == oracle.extend_square(ods, nthreads=min(16, os.cpu_count() or 1))).all()


SCRIPT = r"""
import os, sys
sys.path.insert(0, {root!r})
import numpy as np, torch, torch.distributed as dist
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533", RANK="0", WORLD_SIZE="1")
torch.cuda.set_device(0)
dist.init_process_group("nccl")
from rsmt2d_amd.distributed import RowShardedExtender, hip_backend
import oracle
k, S = 64, 512
ods = np.random.default_rng(3).integers(0, 256, (k, k, S), dtype=np.uint8)
eds = torch.zeros((2 * k, 2 * k, S), dtype=torch.uint8, device="cuda")
eds[:k, :k] = torch.from_numpy(ods).cuda()
torch.cuda.synchronize()
ext = RowShardedExtender(k, S, *hip_backend(0))
ext.extend(eds)
ok = bool((eds.cpu().numpy() == oracle.extend_square(ods)).all())
dist.destroy_process_group()
print("SHARDED_OK" if ok else "SHARDED_MISMATCH")
"""


def test_row_sharded_extender_rccl_world1():
    pytest.importorskip("torch")
    r = subprocess.run([sys.executable, "-c", SCRIPT.format(root=ROOT)], capture_output=True, text=True, timeout=300)
    assert "SHARDED_OK" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("k,S,w", [(128, 512, 64), (100, 576, 40), (256, 512, 128)])
def test_encode_batch_dev_compact_columns(lib, k, S, w):
    """rsm_encode_batch_dev over a compact [k][w][S] column slice (the all-to-all
    schedule's layout) -> [k][w][S] parity, vs the oracle column by column."""
    top = oracle.splitmix64_bytes(k * w * S, seed=k + w).reshape(k, w, S)
    src = R.DeviceBuffer(k * w * S)
    dst = R.DeviceBuffer(k * w * S)
    src.upload(top)
    R._check(lib.rsm_encode_batch_dev(src.ctx, src.ptr, dst.ptr, k, S, w, S, w * S, None))
    R._check(lib.rsm_sync(src.ctx))
    got = dst.download().reshape(k, w, S)
    for c in range(0, w, max(1, w // 8)):
        want = oracle.encode([top[r, c].tobytes() for r in range(k)])
        assert [got[r, c].tobytes() for r in range(k)] == want, c
    src.free()
    dst.free()


SCRIPT_T = r"""
import os, sys
sys.path.insert(0, {root!r})
import numpy as np, torch, torch.distributed as dist
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29534", RANK="0", WORLD_SIZE="1")
torch.cuda.set_device(0)
dist.init_process_group("nccl")
from rsmt2d_amd.distributed import TransposeShardedExtender, hip_transpose_backend
import oracle
k, S = {k}, 512
ods = np.random.default_rng(4).integers(0, 256, (k, k, S), dtype=np.uint8)
rows = torch.zeros((k, 2 * k, S), dtype=torch.uint8, device="cuda")
rows[:, :k] = torch.from_numpy(ods).cuda()
top = torch.zeros((k, 2 * k, S), dtype=torch.uint8, device="cuda")
bottom = torch.zeros_like(top)
torch.cuda.synchronize()
ext = TransposeShardedExtender(k, S, *hip_transpose_backend(0))
ext.extend(rows, top, bottom)
want = oracle.extend_square(ods, nthreads=8)
ok = bool((top.cpu().numpy() == want[:k]).all() and (bottom.cpu().numpy() == want[k:]).all())
dist.destroy_process_group()
print("TRANSPOSE_OK" if ok else "TRANSPOSE_MISMATCH")
"""


@pytest.mark.parametrize("k", [128, 256])
def test_transpose_sharded_extender_rccl_world1(k):
    """k = 128: row pass + block copy (GF(2^8)); k = 256: the encoder writes the send block."""
    pytest.importorskip("torch")
    r = subprocess.run([sys.executable, "-c", SCRIPT_T.format(root=ROOT, k=k)], capture_output=True, text=True,
                       timeout=300)
    assert "TRANSPOSE_OK" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("k,S,row0,nrows,nblocks", [(256, 512, 64, 32, 8), (512, 512, 0, 64, 8), (192, 128, 48, 48, 4),
                                                    (256, 64, 0, 256, 16), (256, 64, 0, 40, 32), (128, 512, 16, 16, 8),
                                                    (100, 320, 10, 25, 4), (1024, 64, 128, 128, 8)])
def test_extend_rows_blocks_dev(lib, k, S, row0, nrows, nblocks):
    """rsm_extend_rows_blocks_dev == rsm_extend_rows_dev plus the rows cut into column
    blocks (the all-to-all send buffer): encoder side output (GF(2^16), k <= 512, k and
    block width multiples of 32) and the copy form (GF(2^8); 16-column blocks; k > 512).
    The block buffer starts as garbage, so a cell the encoder fails to store shows up."""
    W = 2 * k
    n = W * W * S
    cb = W // nblocks
    a, b = R.DeviceBuffer(n), R.DeviceBuffer(n)
    blocks = R.DeviceBuffer(nrows * W * S)
    a.fill_random(k + nrows)
    blocks.fill_random(5)
    R._check(lib.rsm_sync(a.ctx))
    R._check(lib.rsm_memcpy(a.ctx, b.ptr, a.ptr, n, 2))
    R._check(lib.rsm_extend_rows_dev(a.ctx, a.ptr, k, S, row0, nrows, None))
    R._check(lib.rsm_extend_rows_blocks_dev(b.ctx, b.ptr, k, S, row0, nrows, blocks.ptr, nblocks, None))
    R._check(lib.rsm_sync(a.ctx))
    want = a.download().reshape(W, W, S)
    assert (b.download().reshape(W, W, S) == want).all()
    got = blocks.download().reshape(nblocks, nrows, cb, S)
    mine = want[row0:row0 + nrows]
    for h in range(nblocks):
        assert (got[h] == mine[:, h * cb:(h + 1) * cb]).all(), h
    if k * S <= 256 * 64:  # the rows against the oracle (each row depends on its own Q0 cells only)
        assert (oracle.extend_square(want[:k, :k].copy(), nthreads=8)[row0:row0 + nrows] == mine).all()
    for x in (a, b, blocks):
        x.free()
