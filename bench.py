#!/usr/bin/env python3
"""bench.py -- device-resident 2D Reed-Solomon EDS encode on MI355X.

Metric (BASELINE.json): GiB/s of device-resident 2D RS encode, k=128 square,
512 B shares (config 2: 128x128 -> 256x256, GF(2^8)), plus % of HBM peak.

A "step" = ComputeExtendedDataSquare's arithmetic (erasureExtendSquare,
extendeddatasquare.go:154-227) over one batch of `--batch` independent squares
already resident in HBM (the EDS buffer holds each ODS in its top-left quadrant,
as the Go EDS aliases its input).  The batch (16 x 32 MiB = 512 MiB by default) is
larger than the 256 MiB Infinity Cache, so steps do not run out of cache.
value = ODS bytes encoded per second over all ranks (GiB/s).

N > 1 GPUs (one process per GPU, torch.distributed): every rank encodes its own
batch of independent squares -- the work partitions by square with no data-path
exchange, so scaling is "weak".

Extra JSON objects: "roofline" (dominant kernel, HIP-event timed on the launch
stream), "step_roofline" (whole 2D encode vs SURVEY's algorithmic bytes 4k^2 S),
"cpu_baseline" (the C oracle restatement -- kind "port" -- on this host's cores),
"host_path" (PCIe-inclusive rate through rsm_extend_square; never `value`).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
WORKLOADS = {
    "c2": dict(k=128, S=512, desc="128x128->256x256 square, 512 B shares, GF(2^8)"),
    "c4": dict(k=256, S=2048, desc="256x256->512x512 square, 2048 B shares, GF(2^16)"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    p.add_argument("--batch", type=int, default=0, help="squares per step (default: >= 512 MiB of EDS)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-c5", action="store_true", help="skip the config-5 (sharded 512x512 square) line")
    p.add_argument("--no-c3", action="store_true", help="skip the config-3 (Repair) timings")
    p.add_argument("--no-roots", action="store_true", help="skip the extension + Merkle roots timing")
    p.add_argument("--dist", action="store_true",
                   help="initialise torch.distributed even at N=1 (rehearses the sharded c5 path on one GPU)")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--one-stream", action="store_true", help="GF(2^8): do not alternate steps over two streams")
    p.add_argument("--streams", type=int, default=2, help="GF(2^8): streams the steps rotate over")
    p.add_argument("--buffers", type=int, default=2, help="batches (EDS buffers) the steps rotate over")
    p.add_argument("--row-grid", type=int, default=224,
                   help="GF(2^8) M=128 with >1 stream: CUs of the row-pass persistent grid (0 = all); the "
                        "remaining CUs run the other stream's column pass (profiles/r01h_grid_ab.txt)")
    p.add_argument("--schedule", choices=["pipelined", "two-launch"], default="two-launch",
                   help="GF(2^8) M=128: 'pipelined' = one launch per step running the next batch's row pass "
                        "with this batch's column pass (rsm_extend_pipeline_dev; A/B, slower than two launches "
                        "alternating over two streams: profiles/r01g_pipeline_ab.txt)")
    return p.parse_args()


def cpu_baseline(k, S, seconds):
    """The oracle's C restatement of the reference path, multithreaded over codewords."""
    import numpy as np
    import oracle
    threads = min(16, os.cpu_count() or 1)
    ods = oracle.splitmix64_bytes(k * k * S).reshape(k, k, S)
    oracle.extend_square(ods, nthreads=threads)  # warm
    n, t0 = 0, time.perf_counter()
    while True:
        oracle.extend_square(ods, nthreads=threads)
        n += 1
        dt = time.perf_counter() - t0
        if dt >= seconds:
            break
    return {"value": round(n * k * k * S / dt / 2**30, 4), "unit": "GiB/s", "cores": threads,
            "kind": "port",
            "sample": f"{n} squares k={k} S={S} through oracle/leopard_oracle.c (scalar C restatement of "
                      f"klauspost leopard, {threads} threads over codewords); the Go reference cannot run here"}


def bench_c5(world, rank, local, dist, steps, L, R):
    """Config 5: one 512x512 -> 1024x1024 square (GF(2^16), 512 B shares).  N=1: the
    whole square on one GPU; N>1: rows sharded over the N GPUs, then an RCCL
    all-to-all hands every GPU its column slice of the top half (SURVEY §8(e) Option B,
    rsmt2d_amd.distributed.TransposeShardedExtender); the all-gather schedule (Option
    A) is timed beside it.  Strong scaling of a single square."""
    k, S = 512, 512
    W = 2 * k
    steps = max(3, min(steps, 10))
    if dist is None:
        ctx = R.device_context(local)
        buf = R.DeviceBuffer(W * W * S, local)
        buf.fill_random(0xC5)
        R._check(L.rsm_extend_squares_dev(ctx, buf.ptr, k, S, 1, None))
        R._check(L.rsm_sync(ctx))
        t0 = time.perf_counter()
        for _ in range(steps):
            R._check(L.rsm_extend_squares_dev(ctx, buf.ptr, k, S, 1, None))
        R._check(L.rsm_sync(ctx))
        dt = (time.perf_counter() - t0) / steps
        buf.free()
    else:
        import torch
        from rsmt2d_amd.distributed import (RowShardedExtender, TransposeShardedExtender, hip_backend,
                                            hip_transpose_backend)
        dev = torch.device("cuda", local)
        g = torch.Generator(device=dev)
        g.manual_seed(0xC5 + rank)

        def timed(fn):
            fn()
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(steps):
                fn()
            torch.cuda.synchronize()
            dist.barrier()
            t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t.item()) / steps

        # Option B (primary): all-to-all of column slices
        tx = TransposeShardedExtender(k, S, *hip_transpose_backend(local))
        n, w = k // world, W // world
        rows = torch.zeros((n, W, S), dtype=torch.uint8, device=dev)
        rows[:, :k] = torch.randint(0, 256, (n, k, S), dtype=torch.uint8, device=dev, generator=g)
        top = torch.empty((k, w, S), dtype=torch.uint8, device=dev)
        bottom = torch.empty_like(top)
        torch.cuda.synchronize()
        dt = timed(lambda: tx.extend(rows, top, bottom))
        del rows, top, bottom
        # Option A (north_star's all-gather of the top half), for comparison
        eds = torch.zeros((W, W, S), dtype=torch.uint8, device=dev)
        ext = RowShardedExtender(k, S, *hip_backend(local))
        r0, r1 = ext.rows
        eds[r0:r1, :k] = torch.randint(0, 256, (r1 - r0, k, S), dtype=torch.uint8, device=dev, generator=g)
        torch.cuda.synchronize()
        dt_ag = timed(lambda: ext.extend(eds))
        del eds
    out = {"workload": "c5: 512x512->1024x1024 square, 512 B shares, GF(2^16)"
                       + ("" if world == 1 else f", rows sharded over {world} GPUs + RCCL all-to-all of column slices"),
           "n_gpus": world, "ms_per_square": round(dt * 1e3, 4), "ods_GiB_s": round(k * k * S / dt / 2**30, 3),
           "scaling": "strong (one square)"}
    if dist is not None:
        out["received_bytes_per_gpu"] = (world - 1) * (k // world) * (W // world) * S
        out["allgather_ms_per_square"] = round(dt_ag * 1e3, 4)
        out["allgather_received_bytes_per_gpu"] = (world - 1) * (k // world) * W * S
    return out


def bench_c3(local, L, R, repeats=5):
    """Config 3: k=128, S=512, exactly k of the 2k cells of every
    row erased (BenchmarkRepair's scheme, extendeddatacrossword_test.go:443-453),
    honest DefaultTree roots.  Two timings:
      decode_sweep -- the device decode of all 2k rows alone (rsm_decode_vectors_dev
                      over a device-resident EDS + presence mask, HIP-synchronised);
      repair       -- (*ExtendedDataSquare).Repair end to end as BenchmarkRepair
                      times it (import untimed): upload, device sweeps, full
                      re-extension check, DefaultTree roots of every row/col
                      (on the device), copy back.
    Replicas only: Repair is not sharded."""
    import ctypes
    import numpy as np
    k, S = 128, 512
    W = 2 * k
    ctx = R.device_context(local)
    rng = np.random.default_rng(0xC3)
    # original EDS from the device extension of a seeded ODS
    buf = R.DeviceBuffer(W * W * S, local)
    buf.fill_random(0xC3)
    R._check(L.rsm_extend_squares_dev(ctx, buf.ptr, k, S, 1, None))
    R._check(L.rsm_sync(ctx))
    full = buf.download(W * W * S).reshape(W, W, S)
    present = np.ones((W, W), np.uint8)
    for r in range(W):
        present[r, rng.choice(W, size=k, replace=False)] = 0

    # honest roots
    base = full.ctypes.data
    ptrs = (ctypes.c_void_p * (W * W))(*[base + i * S for i in range(W * W)])
    lens = (ctypes.c_uint32 * (W * W))(*([S] * (W * W)))
    h = ctypes.c_void_p()
    R._check(L.rsm_eds_import(None, ptrs, lens, W * W, ctypes.byref(h)))
    roots = {}
    for axis in (0, 1):
        out = ctypes.create_string_buffer(W * 32)
        rl = ctypes.c_uint32()
        R._check(L.rsm_eds_roots(h, axis, None, None, out, 32, ctypes.byref(rl)))  # NULL = DefaultTree
        roots[axis] = out.raw
    L.rsm_eds_free(h)

    # (1) device decode sweep alone
    damaged = full * present[:, :, None]
    buf.upload(damaged)
    pres_d = R.DeviceBuffer(W * W, local)
    pres_d.upload(present)
    idx_d = R.DeviceBuffer(4 * W, local)
    idx_d.upload(np.arange(W, dtype=np.uint32))
    sweep = lambda: R._check(L.rsm_decode_vectors_dev(ctx, buf.ptr, pres_d.ptr, k, S, 0, idx_d.ptr, W, None))
    sweep()
    R._check(L.rsm_sync(ctx))
    if not np.array_equal(buf.download(W * W * S).reshape(W, W, S), full):
        raise SystemExit("bench c3: device decode sweep differs from the original EDS")
    n_sw = 50
    t0 = time.perf_counter()
    for _ in range(n_sw):
        sweep()
    R._check(L.rsm_sync(ctx))
    t_sweep = (time.perf_counter() - t0) / n_sw
    for b in (buf, pres_d, idx_d):
        b.free()

    # (2) end-to-end Repair (import untimed, as BenchmarkRepair)
    flat_ptrs = (ctypes.c_void_p * (W * W))(*[base + i * S if present.flat[i] else None for i in range(W * W)])
    flat_lens = (ctypes.c_uint32 * (W * W))(*[S if present.flat[i] else 0 for i in range(W * W)])
    times, stats = [], R.RepairStats()
    for _ in range(repeats):
        h = ctypes.c_void_p()
        R._check(L.rsm_eds_import(None, flat_ptrs, flat_lens, W * W, ctypes.byref(h)))
        R._check(L.rsm_eds_set_context(h, ctx))
        byz = R._Byz()
        t0 = time.perf_counter()
        R._check(L.rsm_eds_repair(h, roots[0], roots[1], 32, None, None, ctypes.byref(byz)))
        times.append(time.perf_counter() - t0)
        R._check(L.rsm_eds_repair_stats(h, ctypes.byref(stats)))
        if repeats and len(times) == 1:
            got = np.empty((W, W, S), np.uint8)
            pr = np.empty((W, W), np.uint8)
            R._check(L.rsm_eds_flattened(h, got.ctypes.data, pr.ctypes.data))
            if not (pr.all() and np.array_equal(got, full)):
                raise SystemExit("bench c3: repaired EDS differs from the original")
        L.rsm_eds_free(h)
    t_rep = sorted(times)[len(times) // 2]
    algo = W * W * S  # present shares read + missing shares written
    return {"workload": "c3: k=128, S=512, 128 of 256 cells erased in every row (BenchmarkRepair scheme)",
            "decode_sweep_us": round(t_sweep * 1e6, 2),
            "decode_sweep_GB_s": round(algo / t_sweep / 1e9, 1),
            "decode_sweep_frac": round(algo / t_sweep / 1e9 / HBM_PEAK_GBS, 4),
            "repair_ms": round(t_rep * 1e3, 3), "repair_samples": repeats,
            "repair_fast_path": int(stats.fast_path), "repair_sweeps": int(stats.sweeps),
            "note": "repair = rsm_eds_repair end to end (H2D, device sweeps, device re-extension check, "
                    "device DefaultTree roots of all 512 vectors, D2H into the EDS buffer); median of samples"}


def bench_roots(local, L, R, buf, k, S, B, steps):
    """BenchmarkExtensionWithRoots (extendeddatasquare_test.go:309-334): the 2D
    extension plus RowRoots + ColRoots (DefaultTree) of every square, all on the
    device (rsm_extend_squares_dev + one rsm_roots_squares_dev for the batch)."""
    ctx = R.device_context(local)
    W = 2 * k
    roots = R.DeviceBuffer(2 * W * 32 * B, local)

    def run():
        R._check(L.rsm_extend_squares_dev(ctx, buf.ptr, k, S, B, None))
        R._check(L.rsm_roots_squares_dev(ctx, buf.ptr, W, S, B, roots.ptr, None))

    run()
    R._check(L.rsm_sync(ctx))
    n = max(3, min(steps, 10))
    t0 = time.perf_counter()
    for _ in range(n):
        run()
    R._check(L.rsm_sync(ctx))
    dt = (time.perf_counter() - t0) / n
    t0 = time.perf_counter()
    for _ in range(n):
        R._check(L.rsm_roots_squares_dev(ctx, buf.ptr, W, S, B, roots.ptr, None))
    R._check(L.rsm_sync(ctx))
    dr = (time.perf_counter() - t0) / n
    roots.free()
    return {"workload": f"extension + DefaultTree row/col roots, k={k}, S={S}, {B} squares per step",
            "ms_per_square": round(dt / B * 1e3, 4), "ods_GiB_s": round(B * k * k * S / dt / 2**30, 3),
            "roots_only_ms_per_square": round(dr / B * 1e3, 4),
            "note": "leaf SHA-256 per cell (shared by its row and column tree) + per-tree node hashes on the GPU, "
                    "one launch pair per batch"}


def main():
    a = parse()
    import numpy as np

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1 or a.dist:
        # torch.distributed only for the timing barrier and the max-over-ranks of the
        # elapsed time (the workload itself has no data-path exchange).  torch's own HIP
        # runtime must initialise before librsmt2d_hip.so is loaded.
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(backend="nccl", init_method="env://")
        dev = torch.device("cuda", local)
    import rsmt2d_amd as R

    wl = WORKLOADS[a.workload]
    k, S = wl["k"], wl["S"]
    W = 2 * k
    sq_bytes = W * W * S
    B = a.batch or max(1, (512 << 20) // sq_bytes)
    L = R.library()
    ctx = R.device_context(local)

    # synthetic ODS: seeded uniform bytes (SplitMix64) generated on the device; each
    # square's top-left quadrant is its ODS (the other quadrants are overwritten).
    # Two batches are used alternately, so a step never finds the previous step's
    # squares in the 256 MiB Infinity Cache (rotate > 512 MiB).
    bufs = [R.DeviceBuffer(B * sq_bytes, local) for _ in range(max(2, a.buffers))]
    for i, b in enumerate(bufs):
        b.fill_random(0x52534D543244 + 2 * rank + i)
    R._check(L.rsm_sync(ctx))
    buf = bufs[0]
    nstep = [0]
    # GF(2^8): consecutive steps alternate between two streams (each step's row and
    # column passes stay ordered on its own stream), so one step's column-pass tail
    # overlaps the next step's row-pass prologue.  GF(2^16) shares the context's work
    # arrays between launches: one stream.
    import ctypes
    streams = [None]
    if k <= 128 and not a.one_stream:
        for _ in range(max(1, a.streams) - 1):
            s2 = ctypes.c_void_p()
            R._check(L.rsm_stream_create(ctx, ctypes.byref(s2)))
            streams.append(s2)

    pipelined = a.schedule == "pipelined" and 64 < k <= 128

    row_grid = a.row_grid if (len(streams) > 1 and 64 < k <= 128) else 0
    L.rsm_set_pass_grid(0, row_grid)

    def step():
        i = nstep[0]
        nstep[0] += 1
        R._check(L.rsm_extend_squares_dev(ctx, bufs[i % len(bufs)].ptr, k, S, B, streams[i % len(streams)]))

    def run(n):
        if not pipelined:
            for _ in range(n):
                step()
            return
        # n complete extensions in n + 1 launches: launch i runs batch i+1's row pass
        # and batch i's column pass (batches alternate between the two buffers)
        R._check(L.rsm_extend_pipeline_dev(ctx, bufs[0].ptr, None, k, S, B, None))
        for i in range(n):
            rows = bufs[(i + 1) & 1].ptr if i + 1 < n else None
            R._check(L.rsm_extend_pipeline_dev(ctx, rows, bufs[i & 1].ptr, k, S, B, None))

    def sync_all():
        R._check(L.rsm_sync(ctx))
        for st in streams[1:]:
            R._check(L.rsm_stream_sync(st))

    run(max(1, a.warmup))
    sync_all()
    # correctness gate on one square before timing (the oracle is the checker only)
    if rank == 0:
        import oracle
        got = buf.download(sq_bytes).reshape(W, W, S)
        want = oracle.extend_square(got[:k, :k].copy(), nthreads=min(16, os.cpu_count() or 1))
        if not np.array_equal(got, want):
            raise SystemExit("bench: GPU EDS differs from oracle -- refusing to report")

    def barrier():
        if dist is not None:
            dist.barrier()
            torch.cuda.synchronize()

    barrier()
    sync_all()
    t0 = time.perf_counter()
    run(a.steps)
    sync_all()
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # per-kernel durations: HIP events on the launch stream (the context stream)
    import ctypes
    row_ms, col_ms, step_ms = ctypes.c_float(), ctypes.c_float(), ctypes.c_float()
    rms, cms, sms = [], [], []
    for r in range(max(6, min(a.steps, 20))):  # row, column, then one production step per call
        R._check(L.rsm_time_extend(ctx, bufs[r & 1].ptr, k, S, B, 1, ctypes.byref(row_ms), ctypes.byref(col_ms),
                                   ctypes.byref(step_ms)))
        rms.append(row_ms.value)
        cms.append(col_ms.value)
        sms.append(step_ms.value)
    t_row, t_col = sum(rms) / len(rms) / 1e3, sum(cms) / len(cms) / 1e3
    t_fused = sum(sms) / len(sms) / 1e3
    fused = bool(L.rsm_extend_fused(k, S))
    t_pipe = None
    if pipelined:
        pms = ctypes.c_float()
        R._check(L.rsm_time_pipeline(ctx, bufs[1].ptr, bufs[0].ptr, k, S, B, max(6, min(a.steps, 20)),
                                     ctypes.byref(pms)))
        t_pipe = pms.value / 1e3

    ods_bytes = k * k * S
    total = world * B * a.steps * ods_bytes
    value = total / elapsed / 2**30
    ms_per_step = elapsed / a.steps * 1e3
    algo_step = 4 * ods_bytes * B  # read Q0 once, write Q1+Q2+Q3
    col_bytes = 4 * ods_bytes * B  # column pass: [Q0|Q1] in, [Q2|Q3] out
    row_bytes = 2 * ods_bytes * B  # row pass: Q0 in, Q1 out
    bitsliced = 64 < k <= 128
    kname = ("encode_gf8_bs128u_kernel" if bitsliced else "encode_gf8_kernel" if k <= 64
             else "enc16_a/b/c (GF(2^16) passes)")
    col_dom = t_col >= t_row
    dominant = ((kname + " column pass", col_bytes, t_col) if col_dom else (kname + " row pass", row_bytes, t_row))
    if fused:
        # opt-in: ONE launch per step runs both passes (encode_gf8_bs128f_kernel);
        # its algorithmic bytes are the step's 4k^2 S
        kname = "encode_gf8_bs128f_kernel"
        dominant = (kname + " (fused row + column passes)", algo_step, t_fused)
    if pipelined:
        # one launch per step: batch i+1's row pass + batch i's column pass
        # (encode_gf8_bs128p_kernel) -- one step's worth of algorithmic bytes, 4k^2 S B
        kname = "encode_gf8_bs128p_kernel"
        dominant = (kname + " (row pass of batch i+1 + column pass of batch i)", algo_step, t_pipe)
    ach = dominant[1] / dominant[2] / 1e9
    # HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC
    # passes (scripts/pmc_summary.py; FETCH_SIZE x2 gfx950 correction), matched by
    # kernel name (<MODE, PASS>: PASS 1 = column pass) -- null when no matching
    # profile exists (e.g. the multi-kernel GF(2^16) passes).
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if bitsliced and os.path.exists(pmc_path):
        # production template <MODE 40, PASS>; A/B modes (RSM_BS_MODE) launch PASS 1
        want = "encode_gf8_bs128u_kernel<%s, %d>" % (os.environ.get("RSM_BS_MODE", "40"), 1 if col_dom else 0)
        sets = (W if col_dom else k) * B * S // 2048
        if fused:
            want, sets = "encode_gf8_bs128f_kernel<40>", 3 * k * B * S // 2048
        if pipelined:
            want, sets = "encode_gf8_bs128p_kernel<40>", 3 * k * B * S // 2048
        grid_threads = min(sets, 256) * 512  # persistent grid: one 512-thread workgroup per CU
        for row in json.load(open(pmc_path)).get("launches", []):
            if want in row["kernel"] and row["grid_threads"] == grid_threads:
                traffic = int(row["traffic_bytes"])
    out = {
        "metric": "GiB/s device-resident 2D RS encode, k=128 square, 512 B shares; % HBM peak",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8" if k <= 128 else "u16",
        "data": "synthetic (seeded SplitMix64 bytes, device-generated)",
        "config": {"workload": f"{a.workload}: {wl['desc']}", "k": k, "share_size": S,
                   "squares_per_step": B, "eds_bytes_per_step": B * sq_bytes,
                   "parallelism": f"independent squares per GPU x{world}",
                   "schedule": "pipelined" if pipelined else "two-launch",
                   "streams": len(streams), "row_pass_grid": row_grid or None},
        "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel": dominant[0], "avg_launch_us": round(dominant[2] * 1e6, 2),
                     "bytes_per_launch": dominant[1]},
        "step_roofline": {"algorithmic_bytes": algo_step,
                          "achieved": round(algo_step / (elapsed / a.steps) / 1e9, 1),
                          "frac": round(algo_step / (elapsed / a.steps) / 1e9 / HBM_PEAK_GBS, 4),
                          "row_pass_us": round(t_row * 1e6, 2), "col_pass_us": round(t_col * 1e6, 2),
                          "one_step_launch_us": round(t_fused * 1e6, 2), "fused": fused,
                          "schedule": "pipelined" if pipelined else "two-launch",
                          "pipelined_launch_us": round(t_pipe * 1e6, 2) if t_pipe else None},
    }
    if rank == 0 and world == 1:
        # PCIe-inclusive host-memory rate (ComputeExtendedDataSquare from host buffers)
        ods = np.random.default_rng(1).integers(0, 256, (k, k, S), dtype=np.uint8)
        eh = np.empty((W, W, S), np.uint8)
        R._check(L.rsm_extend_square(ctx, ods.ctypes.data, k, S, eh.ctypes.data))
        t1, n = time.perf_counter(), 0
        while time.perf_counter() - t1 < 1.0:
            R._check(L.rsm_extend_square(ctx, ods.ctypes.data, k, S, eh.ctypes.data))
            n += 1
        out["host_path"] = {"value": round(n * ods_bytes / (time.perf_counter() - t1) / 2**30, 3), "unit": "GiB/s",
                            "note": "rsm_extend_square: pageable host ODS -> H2D -> extend -> D2H EDS, one square"}
        out["cpu_baseline"] = None if a.no_cpu_baseline else cpu_baseline(k, S, a.cpu_seconds)
    if rank == 0 and world == 1 and not a.no_roots:
        out["with_roots"] = bench_roots(local, L, R, buf, k, S, B, a.steps)
    for b in bufs:
        b.free()
    for st in streams[1:]:
        R._check(L.rsm_stream_destroy(ctx, st))
    if rank == 0 and world == 1 and not a.no_c3:
        out["c3"] = bench_c3(local, L, R)
    if not a.no_c5:
        out["c5"] = bench_c5(world, rank, local, dist, a.steps, L, R)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
