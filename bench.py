#!/usr/bin/env python3
"""bench.py -- device-resident 2D Reed-Solomon EDS encode on MI355X.

Metric (BASELINE.json): GiB/s of device-resident 2D RS encode, k=128 square,
512 B shares (config 2: 128x128 -> 256x256, GF(2^8)), plus % of HBM peak.

A "step" = ComputeExtendedDataSquare's arithmetic (erasureExtendSquare,
extendeddatasquare.go:154-227) over one batch of `--batch` independent squares
already resident in HBM (the EDS buffer holds each ODS in its top-left quadrant,
as the Go EDS aliases its input).  c2 default: 512 squares (16 GiB of EDS) per step
as ONE queue-driven launch (both passes, extend_gf8_bs128s_kernel: half-split
bit-sliced sets), steps rotating over 3 streams and 3 buffers
(48 GiB of the 288 GB), so no step finds its squares in the 256 MiB Infinity Cache.
value = ODS bytes encoded per second over all ranks (GiB/s).

N > 1 GPUs (one process per GPU, torch.distributed): every rank encodes its own
batch of independent squares -- the work partitions by square with no data-path
exchange, so scaling is "weak".

Extra JSON objects: "roofline" (dominant kernel, HIP-event timed on the launch
stream), "step_roofline" (whole 2D encode vs SURVEY's algorithmic bytes 4k^2 S),
"cpu_baseline" (the C restatement of the reference path -- AVX-512 + GFNI where the host has
it, else AVX2 -- kind "port", on every CPU this process may run on: sched_getaffinity),
"host_path" (PCIe-inclusive rates, pinned+overlapped and pageable; never `value`),
"codec" (per-codeword Encode latency and 64-thread concurrent rate).
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
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    p.add_argument("--batch", type=int, default=0, help="squares per step (default: >= 1 GiB of EDS; steps rotate over --buffers batches, so a step never finds its squares in the 256 MiB Infinity Cache)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-c5", action="store_true", help="skip the config-5 (sharded 512x512 square) line")
    p.add_argument("--no-c3", action="store_true", help="skip the config-3 (Repair) timings")
    p.add_argument("--no-c4", action="store_true", help="skip the config-4 (k=256, S=2048, GF(2^16)) line")
    p.add_argument("--no-gf16-repair", action="store_true", help="skip the k=256/512 Repair timings")
    p.add_argument("--no-roots", action="store_true", help="skip the extension + Merkle roots timing")
    p.add_argument("--no-extras", action="store_true", help="skip host-path and Codec-latency lines")
    p.add_argument("--headline-only", action="store_true",
                   help="only the headline line (no sub-lines, no CPU baseline): the command the committed "
                        "rocprofv3 kernel-trace / PMC summaries are taken from")
    p.add_argument("--dist", action="store_true",
                   help="initialise torch.distributed even at N=1 (rehearses the sharded c5 path on one GPU)")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--one-stream", action="store_true", help="GF(2^8): do not alternate steps over two streams")
    p.add_argument("--streams", type=int, default=0,
                   help="GF(2^8): streams the steps rotate over (default 3 for the single-launch k=128 "
                        "schedule, 2 for the two-launch one)")
    p.add_argument("--buffers", type=int, default=0, help="batches (EDS buffers) the steps rotate over "
                   "(default: one per stream, at least 2)")
    p.add_argument("--two-launch", action="store_true",
                   help="k=128: the round-1 schedule (row pass launch + column pass launch) instead of the "
                        "single queue-driven launch")
    p.add_argument("--row-grid", type=int, default=224,
                   help="GF(2^8) M=128 with >1 stream: CUs of the row-pass persistent grid (0 = all); the "
                        "remaining CUs run the other stream's column pass (profiles/r01h_grid_ab.txt)")
    a = p.parse_args()
    a.no_single = a.headline_only
    if a.headline_only:
        a.no_cpu_baseline = a.no_c5 = a.no_c3 = a.no_c4 = a.no_gf16_repair = a.no_roots = a.no_extras = True
    return a


def cpu_info():
    model, cores = None, os.cpu_count()
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return model, cores


def cpu_baseline(k, S, seconds):
    """The reference path restated on the host CPU (oracle/leopard_oracle.c with
    klauspost's fastest x86 leopard8 technique where the CPU has it: AVX-512 rows,
    GF2P8AFFINEQB multiplies, fused butterflies -- libleopard_gfni.so; else the AVX2
    pshufb build), multithreaded over codewords with the reference's two-phase
    schedule, writing into a reused EDS buffer (no page faults in the timed loop).
    Threads: the CPUs this job may actually use -- its affinity mask
    (os.sched_getaffinity; os.cpu_count() is the whole machine), capped by its cgroup
    CPU share -- the cgroup quota (cpu.max) when one is set, else the share the
    harness declares for worker pools (OMP_NUM_THREADS): on the GPU box the mask is all
    256 host CPUs but the share is 16, and 256 threads there ran at 5.8 GiB/s against
    18-19 for 16 (profiles/r04f_bench.json).  The mask, the quota, a short run with one
    thread per CPU of the mask, the single-thread rate and its linear all-host-CPUs
    extrapolation are reported beside it.  Not the reference: its Go/klauspost code
    cannot run here."""
    import numpy as np
    import oracle
    ncpu = os.cpu_count() or 1
    try:
        mask = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        mask = list(range(ncpu))
    # the job's CPU share: its cgroup quota, else the share the harness declares for
    # worker pools (OMP_NUM_THREADS), else the whole affinity mask
    quota, share_src = _cgroup_cpu_quota(), "cgroup cpu.max"
    if not quota and os.environ.get("OMP_NUM_THREADS", "").isdigit():
        quota, share_src = int(os.environ["OMP_NUM_THREADS"]), "OMP_NUM_THREADS"
    threads = max(1, min(len(mask), quota) if quota else len(mask))
    gfni = oracle.gfni_supported() and k <= 128
    ext = oracle.extend_square_gfni if gfni else oracle.extend_square_simd if k <= 128 else None
    ods = oracle.splitmix64_bytes(k * k * S).reshape(k, k, S)
    out = np.empty((2 * k, 2 * k, S), np.uint8)

    def rate(nth, secs):
        """Squares per second with `nth` host threads, each extending whole squares on
        its own (the bench workload is independent squares: one square per thread is
        the CPU's natural schedule; splitting one 8 MiB square's codewords over 16
        threads scaled 2.2x, r03i)."""
        import threading
        outs = [np.empty_like(out) for _ in range(nth)]
        done = [0] * nth
        stop = [False]

        def work(i):
            run = (lambda: ext(ods, nthreads=1, out=outs[i])) if ext else (lambda: oracle.extend_square(ods, nthreads=1))
            while not stop[0]:
                run()
                done[i] += 1

        for i in range(nth):  # warm (page in every output buffer)
            (ext(ods, nthreads=1, out=outs[i]) if ext else oracle.extend_square(ods, nthreads=1))
        ths = [threading.Thread(target=work, args=(i,)) for i in range(nth)]
        t0 = time.perf_counter()
        for t in ths:
            t.start()
        time.sleep(secs)
        stop[0] = True
        for t in ths:
            t.join()
        return sum(done), time.perf_counter() - t0

    n, dt = rate(threads, seconds)
    n1, dt1 = rate(1, max(2.0, seconds / 4))
    nm, dtm = rate(len(mask), max(2.0, seconds / 4)) if len(mask) != threads else (n, dt)
    model, _ = cpu_info()
    tech = ("AVX-512 + GFNI (GF2P8AFFINEQB multiplies, fused butterflies)" if gfni
            else "AVX2 pshufb nibble tables" if ext else "scalar tables")
    return {"value": round(n * k * k * S / dt / 2**30, 4), "unit": "GiB/s", "cores": threads,
            "kind": "port", "cpu_model": model, "host_cpus": ncpu, "affinity": _ranges(mask),
            "cpu_share": quota, "cpu_share_source": share_src if quota else None,
            "affinity_threads_GiB_s": round(nm * k * k * S / dtm / 2**30, 4),
            "single_thread_GiB_s": round(n1 * k * k * S / dt1 / 2**30, 4),
            "all_cores_estimate_GiB_s": round(n1 * k * k * S / dt1 / 2**30 * ncpu, 1),
            "sample": f"{n} squares k={k} S={S} ({dt:.1f} s) through oracle/leopard_oracle.c ({tech}; restatement "
                      f"of klauspost leopard8, not the reference), {threads} threads (the affinity mask of "
                      f"{len(mask)} CPUs capped by the job's CPU share {quota} from {share_src}) each extending "
                      f"whole squares; "
                      f"affinity_threads: {len(mask)} threads, {nm} squares in {dtm:.1f} s; single thread: {n1} "
                      f"squares in {dt1:.1f} s; all_cores_estimate = single-thread rate x {ncpu} host CPUs "
                      f"(linear, not measured)"}


def _cgroup_cpu_quota():
    """CPUs of this job's cgroup CPU quota (cgroup v2 cpu.max "quota period", v1
    cfs_quota_us / cfs_period_us), rounded up; None when unlimited or unreadable."""
    import math
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else max(1, math.ceil(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else max(1, math.ceil(q / per))
    except (OSError, ValueError):
        return None


def _ranges(cpus):
    """[0, 1, 2, 5] -> "0-2,5" (an affinity mask as taskset prints it)."""
    out, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(out)


def pct(xs, q):
    xs = sorted(xs)
    if not xs:
        return None
    i = min(len(xs) - 1, max(0, int(round(q * (len(xs) - 1)))))
    return xs[i]


def bench_codec(local, L, R, k=128, S=512, calls=400, threads=64):
    """Per-codeword Encode (codec_test.go:15-35 BenchmarkEncoding, k=128, 512 B):
    latency of one rsm_encode from host memory on an idle GPU, and aggregate rate
    with `threads` host threads calling concurrently (rsmt2d's 2k goroutines).  Also
    Decode in BenchmarkDecoding's shape (codec_test.go:50-92: the 2k shares of a k =
    128 codeword with k/2 of them nil at random), every result checked."""
    import ctypes
    import threading
    import numpy as np
    ctx = R.device_context(local)
    rng = np.random.default_rng(7)

    def mk():
        data = rng.integers(0, 256, (k, S), dtype=np.uint8)
        par = np.empty((k, S), np.uint8)
        dp = (ctypes.c_void_p * k)(*[data.ctypes.data + i * S for i in range(k)])
        pp = (ctypes.c_void_p * k)(*[par.ctypes.data + i * S for i in range(k)])
        return data, par, dp, pp

    d, p, dp, pp = mk()
    for _ in range(20):
        R._check(L.rsm_encode(ctx, dp, k, S, pp))
    lat = []
    for _ in range(calls):
        t0 = time.perf_counter()
        R._check(L.rsm_encode(ctx, dp, k, S, pp))
        lat.append(time.perf_counter() - t0)
    per = max(1, calls // 2)
    bufs = [mk() for _ in range(threads)]
    errs = []

    def worker(i):
        _, _, a, b = bufs[i]
        for _ in range(per):
            rc = L.rsm_encode(ctx, a, k, S, b)
            if rc:
                errs.append(rc)

    ths = [threading.Thread(target=worker, args=(i,)) for i in range(threads)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    dt = time.perf_counter() - t0
    if errs:
        raise SystemExit(f"bench codec: concurrent rsm_encode failed {errs[:3]}")
    n = threads * per
    # BenchmarkDecoding: k/2 of the 2k shares nil
    full = np.concatenate([d, p])
    present = np.ones(2 * k, np.uint8)
    present[rng.choice(2 * k, size=k // 2, replace=False)] = 0
    work = np.empty_like(full)
    wp = (ctypes.c_void_p * (2 * k))(*[work.ctypes.data + i * S for i in range(2 * k)])
    dlat = []
    for i in range(calls + 20):
        work[:] = full * present[:, None]
        t0 = time.perf_counter()
        R._check(L.rsm_decode(ctx, wp, present.ctypes.data, 2 * k, S))
        if i >= 20:
            dlat.append(time.perf_counter() - t0)
        if i == 0 and not np.array_equal(work, full):
            raise SystemExit("bench codec: rsm_decode result differs")
    return {"workload": f"per-codeword Encode k={k} S={S} from host memory (BenchmarkEncoding shape)",
            "latency_us_p50": round(pct(lat, 0.5) * 1e6, 1), "latency_us_p10": round(pct(lat, 0.1) * 1e6, 1),
            "latency_us_p90": round(pct(lat, 0.9) * 1e6, 1),
            "concurrent_threads": threads, "concurrent_codewords_per_s": round(n / dt, 1),
            "concurrent_GiB_s": round(n * k * S / dt / 2**30, 3),
            "decode_workload": f"per-codeword Decode of 2k={2 * k} shares, {k // 2} nil (BenchmarkDecoding shape)",
            "decode_latency_us_p50": round(pct(dlat, 0.5) * 1e6, 1),
            "decode_latency_us_p10": round(pct(dlat, 0.1) * 1e6, 1),
            "decode_latency_us_p90": round(pct(dlat, 0.9) * 1e6, 1)}


def bench_fraud_proof(local, L, R, k=128, S=512, reps=300):
    """Fraud-proof verification (extendeddatacrossword_test.go:116-163)
    as a light client runs it on one byzantine row of a c2 square: Decode the 2k
    shares of the proof (k of them nil), DefaultTree root of the rebuilt vector
    (compared with the row root), re-Encode the first k and compare the parity half.
    Latency of the whole check from host memory, one proof at a time."""
    import ctypes
    import numpy as np
    ctx = R.device_context(local)
    rng = np.random.default_rng(0xF4)
    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
    par = np.empty((k, S), np.uint8)
    dp = (ctypes.c_void_p * k)(*[data.ctypes.data + i * S for i in range(k)])
    pp = (ctypes.c_void_p * k)(*[par.ctypes.data + i * S for i in range(k)])
    R._check(L.rsm_encode(ctx, dp, k, S, pp))
    full = np.concatenate([data, par])
    present = np.ones(2 * k, np.uint8)
    present[rng.choice(2 * k, size=k, replace=False)] = 0
    work = np.empty_like(full)
    wp = (ctypes.c_void_p * (2 * k))(*[work.ctypes.data + i * S for i in range(2 * k)])
    p2 = np.empty((k, S), np.uint8)
    pp2 = (ctypes.c_void_p * k)(*[p2.ctypes.data + i * S for i in range(k)])
    root = ctypes.create_string_buffer(64)
    rlen = ctypes.c_uint32()
    lat, t_dec = [], []
    for i in range(reps + 20):
        work[:] = full * present[:, None]
        t0 = time.perf_counter()
        R._check(L.rsm_decode(ctx, wp, present.ctypes.data, 2 * k, S))
        t1 = time.perf_counter()
        rlen.value = 64
        R._check(L.rsm_default_tree_root(None, 0, 0, wp, 2 * k, S, root, ctypes.byref(rlen)))
        R._check(L.rsm_encode(ctx, wp, k, S, pp2))
        ok = np.array_equal(p2, work[k:])
        t2 = time.perf_counter()
        if not ok or not np.array_equal(work, full):
            raise SystemExit("bench fraud proof: rebuilt vector differs")
        if i >= 20:
            lat.append(t2 - t0)
            t_dec.append(t1 - t0)
    return {"workload": f"fraud-proof check of one row, k={k} S={S}: Decode of 2k shares (k nil) + DefaultTree "
                        "root + re-Encode + parity compare (extendeddatacrossword_test.go:116-163)",
            "latency_us_p50": round(pct(lat, 0.5) * 1e6, 1), "latency_us_p10": round(pct(lat, 0.1) * 1e6, 1),
            "latency_us_p90": round(pct(lat, 0.9) * 1e6, 1), "decode_us_p50": round(pct(t_dec, 0.5) * 1e6, 1),
            "proofs": reps}


def bench_host_path(local, L, R, k, S, squares=8, seconds=2.0):
    """ComputeExtendedDataSquare from host memory (north_star: rate including
    hipMemcpyAsync both ways).  pinned: rsm_extend_squares_host over `squares`
    squares in pinned arenas (H2D / extension / D2H of different squares overlap on
    three streams; only Q1..Q3 come back); pageable: rsm_extend_square one square
    at a time from numpy memory."""
    import ctypes
    import numpy as np
    ctx = R.device_context(local)
    W = 2 * k
    ob, eb = k * k * S, W * W * S
    hp_o, hp_e = ctypes.c_void_p(), ctypes.c_void_p()
    R._check(L.rsm_host_alloc(ctx, ob * squares, ctypes.byref(hp_o)))
    R._check(L.rsm_host_alloc(ctx, eb * squares, ctypes.byref(hp_e)))
    ods = np.ctypeslib.as_array((ctypes.c_uint8 * (ob * squares)).from_address(hp_o.value))
    ods[:] = np.random.default_rng(3).integers(0, 256, ob * squares, dtype=np.uint8)
    R._check(L.rsm_extend_squares_host(ctx, hp_o, k, S, squares, hp_e))
    eds = np.ctypeslib.as_array((ctypes.c_uint8 * eb).from_address(hp_e.value)).reshape(W, W, S)
    import oracle
    if not np.array_equal(eds, oracle.extend_square(ods[:ob].reshape(k, k, S), nthreads=8)):
        raise SystemExit("bench host path: pinned batch differs from the oracle")
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        R._check(L.rsm_extend_squares_host(ctx, hp_o, k, S, squares, hp_e))
        n += 1
    pinned = n * squares * ob / (time.perf_counter() - t0) / 2**30
    R._check(L.rsm_host_free(ctx, hp_o))
    R._check(L.rsm_host_free(ctx, hp_e))
    o1 = np.random.default_rng(1).integers(0, 256, (k, k, S), dtype=np.uint8)
    e1 = np.empty((W, W, S), np.uint8)
    R._check(L.rsm_extend_square(ctx, o1.ctypes.data, k, S, e1.ctypes.data))
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds / 2:
        R._check(L.rsm_extend_square(ctx, o1.ctypes.data, k, S, e1.ctypes.data))
        n += 1
    pageable = n * ob / (time.perf_counter() - t0) / 2**30
    return {"pinned_GiB_s": round(pinned, 3), "pageable_GiB_s": round(pageable, 3), "unit": "GiB/s ODS",
            "pcie_bytes_per_square": ob + 3 * ob,
            "note": f"pinned = rsm_extend_squares_host over {squares} squares per call (3 streams: H2D, extension and "
                    "D2H of different squares overlap; Q0 is not copied back); pageable = rsm_extend_square per square"}


def bench_c5_c_abi(G, L, R, steps, k=512, S=512):
    """Config 5 through the C ABI a cgo ComputeExtendedDataSquare would call
    (rsm_multi_*: ONE process drives all G GPUs, an RCCL clique from ncclCommInitAll,
    extendeddatasquare.go:50-77): (1) device-resident rsm_multi_extend_dev (row pass of
    each GPU's k/G rows, RCCL exchange, column pass of its 2k/G columns; per-GPU HIP
    events on the context streams, the slowest GPU's span), both schedules; (2) host to
    host from a pinned arena (rsm_multi_extend_square_inplace on rsm_multi_host_alloc
    memory: Q0 rows up, Q1 rows and the bottom-half column slice down, one DMA each per
    GPU) and from pageable numpy memory (rsm_multi_extend_square); the pinned EDS is
    checked against the oracle at G = 1 and through the square's parity identity (every
    column of the result re-encodes to itself: Q3 from Q1 columns) otherwise."""
    import ctypes
    import numpy as np
    W = 2 * k
    steps = max(3, min(steps, 10))
    m = ctypes.c_void_p()
    devs = (ctypes.c_int * G)(*range(G))
    R._check(L.rsm_multi_create(devs, G, ctypes.byref(m)))
    out = {"workload": f"c5 through the C ABI: one process, {G} GPU(s), RCCL clique (ncclCommInitAll)",
           "n_gpus": G}
    try:
        ctxs = [L.rsm_multi_context(m, g) for g in range(G)]
        bufs = []
        for g in range(G):
            p = ctypes.c_void_p()
            R._check(L.rsm_dev_alloc(ctxs[g], W * W * S, ctypes.byref(p)))
            R._check(L.rsm_dev_fill_random(ctxs[g], p, W * W * S, 0xC5C5 + g))
            bufs.append(p.value)
        arr = (ctypes.c_void_p * G)(*bufs)
        ev = [[ctypes.c_void_p(), ctypes.c_void_p()] for _ in range(G)]
        for g in range(G):
            for e in ev[g]:
                R._check(L.rsm_event_create(ctxs[g], ctypes.byref(e)))
        for name, sched in (("allgather", 0), ("alltoall", 1)):
            R._check(L.rsm_multi_extend_dev(m, arr, k, S, sched))  # warm (RCCL connections)
            R._check(L.rsm_multi_sync(m))
            t0 = time.perf_counter()
            for g in range(G):
                R._check(L.rsm_event_record(ctxs[g], ev[g][0], None))
            for _ in range(steps):
                R._check(L.rsm_multi_extend_dev(m, arr, k, S, sched))
            for g in range(G):
                R._check(L.rsm_event_record(ctxs[g], ev[g][1], None))
            R._check(L.rsm_multi_sync(m))
            wall = (time.perf_counter() - t0) / steps
            spans = []
            ms = ctypes.c_float()
            for g in range(G):
                R._check(L.rsm_event_elapsed_ms(ev[g][0], ev[g][1], ctypes.byref(ms)))
                spans.append(ms.value / steps)
            dt = max(spans) / 1e3
            out[f"dev_{name}_ms_per_square"] = round(dt * 1e3, 4)
            out[f"dev_{name}_ods_GiB_s"] = round(k * k * S / dt / 2**30, 3)
            out[f"dev_{name}_host_wall_ms"] = round(wall * 1e3, 4)
        for g in range(G):
            for e in ev[g]:
                L.rsm_event_destroy(e)
            R._check(L.rsm_dev_free(ctxs[g], ctypes.c_void_p(bufs[g])))
        # host to host: pinned in place, then pageable
        import oracle
        ods = oracle.splitmix64_bytes(k * k * S, seed=0xC5).reshape(k, k, S)
        hp = ctypes.c_void_p()
        R._check(L.rsm_multi_host_alloc(m, W * W * S, ctypes.byref(hp)))
        try:
            eds = np.ctypeslib.as_array((ctypes.c_uint8 * (W * W * S)).from_address(hp.value)).reshape(W, W, S)
            eds[:k, :k] = ods
            R._check(L.rsm_multi_extend_square_inplace(m, hp, k, S, 1))
            if G == 1:
                ok = np.array_equal(eds, oracle.extend_square(ods, nthreads=16))
            else:
                # rows of the result re-encode to themselves (an independent check of Q1 and,
                # with the column identity below, of Q2/Q3) -- the oracle's whole square
                # takes ~1 s of host CPU per 16 threads, spent once at G = 1
                def reenc(v):  # the parity half the oracle's Encode gives for the first half of v
                    return np.frombuffer(b"".join(oracle.encode(list(v[:k]))), np.uint8).reshape(k, S)
                ok = all(np.array_equal(reenc(eds[r]), eds[r, k:]) for r in (0, k - 1, k, W - 1)) and \
                    all(np.array_equal(reenc(eds[:, c]), eds[k:, c]) for c in (0, W - 1))
            if not ok:
                raise SystemExit("bench c5 c_abi: pinned in-place EDS differs from the oracle")
            t0 = time.perf_counter()
            for _ in range(3):
                R._check(L.rsm_multi_extend_square_inplace(m, hp, k, S, 1))
            pinned = (time.perf_counter() - t0) / 3
        finally:
            R._check(L.rsm_multi_host_free(m, hp))
        e2 = np.empty((W, W, S), np.uint8)
        R._check(L.rsm_multi_extend_square(m, ods.ctypes.data, k, S, e2.ctypes.data, 1))
        t0 = time.perf_counter()
        for _ in range(3):
            R._check(L.rsm_multi_extend_square(m, ods.ctypes.data, k, S, e2.ctypes.data, 1))
        pageable = (time.perf_counter() - t0) / 3
        pcie = k * k * S + 3 * k * k * S
        out["pinned_host_ms_per_square"] = round(pinned * 1e3, 3)
        out["pinned_host_pcie_GB_s"] = round(pcie / pinned / 1e9, 2)
        out["pageable_host_ms_per_square"] = round(pageable * 1e3, 3)
        out["pcie_bytes_per_square"] = pcie
        out["note"] = ("dev_* = rsm_multi_extend_dev (device-resident, slowest GPU's event span); pinned = "
                       "rsm_multi_extend_square_inplace on an rsm_multi_host_alloc arena (all-to-all schedule; Q0 up, "
                       "Q1..Q3 down: pcie_bytes over all GPUs' links); pageable = rsm_multi_extend_square")
    finally:
        L.rsm_multi_destroy(m)
    return out


def bench_c5_g8_projection(ctx, buf, L, R, k, S, G=8, reps=20, device=0):
    """One rank's compute at G = 8 GPUs, timed on this one GPU (the
    row-sharded schedule of rsm_multi_extend_dev, extendeddatasquare.go:204-207):
    rsm_extend_rows_blocks_dev of k/G Q0 rows (the row pass of one shard, writing the
    all-to-all send blocks itself: no pack pass) and rsm_extend_cols_dev of 2k/G columns
    (its column slice after the exchange), device events around `reps` back-to-back calls
    each; the plain row pass (rsm_extend_rows_dev) is timed beside it.  The exchange is NOT measured (no
    multi-GPU node here): its bytes per GPU are reported, and `exchange_est_ms` prices
    them at the 7 xGMI links' 153 GB/s peak each (a lower bound on the exchange)."""
    import ctypes
    W = 2 * k
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    R._check(L.rsm_event_create(ctx, ctypes.byref(e0)))
    R._check(L.rsm_event_create(ctx, ctypes.byref(e1)))
    ms = ctypes.c_float()
    times = {}
    send = R.DeviceBuffer((k // G) * W * S, device)
    try:
        for name, fn in (("rows", lambda: L.rsm_extend_rows_blocks_dev(ctx, buf.ptr, k, S, 0, k // G, send.ptr, G,
                                                                        None)),
                         ("rows_plain", lambda: L.rsm_extend_rows_dev(ctx, buf.ptr, k, S, 0, k // G, None)),
                         ("cols", lambda: L.rsm_extend_cols_dev(ctx, buf.ptr, k, S, 0, W // G, None))):
            R._check(fn())
            R._check(L.rsm_event_record(ctx, e0, None))
            for _ in range(reps):
                R._check(fn())
            R._check(L.rsm_event_record(ctx, e1, None))
            R._check(L.rsm_sync(ctx))
            R._check(L.rsm_event_elapsed_ms(e0, e1, ctypes.byref(ms)))
            times[name] = ms.value / reps
    finally:
        L.rsm_event_destroy(e0)
        L.rsm_event_destroy(e1)
        send.free()
    ag = (G - 1) * (k // G) * W * S     # all-gather of the top half: received per GPU
    a2a = (G - 1) * (k // G) * (W // G) * S  # all-to-all of column blocks: received per GPU
    link = 7 * 153e9
    comp = times["rows"] + times["cols"]
    return {"label": "projection, exchange not measured: one rank's compute at G = 8 on one GPU",
            "rows_ms": round(times["rows"], 4), "rows_plain_ms": round(times["rows_plain"], 4), "rows": k // G, "row_tasks": (k // G) * ((S + 255) // 256),
            "cols_ms": round(times["cols"], 4), "cols": W // G,
            "compute_ms": round(comp, 4),
            "allgather_received_bytes_per_gpu": ag, "alltoall_received_bytes_per_gpu": a2a,
            "exchange_est_ms": {"allgather": round(ag / link * 1e3, 4), "alltoall": round(a2a / link * 1e3, 4)},
            "projected_ms_per_square": {"allgather": round(comp + ag / link * 1e3, 4),
                                        "alltoall": round(comp + a2a / link * 1e3, 4)},
            "projected_ods_GiB_s_alltoall": round(k * k * S / ((comp + a2a / link * 1e3) / 1e3) / 2**30, 1)}


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
        for _ in range(3):  # warm-up squares (clocks ramp up after the bench's earlier lines)
            R._check(L.rsm_extend_squares_dev(ctx, buf.ptr, k, S, 1, None))
        R._check(L.rsm_sync(ctx))
        reps = max(3, min(4 * steps, 40))  # ~18 ms of back-to-back squares: steadier than 10
        t0 = time.perf_counter()
        for _ in range(reps):
            R._check(L.rsm_extend_squares_dev(ctx, buf.ptr, k, S, 1, None))
        R._check(L.rsm_sync(ctx))
        dt = (time.perf_counter() - t0) / reps
        g8 = bench_c5_g8_projection(ctx, buf, L, R, k, S, device=local)
        buf.free()
        # the C-ABI multi-GPU entry point with a clique of one
        multi = bench_c5_c_abi(1, L, R, steps)
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
        torch.cuda.synchronize()
        # the C-ABI path a cgo caller uses (one process drives every GPU): rank 0 runs it
        # over all `world` GPUs while the other ranks wait at a CPU (gloo) barrier, so no
        # collective of theirs occupies the GPUs meanwhile
        cpu_group = dist.new_group(backend="gloo")
        c_abi = None
        if rank == 0:
            try:
                if torch.cuda.device_count() < world:
                    c_abi = {"error": f"rank 0 sees {torch.cuda.device_count()} of the {world} GPUs "
                                      "(HIP_VISIBLE_DEVICES): the one-process clique cannot be formed"}
                else:
                    c_abi = bench_c5_c_abi(world, L, R, steps)
            except Exception as e:  # noqa: BLE001 -- reported in the line, the headline stands
                c_abi = {"error": f"{type(e).__name__}: {e}"}
        dist.barrier(group=cpu_group)
    out = {"workload": "c5: 512x512->1024x1024 square, 512 B shares, GF(2^16)"
                       + ("" if world == 1 else f", rows sharded over {world} GPUs + RCCL all-to-all of column slices"),
           "n_gpus": world, "ms_per_square": round(dt * 1e3, 4), "ods_GiB_s": round(k * k * S / dt / 2**30, 3),
           "scaling": "strong (one square)",
           "frac": round(4 * k * k * S / dt / 1e9 / HBM_PEAK_GBS, 4)}
    if world == 1:
        tr = gf16_square_traffic("enc16h512_kernel")
        if tr:
            out["traffic"] = tr
    if dist is None:
        out["c_abi"] = multi
        out["g8_projection"] = g8
    if dist is not None:
        if rank == 0:
            out["c_abi"] = c_abi
        out["received_bytes_per_gpu"] = (world - 1) * (k // world) * (W // world) * S
        out["allgather_ms_per_square"] = round(dt_ag * 1e3, 4)
        out["allgather_received_bytes_per_gpu"] = (world - 1) * (k // world) * W * S
    return out


def bench_c3(local, L, R, repeats=5, k=128, S=512):
    """Config 3: k=128, S=512, exactly k of the 2k cells of every
    row erased (BenchmarkRepair's scheme, extendeddatacrossword_test.go:443-453),
    honest DefaultTree roots; also run at k = 256 and 512 (GF(2^16), BenchmarkRepair's
    larger ODS sizes).  Two timings:
      decode_sweep -- the device decode of all 2k rows alone (rsm_decode_vectors_dev
                      over a device-resident EDS + presence mask, HIP-synchronised);
      repair       -- (*ExtendedDataSquare).Repair end to end as BenchmarkRepair
                      times it (import untimed): zero-copy decode sweeps over
                      PCIe (present cells up, rebuilt cells back), column
                      re-encode check, DefaultTree roots of every row/col (on
                      the device).
    Replicas only: Repair is not sharded."""
    import ctypes
    import numpy as np
    W = 2 * k
    ctx = R.device_context(local)
    rng = np.random.default_rng(0xC3 + k)
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
    n_sw = 50 if k <= 128 else 10
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
    return {"workload": f"{'c3: ' if k == 128 else ''}k={k}, S={S}, {k} of {W} cells erased in every row "
                        f"(BenchmarkRepair scheme, GF(2^{8 if k <= 128 else 16}))",
            "decode_sweep_us": round(t_sweep * 1e6, 2),
            "decode_sweep_GB_s": round(algo / t_sweep / 1e9, 1),
            "decode_sweep_frac": round(algo / t_sweep / 1e9 / HBM_PEAK_GBS, 4),
            "repair_ms": round(t_rep * 1e3, 3), "repair_samples": repeats,
            "repair_fast_path": int(stats.fast_path), "repair_sweeps": int(stats.sweeps),
            "note": "repair = rsm_eds_repair end to end on a host EDS (zero-copy decode sweeps: present cells "
                    "read over PCIe, rebuilt cells written back; device column re-encode check; device "
                    "DefaultTree roots of all 512 vectors); median of samples"}


def bench_single_square(local, L, R, k=128, S=512, reps=200):
    """What a cgo ComputeExtendedDataSquare of ONE square gets (extendeddatasquare.go:
    50-77) from device memory: rsm_extend_squares_dev with count = 1 -- the latency form
    (encode_gf8_split_kernel: rows + Q0 columns in one launch over every CU, Q1 columns
    in a second) -- launches back to back on one stream, so each one's device time is its
    latency.  Oracle-checked.  Beside it the queue-driven launch for the same square and
    a count sweep of both forms (where rsm_ctx_set_split_max's default comes from)."""
    import ctypes
    import numpy as np
    import oracle
    ctx = R.device_context(local)
    W = 2 * k
    buf = R.DeviceBuffer(W * W * S * 8, local)
    buf.fill_random(0x55)
    R._check(L.rsm_extend_squares_dev(ctx, buf.ptr, k, S, 1, None))
    R._check(L.rsm_sync(ctx))
    got = buf.download(W * W * S).reshape(W, W, S)
    if not np.array_equal(got, oracle.extend_square(got[:k, :k].copy(), nthreads=8)):
        raise SystemExit("bench single square: GPU EDS differs from the oracle")
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    R._check(L.rsm_event_create(ctx, ctypes.byref(e0)))
    R._check(L.rsm_event_create(ctx, ctypes.byref(e1)))

    def dev_us(count, n):
        R._check(L.rsm_extend_squares_dev(ctx, buf.ptr, k, S, count, None))  # warm
        R._check(L.rsm_event_record(ctx, e0, None))
        for _ in range(n):
            R._check(L.rsm_extend_squares_dev(ctx, buf.ptr, k, S, count, None))
        R._check(L.rsm_event_record(ctx, e1, None))
        ms = ctypes.c_float()
        R._check(L.rsm_event_elapsed_ms(e0, e1, ctypes.byref(ms)))
        return ms.value / n * 1e3

    t_dev = dev_us(1, reps) / 1e6
    prev = ctypes.c_int(0)
    R._check(L.rsm_ctx_set_split_max(ctx, 0, ctypes.byref(prev)))
    t_queue = dev_us(1, reps)
    sweep = {}
    for c in (2, 4, 8):
        R._check(L.rsm_ctx_set_split_max(ctx, 0, None))
        q = dev_us(c, 50)
        R._check(L.rsm_ctx_set_split_max(ctx, 8, None))
        sp = dev_us(c, 50)
        sweep[str(c)] = {"split_us": round(sp, 2), "queue_us": round(q, 2)}
    R._check(L.rsm_ctx_set_split_max(ctx, prev.value, None))
    lat = []
    for _ in range(50):  # host-observed: launch + completion of one square
        t0 = time.perf_counter()
        R._check(L.rsm_extend_squares_dev(ctx, buf.ptr, k, S, 1, None))
        R._check(L.rsm_sync(ctx))
        lat.append(time.perf_counter() - t0)
    for e in (e0, e1):
        L.rsm_event_destroy(e)
    buf.free()
    return {"workload": f"one k={k} S={S} square, device-resident (count = 1)",
            "single_square_us": round(t_dev * 1e6, 2), "host_observed_us_p50": round(pct(lat, 0.5) * 1e6, 1),
            "frac": round(4 * k * k * S / t_dev / 1e9 / HBM_PEAK_GBS, 4),
            "kernel": "encode_gf8_split16_kernel x 2 launches (latency form, 16 waves per task; batches: encode_gf8_split_kernel<8>)",
            "queue_form_us": round(t_queue, 2), "count_sweep_us": sweep,
            "note": "device time per launch of back-to-back launches on one stream; host_observed = "
                    "rsm_extend_squares_dev + rsm_sync round trip; queue_form = the single queue-driven "
                    "launch (rsm_ctx_set_split_max 0)"}


def bench_small_squares(local, L, R, S=512, ks=(4, 8, 16, 32, 64)):
    """BenchmarkExtensionEncoding's small squares (extendeddatasquare_test.go:279-302:
    k = 4 .. 64 at shareSize 512, GF(2^8) byte-table kernels): per k, one square per
    call (what a cgo ComputeExtendedDataSquare gets, device-resident: back-to-back calls
    on one stream, device time per call) and a batch of squares per call (1 GiB of EDS)
    as throughput.  Every k is oracle-checked first."""
    import ctypes
    import numpy as np
    import oracle
    ctx = R.device_context(local)
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    R._check(L.rsm_event_create(ctx, ctypes.byref(e0)))
    R._check(L.rsm_event_create(ctx, ctypes.byref(e1)))

    def dev_ms(ptr, k, count, n):
        R._check(L.rsm_extend_squares_dev(ctx, ptr, k, S, count, None))  # warm
        R._check(L.rsm_event_record(ctx, e0, None))
        for _ in range(n):
            R._check(L.rsm_extend_squares_dev(ctx, ptr, k, S, count, None))
        R._check(L.rsm_event_record(ctx, e1, None))
        ms = ctypes.c_float()
        R._check(L.rsm_event_elapsed_ms(e0, e1, ctypes.byref(ms)))
        return ms.value / n

    out = {}
    for k in ks:
        W = 2 * k
        sq = W * W * S
        B = max(1, (1 << 30) // sq)
        buf = R.DeviceBuffer(B * sq, local)
        buf.fill_random(0x5A + k)
        R._check(L.rsm_extend_squares_dev(ctx, buf.ptr, k, S, B, None))
        R._check(L.rsm_sync(ctx))
        for i in (0, B - 1):
            got = buf.download(sq, i * sq).reshape(W, W, S)
            if not np.array_equal(got, oracle.extend_square(got[:k, :k].copy(), nthreads=8)):
                raise SystemExit(f"bench small squares: GPU EDS (k={k}) differs from the oracle")
        one = dev_ms(buf.ptr, k, 1, 200)
        batch = dev_ms(buf.ptr, k, B, 10)
        buf.free()
        out[str(k)] = {"single_square_us": round(one * 1e3, 2), "batch_squares": B,
                       "batch_us_per_square": round(batch * 1e3 / B, 3),
                       "batch_ods_GiB_s": round(k * k * S * B / (batch / 1e3) / 2**30, 2),
                       "batch_frac": round(4 * k * k * S * B / (batch / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
    for e in (e0, e1):
        L.rsm_event_destroy(e)
    return {"workload": f"BenchmarkExtensionEncoding k = {', '.join(map(str, ks))} at S = {S} (GF(2^8))",
            "kernel": "single: encode_gf8_splitm_kernel<M, NW> latency form for k = 9..64 (two launches), "
                      "encode_gf8_kernel<M> row pass then column pass for k <= 8; batch (more than 64 squares): "
                      "encode_gf8_kernel<M>", "by_k": out,
            "note": "single = one square per rsm_extend_squares_dev (device time of back-to-back calls on one "
                    "stream); batch = 1 GiB of EDS per call; frac = 4 k^2 S per square / time / 8 TB/s"}


def gf16_square_traffic(kernel):
    """HBM bytes per square of the GF(2^16) encoder `kernel` (row + column launch) from the
    committed counter passes (profiles/r06r_gf16_enc_pmc.json: rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE over scripts/diag/run_gf16.py, one square per call: c4 for enc16h_kernel, c5
    for enc16h512_kernel), or None when the file lacks the kernel."""
    try:
        rows = json.load(open(os.path.join(ROOT, "profiles", "r06r_gf16_enc_pmc.json")))["launches"]
    except (OSError, ValueError, KeyError):
        return None
    t = [r["traffic_bytes"] for r in rows if f"::{kernel}<" in r["kernel"]]
    return {"traffic_bytes_per_square": round(sum(t)), "source": "profiles/r06r_gf16_enc_pmc.json"} if len(t) == 2 else None


def bench_c4(local, L, R, steps, B=2, k=256, S=2048):
    """Config 4: 256x256 -> 512x512 squares of 2048 B shares (GF(2^16), enc16h_kernel: m = 256),
    device-resident, B squares (1 GiB of EDS) per step, steps alternating over two
    buffers so no step finds its squares in the 256 MiB Infinity Cache.  With S = 512
    the same code times BenchmarkExtensionEncoding's own k = 256 shape
    (extendeddatasquare_test.go:282-305, shareSize 512; B = 8 squares = 1 GiB)."""
    import ctypes
    import numpy as np
    import oracle
    W = 2 * k
    sq = W * W * S
    ctx = R.device_context(local)
    bufs = [R.DeviceBuffer(B * sq, local) for _ in range(2)]
    for i, b in enumerate(bufs):
        b.fill_random(0xC4 + i)
    R._check(L.rsm_sync(ctx))
    for b in bufs:
        R._check(L.rsm_extend_squares_dev(ctx, b.ptr, k, S, B, None))
    R._check(L.rsm_sync(ctx))
    got = bufs[0].download(sq).reshape(W, W, S)
    if not np.array_equal(got, oracle.extend_square(got[:k, :k].copy(), nthreads=16)):
        raise SystemExit("bench c4: GPU EDS differs from the oracle")
    n = max(4, min(steps, 20))
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    R._check(L.rsm_event_create(ctx, ctypes.byref(e0)))
    R._check(L.rsm_event_create(ctx, ctypes.byref(e1)))
    R._check(L.rsm_event_record(ctx, e0, None))
    for i in range(n):
        R._check(L.rsm_extend_squares_dev(ctx, bufs[i % 2].ptr, k, S, B, None))
    R._check(L.rsm_event_record(ctx, e1, None))
    ms = ctypes.c_float()
    R._check(L.rsm_event_elapsed_ms(e0, e1, ctypes.byref(ms)))
    dt = ms.value / n / 1e3
    for e in (e0, e1):
        L.rsm_event_destroy(e)
    for b in bufs:
        b.free()
    algo = 4 * k * k * S * B
    tr = gf16_square_traffic("enc16h_kernel") if (k, S) == (256, 2048) else None
    return {**({"traffic": tr} if tr else {}),
            "workload": (f"{'c4: ' if (k, S) == (256, 2048) else ''}{k}x{k}->{W}x{W} squares, {S} B shares, "
                         "GF(2^16)"), "squares_per_step": B,
            "ms_per_square": round(dt / B * 1e3, 4), "ods_GiB_s": round(k * k * S * B / dt / 2**30, 3),
            "frac": round(algo / dt / 1e9 / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_square": 4 * k * k * S,
            "kernel": ("enc16h_kernel (m = 256, half-wave form)" if (1 << (k - 1).bit_length()) == 256
                       else f"enc16_kernel<{1 << (k - 1).bit_length()}>") + " (row pass, column pass)"}


def bench_eds_roots(local, L, R, S=512, ods_sizes=(32, 64, 128, 256, 512), reps=20, ns=29):
    """BenchmarkEDSRootsWithDefaultTree and BenchmarkEDSRootsWithErasuredNMT
    (datasquare_test.go:415-473): the 2W row and column roots of ONE square of width
    W = 2 * ods (64 .. 1024 shares of 512 B), no extension, from device memory --
    rsm_roots_dev / rsm_nmt_roots_dev back to back on one stream, device time per call.
    Synthetic square: random payload with namespaces non-decreasing along every row and
    column (big-endian cell index, as genRandSortedDS gives); row 0 and column W - 1 of
    each width checked against the host DefaultTree and oracle/nmt.py before timing."""
    import ctypes
    import numpy as np
    import oracle.nmt as onmt
    ctx = R.device_context(local)
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    R._check(L.rsm_event_create(ctx, ctypes.byref(e0)))
    R._check(L.rsm_event_create(ctx, ctypes.byref(e1)))

    def dev_us(call):
        call()  # warm
        R._check(L.rsm_event_record(ctx, e0, None))
        for _ in range(reps):
            call()
        R._check(L.rsm_event_record(ctx, e1, None))
        ms = ctypes.c_float()
        R._check(L.rsm_event_elapsed_ms(e0, e1, ctypes.byref(ms)))
        return ms.value * 1e3 / reps

    rng = np.random.default_rng(0xED5)
    by = {}
    for o in ods_sizes:
        W = 2 * o
        sq = rng.integers(0, 256, (W, W, S), dtype=np.uint8)
        idx = np.arange(W * W, dtype=np.uint64).reshape(W, W)
        for b in range(8):
            sq[:, :, ns - 1 - b] = ((idx >> np.uint64(8 * b)) & np.uint64(0xFF)).astype(np.uint8)
        sq[:, :, : ns - 8] = 0
        buf = R.DeviceBuffer(W * W * S, local)
        buf.upload(sq)
        RL = 2 * ns + 32
        droots = R.DeviceBuffer(2 * W * 32, local)
        nroots = R.DeviceBuffer(2 * W * RL, local)
        status = R.DeviceBuffer(2 * W * 4, local)
        p = R.NmtParams(ns, 1, o)
        default = lambda: R._check(L.rsm_roots_dev(ctx, buf.ptr, W, S, droots.ptr, None))
        nmt = lambda: R._check(L.rsm_nmt_roots_dev(ctx, buf.ptr, W, S, ctypes.byref(p), nroots.ptr, status.ptr, None))
        default()
        nmt()
        R._check(L.rsm_sync(ctx))
        gd = droots.download(2 * W * 32).reshape(2 * W, 32)
        gn = nroots.download(2 * W * RL).reshape(2 * W, RL)
        st = status.download(2 * W * 4).view(np.uint32)
        for axis, i in ((0, 0), (1, W - 1)):
            vec = [bytes(c) for c in (sq[i] if axis == 0 else sq[:, i])]
            if bytes(gd[axis * W + i]) != R._default_root(vec):
                raise SystemExit("bench eds roots: device DefaultTree root differs from the host tree")
            if bytes(gn[axis * W + i]) != onmt.erasured_root(vec, i, o, ns) or st.any():
                raise SystemExit("bench eds roots: device NMT root differs from the restatement")
        by[str(o)] = {"eds_width": W, "default_tree_us": round(dev_us(default), 1), "nmt_us": round(dev_us(nmt), 1)}
        for b in (buf, droots, nroots, status):
            b.free()
    return {"workload": "BenchmarkEDSRootsWithDefaultTree / WithErasuredNMT: the 2W roots of one square of "
                        f"{S} B shares, ODS width 32..512 (no extension)",
            "by_ods": by,
            "note": "device time per call of back-to-back rsm_roots_dev / rsm_nmt_roots_dev on one stream "
                    "(one leaf launch + one tree launch each; namespace 29 B, IgnoreMaxNamespace)"}


def bench_extension_with_roots(local, L, R, S=512, ks=(4, 8, 16, 32, 64, 128, 256, 512), reps=10):
    """BenchmarkExtensionWithRoots (extendeddatasquare_test.go:309-333): ONE square's
    extension and its DefaultTree row and column roots, from device memory
    (rsm_extend_squares_dev count = 1, then rsm_roots_dev), k = 4 .. 512 at 512 B shares
    (GF(2^16) past k = 128); device time per square of back-to-back pairs on one stream.
    The k = 16 square is checked against the oracle extension and the host DefaultTree."""
    import ctypes
    import numpy as np
    import oracle
    ctx = R.device_context(local)
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    R._check(L.rsm_event_create(ctx, ctypes.byref(e0)))
    R._check(L.rsm_event_create(ctx, ctypes.byref(e1)))
    by = {}
    for k in ks:
        W = 2 * k
        buf = R.DeviceBuffer(W * W * S, local)
        buf.fill_random(0xE5 + k)
        roots = R.DeviceBuffer(2 * W * 32, local)

        def pair():
            R._check(L.rsm_extend_squares_dev(ctx, buf.ptr, k, S, 1, None))
            R._check(L.rsm_roots_dev(ctx, buf.ptr, W, S, roots.ptr, None))

        pair()
        R._check(L.rsm_sync(ctx))
        if k == 16:
            got = buf.download(W * W * S).reshape(W, W, S)
            if not np.array_equal(got, oracle.extend_square(got[:k, :k].copy(), nthreads=8)):
                raise SystemExit("bench extension with roots: GPU EDS differs from the oracle")
            rr = roots.download(2 * W * 32).reshape(2 * W, 32)
            if bytes(rr[0]) != R._default_root([bytes(c) for c in got[0]]):
                raise SystemExit("bench extension with roots: device root differs from the host tree")
        R._check(L.rsm_event_record(ctx, e0, None))
        for _ in range(reps):
            pair()
        R._check(L.rsm_event_record(ctx, e1, None))
        ms = ctypes.c_float()
        R._check(L.rsm_event_elapsed_ms(e0, e1, ctypes.byref(ms)))
        by[str(k)] = round(ms.value * 1e3 / reps, 1)
        buf.free()
        roots.free()
    return {"workload": f"BenchmarkExtensionWithRoots: one square extended + DefaultTree roots, {S} B shares",
            "us_per_square_by_k": by,
            "note": "device time per (rsm_extend_squares_dev count=1 + rsm_roots_dev) of back-to-back pairs"}


def bench_nmt_roots(local, L, R, k, S, squares=32, reps=5, ns=29):
    """The same with Celestia's tree: extension + NMT row/column roots (celestiaorg/nmt
    v0.24.3 as rsmt2d's erasured wrappers push it: namespace 29 bytes, parity namespace
    0xFF.. outside Q0, IgnoreMaxNamespace) of `squares` squares, all on the
    device (rsm_extend_squares_dev for the batch + one rsm_nmt_roots_dev per square).
    Synthetic ODS: random payload, namespaces non-decreasing along every row and column
    (big-endian cell index), as a valid block has them; rsm_nmt_roots_squares_dev does
    the batch in one launch pair.  The first square's roots are checked against the host
    restatement (oracle/nmt.py) before timing."""
    import ctypes
    import numpy as np
    ctx = R.device_context(local)
    W = 2 * k
    sq = W * W * S
    rng = np.random.default_rng(0x4E4D54)
    ods = rng.integers(0, 256, (k, k, S), dtype=np.uint8)
    idx = np.arange(k * k, dtype=np.uint64).reshape(k, k)
    for b in range(8):  # namespace = cell index, big-endian in the last 8 of its ns bytes
        ods[:, :, ns - 1 - b] = ((idx >> np.uint64(8 * b)) & np.uint64(0xFF)).astype(np.uint8)
    ods[:, :, : ns - 8] = 0
    full = np.zeros((W, W, S), np.uint8)
    full[:k, :k] = ods
    buf = R.DeviceBuffer(squares * sq, local)
    for i in range(squares):
        buf.upload(full, i * sq)
    roots = R.DeviceBuffer(squares * 2 * W * (2 * ns + 32), local)
    status = R.DeviceBuffer(squares * 2 * W * 4, local)
    p = R.NmtParams(ns, 1, k)

    def nmt_roots():
        R._check(L.rsm_nmt_roots_squares_dev(ctx, buf.ptr, W, S, squares, ctypes.byref(p), roots.ptr, status.ptr, None))

    def run():
        R._check(L.rsm_extend_squares_dev(ctx, buf.ptr, k, S, squares, None))
        nmt_roots()

    run()
    R._check(L.rsm_sync(ctx))
    got = roots.download(2 * W * (2 * ns + 32)).reshape(2 * W, 2 * ns + 32)
    st = status.download(squares * 2 * W * 4).view(np.uint32)
    eds = buf.download(sq).reshape(W, W, S)
    import oracle.nmt as onmt
    for axis, i in ((0, 0), (1, W - 1)):
        vec = eds[i] if axis == 0 else eds[:, i]
        want = onmt.erasured_root([bytes(c) for c in vec], i, k, ns)
        if bytes(got[axis * W + i]) != want or st.any():
            raise SystemExit("bench nmt roots: device root differs from the restatement")
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    R._check(L.rsm_sync(ctx))
    dt = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    for _ in range(reps):
        nmt_roots()
    R._check(L.rsm_sync(ctx))
    dr = (time.perf_counter() - t0) / reps
    for b in (buf, roots, status):
        b.free()
    return {"workload": f"extension + NMT row/col roots (namespace {ns} B), k={k}, S={S}, {squares} squares per step",
            "ms_per_square": round(dt / squares * 1e3, 4), "ods_GiB_s": round(squares * k * k * S / dt / 2**30, 3),
            "roots_only_ms_per_square": round(dr / squares * 1e3, 4),
            "note": "rsm_nmt_roots_squares_dev: one leaf launch (ns||share per cell, shared by its row and column "
                    "tree) and one tree launch (min/max namespace nodes) for the batch; roots of square 0 checked "
                    "against oracle/nmt.py"}


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
    import ctypes
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
    # k = 128: one queue-driven launch per step (both passes; rsm_extend_squares_dev
    # takes it for batches of >= 2 squares) unless --two-launch
    single = k == 128 and not a.two_launch and not a.one_stream
    # k = 128: 512 squares (16 GiB of EDS) per launch -- the launch's start-up and tail
    # are paid once per 512 squares (7.90 us per square against 8.01 at 256, same box,
    # profiles/r04d_c2_variants_qab.jsonl)
    B = a.batch or (512 if single else max(1, (1 << 30) // sq_bytes))
    nstreams = 1 if a.one_stream else (a.streams or (3 if single else 2))
    L = R.library()
    ctx = R.device_context(local)

    # synthetic ODS: seeded uniform bytes (SplitMix64) generated on the device; each
    # square's top-left quadrant is its ODS (the other quadrants are overwritten).
    # Batches are used in rotation, so a step never finds the previous step's
    # squares in the 256 MiB Infinity Cache (rotate > 512 MiB).
    bufs = [R.DeviceBuffer(B * sq_bytes, local) for _ in range(max(2, a.buffers or nstreams))]
    for i, b in enumerate(bufs):
        b.fill_random(0x52534D543244 + 2 * rank + i)
    R._check(L.rsm_sync(ctx))
    buf = bufs[0]
    # GF(2^8): consecutive steps alternate between two streams (each step's row and
    # column passes stay ordered on its own stream), so one step's column-pass tail
    # overlaps the next step's row-pass prologue.  (Every stream owns its scratch.)
    streams = [None]
    if not a.one_stream:
        for _ in range(max(1, nstreams) - 1):
            s2 = ctypes.c_void_p()
            R._check(L.rsm_stream_create(ctx, ctypes.byref(s2)))
            streams.append(s2)
    row_grid = a.row_grid if (len(streams) > 1 and 64 < k <= 128 and not single) else 0
    prev_grid = ctypes.c_int()
    R._check(L.rsm_ctx_set_pass_grid(ctx, 0, row_grid, ctypes.byref(prev_grid)))

    def new_event():
        e = ctypes.c_void_p()
        R._check(L.rsm_event_create(ctx, ctypes.byref(e)))
        return e

    nstep = [0]

    def step(ev=None):
        i = nstep[0]
        nstep[0] += 1
        st, b = streams[i % len(streams)], bufs[i % len(bufs)].ptr
        if ev is None:
            if single:
                R._check(L.rsm_extend_squares_dev(ctx, b, k, S, B, st))
            else:  # the two launches (rsm_extend_squares_dev would take the queue path)
                R._check(L.rsm_extend_squares_phase_dev(ctx, b, k, S, B, 1, st))
                R._check(L.rsm_extend_squares_phase_dev(ctx, b, k, S, B, 2, st))
            return
        if single:
            # the production step: ONE launch (both passes), an event either side
            R._check(L.rsm_event_record(ctx, ev[0], st))
            R._check(L.rsm_extend_squares_dev(ctx, b, k, S, B, st))
            R._check(L.rsm_event_record(ctx, ev[2], st))
            return
        # the production step (two launches) with an event at each launch boundary
        R._check(L.rsm_event_record(ctx, ev[0], st))
        R._check(L.rsm_extend_squares_phase_dev(ctx, b, k, S, B, 1, st))
        R._check(L.rsm_event_record(ctx, ev[1], st))
        R._check(L.rsm_extend_squares_phase_dev(ctx, b, k, S, B, 2, st))
        R._check(L.rsm_event_record(ctx, ev[2], st))

    def sync_all():
        # every stream's stuck-wait report is checked at each sync point (rsm_sync covers
        # the context stream, rsm_stream_check the extra ones)
        R._check(L.rsm_sync(ctx))
        for st in streams[1:]:
            R._check(L.rsm_stream_check(ctx, st))

    # the first warmup step, then the correctness gate on its output (the oracle is the
    # checker only), then the remaining warmup steps: the timed steps follow warm steps
    # directly (a GPU left idle during the CPU-side gate drops its clocks)
    step()
    sync_all()
    if rank == 0:
        import oracle
        for j in sorted({0, B - 1}):  # first and last square of the batch
            got = buf.download(sq_bytes, j * sq_bytes).reshape(W, W, S)
            want = oracle.extend_square(got[:k, :k].copy(), nthreads=min(16, os.cpu_count() or 1))
            if not np.array_equal(got, want):
                raise SystemExit("bench: GPU EDS differs from oracle -- refusing to report")
    for _ in range(max(0, a.warmup - 1)):
        step()
    sync_all()

    def barrier():
        if dist is not None:
            dist.barrier()
            torch.cuda.synchronize()

    events = [[new_event() for _ in range(3)] for _ in range(a.steps)]
    barrier()
    sync_all()
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(events[i])
    sync_all()
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # per-launch durations of THIS timed run (events on the launch streams)
    rows, cols, spans = [], [], []
    ms = ctypes.c_float()
    # union of the timed launches on the device clock: from the first launch's start
    # event to the LATEST end event of any step (with several streams an earlier
    # launch on another stream can end after the last-enqueued one)
    union_s = 0.0
    for ev in events:
        R._check(L.rsm_event_elapsed_ms(events[0][0], ev[2], ctypes.byref(ms)))
        union_s = max(union_s, ms.value / 1e3)
    for ev in events:
        if not single:
            R._check(L.rsm_event_elapsed_ms(ev[0], ev[1], ctypes.byref(ms)))
            rows.append(ms.value / 1e3)
            R._check(L.rsm_event_elapsed_ms(ev[1], ev[2], ctypes.byref(ms)))
            cols.append(ms.value / 1e3)
        R._check(L.rsm_event_elapsed_ms(ev[0], ev[2], ctypes.byref(ms)))
        spans.append(ms.value / 1e3)
        for e in ev:
            L.rsm_event_destroy(e)
    t_row = sum(rows) / len(rows) if rows else 0.0
    t_col = sum(cols) / len(cols) if cols else 0.0
    t_span = sum(spans) / len(spans)
    # the same launches alone on one stream (no overlap with another step)
    r_ms, c_ms, s_ms = ctypes.c_float(), ctypes.c_float(), ctypes.c_float()
    R._check(L.rsm_time_extend(ctx, bufs[0].ptr, k, S, B, 10, ctypes.byref(r_ms), ctypes.byref(c_ms),
                               ctypes.byref(s_ms)))
    iso_single = None
    if single:
        e0, e1 = new_event(), new_event()
        R._check(L.rsm_event_record(ctx, e0, None))
        for _ in range(5):
            R._check(L.rsm_extend_squares_dev(ctx, bufs[0].ptr, k, S, B, None))
        R._check(L.rsm_event_record(ctx, e1, None))
        R._check(L.rsm_event_elapsed_ms(e0, e1, ctypes.byref(ms)))
        iso_single = ms.value / 5 / 1e3
        for e in (e0, e1):
            L.rsm_event_destroy(e)
    R._check(L.rsm_ctx_set_pass_grid(ctx, 0, prev_grid.value, None))

    ods_bytes = k * k * S
    total = world * B * a.steps * ods_bytes
    value = total / elapsed / 2**30
    ms_per_step = elapsed / a.steps * 1e3
    algo_step = 4 * ods_bytes * B  # read Q0 once, write Q1+Q2+Q3
    col_bytes = 4 * ods_bytes * B  # column pass: [Q0|Q1] in, [Q2|Q3] out
    row_bytes = 2 * ods_bytes * B  # row pass: Q0 in, Q1 out
    bitsliced = 64 < k <= 128
    kname = ("encode_gf8_bs128u_kernel" if bitsliced else "encode_gf8_kernel" if k <= 64
             else "enc16_kernel (GF(2^16) single pass)")
    col_dom = t_col >= t_row
    if single:
        # the step IS one launch of the dominant kernel; with 3 streams the launches
        # run concurrently (each on a share of the CUs), so the kernel's rate is the
        # algorithmic bytes of all timed launches over their union on the device clock
        dominant = ("extend_gf8_bs128s_kernel (one launch: both passes)", algo_step, union_s / a.steps)
    else:
        dominant = ((kname + " column pass", col_bytes, t_col) if col_dom else (kname + " row pass", row_bytes, t_row))
    ach = dominant[1] / dominant[2] / 1e9
    # HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC
    # passes (scripts/pmc_summary.py; FETCH_SIZE x2 gfx950 correction), matched by
    # kernel name (<MODE, PASS>: PASS 1 = column pass) -- null when no matching
    # profile exists (e.g. the multi-kernel GF(2^16) passes).
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if bitsliced and os.path.exists(pmc_path):
        if single:
            want = "extend_gf8_bs128s_kernel<"  # any mode (production: <16777216>, fixed lane offsets)
            sets = 3 * k * B * S // 2048
        else:
            want = "encode_gf8_bs128u_kernel<%d, %d>" % ((184, 1) if col_dom else (104, 0))
            sets = (W if col_dom else k) * B * S // 2048
        grid_threads = min(sets, 256) * 512  # persistent grid: one 512-thread workgroup per CU
        for row in json.load(open(pmc_path)).get("launches", []):
            # persistent launches of every batch size share one grid: accept the row
            # only if it is plausibly this batch (0.9x - 2x the algorithmic bytes)
            if want in row["kernel"] and row["grid_threads"] == grid_threads and \
                    0.9 <= row["traffic_bytes"] / dominant[1] <= 2.0:
                traffic = int(row["traffic_bytes"])
    us = lambda x: round(x * 1e6, 2)
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
                   "squares_per_step": B, "eds_bytes_per_step": B * sq_bytes, "buffers": len(bufs),
                   "parallelism": f"independent squares per GPU x{world}",
                   "schedule": "single-launch queue (both passes)" if single else "two-launch",
                   "streams": len(streams), "row_pass_grid": row_grid or None},
        "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel": dominant[0],
                     **({"union_us_per_launch": us(union_s / a.steps),
                         "concurrent_span_us": us(t_span)} if single else {"avg_launch_us": us(dominant[2])}),
                     "bytes_per_launch": dominant[1],
                     "source": (f"HIP events around every launch of the {a.steps} timed steps; {len(streams)} "
                                "concurrent launches share the CUs, so achieved = bytes of all timed launches / "
                                f"their union on the device clock ({us(union_s / a.steps)} us per launch)")
                     if single else f"HIP events around every launch of the {a.steps} timed steps"},
        "step_roofline": {"algorithmic_bytes": algo_step,
                          "achieved": round(algo_step / (elapsed / a.steps) / 1e9, 1),
                          "frac": round(algo_step / (elapsed / a.steps) / 1e9 / HBM_PEAK_GBS, 4),
                          **({} if single else {
                              "row_pass_us": {"mean": us(t_row), "p10": us(pct(rows, .1)), "p50": us(pct(rows, .5)),
                                              "p90": us(pct(rows, .9))},
                              "col_pass_us": {"mean": us(t_col), "p10": us(pct(cols, .1)), "p50": us(pct(cols, .5)),
                                              "p90": us(pct(cols, .9))}}),
                          "step_span_us": {"mean": us(t_span), "p10": us(pct(spans, .1)), "p50": us(pct(spans, .5)),
                                           "p90": us(pct(spans, .9))},
                          "isolated_one_stream_us": dict(
                              ({"single_launch": us(iso_single)} if single else {}),
                              two_launch_row=round(r_ms.value * 1e3, 2), two_launch_col=round(c_ms.value * 1e3, 2))},
    }
    if rank == 0 and world == 1:
        model, ncpu = cpu_info()
        out["host"] = {"cpu_model": model, "cpus": ncpu}
        if not a.no_extras:
            out["host_path"] = bench_host_path(local, L, R, k, S, squares=8 if k <= 128 else 2)
            if k <= 128:
                out["codec"] = bench_codec(local, L, R)
                out["fraud_proof"] = bench_fraud_proof(local, L, R)
        out["cpu_baseline"] = None if a.no_cpu_baseline else cpu_baseline(k, S, a.cpu_seconds)
        cb = out["cpu_baseline"]
        if cb:
            # GPU / CPU against the measured run capped to the job's CPU share (cb["value"]),
            # against the run on every CPU of the affinity mask, and against the linear
            # all-host-CPUs extrapolation of the single-thread rate
            cb["gpu_over_cpu"] = round(value / cb["value"], 2)
            if cb.get("affinity_threads_GiB_s"):
                cb["gpu_over_cpu_affinity_threads"] = round(value / cb["affinity_threads_GiB_s"], 2)
            cb["gpu_over_cpu_all_cores_estimate"] = round(value / cb["all_cores_estimate_GiB_s"], 2)
    if rank == 0 and world == 1 and not a.no_roots:
        out["with_roots"] = bench_roots(local, L, R, buf, k, S, B, a.steps)
        out["with_nmt_roots"] = bench_nmt_roots(local, L, R, k, S)
        out["eds_roots"] = bench_eds_roots(local, L, R)
        out["extension_with_roots"] = bench_extension_with_roots(local, L, R)
    for b in bufs:
        b.free()
    for st in streams[1:]:
        R._check(L.rsm_stream_destroy(ctx, st))
    if rank == 0 and world == 1 and k == 128 and not a.no_single:
        out["single_square"] = bench_single_square(local, L, R)
        out["small_squares"] = bench_small_squares(local, L, R)
        if not a.no_c4:
            out["c4"] = bench_c4(local, L, R, a.steps)
            # BenchmarkExtensionEncoding's k = 256 square at its shareSize 512 (GF(2^16))
            out["gf16_k256_s512"] = bench_c4(local, L, R, a.steps, B=8, k=256, S=512)
    if rank == 0 and world == 1 and not a.no_c3:
        out["c3"] = bench_c3(local, L, R)
        if not a.no_gf16_repair:
            out["repair_gf16"] = [bench_c3(local, L, R, repeats=3, k=kk) for kk in (256, 512)]
    if not a.no_c5:
        if world == 1:
            out["c5"] = bench_c5(world, rank, local, dist, a.steps, L, R)
        else:
            # N > 1: the c5 sub-line (strong scaling of one sharded square, RCCL exchange)
            # is measured after the headline; an error raised on every rank (the usual
            # failure of a collective) is reported in the line instead of losing the
            # headline measured above
            try:
                out["c5"] = bench_c5(world, rank, local, dist, a.steps, L, R)
            except Exception as e:  # noqa: BLE001
                out["c5"] = {"error": f"{type(e).__name__}: {e}"}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
