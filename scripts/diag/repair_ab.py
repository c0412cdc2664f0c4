"""Repair timing (diagnostic library): BenchmarkRepair's scheme (k of the 2k cells of every
row erased, extendeddatacrossword_test.go:443-453), S = 512, k = 128 / 256 / 512, repaired
through rsm_eds_repair (zero-copy sweeps); every repaired square is compared with the
original.  One JSON line per (k, rep).  The A/B lines in profiles/r05h_repair_transport_ab.jsonl
(split transport) and profiles/r05t_repair_concurrent_ab.jsonl (the halves on two lanes)
were taken with diagnostic modes of rsm_eds_repair that were removed once measured slower.
REPAB_KS picks the k values, REPAB_MODES the rsm_diag_set_repair_mode values (default 0).
usage: python3 scripts/diag/repair_ab.py"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import rsmt2d_amd as R  # noqa: E402

D = R.diag_library()


def chk(rc):
    R._check_with(D, rc)


def main():
    ctx = ctypes.c_void_p()
    chk(D.rsm_ctx_create(0, ctypes.byref(ctx)))
    for k in [int(x) for x in os.environ.get("REPAB_KS", "128,256,512").split(",")]:
        S, W = 512, 2 * k
        n = W * W * S
        buf = ctypes.c_void_p()
        chk(D.rsm_dev_alloc(ctx, n, ctypes.byref(buf)))
        chk(D.rsm_dev_fill_random(ctx, buf.value, n, 0xAB + k))
        chk(D.rsm_extend_squares_dev(ctx, buf.value, k, S, 1, None))
        chk(D.rsm_sync(ctx))
        full = np.empty((W, W, S), np.uint8)
        chk(D.rsm_memcpy(ctx, full.ctypes.data, buf.value, n, 1))
        chk(D.rsm_dev_free(ctx, buf))
        rng = np.random.default_rng(k)
        present = np.ones((W, W), np.uint8)
        for r in range(W):
            present[r, rng.choice(W, size=k, replace=False)] = 0
        base = full.ctypes.data
        ptrs = np.arange(W * W, dtype=np.uint64) * np.uint64(S) + np.uint64(base)
        lens = np.full(W * W, S, np.uint32)
        h = ctypes.c_void_p()
        chk(D.rsm_eds_import(ctx.value, ptrs.ctypes.data, lens.ctypes.data, W * W, ctypes.byref(h)))
        roots = {}
        for axis in (0, 1):
            out = np.empty(W * 32, np.uint8)
            rl = ctypes.c_uint32()
            chk(D.rsm_eds_roots(h, axis, None, None, out.ctypes.data, 32, ctypes.byref(rl)))
            roots[axis] = out
        D.rsm_eds_free(h)
        fptrs = ptrs.copy()
        fptrs[present.reshape(-1) == 0] = 0
        reps = int(os.environ.get("REPAB_REPS", "5"))
        for rep in range(2):
            for mode in [int(x) for x in os.environ.get("REPAB_MODES", "0").split(",")]:
                chk(D.rsm_diag_set_repair_mode(mode))
                times, fast, ok = [], 0, True
                for i in range(reps):
                    h = ctypes.c_void_p()
                    chk(D.rsm_eds_import(ctx.value, fptrs.ctypes.data, lens.ctypes.data, W * W, ctypes.byref(h)))
                    byz = R._Byz()
                    t0 = time.perf_counter()
                    chk(D.rsm_eds_repair(h, roots[0].ctypes.data, roots[1].ctypes.data, 32, None, None, ctypes.byref(byz)))
                    times.append(time.perf_counter() - t0)
                    st = R.RepairStats()
                    chk(D.rsm_eds_repair_stats(h, ctypes.byref(st)))
                    fast = st.fast_path
                    if i == 0:
                        got = np.empty_like(full)
                        chk(D.rsm_eds_flattened(h, got.ctypes.data, None))
                        ok = bool(np.array_equal(got, full))
                    D.rsm_eds_free(h)
                print(json.dumps({"k": k, "S": S, "mode": mode, "rep": rep,
                                  "repair_ms_p50": round(sorted(times)[len(times) // 2] * 1e3, 3),
                                  "repair_ms_min": round(min(times) * 1e3, 3), "fast_path": fast,
                                  "repaired_equal": ok}), flush=True)
    chk(D.rsm_diag_set_repair_mode(0))


if __name__ == "__main__":
    main()
