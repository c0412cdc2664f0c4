"""GF(2^16) encoder A/B (diagnostic library): device time per c5 square (k = 512,
S = 512) with the m = 512 encoder forms of rsm_diag_set_enc16_e64 (the list is in
include/rsmt2d_hip_diag.h); every output is checked against the first form's.  One JSON line
per configuration.  GF16AB_FORMS (comma list) picks the m = 512 forms, GF16AB_REPS the
repetitions, GF16AB_C4=0 skips the c4 part, GF16AB_C4FORMS its forms (single-form runs under rocprofv3 --pmc).
usage: python3 scripts/diag/gf16_ab.py"""
import ctypes
import json
import os
import sys

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
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    chk(D.rsm_event_create(ctx, ctypes.byref(e0)))
    chk(D.rsm_event_create(ctx, ctypes.byref(e1)))
    k, S = 512, 512
    n = (2 * k) ** 2 * S
    p = ctypes.c_void_p()
    chk(D.rsm_dev_alloc(ctx, n, ctypes.byref(p)))
    outs = {}
    forms = [int(f) for f in os.environ.get("GF16AB_FORMS", "2,4,0").split(",")]
    base = forms[0]
    for rep in range(int(os.environ.get("GF16AB_REPS", "2"))):
        for e64 in forms:
            chk(D.rsm_diag_set_enc16_e64(e64))
            chk(D.rsm_dev_fill_random(ctx, p.value, n, 7))
            chk(D.rsm_extend_squares_dev(ctx, p.value, k, S, 1, None))
            chk(D.rsm_sync(ctx))
            out = np.empty(n, np.uint8)
            chk(D.rsm_memcpy(ctx, out.ctypes.data, p.value, n, 1))
            outs[e64] = out
            reps = 20
            chk(D.rsm_event_record(ctx, e0, None))
            for _ in range(reps):
                chk(D.rsm_extend_squares_dev(ctx, p.value, k, S, 1, None))
            chk(D.rsm_event_record(ctx, e1, None))
            chk(D.rsm_sync(ctx))
            ms = ctypes.c_float()
            chk(D.rsm_event_elapsed_ms(e0, e1, ctypes.byref(ms)))
            print(json.dumps({"form": e64, "rep": rep, "c5_ms_per_square": round(ms.value / reps, 4),
                              f"same_as_form{base}": bool(np.array_equal(outs[e64], outs[base]))}), flush=True)
    chk(D.rsm_diag_set_enc16_e64(0))
    if os.environ.get("GF16AB_C4", "1") == "0":
        return
    # c4 (k = 256, S = 2048, 2 squares per step): m = 256 as 16 waves x 16 elements
    # (production since round 4, form 0) or 8 x 32 (form 7)
    k, S, B = 256, 2048, 2
    n = (2 * k) ** 2 * S * B
    q = ctypes.c_void_p()
    chk(D.rsm_dev_alloc(ctx, n, ctypes.byref(q)))
    outs = {}
    c4forms = [int(f) for f in os.environ.get("GF16AB_C4FORMS", "7,0").split(",")]
    for rep in range(2):
        for form in c4forms:
            chk(D.rsm_diag_set_enc16_e64(form))
            chk(D.rsm_dev_fill_random(ctx, q.value, n, 11))
            chk(D.rsm_extend_squares_dev(ctx, q.value, k, S, B, None))
            chk(D.rsm_sync(ctx))
            out = np.empty(n, np.uint8)
            chk(D.rsm_memcpy(ctx, out.ctypes.data, q.value, n, 1))
            outs[form] = out
            reps = 10
            chk(D.rsm_event_record(ctx, e0, None))
            for _ in range(reps):
                chk(D.rsm_extend_squares_dev(ctx, q.value, k, S, B, None))
            chk(D.rsm_event_record(ctx, e1, None))
            chk(D.rsm_sync(ctx))
            ms = ctypes.c_float()
            chk(D.rsm_event_elapsed_ms(e0, e1, ctypes.byref(ms)))
            t = ms.value / reps / B
            print(json.dumps({"c4_form": form, "rep": rep, "c4_ms_per_square": round(t, 4),
                              "frac": round(4 * k * k * S / (t / 1e3) / 8e12, 4),
                              f"same_as_form{c4forms[0]}": bool(np.array_equal(out, outs[c4forms[0]]))}), flush=True)
    chk(D.rsm_diag_set_enc16_e64(0))
    chk(D.rsm_dev_free(ctx, q))


if __name__ == "__main__":
    main()
