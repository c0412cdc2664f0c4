"""A short single-square workload for counter passes (the shape one cgo
ComputeExtendedDataSquare call sees, extendeddatasquare.go:50-77): N device-resident
extensions of ONE k = 128, S = 512 square (rsm_extend_squares_dev with count = 1: the
latency form, two launches of encode_gf8_split16_kernel; RUN_SINGLE_WAVES picks the
form in the diagnostic library).
usage: [RUN_SINGLE_WAVES=16,16] python3 scripts/diag/run_single.py [N]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import rsmt2d_amd as R  # noqa: E402


def main(n):
    waves = os.environ.get("RUN_SINGLE_WAVES")  # "a,b": the diagnostic library's split waves per launch
    if waves:
        import ctypes
        L = R.diag_library()
        h = ctypes.c_void_p()
        R._check_with(L, L.rsm_ctx_create(0, ctypes.byref(h)))
        ctx = h.value
        R._check_with(L, L.rsm_diag_set_split_waves(*[int(x) for x in waves.split(",")]))
    else:
        L = R.library()
        ctx = R.device_context(0)
    k, S = 128, 512
    W = 2 * k
    buf = R.DeviceBuffer(W * W * S)
    buf.fill_random(k)
    for _ in range(n):
        R._check_with(L, L.rsm_extend_squares_dev(ctx, buf.ptr, k, S, 1, None))
    R._check_with(L, L.rsm_sync(ctx))
    buf.free()
    print("ok")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
