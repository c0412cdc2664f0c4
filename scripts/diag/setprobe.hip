// setprobe.hip -- diagnostic (NOT part of librsmt2d_hip.so): where the compute time of
// one bit-sliced M = 128 set goes.  One 8-wave workgroup per CU runs N iterations of a
// piece of the production set program on registers only (no global memory):
//   0: the whole set (16 transposes in, small IFFT, 8 exchange rounds, large
//      IFFT/FFT, 8 rounds back, small FFT, 16 transposes out)
//   1: butterflies only (small IFFT + large IFFT/FFT + small FFT)
//   2: transposes only (32)
//   3: LDS exchange only (16 rounds, 32 barriers)
//   4: large IFFT/FFT only
//   5/6: transposes, two symbols interleaved per asm block (masks in SGPRs / VGPRs)
//   7: exchange, two planes per round (ds_write_b64 / ds_read_b64, 64 KiB buffer)
//   8: exchange, one plane per step, double-buffered (reads of p + writes of p+1, one barrier)
//   9-14: 128 independent instructions of one kind per wave (per-instruction issue cost)
//   15: exchange, two planes per round, hand-written ds_write_b64 / ds_read_b64 (64 KiB)
// Usage: setprobe [iters]; prints one JSON line per variant (us per set per CU).
#include "../../rsmt2d_amd/csrc/kernels_gf8_bs.hip"
#include <cstdio>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

namespace rsm {
namespace {
__device__ __forceinline__ void transpose8x2_s(uint32_t (&w)[8], uint32_t (&u)[8]) {
    uint32_t t0, t1, t2, t3, t4, t5, t6, t7;
    asm volatile(
        "v_lshlrev_b32 %16, 4, %4\n\t"
        "v_lshlrev_b32 %20, 4, %12\n\t"
        "v_lshrrev_b32 %17, 4, %0\n\t"
        "v_lshrrev_b32 %21, 4, %8\n\t"
        "v_lshlrev_b32 %18, 4, %5\n\t"
        "v_lshlrev_b32 %22, 4, %13\n\t"
        "v_lshrrev_b32 %19, 4, %1\n\t"
        "v_lshrrev_b32 %23, 4, %9\n\t"
        "v_bfi_b32 %0, %25, %16, %0\n\t"
        "v_bfi_b32 %8, %25, %20, %8\n\t"
        "v_bfi_b32 %4, %24, %17, %4\n\t"
        "v_bfi_b32 %12, %24, %21, %12\n\t"
        "v_bfi_b32 %1, %25, %18, %1\n\t"
        "v_bfi_b32 %9, %25, %22, %9\n\t"
        "v_bfi_b32 %5, %24, %19, %5\n\t"
        "v_bfi_b32 %13, %24, %23, %13\n\t"
        "v_lshlrev_b32 %16, 4, %6\n\t"
        "v_lshlrev_b32 %20, 4, %14\n\t"
        "v_lshrrev_b32 %17, 4, %2\n\t"
        "v_lshrrev_b32 %21, 4, %10\n\t"
        "v_lshlrev_b32 %18, 4, %7\n\t"
        "v_lshlrev_b32 %22, 4, %15\n\t"
        "v_lshrrev_b32 %19, 4, %3\n\t"
        "v_lshrrev_b32 %23, 4, %11\n\t"
        "v_bfi_b32 %2, %25, %16, %2\n\t"
        "v_bfi_b32 %10, %25, %20, %10\n\t"
        "v_bfi_b32 %6, %24, %17, %6\n\t"
        "v_bfi_b32 %14, %24, %21, %14\n\t"
        "v_bfi_b32 %3, %25, %18, %3\n\t"
        "v_bfi_b32 %11, %25, %22, %11\n\t"
        "v_bfi_b32 %7, %24, %19, %7\n\t"
        "v_bfi_b32 %15, %24, %23, %15\n\t"
        "v_lshlrev_b32 %16, 2, %2\n\t"
        "v_lshlrev_b32 %20, 2, %10\n\t"
        "v_lshrrev_b32 %17, 2, %0\n\t"
        "v_lshrrev_b32 %21, 2, %8\n\t"
        "v_lshlrev_b32 %18, 2, %3\n\t"
        "v_lshlrev_b32 %22, 2, %11\n\t"
        "v_lshrrev_b32 %19, 2, %1\n\t"
        "v_lshrrev_b32 %23, 2, %9\n\t"
        "v_bfi_b32 %0, %27, %16, %0\n\t"
        "v_bfi_b32 %8, %27, %20, %8\n\t"
        "v_bfi_b32 %2, %26, %17, %2\n\t"
        "v_bfi_b32 %10, %26, %21, %10\n\t"
        "v_bfi_b32 %1, %27, %18, %1\n\t"
        "v_bfi_b32 %9, %27, %22, %9\n\t"
        "v_bfi_b32 %3, %26, %19, %3\n\t"
        "v_bfi_b32 %11, %26, %23, %11\n\t"
        "v_lshlrev_b32 %16, 2, %6\n\t"
        "v_lshlrev_b32 %20, 2, %14\n\t"
        "v_lshrrev_b32 %17, 2, %4\n\t"
        "v_lshrrev_b32 %21, 2, %12\n\t"
        "v_lshlrev_b32 %18, 2, %7\n\t"
        "v_lshlrev_b32 %22, 2, %15\n\t"
        "v_lshrrev_b32 %19, 2, %5\n\t"
        "v_lshrrev_b32 %23, 2, %13\n\t"
        "v_bfi_b32 %4, %27, %16, %4\n\t"
        "v_bfi_b32 %12, %27, %20, %12\n\t"
        "v_bfi_b32 %6, %26, %17, %6\n\t"
        "v_bfi_b32 %14, %26, %21, %14\n\t"
        "v_bfi_b32 %5, %27, %18, %5\n\t"
        "v_bfi_b32 %13, %27, %22, %13\n\t"
        "v_bfi_b32 %7, %26, %19, %7\n\t"
        "v_bfi_b32 %15, %26, %23, %15\n\t"
        "v_lshlrev_b32 %16, 1, %1\n\t"
        "v_lshlrev_b32 %20, 1, %9\n\t"
        "v_lshrrev_b32 %17, 1, %0\n\t"
        "v_lshrrev_b32 %21, 1, %8\n\t"
        "v_lshlrev_b32 %18, 1, %3\n\t"
        "v_lshlrev_b32 %22, 1, %11\n\t"
        "v_lshrrev_b32 %19, 1, %2\n\t"
        "v_lshrrev_b32 %23, 1, %10\n\t"
        "v_bfi_b32 %0, %29, %16, %0\n\t"
        "v_bfi_b32 %8, %29, %20, %8\n\t"
        "v_bfi_b32 %1, %28, %17, %1\n\t"
        "v_bfi_b32 %9, %28, %21, %9\n\t"
        "v_bfi_b32 %2, %29, %18, %2\n\t"
        "v_bfi_b32 %10, %29, %22, %10\n\t"
        "v_bfi_b32 %3, %28, %19, %3\n\t"
        "v_bfi_b32 %11, %28, %23, %11\n\t"
        "v_lshlrev_b32 %16, 1, %5\n\t"
        "v_lshlrev_b32 %20, 1, %13\n\t"
        "v_lshrrev_b32 %17, 1, %4\n\t"
        "v_lshrrev_b32 %21, 1, %12\n\t"
        "v_lshlrev_b32 %18, 1, %7\n\t"
        "v_lshlrev_b32 %22, 1, %15\n\t"
        "v_lshrrev_b32 %19, 1, %6\n\t"
        "v_lshrrev_b32 %23, 1, %14\n\t"
        "v_bfi_b32 %4, %29, %16, %4\n\t"
        "v_bfi_b32 %12, %29, %20, %12\n\t"
        "v_bfi_b32 %5, %28, %17, %5\n\t"
        "v_bfi_b32 %13, %28, %21, %13\n\t"
        "v_bfi_b32 %6, %29, %18, %6\n\t"
        "v_bfi_b32 %14, %29, %22, %14\n\t"
        "v_bfi_b32 %7, %28, %19, %7\n\t"
        "v_bfi_b32 %15, %28, %23, %15\n\t"
        : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]), "+v"(w[7]),
          "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5]), "+v"(u[6]), "+v"(u[7]),
          "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3), "=&v"(t4), "=&v"(t5), "=&v"(t6), "=&v"(t7)
        : "s"(0x0F0F0F0Fu), "s"(0xF0F0F0F0u), "s"(0x33333333u), "s"(0xCCCCCCCCu), "s"(0x55555555u),
          "s"(0xAAAAAAAAu));
}
__device__ __forceinline__ void transpose8x2_v(uint32_t (&w)[8], uint32_t (&u)[8]) {
    uint32_t t0, t1, t2, t3, t4, t5, t6, t7;
    asm volatile(
        "v_lshlrev_b32 %16, 4, %4\n\t"
        "v_lshlrev_b32 %20, 4, %12\n\t"
        "v_lshrrev_b32 %17, 4, %0\n\t"
        "v_lshrrev_b32 %21, 4, %8\n\t"
        "v_lshlrev_b32 %18, 4, %5\n\t"
        "v_lshlrev_b32 %22, 4, %13\n\t"
        "v_lshrrev_b32 %19, 4, %1\n\t"
        "v_lshrrev_b32 %23, 4, %9\n\t"
        "v_bfi_b32 %0, %25, %16, %0\n\t"
        "v_bfi_b32 %8, %25, %20, %8\n\t"
        "v_bfi_b32 %4, %24, %17, %4\n\t"
        "v_bfi_b32 %12, %24, %21, %12\n\t"
        "v_bfi_b32 %1, %25, %18, %1\n\t"
        "v_bfi_b32 %9, %25, %22, %9\n\t"
        "v_bfi_b32 %5, %24, %19, %5\n\t"
        "v_bfi_b32 %13, %24, %23, %13\n\t"
        "v_lshlrev_b32 %16, 4, %6\n\t"
        "v_lshlrev_b32 %20, 4, %14\n\t"
        "v_lshrrev_b32 %17, 4, %2\n\t"
        "v_lshrrev_b32 %21, 4, %10\n\t"
        "v_lshlrev_b32 %18, 4, %7\n\t"
        "v_lshlrev_b32 %22, 4, %15\n\t"
        "v_lshrrev_b32 %19, 4, %3\n\t"
        "v_lshrrev_b32 %23, 4, %11\n\t"
        "v_bfi_b32 %2, %25, %16, %2\n\t"
        "v_bfi_b32 %10, %25, %20, %10\n\t"
        "v_bfi_b32 %6, %24, %17, %6\n\t"
        "v_bfi_b32 %14, %24, %21, %14\n\t"
        "v_bfi_b32 %3, %25, %18, %3\n\t"
        "v_bfi_b32 %11, %25, %22, %11\n\t"
        "v_bfi_b32 %7, %24, %19, %7\n\t"
        "v_bfi_b32 %15, %24, %23, %15\n\t"
        "v_lshlrev_b32 %16, 2, %2\n\t"
        "v_lshlrev_b32 %20, 2, %10\n\t"
        "v_lshrrev_b32 %17, 2, %0\n\t"
        "v_lshrrev_b32 %21, 2, %8\n\t"
        "v_lshlrev_b32 %18, 2, %3\n\t"
        "v_lshlrev_b32 %22, 2, %11\n\t"
        "v_lshrrev_b32 %19, 2, %1\n\t"
        "v_lshrrev_b32 %23, 2, %9\n\t"
        "v_bfi_b32 %0, %27, %16, %0\n\t"
        "v_bfi_b32 %8, %27, %20, %8\n\t"
        "v_bfi_b32 %2, %26, %17, %2\n\t"
        "v_bfi_b32 %10, %26, %21, %10\n\t"
        "v_bfi_b32 %1, %27, %18, %1\n\t"
        "v_bfi_b32 %9, %27, %22, %9\n\t"
        "v_bfi_b32 %3, %26, %19, %3\n\t"
        "v_bfi_b32 %11, %26, %23, %11\n\t"
        "v_lshlrev_b32 %16, 2, %6\n\t"
        "v_lshlrev_b32 %20, 2, %14\n\t"
        "v_lshrrev_b32 %17, 2, %4\n\t"
        "v_lshrrev_b32 %21, 2, %12\n\t"
        "v_lshlrev_b32 %18, 2, %7\n\t"
        "v_lshlrev_b32 %22, 2, %15\n\t"
        "v_lshrrev_b32 %19, 2, %5\n\t"
        "v_lshrrev_b32 %23, 2, %13\n\t"
        "v_bfi_b32 %4, %27, %16, %4\n\t"
        "v_bfi_b32 %12, %27, %20, %12\n\t"
        "v_bfi_b32 %6, %26, %17, %6\n\t"
        "v_bfi_b32 %14, %26, %21, %14\n\t"
        "v_bfi_b32 %5, %27, %18, %5\n\t"
        "v_bfi_b32 %13, %27, %22, %13\n\t"
        "v_bfi_b32 %7, %26, %19, %7\n\t"
        "v_bfi_b32 %15, %26, %23, %15\n\t"
        "v_lshlrev_b32 %16, 1, %1\n\t"
        "v_lshlrev_b32 %20, 1, %9\n\t"
        "v_lshrrev_b32 %17, 1, %0\n\t"
        "v_lshrrev_b32 %21, 1, %8\n\t"
        "v_lshlrev_b32 %18, 1, %3\n\t"
        "v_lshlrev_b32 %22, 1, %11\n\t"
        "v_lshrrev_b32 %19, 1, %2\n\t"
        "v_lshrrev_b32 %23, 1, %10\n\t"
        "v_bfi_b32 %0, %29, %16, %0\n\t"
        "v_bfi_b32 %8, %29, %20, %8\n\t"
        "v_bfi_b32 %1, %28, %17, %1\n\t"
        "v_bfi_b32 %9, %28, %21, %9\n\t"
        "v_bfi_b32 %2, %29, %18, %2\n\t"
        "v_bfi_b32 %10, %29, %22, %10\n\t"
        "v_bfi_b32 %3, %28, %19, %3\n\t"
        "v_bfi_b32 %11, %28, %23, %11\n\t"
        "v_lshlrev_b32 %16, 1, %5\n\t"
        "v_lshlrev_b32 %20, 1, %13\n\t"
        "v_lshrrev_b32 %17, 1, %4\n\t"
        "v_lshrrev_b32 %21, 1, %12\n\t"
        "v_lshlrev_b32 %18, 1, %7\n\t"
        "v_lshlrev_b32 %22, 1, %15\n\t"
        "v_lshrrev_b32 %19, 1, %6\n\t"
        "v_lshrrev_b32 %23, 1, %14\n\t"
        "v_bfi_b32 %4, %29, %16, %4\n\t"
        "v_bfi_b32 %12, %29, %20, %12\n\t"
        "v_bfi_b32 %5, %28, %17, %5\n\t"
        "v_bfi_b32 %13, %28, %21, %13\n\t"
        "v_bfi_b32 %6, %29, %18, %6\n\t"
        "v_bfi_b32 %14, %29, %22, %14\n\t"
        "v_bfi_b32 %7, %28, %19, %7\n\t"
        "v_bfi_b32 %15, %28, %23, %15\n\t"
        : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]), "+v"(w[7]),
          "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5]), "+v"(u[6]), "+v"(u[7]),
          "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3), "=&v"(t4), "=&v"(t5), "=&v"(t6), "=&v"(t7)
        : "v"(0x0F0F0F0Fu), "v"(0xF0F0F0F0u), "v"(0x33333333u), "v"(0xCCCCCCCCu), "v"(0x55555555u),
          "v"(0xAAAAAAAAu));
}

__device__ __forceinline__ void alu_lshl(uint32_t (&X)[16][8]) {
    asm volatile(
        "v_lshlrev_b32 %0, 4, %5\n\t"
        "v_lshlrev_b32 %1, 4, %6\n\t"
        "v_lshlrev_b32 %2, 4, %7\n\t"
        "v_lshlrev_b32 %3, 4, %8\n\t"
        "v_lshlrev_b32 %4, 4, %9\n\t"
        "v_lshlrev_b32 %5, 4, %10\n\t"
        "v_lshlrev_b32 %6, 4, %11\n\t"
        "v_lshlrev_b32 %7, 4, %12\n\t"
        "v_lshlrev_b32 %8, 4, %13\n\t"
        "v_lshlrev_b32 %9, 4, %14\n\t"
        "v_lshlrev_b32 %10, 4, %15\n\t"
        "v_lshlrev_b32 %11, 4, %0\n\t"
        "v_lshlrev_b32 %12, 4, %1\n\t"
        "v_lshlrev_b32 %13, 4, %2\n\t"
        "v_lshlrev_b32 %14, 4, %3\n\t"
        "v_lshlrev_b32 %15, 4, %4\n\t"
        "v_lshlrev_b32 %0, 4, %5\n\t"
        "v_lshlrev_b32 %1, 4, %6\n\t"
        "v_lshlrev_b32 %2, 4, %7\n\t"
        "v_lshlrev_b32 %3, 4, %8\n\t"
        "v_lshlrev_b32 %4, 4, %9\n\t"
        "v_lshlrev_b32 %5, 4, %10\n\t"
        "v_lshlrev_b32 %6, 4, %11\n\t"
        "v_lshlrev_b32 %7, 4, %12\n\t"
        "v_lshlrev_b32 %8, 4, %13\n\t"
        "v_lshlrev_b32 %9, 4, %14\n\t"
        "v_lshlrev_b32 %10, 4, %15\n\t"
        "v_lshlrev_b32 %11, 4, %0\n\t"
        "v_lshlrev_b32 %12, 4, %1\n\t"
        "v_lshlrev_b32 %13, 4, %2\n\t"
        "v_lshlrev_b32 %14, 4, %3\n\t"
        "v_lshlrev_b32 %15, 4, %4\n\t"
        "v_lshlrev_b32 %0, 4, %5\n\t"
        "v_lshlrev_b32 %1, 4, %6\n\t"
        "v_lshlrev_b32 %2, 4, %7\n\t"
        "v_lshlrev_b32 %3, 4, %8\n\t"
        "v_lshlrev_b32 %4, 4, %9\n\t"
        "v_lshlrev_b32 %5, 4, %10\n\t"
        "v_lshlrev_b32 %6, 4, %11\n\t"
        "v_lshlrev_b32 %7, 4, %12\n\t"
        "v_lshlrev_b32 %8, 4, %13\n\t"
        "v_lshlrev_b32 %9, 4, %14\n\t"
        "v_lshlrev_b32 %10, 4, %15\n\t"
        "v_lshlrev_b32 %11, 4, %0\n\t"
        "v_lshlrev_b32 %12, 4, %1\n\t"
        "v_lshlrev_b32 %13, 4, %2\n\t"
        "v_lshlrev_b32 %14, 4, %3\n\t"
        "v_lshlrev_b32 %15, 4, %4\n\t"
        "v_lshlrev_b32 %0, 4, %5\n\t"
        "v_lshlrev_b32 %1, 4, %6\n\t"
        "v_lshlrev_b32 %2, 4, %7\n\t"
        "v_lshlrev_b32 %3, 4, %8\n\t"
        "v_lshlrev_b32 %4, 4, %9\n\t"
        "v_lshlrev_b32 %5, 4, %10\n\t"
        "v_lshlrev_b32 %6, 4, %11\n\t"
        "v_lshlrev_b32 %7, 4, %12\n\t"
        "v_lshlrev_b32 %8, 4, %13\n\t"
        "v_lshlrev_b32 %9, 4, %14\n\t"
        "v_lshlrev_b32 %10, 4, %15\n\t"
        "v_lshlrev_b32 %11, 4, %0\n\t"
        "v_lshlrev_b32 %12, 4, %1\n\t"
        "v_lshlrev_b32 %13, 4, %2\n\t"
        "v_lshlrev_b32 %14, 4, %3\n\t"
        "v_lshlrev_b32 %15, 4, %4\n\t"
        "v_lshlrev_b32 %0, 4, %5\n\t"
        "v_lshlrev_b32 %1, 4, %6\n\t"
        "v_lshlrev_b32 %2, 4, %7\n\t"
        "v_lshlrev_b32 %3, 4, %8\n\t"
        "v_lshlrev_b32 %4, 4, %9\n\t"
        "v_lshlrev_b32 %5, 4, %10\n\t"
        "v_lshlrev_b32 %6, 4, %11\n\t"
        "v_lshlrev_b32 %7, 4, %12\n\t"
        "v_lshlrev_b32 %8, 4, %13\n\t"
        "v_lshlrev_b32 %9, 4, %14\n\t"
        "v_lshlrev_b32 %10, 4, %15\n\t"
        "v_lshlrev_b32 %11, 4, %0\n\t"
        "v_lshlrev_b32 %12, 4, %1\n\t"
        "v_lshlrev_b32 %13, 4, %2\n\t"
        "v_lshlrev_b32 %14, 4, %3\n\t"
        "v_lshlrev_b32 %15, 4, %4\n\t"
        "v_lshlrev_b32 %0, 4, %5\n\t"
        "v_lshlrev_b32 %1, 4, %6\n\t"
        "v_lshlrev_b32 %2, 4, %7\n\t"
        "v_lshlrev_b32 %3, 4, %8\n\t"
        "v_lshlrev_b32 %4, 4, %9\n\t"
        "v_lshlrev_b32 %5, 4, %10\n\t"
        "v_lshlrev_b32 %6, 4, %11\n\t"
        "v_lshlrev_b32 %7, 4, %12\n\t"
        "v_lshlrev_b32 %8, 4, %13\n\t"
        "v_lshlrev_b32 %9, 4, %14\n\t"
        "v_lshlrev_b32 %10, 4, %15\n\t"
        "v_lshlrev_b32 %11, 4, %0\n\t"
        "v_lshlrev_b32 %12, 4, %1\n\t"
        "v_lshlrev_b32 %13, 4, %2\n\t"
        "v_lshlrev_b32 %14, 4, %3\n\t"
        "v_lshlrev_b32 %15, 4, %4\n\t"
        "v_lshlrev_b32 %0, 4, %5\n\t"
        "v_lshlrev_b32 %1, 4, %6\n\t"
        "v_lshlrev_b32 %2, 4, %7\n\t"
        "v_lshlrev_b32 %3, 4, %8\n\t"
        "v_lshlrev_b32 %4, 4, %9\n\t"
        "v_lshlrev_b32 %5, 4, %10\n\t"
        "v_lshlrev_b32 %6, 4, %11\n\t"
        "v_lshlrev_b32 %7, 4, %12\n\t"
        "v_lshlrev_b32 %8, 4, %13\n\t"
        "v_lshlrev_b32 %9, 4, %14\n\t"
        "v_lshlrev_b32 %10, 4, %15\n\t"
        "v_lshlrev_b32 %11, 4, %0\n\t"
        "v_lshlrev_b32 %12, 4, %1\n\t"
        "v_lshlrev_b32 %13, 4, %2\n\t"
        "v_lshlrev_b32 %14, 4, %3\n\t"
        "v_lshlrev_b32 %15, 4, %4\n\t"
        "v_lshlrev_b32 %0, 4, %5\n\t"
        "v_lshlrev_b32 %1, 4, %6\n\t"
        "v_lshlrev_b32 %2, 4, %7\n\t"
        "v_lshlrev_b32 %3, 4, %8\n\t"
        "v_lshlrev_b32 %4, 4, %9\n\t"
        "v_lshlrev_b32 %5, 4, %10\n\t"
        "v_lshlrev_b32 %6, 4, %11\n\t"
        "v_lshlrev_b32 %7, 4, %12\n\t"
        "v_lshlrev_b32 %8, 4, %13\n\t"
        "v_lshlrev_b32 %9, 4, %14\n\t"
        "v_lshlrev_b32 %10, 4, %15\n\t"
        "v_lshlrev_b32 %11, 4, %0\n\t"
        "v_lshlrev_b32 %12, 4, %1\n\t"
        "v_lshlrev_b32 %13, 4, %2\n\t"
        "v_lshlrev_b32 %14, 4, %3\n\t"
        "v_lshlrev_b32 %15, 4, %4\n\t"
        : "+v"(X[0][0]), "+v"(X[0][1]), "+v"(X[0][2]), "+v"(X[0][3]), "+v"(X[0][4]), "+v"(X[0][5]), "+v"(X[0][6]), "+v"(X[0][7]), "+v"(X[1][0]), "+v"(X[1][1]), "+v"(X[1][2]), "+v"(X[1][3]), "+v"(X[1][4]), "+v"(X[1][5]), "+v"(X[1][6]), "+v"(X[1][7])
        : "s"(0x0F0F0F0Fu));
}
__device__ __forceinline__ void alu_bfi(uint32_t (&X)[16][8]) {
    asm volatile(
        "v_bfi_b32 %0, %16, %5, %0\n\t"
        "v_bfi_b32 %1, %16, %6, %1\n\t"
        "v_bfi_b32 %2, %16, %7, %2\n\t"
        "v_bfi_b32 %3, %16, %8, %3\n\t"
        "v_bfi_b32 %4, %16, %9, %4\n\t"
        "v_bfi_b32 %5, %16, %10, %5\n\t"
        "v_bfi_b32 %6, %16, %11, %6\n\t"
        "v_bfi_b32 %7, %16, %12, %7\n\t"
        "v_bfi_b32 %8, %16, %13, %8\n\t"
        "v_bfi_b32 %9, %16, %14, %9\n\t"
        "v_bfi_b32 %10, %16, %15, %10\n\t"
        "v_bfi_b32 %11, %16, %0, %11\n\t"
        "v_bfi_b32 %12, %16, %1, %12\n\t"
        "v_bfi_b32 %13, %16, %2, %13\n\t"
        "v_bfi_b32 %14, %16, %3, %14\n\t"
        "v_bfi_b32 %15, %16, %4, %15\n\t"
        "v_bfi_b32 %0, %16, %5, %0\n\t"
        "v_bfi_b32 %1, %16, %6, %1\n\t"
        "v_bfi_b32 %2, %16, %7, %2\n\t"
        "v_bfi_b32 %3, %16, %8, %3\n\t"
        "v_bfi_b32 %4, %16, %9, %4\n\t"
        "v_bfi_b32 %5, %16, %10, %5\n\t"
        "v_bfi_b32 %6, %16, %11, %6\n\t"
        "v_bfi_b32 %7, %16, %12, %7\n\t"
        "v_bfi_b32 %8, %16, %13, %8\n\t"
        "v_bfi_b32 %9, %16, %14, %9\n\t"
        "v_bfi_b32 %10, %16, %15, %10\n\t"
        "v_bfi_b32 %11, %16, %0, %11\n\t"
        "v_bfi_b32 %12, %16, %1, %12\n\t"
        "v_bfi_b32 %13, %16, %2, %13\n\t"
        "v_bfi_b32 %14, %16, %3, %14\n\t"
        "v_bfi_b32 %15, %16, %4, %15\n\t"
        "v_bfi_b32 %0, %16, %5, %0\n\t"
        "v_bfi_b32 %1, %16, %6, %1\n\t"
        "v_bfi_b32 %2, %16, %7, %2\n\t"
        "v_bfi_b32 %3, %16, %8, %3\n\t"
        "v_bfi_b32 %4, %16, %9, %4\n\t"
        "v_bfi_b32 %5, %16, %10, %5\n\t"
        "v_bfi_b32 %6, %16, %11, %6\n\t"
        "v_bfi_b32 %7, %16, %12, %7\n\t"
        "v_bfi_b32 %8, %16, %13, %8\n\t"
        "v_bfi_b32 %9, %16, %14, %9\n\t"
        "v_bfi_b32 %10, %16, %15, %10\n\t"
        "v_bfi_b32 %11, %16, %0, %11\n\t"
        "v_bfi_b32 %12, %16, %1, %12\n\t"
        "v_bfi_b32 %13, %16, %2, %13\n\t"
        "v_bfi_b32 %14, %16, %3, %14\n\t"
        "v_bfi_b32 %15, %16, %4, %15\n\t"
        "v_bfi_b32 %0, %16, %5, %0\n\t"
        "v_bfi_b32 %1, %16, %6, %1\n\t"
        "v_bfi_b32 %2, %16, %7, %2\n\t"
        "v_bfi_b32 %3, %16, %8, %3\n\t"
        "v_bfi_b32 %4, %16, %9, %4\n\t"
        "v_bfi_b32 %5, %16, %10, %5\n\t"
        "v_bfi_b32 %6, %16, %11, %6\n\t"
        "v_bfi_b32 %7, %16, %12, %7\n\t"
        "v_bfi_b32 %8, %16, %13, %8\n\t"
        "v_bfi_b32 %9, %16, %14, %9\n\t"
        "v_bfi_b32 %10, %16, %15, %10\n\t"
        "v_bfi_b32 %11, %16, %0, %11\n\t"
        "v_bfi_b32 %12, %16, %1, %12\n\t"
        "v_bfi_b32 %13, %16, %2, %13\n\t"
        "v_bfi_b32 %14, %16, %3, %14\n\t"
        "v_bfi_b32 %15, %16, %4, %15\n\t"
        "v_bfi_b32 %0, %16, %5, %0\n\t"
        "v_bfi_b32 %1, %16, %6, %1\n\t"
        "v_bfi_b32 %2, %16, %7, %2\n\t"
        "v_bfi_b32 %3, %16, %8, %3\n\t"
        "v_bfi_b32 %4, %16, %9, %4\n\t"
        "v_bfi_b32 %5, %16, %10, %5\n\t"
        "v_bfi_b32 %6, %16, %11, %6\n\t"
        "v_bfi_b32 %7, %16, %12, %7\n\t"
        "v_bfi_b32 %8, %16, %13, %8\n\t"
        "v_bfi_b32 %9, %16, %14, %9\n\t"
        "v_bfi_b32 %10, %16, %15, %10\n\t"
        "v_bfi_b32 %11, %16, %0, %11\n\t"
        "v_bfi_b32 %12, %16, %1, %12\n\t"
        "v_bfi_b32 %13, %16, %2, %13\n\t"
        "v_bfi_b32 %14, %16, %3, %14\n\t"
        "v_bfi_b32 %15, %16, %4, %15\n\t"
        "v_bfi_b32 %0, %16, %5, %0\n\t"
        "v_bfi_b32 %1, %16, %6, %1\n\t"
        "v_bfi_b32 %2, %16, %7, %2\n\t"
        "v_bfi_b32 %3, %16, %8, %3\n\t"
        "v_bfi_b32 %4, %16, %9, %4\n\t"
        "v_bfi_b32 %5, %16, %10, %5\n\t"
        "v_bfi_b32 %6, %16, %11, %6\n\t"
        "v_bfi_b32 %7, %16, %12, %7\n\t"
        "v_bfi_b32 %8, %16, %13, %8\n\t"
        "v_bfi_b32 %9, %16, %14, %9\n\t"
        "v_bfi_b32 %10, %16, %15, %10\n\t"
        "v_bfi_b32 %11, %16, %0, %11\n\t"
        "v_bfi_b32 %12, %16, %1, %12\n\t"
        "v_bfi_b32 %13, %16, %2, %13\n\t"
        "v_bfi_b32 %14, %16, %3, %14\n\t"
        "v_bfi_b32 %15, %16, %4, %15\n\t"
        "v_bfi_b32 %0, %16, %5, %0\n\t"
        "v_bfi_b32 %1, %16, %6, %1\n\t"
        "v_bfi_b32 %2, %16, %7, %2\n\t"
        "v_bfi_b32 %3, %16, %8, %3\n\t"
        "v_bfi_b32 %4, %16, %9, %4\n\t"
        "v_bfi_b32 %5, %16, %10, %5\n\t"
        "v_bfi_b32 %6, %16, %11, %6\n\t"
        "v_bfi_b32 %7, %16, %12, %7\n\t"
        "v_bfi_b32 %8, %16, %13, %8\n\t"
        "v_bfi_b32 %9, %16, %14, %9\n\t"
        "v_bfi_b32 %10, %16, %15, %10\n\t"
        "v_bfi_b32 %11, %16, %0, %11\n\t"
        "v_bfi_b32 %12, %16, %1, %12\n\t"
        "v_bfi_b32 %13, %16, %2, %13\n\t"
        "v_bfi_b32 %14, %16, %3, %14\n\t"
        "v_bfi_b32 %15, %16, %4, %15\n\t"
        "v_bfi_b32 %0, %16, %5, %0\n\t"
        "v_bfi_b32 %1, %16, %6, %1\n\t"
        "v_bfi_b32 %2, %16, %7, %2\n\t"
        "v_bfi_b32 %3, %16, %8, %3\n\t"
        "v_bfi_b32 %4, %16, %9, %4\n\t"
        "v_bfi_b32 %5, %16, %10, %5\n\t"
        "v_bfi_b32 %6, %16, %11, %6\n\t"
        "v_bfi_b32 %7, %16, %12, %7\n\t"
        "v_bfi_b32 %8, %16, %13, %8\n\t"
        "v_bfi_b32 %9, %16, %14, %9\n\t"
        "v_bfi_b32 %10, %16, %15, %10\n\t"
        "v_bfi_b32 %11, %16, %0, %11\n\t"
        "v_bfi_b32 %12, %16, %1, %12\n\t"
        "v_bfi_b32 %13, %16, %2, %13\n\t"
        "v_bfi_b32 %14, %16, %3, %14\n\t"
        "v_bfi_b32 %15, %16, %4, %15\n\t"
        : "+v"(X[0][0]), "+v"(X[0][1]), "+v"(X[0][2]), "+v"(X[0][3]), "+v"(X[0][4]), "+v"(X[0][5]), "+v"(X[0][6]), "+v"(X[0][7]), "+v"(X[1][0]), "+v"(X[1][1]), "+v"(X[1][2]), "+v"(X[1][3]), "+v"(X[1][4]), "+v"(X[1][5]), "+v"(X[1][6]), "+v"(X[1][7])
        : "s"(0x0F0F0F0Fu));
}
__device__ __forceinline__ void alu_bitop3(uint32_t (&X)[16][8]) {
    asm volatile(
        "v_bitop3_b32 %0, %0, %5, %11 bitop3:0x96\n\t"
        "v_bitop3_b32 %1, %1, %6, %12 bitop3:0x96\n\t"
        "v_bitop3_b32 %2, %2, %7, %13 bitop3:0x96\n\t"
        "v_bitop3_b32 %3, %3, %8, %14 bitop3:0x96\n\t"
        "v_bitop3_b32 %4, %4, %9, %15 bitop3:0x96\n\t"
        "v_bitop3_b32 %5, %5, %10, %0 bitop3:0x96\n\t"
        "v_bitop3_b32 %6, %6, %11, %1 bitop3:0x96\n\t"
        "v_bitop3_b32 %7, %7, %12, %2 bitop3:0x96\n\t"
        "v_bitop3_b32 %8, %8, %13, %3 bitop3:0x96\n\t"
        "v_bitop3_b32 %9, %9, %14, %4 bitop3:0x96\n\t"
        "v_bitop3_b32 %10, %10, %15, %5 bitop3:0x96\n\t"
        "v_bitop3_b32 %11, %11, %0, %6 bitop3:0x96\n\t"
        "v_bitop3_b32 %12, %12, %1, %7 bitop3:0x96\n\t"
        "v_bitop3_b32 %13, %13, %2, %8 bitop3:0x96\n\t"
        "v_bitop3_b32 %14, %14, %3, %9 bitop3:0x96\n\t"
        "v_bitop3_b32 %15, %15, %4, %10 bitop3:0x96\n\t"
        "v_bitop3_b32 %0, %0, %5, %11 bitop3:0x96\n\t"
        "v_bitop3_b32 %1, %1, %6, %12 bitop3:0x96\n\t"
        "v_bitop3_b32 %2, %2, %7, %13 bitop3:0x96\n\t"
        "v_bitop3_b32 %3, %3, %8, %14 bitop3:0x96\n\t"
        "v_bitop3_b32 %4, %4, %9, %15 bitop3:0x96\n\t"
        "v_bitop3_b32 %5, %5, %10, %0 bitop3:0x96\n\t"
        "v_bitop3_b32 %6, %6, %11, %1 bitop3:0x96\n\t"
        "v_bitop3_b32 %7, %7, %12, %2 bitop3:0x96\n\t"
        "v_bitop3_b32 %8, %8, %13, %3 bitop3:0x96\n\t"
        "v_bitop3_b32 %9, %9, %14, %4 bitop3:0x96\n\t"
        "v_bitop3_b32 %10, %10, %15, %5 bitop3:0x96\n\t"
        "v_bitop3_b32 %11, %11, %0, %6 bitop3:0x96\n\t"
        "v_bitop3_b32 %12, %12, %1, %7 bitop3:0x96\n\t"
        "v_bitop3_b32 %13, %13, %2, %8 bitop3:0x96\n\t"
        "v_bitop3_b32 %14, %14, %3, %9 bitop3:0x96\n\t"
        "v_bitop3_b32 %15, %15, %4, %10 bitop3:0x96\n\t"
        "v_bitop3_b32 %0, %0, %5, %11 bitop3:0x96\n\t"
        "v_bitop3_b32 %1, %1, %6, %12 bitop3:0x96\n\t"
        "v_bitop3_b32 %2, %2, %7, %13 bitop3:0x96\n\t"
        "v_bitop3_b32 %3, %3, %8, %14 bitop3:0x96\n\t"
        "v_bitop3_b32 %4, %4, %9, %15 bitop3:0x96\n\t"
        "v_bitop3_b32 %5, %5, %10, %0 bitop3:0x96\n\t"
        "v_bitop3_b32 %6, %6, %11, %1 bitop3:0x96\n\t"
        "v_bitop3_b32 %7, %7, %12, %2 bitop3:0x96\n\t"
        "v_bitop3_b32 %8, %8, %13, %3 bitop3:0x96\n\t"
        "v_bitop3_b32 %9, %9, %14, %4 bitop3:0x96\n\t"
        "v_bitop3_b32 %10, %10, %15, %5 bitop3:0x96\n\t"
        "v_bitop3_b32 %11, %11, %0, %6 bitop3:0x96\n\t"
        "v_bitop3_b32 %12, %12, %1, %7 bitop3:0x96\n\t"
        "v_bitop3_b32 %13, %13, %2, %8 bitop3:0x96\n\t"
        "v_bitop3_b32 %14, %14, %3, %9 bitop3:0x96\n\t"
        "v_bitop3_b32 %15, %15, %4, %10 bitop3:0x96\n\t"
        "v_bitop3_b32 %0, %0, %5, %11 bitop3:0x96\n\t"
        "v_bitop3_b32 %1, %1, %6, %12 bitop3:0x96\n\t"
        "v_bitop3_b32 %2, %2, %7, %13 bitop3:0x96\n\t"
        "v_bitop3_b32 %3, %3, %8, %14 bitop3:0x96\n\t"
        "v_bitop3_b32 %4, %4, %9, %15 bitop3:0x96\n\t"
        "v_bitop3_b32 %5, %5, %10, %0 bitop3:0x96\n\t"
        "v_bitop3_b32 %6, %6, %11, %1 bitop3:0x96\n\t"
        "v_bitop3_b32 %7, %7, %12, %2 bitop3:0x96\n\t"
        "v_bitop3_b32 %8, %8, %13, %3 bitop3:0x96\n\t"
        "v_bitop3_b32 %9, %9, %14, %4 bitop3:0x96\n\t"
        "v_bitop3_b32 %10, %10, %15, %5 bitop3:0x96\n\t"
        "v_bitop3_b32 %11, %11, %0, %6 bitop3:0x96\n\t"
        "v_bitop3_b32 %12, %12, %1, %7 bitop3:0x96\n\t"
        "v_bitop3_b32 %13, %13, %2, %8 bitop3:0x96\n\t"
        "v_bitop3_b32 %14, %14, %3, %9 bitop3:0x96\n\t"
        "v_bitop3_b32 %15, %15, %4, %10 bitop3:0x96\n\t"
        "v_bitop3_b32 %0, %0, %5, %11 bitop3:0x96\n\t"
        "v_bitop3_b32 %1, %1, %6, %12 bitop3:0x96\n\t"
        "v_bitop3_b32 %2, %2, %7, %13 bitop3:0x96\n\t"
        "v_bitop3_b32 %3, %3, %8, %14 bitop3:0x96\n\t"
        "v_bitop3_b32 %4, %4, %9, %15 bitop3:0x96\n\t"
        "v_bitop3_b32 %5, %5, %10, %0 bitop3:0x96\n\t"
        "v_bitop3_b32 %6, %6, %11, %1 bitop3:0x96\n\t"
        "v_bitop3_b32 %7, %7, %12, %2 bitop3:0x96\n\t"
        "v_bitop3_b32 %8, %8, %13, %3 bitop3:0x96\n\t"
        "v_bitop3_b32 %9, %9, %14, %4 bitop3:0x96\n\t"
        "v_bitop3_b32 %10, %10, %15, %5 bitop3:0x96\n\t"
        "v_bitop3_b32 %11, %11, %0, %6 bitop3:0x96\n\t"
        "v_bitop3_b32 %12, %12, %1, %7 bitop3:0x96\n\t"
        "v_bitop3_b32 %13, %13, %2, %8 bitop3:0x96\n\t"
        "v_bitop3_b32 %14, %14, %3, %9 bitop3:0x96\n\t"
        "v_bitop3_b32 %15, %15, %4, %10 bitop3:0x96\n\t"
        "v_bitop3_b32 %0, %0, %5, %11 bitop3:0x96\n\t"
        "v_bitop3_b32 %1, %1, %6, %12 bitop3:0x96\n\t"
        "v_bitop3_b32 %2, %2, %7, %13 bitop3:0x96\n\t"
        "v_bitop3_b32 %3, %3, %8, %14 bitop3:0x96\n\t"
        "v_bitop3_b32 %4, %4, %9, %15 bitop3:0x96\n\t"
        "v_bitop3_b32 %5, %5, %10, %0 bitop3:0x96\n\t"
        "v_bitop3_b32 %6, %6, %11, %1 bitop3:0x96\n\t"
        "v_bitop3_b32 %7, %7, %12, %2 bitop3:0x96\n\t"
        "v_bitop3_b32 %8, %8, %13, %3 bitop3:0x96\n\t"
        "v_bitop3_b32 %9, %9, %14, %4 bitop3:0x96\n\t"
        "v_bitop3_b32 %10, %10, %15, %5 bitop3:0x96\n\t"
        "v_bitop3_b32 %11, %11, %0, %6 bitop3:0x96\n\t"
        "v_bitop3_b32 %12, %12, %1, %7 bitop3:0x96\n\t"
        "v_bitop3_b32 %13, %13, %2, %8 bitop3:0x96\n\t"
        "v_bitop3_b32 %14, %14, %3, %9 bitop3:0x96\n\t"
        "v_bitop3_b32 %15, %15, %4, %10 bitop3:0x96\n\t"
        "v_bitop3_b32 %0, %0, %5, %11 bitop3:0x96\n\t"
        "v_bitop3_b32 %1, %1, %6, %12 bitop3:0x96\n\t"
        "v_bitop3_b32 %2, %2, %7, %13 bitop3:0x96\n\t"
        "v_bitop3_b32 %3, %3, %8, %14 bitop3:0x96\n\t"
        "v_bitop3_b32 %4, %4, %9, %15 bitop3:0x96\n\t"
        "v_bitop3_b32 %5, %5, %10, %0 bitop3:0x96\n\t"
        "v_bitop3_b32 %6, %6, %11, %1 bitop3:0x96\n\t"
        "v_bitop3_b32 %7, %7, %12, %2 bitop3:0x96\n\t"
        "v_bitop3_b32 %8, %8, %13, %3 bitop3:0x96\n\t"
        "v_bitop3_b32 %9, %9, %14, %4 bitop3:0x96\n\t"
        "v_bitop3_b32 %10, %10, %15, %5 bitop3:0x96\n\t"
        "v_bitop3_b32 %11, %11, %0, %6 bitop3:0x96\n\t"
        "v_bitop3_b32 %12, %12, %1, %7 bitop3:0x96\n\t"
        "v_bitop3_b32 %13, %13, %2, %8 bitop3:0x96\n\t"
        "v_bitop3_b32 %14, %14, %3, %9 bitop3:0x96\n\t"
        "v_bitop3_b32 %15, %15, %4, %10 bitop3:0x96\n\t"
        "v_bitop3_b32 %0, %0, %5, %11 bitop3:0x96\n\t"
        "v_bitop3_b32 %1, %1, %6, %12 bitop3:0x96\n\t"
        "v_bitop3_b32 %2, %2, %7, %13 bitop3:0x96\n\t"
        "v_bitop3_b32 %3, %3, %8, %14 bitop3:0x96\n\t"
        "v_bitop3_b32 %4, %4, %9, %15 bitop3:0x96\n\t"
        "v_bitop3_b32 %5, %5, %10, %0 bitop3:0x96\n\t"
        "v_bitop3_b32 %6, %6, %11, %1 bitop3:0x96\n\t"
        "v_bitop3_b32 %7, %7, %12, %2 bitop3:0x96\n\t"
        "v_bitop3_b32 %8, %8, %13, %3 bitop3:0x96\n\t"
        "v_bitop3_b32 %9, %9, %14, %4 bitop3:0x96\n\t"
        "v_bitop3_b32 %10, %10, %15, %5 bitop3:0x96\n\t"
        "v_bitop3_b32 %11, %11, %0, %6 bitop3:0x96\n\t"
        "v_bitop3_b32 %12, %12, %1, %7 bitop3:0x96\n\t"
        "v_bitop3_b32 %13, %13, %2, %8 bitop3:0x96\n\t"
        "v_bitop3_b32 %14, %14, %3, %9 bitop3:0x96\n\t"
        "v_bitop3_b32 %15, %15, %4, %10 bitop3:0x96\n\t"
        : "+v"(X[0][0]), "+v"(X[0][1]), "+v"(X[0][2]), "+v"(X[0][3]), "+v"(X[0][4]), "+v"(X[0][5]), "+v"(X[0][6]), "+v"(X[0][7]), "+v"(X[1][0]), "+v"(X[1][1]), "+v"(X[1][2]), "+v"(X[1][3]), "+v"(X[1][4]), "+v"(X[1][5]), "+v"(X[1][6]), "+v"(X[1][7])
        : "s"(0x0F0F0F0Fu));
}
__device__ __forceinline__ void alu_xor(uint32_t (&X)[16][8]) {
    asm volatile(
        "v_xor_b32 %0, %0, %5\n\t"
        "v_xor_b32 %1, %1, %6\n\t"
        "v_xor_b32 %2, %2, %7\n\t"
        "v_xor_b32 %3, %3, %8\n\t"
        "v_xor_b32 %4, %4, %9\n\t"
        "v_xor_b32 %5, %5, %10\n\t"
        "v_xor_b32 %6, %6, %11\n\t"
        "v_xor_b32 %7, %7, %12\n\t"
        "v_xor_b32 %8, %8, %13\n\t"
        "v_xor_b32 %9, %9, %14\n\t"
        "v_xor_b32 %10, %10, %15\n\t"
        "v_xor_b32 %11, %11, %0\n\t"
        "v_xor_b32 %12, %12, %1\n\t"
        "v_xor_b32 %13, %13, %2\n\t"
        "v_xor_b32 %14, %14, %3\n\t"
        "v_xor_b32 %15, %15, %4\n\t"
        "v_xor_b32 %0, %0, %5\n\t"
        "v_xor_b32 %1, %1, %6\n\t"
        "v_xor_b32 %2, %2, %7\n\t"
        "v_xor_b32 %3, %3, %8\n\t"
        "v_xor_b32 %4, %4, %9\n\t"
        "v_xor_b32 %5, %5, %10\n\t"
        "v_xor_b32 %6, %6, %11\n\t"
        "v_xor_b32 %7, %7, %12\n\t"
        "v_xor_b32 %8, %8, %13\n\t"
        "v_xor_b32 %9, %9, %14\n\t"
        "v_xor_b32 %10, %10, %15\n\t"
        "v_xor_b32 %11, %11, %0\n\t"
        "v_xor_b32 %12, %12, %1\n\t"
        "v_xor_b32 %13, %13, %2\n\t"
        "v_xor_b32 %14, %14, %3\n\t"
        "v_xor_b32 %15, %15, %4\n\t"
        "v_xor_b32 %0, %0, %5\n\t"
        "v_xor_b32 %1, %1, %6\n\t"
        "v_xor_b32 %2, %2, %7\n\t"
        "v_xor_b32 %3, %3, %8\n\t"
        "v_xor_b32 %4, %4, %9\n\t"
        "v_xor_b32 %5, %5, %10\n\t"
        "v_xor_b32 %6, %6, %11\n\t"
        "v_xor_b32 %7, %7, %12\n\t"
        "v_xor_b32 %8, %8, %13\n\t"
        "v_xor_b32 %9, %9, %14\n\t"
        "v_xor_b32 %10, %10, %15\n\t"
        "v_xor_b32 %11, %11, %0\n\t"
        "v_xor_b32 %12, %12, %1\n\t"
        "v_xor_b32 %13, %13, %2\n\t"
        "v_xor_b32 %14, %14, %3\n\t"
        "v_xor_b32 %15, %15, %4\n\t"
        "v_xor_b32 %0, %0, %5\n\t"
        "v_xor_b32 %1, %1, %6\n\t"
        "v_xor_b32 %2, %2, %7\n\t"
        "v_xor_b32 %3, %3, %8\n\t"
        "v_xor_b32 %4, %4, %9\n\t"
        "v_xor_b32 %5, %5, %10\n\t"
        "v_xor_b32 %6, %6, %11\n\t"
        "v_xor_b32 %7, %7, %12\n\t"
        "v_xor_b32 %8, %8, %13\n\t"
        "v_xor_b32 %9, %9, %14\n\t"
        "v_xor_b32 %10, %10, %15\n\t"
        "v_xor_b32 %11, %11, %0\n\t"
        "v_xor_b32 %12, %12, %1\n\t"
        "v_xor_b32 %13, %13, %2\n\t"
        "v_xor_b32 %14, %14, %3\n\t"
        "v_xor_b32 %15, %15, %4\n\t"
        "v_xor_b32 %0, %0, %5\n\t"
        "v_xor_b32 %1, %1, %6\n\t"
        "v_xor_b32 %2, %2, %7\n\t"
        "v_xor_b32 %3, %3, %8\n\t"
        "v_xor_b32 %4, %4, %9\n\t"
        "v_xor_b32 %5, %5, %10\n\t"
        "v_xor_b32 %6, %6, %11\n\t"
        "v_xor_b32 %7, %7, %12\n\t"
        "v_xor_b32 %8, %8, %13\n\t"
        "v_xor_b32 %9, %9, %14\n\t"
        "v_xor_b32 %10, %10, %15\n\t"
        "v_xor_b32 %11, %11, %0\n\t"
        "v_xor_b32 %12, %12, %1\n\t"
        "v_xor_b32 %13, %13, %2\n\t"
        "v_xor_b32 %14, %14, %3\n\t"
        "v_xor_b32 %15, %15, %4\n\t"
        "v_xor_b32 %0, %0, %5\n\t"
        "v_xor_b32 %1, %1, %6\n\t"
        "v_xor_b32 %2, %2, %7\n\t"
        "v_xor_b32 %3, %3, %8\n\t"
        "v_xor_b32 %4, %4, %9\n\t"
        "v_xor_b32 %5, %5, %10\n\t"
        "v_xor_b32 %6, %6, %11\n\t"
        "v_xor_b32 %7, %7, %12\n\t"
        "v_xor_b32 %8, %8, %13\n\t"
        "v_xor_b32 %9, %9, %14\n\t"
        "v_xor_b32 %10, %10, %15\n\t"
        "v_xor_b32 %11, %11, %0\n\t"
        "v_xor_b32 %12, %12, %1\n\t"
        "v_xor_b32 %13, %13, %2\n\t"
        "v_xor_b32 %14, %14, %3\n\t"
        "v_xor_b32 %15, %15, %4\n\t"
        "v_xor_b32 %0, %0, %5\n\t"
        "v_xor_b32 %1, %1, %6\n\t"
        "v_xor_b32 %2, %2, %7\n\t"
        "v_xor_b32 %3, %3, %8\n\t"
        "v_xor_b32 %4, %4, %9\n\t"
        "v_xor_b32 %5, %5, %10\n\t"
        "v_xor_b32 %6, %6, %11\n\t"
        "v_xor_b32 %7, %7, %12\n\t"
        "v_xor_b32 %8, %8, %13\n\t"
        "v_xor_b32 %9, %9, %14\n\t"
        "v_xor_b32 %10, %10, %15\n\t"
        "v_xor_b32 %11, %11, %0\n\t"
        "v_xor_b32 %12, %12, %1\n\t"
        "v_xor_b32 %13, %13, %2\n\t"
        "v_xor_b32 %14, %14, %3\n\t"
        "v_xor_b32 %15, %15, %4\n\t"
        "v_xor_b32 %0, %0, %5\n\t"
        "v_xor_b32 %1, %1, %6\n\t"
        "v_xor_b32 %2, %2, %7\n\t"
        "v_xor_b32 %3, %3, %8\n\t"
        "v_xor_b32 %4, %4, %9\n\t"
        "v_xor_b32 %5, %5, %10\n\t"
        "v_xor_b32 %6, %6, %11\n\t"
        "v_xor_b32 %7, %7, %12\n\t"
        "v_xor_b32 %8, %8, %13\n\t"
        "v_xor_b32 %9, %9, %14\n\t"
        "v_xor_b32 %10, %10, %15\n\t"
        "v_xor_b32 %11, %11, %0\n\t"
        "v_xor_b32 %12, %12, %1\n\t"
        "v_xor_b32 %13, %13, %2\n\t"
        "v_xor_b32 %14, %14, %3\n\t"
        "v_xor_b32 %15, %15, %4\n\t"
        : "+v"(X[0][0]), "+v"(X[0][1]), "+v"(X[0][2]), "+v"(X[0][3]), "+v"(X[0][4]), "+v"(X[0][5]), "+v"(X[0][6]), "+v"(X[0][7]), "+v"(X[1][0]), "+v"(X[1][1]), "+v"(X[1][2]), "+v"(X[1][3]), "+v"(X[1][4]), "+v"(X[1][5]), "+v"(X[1][6]), "+v"(X[1][7])
        : "s"(0x0F0F0F0Fu));
}
__device__ __forceinline__ void alu_perm(uint32_t (&X)[16][8]) {
    asm volatile(
        "v_perm_b32 %0, %5, %11, %16\n\t"
        "v_perm_b32 %1, %6, %12, %16\n\t"
        "v_perm_b32 %2, %7, %13, %16\n\t"
        "v_perm_b32 %3, %8, %14, %16\n\t"
        "v_perm_b32 %4, %9, %15, %16\n\t"
        "v_perm_b32 %5, %10, %0, %16\n\t"
        "v_perm_b32 %6, %11, %1, %16\n\t"
        "v_perm_b32 %7, %12, %2, %16\n\t"
        "v_perm_b32 %8, %13, %3, %16\n\t"
        "v_perm_b32 %9, %14, %4, %16\n\t"
        "v_perm_b32 %10, %15, %5, %16\n\t"
        "v_perm_b32 %11, %0, %6, %16\n\t"
        "v_perm_b32 %12, %1, %7, %16\n\t"
        "v_perm_b32 %13, %2, %8, %16\n\t"
        "v_perm_b32 %14, %3, %9, %16\n\t"
        "v_perm_b32 %15, %4, %10, %16\n\t"
        "v_perm_b32 %0, %5, %11, %16\n\t"
        "v_perm_b32 %1, %6, %12, %16\n\t"
        "v_perm_b32 %2, %7, %13, %16\n\t"
        "v_perm_b32 %3, %8, %14, %16\n\t"
        "v_perm_b32 %4, %9, %15, %16\n\t"
        "v_perm_b32 %5, %10, %0, %16\n\t"
        "v_perm_b32 %6, %11, %1, %16\n\t"
        "v_perm_b32 %7, %12, %2, %16\n\t"
        "v_perm_b32 %8, %13, %3, %16\n\t"
        "v_perm_b32 %9, %14, %4, %16\n\t"
        "v_perm_b32 %10, %15, %5, %16\n\t"
        "v_perm_b32 %11, %0, %6, %16\n\t"
        "v_perm_b32 %12, %1, %7, %16\n\t"
        "v_perm_b32 %13, %2, %8, %16\n\t"
        "v_perm_b32 %14, %3, %9, %16\n\t"
        "v_perm_b32 %15, %4, %10, %16\n\t"
        "v_perm_b32 %0, %5, %11, %16\n\t"
        "v_perm_b32 %1, %6, %12, %16\n\t"
        "v_perm_b32 %2, %7, %13, %16\n\t"
        "v_perm_b32 %3, %8, %14, %16\n\t"
        "v_perm_b32 %4, %9, %15, %16\n\t"
        "v_perm_b32 %5, %10, %0, %16\n\t"
        "v_perm_b32 %6, %11, %1, %16\n\t"
        "v_perm_b32 %7, %12, %2, %16\n\t"
        "v_perm_b32 %8, %13, %3, %16\n\t"
        "v_perm_b32 %9, %14, %4, %16\n\t"
        "v_perm_b32 %10, %15, %5, %16\n\t"
        "v_perm_b32 %11, %0, %6, %16\n\t"
        "v_perm_b32 %12, %1, %7, %16\n\t"
        "v_perm_b32 %13, %2, %8, %16\n\t"
        "v_perm_b32 %14, %3, %9, %16\n\t"
        "v_perm_b32 %15, %4, %10, %16\n\t"
        "v_perm_b32 %0, %5, %11, %16\n\t"
        "v_perm_b32 %1, %6, %12, %16\n\t"
        "v_perm_b32 %2, %7, %13, %16\n\t"
        "v_perm_b32 %3, %8, %14, %16\n\t"
        "v_perm_b32 %4, %9, %15, %16\n\t"
        "v_perm_b32 %5, %10, %0, %16\n\t"
        "v_perm_b32 %6, %11, %1, %16\n\t"
        "v_perm_b32 %7, %12, %2, %16\n\t"
        "v_perm_b32 %8, %13, %3, %16\n\t"
        "v_perm_b32 %9, %14, %4, %16\n\t"
        "v_perm_b32 %10, %15, %5, %16\n\t"
        "v_perm_b32 %11, %0, %6, %16\n\t"
        "v_perm_b32 %12, %1, %7, %16\n\t"
        "v_perm_b32 %13, %2, %8, %16\n\t"
        "v_perm_b32 %14, %3, %9, %16\n\t"
        "v_perm_b32 %15, %4, %10, %16\n\t"
        "v_perm_b32 %0, %5, %11, %16\n\t"
        "v_perm_b32 %1, %6, %12, %16\n\t"
        "v_perm_b32 %2, %7, %13, %16\n\t"
        "v_perm_b32 %3, %8, %14, %16\n\t"
        "v_perm_b32 %4, %9, %15, %16\n\t"
        "v_perm_b32 %5, %10, %0, %16\n\t"
        "v_perm_b32 %6, %11, %1, %16\n\t"
        "v_perm_b32 %7, %12, %2, %16\n\t"
        "v_perm_b32 %8, %13, %3, %16\n\t"
        "v_perm_b32 %9, %14, %4, %16\n\t"
        "v_perm_b32 %10, %15, %5, %16\n\t"
        "v_perm_b32 %11, %0, %6, %16\n\t"
        "v_perm_b32 %12, %1, %7, %16\n\t"
        "v_perm_b32 %13, %2, %8, %16\n\t"
        "v_perm_b32 %14, %3, %9, %16\n\t"
        "v_perm_b32 %15, %4, %10, %16\n\t"
        "v_perm_b32 %0, %5, %11, %16\n\t"
        "v_perm_b32 %1, %6, %12, %16\n\t"
        "v_perm_b32 %2, %7, %13, %16\n\t"
        "v_perm_b32 %3, %8, %14, %16\n\t"
        "v_perm_b32 %4, %9, %15, %16\n\t"
        "v_perm_b32 %5, %10, %0, %16\n\t"
        "v_perm_b32 %6, %11, %1, %16\n\t"
        "v_perm_b32 %7, %12, %2, %16\n\t"
        "v_perm_b32 %8, %13, %3, %16\n\t"
        "v_perm_b32 %9, %14, %4, %16\n\t"
        "v_perm_b32 %10, %15, %5, %16\n\t"
        "v_perm_b32 %11, %0, %6, %16\n\t"
        "v_perm_b32 %12, %1, %7, %16\n\t"
        "v_perm_b32 %13, %2, %8, %16\n\t"
        "v_perm_b32 %14, %3, %9, %16\n\t"
        "v_perm_b32 %15, %4, %10, %16\n\t"
        "v_perm_b32 %0, %5, %11, %16\n\t"
        "v_perm_b32 %1, %6, %12, %16\n\t"
        "v_perm_b32 %2, %7, %13, %16\n\t"
        "v_perm_b32 %3, %8, %14, %16\n\t"
        "v_perm_b32 %4, %9, %15, %16\n\t"
        "v_perm_b32 %5, %10, %0, %16\n\t"
        "v_perm_b32 %6, %11, %1, %16\n\t"
        "v_perm_b32 %7, %12, %2, %16\n\t"
        "v_perm_b32 %8, %13, %3, %16\n\t"
        "v_perm_b32 %9, %14, %4, %16\n\t"
        "v_perm_b32 %10, %15, %5, %16\n\t"
        "v_perm_b32 %11, %0, %6, %16\n\t"
        "v_perm_b32 %12, %1, %7, %16\n\t"
        "v_perm_b32 %13, %2, %8, %16\n\t"
        "v_perm_b32 %14, %3, %9, %16\n\t"
        "v_perm_b32 %15, %4, %10, %16\n\t"
        "v_perm_b32 %0, %5, %11, %16\n\t"
        "v_perm_b32 %1, %6, %12, %16\n\t"
        "v_perm_b32 %2, %7, %13, %16\n\t"
        "v_perm_b32 %3, %8, %14, %16\n\t"
        "v_perm_b32 %4, %9, %15, %16\n\t"
        "v_perm_b32 %5, %10, %0, %16\n\t"
        "v_perm_b32 %6, %11, %1, %16\n\t"
        "v_perm_b32 %7, %12, %2, %16\n\t"
        "v_perm_b32 %8, %13, %3, %16\n\t"
        "v_perm_b32 %9, %14, %4, %16\n\t"
        "v_perm_b32 %10, %15, %5, %16\n\t"
        "v_perm_b32 %11, %0, %6, %16\n\t"
        "v_perm_b32 %12, %1, %7, %16\n\t"
        "v_perm_b32 %13, %2, %8, %16\n\t"
        "v_perm_b32 %14, %3, %9, %16\n\t"
        "v_perm_b32 %15, %4, %10, %16\n\t"
        : "+v"(X[0][0]), "+v"(X[0][1]), "+v"(X[0][2]), "+v"(X[0][3]), "+v"(X[0][4]), "+v"(X[0][5]), "+v"(X[0][6]), "+v"(X[0][7]), "+v"(X[1][0]), "+v"(X[1][1]), "+v"(X[1][2]), "+v"(X[1][3]), "+v"(X[1][4]), "+v"(X[1][5]), "+v"(X[1][6]), "+v"(X[1][7])
        : "s"(0x0F0F0F0Fu));
}
__device__ __forceinline__ void alu_bfiv(uint32_t (&X)[16][8]) {
    asm volatile(
        "v_bfi_b32 %0, %11, %5, %0\n\t"
        "v_bfi_b32 %1, %12, %6, %1\n\t"
        "v_bfi_b32 %2, %13, %7, %2\n\t"
        "v_bfi_b32 %3, %14, %8, %3\n\t"
        "v_bfi_b32 %4, %15, %9, %4\n\t"
        "v_bfi_b32 %5, %0, %10, %5\n\t"
        "v_bfi_b32 %6, %1, %11, %6\n\t"
        "v_bfi_b32 %7, %2, %12, %7\n\t"
        "v_bfi_b32 %8, %3, %13, %8\n\t"
        "v_bfi_b32 %9, %4, %14, %9\n\t"
        "v_bfi_b32 %10, %5, %15, %10\n\t"
        "v_bfi_b32 %11, %6, %0, %11\n\t"
        "v_bfi_b32 %12, %7, %1, %12\n\t"
        "v_bfi_b32 %13, %8, %2, %13\n\t"
        "v_bfi_b32 %14, %9, %3, %14\n\t"
        "v_bfi_b32 %15, %10, %4, %15\n\t"
        "v_bfi_b32 %0, %11, %5, %0\n\t"
        "v_bfi_b32 %1, %12, %6, %1\n\t"
        "v_bfi_b32 %2, %13, %7, %2\n\t"
        "v_bfi_b32 %3, %14, %8, %3\n\t"
        "v_bfi_b32 %4, %15, %9, %4\n\t"
        "v_bfi_b32 %5, %0, %10, %5\n\t"
        "v_bfi_b32 %6, %1, %11, %6\n\t"
        "v_bfi_b32 %7, %2, %12, %7\n\t"
        "v_bfi_b32 %8, %3, %13, %8\n\t"
        "v_bfi_b32 %9, %4, %14, %9\n\t"
        "v_bfi_b32 %10, %5, %15, %10\n\t"
        "v_bfi_b32 %11, %6, %0, %11\n\t"
        "v_bfi_b32 %12, %7, %1, %12\n\t"
        "v_bfi_b32 %13, %8, %2, %13\n\t"
        "v_bfi_b32 %14, %9, %3, %14\n\t"
        "v_bfi_b32 %15, %10, %4, %15\n\t"
        "v_bfi_b32 %0, %11, %5, %0\n\t"
        "v_bfi_b32 %1, %12, %6, %1\n\t"
        "v_bfi_b32 %2, %13, %7, %2\n\t"
        "v_bfi_b32 %3, %14, %8, %3\n\t"
        "v_bfi_b32 %4, %15, %9, %4\n\t"
        "v_bfi_b32 %5, %0, %10, %5\n\t"
        "v_bfi_b32 %6, %1, %11, %6\n\t"
        "v_bfi_b32 %7, %2, %12, %7\n\t"
        "v_bfi_b32 %8, %3, %13, %8\n\t"
        "v_bfi_b32 %9, %4, %14, %9\n\t"
        "v_bfi_b32 %10, %5, %15, %10\n\t"
        "v_bfi_b32 %11, %6, %0, %11\n\t"
        "v_bfi_b32 %12, %7, %1, %12\n\t"
        "v_bfi_b32 %13, %8, %2, %13\n\t"
        "v_bfi_b32 %14, %9, %3, %14\n\t"
        "v_bfi_b32 %15, %10, %4, %15\n\t"
        "v_bfi_b32 %0, %11, %5, %0\n\t"
        "v_bfi_b32 %1, %12, %6, %1\n\t"
        "v_bfi_b32 %2, %13, %7, %2\n\t"
        "v_bfi_b32 %3, %14, %8, %3\n\t"
        "v_bfi_b32 %4, %15, %9, %4\n\t"
        "v_bfi_b32 %5, %0, %10, %5\n\t"
        "v_bfi_b32 %6, %1, %11, %6\n\t"
        "v_bfi_b32 %7, %2, %12, %7\n\t"
        "v_bfi_b32 %8, %3, %13, %8\n\t"
        "v_bfi_b32 %9, %4, %14, %9\n\t"
        "v_bfi_b32 %10, %5, %15, %10\n\t"
        "v_bfi_b32 %11, %6, %0, %11\n\t"
        "v_bfi_b32 %12, %7, %1, %12\n\t"
        "v_bfi_b32 %13, %8, %2, %13\n\t"
        "v_bfi_b32 %14, %9, %3, %14\n\t"
        "v_bfi_b32 %15, %10, %4, %15\n\t"
        "v_bfi_b32 %0, %11, %5, %0\n\t"
        "v_bfi_b32 %1, %12, %6, %1\n\t"
        "v_bfi_b32 %2, %13, %7, %2\n\t"
        "v_bfi_b32 %3, %14, %8, %3\n\t"
        "v_bfi_b32 %4, %15, %9, %4\n\t"
        "v_bfi_b32 %5, %0, %10, %5\n\t"
        "v_bfi_b32 %6, %1, %11, %6\n\t"
        "v_bfi_b32 %7, %2, %12, %7\n\t"
        "v_bfi_b32 %8, %3, %13, %8\n\t"
        "v_bfi_b32 %9, %4, %14, %9\n\t"
        "v_bfi_b32 %10, %5, %15, %10\n\t"
        "v_bfi_b32 %11, %6, %0, %11\n\t"
        "v_bfi_b32 %12, %7, %1, %12\n\t"
        "v_bfi_b32 %13, %8, %2, %13\n\t"
        "v_bfi_b32 %14, %9, %3, %14\n\t"
        "v_bfi_b32 %15, %10, %4, %15\n\t"
        "v_bfi_b32 %0, %11, %5, %0\n\t"
        "v_bfi_b32 %1, %12, %6, %1\n\t"
        "v_bfi_b32 %2, %13, %7, %2\n\t"
        "v_bfi_b32 %3, %14, %8, %3\n\t"
        "v_bfi_b32 %4, %15, %9, %4\n\t"
        "v_bfi_b32 %5, %0, %10, %5\n\t"
        "v_bfi_b32 %6, %1, %11, %6\n\t"
        "v_bfi_b32 %7, %2, %12, %7\n\t"
        "v_bfi_b32 %8, %3, %13, %8\n\t"
        "v_bfi_b32 %9, %4, %14, %9\n\t"
        "v_bfi_b32 %10, %5, %15, %10\n\t"
        "v_bfi_b32 %11, %6, %0, %11\n\t"
        "v_bfi_b32 %12, %7, %1, %12\n\t"
        "v_bfi_b32 %13, %8, %2, %13\n\t"
        "v_bfi_b32 %14, %9, %3, %14\n\t"
        "v_bfi_b32 %15, %10, %4, %15\n\t"
        "v_bfi_b32 %0, %11, %5, %0\n\t"
        "v_bfi_b32 %1, %12, %6, %1\n\t"
        "v_bfi_b32 %2, %13, %7, %2\n\t"
        "v_bfi_b32 %3, %14, %8, %3\n\t"
        "v_bfi_b32 %4, %15, %9, %4\n\t"
        "v_bfi_b32 %5, %0, %10, %5\n\t"
        "v_bfi_b32 %6, %1, %11, %6\n\t"
        "v_bfi_b32 %7, %2, %12, %7\n\t"
        "v_bfi_b32 %8, %3, %13, %8\n\t"
        "v_bfi_b32 %9, %4, %14, %9\n\t"
        "v_bfi_b32 %10, %5, %15, %10\n\t"
        "v_bfi_b32 %11, %6, %0, %11\n\t"
        "v_bfi_b32 %12, %7, %1, %12\n\t"
        "v_bfi_b32 %13, %8, %2, %13\n\t"
        "v_bfi_b32 %14, %9, %3, %14\n\t"
        "v_bfi_b32 %15, %10, %4, %15\n\t"
        "v_bfi_b32 %0, %11, %5, %0\n\t"
        "v_bfi_b32 %1, %12, %6, %1\n\t"
        "v_bfi_b32 %2, %13, %7, %2\n\t"
        "v_bfi_b32 %3, %14, %8, %3\n\t"
        "v_bfi_b32 %4, %15, %9, %4\n\t"
        "v_bfi_b32 %5, %0, %10, %5\n\t"
        "v_bfi_b32 %6, %1, %11, %6\n\t"
        "v_bfi_b32 %7, %2, %12, %7\n\t"
        "v_bfi_b32 %8, %3, %13, %8\n\t"
        "v_bfi_b32 %9, %4, %14, %9\n\t"
        "v_bfi_b32 %10, %5, %15, %10\n\t"
        "v_bfi_b32 %11, %6, %0, %11\n\t"
        "v_bfi_b32 %12, %7, %1, %12\n\t"
        "v_bfi_b32 %13, %8, %2, %13\n\t"
        "v_bfi_b32 %14, %9, %3, %14\n\t"
        "v_bfi_b32 %15, %10, %4, %15\n\t"
        : "+v"(X[0][0]), "+v"(X[0][1]), "+v"(X[0][2]), "+v"(X[0][3]), "+v"(X[0][4]), "+v"(X[0][5]), "+v"(X[0][6]), "+v"(X[0][7]), "+v"(X[1][0]), "+v"(X[1][1]), "+v"(X[1][2]), "+v"(X[1][3]), "+v"(X[1][4]), "+v"(X[1][5]), "+v"(X[1][6]), "+v"(X[1][7])
        : "s"(0x0F0F0F0Fu));
}

// exchange, one plane per step, double-buffered (two 32 KiB [symbol][lane] buffers):
// step p issues the reads of plane p and the writes of plane p + 1, then one barrier
template <bool TO_LARGE>
__device__ __forceinline__ void xch_db(uint32_t (&X)[16][8], uint32_t* lds, uint32_t A, uint32_t lane) {
    auto wa = [&](int j) { return TO_LARGE ? (16u * A + j) * 64u + lane : (8u * j + A) * 64u + lane; };
    auto ra = [&](int j) { return TO_LARGE ? (8u * j + A) * 64u + lane : (16u * A + j) * 64u + lane; };
    uint32_t R[16];
    bs8::sfor<16>([&](auto J) { lds[wa(J)] = X[decltype(J)::value][0]; });
    __syncthreads();
    bs8::sfor<8>([&](auto Pp) {
        constexpr int p = decltype(Pp)::value;
        uint32_t* cur = lds + (p & 1) * 8192u;
        uint32_t* nxt = lds + ((p + 1) & 1) * 8192u;
        bs8::sfor<16>([&](auto J) { R[decltype(J)::value] = cur[ra(J)]; });
        if constexpr (p < 7) bs8::sfor<16>([&](auto J) { nxt[wa(J)] = X[decltype(J)::value][p + 1]; });
        bs8::sfor<16>([&](auto J) { X[decltype(J)::value][p] = R[decltype(J)::value]; });
        __syncthreads();
    });
}

// hand-written two-plane exchange: [symbol][lane] x 8 B, ds_write_b64 / ds_read_b64 with
// immediate offsets (small e = 16A + j: 8192 A + 512 j; large e = 8h + A: 512 A + 4096 h)
typedef uint32_t v2u_ __attribute__((ext_vector_type(2)));
#define XW64(j, o) "ds_write_b64 %16, %" #j " offset:" #o "\n\t"
#define XR64(j, o) "ds_read_b64 %" #j ", %17 offset:" #o "\n\t"
#define XSMALL(W) W(0, 0) W(1, 512) W(2, 1024) W(3, 1536) W(4, 2048) W(5, 2560) W(6, 3072) W(7, 3584) \
    W(8, 4096) W(9, 4608) W(10, 5120) W(11, 5632) W(12, 6144) W(13, 6656) W(14, 7168) W(15, 7680)
#define XLARGE(W) W(0, 0) W(1, 4096) W(2, 8192) W(3, 12288) W(4, 16384) W(5, 20480) W(6, 24576) W(7, 28672) \
    W(8, 32768) W(9, 36864) W(10, 40960) W(11, 45056) W(12, 49152) W(13, 53248) W(14, 57344) W(15, 61440)
template <bool TO_LARGE>
__device__ __forceinline__ void xch64(v2u_ (&Y)[16], uint32_t wb, uint32_t rb) {
    if constexpr (TO_LARGE)
        asm volatile(XSMALL(XW64) "s_waitcnt lgkmcnt(0)\n\ts_barrier\n\t" XLARGE(XR64) "s_waitcnt lgkmcnt(0)\n\ts_barrier"
                     : "+v"(Y[0]), "+v"(Y[1]), "+v"(Y[2]), "+v"(Y[3]), "+v"(Y[4]), "+v"(Y[5]), "+v"(Y[6]), "+v"(Y[7]),
                       "+v"(Y[8]), "+v"(Y[9]), "+v"(Y[10]), "+v"(Y[11]), "+v"(Y[12]), "+v"(Y[13]), "+v"(Y[14]), "+v"(Y[15])
                     : "v"(wb), "v"(rb) : "memory");
    else
        asm volatile(XLARGE(XW64) "s_waitcnt lgkmcnt(0)\n\ts_barrier\n\t" XSMALL(XR64) "s_waitcnt lgkmcnt(0)\n\ts_barrier"
                     : "+v"(Y[0]), "+v"(Y[1]), "+v"(Y[2]), "+v"(Y[3]), "+v"(Y[4]), "+v"(Y[5]), "+v"(Y[6]), "+v"(Y[7]),
                       "+v"(Y[8]), "+v"(Y[9]), "+v"(Y[10]), "+v"(Y[11]), "+v"(Y[12]), "+v"(Y[13]), "+v"(Y[14]), "+v"(Y[15])
                     : "v"(wb), "v"(rb) : "memory");
}
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
// exchange with two planes per round through a 64 KiB [symbol][lane] x 8 B buffer
template <int q>
__device__ __forceinline__ void xch2_to_large(uint32_t (&X)[16][8], uint32_t* lds, uint32_t A, uint32_t lane) {
    v2u* E = reinterpret_cast<v2u*>(lds);
    bs8::sfor<16>([&](auto J) { constexpr int j = decltype(J)::value; E[(16u * A + j) * 64u + lane] = v2u{X[j][2 * q], X[j][2 * q + 1]}; });
    __syncthreads();
    bs8::sfor<16>([&](auto H) { constexpr int h = decltype(H)::value; const v2u v = E[(8u * h + A) * 64u + lane]; X[h][2 * q] = v.x; X[h][2 * q + 1] = v.y; });
    __syncthreads();
}
template <int q>
__device__ __forceinline__ void xch2_to_small(uint32_t (&X)[16][8], uint32_t* lds, uint32_t A, uint32_t lane) {
    v2u* E = reinterpret_cast<v2u*>(lds);
    bs8::sfor<16>([&](auto H) { constexpr int h = decltype(H)::value; E[(8u * h + A) * 64u + lane] = v2u{X[h][2 * q], X[h][2 * q + 1]}; });
    __syncthreads();
    bs8::sfor<16>([&](auto J) { constexpr int j = decltype(J)::value; const v2u v = E[(16u * A + j) * 64u + lane]; X[j][2 * q] = v.x; X[j][2 * q + 1] = v.y; });
    __syncthreads();
}
template <int V>
__global__ __launch_bounds__(512, 1) void setprobe_kernel(uint32_t iters, uint32_t* sink) {
    __shared__ uint32_t lds[(kDmaBytes + kXchBytes) / 4];
    const uint32_t lds_base = (uint32_t)(uintptr_t)lds;
    const uint32_t A = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t s_small = __builtin_amdgcn_readfirstlane(lds_base + 4096u * A);
    const uint32_t s_large = __builtin_amdgcn_readfirstlane(lds_base + 256u * A);
    const uint32_t e_small = s_small + lane * 4u, e_large = s_large + lane * 4u;
    uint32_t X[16][8];
    bs8::sfor<16>([&](auto J) {
        bs8::sfor<8>([&](auto I) {
            X[decltype(J)::value][decltype(I)::value] = threadIdx.x * 2654435761u + 97u * decltype(J)::value + decltype(I)::value;
        });
    });
    for (uint32_t n = 0; n < iters; ++n) {
        if constexpr (V == 15) {
            // X held as 64 two-plane pairs (the layout a b64 exchange needs)
            v2u_ (&Y)[16][4] = *reinterpret_cast<v2u_ (*)[16][4]>(&X);
            const uint32_t wsm = lds_base + 8192u * A + lane * 8u, wlg = lds_base + 512u * A + lane * 8u;
            bs8::sfor<4>([&](auto Q) {
                v2u_ T[16];
                bs8::sfor<16>([&](auto J) { T[decltype(J)::value] = Y[decltype(J)::value][decltype(Q)::value]; });
                xch64<true>(T, wsm, wlg);
                bs8::sfor<16>([&](auto J) { Y[decltype(J)::value][decltype(Q)::value] = T[decltype(J)::value]; });
            });
            bs8::sfor<4>([&](auto Q) {
                v2u_ T[16];
                bs8::sfor<16>([&](auto J) { T[decltype(J)::value] = Y[decltype(J)::value][decltype(Q)::value]; });
                xch64<false>(T, wlg, wsm);
                bs8::sfor<16>([&](auto J) { Y[decltype(J)::value][decltype(Q)::value] = T[decltype(J)::value]; });
            });
        }
        if constexpr (V == 8) { xch_db<true>(X, lds, A, lane); xch_db<false>(X, lds, A, lane); }
        if constexpr (V == 9) alu_lshl(X);
        if constexpr (V == 10) alu_bfi(X);
        if constexpr (V == 11) alu_bitop3(X);
        if constexpr (V == 12) alu_xor(X);
        if constexpr (V == 13) alu_perm(X);
        if constexpr (V == 14) alu_bfiv(X);
        if constexpr (V == 0 || V == 2) bs8::sfor<16>([&](auto J) { bs8::transpose8_dev(X[decltype(J)::value]); });
        if constexpr (V == 0 || V == 1) bs8::small_ifft_all(X, A);
        if constexpr (V == 0 || V == 3)
            bs8::sfor<8>([&](auto Pp) { xch_to_large<decltype(Pp)::value, true>(X, e_small, s_small, e_large); });
        if constexpr (V <= 1 || V == 4) bs8::large_ifft_fft(X);
        if constexpr (V == 0 || V == 3)
            bs8::sfor<8>([&](auto Pp) { xch_to_small<decltype(Pp)::value, true>(X, e_large, s_large, e_small); });
        if constexpr (V == 0 || V == 1) bs8::small_fft_all(X, A);
        if constexpr (V == 5) bs8::sfor<8>([&](auto J) { transpose8x2_s(X[2 * decltype(J)::value], X[2 * decltype(J)::value + 1]); });
        if constexpr (V == 5) bs8::sfor<8>([&](auto J) { transpose8x2_s(X[2 * decltype(J)::value], X[2 * decltype(J)::value + 1]); });
        if constexpr (V == 6) bs8::sfor<8>([&](auto J) { transpose8x2_v(X[2 * decltype(J)::value], X[2 * decltype(J)::value + 1]); });
        if constexpr (V == 6) bs8::sfor<8>([&](auto J) { transpose8x2_v(X[2 * decltype(J)::value], X[2 * decltype(J)::value + 1]); });
        if constexpr (V == 7) {
            bs8::sfor<4>([&](auto Q) { xch2_to_large<decltype(Q)::value>(X, lds, A, lane); });
            bs8::sfor<4>([&](auto Q) { xch2_to_small<decltype(Q)::value>(X, lds, A, lane); });
        }
        if constexpr (V == 0 || V == 2) bs8::sfor<16>([&](auto J) { bs8::transpose8_dev(X[decltype(J)::value]); });
    }
    uint32_t acc = 0;
    bs8::sfor<16>([&](auto J) { bs8::sfor<8>([&](auto I) { acc ^= X[decltype(J)::value][decltype(I)::value]; }); });
    sink[blockIdx.x * 512 + threadIdx.x] = acc;
}
}  // namespace
}  // namespace rsm

int main(int argc, char** argv) {
    const uint32_t iters = argc > 1 ? atoi(argv[1]) : 64;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t* sink;
    CK(hipMalloc(&sink, (size_t)cus * 512 * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* names[] = {"set", "butterflies", "transposes", "exchange", "large", "transposes_x2_sgpr", "transposes_x2_vgpr", "exchange_b64", "exchange_dbuf", "alu_lshl_x128", "alu_bfi_sgpr_x128", "alu_bitop3_x128", "alu_xor_x128", "alu_perm_x128", "alu_bfi_vgpr_x128", "exchange_b64_asm"};
    for (int v = 0; v < 16; ++v) {
        std::vector<float> ts;
        for (int r = 0; r < 8; ++r) {
            CK(hipEventRecord(e0, 0));
            switch (v) {
                case 0: hipLaunchKernelGGL(rsm::setprobe_kernel<0>, dim3(cus), dim3(512), 0, 0, iters, sink); break;
                case 1: hipLaunchKernelGGL(rsm::setprobe_kernel<1>, dim3(cus), dim3(512), 0, 0, iters, sink); break;
                case 2: hipLaunchKernelGGL(rsm::setprobe_kernel<2>, dim3(cus), dim3(512), 0, 0, iters, sink); break;
                case 3: hipLaunchKernelGGL(rsm::setprobe_kernel<3>, dim3(cus), dim3(512), 0, 0, iters, sink); break;
                case 4: hipLaunchKernelGGL(rsm::setprobe_kernel<4>, dim3(cus), dim3(512), 0, 0, iters, sink); break;
                case 5: hipLaunchKernelGGL(rsm::setprobe_kernel<5>, dim3(cus), dim3(512), 0, 0, iters, sink); break;
                case 6: hipLaunchKernelGGL(rsm::setprobe_kernel<6>, dim3(cus), dim3(512), 0, 0, iters, sink); break;
                case 7: hipLaunchKernelGGL(rsm::setprobe_kernel<7>, dim3(cus), dim3(512), 0, 0, iters, sink); break;
                case 8: hipLaunchKernelGGL(rsm::setprobe_kernel<8>, dim3(cus), dim3(512), 0, 0, iters, sink); break;
                case 9: hipLaunchKernelGGL(rsm::setprobe_kernel<9>, dim3(cus), dim3(512), 0, 0, iters, sink); break;
                case 10: hipLaunchKernelGGL(rsm::setprobe_kernel<10>, dim3(cus), dim3(512), 0, 0, iters, sink); break;
                case 11: hipLaunchKernelGGL(rsm::setprobe_kernel<11>, dim3(cus), dim3(512), 0, 0, iters, sink); break;
                case 12: hipLaunchKernelGGL(rsm::setprobe_kernel<12>, dim3(cus), dim3(512), 0, 0, iters, sink); break;
                case 13: hipLaunchKernelGGL(rsm::setprobe_kernel<13>, dim3(cus), dim3(512), 0, 0, iters, sink); break;
                case 14: hipLaunchKernelGGL(rsm::setprobe_kernel<14>, dim3(cus), dim3(512), 0, 0, iters, sink); break;
                case 15: hipLaunchKernelGGL(rsm::setprobe_kernel<15>, dim3(cus), dim3(512), 0, 0, iters, sink); break;
            }
            CK(hipGetLastError());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 2) ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        printf("{\"probe\": \"setprobe\", \"variant\": \"%s\", \"iters\": %u, \"cus\": %d, \"us_per_set\": %.3f}\n", names[v],
               iters, cus, ts[ts.size() / 2] * 1e3 / iters);
        fflush(stdout);
    }
    CK(hipFree(sink));
    return 0;
}
