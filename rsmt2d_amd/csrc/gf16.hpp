// gf16.hpp -- GF(2^16) tables and device resources shared by host and kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace rsm {

// v_perm_b32 tables for y -> y * exp(L) on packed GF(2^16) symbols.  The 16-bit
// symbol is cut into six chunks (lo byte bits [0,3) [3,6) [6,8), hi byte bits
// [0,3) [3,6) [6,8)); chunk c has an output-lo and an output-hi byte table of up
// to 8 entries held as two dwords each: w[4c+0..1] = lo table, w[4c+2..3] = hi.
struct alignas(16) PermTab16 {
    uint32_t w[24];
};

// Twiddle tables by skew index for the single-pass encoder: skewperm[i] =
// perm[skew[i]], or all-zero where skew[i] is the modulus (the butterfly's
// multiply is skipped), so a butterfly's table is ONE uniform load with no
// dependent skew lookup and no branch.  Indices < kSkewPermN cover m <= 1024.
constexpr uint32_t kSkewPermN = 2048;

// The device LogWalsh buffer holds the 65536-entry table, then at kLwFoldOff + N - 512
// the table folded to N = 512 .. 32768 points: fold_N[r] = sum_q logwalsh[qN + r] (mod
// 65535), which the decoders' N-point error locators use (kernels_gf16.hip; N = 65536
// reads the table itself).
constexpr uint32_t kLwFoldOff = 65536;

struct Gf16Host {
    std::vector<uint16_t> exp, log, skew, logwalsh;
    std::vector<uint16_t> lwfold;     // fold_512, fold_1024, ..., fold_32768
    std::vector<PermTab16> perm;      // 65536 entries
    std::vector<PermTab16> skewperm;  // kSkewPermN entries
};
const Gf16Host& gf16_host();

// Device copies + scratch, owned by a context.
struct Gf16Dev {
    const PermTab16* perm = nullptr;  // [65536]
    const uint16_t* skew = nullptr;   // [65535]
    const uint16_t* logwalsh = nullptr;
    const PermTab16* skewperm = nullptr;  // [kSkewPermN]
    uint32_t cus = 256;                   // persistent-grid size (the context's CUs)
    uint8_t* scratch = nullptr;       // work arrays
    uint64_t scratch_bytes = 0;
    uint16_t* errs = nullptr;         // decoder error locators [count][n]
    uint64_t errs_bytes = 0;
};

}  // namespace rsm
