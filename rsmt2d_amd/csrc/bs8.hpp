// bs8.hpp -- bit-sliced GF(2^8) Leopard encode arithmetic (host + device).
//
// Representation: 32 bytes of one symbol position range are held as 8 u32
// bit-planes (plane i = bit i of each of the 32 bytes).  Multiplication by a
// compile-time constant exp(L) is then a fixed GF(2)-linear map of the planes:
//   out_i = XOR_{j : bit i of (2^j * exp(L)) = 1} y_j
// written as v_bitop3_b32 (3-input XOR) networks with up to three shared
// temporaries, searched at build time (gen/bs8_net.hpp) -- ~15 VALU per 32 bytes,
// against 80 for the byte-table (v_perm) multiply.
//
// The additive-FFT schedule is the one of kernels_gf8.hip (IFFT_DIT layers
// d = 1..M/2 with skew offset M-1, then FFT_DIT layers M/2..1 with offset -1;
// SURVEY.md Appendix A.4, klauspost leopard8.go ifftDITEncoder8/fftDIT8), split
// for M = 128 into
//   small layers d = 1, 2, 4   on 16 consecutive symbols e = 16a + j  (fixed a)
//   large layers d = 8 .. 64   on 16 strided symbols   e = 8h + g    (fixed g)
// so that a thread never needs more than 16 symbols x 8 planes = 128 registers,
// and every twiddle is a compile-time constant within a (small: a / large: all)
// specialisation.  This header holds the arithmetic only; the data movement
// (global loads, the LDS exchange between the two layouts) is in
// kernels_gf8_bs.hip, and tests/native/bs8_host.cpp runs the same templates on
// the CPU against the oracle.
#pragma once
#include <cstdint>
#include <utility>
#include "gf_tables.hpp"

#if defined(__HIPCC__)
#define RSM_HD __host__ __device__ __forceinline__
#else
#define RSM_HD inline __attribute__((always_inline))
#endif

namespace rsm::bs8 {

template <int N, typename F>
RSM_HD void sfor(F&& f) {
    [&]<int... I>(std::integer_sequence<int, I...>) {
        (f(std::integral_constant<int, I>{}), ...);
    }(std::make_integer_sequence<int, N>{});
}

#if defined(__HIPCC__)
// Device butterflies: one generated asm block each (bs8_asm.inc, from
// gen/gen_bs8_asm.cpp).  One block per butterfly instead of one statement per
// instruction: the compiler pads every asm boundary with an s_nop (a 4-cycle
// issue slot).
#define RSM_BS8_DEV __device__ __forceinline__
template <unsigned L>
RSM_BS8_DEV void ifft2_asm(uint32_t (&x)[8], uint32_t (&y)[8]);
template <unsigned L>
RSM_BS8_DEV void fft2_asm(uint32_t (&x)[8], uint32_t (&y)[8]);
template <unsigned L>
RSM_BS8_DEV void mid2_asm(uint32_t (&x)[8], uint32_t (&y)[8]);
#include "bs8_asm.inc"
// small-layout layers of all eight waves, one asm statement each (branch on A inside)
#include "bs8_small.inc"
#endif

// Host reference: the same networks, interpreted from the generated table.
#include "bs8_net.inc"
template <unsigned L>
inline void muladd_host(uint32_t (&x)[8], const uint32_t (&y)[8]) {
    uint32_t r[24] = {};  // x, y, up to 8 temporaries
    for (int i = 0; i < 8; ++i) r[i] = x[i], r[8 + i] = y[i];
    for (int n = 0; n < kNetLen[L]; ++n) {
        const NetOp& o = kNet[L][n];
        const uint32_t v = o.kind == 0 ? r[o.a] : o.kind == 3 ? (r[o.a] ^ r[o.b] ^ r[o.c]) : (r[o.a] ^ r[o.b]);
        r[o.dst] = o.kind >= 2 ? v : (r[o.dst] ^ v);
    }
    for (int i = 0; i < 8; ++i) x[i] = r[i];
}

// IFFT_DIT2: y ^= x; x ^= y*L.   FFT_DIT2: x ^= y*L; y ^= x.   L == 255: XOR only.
// MID: y ^= x; x ^= y*L; y ^= x -- an IFFT_DIT2 (twiddle L1) directly followed by an
// FFT_DIT2 (L2) on the same pair, since x ^= L1*y' ^ L2*y' = (exp L1 + exp L2)*y'.
template <unsigned L>
RSM_HD void ifft2(uint32_t (&x)[8], uint32_t (&y)[8]) {
#if defined(__HIP_DEVICE_COMPILE__)
    ifft2_asm<L>(x, y);
#else
    for (int i = 0; i < 8; ++i) y[i] ^= x[i];
    if constexpr (L != 255u) muladd_host<L>(x, y);
#endif
}
template <unsigned L>
RSM_HD void fft2(uint32_t (&x)[8], uint32_t (&y)[8]) {
#if defined(__HIP_DEVICE_COMPILE__)
    fft2_asm<L>(x, y);
#else
    if constexpr (L != 255u) muladd_host<L>(x, y);
    for (int i = 0; i < 8; ++i) y[i] ^= x[i];
#endif
}
template <unsigned L>
RSM_HD void mid2(uint32_t (&x)[8], uint32_t (&y)[8]) {
#if defined(__HIP_DEVICE_COMPILE__)
    mid2_asm<L>(x, y);
#else
    for (int i = 0; i < 8; ++i) y[i] ^= x[i];
    if constexpr (L != 255u) muladd_host<L>(x, y);
    for (int i = 0; i < 8; ++i) y[i] ^= x[i];
#endif
}

// Leopard's log of zero is 255; the log of exp(L1) + exp(L2).
constexpr unsigned elem_of_log(unsigned L) { return L == 255u ? 0u : kGf8.exp[L]; }
constexpr unsigned log_of_sum(unsigned L1, unsigned L2) {
    return (elem_of_log(L1) ^ elem_of_log(L2)) == 0 ? 255u : kGf8.log[elem_of_log(L1) ^ elem_of_log(L2)];
}

// 8x8 bit-matrix transpose applied to each of the 4 byte lanes of 8 words:
// afterwards bit q of byte b of w[p] = bit p of byte b of the original w[q].
// An involution: the same network converts bytes -> planes and planes -> bytes.
RSM_HD void swapbits(uint32_t& a, uint32_t& b, int s, uint32_t m) {
    const uint32_t t = ((a >> s) ^ b) & m;
    b ^= t;
    a ^= t << s;
}
RSM_HD void transpose8(uint32_t (&w)[8]) {
    swapbits(w[0], w[4], 4, 0x0F0F0F0Fu);
    swapbits(w[1], w[5], 4, 0x0F0F0F0Fu);
    swapbits(w[2], w[6], 4, 0x0F0F0F0Fu);
    swapbits(w[3], w[7], 4, 0x0F0F0F0Fu);
    swapbits(w[0], w[2], 2, 0x33333333u);
    swapbits(w[1], w[3], 2, 0x33333333u);
    swapbits(w[4], w[6], 2, 0x33333333u);
    swapbits(w[5], w[7], 2, 0x33333333u);
    swapbits(w[0], w[1], 1, 0x55555555u);
    swapbits(w[2], w[3], 1, 0x55555555u);
    swapbits(w[4], w[5], 1, 0x55555555u);
    swapbits(w[6], w[7], 1, 0x55555555u);
}

#if defined(__HIPCC__)
// Device 8x8 transpose as one asm block: per swap t1 = b << s, t2 = a >> s,
// a = sel(m << s ? t1 : a), b = sel(m ? t2 : b), two swaps interleaved so
// consecutive instructions are independent.  Same permutation as transpose8.
// On gfx950 every shift and v_bfi_b32 issues at half rate (4.5 cycles per wave
// instruction with two waves per SIMD) while v_bitop3_b32 and v_add_u32 issue at
// full rate (2.4-2.9; profiles/r02d_aluprobe.jsonl), so the select is a
// v_bitop3_b32 (truth table 0xD8: S2 ? S1 : S0) and the s = 1 left shift a
// v_add_u32 (b + b).
#define RSM_T8_SHL(d, b, s) "v_lshlrev_b32 %" #d ", " #s ", %" #b "\n\t"
#define RSM_T8_SHL1(d, b, s) "v_add_u32 %" #d ", %" #b ", %" #b "\n\t"
#define RSM_T8_PAIRS(SHL, a0, b0, a1, b1, s, m, mh)    \
    SHL(8, b0, s)                                    \
    "v_lshrrev_b32 %9, " #s ", %" #a0 "\n\t"           \
    SHL(10, b1, s)                                   \
    "v_lshrrev_b32 %11, " #s ", %" #a1 "\n\t"          \
    "v_bitop3_b32 %" #a0 ", %" #a0 ", %8, %" #mh " bitop3:0xd8\n\t" \
    "v_bitop3_b32 %" #b0 ", %" #b0 ", %9, %" #m " bitop3:0xd8\n\t"  \
    "v_bitop3_b32 %" #a1 ", %" #a1 ", %10, %" #mh " bitop3:0xd8\n\t" \
    "v_bitop3_b32 %" #b1 ", %" #b1 ", %11, %" #m " bitop3:0xd8\n\t"
__device__ __forceinline__ void transpose8_dev(uint32_t (&w)[8]) {
    uint32_t t0, t1, t2, t3;
    asm volatile(
        RSM_T8_PAIRS(RSM_T8_SHL, 0, 4, 1, 5, 4, 12, 13)
        RSM_T8_PAIRS(RSM_T8_SHL, 2, 6, 3, 7, 4, 12, 13)
        RSM_T8_PAIRS(RSM_T8_SHL, 0, 2, 1, 3, 2, 14, 15)
        RSM_T8_PAIRS(RSM_T8_SHL, 4, 6, 5, 7, 2, 14, 15)
        RSM_T8_PAIRS(RSM_T8_SHL1, 0, 1, 2, 3, 1, 16, 17)
        RSM_T8_PAIRS(RSM_T8_SHL1, 4, 5, 6, 7, 1, 16, 17)
        : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]), "+v"(w[7]),
          "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3)
        : "s"(0x0F0F0F0Fu), "s"(0xF0F0F0F0u), "s"(0x33333333u), "s"(0xCCCCCCCCu), "s"(0x55555555u),
          "s"(0xAAAAAAAAu));
}
#undef RSM_T8_SHL
#undef RSM_T8_SHL1
#undef RSM_T8_PAIRS
#endif

constexpr int kM = 128;        // transform size handled here (65 <= k <= 128)
constexpr int kOffEnc = kM - 1;  // encoder IFFT skew offset

// Small layers: registers j = 0..15 hold symbols e = 16A + j.
template <int A>
RSM_HD void small_ifft(uint32_t (&X)[16][8]) {
    sfor<3>([&](auto LG) {
        constexpr int d = 1 << decltype(LG)::value;
        sfor<16 / (2 * d)>([&](auto B) {
            constexpr int b = decltype(B)::value * 2 * d;
            constexpr unsigned L = kGf8.skew[kOffEnc + 16 * A + b + d];
            sfor<d>([&](auto Q) { ifft2<L>(X[b + decltype(Q)::value], X[b + decltype(Q)::value + d]); });
        });
    });
}
template <int A>
RSM_HD void small_fft(uint32_t (&X)[16][8]) {
    sfor<3>([&](auto LG) {
        constexpr int d = 4 >> decltype(LG)::value;
        sfor<16 / (2 * d)>([&](auto B) {
            constexpr int b = decltype(B)::value * 2 * d;
            constexpr unsigned L = kGf8.skew[-1 + 16 * A + b + d];
            sfor<d>([&](auto Q) { fft2<L>(X[b + decltype(Q)::value], X[b + decltype(Q)::value + d]); });
        });
    });
}

// Large layers: registers h = 0..15 hold symbols e = 8h + g (any g < 8): the
// pairing bit is a bit of h and the block start 8*(h & ~(2dh-1)) does not
// depend on g, so one code path serves every g.  The encoder's last IFFT layer
// (d = 64, SKEW[kOffEnc + 64]) and first FFT layer (d = 64, SKEW[63]) act on the
// same pairs with nothing in between: one merged butterfly, one multiply.
inline constexpr unsigned kMidLog = log_of_sum(kGf8.skew[kOffEnc + 64], kGf8.skew[63]);
RSM_HD void large_ifft_fft(uint32_t (&X)[16][8]) {
    sfor<3>([&](auto LG) {  // IFFT d = 8, 16, 32
        constexpr int dh = 1 << decltype(LG)::value;
        sfor<16 / (2 * dh)>([&](auto B) {
            constexpr int hb = decltype(B)::value * 2 * dh;
            constexpr unsigned L = kGf8.skew[kOffEnc + 8 * hb + 8 * dh];
            sfor<dh>([&](auto Q) { ifft2<L>(X[hb + decltype(Q)::value], X[hb + decltype(Q)::value + dh]); });
        });
    });
    sfor<8>([&](auto Q) { mid2<kMidLog>(X[decltype(Q)::value], X[decltype(Q)::value + 8]); });
    sfor<3>([&](auto LG) {  // FFT d = 32, 16, 8
        constexpr int dh = 4 >> decltype(LG)::value;
        sfor<16 / (2 * dh)>([&](auto B) {
            constexpr int hb = decltype(B)::value * 2 * dh;
            constexpr unsigned L = kGf8.skew[-1 + 8 * hb + 8 * dh];
            sfor<dh>([&](auto Q) { fft2<L>(X[hb + decltype(Q)::value], X[hb + decltype(Q)::value + dh]); });
        });
    });
}

// ---------------------------------------------------------------------------
// Half-split schedule (production queue kernel since round 3).  Symbol bit 6
// splits the 128-point transform into two halves that are independent in every
// layer except the merged middle pair, so each phase below works on one half
// (registers 8G..8G+7) while the other half's LDS exchange is in flight.
//   small layout S': wave A, register j: e = (j & 7) + 8A + 64 (j >> 3)
//                    (bits 0-2 in registers, 3-5 the wave, bit 6 the half)
//   large layout L : wave w, register h: e = w + 8h (as above)
// The exchange of half G is a transpose: wave u's register 8G + v goes to wave v's
// register 8G + u (both directions).
template <int A, int G>
RSM_HD void small_ifft_h(uint32_t (&X)[16][8]) {
    sfor<3>([&](auto LG) {
        constexpr int d = 1 << decltype(LG)::value;
        sfor<8 / (2 * d)>([&](auto B) {
            constexpr int b = decltype(B)::value * 2 * d;
            constexpr unsigned L = kGf8.skew[kOffEnc + 8 * A + 64 * G + b + d];
            sfor<d>([&](auto Q) {
                ifft2<L>(X[8 * G + b + decltype(Q)::value], X[8 * G + b + decltype(Q)::value + d]);
            });
        });
    });
}
template <int A, int G>
RSM_HD void small_fft_h(uint32_t (&X)[16][8]) {
    sfor<3>([&](auto LG) {
        constexpr int d = 4 >> decltype(LG)::value;
        sfor<8 / (2 * d)>([&](auto B) {
            constexpr int b = decltype(B)::value * 2 * d;
            constexpr unsigned L = kGf8.skew[-1 + 8 * A + 64 * G + b + d];
            sfor<d>([&](auto Q) {
                fft2<L>(X[8 * G + b + decltype(Q)::value], X[8 * G + b + decltype(Q)::value + d]);
            });
        });
    });
}
template <int G>
RSM_HD void large_ifft_h(uint32_t (&X)[16][8]) {  // IFFT d = 8, 16, 32 on h in [8G, 8G + 8)
    sfor<3>([&](auto LG) {
        constexpr int dh = 1 << decltype(LG)::value;
        sfor<8 / (2 * dh)>([&](auto B) {
            constexpr int hb = 8 * G + decltype(B)::value * 2 * dh;
            constexpr unsigned L = kGf8.skew[kOffEnc + 8 * hb + 8 * dh];
            sfor<dh>([&](auto Q) { ifft2<L>(X[hb + decltype(Q)::value], X[hb + decltype(Q)::value + dh]); });
        });
    });
}
RSM_HD void large_mid(uint32_t (&X)[16][8]) {
    sfor<8>([&](auto Q) { mid2<kMidLog>(X[decltype(Q)::value], X[decltype(Q)::value + 8]); });
}
template <int G>
RSM_HD void large_fft_h(uint32_t (&X)[16][8]) {  // FFT d = 32, 16, 8 on h in [8G, 8G + 8)
    sfor<3>([&](auto LG) {
        constexpr int dh = 4 >> decltype(LG)::value;
        sfor<8 / (2 * dh)>([&](auto B) {
            constexpr int hb = 8 * G + decltype(B)::value * 2 * dh;
            constexpr unsigned L = kGf8.skew[-1 + 8 * hb + 8 * dh];
            sfor<dh>([&](auto Q) { fft2<L>(X[hb + decltype(Q)::value], X[hb + decltype(Q)::value + dh]); });
        });
    });
}

}  // namespace rsm::bs8
