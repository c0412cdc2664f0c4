// kernels_gf8.hip -- CDNA4 (gfx950) Leopard GF(2^8) Reed-Solomon kernels.
//
// Replaces the per-codeword klauspost leopard8 encode/reconstruct that rsmt2d's
// LeoRSCodec calls (leopard.go:28-59) with batched launches over a
// device-resident extended data square (datasquare.go's grid as one contiguous
// [W][W][S] HBM buffer, W = 2k).
//
// Work decomposition ("wave task"): one wavefront owns one codeword (a row or a
// column of the square) x one 256-byte chunk of the share width.  Lane l holds
// byte positions [chunk*256 + 4l, +4) of EVERY symbol of the codeword in
// registers (u32 = 4 independent GF(2^8) symbols), so all butterflies are
// lane-local and every lane of the wave applies the same twiddle: the whole
// additive FFT is unrolled at compile time (template on the power-of-two size
// M) and each twiddle multiply is a fixed 3 x v_perm_b32 table lookup.  Global
// loads/stores are one dword per lane per share = 256 contiguous bytes per wave
// instruction.  No LDS, no cross-lane traffic in the FFT body.
//
// Algorithm restated from SURVEY.md Appendix A (klauspost/reedsolomon v1.14.1
// leopard8.go ifftDITEncoder8/fftDIT8/reconstruct); the radix-4 loop nesting of
// the reference is rewritten layer-by-layer, which performs the identical
// butterflies (groups are disjoint), and truncated groups are computed on
// zero-padding (exact: see DESIGN.md "Truncation").
#include <hip/hip_runtime.h>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <utility>
#include "gf_tables.hpp"
#include "rsm_kernels.hpp"

namespace rsm {

template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    [&]<int... I>(std::integer_sequence<int, I...>) {
        (f(std::integral_constant<int, I>{}), ...);
    }(std::make_integer_sequence<int, N>{});
}

// ---------------------------------------------------------------------------
// GF(2^8) multiply of 4 packed symbols by the constant exp(L).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // gfx950 v_bitop3_b32: a ^ b ^ c
}

// A table dword materialised in a VGPR right where it is used.  v_perm_b32 may
// read only one SGPR (gfx9 constant-bus limit), so one half of each 8-entry
// table must be a VGPR; left to itself the compiler hoists all ~250 distinct
// constants to the kernel entry and runs out of registers.
template <uint32_t C>
__device__ __forceinline__ uint32_t vconst() {
    uint32_t v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "i"(C));
    return v;
}

// x ^= y * exp(L), as ONE scheduling unit: the compiler, left to schedule the
// twelve instructions freely, computes the partial products of many butterflies
// ahead of their use and needs ~70 extra VGPRs; as a unit the temporaries die
// inside it.  Pure register ops (no memory, no special hazards: VALU->VALU and
// SALU->VALU dependencies are interlocked), so it is not volatile.
// The two VGPR table halves (ta = a_lo, tb = b_lo) are materialised once per FFT
// block by the caller and shared by the block's d butterflies.
template <unsigned L>
__device__ __forceinline__ void gf8_muladd_ct(uint32_t& x, uint32_t y, uint32_t ta, uint32_t tb) {
    constexpr PermTab t = make_perm_tab(L);
    uint32_t sa, sb, sc;
    asm("v_lshrrev_b32 %[sb], 3, %[y]\n\t"
        "v_lshrrev_b32 %[sc], 6, %[y]\n\t"
        "v_and_b32 %[sa], %[m7], %[y]\n\t"
        "v_and_b32 %[sb], %[m7], %[sb]\n\t"
        "v_and_b32 %[sc], %[m3], %[sc]\n\t"
        "v_perm_b32 %[sa], %[ahi], %[ta], %[sa]\n\t"
        "v_perm_b32 %[sb], %[bhi], %[tb], %[sb]\n\t"
        "v_perm_b32 %[sc], %[cc], %[cc], %[sc]\n\t"
        "v_bitop3_b32 %[x], %[x], %[sa], %[sb] bitop3:0x96\n\t"
        "v_xor_b32 %[x], %[x], %[sc]"
        : [x] "+v"(x), [sa] "=&v"(sa), [sb] "=&v"(sb), [sc] "=&v"(sc)
        : [y] "v"(y), [ta] "v"(ta), [tb] "v"(tb), [m7] "i"(0x07070707), [m3] "i"(0x03030303),
          [ahi] "s"(t.a_hi), [bhi] "s"(t.b_hi), [cc] "s"(t.c));
}
template <unsigned L>
__device__ __forceinline__ void gf8_muladd_ct(uint32_t& x, uint32_t y) {
    constexpr PermTab t = make_perm_tab(L);
    gf8_muladd_ct<L>(x, y, vconst<t.a_lo>(), vconst<t.b_lo>());
}

// Two multiplies share their selector shifts: ONE v_lshrrev_b64 per shift amount on the
// pair (y1:y0) -- it issues at the rate of a 32-bit shift (profiles/r03_alu64.jsonl), so
// two multiplies take 2 half-rate shifts instead of 4.  The bits y1 pushes into y0's top
// byte are masked off with the selector bits.  Callers pair registers 2i, 2i + 1 of their
// point arrays (an even-aligned register pair needs no copies).
#ifdef RSM_GF8_NO_PAIR  // (diagnostic A/B builds only: every multiply shifts its own selectors)
constexpr bool kGf8Pair = false;
#else
constexpr bool kGf8Pair = true;
#endif
struct Shift2 {
    uint32_t b0, b1, c0, c1;  // y0 >> 3, y1 >> 3, y0 >> 6, y1 >> 6 (junk above the selector bits)
};
__device__ __forceinline__ Shift2 shift2(uint32_t y0, uint32_t y1) {
    const uint64_t y = ((uint64_t)y1 << 32) | y0;
    uint64_t s3, s6;
    asm("v_lshrrev_b64 %0, 3, %2\n\tv_lshrrev_b64 %1, 6, %2" : "=&v"(s3), "=&v"(s6) : "v"(y));
    return Shift2{(uint32_t)s3, (uint32_t)(s3 >> 32), (uint32_t)s6, (uint32_t)(s6 >> 32)};
}
// x ^= y * exp(L) from y and its pre-shifted selector sources y3 = y >> 3, y6 = y >> 6
// (one scheduling unit, as gf8_muladd_ct)
template <unsigned L>
__device__ __forceinline__ void gf8_muladd_sel(uint32_t& x, uint32_t y, uint32_t y3, uint32_t y6, uint32_t ta, uint32_t tb) {
    constexpr PermTab t = make_perm_tab(L);
    uint32_t sa, sb, sc;
    asm("v_and_b32 %[sa], %[m7], %[y]\n\t"
        "v_and_b32 %[sb], %[m7], %[y3]\n\t"
        "v_and_b32 %[sc], %[m3], %[y6]\n\t"
        "v_perm_b32 %[sa], %[ahi], %[ta], %[sa]\n\t"
        "v_perm_b32 %[sb], %[bhi], %[tb], %[sb]\n\t"
        "v_perm_b32 %[sc], %[cc], %[cc], %[sc]\n\t"
        "v_bitop3_b32 %[x], %[x], %[sa], %[sb] bitop3:0x96\n\t"
        "v_xor_b32 %[x], %[x], %[sc]"
        : [x] "+v"(x), [sa] "=&v"(sa), [sb] "=&v"(sb), [sc] "=&v"(sc)
        : [y] "v"(y), [y3] "v"(y3), [y6] "v"(y6), [ta] "v"(ta), [tb] "v"(tb), [m7] "i"(0x07070707),
          [m3] "i"(0x03030303), [ahi] "s"(t.a_hi), [bhi] "s"(t.b_hi), [cc] "s"(t.c));
}
// x0 ^= y0 * exp(L0), x1 ^= y1 * exp(L1) (tables ta0/tb0, ta1/tb1 as gf8_muladd_ct's)
template <unsigned L0, unsigned L1>
__device__ __forceinline__ void gf8_muladd2_ct(uint32_t& x0, uint32_t& x1, uint32_t y0, uint32_t y1, uint32_t ta0,
                                               uint32_t tb0, uint32_t ta1, uint32_t tb1) {
    const Shift2 q = shift2(y0, y1);
    gf8_muladd_sel<L0>(x0, y0, q.b0, q.c0, ta0, tb0);
    gf8_muladd_sel<L1>(x1, y1, q.b1, q.c1, ta1, tb1);
}
template <unsigned L0, unsigned L1>
__device__ __forceinline__ void gf8_muladd2_ct(uint32_t& x0, uint32_t& x1, uint32_t y0, uint32_t y1) {
    constexpr PermTab t0 = make_perm_tab(L0), t1 = make_perm_tab(L1);
    const uint32_t ta0 = vconst<t0.a_lo>(), tb0 = vconst<t0.b_lo>();
    if constexpr (L0 == L1) gf8_muladd2_ct<L0, L1>(x0, x1, y0, y1, ta0, tb0, ta0, tb0);
    else gf8_muladd2_ct<L0, L1>(x0, x1, y0, y1, ta0, tb0, vconst<t1.a_lo>(), vconst<t1.b_lo>());
}

// Runtime (wave-uniform) log constant: tables for all 256 logs in constant memory.
struct PermTabAll {
    PermTab t[256];
};
constexpr PermTabAll make_perm_all() {
    PermTabAll a{};
    for (unsigned L = 0; L < 256; ++L) a.t[L] = make_perm_tab(L);
    return a;
}
__constant__ PermTabAll d_perm8 = make_perm_all();
__constant__ Gf8Tables d_gf8 = kGf8;

// Pins a wave-uniform value to an SGPR at this point of the program; used so the
// per-symbol constant-memory table loads below are issued where they are needed
// instead of all being hoisted to the kernel entry (hundreds of SGPRs).
__device__ __forceinline__ uint32_t pin_sgpr(uint32_t x) {
    asm volatile("; pin %0" : "+s"(x));
    return x;
}

__device__ __forceinline__ uint32_t gf8_mul_rt(uint32_t y, unsigned L) {
    const PermTab t = d_perm8.t[pin_sgpr(L)];
    const uint32_t sa = y & 0x07070707u;
    const uint32_t sb = (y >> 3) & 0x07070707u;
    const uint32_t sc = (y >> 6) & 0x03030303u;
    return xor3(__builtin_amdgcn_perm(t.a_hi, t.a_lo, sa), __builtin_amdgcn_perm(t.b_hi, t.b_lo, sb),
                __builtin_amdgcn_perm(t.c, t.c, sc));
}

// IFFT_DIT2 (y ^= x; x ^= y*L) and FFT_DIT2 (x ^= y*L; y ^= x); L == 255 means
// a zero twiddle: XOR half only (klauspost ifftDIT4/fftDIT4 "log_m == modulus").
template <unsigned L>
__device__ __forceinline__ void ifft2(uint32_t& x, uint32_t& y) {
    y ^= x;
    if constexpr (L != 255u) gf8_muladd_ct<L>(x, y);
}
template <unsigned L>
__device__ __forceinline__ void fft2(uint32_t& x, uint32_t& y) {
    if constexpr (L != 255u) gf8_muladd_ct<L>(x, y);
    y ^= x;
}
// the same for two butterflies of one block whose y registers form a pair (shift2)
template <unsigned L>
__device__ __forceinline__ void ifft2x2(uint32_t& x0, uint32_t& x1, uint32_t& y0, uint32_t& y1) {
    y0 ^= x0;
    y1 ^= x1;
    if constexpr (L != 255u) gf8_muladd2_ct<L, L>(x0, x1, y0, y1);
}
template <unsigned L>
__device__ __forceinline__ void fft2x2(uint32_t& x0, uint32_t& x1, uint32_t& y0, uint32_t& y1) {
    if constexpr (L != 255u) gf8_muladd2_ct<L, L>(x0, x1, y0, y1);
    y0 ^= x0;
    y1 ^= x1;
}

// Inverse transform over N points, layer d = 1, 2, ..., N/2; block b uses
// SKEW[OFF + b + d]  (encoder: OFF = m - 1; decoder: OFF = -1).
template <int N, int OFF>
__device__ __forceinline__ void ifft_layers(uint32_t (&w)[N]) {
    static_for<16>([&](auto LG) {
        constexpr int lg = decltype(LG)::value;
        if constexpr ((1 << lg) < N) {
            constexpr int d = 1 << lg;
            static_for<N / (2 * d)>([&](auto B) {
                constexpr int b = decltype(B)::value * 2 * d;
                constexpr unsigned L = kGf8.skew[OFF + b + d];
                if constexpr (L == 255u) {
                    static_for<d>([&](auto Q) { w[b + decltype(Q)::value + d] ^= w[b + decltype(Q)::value]; });
                } else if constexpr (d >= 2 && kGf8Pair) {  // butterfly pairs: y registers i + d, i + d + 1
                    constexpr PermTab t = make_perm_tab(L);
                    const uint32_t ta = vconst<t.a_lo>(), tb = vconst<t.b_lo>();
                    static_for<d / 2>([&](auto Q) {
                        constexpr int i = b + 2 * decltype(Q)::value;
                        w[i + d] ^= w[i];
                        w[i + 1 + d] ^= w[i + 1];
                        gf8_muladd2_ct<L, L>(w[i], w[i + 1], w[i + d], w[i + 1 + d], ta, tb, ta, tb);
                    });
                } else {
                    constexpr PermTab t = make_perm_tab(L);
                    const uint32_t ta = vconst<t.a_lo>(), tb = vconst<t.b_lo>();
                    static_for<d>([&](auto Q) {
                        constexpr int i = b + decltype(Q)::value;
                        w[i + d] ^= w[i];
                        gf8_muladd_ct<L>(w[i], w[i + d], ta, tb);
                    });
                }
            });
        }
    });
}

// Forward transform, layer d = N/2, ..., 1; block b uses SKEW[OFF + b + d]
// (full transforms: OFF = -1; upper half of a 2N-point decoder transform: OFF = N - 1).
template <int N, int OFF = -1>
__device__ __forceinline__ void fft_layers(uint32_t (&w)[N]) {
    static_for<16>([&](auto LG) {
        constexpr int lg = 15 - decltype(LG)::value;
        if constexpr ((1 << lg) < N) {
            constexpr int d = 1 << lg;
            static_for<N / (2 * d)>([&](auto B) {
                constexpr int b = decltype(B)::value * 2 * d;
                constexpr unsigned L = kGf8.skew[OFF + b + d];
                if constexpr (L == 255u) {
                    static_for<d>([&](auto Q) { w[b + decltype(Q)::value + d] ^= w[b + decltype(Q)::value]; });
                } else if constexpr (d >= 2 && kGf8Pair) {  // butterfly pairs: y registers i + d, i + d + 1
                    constexpr PermTab t = make_perm_tab(L);
                    const uint32_t ta = vconst<t.a_lo>(), tb = vconst<t.b_lo>();
                    static_for<d / 2>([&](auto Q) {
                        constexpr int i = b + 2 * decltype(Q)::value;
                        gf8_muladd2_ct<L, L>(w[i], w[i + 1], w[i + d], w[i + 1 + d], ta, tb, ta, tb);
                        w[i + d] ^= w[i];
                        w[i + 1 + d] ^= w[i + 1];
                    });
                } else {
                    constexpr PermTab t = make_perm_tab(L);
                    const uint32_t ta = vconst<t.a_lo>(), tb = vconst<t.b_lo>();
                    static_for<d>([&](auto Q) {
                        constexpr int i = b + decltype(Q)::value;
                        gf8_muladd_ct<L>(w[i], w[i + d], ta, tb);
                        w[i + d] ^= w[i];
                    });
                }
            });
        }
    });
}

__device__ __forceinline__ uint64_t cw_rel(const CodewordSet& cs, uint32_t q) {
    if (cs.indices != nullptr) return (uint64_t)cs.indices[q] * cs.cw_stride;
    const uint32_t sq = q / cs.per_square;
    const uint32_t t = q - sq * cs.per_square;
    return (uint64_t)sq * cs.square_stride + (uint64_t)t * cs.cw_stride;
}

// Offsets at or beyond kOob are out of range for every buffer resource below:
// loads there return 0 and stores are dropped, so inactive lanes / padded symbols
// need no exec-mask branches.
constexpr uint32_t kOob = 0x80000000u;

// Buffer resource over a wave-uniform base: 32-bit per-lane voffset + SGPR soffset
// per symbol keeps address arithmetic off the VGPR file (guide T8/T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void* u = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(u, (short)0, (int)kOob, 0x00020000);
}

// ---------------------------------------------------------------------------
// Encode: k data symbols -> k parity symbols per byte position, for every
// codeword of a CodewordSet.  M = ceilPow2(k).
// ---------------------------------------------------------------------------
template <int M>
__global__ __launch_bounds__(256, 3) void encode_gf8_kernel(CodewordSet cs) {
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t chunks = cs.chunks;
    if (wave >= cs.count * chunks) return;
    const uint32_t q = wave / chunks;
    const uint32_t chunk = wave - q * chunks;
    const uint32_t off0 = chunk * 256u + lane * 4u;
    const uint32_t off = off0 < cs.S ? off0 : kOob;
    const uint64_t rel = cw_rel(cs, q);
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(cs.base + rel);
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(cs.out_base + rel);
    const uint32_t k = cs.k;
    const uint32_t es = (uint32_t)cs.elem_stride;

    uint32_t w[M];
    static_for<M>([&](auto E) {
        constexpr int e = decltype(E)::value;
        w[e] = __builtin_amdgcn_raw_buffer_load_b32(rs, off, e < (int)k ? e * es : kOob, 0);
    });
    if constexpr (M > 1) {
        ifft_layers<M, M - 1>(w);
        fft_layers<M>(w);
    }
    const uint32_t oo = (uint32_t)cs.out_offset;
    static_for<M>([&](auto E) {
        constexpr int e = decltype(E)::value;
        __builtin_amdgcn_raw_buffer_store_b32(w[e], ro, off, e < (int)k ? oo + e * es : kOob, 0);
    });
}

// Wide form (codewords whose halves span more than kOffsetLimit: columns of squares
// over 4 GiB): a 64-bit base per symbol, the same butterflies; a capped grid of
// one-wave workgroups loops over the tasks (M registers of state per lane).
template <int M>
__global__ __launch_bounds__(64) void encode_gf8_wide_kernel(CodewordSet cs) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t chunks = cs.chunks, k = cs.k;
    const uint32_t tasks = cs.count * chunks;
    for (uint32_t t = blockIdx.x; t < tasks; t += gridDim.x) {
        const uint32_t task = __builtin_amdgcn_readfirstlane(t);
        const uint32_t q = task / chunks;
        const uint32_t chunk = task - q * chunks;
        const uint32_t off0 = chunk * 256u + lane * 4u;
        const uint32_t off = off0 < cs.S ? off0 : kOob;
        const uint64_t rel = cw_rel(cs, q);
        uint32_t w[M];
        static_for<M>([&](auto E) {
            constexpr int e = decltype(E)::value;
            w[e] = (uint32_t)e < k ? __builtin_amdgcn_raw_buffer_load_b32(
                                         make_rsrc(cs.base + rel + (uint64_t)e * cs.elem_stride), off, 0, 0)
                                   : 0u;
        });
        if constexpr (M > 1) {
            ifft_layers<M, M - 1>(w);
            fft_layers<M>(w);
        }
        static_for<M>([&](auto E) {
            constexpr int e = decltype(E)::value;
            if ((uint32_t)e < k)
                __builtin_amdgcn_raw_buffer_store_b32(
                    w[e], make_rsrc(cs.out_base + rel + cs.out_offset + (uint64_t)e * cs.elem_stride), off, 0, 0);
        });
    }
}

// ---------------------------------------------------------------------------
// Decode (reconstruct, recoverAll): fills every missing symbol of the listed
// codewords in place.  Element e of codeword q: e < k data, k <= e < 2k parity.
// presence: byte per cell of the square ([W][W], non-zero = present).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t addmod8(uint32_t a, uint32_t b) {
    uint32_t s = a + b;
    return (s + (s >> 8)) & 255u;
}
__device__ __forceinline__ uint32_t submod8(uint32_t a, uint32_t b) {
    uint32_t d = a - b;
    return (d + (d >> 8)) & 255u;
}

// x of lane (lane ^ 2^LD), all 64 lanes active.  Lane-crossing without LDS round
// trips where the hardware has a direct form (ds_bpermute, the previous form, put
// 24 dependent LDS round trips on the decoder's error-locator path):
//   ^1, ^2: DPP quad_perm;  ^4: row_half_mirror (^7) then quad_perm [3,2,1,0] (^3);
//   ^8: DPP row_ror:8;  ^16: ds_swizzle SWAP 16;  ^32: v_permlane32_swap (gfx950).
template <int LD>
__device__ __forceinline__ uint32_t lane_xor(uint32_t x, uint32_t lane) {
    if constexpr (LD == 0) return __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, true);
    else if constexpr (LD == 1) return __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, true);
    else if constexpr (LD == 2)
        return __builtin_amdgcn_mov_dpp(__builtin_amdgcn_mov_dpp(x, 0x141, 0xF, 0xF, true), 0x1B, 0xF, 0xF, true);
    else if constexpr (LD == 3) return __builtin_amdgcn_mov_dpp(x, 0x128, 0xF, 0xF, true);
    else if constexpr (LD == 4) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x401F);
    else {
        const auto s = __builtin_amdgcn_permlane32_swap(x, x, false, false);  // [x_lo, x_lo], [x_hi, x_hi]
        return lane < 32u ? s[1] : s[0];
    }
}

// FWHT over 256 log-domain entries held 4 per lane (entry 4*lane + j in e[j]).
__device__ __forceinline__ void fwht256(uint32_t (&e)[4], uint32_t lane) {
    // dist 1, 2 inside the lane
    {
        uint32_t a0 = addmod8(e[0], e[1]), a1 = submod8(e[0], e[1]);
        uint32_t a2 = addmod8(e[2], e[3]), a3 = submod8(e[2], e[3]);
        e[0] = addmod8(a0, a2); e[2] = submod8(a0, a2);
        e[1] = addmod8(a1, a3); e[3] = submod8(a1, a3);
    }
    // dist 4..128 across lanes (partner lane = lane ^ (dist/4))
    static_for<6>([&](auto LDc) {
        constexpr int ld = decltype(LDc)::value;
        const bool upper = (lane & (1u << ld)) != 0;
        uint32_t p[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) p[j] = lane_xor<ld>(e[j], lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) e[j] = upper ? submod8(p[j], e[j]) : addmod8(e[j], p[j]);
    });
}

// Formal derivative restricted to one half (size H) of the 2H-point decoder
// transform: out[j] = in[j] ^ XOR_{t: bit t of j == 0, j + 2^t < H} in[j + 2^t].
// (The sequential reference loop, extendeddatacrossword -> leopard reconstruct
// "work <- FormalDerivative(work, n)", reads only not-yet-updated elements, so it
// equals this closed form; the 2^log2(H) cross-half term is added separately.)
template <int H>
__device__ __forceinline__ void derivative_half(uint32_t (&w)[H]) {
    static_for<H>([&](auto J) {
        constexpr int j = decltype(J)::value;
        static_for<16>([&](auto T) {
            constexpr int t = decltype(T)::value;
            if constexpr ((1 << t) < H && ((j >> t) & 1) == 0 && j + (1 << t) < H) w[j] ^= w[j + (1 << t)];
        });
    });
}

// One wavefront per (codeword, 256-byte chunk).  The n = 2m point decoder
// transform is run as two m-point halves: layers below m stay inside a half, so
// only one half lives in registers at a time and the other is parked in LDS
// (m x 64 dwords, lane-major: conflict-free).
// Cells: narrow form -- one buffer resource per half of the codeword (data cells
// e < k, parity cells k + i), 32-bit offsets i * cell_step * S within the half
// (narrow_fits); WIDE -- a 64-bit base per cell, cells `pitch` bytes apart.
template <int M, bool WIDE>
__device__ __forceinline__ void decode_gf8_task(const DecodeSet& ds, uint32_t wave, uint32_t (&park)[M][64]) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t chunks = ds.chunks;
    const uint32_t qi = wave / chunks;
    const uint32_t chunk = wave - qi * chunks;
    const uint32_t k = ds.k;
    const uint32_t W = 2u * k;
    const uint32_t vec = ds.indices[qi];
    // element e lives at cell (r, c): row vector -> (vec, e); col vector -> (e, vec)
    const uint64_t cell0 = ds.axis == 0 ? (uint64_t)vec * W : (uint64_t)vec;
    const uint64_t cell_step = ds.axis == 0 ? 1u : (uint64_t)W;

    // --- presence of the 2k elements as 64-bit ballots (wave-uniform) ---
    uint64_t pres[(2 * M + 63) / 64];
#pragma unroll
    for (int g = 0; g < (2 * M + 63) / 64; ++g) {
        const uint32_t e = g * 64u + lane;
        const bool p = e < W && ds.presence[cell0 + e * cell_step] != 0;
        pres[g] = __ballot(p);
    }
    auto present = [&](uint32_t e) -> bool { return (pres[e >> 6] >> (e & 63u)) & 1u; };

    // --- error locator (log domain), klauspost reconstruct: lane holds entries
    //     4*lane .. 4*lane+3 of the 256-entry table ---
    uint32_t er[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t i = lane * 4u + j;
        uint32_t v = 0;
        if (i < k) v = present(k + i) ? 0u : 1u;                     // parity i missing
        else if (i < (uint32_t)M) v = 1u;                            // recovery padding
        else if (i < (uint32_t)M + k) v = present(i - M) ? 0u : 1u;  // data i-M missing
        er[j] = v;
    }
    fwht256(er, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) er[j] = (er[j] * d_gf8.logwalsh[lane * 4u + j]) % 255u;
    fwht256(er, lane);
    const uint32_t er_packed = er[0] | (er[1] << 8) | (er[2] << 16) | (er[3] << 24);
    auto err_at = [&](int i) -> uint32_t {
        const uint32_t v = __builtin_amdgcn_readlane(er_packed, i >> 2);
        return (v >> (8 * (i & 3))) & 255u;
    };

    const uint32_t off0 = chunk * 256u + lane * 4u;
    const uint32_t off = off0 < ds.S ? off0 : kOob;
    const uint64_t pitch = WIDE && ds.pitch ? ds.pitch : ds.S;
    const __amdgpu_buffer_rsrc_t rd = make_rsrc(ds.base + cell0 * pitch);                            // data half
    const __amdgpu_buffer_rsrc_t rp = make_rsrc(ds.base + (cell0 + (uint64_t)k * cell_step) * pitch);  // parity half
    auto soff = [&](uint32_t i) -> uint32_t { return pin_sgpr((uint32_t)((uint64_t)i * cell_step * ds.S)); };
    // symbol i of a half (par: parity cell k + i, else data cell i)
    auto cell_rsrc = [&](uint32_t i, bool par) {
        return make_rsrc(ds.base + (cell0 + ((par ? (uint64_t)k : 0ull) + i) * cell_step) * pitch);
    };
    auto ld = [&](uint32_t i, bool par, bool ok) -> uint32_t {
        if constexpr (WIDE) return ok ? __builtin_amdgcn_raw_buffer_load_b32(cell_rsrc(i, par), off, 0, 0) : 0u;
        else return __builtin_amdgcn_raw_buffer_load_b32(par ? rp : rd, off, ok ? soff(i) : kOob, 0);
    };
    auto st = [&](uint32_t i, bool par, uint32_t v) {
        if constexpr (WIDE) __builtin_amdgcn_raw_buffer_store_b32(v, cell_rsrc(i, par), off, 0, 0);
        else __builtin_amdgcn_raw_buffer_store_b32(v, par ? rp : rd, off, soff(i), 0);
    };

    constexpr unsigned LM = kGf8.skew[M - 1];  // twiddle of the layer joining the halves
    uint32_t w[M];

    // 1. upper half: original data, scaled by the error locator; IFFT layers < M
    static_for<M>([&](auto E) {
        constexpr int e = decltype(E)::value;
        w[e] = ld(e, false, (uint32_t)e < k && present(e));
    });
    static_for<M>([&](auto E) {
        constexpr int e = decltype(E)::value;
        if ((uint32_t)e < k && present(e)) w[e] = gf8_mul_rt(w[e], err_at(M + e));
    });
    ifft_layers<M, M - 1>(w);
    static_for<M>([&](auto E) { park[decltype(E)::value][lane] = w[decltype(E)::value]; });

    // 2. lower half: recovery (parity) data; IFFT layers < M
    static_for<M>([&](auto E) {
        constexpr int e = decltype(E)::value;
        w[e] = ld(e, true, (uint32_t)e < k && present(k + e));
    });
    static_for<M>([&](auto E) {
        constexpr int e = decltype(E)::value;
        if ((uint32_t)e < k && present(k + e)) w[e] = gf8_mul_rt(w[e], err_at(e));
    });
    ifft_layers<M, -1>(w);

    // 3. IFFT layer M (pairs i, i+M), then derivative of the lower half plus the
    //    cross-half term x[j + M].
    static_for<M>([&](auto E) {
        constexpr int i = decltype(E)::value;
        uint32_t bv = park[i][lane];
        ifft2<LM>(w[i], bv);
        park[i][lane] = bv;
    });
    derivative_half<M>(w);
    static_for<M>([&](auto E) {
        constexpr int i = decltype(E)::value;
        const uint32_t bv = park[i][lane];
        w[i] ^= bv;
        park[i][lane] = w[i];  // park the finished lower half ...
        w[i] = bv;             // ... and bring the upper half into registers
    });

    // 4. derivative of the upper half; FFT layer M; FFT layers < M of the upper half
    derivative_half<M>(w);
    static_for<M>([&](auto E) {
        constexpr int i = decltype(E)::value;
        uint32_t av = park[i][lane];
        fft2<LM>(av, w[i]);
        park[i][lane] = av;
    });
    fft_layers<M, M - 1>(w);
    static_for<M>([&](auto E) {
        constexpr int e = decltype(E)::value;
        if ((uint32_t)e < k && !present(e)) st(e, false, gf8_mul_rt(w[e], 255u - err_at(M + e)));
    });

    // 5. lower half: FFT layers < M, reveal missing parity
    static_for<M>([&](auto E) { w[decltype(E)::value] = park[decltype(E)::value][lane]; });
    fft_layers<M, -1>(w);
    static_for<M>([&](auto E) {
        constexpr int e = decltype(E)::value;
        if ((uint32_t)e < k && !present(k + e)) st(e, true, gf8_mul_rt(w[e], 255u - err_at(e)));
    });
}

template <int M>
__global__ __launch_bounds__(64) void decode_gf8_kernel(DecodeSet ds) {
    __shared__ uint32_t park[M][64];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x);
    if (wave >= ds.count * ds.chunks) return;
    decode_gf8_task<M, false>(ds, wave, park);
}

// wide form: a capped grid of one-wave workgroups loops over the tasks (one wave
// per workgroup: the LDS park is reused in program order, no barrier needed)
template <int M>
__global__ __launch_bounds__(64) void decode_gf8_wide_kernel(DecodeSet ds) {
    __shared__ uint32_t park[M][64];
    const uint32_t tasks = ds.count * ds.chunks;
    for (uint32_t t = blockIdx.x; t < tasks; t += gridDim.x)
        decode_gf8_task<M, true>(ds, __builtin_amdgcn_readfirstlane(t), park);
}

// ---------------------------------------------------------------------------
// Split decoder for M = 128 (65 <= k <= 128, n = 256 points): one NW-wave
// workgroup per (codeword, 256-byte chunk), PW = 256 / NW points per wave.
//   S layout: wave w holds points e = PW w + j (j < PW): decoder IFFT layers
//             d < PW and FFT layers PW/2..1 (twiddles depend on w: one
//             compile-time variant per wave, selected by a wave-uniform branch);
//   L layout: wave w holds e = NW h + w (h < PW): IFFT layers PW..128, the formal
//             derivative and FFT layers 128..PW (twiddles independent of w).
// The derivative (closed form out[e] = in[e] ^ XOR_{t: e_t = 0} in[e + 2^t], see
// derivative_half) needs, in L, the partners across the low log2(NW) bits from
// the other waves: all waves publish their post-IFFT points to LDS once, then each
// adds the (original) partner values.  LDS: [256 points][64 lanes] dwords = 64 KiB
// + 15 KiB of multiply tables, so two workgroups share a CU (158 of 160 KiB).  Production NW = 16 (8 waves per SIMD: the
// shift/and/perm/xor chains of the byte-table multiplies need the latency cover;
// c3 sweep 42.5 / 33.7 / 32.0 us at NW = 4 / 8 / 16).
// ---------------------------------------------------------------------------
template <int PW, int W>
__device__ __forceinline__ void split_ifft_low(uint32_t (&v)[PW]) { ifft_layers<PW, PW * W - 1>(v); }
template <int PW, int W>
__device__ __forceinline__ void split_fft_low(uint32_t (&v)[PW]) { fft_layers<PW, PW * W - 1>(v); }

// wave-uniform dispatch of the per-wave twiddle variant
template <int NW, int PW, bool FFT>
__device__ __forceinline__ void split_low(uint32_t (&v)[PW], uint32_t w) {
    static_for<NW>([&](auto Wc) {
        constexpr int W = decltype(Wc)::value;
        if (w == (uint32_t)W) {
            if constexpr (FFT) split_fft_low<PW, W>(v);
            else split_ifft_low<PW, W>(v);
        }
    });
}

// L layout, layer d >= PW: e = NW h + w, so the partner e + d is register h + d / NW
// of the same wave; block start 2d * floor(e / 2d) = 2d * floor(h / (2d / NW)).
template <int NW, int PW, bool FFT>
__device__ __forceinline__ void split_high(uint32_t (&v)[PW]) {
    static_for<8>([&](auto LG) {
        constexpr int d = FFT ? (128 >> decltype(LG)::value) : (1 << decltype(LG)::value);
        if constexpr (d >= PW && d <= 128) {
            constexpr int sd = d / NW;
            static_for<PW>([&](auto H) {
                constexpr int h = decltype(H)::value;
                if constexpr (((h / sd) & 1) == 0) {
                    constexpr int b = 2 * d * (h / (2 * sd));
                    constexpr unsigned L = kGf8.skew[b + d - 1];
                    if constexpr (sd >= 2 && kGf8Pair) {  // pairs h, h + 1 of one block (shift2)
                        if constexpr ((h & 1) == 0) {
                            if constexpr (FFT) fft2x2<L>(v[h], v[h + 1], v[h + sd], v[h + sd + 1]);
                            else ifft2x2<L>(v[h], v[h + 1], v[h + sd], v[h + sd + 1]);
                        }
                    } else if constexpr (FFT) {
                        fft2<L>(v[h], v[h + sd]);
                    } else {
                        ifft2<L>(v[h], v[h + sd]);
                    }
                }
            });
        }
    });
}

// y * exp(L) with the table in registers (VGPR operands: read from LDS)
__device__ __forceinline__ uint32_t gf8_mul_tab(uint32_t y, const PermTab& t) {
    const uint32_t sa = y & 0x07070707u;
    const uint32_t sb = (y >> 3) & 0x07070707u;
    const uint32_t sc = (y >> 6) & 0x03030303u;
    return xor3(__builtin_amdgcn_perm(t.a_hi, t.a_lo, sa), __builtin_amdgcn_perm(t.b_hi, t.b_lo, sb),
                __builtin_amdgcn_perm(t.c, t.c, sc));
}

// two points at once, sharing their selector shifts (shift2)
__device__ __forceinline__ void gf8_mul_tab2(uint32_t& y0, uint32_t& y1, const PermTab& t0, const PermTab& t1) {
    const Shift2 q = shift2(y0, y1);
    const uint32_t a0 = y0 & 0x07070707u, a1 = y1 & 0x07070707u;
    const uint32_t b0 = q.b0 & 0x07070707u, b1 = q.b1 & 0x07070707u;
    const uint32_t c0 = q.c0 & 0x03030303u, c1 = q.c1 & 0x03030303u;
    y0 = xor3(__builtin_amdgcn_perm(t0.a_hi, t0.a_lo, a0), __builtin_amdgcn_perm(t0.b_hi, t0.b_lo, b0),
              __builtin_amdgcn_perm(t0.c, t0.c, c0));
    y1 = xor3(__builtin_amdgcn_perm(t1.a_hi, t1.a_lo, a1), __builtin_amdgcn_perm(t1.b_hi, t1.b_lo, b1),
              __builtin_amdgcn_perm(t1.c, t1.c, c1));
}

// bits [o, o + 64) of the 256-bit presence mask (zeros past the end)
__device__ __forceinline__ uint64_t pres_bits(const uint64_t (&pres)[4], uint32_t o) {
    const uint32_t q = o >> 6, r = o & 63u;
    const uint64_t lo = q < 4u ? pres[q] >> r : 0ull;
    const uint64_t hi = (r && q + 1u < 4u) ? pres[q + 1u] << (64u - r) : 0ull;
    return lo | hi;
}

// per-point multiply tables of one codeword: [0] scale by err[e] (all-zero for an
// absent point, so its bytes -- whatever the buffer holds -- enter as 0), [1]
// reveal by 255 - err[e].  Written once by wave 0; every wave reads them with
// uniform LDS broadcasts instead of a dependent scalar table load per point.
// diagnostic phase stamp (RSM_DIAG builds, ds.trace set): thread 0, 100 MHz clock
__device__ __forceinline__ void dec_stamp(const DecodeSet& ds, int i) {
#ifdef RSM_DIAG
    if (ds.trace && threadIdx.x == 0) {
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(ds.trace, (short)0, 0x7FFFFFFF, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32((uint32_t)__builtin_amdgcn_s_memrealtime(), r,
                                              (blockIdx.x * kDecTraceWords + i) * 4u, 0, 0);
    }
#else
    (void)ds;
    (void)i;
#endif
}

// WE ("wave error locator", round 5): every wave computes the error locator itself
// (the 256-entry FWHT pair, beside the other waves' identical copies) and multiplies
// its points by tables read with scalar loads (d_perm8, scalar-cache resident), so no
// wave waits for wave 0's locator, its per-point table resolution or the barrier
// after it; without WE wave 0 stages the tables in LDS (ptab) for all waves.
template <int NW, bool ZC, bool WE = false>
__device__ __forceinline__ void decode_split_task(const DecodeSet& ds, uint32_t task, uint32_t (&xch)[256][64],
                                                  PermTab (&ptab)[2][256], PermTab (&stab)[257]) {
    constexpr int PW = 256 / NW, HALF = NW / 2;
    if constexpr (!ZC) dec_stamp(ds, 0);
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t chunks = ds.chunks;
    const uint32_t qi = task / chunks;
    const uint32_t chunk = task - qi * chunks;
    const uint32_t k = ds.k;
    const uint32_t Wd = 2u * k;
    const uint32_t vec = __builtin_amdgcn_readfirstlane(ds.indices[qi]);
    const uint64_t cell0 = ds.axis == 0 ? (uint64_t)vec * Wd : (uint64_t)vec;
    const uint64_t cell_step = ds.axis == 0 ? 1u : (uint64_t)Wd;

    // This wave's points e = PW w + j are PW consecutive cell positions: recovery
    // (parity) i = e for w < NW/2, original (data) i = e - 128 for w >= NW/2; point j
    // is valid when i < k.  From HBM their loads go out first (independent of the
    // presence mask and the error locator, whose latency they overlap; an absent
    // point's bytes are multiplied by zero).  Zero-copy (ZC: inputs from host-mapped
    // memory over PCIe), only the present points are read: the presence mask comes
    // first, and the PCIe bytes halve.
    const uint32_t off0 = chunk * 256u + lane * 4u;
    const uint32_t off = off0 < ds.S ? off0 : kOob;
    // this wave's half of the codeword (parity cells k + i for w < NW/2, data cells i
    // otherwise) has its own 64-bit base; offsets within it are 32-bit (narrow_fits)
    const uint64_t hcell = (cell0 + (w < HALF ? (uint64_t)k * cell_step : 0ull)) * ds.S;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(ds.base + hcell);
    const bool mirror = ds.mirror != nullptr;  // rebuilt cells also written there
    const __amdgpu_buffer_rsrc_t ri = make_rsrc((ZC ? ds.in_base : ds.base) + hcell);
    const uint32_t ib = (w % HALF) * PW;
    const uint32_t nvalid = ib >= k ? 0u : (k - ib >= (uint32_t)PW ? (uint32_t)PW : k - ib);
    const uint32_t pstep = (uint32_t)(cell_step * ds.S);
    const uint32_t pbase = ib * pstep;
    const uint64_t valid = nvalid == 64u ? ~0ull : ((1ull << nvalid) - 1ull);
    uint32_t v[PW];
    auto load_points = [&](uint64_t mask) {
        static_for<PW>([&](auto J) {
            constexpr int j = decltype(J)::value;
            const uint32_t so = ((mask >> j) & 1ull) ? pbase + (uint32_t)j * pstep : kOob;
            v[j] = __builtin_amdgcn_raw_buffer_load_b32(ri, off, so, 0);
        });
    };
    // presence bytes first: the ballots (and wave 0's error locator) wait only for them,
    // while the points' loads -- issued right behind, an asm barrier keeps the order --
    // are still in flight (vmcnt retires in order: presence loads queued behind the
    // points made the locator wait for every point, 6.5 of 26 us per task,
    // profiles/r03_trace_decode.jsonl)
    // (diagnostic A/B, RSM_DIAG with ds.delay == kDecFloor: the setup-free floor of a
    // pre-pass design -- no presence loads, no error locator: a zero locator and every
    // other point present (BenchmarkRepair's count), wrong
    // output -- the time a decode kernel would take if a separate
    // per-codeword pre-pass had resolved presence and locator before it)
#ifdef RSM_DIAG
    const bool floor = WE && ds.delay == kDecFloor;
#else
    constexpr bool floor = false;
#endif
    uint32_t pv[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const uint32_t e = g * 64u + lane;
        pv[g] = e < Wd ? (floor ? ((e + vec) & 1u) : ds.presence[cell0 + e * cell_step]) : 0u;
    }
    // wave 0's error-locator weights and the 256 multiply tables (5 KiB, staged into
    // LDS for the per-point gathers below), also ahead of the points
    uint32_t lw[4] = {0, 0, 0, 0};
    constexpr int kTabWords = 256 * 5 / 64;
    uint32_t sv[kTabWords];
    if constexpr (WE) {
#pragma unroll
        for (int j = 0; j < 4; ++j) lw[j] = d_gf8.logwalsh[lane * 4u + j];
    } else if (w == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) lw[j] = d_gf8.logwalsh[lane * 4u + j];
        const uint32_t* tw = reinterpret_cast<const uint32_t*>(&d_perm8.t[0]);
#pragma unroll
        for (int i = 0; i < kTabWords; ++i) sv[i] = tw[i * 64 + lane];
    }
    asm volatile("" ::: "memory");
#ifdef RSM_DIAG
    if constexpr (!ZC) {
        if (ds.delay && ds.delay != kDecFloor && blockIdx.x >= gridDim.x / 2u) {  // A/B: stagger the two halves' loads
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (__builtin_amdgcn_s_memrealtime() - t0 < ds.delay) __builtin_amdgcn_s_sleep(2);
        }
    }
#endif
    if constexpr (!ZC) load_points(valid);
    if (!WE && w == 0) {
        uint32_t* st = reinterpret_cast<uint32_t*>(&stab[0]);
#pragma unroll
        for (int i = 0; i < kTabWords; ++i) st[i * 64 + lane] = sv[i];
        if (lane < 5u) st[256 * 5 + lane] = 0u;  // entry 256: the zero multiplier
    }

    uint64_t pres[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) pres[g] = __ballot(pv[g] != 0);
    auto present = [&](uint32_t e) -> bool { return (pres[e >> 6] >> (e & 63u)) & 1u; };
    const uint64_t have = pres_bits(pres, w < HALF ? k + ib : ib) & valid;
    if constexpr (!ZC) dec_stamp(ds, 1);
    if constexpr (ZC) load_points(have);

    // error locator (log domain), as decode_gf8_kernel: entries 4 lane .. 4 lane + 3;
    // wave 0 alone: it resolves each point's multiply table (ptab: the staged table of
    // exp(err) / exp(-err), so every wave's per-point multiply is ONE uniform LDS read)
    // the staged table of its own points
    uint32_t er_packed = 0;  // (WE) this wave's copy of the locator, 4 entries per lane
    if constexpr (WE) {
        uint32_t er[4] = {0u, 0u, 0u, 0u};
        if (!floor) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t i = lane * 4u + j;
            uint32_t x = 0;
            if (i < k) x = present(k + i) ? 0u : 1u;
            else if (i < 128u) x = 1u;
            else if (i < 128u + k) x = present(i - 128u) ? 0u : 1u;
            er[j] = x;
        }
        fwht256(er, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) er[j] = (er[j] * lw[j]) % 255u;
        fwht256(er, lane);
        }
        er_packed = er[0] | (er[1] << 8) | (er[2] << 16) | (er[3] << 24);
    } else if (w == 0) {
        uint32_t er[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t i = lane * 4u + j;
            uint32_t x = 0;
            if (i < k) x = present(k + i) ? 0u : 1u;
            else if (i < 128u) x = 1u;
            else if (i < 128u + k) x = present(i - 128u) ? 0u : 1u;
            er[j] = x;
        }
        fwht256(er, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) er[j] = (er[j] * lw[j]) % 255u;
        fwht256(er, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t e = lane * 4u + j;  // point e: a present, valid input?
            const uint32_t i = e < 128u ? e : e - 128u;
            const bool in = i < k && present(e < 128u ? k + e : i);
            ptab[0][e] = stab[in ? er[j] : 256u];  // scale by exp(err), 256: absent -> 0
            ptab[1][e] = stab[255u - er[j]];       // reveal
        }
    }
    if constexpr (ZC) {  // the present cells also land in the device square
        static_for<PW>([&](auto J) {
            constexpr int j = decltype(J)::value;
            const uint32_t so = ((have >> j) & 1ull) ? pbase + (uint32_t)j * pstep : kOob;
            __builtin_amdgcn_raw_buffer_store_b32(v[j], rs, off, so, 0);
        });
    }
    if constexpr (!WE) __syncthreads();
    if constexpr (!ZC) dec_stamp(ds, 2);
    // (WE) locator entry of point e: byte e & 3 of lane e >> 2 (a wave-uniform readlane)
    auto err_of = [&](uint32_t e) -> uint32_t {
        return (__builtin_amdgcn_readlane(er_packed, e >> 2) >> (8u * (e & 3u))) & 255u;
    };

    // 1. S layout: scale every point by the error locator (absent -> 0)
    static_for<PW>([&](auto J) {
        constexpr int j = decltype(J)::value;
        if constexpr (WE) v[j] = ((have >> j) & 1ull) ? gf8_mul_rt(v[j], err_of(PW * w + j)) : 0u;
        else if constexpr (ZC || !kGf8Pair) v[j] = gf8_mul_tab(v[j], ptab[0][PW * w + j]);  // (paired: spills at NW = 4)
        else if constexpr ((j & 1) == 0) gf8_mul_tab2(v[j], v[j + 1], ptab[0][PW * w + j], ptab[0][PW * w + j + 1]);
    });
    // 2. IFFT layers 1..PW/2 (per-wave twiddles)
    split_low<NW, PW, false>(v, w);
    if constexpr (!ZC) dec_stamp(ds, 3);
    // 3. S -> L
    static_for<PW>([&](auto J) { xch[PW * w + decltype(J)::value][lane] = v[decltype(J)::value]; });
    __syncthreads();
    static_for<PW>([&](auto H) { v[decltype(H)::value] = xch[NW * decltype(H)::value + w][lane]; });
    __syncthreads();
    // 4. IFFT layers PW..128; formal derivative
    split_high<NW, PW, false>(v);
    static_for<PW>([&](auto H) { xch[NW * decltype(H)::value + w][lane] = v[decltype(H)::value]; });
    __syncthreads();
    static_for<PW>([&](auto H) {  // partners across the high bits: same wave, registers h + 2^t
        constexpr int h = decltype(H)::value;
        static_for<8>([&](auto T) {
            constexpr int t = decltype(T)::value;
            if constexpr ((1 << t) < PW && ((h >> t) & 1) == 0) v[h] ^= v[h + (1 << t)];
        });
    });
    static_for<8>([&](auto B) {  // partners across the low bits: wave w + 2^b (bit b of e is 0)
        constexpr int bit = 1 << decltype(B)::value;
        if constexpr (bit < NW)
            if ((w & (uint32_t)bit) == 0)
                static_for<PW>([&](auto H) {
                    v[decltype(H)::value] ^= xch[NW * decltype(H)::value + w + bit][lane];
                });
    });
    if constexpr (!ZC) dec_stamp(ds, 4);
    // 5. FFT layers 128..PW; L -> S
    split_high<NW, PW, true>(v);
    __syncthreads();
    static_for<PW>([&](auto H) { xch[NW * decltype(H)::value + w][lane] = v[decltype(H)::value]; });
    __syncthreads();
    static_for<PW>([&](auto J) { v[decltype(J)::value] = xch[PW * w + decltype(J)::value][lane]; });
    if constexpr (!ZC) dec_stamp(ds, 5);
    // 6. FFT layers PW/2..1; reveal the missing points of this wave
    split_low<NW, PW, true>(v, w);
    if constexpr (!ZC) dec_stamp(ds, 6);
    const uint64_t reveal = valid & ~have;
    const __amdgpu_buffer_rsrc_t rm = make_rsrc((mirror ? ds.mirror : ds.base) + hcell);
    uint32_t sbase = pbase, sstep = pstep;
    asm volatile("" : "+s"(sbase), "+s"(sstep));
    static_for<PW / 2>([&](auto J2) {  // points j, j + 1 (gf8_mul_tab2: shared selector shifts)
        constexpr int j = 2 * decltype(J2)::value;
        const uint32_t e = PW * w + j;
        uint32_t x[2];
        if constexpr (WE) {
            x[0] = ((reveal >> j) & 1ull) ? gf8_mul_rt(v[j], 255u - err_of(e)) : 0u;
            x[1] = ((reveal >> (j + 1)) & 1ull) ? gf8_mul_rt(v[j + 1], 255u - err_of(e + 1)) : 0u;
        } else if constexpr (ZC || !kGf8Pair) {
            x[0] = gf8_mul_tab(v[j], ptab[1][e]);
            x[1] = gf8_mul_tab(v[j + 1], ptab[1][e + 1]);
        } else {
            x[0] = v[j];
            x[1] = v[j + 1];
            gf8_mul_tab2(x[0], x[1], ptab[1][e], ptab[1][e + 1]);
        }
        static_for<2>([&](auto U) {
            constexpr int u = decltype(U)::value;
            const uint32_t so = ((reveal >> (j + u)) & 1ull) ? sbase + (uint32_t)(j + u) * sstep : kOob;
            __builtin_amdgcn_raw_buffer_store_b32(x[u], rs, off, so, 0);
            if (mirror) __builtin_amdgcn_raw_buffer_store_b32(x[u], rm, off, so, 0);
        });
    });
    if constexpr (!ZC) dec_stamp(ds, 7);
}

constexpr int kSplitWaves = 16;

// one workgroup per task (device-resident square)
template <int NW, bool WE = false>
__global__ __launch_bounds__(64 * NW, NW / 2) void decode_gf8_split_kernel(DecodeSet ds) {
    __shared__ uint32_t xch[256][64];
    __shared__ PermTab ptab[WE ? 1 : 2][256];  // (unused by WE)
    __shared__ PermTab stab[WE ? 1 : 257];
    decode_split_task<NW, false, WE>(ds, blockIdx.x, xch, reinterpret_cast<PermTab (&)[2][256]>(ptab),
                                     reinterpret_cast<PermTab (&)[257]>(stab));
}

// zero-copy form: a capped grid loops over the tasks
template <int NW>
__global__ __launch_bounds__(64 * NW, NW / 2) void decode_gf8_split_zc_kernel(DecodeSet ds) {
    __shared__ uint32_t xch[256][64];
    __shared__ PermTab ptab[2][256];
    __shared__ PermTab stab[257];
    const uint32_t tasks = ds.count * ds.chunks;
    for (uint32_t task = blockIdx.x; task < tasks; task += gridDim.x) {
        decode_split_task<NW, true>(ds, __builtin_amdgcn_readfirstlane(task), xch, ptab, stab);
        __syncthreads();  // LDS (xch, ptab, stab) is reused by the next task
    }
}


// ---------------------------------------------------------------------------
// Split encoder for M = 128 (65 <= k <= 128): the LATENCY form, for one or a few
// squares (a single square has only 96 sets of the bit-sliced kernel's 2 KiB width,
// and its row -> column dependency puts two ~16 us sets on the critical path).  One
// NW-wave workgroup per (codeword, 256-byte chunk), the codewords of up to two
// CodewordSets in one grid (rows of Q0 -> Q1 together with columns of Q0 -> Q2), so
// a square's first phase fills every CU; PW = 128 / NW points per wave:
//   S layout: wave w holds points e = PW w + j (j < PW): IFFT layers d < PW (offset
//             m - 1 = 127) and FFT layers PW/2..1 (offset -1) with per-wave twiddles
//             (one compile-time variant per wave, chosen by a wave-uniform branch);
//   L layout: wave w holds e = NW h + w (h < PW): IFFT layers PW..64 and FFT layers
//             64..PW (the top pair merged), twiddles independent of w (d >= PW >= NW).
// Same butterflies as encode_gf8_kernel<128> (klauspost leopard8
// ifftDITEncoder8 / fftDIT8), so the same parity; LDS [128 points][64 lanes] dwords.
// ---------------------------------------------------------------------------
constexpr int ilog2_ct(int x) { return x <= 1 ? 0 : 1 + ilog2_ct(x / 2); }
constexpr unsigned log_of_sum8(unsigned L1, unsigned L2) {
    const unsigned a = L1 == 255u ? 0u : kGf8.exp[L1], b = L2 == 255u ? 0u : kGf8.exp[L2];
    return (a ^ b) == 0u ? 255u : kGf8.log[a ^ b];
}
template <int NW, int PW, bool FFT, int M = 128>
__device__ __forceinline__ void enc_split_high(uint32_t (&v)[PW]) {
    constexpr int NL = ilog2_ct(M) - 1;  // layers d = 1 .. M/4
    static_for<NL>([&](auto LG) {  // d = max(PW, NW) .. M/4: the top layer d = M/2 is enc_split_mid
        constexpr int d = FFT ? ((M / 4) >> decltype(LG)::value) : (1 << decltype(LG)::value);
        if constexpr (d >= PW && d >= NW) {
            constexpr int sd = d / NW;
            static_for<PW>([&](auto H) {
                constexpr int h = decltype(H)::value;
                if constexpr (((h / sd) & 1) == 0) {
                    constexpr int b = 2 * d * (h / (2 * sd));
                    constexpr unsigned L = kGf8.skew[(FFT ? -1 : M - 1) + b + d];
                    if constexpr (sd >= 2 && kGf8Pair) {  // pairs h, h + 1 of one block (shift2)
                        if constexpr ((h & 1) == 0) {
                            if constexpr (FFT) fft2x2<L>(v[h], v[h + 1], v[h + sd], v[h + sd + 1]);
                            else ifft2x2<L>(v[h], v[h + 1], v[h + sd], v[h + sd + 1]);
                        }
                    } else if constexpr (FFT) {
                        fft2<L>(v[h], v[h + sd]);
                    } else {
                        ifft2<L>(v[h], v[h + sd]);
                    }
                }
            });
        }
    });
}
// The last IFFT layer and the first FFT layer (d = 64) join the same pairs: one
// multiply by exp(L1) + exp(L2) instead of two (bs8.hpp mid2, by linearity):
// y ^= x; x ^= y * (exp L1 + exp L2); y ^= x.
template <int NW, int PW, int M = 128>
__device__ __forceinline__ void enc_split_mid(uint32_t (&v)[PW]) {
    constexpr int sd = (M / 2) / NW;
    constexpr unsigned L = log_of_sum8(kGf8.skew[M - 1 + M / 2], kGf8.skew[-1 + M / 2]);
    static_for<PW>([&](auto H) {
        constexpr int h = decltype(H)::value;
        if constexpr (kGf8Pair && sd >= 2 && ((h / sd) & 1) == 0 && (h & 1) == 0) {  // pairs h, h + 1 (shift2)
            v[h + sd] ^= v[h];
            v[h + sd + 1] ^= v[h + 1];
            if constexpr (L != 255u) gf8_muladd2_ct<L, L>(v[h], v[h + 1], v[h + sd], v[h + sd + 1]);
            v[h + sd] ^= v[h];
            v[h + sd + 1] ^= v[h + 1];
        } else if constexpr ((!kGf8Pair || sd < 2) && ((h / sd) & 1) == 0) {
            v[h + sd] ^= v[h];
            if constexpr (L != 255u) gf8_muladd_ct<L>(v[h], v[h + sd]);
            v[h + sd] ^= v[h];
        }
    });
}
template <int NW, int PW, bool FFT, int M = 128>
__device__ __forceinline__ void enc_split_low(uint32_t (&v)[PW], uint32_t w) {
    static_for<NW>([&](auto Wc) {
        constexpr int W = decltype(Wc)::value;
        if (w == (uint32_t)W) {
            if constexpr (FFT) fft_layers<PW, PW * W - 1>(v);
            else ifft_layers<PW, M - 1 + PW * W>(v);
        }
    });
}

struct SplitEncPlan {
    CodewordSet cs[3];
    uint32_t n0, n1, n2;  // tasks of cs[0], cs[1], cs[2] (in this order of block index)
    // fused form (one square: every workgroup co-resident): cs[0] = rows of Q0 -> Q1,
    // cs[1] = columns of Q0 -> Q2, cs[2] = columns of Q1 -> Q3, whose workgroups wait
    // for every row task (ctr[0] == n0); ctr[32] counts finished Q1-column tasks, the
    // last one re-zeroes both words; err: pinned host word set by a stuck wait
    uint32_t* ctr;
    uint32_t* err;
    uint32_t fused;
};
constexpr uint32_t kSplitSpinLimit = 1u << 20;  // polls (~1 s) before a wait is declared stuck
constexpr uint32_t kSplitFlag0 = 256;  // the fused form's 64 done flags: words 256 + 16 x (1280 words in all)

template <int NW>
__global__ __launch_bounds__(64 * NW) void encode_gf8_split_kernel(SplitEncPlan p) {
    constexpr int PW = 128 / NW;
    // every layer d < PW is in S and every d >= PW must be in-register in L (d a
    // multiple of NW): PW >= NW
    static_assert(PW * NW == 128 && PW >= NW, "split encoder shape");
    __shared__ uint32_t xch[128][64];
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t task = blockIdx.x;
    const uint32_t kind = task < p.n0 ? 0u : (task < p.n0 + p.n1 ? 1u : 2u);
    task -= kind == 0u ? 0u : (kind == 1u ? p.n0 : p.n0 + p.n1);
    const CodewordSet& cs = p.cs[kind];
    const bool fused = p.fused != 0u;
    // fused form: the rows and the Q1 columns are the critical path, the Q0 columns
    // fill the issue slots they leave (wave priority)
    if (fused && kind != 1u) __builtin_amdgcn_s_setprio(3);
    if (fused && kind == 2u) {
        // wait for every row task's Q1: the row task whose counter add comes last sets
        // 64 replicated done flags (one 64-B line each, kSplitFlag0 + 16 x), and this
        // workgroup polls its own line -- 256 pollers on the counter word itself slowed
        // the row tasks' memory traffic; then ONE agent acquire before the barrier that
        // precedes this workgroup's loads (hand-off argument)
        if (threadIdx.x == 0) {
            uint32_t n = 0;
            const uint32_t* flag = p.ctr + kSplitFlag0 + 16u * (blockIdx.x & 63u);
            while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
                if (++n >= kSplitSpinLimit) {
                    __hip_atomic_store(p.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        __syncthreads();
    }
    const uint32_t chunks = cs.chunks;
    const uint32_t q = task / chunks;
    const uint32_t chunk = task - q * chunks;
    const uint32_t off0 = chunk * 256u + lane * 4u;
    const uint32_t off = off0 < cs.S ? off0 : kOob;
    const uint64_t rel = cw_rel(cs, q);
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(cs.base + rel);
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(cs.out_base + rel);
    const uint32_t k = cs.k, es = (uint32_t)cs.elem_stride, oo = (uint32_t)cs.out_offset;
    uint32_t v[PW];
    static_for<PW>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t e = PW * w + j;
        v[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, off, e < k ? e * es : kOob, 0);
    });
    enc_split_low<NW, PW, false>(v, w);
    static_for<PW>([&](auto J) { xch[PW * w + decltype(J)::value][lane] = v[decltype(J)::value]; });
    __syncthreads();
    static_for<PW>([&](auto H) { v[decltype(H)::value] = xch[NW * decltype(H)::value + w][lane]; });
    enc_split_high<NW, PW, false>(v);
    enc_split_mid<NW, PW>(v);
    enc_split_high<NW, PW, true>(v);
    __syncthreads();
    static_for<PW>([&](auto H) { xch[NW * decltype(H)::value + w][lane] = v[decltype(H)::value]; });
    __syncthreads();
    static_for<PW>([&](auto J) { v[decltype(J)::value] = xch[PW * w + decltype(J)::value][lane]; });
    enc_split_low<NW, PW, true>(v, w);
    const bool handoff = fused && kind == 0u;  // Q1 of the fused form: write-through (sc1)
    static_for<PW>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t e = PW * w + j;
        const uint32_t so = e < k ? oo + e * es : kOob;
        if (handoff) __builtin_amdgcn_raw_buffer_store_b32(v[j], ro, off, so, 16);
        else __builtin_amdgcn_raw_buffer_store_b32(v[j], ro, off, so, 0);
    });
    if (handoff) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // the last row task (its add returns n0 - 1: every other row task's add, each
        // behind its own write-through stores, came before) sets the 64 done flags,
        // one lane per line, after its add has returned
        uint32_t last = 0;
        if (threadIdx.x == 0)
            last = __hip_atomic_fetch_add(p.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == p.n0 - 1u;
        if (threadIdx.x < 64u && __builtin_amdgcn_readfirstlane(last))
            __hip_atomic_store(p.ctr + kSplitFlag0 + 16u * threadIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (fused && kind == 2u && threadIdx.x < 64u) {
        uint32_t last = 0;
        if (threadIdx.x == 0)
            last = __hip_atomic_fetch_add(p.ctr + 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == p.n2 - 1u;
        if (__builtin_amdgcn_readfirstlane(last)) {  // every waiter is past its wait: re-zero for the next launch
            __hip_atomic_store(p.ctr + kSplitFlag0 + 16u * threadIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (threadIdx.x == 0) {
                __hip_atomic_store(p.ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(p.ctr + 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}
// ---------------------------------------------------------------------------
// 16-wave latency form (round 6; production for one square and the per-codeword codec,
// kSplitWavesOne; diagnostic builds: rsm_diag_set_split_waves 16): PW = 8 points per wave, so each wave's chain of butterflies is half as long and a launch
// has twice the waves to hide its latencies.  Three register bits cannot hold the
// layer bits 3..6 in one window, so there are three layouts:
//   S: wave w, register j: e = 8w + j                         IFFT d = 1, 2, 4; FFT 4, 2, 1
//   M: wave w, register r: e = (w & 7) + 64 (w >> 3) + 8 m(r)  IFFT d = 8; FFT d = 8
//      m(r) = e bits 3..5 = r bits (1, 0, 2): the two d = 8 butterflies of a register
//      quad have adjacent y registers, so they share their selector shifts
//   L: wave w, register h: e = w + 16 h                       IFFT d = 16, 32, the merged
//                                                             d = 64 pair, FFT 32, 16
// Four LDS exchanges through two alternating [128][64] buffers: one barrier each (a
// buffer is rewritten only after the barrier of the exchange in between, which every
// wave reaches after its reads of that buffer).
// ---------------------------------------------------------------------------
__device__ __forceinline__ constexpr uint32_t split16_m(int r) {
    return 8u * (uint32_t)(((r >> 1) & 1) | ((r & 1) << 1) | (r & 4));
}
// d = 8 in M: quads (R, R+1 | R+2, R+3), x = e bit 3 clear; U = w >> 3 (e bit 6)
template <int U, bool FFT>
__device__ __forceinline__ void split16_layer8(uint32_t (&v)[8]) {
    static_for<2>([&](auto B2) {
        constexpr int R = 4 * decltype(B2)::value;
        constexpr int blk = 64 * U + 32 * decltype(B2)::value;  // block start for e bit 4 = 0; + 16 for bit 4 = 1
        constexpr unsigned L0 = kGf8.skew[(FFT ? -1 : 127) + blk + 8];
        constexpr unsigned L1 = kGf8.skew[(FFT ? -1 : 127) + blk + 16 + 8];
        if constexpr (!FFT) {
            v[R + 2] ^= v[R];
            v[R + 3] ^= v[R + 1];
        }
        if constexpr (L0 != 255u && L1 != 255u) {
            gf8_muladd2_ct<L0, L1>(v[R], v[R + 1], v[R + 2], v[R + 3]);
        } else {
            if constexpr (L0 != 255u) gf8_muladd_ct<L0>(v[R], v[R + 2]);
            if constexpr (L1 != 255u) gf8_muladd_ct<L1>(v[R + 1], v[R + 3]);
        }
        if constexpr (FFT) {
            v[R + 2] ^= v[R];
            v[R + 3] ^= v[R + 1];
        }
    });
}

// S-layout twiddles of the 16-wave form as per-wave runtime tables (round 6, A/B): one
// code path for all 16 waves instead of 16 compile-time variants (~16x the S-layout
// code), to test whether the short launches wait on instruction-cache misses.  Wave w's tables (scalar loads, SGPR operands): [dir]
// [d = 1: blocks 0..3 | d = 2: blocks 0..1 | d = 4], an all-zero table for SKEW = 255.
struct Split16Tw {
    PermTab t[2][7];
};
struct Split16TwAll {
    Split16Tw w[16];
};
constexpr Split16TwAll make_split16_tw() {
    Split16TwAll a{};
    for (int w = 0; w < 16; ++w)
        for (int dir = 0; dir < 2; ++dir)
            for (int lg = 0; lg < 3; ++lg) {
                const int d = 1 << lg;
                for (int B = 0; B < 8 / (2 * d); ++B) {
                    const int ti = lg == 0 ? B : (lg == 1 ? 4 + B : 6);
                    const unsigned L = kGf8.skew[(dir ? 8 * w - 1 : 127 + 8 * w) + 2 * d * B + d];
                    a.w[w].t[dir][ti] = L == 255u ? PermTab{} : make_perm_tab(L);
                }
            }
    return a;
}
__constant__ Split16TwAll d_split16_tw = make_split16_tw();

// x ^= y * t with a wave-uniform runtime table t (SGPRs) and its VGPR halves ta / tb, from
// y and its pre-shifted selector sources (as gf8_muladd_sel)
__device__ __forceinline__ void gf8_muladd_sel_rt(uint32_t& x, uint32_t y, uint32_t y3, uint32_t y6, const PermTab& t,
                                                  uint32_t ta, uint32_t tb) {
    uint32_t sa, sb, sc;
    asm("v_and_b32 %[sa], %[m7], %[y]\n\t"
        "v_and_b32 %[sb], %[m7], %[y3]\n\t"
        "v_and_b32 %[sc], %[m3], %[y6]\n\t"
        "v_perm_b32 %[sa], %[ahi], %[ta], %[sa]\n\t"
        "v_perm_b32 %[sb], %[bhi], %[tb], %[sb]\n\t"
        "v_perm_b32 %[sc], %[cc], %[cc], %[sc]\n\t"
        "v_bitop3_b32 %[x], %[x], %[sa], %[sb] bitop3:0x96\n\t"
        "v_xor_b32 %[x], %[x], %[sc]"
        : [x] "+v"(x), [sa] "=&v"(sa), [sb] "=&v"(sb), [sc] "=&v"(sc)
        : [y] "v"(y), [y3] "v"(y3), [y6] "v"(y6), [ta] "v"(ta), [tb] "v"(tb), [m7] "i"(0x07070707),
          [m3] "i"(0x03030303), [ahi] "s"(t.a_hi), [bhi] "s"(t.b_hi), [cc] "s"(t.c));
}
// S layout, all three layers of one direction, with wave w's runtime tables
template <bool FFT>
__device__ __forceinline__ void split16_low_rt(uint32_t (&v)[8], const Split16Tw& tw) {
    static_for<3>([&](auto LGi) {
        constexpr int lg = FFT ? 2 - decltype(LGi)::value : decltype(LGi)::value;
        constexpr int d = 1 << lg;
        static_for<8 / (2 * d)>([&](auto B) {
            constexpr int b = decltype(B)::value * 2 * d;
            constexpr int ti = lg == 0 ? decltype(B)::value : (lg == 1 ? 4 + decltype(B)::value : 6);
            const PermTab t = tw.t[FFT ? 1 : 0][ti];
            const uint32_t ta = t.a_lo, tb = t.b_lo;
            if constexpr (d == 1) {
                if constexpr (!FFT) v[b + 1] ^= v[b];
                const uint32_t y = v[b + 1];
                gf8_muladd_sel_rt(v[b], y, y >> 3, y >> 6, t, ta, tb);
                if constexpr (FFT) v[b + 1] ^= v[b];
            } else {
                static_for<d / 2>([&](auto Q) {
                    constexpr int i = b + 2 * decltype(Q)::value;
                    if constexpr (!FFT) {
                        v[i + d] ^= v[i];
                        v[i + 1 + d] ^= v[i + 1];
                    }
                    const Shift2 q = shift2(v[i + d], v[i + 1 + d]);
                    gf8_muladd_sel_rt(v[i], v[i + d], q.b0, q.c0, t, ta, tb);
                    gf8_muladd_sel_rt(v[i + 1], v[i + 1 + d], q.b1, q.c1, t, ta, tb);
                    if constexpr (FFT) {
                        v[i + d] ^= v[i];
                        v[i + 1 + d] ^= v[i + 1];
                    }
                });
            }
        });
    });
}
// Measured slower than the 16 compile-time variants (21.8 against 21.1 us per square, same
// box, profiles/r06o_split16_ab.jsonl): the instruction cache was not what the short
// launches wait on.  Diagnostic A/B builds only.
#ifdef RSM_SPLIT16_RT
constexpr bool kSplit16Rt = true;
#else
constexpr bool kSplit16Rt = false;
#endif

__global__ __launch_bounds__(1024, 8) void encode_gf8_split16_kernel(SplitEncPlan p) {
    constexpr int NW = 16, PW = 8;
    __shared__ uint32_t xch[2][128][64];
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t task = blockIdx.x;
    const uint32_t kind = task < p.n0 ? 0u : 1u;
    task -= kind == 0u ? 0u : p.n0;
    const CodewordSet& cs = p.cs[kind];
    const uint32_t chunks = cs.chunks;
    const uint32_t q = task / chunks;
    const uint32_t chunk = task - q * chunks;
    const uint32_t off0 = chunk * 256u + lane * 4u;
    const uint32_t off = off0 < cs.S ? off0 : kOob;
    const uint64_t rel = cw_rel(cs, q);
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(cs.base + rel);
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(cs.out_base + rel);
    const uint32_t k = cs.k, es = (uint32_t)cs.elem_stride, oo = (uint32_t)cs.out_offset;
    const uint32_t mb = (w & 7u) + 64u * (w >> 3);  // M layout: e of register r = mb + split16_m(r)
    uint32_t v[PW];
    static_for<PW>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t e = PW * w + j;
        v[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, off, e < k ? e * es : kOob, 0);
    });
    if constexpr (kSplit16Rt) split16_low_rt<false>(v, d_split16_tw.w[w]);  // S: IFFT d = 1, 2, 4
    else enc_split_low<NW, PW, false>(v, w);
    static_for<PW>([&](auto J) { xch[0][PW * w + decltype(J)::value][lane] = v[decltype(J)::value]; });
    __syncthreads();
    static_for<PW>([&](auto R) { v[decltype(R)::value] = xch[0][mb + split16_m(decltype(R)::value)][lane]; });
    if (w < 8u) split16_layer8<0, false>(v);  // M: IFFT d = 8
    else split16_layer8<1, false>(v);
    static_for<PW>([&](auto R) { xch[1][mb + split16_m(decltype(R)::value)][lane] = v[decltype(R)::value]; });
    __syncthreads();
    static_for<PW>([&](auto H) { v[decltype(H)::value] = xch[1][w + NW * decltype(H)::value][lane]; });
    enc_split_high<NW, PW, false>(v);  // L: IFFT d = 16, 32; merged d = 64; FFT 32, 16
    enc_split_mid<NW, PW>(v);
    enc_split_high<NW, PW, true>(v);
    static_for<PW>([&](auto H) { xch[0][w + NW * decltype(H)::value][lane] = v[decltype(H)::value]; });
    __syncthreads();
    static_for<PW>([&](auto R) { v[decltype(R)::value] = xch[0][mb + split16_m(decltype(R)::value)][lane]; });
    if (w < 8u) split16_layer8<0, true>(v);  // M: FFT d = 8
    else split16_layer8<1, true>(v);
    static_for<PW>([&](auto R) { xch[1][mb + split16_m(decltype(R)::value)][lane] = v[decltype(R)::value]; });
    __syncthreads();
    static_for<PW>([&](auto J) { v[decltype(J)::value] = xch[1][PW * w + decltype(J)::value][lane]; });
    if constexpr (kSplit16Rt) split16_low_rt<true>(v, d_split16_tw.w[w]);  // S: FFT d = 4, 2, 1
    else enc_split_low<NW, PW, true>(v, w);
    static_for<PW>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t e = PW * w + j;
        __builtin_amdgcn_raw_buffer_store_b32(v[j], ro, off, e < k ? oo + e * es : kOob, 0);
    });
}

// ---------------------------------------------------------------------------
// Latency form for M = 16, 32 and 64 (9 <= k <= 64, round 6): one NW-wave workgroup per
// (codeword, 256-byte chunk) with the layouts of encode_gf8_split_kernel (S: e = PW w + j,
// L: e = NW h + w, the top pair merged), so one square's codewords spread over NW times
// the waves of the byte-table kernel's one-wave-per-task form, whose single wave per
// SIMD runs the whole transform as one dependent chain.  No fused form.
// ---------------------------------------------------------------------------
template <int M, int NW>
__global__ __launch_bounds__(64 * NW) void encode_gf8_splitm_kernel(SplitEncPlan p) {
    constexpr int PW = M / NW;
    static_assert(PW * NW == M && PW >= NW, "split encoder shape");
    __shared__ uint32_t xch[M][64];
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t task = blockIdx.x;
    const uint32_t kind = task < p.n0 ? 0u : 1u;
    task -= kind == 0u ? 0u : p.n0;
    const CodewordSet& cs = p.cs[kind];
    const uint32_t chunks = cs.chunks;
    const uint32_t q = task / chunks;
    const uint32_t chunk = task - q * chunks;
    const uint32_t off0 = chunk * 256u + lane * 4u;
    const uint32_t off = off0 < cs.S ? off0 : kOob;
    const uint64_t rel = cw_rel(cs, q);
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(cs.base + rel);
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(cs.out_base + rel);
    const uint32_t k = cs.k, es = (uint32_t)cs.elem_stride, oo = (uint32_t)cs.out_offset;
    uint32_t v[PW];
    static_for<PW>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t e = PW * w + j;
        v[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, off, e < k ? e * es : kOob, 0);
    });
    enc_split_low<NW, PW, false, M>(v, w);
    static_for<PW>([&](auto J) { xch[PW * w + decltype(J)::value][lane] = v[decltype(J)::value]; });
    __syncthreads();
    static_for<PW>([&](auto H) { v[decltype(H)::value] = xch[NW * decltype(H)::value + w][lane]; });
    enc_split_high<NW, PW, false, M>(v);
    enc_split_mid<NW, PW, M>(v);
    enc_split_high<NW, PW, true, M>(v);
    __syncthreads();
    static_for<PW>([&](auto H) { xch[NW * decltype(H)::value + w][lane] = v[decltype(H)::value]; });
    __syncthreads();
    static_for<PW>([&](auto J) { v[decltype(J)::value] = xch[PW * w + decltype(J)::value][lane]; });
    enc_split_low<NW, PW, true, M>(v, w);
    static_for<PW>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t e = PW * w + j;
        __builtin_amdgcn_raw_buffer_store_b32(v[j], ro, off, e < k ? oo + e * es : kOob, 0);
    });
}

// waves per (codeword, chunk): chosen by the caller -- 16 (encode_gf8_split16_kernel) for
// one square and the per-codeword codec, 8 for batches (8 against 4: single square 21.1
// against 25.3 us, profiles/r03_single.jsonl; 16 against 8: DESIGN.md §4 latency form,
// round 6); diagnostic builds take rsm_diag_set_split_waves (A/B of 2 / 4 / 8 / 16 per
// launch; 0 = the caller's choice)
#ifdef RSM_DIAG
static std::atomic<int> g_split_nw[2] = {0, 0};
static std::atomic<bool> g_split_fused{false};
void set_split_diag_waves(int first, int second) {
    g_split_nw[0].store(first);
    g_split_nw[1].store(second);
}
void set_split_diag_fused(bool on) { g_split_fused.store(on); }
bool split_fused_enabled() { return g_split_fused.load(); }
#else
// the one-launch form with its device-side wait measured SLOWER than two launches
// (30.1 vs 22.2 us: the write-through Q1 stores leave L2 and the Q1-column workgroups
// read them back from the Infinity Cache; profiles/r03_single.jsonl) -- diagnostic only
bool split_fused_enabled() { return false; }
#endif

static hipError_t launch_split(const SplitEncPlan& p, uint32_t tasks, int nw, hipStream_t st) {
    switch (nw) {
        case 2: hipLaunchKernelGGL(encode_gf8_split_kernel<2>, dim3(tasks), dim3(128), 0, st, p); break;
        case 8: hipLaunchKernelGGL(encode_gf8_split_kernel<8>, dim3(tasks), dim3(512), 0, st, p); break;
        case 16:  // (no fused form: the 16-wave kernel takes up to two sets, no hand-off)
            if (p.fused) hipLaunchKernelGGL(encode_gf8_split_kernel<8>, dim3(tasks), dim3(512), 0, st, p);
            else hipLaunchKernelGGL(encode_gf8_split16_kernel, dim3(tasks), dim3(1024), 0, st, p);
            break;
        default: hipLaunchKernelGGL(encode_gf8_split_kernel<4>, dim3(tasks), dim3(256), 0, st, p); break;
    }
    return hipGetLastError();
}
static int split_waves(int launch, int nw) {
#ifdef RSM_DIAG
    const int n = g_split_nw[launch].load();
    return n ? n : nw;
#else
    (void)launch;
    return nw;
#endif
}
static void split_set(SplitEncPlan& p, int i, const CodewordSet& c, uint32_t& n) {
    p.cs[i] = rebased(c);  // parity from its own base: offsets span one half (narrow_fits)
    p.cs[i].chunks = (c.S + 255) / 256;
    n = p.cs[i].count * p.cs[i].chunks;
}

hipError_t launch_encode_gf8_split(const CodewordSet& a, const CodewordSet* b, hipStream_t st, int nw) {
    const uint32_t M = ceil_pow2(a.k);
    if ((M != 16 && M != 32 && M != 64 && M != 128) || (b && ceil_pow2(b->k) != M)) return hipErrorInvalidValue;
    SplitEncPlan p{};
    split_set(p, 0, a, p.n0);
    if (b) split_set(p, 1, *b, p.n1);
    const uint64_t tasks = (uint64_t)p.n0 + p.n1;
    if (tasks == 0) return hipSuccess;
    if (M == 64) {  // (nw: 8 waves of 8 points; the only shape with PW >= NW and more than 4 waves)
        hipLaunchKernelGGL((encode_gf8_splitm_kernel<64, 8>), dim3((uint32_t)tasks), dim3(512), 0, st, p);
        return hipGetLastError();
    }
    if (M == 32) {  // 4 waves of 8 points
        hipLaunchKernelGGL((encode_gf8_splitm_kernel<32, 4>), dim3((uint32_t)tasks), dim3(256), 0, st, p);
        return hipGetLastError();
    }
    if (M == 16) {  // 4 waves of 4 points
        hipLaunchKernelGGL((encode_gf8_splitm_kernel<16, 4>), dim3((uint32_t)tasks), dim3(256), 0, st, p);
        return hipGetLastError();
    }
    return launch_split(p, (uint32_t)tasks, split_waves(b ? 0 : 1, nw), st);
}

hipError_t launch_extend_gf8_split_fused(const CodewordSet& rows, const CodewordSet& c0, const CodewordSet& c1,
                                         uint32_t* ctr, uint32_t* err, hipStream_t st) {
    if (ceil_pow2(rows.k) != 128) return hipErrorInvalidValue;
    SplitEncPlan p{};
    split_set(p, 0, rows, p.n0);
    split_set(p, 1, c0, p.n1);
    split_set(p, 2, c1, p.n2);
    p.ctr = ctr;
    p.err = err;
    p.fused = 1;
    const uint64_t tasks = (uint64_t)p.n0 + p.n1 + p.n2;
    if (tasks == 0 || p.n2 == 0) return hipErrorInvalidValue;
    return launch_split(p, (uint32_t)tasks, split_waves(0, 8), st);
}

// ---------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------
template <int M>
static hipError_t launch_enc(const CodewordSet& cs, hipStream_t st) {
    const uint64_t tasks = (uint64_t)cs.count * cs.chunks;
    const uint32_t blocks = (uint32_t)((tasks + 3) / 4);
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(encode_gf8_kernel<M>, dim3(blocks), dim3(256), 0, st, cs);
    return hipGetLastError();
}

// Diagnostic build only: RSM_GF8_KERNEL=table forces the byte-table kernel for
// M = 128 (A/B measurements).  The product library always takes the bit-sliced
// kernel where it applies.
static bool bs128_enabled() {
#ifdef RSM_DIAG
    static const bool on = [] {
        const char* v = getenv("RSM_GF8_KERNEL");
        return !(v && strcmp(v, "table") == 0);
    }();
    return on;
#else
    return true;
#endif
}

hipError_t launch_encode_gf8(const CodewordSet& cs, hipStream_t st) {
    if (bs128_enabled() && bs128_applicable(cs)) return launch_encode_gf8_bs128(cs, st);
    switch (ceil_pow2(cs.k)) {
        case 1: return launch_enc<1>(cs, st);
        case 2: return launch_enc<2>(cs, st);
        case 4: return launch_enc<4>(cs, st);
        case 8: return launch_enc<8>(cs, st);
        case 16: return launch_enc<16>(cs, st);
        case 32: return launch_enc<32>(cs, st);
        case 64: return launch_enc<64>(cs, st);
        case 128: return launch_enc<128>(cs, st);
        default: return hipErrorInvalidValue;
    }
}

// Wide forms: one launch per byte slab of the shares (base advanced to the slab's
// first byte, S = its width; at most 1 GiB, and few enough 256-byte chunks that
// count * chunks stays a 32-bit task index); a capped grid loops over the tasks.
constexpr uint32_t kWideGrid = 2048;
static uint32_t wide_slab(uint32_t count) {
    uint64_t chunks = (1ull << 31) / (count ? count : 1u);
    if (chunks > (1u << 22)) chunks = 1u << 22;  // 1 GiB
    return (uint32_t)(chunks ? chunks : 1u) * 256u;
}
template <int M>
static hipError_t go_enc_wide(const CodewordSet& cs, hipStream_t st) {
    const uint32_t tasks = cs.count * cs.chunks;
    hipLaunchKernelGGL(encode_gf8_wide_kernel<M>, dim3(tasks < kWideGrid ? tasks : kWideGrid), dim3(64), 0, st, cs);
    return hipGetLastError();
}
template <int M>
static hipError_t go_dec_wide(const DecodeSet& ds, hipStream_t st) {
    const uint32_t tasks = ds.count * ds.chunks;
    hipLaunchKernelGGL(decode_gf8_wide_kernel<M>, dim3(tasks < kWideGrid ? tasks : kWideGrid), dim3(64), 0, st, ds);
    return hipGetLastError();
}

hipError_t launch_encode_gf8_wide(const CodewordSet& cs0, hipStream_t st) {
    if (cs0.k == 0 || ceil_pow2(cs0.k) > 128 || cs0.count >= (1u << 31)) return hipErrorInvalidValue;
    const uint32_t slab = wide_slab(cs0.count);
    for (uint64_t c0 = 0; c0 < cs0.S; c0 += slab) {
        CodewordSet cs = cs0;
        cs.base = cs0.base + c0;
        cs.out_base = (cs0.out_base ? cs0.out_base : cs0.base) + c0;
        cs.S = (uint32_t)(cs0.S - c0 < slab ? cs0.S - c0 : slab);
        cs.chunks = (cs.S + 255) / 256;
        hipError_t e;
        switch (ceil_pow2(cs.k)) {
            case 1: e = go_enc_wide<1>(cs, st); break;
            case 2: e = go_enc_wide<2>(cs, st); break;
            case 4: e = go_enc_wide<4>(cs, st); break;
            case 8: e = go_enc_wide<8>(cs, st); break;
            case 16: e = go_enc_wide<16>(cs, st); break;
            case 32: e = go_enc_wide<32>(cs, st); break;
            case 64: e = go_enc_wide<64>(cs, st); break;
            default: e = go_enc_wide<128>(cs, st); break;
        }
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_decode_gf8_wide(const DecodeSet& ds0, hipStream_t st) {
    if (ds0.k == 0 || ceil_pow2(ds0.k) > 128 || ds0.in_base || ds0.mirror) return hipErrorInvalidValue;
    const uint32_t slab = wide_slab(ds0.count);
    for (uint64_t c0 = 0; c0 < ds0.S; c0 += slab) {
        DecodeSet ds = ds0;
        ds.trace = nullptr;
        ds.base = ds0.base + c0;
        ds.pitch = ds0.pitch ? ds0.pitch : ds0.S;
        ds.S = (uint32_t)(ds0.S - c0 < slab ? ds0.S - c0 : slab);
        ds.chunks = (ds.S + 255) / 256;
        hipError_t e;
        switch (ceil_pow2(ds.k)) {
            case 1: e = go_dec_wide<1>(ds, st); break;
            case 2: e = go_dec_wide<2>(ds, st); break;
            case 4: e = go_dec_wide<4>(ds, st); break;
            case 8: e = go_dec_wide<8>(ds, st); break;
            case 16: e = go_dec_wide<16>(ds, st); break;
            case 32: e = go_dec_wide<32>(ds, st); break;
            case 64: e = go_dec_wide<64>(ds, st); break;
            default: e = go_dec_wide<128>(ds, st); break;
        }
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

template <int M>
static hipError_t launch_dec(const DecodeSet& ds, hipStream_t st) {
    const uint64_t tasks = (uint64_t)ds.count * ds.chunks;
    if (tasks == 0) return hipSuccess;
    hipLaunchKernelGGL(decode_gf8_kernel<M>, dim3((uint32_t)tasks), dim3(64), 0, st, ds);
    return hipGetLastError();
}

// The split decoder's locator: per wave (WE) or wave 0 + LDS tables (round 4 form).
// Sweeps (hundreds of tasks, VALU-bound) share wave 0's locator: the per-wave copies
// measured slower (33.3-34.1 against 30.5-31.2 us, profiles/r05d_dec_ab.jsonl).  A few
// tasks (the codec's one codeword, a fraud-proof row: latency-bound, the CU otherwise
// idle) take the per-wave form, no wave waiting on wave 0 and its barrier: codec Decode
// p50 -1.1 us (profiles/r06s_codec_dec_ab.jsonl).
constexpr uint64_t kDecWaveErrTasks = 64;
#ifdef RSM_DIAG
static std::atomic<uint32_t> g_dec8_mode{0};  // 1: the other locator form (A/B), 2: the floor form
void set_dec8_diag_mode(uint32_t m) { g_dec8_mode.store(m); }
static bool dec8_wave_err(uint64_t tasks) {
    const uint32_t m = g_dec8_mode.load();
    if (m == 2) return true;  // the setup-free floor runs on the per-wave form
    return (tasks <= kDecWaveErrTasks) != (m == 1);
}
#else
void set_dec8_diag_mode(uint32_t) {}
static bool dec8_wave_err(uint64_t tasks) { return tasks <= kDecWaveErrTasks; }
#endif
#ifdef RSM_DIAG
static std::atomic<uint32_t*> g_dec_trace{nullptr};
static std::atomic<uint32_t> g_dec_delay{0};
void set_dec_diag_trace(uint32_t* d) { g_dec_trace.store(d); }
uint32_t* dec_diag_trace_ptr() { return g_dec_trace.load(); }
void set_dec_diag_delay(uint32_t ticks) { g_dec_delay.store(ticks); }
#else
void set_dec_diag_trace(uint32_t*) {}
uint32_t* dec_diag_trace_ptr() { return nullptr; }
void set_dec_diag_delay(uint32_t) {}
#endif

hipError_t launch_decode_gf8(const DecodeSet& ds0, hipStream_t st) {
    DecodeSet ds = ds0;
#ifdef RSM_DIAG
    ds.trace = g_dec_trace.load();
    ds.delay = g_dec8_mode.load() == 2 ? kDecFloor : g_dec_delay.load();  // mode 2: the setup-free floor
#else
    ds.trace = nullptr;
    ds.delay = 0;
#endif
    if (ceil_pow2(ds.k) == 128) {  // split form: kSplitWaves waves per (codeword, 256 B chunk)
        const uint64_t tasks = (uint64_t)ds.count * ds.chunks;
        if (tasks == 0) return hipSuccess;
        if (ds.in_base) {
            // zero-copy: PCIe-bound; 4 waves (8 would spill the loop's extra registers)
            const uint32_t grid = ds.grid && ds.grid < tasks ? ds.grid : (uint32_t)tasks;
            hipLaunchKernelGGL(decode_gf8_split_zc_kernel<4>, dim3(grid), dim3(256), 0, st, ds);
        } else {
            constexpr int NW = kSplitWaves;
            if (dec8_wave_err(tasks))
                hipLaunchKernelGGL((decode_gf8_split_kernel<NW, true>), dim3((uint32_t)tasks), dim3(64 * NW), 0, st, ds);
            else
                hipLaunchKernelGGL((decode_gf8_split_kernel<NW, false>), dim3((uint32_t)tasks), dim3(64 * NW), 0, st, ds);
        }
        return hipGetLastError();
    }
    switch (ceil_pow2(ds.k)) {
        case 1: return launch_dec<1>(ds, st);
        case 2: return launch_dec<2>(ds, st);
        case 4: return launch_dec<4>(ds, st);
        case 8: return launch_dec<8>(ds, st);
        case 16: return launch_dec<16>(ds, st);
        case 32: return launch_dec<32>(ds, st);
        case 64: return launch_dec<64>(ds, st);
        case 128: return launch_dec<128>(ds, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace rsm
