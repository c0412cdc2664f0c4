// gf_tables.hpp -- compile-time Leopard GF(2^8) tables for code generation.
//
// The HIP kernels specialise the additive-FFT butterfly network on the
// power-of-two transform size m, so every FFT skew (twiddle log) is a
// compile-time constant and every GF multiply-by-constant becomes a fixed
// v_perm_b32 lookup sequence.  These tables restate the field construction of
// klauspost/reedsolomon v1.14.1 leopard8.go (catid LeopardFF8.cpp), which
// rsmt2d's LeoRSCodec selects for 2k <= 256 shards (leopard.go:65,
// codecs.go:6-10):
//   * LFSR exp/log over poly 0x11D, converted to the Cantor basis
//     {1,214,152,146,86,200,88,230}
//   * FFT skew vector + log-Walsh transform (FFTInitialize)
// Pinned in tests/ against the reference KATs (extendeddatasquare_test.go:39-59).
#pragma once
#include <cstdint>

namespace rsm {

struct Gf8Tables {
    uint8_t exp[256];
    uint8_t log[256];
    uint8_t skew[255];
    uint8_t logwalsh[256];
};

constexpr unsigned gf8_add_mod(unsigned a, unsigned b) {
    unsigned s = a + b;
    return (s + (s >> 8)) & 255u;
}
constexpr unsigned gf8_sub_mod(unsigned a, unsigned b) {
    unsigned d = a - b;
    return (d + (d >> 8)) & 255u;
}

constexpr Gf8Tables make_gf8_tables() {
    Gf8Tables t{};
    constexpr unsigned basis[8] = {1, 214, 152, 146, 86, 200, 88, 230};
    unsigned state = 1;
    for (unsigned i = 0; i < 255; ++i) {
        t.exp[state] = static_cast<uint8_t>(i);
        state <<= 1;
        if (state >= 256) state ^= 0x11Du;
    }
    t.exp[0] = 255;
    t.log[0] = 0;
    for (unsigned i = 0; i < 8; ++i) {
        unsigned w = 1u << i;
        for (unsigned j = 0; j < w; ++j) t.log[j + w] = static_cast<uint8_t>(t.log[j] ^ basis[i]);
    }
    for (unsigned i = 0; i < 256; ++i) t.log[i] = t.exp[t.log[i]];
    for (unsigned i = 0; i < 256; ++i) t.exp[t.log[i]] = static_cast<uint8_t>(i);
    t.exp[255] = t.exp[0];

    auto mul_log = [&](unsigned a, unsigned lb) -> unsigned {
        return a == 0 ? 0u : t.exp[gf8_add_mod(t.log[a], lb)];
    };
    unsigned temp[7] = {};
    for (unsigned i = 1; i < 8; ++i) temp[i - 1] = 1u << i;
    for (unsigned m = 0; m < 7; ++m) {
        unsigned step = 1u << (m + 1);
        t.skew[(1u << m) - 1] = 0;
        for (unsigned i = m; i < 7; ++i) {
            unsigned s = 1u << (i + 1);
            for (unsigned j = (1u << m) - 1; j < s; j += step)
                t.skew[j + s] = static_cast<uint8_t>(t.skew[j] ^ temp[i]);
        }
        temp[m] = 255u - t.log[mul_log(temp[m], t.log[temp[m] ^ 1u])];
        for (unsigned i = m + 1; i < 7; ++i)
            temp[i] = mul_log(temp[i], gf8_add_mod(t.log[temp[i] ^ 1u], temp[m]));
    }
    for (unsigned i = 0; i < 255; ++i) t.skew[i] = t.log[t.skew[i]];
    for (unsigned i = 0; i < 256; ++i) t.logwalsh[i] = t.log[i];
    t.logwalsh[0] = 0;
    // FWHT(LogWalsh, 256, 256)
    unsigned dist = 1, dist4 = 4;
    for (; dist4 <= 256; dist = dist4, dist4 <<= 2)
        for (unsigned r = 0; r < 256; r += dist4)
            for (unsigned i = r; i < r + dist; ++i) {
                unsigned t0 = t.logwalsh[i], t1 = t.logwalsh[i + dist];
                unsigned t2 = t.logwalsh[i + 2 * dist], t3 = t.logwalsh[i + 3 * dist];
                unsigned a;
                a = gf8_add_mod(t0, t1); t1 = gf8_sub_mod(t0, t1); t0 = a;
                a = gf8_add_mod(t2, t3); t3 = gf8_sub_mod(t2, t3); t2 = a;
                a = gf8_add_mod(t0, t2); t2 = gf8_sub_mod(t0, t2); t0 = a;
                a = gf8_add_mod(t1, t3); t3 = gf8_sub_mod(t1, t3); t1 = a;
                t.logwalsh[i] = static_cast<uint8_t>(t0);
                t.logwalsh[i + dist] = static_cast<uint8_t>(t1);
                t.logwalsh[i + 2 * dist] = static_cast<uint8_t>(t2);
                t.logwalsh[i + 3 * dist] = static_cast<uint8_t>(t3);
            }
    return t;
}

inline constexpr Gf8Tables kGf8 = make_gf8_tables();

// Self-checks against SURVEY.md A.2/A.3 (values the survey-time restatement and
// the oracle both reproduce).
static_assert(kGf8.exp[1] == 104 && kGf8.exp[2] == 92 && kGf8.exp[7] == 18);
static_assert(kGf8.log[0] == 255 && kGf8.log[1] == 0 && kGf8.log[2] == 85 && kGf8.log[7] == 136);
static_assert(kGf8.skew[0] == 255 && kGf8.skew[2] == 85 && kGf8.skew[8] == 153 && kGf8.skew[14] == 187);

constexpr unsigned gf8_mul_log(unsigned a, unsigned lb) {
    return a == 0 ? 0u : kGf8.exp[gf8_add_mod(kGf8.log[a], lb)];
}

// v_perm_b32 lookup tables for y -> y * exp(L): the byte is split into chunks
// bits[0:3), bits[3:6), bits[6:8); each chunk indexes an 8- (or 4-) entry byte
// table held in a 64-bit {hi:lo} register pair.  GF multiplication is linear over
// XOR, so the three partial products XOR to the full product.
struct PermTab {
    uint32_t a_lo, a_hi, b_lo, b_hi, c;
};
constexpr uint32_t pack4(unsigned b0, unsigned b1, unsigned b2, unsigned b3) {
    return b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
}
constexpr PermTab make_perm_tab(unsigned L) {
    PermTab p{};
    unsigned ta[8] = {}, tb[8] = {}, tc[4] = {};
    for (unsigned v = 0; v < 8; ++v) {
        ta[v] = gf8_mul_log(v, L);
        tb[v] = gf8_mul_log(v << 3, L);
    }
    for (unsigned v = 0; v < 4; ++v) tc[v] = gf8_mul_log(v << 6, L);
    p.a_lo = pack4(ta[0], ta[1], ta[2], ta[3]);
    p.a_hi = pack4(ta[4], ta[5], ta[6], ta[7]);
    p.b_lo = pack4(tb[0], tb[1], tb[2], tb[3]);
    p.b_hi = pack4(tb[4], tb[5], tb[6], tb[7]);
    p.c = pack4(tc[0], tc[1], tc[2], tc[3]);
    return p;
}

}  // namespace rsm
