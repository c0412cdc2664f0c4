// gf16_tables.cpp -- Leopard GF(2^16) field tables (klauspost/reedsolomon
// v1.14.1 leopard.go, catid LeopardFF16.cpp), built on the host once per
// device and uploaded: exp/log over poly 0x1002D in the Cantor basis, the FFT
// skew vector, LogWalsh, and one v_perm_b32 table set per log value (PermTab16,
// see kernels_gf16.hip) so every multiply-by-constant on the device is a fixed
// sequence of byte permutes.
#include "gf16.hpp"

#include <cstring>
#include <mutex>
#include <vector>

namespace rsm {

namespace {
constexpr unsigned kBits = 16, kOrder = 65536, kMod = 65535;
constexpr unsigned kBasis[kBits] = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
                                    0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};

inline unsigned add_mod(unsigned a, unsigned b) {
    unsigned s = a + b;
    return (s + (s >> kBits)) & kMod;
}
inline unsigned sub_mod(unsigned a, unsigned b) {
    unsigned d = a - b;
    return (d + (d >> kBits)) & kMod;
}
}  // namespace

const Gf16Host& gf16_host() {
    static Gf16Host t;
    static std::once_flag once;
    std::call_once(once, [] {
        t.exp.assign(kOrder, 0);
        t.log.assign(kOrder, 0);
        t.skew.assign(kMod, 0);
        t.logwalsh.assign(kOrder, 0);
        unsigned state = 1;
        for (unsigned i = 0; i < kMod; ++i) {
            t.exp[state] = (uint16_t)i;
            state <<= 1;
            if (state >= kOrder) state ^= 0x1002Du;
        }
        t.exp[0] = kMod;
        t.log[0] = 0;
        for (unsigned i = 0; i < kBits; ++i) {
            unsigned w = 1u << i;
            for (unsigned j = 0; j < w; ++j) t.log[j + w] = (uint16_t)(t.log[j] ^ kBasis[i]);
        }
        for (unsigned i = 0; i < kOrder; ++i) t.log[i] = t.exp[t.log[i]];
        for (unsigned i = 0; i < kOrder; ++i) t.exp[t.log[i]] = (uint16_t)i;
        t.exp[kMod] = t.exp[0];
        auto mul_log = [&](unsigned a, unsigned lb) -> unsigned { return a == 0 ? 0u : t.exp[add_mod(t.log[a], lb)]; };
        unsigned temp[kBits - 1];
        for (unsigned i = 1; i < kBits; ++i) temp[i - 1] = 1u << i;
        for (unsigned m = 0; m < kBits - 1; ++m) {
            unsigned step = 1u << (m + 1);
            t.skew[(1u << m) - 1] = 0;
            for (unsigned i = m; i < kBits - 1; ++i) {
                unsigned s = 1u << (i + 1);
                for (unsigned j = (1u << m) - 1; j < s; j += step) t.skew[j + s] = (uint16_t)(t.skew[j] ^ temp[i]);
            }
            temp[m] = kMod - t.log[mul_log(temp[m], t.log[temp[m] ^ 1u])];
            for (unsigned i = m + 1; i < kBits - 1; ++i) temp[i] = mul_log(temp[i], add_mod(t.log[temp[i] ^ 1u], temp[m]));
        }
        for (unsigned i = 0; i < kMod; ++i) t.skew[i] = t.log[t.skew[i]];
        for (unsigned i = 0; i < kOrder; ++i) t.logwalsh[i] = t.log[i];
        t.logwalsh[0] = 0;
        // FWHT(LogWalsh, order, order)
        for (unsigned dist = 1; dist < kOrder; dist <<= 1)
            for (unsigned r = 0; r < kOrder; r += 2 * dist)
                for (unsigned i = r; i < r + dist; ++i) {
                    unsigned a = t.logwalsh[i], b = t.logwalsh[i + dist];
                    t.logwalsh[i] = (uint16_t)add_mod(a, b);
                    t.logwalsh[i + dist] = (uint16_t)sub_mod(a, b);
                }
        // LogWalsh folded to N points (gf16.hpp kLwFoldOff)
        t.lwfold.assign(kOrder - 512, 0);
        for (unsigned N = 512; N < kOrder; N <<= 1)
            for (unsigned r = 0; r < N; ++r) {
                unsigned s = 0;
                for (unsigned q = r; q < kOrder; q += N) s = add_mod(s, t.logwalsh[q]);
                t.lwfold[N - 512 + r] = (uint16_t)s;
            }
        // v_perm tables: PermTab16 per log value L
        t.perm.assign(kOrder, PermTab16{});
        for (unsigned L = 0; L < kOrder; ++L) {
            PermTab16& p = t.perm[L];
            // chunk shift amounts and widths: a,b,c from the lo byte; d,e,f from the hi byte
            const unsigned shift[6] = {0, 3, 6, 8, 11, 14};
            const unsigned width[6] = {8, 8, 4, 8, 8, 4};
            for (unsigned c = 0; c < 6; ++c) {
                uint8_t lo[8] = {}, hi[8] = {};
                for (unsigned v = 0; v < width[c]; ++v) {
                    unsigned prod = mul_log(v << shift[c], L);
                    lo[v] = (uint8_t)prod;
                    hi[v] = (uint8_t)(prod >> 8);
                }
                uint32_t l0, l1, h0, h1;
                memcpy(&l0, lo, 4); memcpy(&l1, lo + 4, 4);
                memcpy(&h0, hi, 4); memcpy(&h1, hi + 4, 4);
                p.w[4 * c + 0] = l0;  // output-lo table, entries 0..3
                p.w[4 * c + 1] = l1;  // output-lo table, entries 4..7
                p.w[4 * c + 2] = h0;  // output-hi table, entries 0..3
                p.w[4 * c + 3] = h1;  // output-hi table, entries 4..7
            }
        }
        // twiddle tables by skew index (encoder): zero table where the skew is the
        // modulus (that butterfly adds nothing)
        t.skewperm.assign(kSkewPermN, PermTab16{});
        for (unsigned i = 0; i < kSkewPermN; ++i)
            if (t.skew[i] != kOrder - 1) t.skewperm[i] = t.perm[t.skew[i]];
    });
    return t;
}

}  // namespace rsm
