// bs8_net.hpp -- build-time search for short bit-sliced GF(2^8) multiply networks.
//
// A butterfly's multiply x ^= y * exp(L) is, on bit-planes, x_i ^= XOR_{j in row_i} y_j
// for the 8x8 GF(2) matrix of exp(L) (bs8.hpp).  Written directly with 3-input
// XORs that is sum_i ceil(|row_i| / 2) instructions.  Here up to three
// temporaries t = y_a ^ y_b (^ y_c) are chosen -- exhaustively over the pairs and
// triples of planes contained in at least two rows -- so that rows sharing them
// need fewer terms; each row then takes ceil(terms / 2) XORs.  The op lists are
// emitted as device asm (gen_bs8_asm.cpp -> bs8_asm.inc, gen_bs8_small.cpp ->
// bs8_small.inc) and as a host table (bs8_net.inc) that the host reference path
// of bs8.hpp interprets (tests/native/bs8_host.cpp runs it against the oracle).
#pragma once
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>
#include "../gf_tables.hpp"

namespace rsm::gen {

// register codes: 0..7 x planes, 8..15 y planes, 16..18 temporaries
enum OpKind : uint8_t { kXor2 = 0, kXor3 = 1, kSet2 = 2, kSet3 = 3 };
struct Op {
    uint8_t kind, dst, a, b, c;
};

inline void matrix_rows(unsigned L, unsigned (&rows)[8]) {
    for (unsigned i = 0; i < 8; ++i) rows[i] = 0;
    for (unsigned j = 0; j < 8; ++j) {
        const unsigned p = gf8_mul_log(1u << j, L);
        for (unsigned i = 0; i < 8; ++i)
            if ((p >> i) & 1u) rows[i] |= 1u << j;
    }
}

inline int popc(unsigned m) { return __builtin_popcount(m); }

// Cheapest cover of one row by pairwise-disjoint temporaries contained in it:
// returns the XOR count; *used = mask of the chosen temporaries.
inline int row_cost(unsigned row, const unsigned* t, int nt, unsigned* used) {
    int best = (popc(row) + 1) / 2;
    unsigned bu = 0;
    for (unsigned s = 1; s < (1u << nt); ++s) {
        unsigned cover = 0;
        int n = popc(row);
        bool ok = true;
        for (int i = 0; i < nt && ok; ++i)
            if ((s >> i) & 1u) {
                if ((t[i] & row) != t[i] || (cover & t[i])) ok = false;
                cover |= t[i];
                n -= popc(t[i]) - 1;
            }
        if (ok && (n + 1) / 2 < best) best = (n + 1) / 2, bu = s;
    }
    if (used) *used = bu;
    return best;
}

inline int direct_cost(unsigned L) {
    unsigned rows[8];
    matrix_rows(L, rows);
    int c = 0;
    for (unsigned i = 0; i < 8; ++i) c += (popc(rows[i]) + 1) / 2;
    return c;
}

// x_i ^= (M_L y)_i as an op list: temporaries first, then step-major over the
// output planes (consecutive instructions independent).  Memoised per L.
inline const std::vector<Op>& mul_network(unsigned L) {
    static std::vector<Op> memo[256];
    static bool done[256] = {};
    if (done[L]) return memo[L];
    unsigned rows[8];
    matrix_rows(L, rows);
    std::vector<unsigned> cand;
    for (unsigned m = 1; m < 256; ++m) {
        if (popc(m) != 2 && popc(m) != 3) continue;
        int uses = 0;
        for (unsigned i = 0; i < 8; ++i) uses += (rows[i] & m) == m;
        if (uses >= 2) cand.push_back(m);
    }
    int best = direct_cost(L);
    unsigned bt[3] = {};
    int bn = 0;
    auto eval = [&](const unsigned* t, int nt) {
        int c = nt;
        for (unsigned i = 0; i < 8 && c < best; ++i) c += row_cost(rows[i], t, nt, nullptr);
        if (c < best) {
            best = c;
            bn = nt;
            for (int i = 0; i < nt; ++i) bt[i] = t[i];
        }
    };
    const int nc = (int)cand.size();
    for (int a = 0; a < nc; ++a) {
        const unsigned t1[1] = {cand[a]};
        eval(t1, 1);
        for (int b = a + 1; b < nc; ++b) {
            const unsigned t2[2] = {cand[a], cand[b]};
            eval(t2, 2);
            for (int c = b + 1; c < nc; ++c) {
                const unsigned t3[3] = {cand[a], cand[b], cand[c]};
                eval(t3, 3);
            }
        }
    }
    std::vector<Op>& ops = memo[L];
    for (int i = 0; i < bn; ++i) {
        uint8_t p[3] = {0, 0, 0};
        int n = 0;
        for (unsigned j = 0; j < 8; ++j)
            if ((bt[i] >> j) & 1u) p[n++] = (uint8_t)(8 + j);
        ops.push_back(Op{(uint8_t)(n == 2 ? kSet2 : kSet3), (uint8_t)(16 + i), p[0], p[1], p[2]});
    }
    std::vector<std::vector<uint8_t>> terms(8);
    for (unsigned i = 0; i < 8; ++i) {
        unsigned used = 0;
        row_cost(rows[i], bt, bn, &used);
        unsigned rest = rows[i];
        for (int t = 0; t < bn; ++t)
            if ((used >> t) & 1u) {
                terms[i].push_back((uint8_t)(16 + t));
                rest &= ~bt[t];
            }
        for (unsigned j = 0; j < 8; ++j)
            if ((rest >> j) & 1u) terms[i].push_back((uint8_t)(8 + j));
    }
    for (unsigned step = 0; step < 4; ++step)
        for (unsigned i = 0; i < 8; ++i) {
            const auto& t = terms[i];
            if (2 * step + 1 < t.size())
                ops.push_back(Op{kXor3, (uint8_t)i, t[2 * step], t[2 * step + 1], 0});
            else if (2 * step < t.size())
                ops.push_back(Op{kXor2, (uint8_t)i, t[2 * step], 0, 0});
        }
    done[L] = true;
    return ops;
}

// Whole butterflies (kind 0 IFFT_DIT2, 1 FFT_DIT2, 2 MID):
//   IFFT: y ^= x; x ^= M y.      FFT: x ^= M y; y ^= x.
//   MID : y ^= x; x ^= M y; y ^= x -- the encoder's last IFFT layer directly followed
//         by its first FFT layer on the same pairs, L the log of the summed twiddles.
// L == 255 (Leopard's log of zero): no multiply.
inline std::vector<Op> butterfly_ops(int kind, unsigned L) {
    std::vector<Op> ops;
    auto add_yx = [&] {
        for (uint8_t i = 0; i < 8; ++i) ops.push_back(Op{kXor2, (uint8_t)(8 + i), i, 0, 0});
    };
    if (kind != 1) add_yx();
    if (L != 255u) {
        const auto& net = mul_network(L);
        ops.insert(ops.end(), net.begin(), net.end());
    }
    if (kind != 0) add_yx();
    return ops;
}

// One op as gfx950 asm text; map(code) gives the asm operand number.
template <typename F>
inline std::string op_asm(const Op& o, F&& map) {
    char b[96];
    switch (o.kind) {
        case kXor2:
            snprintf(b, sizeof b, "v_xor_b32 %%%d, %%%d, %%%d", map(o.dst), map(o.dst), map(o.a));
            break;
        case kXor3:
            snprintf(b, sizeof b, "v_bitop3_b32 %%%d, %%%d, %%%d, %%%d bitop3:0x96", map(o.dst), map(o.dst), map(o.a),
                     map(o.b));
            break;
        case kSet2:
            snprintf(b, sizeof b, "v_xor_b32 %%%d, %%%d, %%%d", map(o.dst), map(o.a), map(o.b));
            break;
        default:
            snprintf(b, sizeof b, "v_bitop3_b32 %%%d, %%%d, %%%d, %%%d bitop3:0x96", map(o.dst), map(o.a), map(o.b),
                     map(o.c));
            break;
    }
    return b;
}

}  // namespace rsm::gen
