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
#include <algorithm>
#include <set>
#include <vector>
#include "../gf_tables.hpp"

namespace rsm::gen {

// register codes: 0..7 x planes, 8..15 y planes, 16..21 temporaries
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
inline const std::vector<Op>& mul_network_v1(unsigned L) {
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

// Round-3 search (beam over chained temporaries): a temporary is ANY mask one 2- or
// 3-input XOR of the items already available (the y planes and earlier temporaries)
// can make, and a row is the shortest XOR of items equal to it (cancellation allowed),
// costing ceil(items / 2) accumulating 3-input XORs.  Beam of 24 over up to kMaxTemps
// temporaries; the v1 network is kept where it is not beaten.
constexpr int kMaxTemps = 6;
inline int g_beam = 24;  // beam width (the generators keep the default)
struct ItemDist {
    uint8_t d[256];
    uint8_t prev[256], item[256];
};
inline void item_dist(const unsigned* items, int n, ItemDist& t) {
    for (int m = 0; m < 256; ++m) t.d[m] = 255;
    t.d[0] = 0;
    uint8_t front[256], nf[256];
    int nfr = 1, lvl = 0;
    front[0] = 0;
    while (nfr) {
        ++lvl;
        int nn = 0;
        for (int f = 0; f < nfr; ++f)
            for (int i = 0; i < n; ++i) {
                const unsigned x = front[f] ^ items[i];
                if (t.d[x] == 255) {
                    t.d[x] = (uint8_t)lvl;
                    t.prev[x] = front[f];
                    t.item[x] = (uint8_t)i;
                    nf[nn++] = (uint8_t)x;
                }
            }
        for (int i = 0; i < nn; ++i) front[i] = nf[i];
        nfr = nn;
    }
}
inline int net_cost(const unsigned (&rows)[8], const std::vector<unsigned>& temps, ItemDist& t, int ne = 0) {
    unsigned items[8 + kMaxTemps];
    int n = 0;
    for (int j = 0; j < 8; ++j) items[n++] = 1u << j;
    for (unsigned m : temps) items[n++] = m;
    item_dist(items, n, t);
    int c = (int)temps.size();
    for (int i = 0; i < 8; ++i) c += (t.d[rows[i]] + ne + 1) / 2;
    return c;
}
inline std::vector<unsigned> beam_temps(const unsigned (&rows)[8], int* cost_out, int ne = 0) {
    struct St {
        int c;
        std::vector<unsigned> t;
    };
    ItemDist td;
    std::vector<St> states{{net_cost(rows, {}, td, ne), {}}};
    St best = states[0];
    for (int depth = 0; depth < kMaxTemps; ++depth) {
        std::vector<St> cand;
        std::set<std::vector<unsigned>> seen;
        for (const St& s : states) {
            unsigned items[8 + kMaxTemps];
            int n = 0;
            for (int j = 0; j < 8; ++j) items[n++] = 1u << j;
            for (unsigned m : s.t) items[n++] = m;
            ItemDist d;
            item_dist(items, n, d);
            for (unsigned m = 1; m < 256; ++m) {
                if (d.d[m] != 2 && d.d[m] != 3) continue;
                std::vector<unsigned> nt = s.t;
                nt.push_back(m);
                std::vector<unsigned> key = nt;
                std::sort(key.begin(), key.end());
                if (!seen.insert(key).second) continue;
                cand.push_back(St{net_cost(rows, nt, td, ne), nt});
            }
        }
        if (cand.empty()) break;
        std::stable_sort(cand.begin(), cand.end(), [](const St& a, const St& b) { return a.c < b.c; });
        if (cand.size() > (size_t)g_beam) cand.resize((size_t)g_beam);
        states = cand;
        if (states[0].c < best.c) best = states[0];
    }
    *cost_out = best.c;
    return best.t;
}
// x_i ^= (M_L y)_i ^ e0_i ^ ... (ne extra symbols folded in by the block optimizer
// below; extra symbol k, plane i has register code 24 + 8k + i).  ne = 0: the plain
// multiply network (the v1 network where the beam does not beat it).
inline const std::vector<Op>& mul_network_ex(unsigned L, int ne) {
    static std::vector<Op> memo[3][256];
    static bool done[3][256] = {};
    if (done[ne][L]) return memo[ne][L];
    done[ne][L] = true;
    unsigned rows[8];
    matrix_rows(L, rows);
    int c2 = 0;
    const std::vector<unsigned> temps = beam_temps(rows, &c2, ne);
    if (ne == 0) {
        const std::vector<Op>& v1 = mul_network_v1(L);
        if ((int)v1.size() <= c2) return memo[ne][L] = v1;
    }
    std::vector<Op>& ops = memo[ne][L];
    unsigned items[8 + kMaxTemps];
    uint8_t code[8 + kMaxTemps];
    int n = 0;
    for (int j = 0; j < 8; ++j) items[n] = 1u << j, code[n++] = (uint8_t)(8 + j);
    auto rep = [&](unsigned m, int nitems) {  // shortest item list for m over items[0..nitems)
        ItemDist d;
        item_dist(items, nitems, d);
        std::vector<uint8_t> r;
        for (unsigned x = m; x; x = d.prev[x]) r.push_back(code[d.item[x]]);
        return r;
    };
    for (size_t i = 0; i < temps.size(); ++i) {
        const std::vector<uint8_t> r = rep(temps[i], n);
        const uint8_t dst = (uint8_t)(16 + i);
        ops.push_back(r.size() == 2 ? Op{kSet2, dst, r[0], r[1], 0} : Op{kSet3, dst, r[0], r[1], r[2]});
        items[n] = temps[i], code[n++] = dst;
    }
    std::vector<std::vector<uint8_t>> terms(8);
    for (int i = 0; i < 8; ++i) {
        terms[i] = rep(rows[i], n);
        for (int k = 0; k < ne; ++k) terms[i].push_back((uint8_t)(24 + 8 * k + i));
    }
    for (unsigned step = 0; step < 8; ++step)
        for (unsigned i = 0; i < 8; ++i) {
            const auto& t = terms[i];
            if (2 * step + 1 < t.size()) ops.push_back(Op{kXor3, (uint8_t)i, t[2 * step], t[2 * step + 1], 0});
            else if (2 * step < t.size()) ops.push_back(Op{kXor2, (uint8_t)i, t[2 * step], 0, 0});
        }
    return ops;
}
inline const std::vector<Op>& mul_network(unsigned L) { return mul_network_ex(L, 0); }

// number of temporaries an op list writes (codes 16..)
inline int temps_used(const std::vector<Op>& ops) {
    int n = 0;
    for (const Op& o : ops)
        if (o.dst >= 16 && o.dst - 15 > n) n = o.dst - 15;
    return n;
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

// ---------------------------------------------------------------------------
// Block optimizer (round 3q): a block of butterflies (one asm statement) as a list of
// symbol-level ops, ADD (d ^= a, 8 XORs) and MULACC (d ^= M_L a, a network), where
// two rewrites fold an ADD into a neighbouring network's rows (an extra term per row:
// ceil((terms + 1) / 2) instead of ceil(terms / 2) + 1 instructions):
//   forward  MULACC(x, y) ... ADD(x, z)  ->  MULACC(x, y; +z)   (IFFT: the next layer's
//            y ^= x on this x-output; z not written, x not read in between)
//   backward ADD(y, x) ... MULACC(y, w)  ->  MULACC(y, w; +x)   (FFT: y ^= x deferred
//            into the next layer's accumulate on y; x not written, y not read between)
// and two ADDs into one register with nothing in between touching them become one
// 3-input XOR per plane.
struct IrOp {
    int kind;  // 0 ADD d ^= a (+ b if b >= 0: 3-input), 1 MULACC d ^= M_L a (+ extras)
    int d, a, b;
    unsigned L;
    std::vector<int> ex;
};
inline void ir_butterfly(std::vector<IrOp>& ir, int kind, unsigned L, int x, int y) {
    auto add = [&] { ir.push_back(IrOp{0, y, x, -1, 0, {}}); };
    if (kind != 1) add();
    if (L != 255u) ir.push_back(IrOp{1, x, y, -1, L, {}});
    if (kind != 0) add();
}
inline bool ir_reads(const IrOp& o, int r) {
    if (o.a == r || o.b == r || o.d == r) return true;  // d is read too (accumulate)
    for (int e : o.ex) if (e == r) return true;
    return false;
}
inline bool ir_writes(const IrOp& o, int r) { return o.d == r; }
inline void ir_optimize(std::vector<IrOp>& ir) {
    bool changed = true;
    while (changed) {
        changed = false;
        for (size_t i = 0; i < ir.size() && !changed; ++i) {
            IrOp& o = ir[i];
            if (o.kind == 1 && o.ex.size() < 2) {  // forward fold of a later ADD(d, z)
                for (size_t j = i + 1; j < ir.size(); ++j) {
                    const IrOp& q = ir[j];
                    if (q.kind == 0 && q.d == o.d && q.b < 0) {
                        bool ok = true;
                        for (size_t m = i + 1; m < j && ok; ++m)
                            if (ir_reads(ir[m], o.d) || ir_writes(ir[m], q.a)) ok = false;
                        if (ok) {
                            o.ex.push_back(q.a);
                            ir.erase(ir.begin() + (long)j);
                            changed = true;
                        }
                        break;
                    }
                    if (ir_reads(q, o.d)) break;
                }
            }
            if (changed) break;
            if (o.kind == 0 && o.b < 0) {  // backward: defer into a later MULACC on d
                for (size_t j = i + 1; j < ir.size(); ++j) {
                    IrOp& q = ir[j];
                    if (q.kind == 1 && q.d == o.d && q.ex.size() < 2) {
                        bool ok = true;
                        for (size_t m = i + 1; m < j && ok; ++m)
                            if (ir_reads(ir[m], o.d) || ir_writes(ir[m], o.a)) ok = false;
                        if (ok && q.a != o.d) {
                            q.ex.push_back(o.a);
                            ir.erase(ir.begin() + (long)i);
                            changed = true;
                        }
                        break;
                    }
                    if (ir_reads(q, o.d)) {
                        // two ADDs into d with nothing else between: one 3-input XOR
                        if (q.kind == 0 && q.d == o.d && q.b < 0) {
                            bool ok = true;
                            for (size_t m = i + 1; m < j && ok; ++m)
                                if (ir_writes(ir[m], o.a) || ir_writes(ir[m], q.a)) ok = false;
                            if (ok) {
                                q.b = o.a;
                                ir.erase(ir.begin() + (long)i);
                                changed = true;
                            }
                        }
                        break;
                    }
                }
            }
        }
    }
}
// asm text of an optimized block; plane(sym, i) gives the operand of plane i of a
// symbol, temporaries are operands tbase...
template <typename F>
inline void ir_emit(const std::vector<IrOp>& ir, F&& plane, int tbase, std::vector<std::string>& out) {
    char b[128];
    for (const IrOp& o : ir) {
        if (o.kind == 0) {
            for (int i = 0; i < 8; ++i) {
                if (o.b < 0) snprintf(b, sizeof b, "v_xor_b32 %%%d, %%%d, %%%d", plane(o.d, i), plane(o.d, i), plane(o.a, i));
                else
                    snprintf(b, sizeof b, "v_bitop3_b32 %%%d, %%%d, %%%d, %%%d bitop3:0x96", plane(o.d, i), plane(o.d, i),
                             plane(o.a, i), plane(o.b, i));
                out.push_back(b);
            }
            continue;
        }
        auto map = [&](int c) {
            return c < 8 ? plane(o.d, c) : c < 16 ? plane(o.a, c - 8) : c < 24 ? tbase + (c - 16) : plane(o.ex[(c - 24) / 8], (c - 24) % 8);
        };
        for (const Op& n : mul_network_ex(o.L, (int)o.ex.size())) out.push_back(op_asm(n, map));
    }
}
inline int ir_temps(const std::vector<IrOp>& ir) {
    int n = 0;
    for (const IrOp& o : ir)
        if (o.kind == 1) {
            const auto& ops = mul_network_ex(o.L, (int)o.ex.size());
            for (const Op& q : ops)
                if (q.dst >= 16 && q.dst - 15 > n) n = q.dst - 15;
        }
    return n;
}
inline int ir_count(const std::vector<IrOp>& ir) {
    int n = 0;
    for (const IrOp& o : ir) n += o.kind == 0 ? 8 : (int)mul_network_ex(o.L, (int)o.ex.size()).size();
    return n;
}

}  // namespace rsm::gen
