// gen_bs8_small.cpp -- build-time generator of bs8_small.inc: the small-layout
// layers of the bit-sliced M = 128 encode (IFFT d = 1, 2, 4 and FFT d = 4, 2, 1 on
// symbols e = 16A + j, bs8.hpp) for all eight waves A as ONE inline-asm statement
// per direction that branches on A inside the asm.  Every other part of the
// kernel is the same code for all waves, so the eight waves of a workgroup share
// one instruction stream except for these blocks (eight distinct full programs
// overflow the instruction cache: measured 1.8x slower).  The butterflies are the
// networks of bs8_net.hpp (the ones bs8_asm.inc and bs8_net.inc hold).
// Operands: %0..%127 = X[j][i] (operand 8j + i), %128..%130 temporaries, %131 = A (SGPR).
#include <algorithm>
#include <cstdio>
#include <string>
#include <vector>
#include "bs8_net.hpp"

using namespace rsm;
using namespace rsm::gen;

// temporaries a list of butterflies needs (the most any one network uses)
struct Bfly {
    int kind;
    unsigned L;
    int xs, ys;
};
static int temps_of(const std::vector<Bfly>& bs) {
    int n = 0;
    for (const Bfly& b : bs) n = std::max(n, temps_used(butterfly_ops(b.kind, b.L)));
    return n;
}
static void bfly_asm(const Bfly& b, int tbase, std::vector<std::string>& out, int regs_per_sym = 8, int sym0 = 0) {
    auto map = [&](int c) {
        return c < 8 ? regs_per_sym * (b.xs - sym0) + c : c < 16 ? regs_per_sym * (b.ys - sym0) + (c - 8) : tbase + (c - 16);
    };
    for (const Op& o : butterfly_ops(b.kind, b.L)) out.push_back(op_asm(o, map));
}
static void print_temps_decl(int nt) {
    printf("    uint32_t");
    for (int t = 0; t < nt; ++t) printf("%s t%d", t ? "," : "", t);
    printf(";\n");
}
static void print_temps_ops(int nt) {  // the last operands of the output list (nt >= 1)
    for (int t = 0; t < nt; ++t) printf(" \"=&v\"(t%d)%s", t, t + 1 < nt ? "," : "");
}

static std::vector<Bfly> small_list(bool ifft, int a) {
    const int kOffEnc = 127;
    std::vector<Bfly> bs;
    if (ifft) {
        for (int d = 1; d <= 4; d <<= 1)
            for (int b = 0; b < 16; b += 2 * d)
                for (int q = 0; q < d; ++q) bs.push_back({0, kGf8.skew[kOffEnc + 16 * a + b + d], b + q, b + q + d});
    } else {
        for (int d = 4; d >= 1; d >>= 1)
            for (int b = 0; b < 16; b += 2 * d)
                for (int q = 0; q < d; ++q) bs.push_back({1, kGf8.skew[-1 + 16 * a + b + d], b + q, b + q + d});
    }
    return bs;
}
// operands: %0..%127 X, %128.. temporaries, then A
static void emit(const char* name, bool ifft) {
    int nt = 1;
    for (int a = 0; a < 8; ++a) nt = std::max(nt, temps_of(small_list(ifft, a)));
    const int opA = 128 + nt;
    printf("RSM_BS8_DEV void %s(uint32_t (&X)[16][8], uint32_t A) {\n", name);
    print_temps_decl(nt);
    printf("    asm volatile(\n");
    for (int a = 0; a < 7; ++a) printf("        \"s_cmp_eq_u32 %%%d, %d\\n\\ts_cbranch_scc1 .L%s%d_%%=\\n\\t\"\n", opA, a, name, a);
    printf("        \"s_branch .L%s7_%%=\\n\\t\"\n", name);
    for (int a = 0; a < 8; ++a) {
        std::vector<std::string> ins;
        for (const Bfly& b : small_list(ifft, a)) bfly_asm(b, 128, ins);
        printf("        \".L%s%d_%%=:\\n\\t\"\n", name, a);
        for (const auto& s : ins) printf("        \"%s\\n\\t\"\n", s.c_str());
        if (a < 7) printf("        \"s_branch .L%send_%%=\\n\\t\"\n", name);
    }
    printf("        \".L%send_%%=:\"\n        :", name);
    for (int j = 0; j < 16; ++j)
        for (int i = 0; i < 8; ++i) printf(" \"+v\"(X[%d][%d]),", j, i);
    print_temps_ops(nt);
    printf("\n        : \"s\"(A) : \"scc\");\n}\n");
}

// Half-split schedule (bs8.hpp small_ifft_h / small_fft_h): the small layers of ONE
// half G in layout S' (register j of wave A holds e = (j & 7) + 8A + 64 (j >> 3)),
// operands %0..%63 = X[8G + b][i] (operand 8b + i), %64..%66 temporaries, %67 = A.
static std::vector<Bfly> half_list(bool ifft, int G, int a) {
    const int kOffEnc = 127;
    std::vector<Bfly> bs;
    if (ifft) {
        for (int d = 1; d <= 4; d <<= 1)
            for (int b = 0; b < 8; b += 2 * d)
                for (int q = 0; q < d; ++q) bs.push_back({0, kGf8.skew[kOffEnc + 8 * a + 64 * G + b + d], b + q, b + q + d});
    } else {
        for (int d = 4; d >= 1; d >>= 1)
            for (int b = 0; b < 8; b += 2 * d)
                for (int q = 0; q < d; ++q) bs.push_back({1, kGf8.skew[-1 + 8 * a + 64 * G + b + d], b + q, b + q + d});
    }
    return bs;
}
// A list of butterflies as the block optimizer's ops (gen/bs8_net.hpp ir_optimize):
// IFFT layers in ascending index order (a network's next-layer y ^= x folds forward),
// FFT layers in descending order (a y ^= x is deferred into the next layer's
// accumulate on y before its partner is rewritten).
static std::vector<IrOp> block_ir(const std::vector<std::vector<Bfly>>& layers) {
    std::vector<IrOp> ir;
    for (const auto& layer : layers) {
        const bool fft = !layer.empty() && layer[0].kind == 1;
        if (fft)
            for (auto it = layer.rbegin(); it != layer.rend(); ++it) ir_butterfly(ir, it->kind, it->L, it->xs, it->ys);
        else
            for (const Bfly& b : layer) ir_butterfly(ir, b.kind, b.L, b.xs, b.ys);
    }
    ir_optimize(ir);
    return ir;
}
static std::vector<std::vector<Bfly>> by_layer(const std::vector<Bfly>& bs, int per_layer) {
    std::vector<std::vector<Bfly>> L;
    for (size_t i = 0; i < bs.size(); i += per_layer) L.emplace_back(bs.begin() + (long)i, bs.begin() + (long)(i + per_layer));
    return L;
}
static long g_plain = 0, g_opt = 0;  // VALU count of the optimized blocks vs butterfly by butterfly
static std::vector<IrOp> opt_block(const std::vector<Bfly>& bs, int per_layer) {
    std::vector<IrOp> ir = block_ir(by_layer(bs, per_layer));
    for (const Bfly& b : bs) g_plain += (long)butterfly_ops(b.kind, b.L).size();
    g_opt += ir_count(ir);
    return ir;
}

// operands: %0..%63 = X[8G + b][i] (operand 8b + i), %64.. temporaries, then A
static void emit_half(const char* name, bool ifft, int G) {
    std::vector<std::vector<IrOp>> irs;
    int nt = 1;
    for (int a = 0; a < 8; ++a) {
        irs.push_back(opt_block(half_list(ifft, G, a), 4));
        nt = std::max(nt, ir_temps(irs.back()));
    }
    const int opA = 64 + nt;
    printf("RSM_BS8_DEV void %s(uint32_t (&X)[16][8], uint32_t A) {\n", name);
    print_temps_decl(nt);
    printf("    asm volatile(\n");
    for (int a = 0; a < 7; ++a) printf("        \"s_cmp_eq_u32 %%%d, %d\\n\\ts_cbranch_scc1 .L%s%d_%%=\\n\\t\"\n", opA, a, name, a);
    printf("        \"s_branch .L%s7_%%=\\n\\t\"\n", name);
    for (int a = 0; a < 8; ++a) {
        std::vector<std::string> ins;
        ir_emit(irs[a], [](int sym, int i) { return 8 * sym + i; }, 64, ins);
        printf("        \".L%s%d_%%=:\\n\\t\"\n", name, a);
        for (const auto& s : ins) printf("        \"%s\\n\\t\"\n", s.c_str());
        if (a < 7) printf("        \"s_branch .L%send_%%=\\n\\t\"\n", name);
    }
    printf("        \".L%send_%%=:\"\n        :", name);
    for (int j = 8 * G; j < 8 * G + 8; ++j)
        for (int i = 0; i < 8; ++i) printf(" \"+v\"(X[%d][%d]),", j, i);
    print_temps_ops(nt);
    printf("\n        : \"s\"(A) : \"scc\");\n}\n");
}

// Large layers of half 1, the merged middle pair and the large layers of half 0 (the
// work between the second exchange read and the third exchange, bs8.hpp
// large_ifft_h<1> + large_mid + large_fft_h<0>) as ONE optimized block: %0..%127 X,
// %128.. temporaries.
static void emit_lmid(const char* name) {
    const int kOffEnc = 127;
    auto e = [](unsigned L) { return L == 255u ? 0u : (unsigned)kGf8.exp[L]; };
    const unsigned sum = e(kGf8.skew[kOffEnc + 64]) ^ e(kGf8.skew[63]);
    const unsigned mid = sum == 0 ? 255u : (unsigned)kGf8.log[sum];
    std::vector<std::vector<Bfly>> layers;
    for (int dh = 1; dh <= 4; dh <<= 1) {  // IFFT d = 8, 16, 32 on h in [8, 16)
        std::vector<Bfly> l;
        for (int bb = 0; bb < 8; bb += 2 * dh) {
            const int hb = 8 + bb;
            for (int q = 0; q < dh; ++q) l.push_back({0, kGf8.skew[kOffEnc + 8 * hb + 8 * dh], hb + q, hb + q + dh});
        }
        layers.push_back(l);
    }
    {
        std::vector<Bfly> l;
        for (int q = 0; q < 8; ++q) l.push_back({2, mid, q, q + 8});
        layers.push_back(l);
    }
    for (int dh = 4; dh >= 1; dh >>= 1) {  // FFT d = 32, 16, 8 on h in [0, 8)
        std::vector<Bfly> l;
        for (int bb = 0; bb < 8; bb += 2 * dh)
            for (int q = 0; q < dh; ++q) l.push_back({1, kGf8.skew[-1 + 8 * bb + 8 * dh], bb + q, bb + q + dh});
        layers.push_back(l);
    }
    std::vector<IrOp> ir = block_ir(layers);
    for (const auto& l : layers)
        for (const Bfly& b : l) g_plain += (long)butterfly_ops(b.kind, b.L).size();
    g_opt += ir_count(ir);
    const int nt = std::max(1, ir_temps(ir));
    std::vector<std::string> ins;
    ir_emit(ir, [](int sym, int i) { return 8 * sym + i; }, 128, ins);
    printf("RSM_BS8_DEV void %s(uint32_t (&X)[16][8]) {\n", name);
    print_temps_decl(nt);
    printf("    asm volatile(\n");
    for (size_t i = 0; i < ins.size(); ++i) printf("        \"%s%s\"\n", ins[i].c_str(), i + 1 < ins.size() ? "\\n\\t" : "");
    printf("        :");
    for (int j = 0; j < 16; ++j)
        for (int i = 0; i < 8; ++i) printf(" \"+v\"(X[%d][%d]),", j, i);
    print_temps_ops(nt);
    printf(");\n}\n");
}

// Half-split exchange (kernels_gf8_bs.hip, bs_split_wave): half G is a transpose,
// wave u's register 8G + v -> wave v's register 8G + u, through LDS entries
//   (plane pair q = p / 2, destination v, source u) at ((q * 8 + v) * 8 + u) * 512 + lane * 8 + (p % 2) * 4
// (a reader's ds_read_b64 returns planes 2q, 2q + 1 of ONE source symbol, so the pair
// it fills is two registers of the same symbol -- the round-2 mapping paired one plane
// of two symbols, and the allocator paid ~100 v_mov and 12 VGPRs to re-pair them for the
// byte stores; the writers' lanes are 8 B apart: a 2-way bank overlap that costs
// ds_write_b32 nothing).
// xch_write_hG: 64 ds_write_b32, no wait (the caller waits and keeps X live until then);
//   %0..%63 = X[8G + v][p] (operand 8v + p), %64 = lds + lane*8 + u*512, %65 = %64 + 65536.
// xch_read_hG: 32 ds_read_b64 then lgkmcnt(0); outputs %0..%31 = T[u][q] (the pair
//   X[8G + u][2q], X[8G + u][2q + 1]), %32 = lds + lane*8 + v*4096, %33 = %32 + 65536.
static int wr_off(int p, int v) { return (((p / 2) % 2) * 8 + v) * 4096 + (p % 2) * 4; }
static bool wr_hi(int p) { return p >= 4; }
static void emit_xch(int G) {
    printf("RSM_BS8_DEV void xch_write_h%d(uint32_t (&X)[16][8], uint32_t va, uint32_t vb) {\n    asm volatile(\n", G);
    for (int p = 0; p < 8; ++p)
        for (int v = 0; v < 8; ++v)
            printf("        \"ds_write_b32 %%%d, %%%d offset:%d\\n\\t\"\n", wr_hi(p) ? 65 : 64, 8 * v + p, wr_off(p, v));
    printf("        :");
    for (int v = 0; v < 8; ++v)
        for (int p = 0; p < 8; ++p) printf(" \"+v\"(X[%d][%d])%s", 8 * G + v, p, (v == 7 && p == 7) ? "" : ",");
    printf("\n        : \"v\"(va), \"v\"(vb) : \"memory\");\n}\n");
    printf("RSM_BS8_DEV void xch_read_h%d(uint32_t (&X)[16][8], uint32_t ra, uint32_t rb) {\n"
           "    uint64_t T[8][4];\n    asm volatile(\n", G);
    for (int q = 0; q < 4; ++q)
        for (int u = 0; u < 8; ++u)
            printf("        \"ds_read_b64 %%%d, %%%d offset:%d\\n\\t\"\n", 4 * u + q, q < 2 ? 32 : 33, (q % 2) * 32768 + u * 512);
    printf("        \"s_waitcnt lgkmcnt(0)\"\n        :");
    for (int u = 0; u < 8; ++u)
        for (int q = 0; q < 4; ++q) printf(" \"=&v\"(T[%d][%d])%s", u, q, (u == 7 && q == 3) ? "" : ",");
    printf("\n        : \"v\"(ra), \"v\"(rb) : \"memory\");\n");
    printf("    for (int u = 0; u < 8; ++u)\n        for (int q = 0; q < 4; ++q) {\n"
           "            X[%d + u][2 * q] = (uint32_t)T[u][q];\n            X[%d + u][2 * q + 1] = (uint32_t)(T[u][q] >> 32);\n"
           "        }\n}\n", 8 * G, 8 * G);
}

// Bytes <-> planes transposes of the half-split kernel (round 3q): a ROTATE-and-select
// network instead of the shift pairs of bs8.hpp transpose8_dev.  The planes only need
// a common bit layout g(byte) -- every butterfly is bitwise -- not the identity one,
// so each swap of the 8x8 bit transpose moves ONE register by a rotation (v_alignbit,
// half rate on gfx950) and takes both outputs from it with two full-rate selects:
//   'b': r = rotl(b, s); b = M ? a : r; a = M ? r : a
//   'a': r = rotr(a, s); a = M ? r : b; b = M ? b : r
// (M: bit t of every byte set, s = 2^t).  The rotations leave plane p offset by a
// per-plane constant; five fix-up rotations align the planes (the minimum over the
// stage orders and per-pair choices: searched with a bit-label model, kTpFix below).
// Per 8 registers: 17 half-rate + 24 full-rate instructions against 20 + 28 for the
// shift form (16 % fewer VALU cycles).  g: byte b of register r -> bit (8b + r + 1) % 32.
// The inverse runs the steps backwards (same count), so planes -> bytes restores the
// exact byte order the stores need.
static const int kTpFix[8] = {1, 0, 0, 31, 0, 31, 29, 28};     // rotl per plane after the stages
static void tp_ops(bool inverse, const int (&w)[8], int tmp0, int tmp1, int mF0, int mCC, int mAA,
                   std::vector<std::string>& out) {
    static const int pairs[3][4][2] = {{{0, 1}, {2, 3}, {4, 5}, {6, 7}},
                                       {{0, 2}, {1, 3}, {4, 6}, {5, 7}},
                                       {{0, 4}, {1, 5}, {2, 6}, {3, 7}}};
    const char* cfg[3] = {"baab", "bbaa", "bbbb"};  // t = 0, 1, 2
    const int mask[3] = {mAA, mCC, mF0};
    char b[128];
    auto rot = [&](int d, int x, int rotr_amount) {  // d = rotr(x, amount)
        snprintf(b, sizeof b, "v_alignbit_b32 %%%d, %%%d, %%%d, %d", d, x, x, rotr_amount & 31);
        out.push_back(b);
    };
    auto sel = [&](int d, int m, int x, int y) {  // d = m ? x : y
        snprintf(b, sizeof b, "v_bitop3_b32 %%%d, %%%d, %%%d, %%%d bitop3:0xd8", d, y, x, m);
        out.push_back(b);
    };
    if (inverse)
        for (int p = 0; p < 8; ++p)
            if (kTpFix[p]) rot(w[p], w[p], kTpFix[p]);
    for (int si = 0; si < 3; ++si) {
        const int t = inverse ? si : 2 - si, s = 1 << t, M = mask[t];
        for (int q = 0; q < 4; q += 2) {  // two swaps interleaved (independent instructions)
            int tmp[2] = {tmp0, tmp1};
            std::vector<std::string> st[2];
            for (int h = 0; h < 2; ++h) {
                const int a = w[pairs[t][q + h][0]], bb = w[pairs[t][q + h][1]], r = tmp[h];
                const bool cb = cfg[t][q + h] == 'b';
                std::vector<std::string> o;
                std::swap(o, out);
                if (!inverse) {
                    if (cb) { rot(r, bb, 32 - s); sel(bb, M, a, r); sel(a, M, r, a); }
                    else { rot(r, a, s); sel(a, M, r, bb); sel(bb, M, bb, r); }
                } else {
                    if (cb) { sel(r, M, a, bb); sel(a, M, bb, a); rot(bb, r, s); }
                    else { sel(r, M, a, bb); sel(bb, M, bb, a); rot(a, r, 32 - s); }
                }
                std::swap(o, out);
                st[h] = o;
            }
            for (int i = 0; i < 3; ++i) out.push_back(st[0][i]), out.push_back(st[1][i]);
        }
    }
    if (!inverse)
        for (int p = 0; p < 8; ++p)
            if (kTpFix[p]) rot(w[p], w[p], 32 - kTpFix[p]);
}
// standalone tp_fwd_dev / tp_inv_dev (one symbol's 8 registers): %0..%7 w, %8 %9
// temporaries, %10..%12 the masks 0xF0F0F0F0, 0xCCCCCCCC, 0xAAAAAAAA (SGPRs)
static void emit_tp(const char* name, bool inverse) {
    std::vector<std::string> ops;
    const int w[8] = {0, 1, 2, 3, 4, 5, 6, 7};
    tp_ops(inverse, w, 8, 9, 10, 11, 12, ops);
    printf("RSM_BS8_DEV void %s(uint32_t (&w)[8]) {\n    uint32_t t0, t1;\n    asm volatile(\n", name);
    for (size_t i = 0; i < ops.size(); ++i) printf("        \"%s%s\"\n", ops[i].c_str(), i + 1 < ops.size() ? "\\n\\t" : "");
    printf("        : \"+v\"(w[0]), \"+v\"(w[1]), \"+v\"(w[2]), \"+v\"(w[3]), \"+v\"(w[4]), \"+v\"(w[5]), \"+v\"(w[6]), "
           "\"+v\"(w[7]),\n          \"=&v\"(t0), \"=&v\"(t1)\n"
           "        : \"s\"(0xF0F0F0F0u), \"s\"(0xCCCCCCCCu), \"s\"(0xAAAAAAAAu));\n}\n");
}

// Interleaved phases of the half-split schedule: the 64 exchange writes of half W
// (ds_write_b32, entries as in emit_xch) spread evenly through the VALU work of the
// OTHER half, so the LDS takes the writes while the SIMDs compute (a separate asm
// block of 64 writes stalls the wave until the LDS has accepted them).  VALU work:
//   kind 0 / 3: bytes -> planes / planes -> bytes of registers 8(1-W) .. 8(1-W)+7 (tp_ops);
//   kind 1: large IFFT of half 1-W (bs8.hpp large_ifft_h);  kind 2: large FFT of half 1-W.
// Operands: %0..%127 X[j][i] (8j + i), %128..%131 temporaries, %132..%137 the transpose
// masks (SGPRs), %138 / %139 the write addresses (p < 4 / p >= 4).
static void emit_phase(const char* name, int W, int kind) {
    const int V = 1 - W;
    std::vector<std::string> valu, wr;
    auto reg = [](int j, int i) { return 8 * j + i; };
    // temporaries: 2 for tp_ops, 4 for the shift form, the networks' need for butterflies
    std::vector<Bfly> bs;
    if (kind == 1 || kind == 2) {
        const int kOffEnc = 127;
        for (int li = 0; li < 3; ++li) {
            const int dh = kind == 1 ? (1 << li) : (4 >> li);
            for (int bb = 0; bb < 8; bb += 2 * dh) {
                const int hb = 8 * V + bb;
                const unsigned L = kind == 1 ? kGf8.skew[kOffEnc + 8 * hb + 8 * dh] : kGf8.skew[-1 + 8 * hb + 8 * dh];
                for (int q = 0; q < dh; ++q) bs.push_back({kind == 1 ? 0 : 1, L, hb + q, hb + q + dh});
            }
        }
    }
    std::vector<IrOp> ir;
    if (kind == 1 || kind == 2) ir = opt_block(bs, 4);
    const int nt = kind == 4 ? 4 : (kind == 0 || kind == 3) ? 2 : std::max(1, ir_temps(ir));
    // masks: the shift form (kind 4) 0x0F.., 0xF0.., 0x33.., 0xCC.., 0x55.., 0xAA.. at mk .. mk + 5;
    // the rotate-and-select transposes (kinds 0, 3) only 0xF0.., 0xCC.., 0xAA.. at mk .. mk + 2;
    // the butterfly phases none (every SGPR a block holds is one the compiler must
    // otherwise keep elsewhere -- spills to VGPR lanes, reloaded with v_readlane)
    const int nm = kind == 4 ? 6 : (kind == 0 || kind == 3) ? 3 : 0;
    const int mk = 128 + nt;
    const int va = mk + nm, vb = mk + nm + 1;
    for (int p = 0; p < 8; ++p)
        for (int v = 0; v < 8; ++v) {
            char b[96];
            snprintf(b, sizeof b, "ds_write_b32 %%%d, %%%d offset:%d", wr_hi(p) ? vb : va, 8 * (8 * W + v) + p,
                     wr_off(p, v));
            wr.push_back(b);
        }
    if (kind == 0 || kind == 3) {
        // bytes -> planes (kind 0) / planes -> bytes (kind 3): the rotate-and-select
        // network of tp_ops, one symbol after the other
        for (int j = 8 * V; j < 8 * V + 8; ++j) {
            const int w[8] = {reg(j, 0), reg(j, 1), reg(j, 2), reg(j, 3), reg(j, 4), reg(j, 5), reg(j, 6), reg(j, 7)};
            tp_ops(kind == 3, w, 128, 129, mk, mk + 1, mk + 2, valu);
        }
    } else if (kind == 4) {
        // transpose8_dev, same instruction sequence (bs8.hpp): the round-3 shift form, an
        // involution, kept for the diagnostic A/B (bs_split_wave bit 8388608)
        struct G { int a0, b0, a1, b1, s, m, mh; };
        const G gs[6] = {{0, 4, 1, 5, 4, mk, mk + 1}, {2, 6, 3, 7, 4, mk, mk + 1}, {0, 2, 1, 3, 2, mk + 2, mk + 3},
                         {4, 6, 5, 7, 2, mk + 2, mk + 3}, {0, 1, 2, 3, 1, mk + 4, mk + 5}, {4, 5, 6, 7, 1, mk + 4, mk + 5}};
        for (int j = 8 * V; j < 8 * V + 8; ++j)
            for (const G& g : gs) {
                char b[128];
                auto shl = [&](int d, int src) {
                    if (g.s == 1) snprintf(b, sizeof b, "v_add_u32 %%%d, %%%d, %%%d", d, reg(j, src), reg(j, src));
                    else snprintf(b, sizeof b, "v_lshlrev_b32 %%%d, %d, %%%d", d, g.s, reg(j, src));
                    valu.push_back(b);
                };
                shl(128, g.b0);
                snprintf(b, sizeof b, "v_lshrrev_b32 %%129, %d, %%%d", g.s, reg(j, g.a0));
                valu.push_back(b);
                shl(130, g.b1);
                snprintf(b, sizeof b, "v_lshrrev_b32 %%131, %d, %%%d", g.s, reg(j, g.a1));
                valu.push_back(b);
                snprintf(b, sizeof b, "v_bitop3_b32 %%%d, %%%d, %%128, %%%d bitop3:0xd8", reg(j, g.a0), reg(j, g.a0), g.mh);
                valu.push_back(b);
                snprintf(b, sizeof b, "v_bitop3_b32 %%%d, %%%d, %%129, %%%d bitop3:0xd8", reg(j, g.b0), reg(j, g.b0), g.m);
                valu.push_back(b);
                snprintf(b, sizeof b, "v_bitop3_b32 %%%d, %%%d, %%130, %%%d bitop3:0xd8", reg(j, g.a1), reg(j, g.a1), g.mh);
                valu.push_back(b);
                snprintf(b, sizeof b, "v_bitop3_b32 %%%d, %%%d, %%131, %%%d bitop3:0xd8", reg(j, g.b1), reg(j, g.b1), g.m);
                valu.push_back(b);
            }
    } else {
        ir_emit(ir, [](int sym, int i) { return 8 * sym + i; }, 128, valu);
    }
    printf("RSM_BS8_DEV void %s(uint32_t (&X)[16][8], uint32_t va, uint32_t vb) {\n", name);
    print_temps_decl(nt);
    printf("    asm volatile(\n");
    const size_t n = valu.size();
    size_t w = 0;
    for (size_t i = 0; i < n; ++i) {
        // write w goes after VALU instruction floor((w + 1) * n / 65) (evenly spread)
        while (w < wr.size() && (w + 1) * n / (wr.size() + 1) <= i) printf("        \"%s\\n\\t\"\n", wr[w++].c_str());
        printf("        \"%s\\n\\t\"\n", valu[i].c_str());
    }
    while (w < wr.size()) printf("        \"%s\\n\\t\"\n", wr[w++].c_str());
    printf("        \"s_nop 0\"\n        :");
    for (int j = 0; j < 16; ++j)
        for (int i = 0; i < 8; ++i) printf(" \"+v\"(X[%d][%d]),", j, i);
    for (int t = 0; t < nt; ++t) printf(" \"=&v\"(t%d)%s", t, t + 1 < nt ? "," : "");
    printf("\n        : ");
    if (nm == 6)
        printf("\"s\"(0x0F0F0F0Fu), \"s\"(0xF0F0F0F0u), \"s\"(0x33333333u), \"s\"(0xCCCCCCCCu), "
               "\"s\"(0x55555555u), \"s\"(0xAAAAAAAAu), ");
    else if (nm == 3)
        printf("\"s\"(0xF0F0F0F0u), \"s\"(0xCCCCCCCCu), \"s\"(0xAAAAAAAAu), ");
    printf("\"v\"(va), \"v\"(vb) : \"memory\");\n}\n");
}


int main() {
    printf("// GENERATED by gen/gen_bs8_small.cpp -- do not edit.\n");
    emit_xch(0);
    emit_xch(1);
    emit_phase("ph_w0_tr1", 0, 0);    // S' -> L half 0  || transposes of h1 (bytes -> planes)
    emit_phase("ph_w1_lifft0", 1, 1); // S' -> L half 1  || large IFFT of h0
    emit_phase("ph_w0_lfft1", 0, 2);  // L -> S' half 0  || large FFT of h1
    emit_phase("ph_w1_tr0", 1, 3);    // L -> S' half 1  || transposes of h0 (planes -> bytes)
    printf("#ifdef RSM_DIAG\n");
    emit_phase("ph_w0_tr1_old", 0, 4);
    emit_phase("ph_w1_tr0_old", 1, 4);
    printf("#endif\n");
    emit_lmid("lmid_all");
    emit_tp("tp_fwd_dev", false);
    emit_tp("tp_inv_dev", true);
    emit("small_ifft_all", true);
    emit("small_fft_all", false);
    emit_half("small_ifft_h0_all", true, 0);
    emit_half("small_ifft_h1_all", true, 1);
    emit_half("small_fft_h0_all", false, 0);
    emit_half("small_fft_h1_all", false, 1);
    fprintf(stderr, "half-split blocks: %ld VALU butterfly by butterfly, %ld optimized\n", g_plain, g_opt);
    return 0;
}
