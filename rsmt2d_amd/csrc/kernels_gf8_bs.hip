// kernels_gf8_bs.hip -- bit-sliced GF(2^8) encode for M = 128 (65 <= k <= 128).
//
// The byte-table kernel (kernels_gf8.hip) spends ~10 VALU per 4 bytes per GF
// multiply and is VALU-bound.  Here 32 bytes of a symbol are 8 bit-planes and a
// multiply by a constant is a short network of 3-input XORs (bs8.hpp,
// gen/bs8_net.hpp).  A lane can hold 16 symbols x 8 planes (128 VGPRs), not the
// whole 128-symbol codeword, so the transform is split between the 8 wavefronts
// of a workgroup (bs8.hpp):
//
//   set       = 64 lanes x 32 bytes = 2 KiB of share width (e.g. four 512-byte
//               codewords), all 128 symbols of it;
//   wave w    : small layout, symbols e = 16w + j: IFFT layers d = 1,2,4
//   LDS       : exchange, one bit-plane per round ([symbol][lane] x 4 B)
//   wave w    : large layout, symbols e = 8h + w: IFFT d = 8..32, the merged
//               d = 64 pair, FFT d = 32..8
//   LDS back, FFT layers d = 4,2,1, planes -> bytes, store.
//
// All eight waves run ONE instruction stream: only the small layers' twiddles
// depend on w, and each direction is one asm statement that branches on w inside
// (bs8_small.inc).  Eight template copies of the whole per-wave program overflow
// the instruction cache (measured 1.8x slower) and a control-flow merge of the
// 128 planes costs ~250 register copies per wave (measured).
//
// Memory: lane l holds bytes [16l, 16l+16) and [1024+16l, +16) of the set's 2 KiB
// (two dwordx4 per symbol; every wave instruction covers 1 KiB contiguous per
// codeword run).  Same CodewordSet contract as encode_gf8_kernel (row pass,
// column pass, slices); callers with an index list use the byte-table kernel.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <atomic>
#include "bs8.hpp"
#include "rsm_kernels.hpp"

namespace rsm {

namespace {

constexpr uint32_t kOobBs = 0x80000000u;
constexpr uint32_t kSetBytes = 2048;

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// Buffer resource as a plain SGPR quad (the LDS-DMA loads are inline asm).
__device__ __forceinline__ v4u make_srd(const void* p) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    v4u r;
    r.x = __builtin_amdgcn_readfirstlane((uint32_t)a);
    r.y = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) & 0xFFFFu;  // stride 0
    r.z = kOobBs;                                                          // num_records
    r.w = 0x00020000u;
    return r;
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t as_rsrc(v4u srd) {
    void* u = reinterpret_cast<void*>(((uint64_t)srd.y << 32) | srd.x);
    return __builtin_amdgcn_make_buffer_rsrc(u, (short)0, (int)kOobBs, 0x00020000);
}

// Per-set addressing: a set is virtual bytes [2048 t, 2048 t + 2048) of the
// concatenated shares of the CodewordSet; lane l's two 16-byte pieces are at
// set bytes 16l and 1024 + 16l.  off[] are relative to the set's first codeword.
struct SetAddr {
    v4u rs, ro;
    uint32_t off[2];
};

// 32-bit index math (bs128_applicable guarantees count * S < 2^31).
__device__ __forceinline__ SetAddr set_addr(const CodewordSet& cs, uint32_t t, uint32_t lane) {
    SetAddr a;
    const uint32_t S = cs.S, ps = cs.per_square;
    const uint32_t v0 = t * kSetBytes;
    const uint32_t q0 = __builtin_amdgcn_readfirstlane(v0 / S);
    const uint32_t r0 = v0 - q0 * S;
    const uint32_t sq0 = __builtin_amdgcn_readfirstlane(q0 / ps);
    const uint64_t rel0 = (uint64_t)sq0 * cs.square_stride + (uint64_t)(q0 - sq0 * ps) * cs.cw_stride;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint32_t v = r0 + 1024u * h + 16u * lane;  // < S + 2048
        const uint32_t dq = v / S;
        const uint32_t q = q0 + dq;
        const uint32_t sq = q / ps;
        const uint64_t rel = (uint64_t)sq * cs.square_stride + (uint64_t)(q - sq * ps) * cs.cw_stride;
        a.off[h] = q < cs.count ? (uint32_t)(rel - rel0) + (v - dq * S) : kOobBs;
    }
    a.rs = make_srd(cs.base + rel0);
    a.ro = make_srd(cs.out_base + rel0);
    return a;
}

// Per-lane part of set_addr when it is the same for every set (round 3q): the share
// size S divides the set width (2048 B), so every set starts at a codeword boundary
// (r0 = 0) and covers G = 2048 / S whole codewords, and per_square and count are
// multiples of G, so those G codewords lie in one square.  Lane offsets are then
// fixed (codeword dq = v / S of the set, byte v % S, v = 1024 h + 16 lane), and a set
// costs one wave-uniform division instead of four per-lane ones.
struct LaneGeo {
    uint32_t off[2];
    uint32_t shift;  // log2(G)
};
__host__ __device__ inline bool lane_geo_ok(const CodewordSet& cs) {
    const uint32_t S = cs.S;
    if (S == 0 || kSetBytes % S != 0 || (S & (S - 1)) != 0 || cs.indices != nullptr) return false;
    const uint32_t G = kSetBytes / S;
    return cs.per_square % G == 0 && cs.count % G == 0;
}
__device__ __forceinline__ LaneGeo lane_geo(const CodewordSet& cs, uint32_t lane) {
    LaneGeo g{};
    const uint32_t S = cs.S, G = kSetBytes / S;
    g.shift = 31u - (uint32_t)__builtin_clz(G);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint32_t v = 1024u * h + 16u * lane;
        const uint32_t dq = v >> (31u - (uint32_t)__builtin_clz(S));
        g.off[h] = (uint32_t)(dq * cs.cw_stride) + (v & (S - 1u));
    }
    return g;
}
__device__ __forceinline__ SetAddr set_addr_geo(const CodewordSet& cs, const LaneGeo& g, uint32_t t) {
    SetAddr a;
    const uint32_t q0 = t << g.shift;
    const uint32_t sq0 = __builtin_amdgcn_readfirstlane(q0 / cs.per_square);
    const uint64_t rel0 = (uint64_t)sq0 * cs.square_stride + (uint64_t)(q0 - sq0 * cs.per_square) * cs.cw_stride;
    a.off[0] = g.off[0];
    a.off[1] = g.off[1];
    a.rs = make_srd(cs.base + rel0);
    a.ro = make_srd(cs.out_base + rel0);
    return a;
}

__device__ __forceinline__ uint32_t sym_off(uint32_t e, uint32_t k, uint32_t base, uint32_t es) {
    return __builtin_amdgcn_readfirstlane(e < k ? base + e * es : kOobBs);
}

constexpr int kPre = 8;  // symbols j < kPre of each wave arrive by LDS-DMA

// LDS-DMA (buffer_load_dwordx4 ... lds): 16 B per lane to M0 + 16*lane.  Inline
// asm, so the compiler neither tracks nor conservatively drains it; the caller
// waits with an explicit vmcnt.
template <bool NT>
__device__ __forceinline__ void dma16(uint32_t lds_byte, uint32_t voff, v4u srd, uint32_t soff) {
    uint32_t keep;  // M0 is compiler-reserved: save and restore it around the DMA
    if constexpr (NT)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 4\n\t"
                     "buffer_load_dwordx4 %2, %3, %4 offen nt lds\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "s"(lds_byte), "v"(voff), "s"(srd), "s"(soff)
                     : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 4\n\t"
                     "buffer_load_dwordx4 %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "s"(lds_byte), "v"(voff), "s"(srd), "s"(soff)
                     : "memory");
}

// LDS traffic as inline asm with immediate offsets: left to the compiler, the 32
// loop-invariant per-symbol addresses are hoisted out of the set loop into 16+
// VGPRs and the prefetch registers spill.  A read group waits for its own data
// (lgkmcnt(0) inside the statement), so the compiler never sees stale outputs.
template <uint32_t O0, uint32_t STEP>
__device__ __forceinline__ void ds_r16x8(uint32_t base, v4u (&r)[8]) {
    asm volatile(
        "ds_read_b128 %0, %8 offset:%9\n\t"
        "ds_read_b128 %1, %8 offset:%10\n\t"
        "ds_read_b128 %2, %8 offset:%11\n\t"
        "ds_read_b128 %3, %8 offset:%12\n\t"
        "ds_read_b128 %4, %8 offset:%13\n\t"
        "ds_read_b128 %5, %8 offset:%14\n\t"
        "ds_read_b128 %6, %8 offset:%15\n\t"
        "ds_read_b128 %7, %8 offset:%16\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]), "=&v"(r[6]), "=&v"(r[7])
        : "v"(base), "i"(O0), "i"(O0 + STEP), "i"(O0 + 2 * STEP), "i"(O0 + 3 * STEP), "i"(O0 + 4 * STEP),
          "i"(O0 + 5 * STEP), "i"(O0 + 6 * STEP), "i"(O0 + 7 * STEP)
        : "memory");
}

constexpr uint32_t kDmaBytes = 128u * 1024u;
constexpr uint32_t kXchBytes = 32u * 1024u;

// Exchange buffer E [symbol 128][lane 64] x 4 B at LDS offset 0 (so that the
// ds_write_addtid_b32 base fits M0[15:0]); one bit-plane per round.
//   small layout (e = 16A + j): byte 4096 A + 256 j;   large (e = 8h + A): 256 A + 2048 h
// Writes: ds_write_b32 with a per-lane address VGPR (4 LDS cycles per instruction),
// or -- ADDTID -- ds_write_addtid_b32 (address = M0 + offset + 4 * lane, 2 cycles,
// MI355X_MICROARCH.md LDS table), M0 set and restored inside the statement.
#define RSM_XW(j, o) "ds_write_b32 %17, %" #j " offset:" #o "\n\t"
#define RSM_XWT(j, o) "ds_write_addtid_b32 %" #j " offset:" #o "\n\t"
#define RSM_XR(j, o) "ds_read_b32 %" #j ", %18 offset:" #o "\n\t"
#define RSM_XOPS(p)                                                                                             \
    : "+v"(X[0][p]), "+v"(X[1][p]), "+v"(X[2][p]), "+v"(X[3][p]), "+v"(X[4][p]), "+v"(X[5][p]), "+v"(X[6][p]), \
      "+v"(X[7][p]), "+v"(X[8][p]), "+v"(X[9][p]), "+v"(X[10][p]), "+v"(X[11][p]), "+v"(X[12][p]),           \
      "+v"(X[13][p]), "+v"(X[14][p]), "+v"(X[15][p]), "=&s"(keep)                                             \
    : "v"(wb), "v"(rb), "s"(ws)                                                                               \
    : "memory"
#define RSM_M0_SET "s_mov_b32 %16, m0\n\ts_mov_b32 m0, %19\n\ts_nop 0\n\t"
#define RSM_M0_RESTORE "s_mov_b32 m0, %16\n\t"
#define RSM_W_SMALL(W) W(0, 0) W(1, 256) W(2, 512) W(3, 768) W(4, 1024) W(5, 1280) W(6, 1536) W(7, 1792) \
    W(8, 2048) W(9, 2304) W(10, 2560) W(11, 2816) W(12, 3072) W(13, 3328) W(14, 3584) W(15, 3840)
#define RSM_W_LARGE(W) W(0, 0) W(1, 2048) W(2, 4096) W(3, 6144) W(4, 8192) W(5, 10240) W(6, 12288) W(7, 14336) \
    W(8, 16384) W(9, 18432) W(10, 20480) W(11, 22528) W(12, 24576) W(13, 26624) W(14, 28672) W(15, 30720)
#define RSM_SYNC "s_waitcnt lgkmcnt(0)\n\ts_barrier\n\t"
// wb / ws: write base (VGPR with the lane term / SGPR without), rb: read base (VGPR)
template <int p, bool ADDTID>
__device__ __forceinline__ void xch_to_large(uint32_t (&X)[16][8], uint32_t wb, uint32_t ws, uint32_t rb) {
    uint32_t keep;
    if constexpr (ADDTID)
        asm volatile(RSM_M0_SET RSM_W_SMALL(RSM_XWT) RSM_M0_RESTORE RSM_SYNC RSM_W_LARGE(RSM_XR)
                     "s_waitcnt lgkmcnt(0)\n\ts_barrier" RSM_XOPS(p));
    else
        asm volatile(RSM_W_SMALL(RSM_XW) RSM_SYNC RSM_W_LARGE(RSM_XR) "s_waitcnt lgkmcnt(0)\n\ts_barrier"
                     RSM_XOPS(p));
}
template <int p, bool ADDTID>
__device__ __forceinline__ void xch_to_small(uint32_t (&X)[16][8], uint32_t wb, uint32_t ws, uint32_t rb) {
    uint32_t keep;
    if constexpr (ADDTID)
        asm volatile(RSM_M0_SET RSM_W_LARGE(RSM_XWT) RSM_M0_RESTORE RSM_SYNC RSM_W_SMALL(RSM_XR)
                     "s_waitcnt lgkmcnt(0)\n\ts_barrier" RSM_XOPS(p));
    else
        asm volatile(RSM_W_LARGE(RSM_XW) RSM_SYNC RSM_W_SMALL(RSM_XR) "s_waitcnt lgkmcnt(0)\n\ts_barrier"
                     RSM_XOPS(p));
}
#undef RSM_XW
#undef RSM_XWT
#undef RSM_XR
#undef RSM_XOPS
#undef RSM_M0_SET
#undef RSM_M0_RESTORE
#undef RSM_W_SMALL
#undef RSM_W_LARGE
#undef RSM_SYNC

template <bool NT, int J0 = 0, int J1 = kPre>
__device__ __forceinline__ void issue_dma_rt(const CodewordSet& cs, const SetAddr& a, uint32_t lds_base, uint32_t A) {
    const uint32_t k = cs.k, es = (uint32_t)cs.elem_stride;
    bs8::sfor<J1 - J0>([&](auto J) {
        constexpr int j = J0 + decltype(J)::value;
        const uint32_t so = sym_off(16u * A + j, k, 0, es);
        const uint32_t l = __builtin_amdgcn_readfirstlane(lds_base + kXchBytes + A * (kPre * 2048u) + j * 2048u);
        dma16<NT>(l, a.off[0], a.rs, so);
        dma16<NT>(l + 1024u, a.off[1], a.rs, so);
    });
}

template <bool NT>
__device__ __forceinline__ void issue_direct_rt(const CodewordSet& cs, const SetAddr& a, uint32_t A,
                                                uint32_t (&P)[16 - kPre][8]) {
    const uint32_t k = cs.k, es = (uint32_t)cs.elem_stride;
    const __amdgpu_buffer_rsrc_t rs = as_rsrc(a.rs);
    bs8::sfor<16 - kPre>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t so = sym_off(16u * A + kPre + j, k, 0, es);
        const v4u x = __builtin_amdgcn_raw_buffer_load_b128(rs, a.off[0], so, NT ? 2 : 0);
        const v4u y = __builtin_amdgcn_raw_buffer_load_b128(rs, a.off[1], so, NT ? 2 : 0);
        P[j][0] = x.x; P[j][1] = x.y; P[j][2] = x.z; P[j][3] = x.w;
        P[j][4] = y.x; P[j][5] = y.y; P[j][6] = y.z; P[j][7] = y.w;
    });
}

// MODE bits: 8 = exchange writes by ds_write_addtid_b32, 32 = non-temporal loads
// (production: 40), 16 = non-temporal stores (A/B);
// diagnostics: 2 = no arithmetic, 4 = no global memory.
// REV: sets are taken in reverse order (the column pass walks the squares the row
// pass just wrote from the most recent one back, so the first squares it reads are
// still in the 256 MiB Infinity Cache).
template <int MODE>
__device__ __forceinline__ void bs_uni_wave(const CodewordSet& cs, uint32_t sets, uint32_t rev, uint32_t lds_base,
                                            uint32_t A) {
    constexpr bool ARITH = !(MODE & 2), ADDTID = (MODE & 8) != 0, NTS = (MODE & 16) != 0, NTL = (MODE & 32) != 0;
    const bool MEM = !(MODE & 4) || cs.S == 1;  // runtime-false in mode 4 (keeps the code alive)
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t G = gridDim.x;
    const uint32_t k = cs.k, es = (uint32_t)cs.elem_stride, oo = (uint32_t)cs.out_offset;
    // LDS: E (exchange, 32 KiB) at 0, D (LDS-DMA landing zone, 128 KiB) after it
    const uint32_t dread = lds_base + kXchBytes + A * 16384u + lane * 16u;
    const uint32_t s_small = __builtin_amdgcn_readfirstlane(lds_base + 4096u * A);
    const uint32_t s_large = __builtin_amdgcn_readfirstlane(lds_base + 256u * A);
    const uint32_t e_small = s_small + lane * 4u, e_large = s_large + lane * 4u;
    uint32_t X[16][8];
    uint32_t P[16 - kPre][8];

    // rev bit 1: XCD-grouped order -- within every full group of G sets, block b
    // (XCD b % 8 under round-robin placement) takes set (b % 8) * G/8 + b / 8, so the
    // blocks of one XCD stream adjacent strips (speed only: any bijection is correct)
    auto addr = [&](uint32_t tt) {
        if ((rev & 2u) && (G & 7u) == 0 && (tt / G + 1u) * G <= sets) {
            const uint32_t b = tt % G;
            tt = tt - b + (b & 7u) * (G >> 3) + (b >> 3);
        }
        return set_addr(cs, (rev & 1u) ? sets - 1u - tt : tt, lane);
    };
    uint32_t t = blockIdx.x;
    SetAddr a = addr(t);
    if (MEM) {
        issue_dma_rt<NTL>(cs, a, lds_base, A);
        issue_direct_rt<NTL>(cs, a, A, P);
    }
    // vmcnt(0) through the builtin (gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15): the
    // compiler sees it, so its own wait for P at the loop head stays vmcnt(32).  LDS-DMA
    // data is read only after the wave's vmcnt AND a barrier (cdna_hip_programming.md
    // §5.7 item 1).
    __builtin_amdgcn_s_waitcnt(0x0F70);
    asm volatile("s_barrier" ::: "memory");
    for (;;) {
        {
            v4u g[8];
            bs8::sfor<2>([&](auto Hh) {
                constexpr int hh = decltype(Hh)::value;
                ds_r16x8<8192 * hh, 1024>(dread, g);
                bs8::sfor<4>([&](auto J) {
                    constexpr int j = 4 * hh + decltype(J)::value;
                    const v4u x = g[2 * (j & 3)], y = g[2 * (j & 3) + 1];
                    X[j][0] = x.x; X[j][1] = x.y; X[j][2] = x.z; X[j][3] = x.w;
                    X[j][4] = y.x; X[j][5] = y.y; X[j][6] = y.z; X[j][7] = y.w;
                });
            });
        }
        bs8::sfor<16 - kPre>([&](auto J) {
            constexpr int j = decltype(J)::value;
            bs8::sfor<8>([&](auto I) { X[kPre + j][decltype(I)::value] = P[j][decltype(I)::value]; });
        });
        const uint32_t tn = t + G;
        const bool more = tn < sets;
        SetAddr an = a;
        // LATE (MODE 64, A/B): the direct half of the next set's loads is issued after
        // the first exchange instead of with the LDS-DMA half (spreads the reads)
        // A/B: MODE 64 issues the direct half of the next set's loads after the first
        // exchange, 128 after the large layers; 256 splits the LDS-DMA half (symbols
        // j >= kPre/2 after the first exchange) -- spreading the reads over the set
        constexpr bool LATE = (MODE & (64 | 128)) != 0, LATER = (MODE & 128) != 0, SPLIT = (MODE & 256) != 0;
        if (more) {
            an = addr(tn);
            if (MEM) {
                if constexpr (SPLIT) issue_dma_rt<NTL, 0, kPre / 2>(cs, an, lds_base, A);
                else issue_dma_rt<NTL>(cs, an, lds_base, A);
                if constexpr (!LATE) issue_direct_rt<NTL>(cs, an, A, P);
            }
        }
        if constexpr (ARITH) {
            bs8::sfor<16>([&](auto J) { bs8::transpose8_dev(X[decltype(J)::value]); });
            bs8::small_ifft_all(X, A);
        }
        bs8::sfor<8>([&](auto Pp) { xch_to_large<decltype(Pp)::value, ADDTID>(X, e_small, s_small, e_large); });
        if (more && MEM) {
            if constexpr (SPLIT) issue_dma_rt<NTL, kPre / 2, kPre>(cs, an, lds_base, A);
            if constexpr (LATE && !LATER) issue_direct_rt<NTL>(cs, an, A, P);
        }
        if constexpr (ARITH) bs8::large_ifft_fft(X);
        if constexpr (LATER)
            if (more && MEM) issue_direct_rt<NTL>(cs, an, A, P);
        bs8::sfor<8>([&](auto Pp) { xch_to_small<decltype(Pp)::value, ADDTID>(X, e_large, s_large, e_small); });
        if constexpr (ARITH) bs8::small_fft_all(X, A);
        {
            const __amdgpu_buffer_rsrc_t ro = as_rsrc(a.ro);
            bs8::sfor<16>([&](auto J) {
                constexpr int j = decltype(J)::value;
                if constexpr (ARITH) bs8::transpose8_dev(X[j]);
                const uint32_t so = sym_off(16u * A + j, k, oo, es);
                v4u x, y;
                x.x = X[j][0]; x.y = X[j][1]; x.z = X[j][2]; x.w = X[j][3];
                y.x = X[j][4]; y.y = X[j][5]; y.z = X[j][6]; y.w = X[j][7];
                if (MEM) {
                    __builtin_amdgcn_raw_buffer_store_b128(x, ro, a.off[0], so, NTS ? 2 : 0);
                    __builtin_amdgcn_raw_buffer_store_b128(y, ro, a.off[1], so, NTS ? 2 : 0);
                }
                // The next statement is an asm block whose early-clobber temporaries the
                // compiler may place in the data registers of the store just issued; a
                // dwordx4 store reads its data over several cycles and the hazard
                // recognizer does not look inside asm, so pad here (without it the last
                // lane groups of the second store intermittently wrote the temporaries).
                asm volatile("s_nop 2" ::: "memory");
            });
        }
        if (!more) break;
        t = tn;
        a = an;
        // issue order: DMA(t) [16], direct(t) [16], stores(t - G) [32]; then the
        // barrier that makes the landed LDS-DMA data readable
        asm volatile("s_waitcnt vmcnt(32)\n\ts_barrier" ::: "memory");
    }
}

// PASS only names the launch in profiles (0 row pass, 1 column pass / other).
template <int MODE, int PASS>
__global__ __launch_bounds__(512, 1) void encode_gf8_bs128u_kernel(CodewordSet cs, uint32_t sets, uint32_t rev) {
    __shared__ uint32_t lds[(kDmaBytes + kXchBytes) / 4];
    if (blockIdx.x >= sets) return;
    bs_uni_wave<MODE>(cs, sets, rev, (uint32_t)(uintptr_t)lds, __builtin_amdgcn_readfirstlane(threadIdx.x >> 6));
}


// ---------------------------------------------------------------------------
// Queue-driven single-launch extension (QueuePlan, rsm_kernels.hpp): the
// production schedule for batches of k = 128 squares.
//
// Both passes of `count` squares in ONE persistent launch, so the column sets
// re-read Q0 and Q1 while they are still in the 256 MiB Infinity Cache instead of
// from HBM (the two-launch schedule moves 6k^2S per square, this one 4k^2S plus
// whatever misses).  A square's sets are of three kinds:
//   row sets      (rn): Q0 rows -> Q1 rows
//   Q0-col sets   (rn): Q0 columns -> Q2 columns        (no dependency)
//   Q1-col sets   (rn): Q1 columns -> Q3 columns        (need all rn row sets)
// Row and Q0-col sets form the MAIN sequence (one queue head): row sets of
// square s interleaved 1:1 with the Q0-col sets of square s - delay/rn (so both
// read a square's Q0 within a set or two of each other, and the last squares'
// Q0-col sets fill the tail).  A Q1-col set is never dequeued before it is
// ready: the workgroup whose row set completes a square (the last add on the
// square's counter) appends the square to a ready list, and Q1-col sets are
// taken from that list (second head) in preference to main items.
//
// Deadlock freedom: a workgroup waits only when the main sequence is exhausted,
// after publishing its own stored row set; every remaining row set is then held
// by a workgroup that finishes it without waiting, so every claimed Q1-col set
// becomes ready.  A claimed Q1-col set that is not ready yet (two workgroups raced
// for the last ready one) is kept in reserve while the workgroup takes main items.
//
// Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility): row sets store Q1
// `sc1`; every wave waits for its stores (vmcnt), a barrier, then ONE lane adds to
// the square's counter (agent scope); a consumer sees the square in the ready
// list through agent-scope loads, takes an agent acquire, and every wave loads
// after a barrier that follows it.  Waits are bounded: a stuck wait sets the
// error word and lets the launch drain (invalid output, never a hung GPU).
constexpr uint32_t kQMain = 0, kQHead1 = 32, kQReady = 64, kQRes = 96, kQErr = 128, kQExit = 160, kQLeft = 192,
                   kQRows = 224;
constexpr uint32_t kNone = 0xFFFFFFFFu, kQ1 = 0x80000000u, kQExitCheck = 0xFFFFFFFEu;
constexpr uint32_t kSpinLimit = 1u << 20;  // polls (~1 s) before a wait is declared stuck

__device__ __forceinline__ uint32_t q_add(uint32_t* w) {
    return __hip_atomic_fetch_add(w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t q_load(uint32_t* w) {
    return __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t q_sub(uint32_t* w) {
    return __hip_atomic_fetch_sub(w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void q_store(uint32_t* w, uint32_t v) {
    __hip_atomic_store(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// item word -> (row set?, set index in p.rows / p.cols); sq1 is a Q1 item's square
__device__ __forceinline__ void q_item(const QueuePlan& p, uint32_t it, uint32_t sq1, uint32_t& row, uint32_t& set) {
    if (it & kQ1) {
        row = 0u;
        set = sq1 * p.cn + p.rn + (it & ~kQ1) % p.rn;
        return;
    }
    const uint32_t N = p.count * p.rn, D = p.delay;
    uint32_t c;
    if (it < D) {
        row = 1u;
        set = it;
        return;
    }
    const uint32_t v = it - D;
    if (v < 2u * (N - D)) {
        const uint32_t pi = v >> 1;
        if (!(v & 1u)) {
            row = 1u;
            set = D + pi;
            return;
        }
        c = pi;
    } else {
        c = (N - D) + (v - 2u * (N - D));
    }
    row = 0u;
    set = (c / p.rn) * p.cn + c % p.rn;
}

// Thread 0's view of the queue.
struct QClaim {
    uint32_t res = kNone;   // a claimed Q1 item that was not ready yet
    uint32_t main_done = 0;
    uint32_t rc = 0, qh = 0;  // hints: ready squares, Q1 head (loaded half a set earlier)
};

// the square of Q1 item q when it is ready, else kNone
__device__ __forceinline__ uint32_t q_ready(const QueuePlan& p, uint32_t q) {
    const uint32_t s1 = q_load(&p.ctr[kQRows + p.count + q / p.rn]);
    return s1 ? s1 - 1u : kNone;
}

// This set's claim (its result is consumed half a set later).  A Q1 item is
// claimed only while the (stale) hint shows more than `margin` unclaimed ready
// ones, so a claim rarely overtakes the ready list; at the end of the main
// sequence any remaining Q1 item is claimed (and waited for).
__device__ __forceinline__ uint32_t q_claim(const QueuePlan& p, const QClaim& c) {
    if (c.res != kNone) return c.res;
    if (c.qh + p.margin < c.rc * p.rn) return kQ1 | q_add(&p.ctr[kQHead1]);
    if (!c.main_done) return q_add(&p.ctr[kQMain]);
    if (c.qh < c.rc * p.rn) return kQ1 | q_add(&p.ctr[kQHead1]);
    return c.qh < p.nq1 ? kQExitCheck : kNone;
}

// Main sequence exhausted and (as far as thread 0 knows) no ready Q1 item: leave
// the launch if the workgroups that stay still outnumber the unclaimed Q1 items
// (each of them takes one before it may leave: the count of live workgroups never
// drops below the unclaimed items, so none is stranded, and the CUs of the others
// go to the next launch on another stream); otherwise claim a Q1 item (it may have
// to be waited for).  Returns kNone (leave) or the claimed Q1 item.
__device__ __forceinline__ uint32_t q_leave_or_claim(const QueuePlan& p, uint32_t G) {
    const uint32_t e = q_add(&p.ctr[kQLeft]);
    uint32_t qh = q_load(&p.ctr[kQHead1]);
    qh = qh < p.nq1 ? qh : p.nq1;
    if (G - e - 1u >= p.nq1 - qh) return kNone;
    q_sub(&p.ctr[kQLeft]);
    return kQ1 | q_add(&p.ctr[kQHead1]);
}

// Synchronous take (prologue): a main item, else a Q1 item, waited for only when
// `wait` (the workgroup then holds no other item); otherwise rdy = 0 for a Q1 item
// that is not ready (the slow path waits for it after the first set).
__device__ __forceinline__ uint32_t q_wait(const QueuePlan& p, uint32_t it);
__device__ __forceinline__ uint32_t q_take(const QueuePlan& p, QClaim& c, bool wait, uint32_t& sq, uint32_t& rdy,
                                           uint32_t G) {
    sq = 0u;
    rdy = 1u;
    if (!c.main_done) {
        const uint32_t u = q_add(&p.ctr[kQMain]);
        if (u < p.nmain) return u;
        c.main_done = 1u;
    }
    const uint32_t it = q_leave_or_claim(p, G);
    if (it == kNone || (it & ~kQ1) >= p.nq1) return kNone;
    const uint32_t q = it & ~kQ1;
    if (wait) {
        sq = q_wait(p, kQ1 | q);
        if (sq == kNone) {  // stuck (error word set): take nothing, leave
            sq = 0u;
            return kNone;
        }
    } else {
        sq = q_ready(p, q);
        if (sq == kNone) {
            sq = 0u;
            rdy = 0u;
        } else {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
    }
    return kQ1 | q;
}

// Bounded wait for Q1 item `it`; returns its square, or kNone when the wait timed
// out (the error word is set; the caller skips the set -- no loads, no stores -- so
// a stuck wait corrupts no square, and the launch still drains).
__device__ __forceinline__ uint32_t q_wait(const QueuePlan& p, uint32_t it) {
    uint32_t s = kNone;
    for (uint32_t n = 0; (s = q_ready(p, it & ~kQ1)) == kNone; ++n) {
        if (n >= kSpinLimit) {
            q_store(&p.ctr[kQErr], 1u);
            return kNone;
        }
        __builtin_amdgcn_s_sleep(4);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    return s;
}

// The last row set of square sq is stored (old = rn - 1 from its counter add):
// append the square to the ready list.
__device__ __forceinline__ void q_publish(const QueuePlan& p, uint32_t sq) {
    const uint32_t slot = q_add(&p.ctr[kQRes]);
    q_store(&p.ctr[kQRows + p.count + slot], sq + 1u);
    q_add(&p.ctr[kQReady]);
}
__device__ __forceinline__ void q_signal(const QueuePlan& p, uint32_t sq) {
    if (q_add(&p.ctr[kQRows + sq]) == p.rn - 1u) q_publish(p, sq);
}

template <int MODE>
__device__ __forceinline__ void bs_queue_wave(const QueuePlan& p, uint32_t* lds, uint32_t lds_base, uint32_t A) {
    // Where the direct half of the next set's loads is issued: MODE 64 right after
    // the first exchange, 128 the same for row sets only (column sets after the large
    // layers), 256 with the LDS-DMA half at the top of the set; default after the
    // large layers.  MODE 512: Q0 read non-temporal by both its readers (A/B).
    // MODE 1024: after the byte->plane transposes; 2048: after the small IFFT layers
    // (both before the first exchange).  MODE 4096: Q1 read with the default policy.
    constexpr bool ADDTID = (MODE & 8) != 0, ARITH = !(MODE & 2), EARLY = (MODE & 256) != 0,
                   NTQ0 = (MODE & 512) != 0, NTQ1 = !(MODE & 4096);
    // diagnostics (wrong output by design): 32768 no LDS exchange, 65536 no byte<->plane
    // transposes, 131072 no butterflies
    constexpr bool XCH = !(MODE & 32768), TRP = ARITH && !(MODE & 65536), BFL = ARITH && !(MODE & 131072);
    // MODE 8192 (with 2048): row sets after the small IFFT layers, column sets right
    // after the first exchange; 16384 (with 2048): the other way round (A/B)
    constexpr int DPOS = (MODE & 8192) ? 6 : (MODE & 16384) ? 7 : EARLY ? 0 : (MODE & 1024) ? 4 : (MODE & 2048) ? 5
                       : (MODE & 64) ? 1 : (MODE & 128) ? 3 : 2;
    const bool MEM = !(MODE & 4) || p.rows.S == 1;  // runtime-false in mode 4 (keeps the code alive)
    const uint32_t lane = threadIdx.x & 63u;
    const bool t0 = threadIdx.x == 0;
    const uint32_t dread = lds_base + kXchBytes + A * 16384u + lane * 16u;
    const uint32_t s_small = __builtin_amdgcn_readfirstlane(lds_base + 4096u * A);
    const uint32_t s_large = __builtin_amdgcn_readfirstlane(lds_base + 256u * A);
    const uint32_t e_small = s_small + lane * 4u, e_large = s_large + lane * 4u;
    uint32_t X[16][8];
    uint32_t P[16 - kPre][8];
    QClaim qc;

    auto addr = [&](uint32_t row, uint32_t set) { return set_addr(row ? p.rows : p.cols, set, lane); };
    // row sets and Q0-col sets read Q0 with the default policy (the other kind
    // re-reads it from the Infinity Cache); Q1-col sets are the last readers of Q1
    auto issue_dma = [&](uint32_t row, uint32_t q1, const SetAddr& a) {
        if (!MEM) return;
        if (row) issue_dma_rt<NTQ0>(p.rows, a, lds_base, A);
        else if (q1) issue_dma_rt<NTQ1>(p.cols, a, lds_base, A);
        else issue_dma_rt<NTQ0>(p.cols, a, lds_base, A);
    };
    auto issue_direct = [&](uint32_t row, uint32_t q1, const SetAddr& a) {
        if (!MEM) return;
        if (row) issue_direct_rt<NTQ0>(p.rows, a, A, P);
        else if (q1) issue_direct_rt<NTQ1>(p.cols, a, A, P);
        else issue_direct_rt<NTQ0>(p.cols, a, A, P);
    };

    // prologue: the first two items, taken synchronously; the first one loaded
    if (t0) {
        uint32_t sq0 = 0, sq1 = 0, r0 = 1, r1 = 1;
        const uint32_t c0 = q_take(p, qc, true, sq0, r0, gridDim.x);
        const uint32_t c1 = c0 == kNone ? kNone : q_take(p, qc, false, sq1, r1, gridDim.x);
        lds[0] = c0;
        lds[1] = sq0;
        lds[4] = c1;
        lds[5] = sq1;
        lds[6] = r1;
        qc.rc = q_load(&p.ctr[kQReady]);
        qc.qh = q_load(&p.ctr[kQHead1]);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    uint32_t cur = __builtin_amdgcn_readfirstlane(lds[0]);
    const uint32_t csq = __builtin_amdgcn_readfirstlane(lds[1]);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    uint32_t pend = kNone;  // square of a stored-but-unsignalled row set
    if (cur != kNone) {
        uint32_t crow, cset;
        q_item(p, cur, csq, crow, cset);
        {
            const SetAddr a = addr(crow, cset);
            issue_dma(crow, cur & kQ1, a);
            issue_direct(crow, cur & kQ1, a);
        }
        if (t0) {
            lds[0] = lds[4];
            lds[1] = lds[5];
            lds[2] = lds[6];
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        // thread 0, carried across the loop: the pending claim, the next-next item
        // (nn, its square, state 0 ready / 1 readiness load rv pending), the pending
        // row-counter add of a signalled row set
        uint32_t cand = kNone, nn = kNone, nnsq = 0, nst = 0, rv = 0, sig = 0, sig_sq = kNone;
        for (;;) {
            {
                v4u g[8];
                bs8::sfor<2>([&](auto Hh) {
                    constexpr int hh = decltype(Hh)::value;
                    ds_r16x8<8192 * hh, 1024>(dread, g);
                    bs8::sfor<4>([&](auto J) {
                        constexpr int j = 4 * hh + decltype(J)::value;
                        const v4u x = g[2 * (j & 3)], y = g[2 * (j & 3) + 1];
                        X[j][0] = x.x; X[j][1] = x.y; X[j][2] = x.z; X[j][3] = x.w;
                        X[j][4] = y.x; X[j][5] = y.y; X[j][6] = y.z; X[j][7] = y.w;
                    });
                });
            }
            bs8::sfor<16 - kPre>([&](auto J) {
                constexpr int j = decltype(J)::value;
                bs8::sfor<8>([&](auto I) { X[kPre + j][decltype(I)::value] = P[j][decltype(I)::value]; });
            });
            // the slot (E words 0..2) holds the next item; everyone reads it before the
            // first exchange overwrites E
            const uint32_t nxt = __builtin_amdgcn_readfirstlane(lds[0]);
            uint32_t nsq = __builtin_amdgcn_readfirstlane(lds[1]);
            const uint32_t rdy = __builtin_amdgcn_readfirstlane(lds[2]);
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            const bool more = nxt != kNone;
            const bool pre = more && rdy;
            uint32_t nrow = 0, nset = 0;
            SetAddr an{};
            if (pre) {
                q_item(p, nxt, nsq, nrow, nset);
                an = addr(nrow, nset);
                issue_dma(nrow, nxt & kQ1, an);
                if constexpr (DPOS == 0) issue_direct(nrow, nxt & kQ1, an);
            }
            // direct loads issued since the previous set's stores, at the publish point
            const bool dearly = pre && (DPOS <= 1 || DPOS >= 4 || (DPOS == 3 && nrow));  // all issued by the publish point
            // no claim in a workgroup's last set (nothing would take the item)
            if (t0) cand = more ? q_claim(p, qc) : kNone;

            if constexpr (TRP) bs8::sfor<16>([&](auto J) { bs8::transpose8_dev(X[decltype(J)::value]); });
            if constexpr (DPOS == 4)
                if (pre) issue_direct(nrow, nxt & kQ1, an);
            if constexpr (BFL) bs8::small_ifft_all(X, A);
            if constexpr (DPOS == 5)
                if (pre) issue_direct(nrow, nxt & kQ1, an);
            if constexpr (DPOS == 6 || DPOS == 7)
                if (pre && ((DPOS == 6) == (nrow != 0))) issue_direct(nrow, nxt & kQ1, an);
            if constexpr (XCH) bs8::sfor<8>([&](auto Pp) { xch_to_large<decltype(Pp)::value, ADDTID>(X, e_small, s_small, e_large); });
            if constexpr (DPOS == 1 || DPOS == 3)
                if (pre && (DPOS == 1 || nrow)) issue_direct(nrow, nxt & kQ1, an);
            if constexpr (DPOS == 6 || DPOS == 7)
                if (pre && ((DPOS == 6) != (nrow != 0))) issue_direct(nrow, nxt & kQ1, an);
            if constexpr (BFL) bs8::large_ifft_fft(X);

            // publish the row set stored at the end of the previous set (its stores
            // were issued before this set's loads: wait for them only); the counter
            // add's result is consumed after the small layers
            if (pend != kNone) {
                // ops issued since those stores: this set's LDS-DMA loads (16) and, with
                // LATE, its direct loads (16)
                if (dearly) asm volatile("s_waitcnt vmcnt(32)\n\ts_barrier" ::: "memory");
                else if (pre) asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
                if (t0) {
                    sig = q_add(&p.ctr[kQRows + pend]);
                    sig_sq = pend;
                }
                pend = kNone;
            }
            // the claim (issued at the top of the set) becomes the next-next item; a Q1
            // item's readiness is loaded now and read after the small layers
            asm volatile("" : "+v"(cand));
            if (t0) {
                nnsq = 0u;
                nst = 0u;
                uint32_t it = cand;
                if (it != kNone && it != kQExitCheck && !(it & kQ1) && it >= p.nmain) {
                    qc.main_done = 1u;
                    it = qc.res != kNone ? qc.res : kQExitCheck;
                }
                if (it == kQExitCheck) it = q_leave_or_claim(p, gridDim.x);
                if (it == kNone || ((it & kQ1) && (it & ~kQ1) >= p.nq1)) {
                    nn = kNone;
                } else {
                    nn = it;
                    if (it & kQ1) {
                        nst = 1u;
                        rv = q_load(&p.ctr[kQRows + p.count + (it & ~kQ1) / p.rn]);
                    }
                }
                qc.rc = q_load(&p.ctr[kQReady]);
                qc.qh = q_load(&p.ctr[kQHead1]);
            }
            if (pre && (DPOS == 2 || (DPOS == 3 && !nrow))) issue_direct(nrow, nxt & kQ1, an);
            if constexpr (XCH) bs8::sfor<8>([&](auto Pp) { xch_to_small<decltype(Pp)::value, ADDTID>(X, e_large, s_large, e_small); });
            if constexpr (BFL) bs8::small_fft_all(X, A);
            if (t0) {
                asm volatile("" : "+v"(sig), "+v"(rv));
                if (sig_sq != kNone) {
                    if (sig == p.rn - 1u) q_publish(p, sig_sq);
                    sig_sq = kNone;
                }
                uint32_t r = 1u;
                if (nst == 1u) {
                    if (rv != 0u) {
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                        nnsq = rv - 1u;
                        if (nn == qc.res) qc.res = kNone;
                    } else {
                        // not published yet: keep it in reserve and take a main item
                        qc.res = nn;
                        uint32_t u = p.nmain;
                        if (!qc.main_done) u = q_add(&p.ctr[kQMain]);
                        if (u < p.nmain) {
                            nn = u;
                        } else {
                            qc.main_done = 1u;
                            qc.res = kNone;
                            r = 0u;  // main sequence exhausted: the slow path waits for it
                        }
                    }
                }
                lds[0] = nn;
                lds[1] = nnsq;
                lds[2] = r;
            }
            {
                const SetAddr a = addr(crow, cset);
                const __amdgpu_buffer_rsrc_t ro = as_rsrc(a.ro);
                const uint32_t k = p.rows.k;
                const uint32_t oo = (uint32_t)(crow ? p.rows.out_offset : p.cols.out_offset);
                const uint32_t es = (uint32_t)(crow ? p.rows.elem_stride : p.cols.elem_stride);
                // Q1 write-through (sc1: another workgroup reads it soon); Q2/Q3 non-temporal
                const bool rs = crow != 0;
                bs8::sfor<16>([&](auto J) {
                    constexpr int j = decltype(J)::value;
                    if constexpr (TRP) bs8::transpose8_dev(X[j]);
                    const uint32_t so = sym_off(16u * A + j, k, oo, es);
                    v4u x, y;
                    x.x = X[j][0]; x.y = X[j][1]; x.z = X[j][2]; x.w = X[j][3];
                    y.x = X[j][4]; y.y = X[j][5]; y.z = X[j][6]; y.w = X[j][7];
                    if (!MEM) {
                    } else if (rs) {
                        __builtin_amdgcn_raw_buffer_store_b128(x, ro, a.off[0], so, 16);
                        __builtin_amdgcn_raw_buffer_store_b128(y, ro, a.off[1], so, 16);
                    } else {
                        __builtin_amdgcn_raw_buffer_store_b128(x, ro, a.off[0], so, 2);
                        __builtin_amdgcn_raw_buffer_store_b128(y, ro, a.off[1], so, 2);
                    }
                    asm volatile("s_nop 2" ::: "memory");  // store-data hazard, see bs_uni_wave
                });
            }
            if (crow) pend = cset / p.rn;
            if (!more) break;
            if (!pre) {
                // slow path (main sequence exhausted, next Q1 set not ready): publish our
                // own row set first, wait, then load the next set synchronously
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
                if (t0) {
                    if (pend != kNone) q_signal(p, pend);
                    lds[3] = q_wait(p, nxt);
                }
                pend = kNone;
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
                nsq = __builtin_amdgcn_readfirstlane(lds[3]);
                if (nsq == kNone) break;  // stuck wait: skip the set, drain
                q_item(p, nxt, nsq, nrow, nset);
                an = addr(nrow, nset);
                issue_dma(nrow, nxt & kQ1, an);
                issue_direct(nrow, nxt & kQ1, an);
                __builtin_amdgcn_s_waitcnt(0x0F70);
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(32) lgkmcnt(0)\n\ts_barrier" ::: "memory");
            }
            cur = nxt;
            crow = nrow;
            cset = nset;
        }
    }
    // drain: every wave's stores, then the last row set's signal and the exit count;
    // the last workgroup out re-zeroes the queue for the next launch on these words
    // (all its threads: 2 * count words)
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (t0) {
        if (pend != kNone) q_signal(p, pend);
        __builtin_amdgcn_s_waitcnt(0x0F70);
        lds[0] = q_add(&p.ctr[kQExit]) == gridDim.x - 1u ? 1u : 0u;
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (__builtin_amdgcn_readfirstlane(lds[0])) {
        for (uint32_t s = threadIdx.x; s < 2u * p.count; s += blockDim.x) q_store(&p.ctr[kQRows + s], 0u);
        if (t0) {
            if (q_load(&p.ctr[kQErr])) {
                __hip_atomic_store(p.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                q_store(&p.ctr[kQErr], 0u);
            }
            q_store(&p.ctr[kQMain], 0u);
            q_store(&p.ctr[kQHead1], 0u);
            q_store(&p.ctr[kQReady], 0u);
            q_store(&p.ctr[kQRes], 0u);
            q_store(&p.ctr[kQLeft], 0u);
            q_store(&p.ctr[kQExit], 0u);
        }
    }
}

// ---------------------------------------------------------------------------
// Half-split schedule (production since round 3): the same queue, hand-off and
// per-set arithmetic as bs_queue_wave, with the set's 128 symbols split by bit 6
// into two halves that are independent in every layer but the merged middle pair
// (bs8.hpp, "Half-split schedule").  Each LDS exchange moves one half while the
// VALU works on the other, so the exchange (a quarter of the set's time when the
// waves wait for it: profiles/r03_qab.jsonl) overlaps arithmetic.  Production form
// (MODE 0, direct loads only -- "XLOAD"; the LDS-DMA form is diagnostic bit 1048576):
//   top   X[h1] <- P (direct loads of this set's h1, issued at the previous top);
//         direct loads of the NEXT set's h1 -> P; transposes + small IFFT h0
//         (X[h0] was loaded right after the previous set's h0 stores)
//   write h0 -> R            || transposes + small IFFT h1
//   read  h0 (layout L)      ;  write h1 -> R || large IFFT h0
//   read  h1                 ;  large IFFT h1, middle pair, large FFT h0
//   write h0 -> R            || large FFT h1
//   read  h0 (layout S')     ;  write h1 -> R || small FFT h0, planes -> bytes, stores h0,
//                               then direct loads of the NEXT set's h0 into X[h0]
//   read  h1                 ;  small FFT h1, planes -> bytes, stores h1
// LDS: R = [0, 128 KiB) (one half's exchange; in the DMA form also the landing zone
// of the next set's h1); the queue slot words at 128 KiB.  Loads of symbol e of the
// set: h0 registers j < 8 hold e = j + 8A, h1 registers e = (j - 8) + 8A + 64.
// Same-box A/B (profiles/r03_qab.jsonl): direct-load form 8.47 us per square against
// 8.67-8.72 for the LDS-DMA form.
constexpr uint32_t kRBytes = 128u * 1024u;
constexpr uint32_t kSlotW = kRBytes / 4;

__device__ __forceinline__ uint32_t e_split(uint32_t A, int j) {
    return (uint32_t)(j & 7) + 8u * A + 64u * (uint32_t)(j >> 3);
}

// h1 (registers 8..15) of a set by LDS-DMA into wave A's 16 KiB of R
template <bool NT>
__device__ __forceinline__ void split_dma_h1(const CodewordSet& cs, const SetAddr& a, uint32_t lds_base, uint32_t A) {
    const uint32_t k = cs.k, es = (uint32_t)cs.elem_stride;
    bs8::sfor<8>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t so = sym_off(e_split(A, 8 + j), k, 0, es);
        const uint32_t l = __builtin_amdgcn_readfirstlane(lds_base + A * 16384u + j * 2048u);
        dma16<NT>(l, a.off[0], a.rs, so);
        dma16<NT>(l + 1024u, a.off[1], a.rs, so);
    });
}
// half G (registers 8G..8G+7) of a set into P (direct loads)
// The per-symbol offsets are loop-invariant, and hoisted out of the set loop they
// outgrow the SGPR file: the compiler then parks them in VGPR lanes and reloads each
// with a v_readlane (a VALU instruction) per use -- ~80 per set and wave.  Passing k,
// the element stride and the wave index through an empty asm makes them opaque per
// use, so each offset is recomputed right before its load / store by 2-3 scalar ALU
// instructions, which issue beside the VALU work.
__device__ __forceinline__ void opaque_sgpr(uint32_t& k, uint32_t& es, uint32_t& A) {
    asm volatile("" : "+s"(k), "+s"(es), "+s"(A));
}
template <bool NT, int G = 0, bool OPQ = true>
__device__ __forceinline__ void split_direct_h0(const CodewordSet& cs, const SetAddr& a, uint32_t A,
                                                uint32_t (&P)[8][8]) {
    uint32_t k = cs.k, es = (uint32_t)cs.elem_stride;
    if constexpr (OPQ) opaque_sgpr(k, es, A);
    const __amdgpu_buffer_rsrc_t rs = as_rsrc(a.rs);
    bs8::sfor<8>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t so = sym_off(e_split(A, 8 * G + j), k, 0, es);
        const v4u x = __builtin_amdgcn_raw_buffer_load_b128(rs, a.off[0], so, NT ? 2 : 0);
        const v4u y = __builtin_amdgcn_raw_buffer_load_b128(rs, a.off[1], so, NT ? 2 : 0);
        P[j][0] = x.x; P[j][1] = x.y; P[j][2] = x.z; P[j][3] = x.w;
        P[j][4] = y.x; P[j][5] = y.y; P[j][6] = y.z; P[j][7] = y.w;
    });
}
// planes -> bytes and the 16 stores of half G (Q1 write-through, Q2/Q3 non-temporal)
template <int G, bool TRP, bool MEM_ON, bool OLDTP = false, bool PLAINQ1 = false, bool OPQ = true>
__device__ __forceinline__ void split_store_h(uint32_t (&X)[16][8], const SetAddr& a, uint32_t A, uint32_t k,
                                              uint32_t oo, uint32_t es, bool row, bool mem) {
    const __amdgpu_buffer_rsrc_t ro = as_rsrc(a.ro);
    if constexpr (OPQ) {
        opaque_sgpr(k, es, A);
        opaque_sgpr(oo, es, A);
    }
    bs8::sfor<8>([&](auto J) {
        constexpr int j = 8 * G + decltype(J)::value;
        if constexpr (TRP && OLDTP) bs8::transpose8_dev(X[j]);
        else if constexpr (TRP) bs8::tp_inv_dev(X[j]);  // planes (layout of gen_bs8_small tp_ops) -> bytes
        const uint32_t so = sym_off(e_split(A, j), k, oo, es);
        v4u x, y;
        x.x = X[j][0]; x.y = X[j][1]; x.z = X[j][2]; x.w = X[j][3];
        y.x = X[j][4]; y.y = X[j][5]; y.z = X[j][6]; y.w = X[j][7];
        if (!MEM_ON || !mem) {
        } else if (row) {
            __builtin_amdgcn_raw_buffer_store_b128(x, ro, a.off[0], so, PLAINQ1 ? 0 : 16);
            __builtin_amdgcn_raw_buffer_store_b128(y, ro, a.off[1], so, PLAINQ1 ? 0 : 16);
        } else {
            __builtin_amdgcn_raw_buffer_store_b128(x, ro, a.off[0], so, 2);
            __builtin_amdgcn_raw_buffer_store_b128(y, ro, a.off[1], so, 2);
        }
        asm volatile("s_nop 2" ::: "memory");  // store-data hazard, see bs_uni_wave
    });
}
// keep half G's registers allocated until the LDS writes that read them are done
template <int G>
__device__ __forceinline__ void keep_half(uint32_t (&X)[16][8]) {
#pragma unroll
    for (int v = 0; v < 8; ++v)
        asm volatile("" : : "v"(X[8 * G + v][0]), "v"(X[8 * G + v][1]), "v"(X[8 * G + v][2]), "v"(X[8 * G + v][3]),
                     "v"(X[8 * G + v][4]), "v"(X[8 * G + v][5]), "v"(X[8 * G + v][6]), "v"(X[8 * G + v][7]));
}
#define RSM_LDS_SYNC asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")
// diagnostic phase timeline (TRACE): thread 0 records the 100 MHz real-time clock at
// phase boundaries, one row of kTraceWords per (workgroup, set); vector stores only
__device__ __forceinline__ void trace_stamp(const QueuePlan& p, uint32_t it, int w, uint32_t v) {
#ifdef RSM_DIAG
    if (p.trace && it < kTraceSets) {
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(p.trace, (short)0, 0x7FFFFFFF, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32(v, r, ((blockIdx.x * kTraceSets + it) * kTraceWords + w) * 4u, 0, 0);
    }
#endif
}

// XCD-affine queues (diagnostic, MODE bit 33554432): the workgroup reads the XCD it
// runs on (HW_REG_XCC_ID) and serves only the squares s = 8 j + x of that XCD from
// that XCD's own queue words, so a square's Q0 re-read and its Q1 hand-off stay in
// one XCD's L2: Q1 is stored with the default policy (not write-through), and the
// consumer's agent acquire (L1 invalidate) suffices because producer and consumer
// share the L2.  Correct for any placement (each workgroup picks the queue of the XCD
// it actually runs on); complete only when every XCD gets gridDim.x / 8 workgroups
// (the round-robin placement, MI355X_MICROARCH.md) -- the diagnostic checks every
// square.  The host zeroes all queue words before each such launch.
__device__ __forceinline__ QueuePlan xcd_plan(const QueuePlan& p0, uint32_t x) {
    QueuePlan p = p0;
    p.count = p0.count / 8u;
    p.nmain = p0.nmain / 8u;
    p.nq1 = p0.nq1 / 8u;
    for (CodewordSet* cs : {&p.rows, &p.cols}) {
        cs->base += (uint64_t)x * cs->square_stride;
        cs->out_base += (uint64_t)x * cs->square_stride;
        cs->square_stride *= 8u;
        cs->count /= 8u;
    }
    p.ctr = p0.ctr + x * (kQueueFixedWords + 2u * p.count);
    return p;
}

template <int MODE>
__device__ __forceinline__ void bs_split_wave(const QueuePlan& p_in, uint32_t* lds, uint32_t lds_base, uint32_t A) {
    constexpr bool XCDQ = (MODE & 33554432) != 0;
    // 67108864: the per-symbol offsets hoisted by the compiler (round-3 codegen: ~80
    // v_readlane SGPR reloads per set) -- A/B against the opaque per-use form
    constexpr bool OPQ = (MODE & 67108864) == 0;
    // 134217728: static priority 1 for waves 4-7 (the second-dispatched half, the
    // arbitration loser; MI355X_MICROARCH.md "Two waves per SIMD" item 4) -- A/B
    if constexpr ((MODE & 134217728) != 0)
        if (A >= 4u) __builtin_amdgcn_s_setprio(1);
    uint32_t xcc = 0;
    if constexpr (XCDQ) asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const QueuePlan p = XCDQ ? xcd_plan(p_in, xcc & 7u) : p_in;
    const uint32_t G = XCDQ ? gridDim.x / 8u : gridDim.x;  // workgroups serving this queue
    // diagnostics (wrong output by design): 2 no arithmetic, 4 no global memory,
    // 32768 no LDS exchange
    constexpr bool ARITH = !(MODE & 2), XCH = !(MODE & 32768), NTQ0 = false, NTQ1 = true;
    // A/B: 65536 = h0's small FFT and stores after the next set's LDS-DMA issue (a
    // longer DMA lead, the last exchange write not overlapped)
    constexpr bool LATE0 = (MODE & 65536) != 0;
    // 131072: the exchange writes issued as separate blocks (A/B against the
    // production form, which interleaves them with the other half's VALU work)
    constexpr bool IL = ARITH && XCH && !LATE0 && !(MODE & 131072);
    // 262144: no LDS-DMA -- h1 of the next set by direct loads into Q right after this
    // set's h0 stores (the LDS region R then holds only exchanges)
    constexpr bool NODMA = (MODE & 262144) != 0 && !LATE0;
    // production: no LDS-DMA -- P holds h1 of the next set (loaded at the top), h0 of
    // the next set is loaded into X[0..7] right after this set's h0 stores;
    // 1048576: the LDS-DMA form (h1 of the next set lands in R, A/B)
    constexpr bool XLOAD = (MODE & 1048576) == 0 && !NODMA && !LATE0;
    // 524288: phase timeline into p.trace (diagnostic build)
    constexpr bool TRACE = (MODE & 524288) != 0;
    // 4194304: an explicit agent-scope release (buffer_wbl2 sc1 + vmcnt(0)) by the
    // signalling lane before each row set's counter add -- measures what the release
    // would cost on top of the write-through (sc1) Q1 stores the hand-off relies on
    constexpr bool REL = (MODE & 4194304) != 0;
    // 8388608: the round-3 shift-pair transposes (bs8.hpp transpose8_dev) instead of the
    // rotate-and-select network (gen_bs8_small.cpp tp_ops) -- A/B
    constexpr bool OLDTP = (MODE & 8388608) != 0;
    auto tp_fwd = [](uint32_t (&w)[8]) {
        if constexpr (OLDTP) bs8::transpose8_dev(w);
        else bs8::tp_fwd_dev(w);
    };
    auto release = [&]() {
        if constexpr (REL) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    };
    uint32_t it_no = 0;
    auto stamp = [&](int w) {
        if constexpr (TRACE)
            if (threadIdx.x == 0) trace_stamp(p, it_no, w, (uint32_t)__builtin_amdgcn_s_memrealtime());
    };
    const bool MEM = !(MODE & 4) || p.rows.S == 1;  // runtime-false in mode 4 (keeps the code alive)
    const uint32_t lane = threadIdx.x & 63u;
    const bool t0 = threadIdx.x == 0;
    const uint32_t dread = lds_base + A * 16384u + lane * 16u;
    // exchange entries (gen_bs8_small.cpp emit_xch): writer wave A at lane * 8 + A * 512,
    // reader wave A at lane * 8 + A * 4096
    const uint32_t xw = lds_base + lane * 8u + A * 512u, xr = lds_base + lane * 8u + A * 4096u;
    uint32_t* slot = lds + kSlotW;
    uint32_t X[16][8];
    uint32_t P[8][8];
    uint32_t Q[8][8];  // NODMA: h1 of the next set
    QClaim qc;

    // 16777216: fixed per-lane set offsets (the host chose it: lane_geo_ok for rows and
    // columns -- S divides the 2 KiB set width, the production c2 shape)
    constexpr bool GEO = (MODE & 16777216) != 0;
    LaneGeo geo_r{}, geo_c{};
    if constexpr (GEO) geo_r = lane_geo(p.rows, lane), geo_c = lane_geo(p.cols, lane);
    auto addr = [&](uint32_t row, uint32_t set) {
        if constexpr (GEO) return row ? set_addr_geo(p.rows, geo_r, set) : set_addr_geo(p.cols, geo_c, set);
        else return set_addr(row ? p.rows : p.cols, set, lane);
    };
    auto issue_dma = [&](uint32_t row, uint32_t q1, const SetAddr& a) {
        if (!MEM) return;
        if constexpr (NODMA) {
            if (row) split_direct_h0<NTQ0, 1, OPQ>(p.rows, a, A, Q);
            else if (q1) split_direct_h0<NTQ1, 1, OPQ>(p.cols, a, A, Q);
            else split_direct_h0<NTQ0, 1, OPQ>(p.cols, a, A, Q);
            return;
        }
        if (row) split_dma_h1<NTQ0>(p.rows, a, lds_base, A);
        else if (q1) split_dma_h1<NTQ1>(p.cols, a, lds_base, A);
        else split_dma_h1<NTQ0>(p.cols, a, lds_base, A);
    };
    auto issue_direct = [&](uint32_t row, uint32_t q1, const SetAddr& a) {
        if (!MEM) return;
        if constexpr (XLOAD) {  // P = h1
            if (row) split_direct_h0<NTQ0, 1, OPQ>(p.rows, a, A, P);
            else if (q1) split_direct_h0<NTQ1, 1, OPQ>(p.cols, a, A, P);
            else split_direct_h0<NTQ0, 1, OPQ>(p.cols, a, A, P);
            return;
        }
        if (row) split_direct_h0<NTQ0, 0, OPQ>(p.rows, a, A, P);
        else if (q1) split_direct_h0<NTQ1, 0, OPQ>(p.cols, a, A, P);
        else split_direct_h0<NTQ0, 0, OPQ>(p.cols, a, A, P);
    };
    // XLOAD: h0 of a set straight into X[0..7]
    auto issue_x0 = [&](uint32_t row, uint32_t q1, const SetAddr& a) {
        uint32_t (&X0)[8][8] = *reinterpret_cast<uint32_t (*)[8][8]>(&X[0][0]);
        if (!MEM) return;
        if (row) split_direct_h0<NTQ0, 0, OPQ>(p.rows, a, A, X0);
        else if (q1) split_direct_h0<NTQ1, 0, OPQ>(p.cols, a, A, X0);
        else split_direct_h0<NTQ0, 0, OPQ>(p.cols, a, A, X0);
    };

    // prologue: the first two items, taken synchronously; the first one loaded
    if (t0) {
        uint32_t sq0 = 0, sq1 = 0, r0 = 1, r1 = 1;
        const uint32_t c0 = q_take(p, qc, true, sq0, r0, G);
        const uint32_t c1 = c0 == kNone ? kNone : q_take(p, qc, false, sq1, r1, G);
        slot[0] = c0;
        slot[1] = sq0;
        slot[4] = c1;
        slot[5] = sq1;
        slot[6] = r1;
        qc.rc = q_load(&p.ctr[kQReady]);
        qc.qh = q_load(&p.ctr[kQHead1]);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    uint32_t cur = __builtin_amdgcn_readfirstlane(slot[0]);
    const uint32_t csq = __builtin_amdgcn_readfirstlane(slot[1]);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    uint32_t pend = kNone;  // square of a stored-but-unsignalled row set
    if (cur != kNone) {
        uint32_t crow, cset;
        q_item(p, cur, csq, crow, cset);
        {
            const SetAddr a = addr(crow, cset);
            if constexpr (XLOAD) issue_x0(crow, cur & kQ1, a);
            else issue_dma(crow, cur & kQ1, a);
            issue_direct(crow, cur & kQ1, a);
        }
        if (t0) {
            slot[0] = slot[4];
            slot[1] = slot[5];
            slot[2] = slot[6];
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        // thread 0, carried across the loop (as bs_queue_wave)
        uint32_t cand = kNone, nn = kNone, nnsq = 0, nst = 0, rv = 0, sig = 0, sig_sq = kNone;
        for (;;) {
            stamp(0);
            // ---- top: h0 from P (XLOAD: h1 from P, h0 already in X); the next item;
            // its P loads ----
            bs8::sfor<8>([&](auto J) {
                constexpr int j = decltype(J)::value;
                bs8::sfor<8>([&](auto I) { X[(XLOAD ? 8 : 0) + j][decltype(I)::value] = P[j][decltype(I)::value]; });
            });
            const uint32_t nxt = __builtin_amdgcn_readfirstlane(slot[0]);
            uint32_t nsq = __builtin_amdgcn_readfirstlane(slot[1]);
            const uint32_t rdy = __builtin_amdgcn_readfirstlane(slot[2]);
            const bool more = nxt != kNone;
            const bool pre = more && rdy;
            uint32_t nrow = 0, nset = 0;
            SetAddr an{};
            if (pre) {
                q_item(p, nxt, nsq, nrow, nset);
                an = addr(nrow, nset);
                issue_direct(nrow, nxt & kQ1, an);
            }
            // no claim in a workgroup's last set (nothing would take the item)
            if (t0) cand = more ? q_claim(p, qc) : kNone;
            if constexpr (ARITH) {
                bs8::sfor<8>([&](auto J) { tp_fwd(X[decltype(J)::value]); });
                bs8::small_ifft_h0_all(X, A);
            }
            if constexpr (XLOAD) {
            } else if constexpr (NODMA) {
                bs8::sfor<8>([&](auto J) {
                    constexpr int j = decltype(J)::value;
                    bs8::sfor<8>([&](auto I) { X[8 + j][decltype(I)::value] = Q[j][decltype(I)::value]; });
                });
            } else {
            // ---- h1 from the LDS-DMA landing zone (issued at the end of the last set) ----
            // ops issued after it: the previous set's h1 stores (16; LATE0: and its h0
            // stores, 16) and, if pre, this set's direct loads (16)
            if constexpr (LATE0) {
                if (pre) asm volatile("s_waitcnt vmcnt(48)\n\ts_barrier" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(32)\n\ts_barrier" ::: "memory");
            } else {
                if (pre) asm volatile("s_waitcnt vmcnt(32)\n\ts_barrier" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
            }
            {
                v4u g[8];
                bs8::sfor<2>([&](auto Hh) {
                    constexpr int hh = decltype(Hh)::value;
                    ds_r16x8<8192 * hh, 1024>(dread, g);
                    bs8::sfor<4>([&](auto J) {
                        constexpr int j = 8 + 4 * hh + decltype(J)::value;
                        const v4u x = g[2 * (j & 3)], y = g[2 * (j & 3) + 1];
                        X[j][0] = x.x; X[j][1] = x.y; X[j][2] = x.z; X[j][3] = x.w;
                        X[j][4] = y.x; X[j][5] = y.y; X[j][6] = y.z; X[j][7] = y.w;
                    });
                });
            }
            asm volatile("s_barrier" ::: "memory");  // every wave has read R
            }
            stamp(1);
            // ---- S' -> L, half 0 || small layers of h1 ----
            if constexpr (IL) {
#ifdef RSM_DIAG
                if constexpr (OLDTP) bs8::ph_w0_tr1_old(X, xw, xw + 65536u);
                else
#endif
                bs8::ph_w0_tr1(X, xw, xw + 65536u);
                bs8::small_ifft_h1_all(X, A);
            } else {
                if constexpr (XCH) bs8::xch_write_h0(X, xw, xw + 65536u);
                if constexpr (ARITH) {
                    bs8::sfor<8>([&](auto J) { tp_fwd(X[8 + decltype(J)::value]); });
                    bs8::small_ifft_h1_all(X, A);
                }
            }
            stamp(2);
            RSM_LDS_SYNC;
            stamp(3);
            keep_half<0>(X);
            if constexpr (XCH) bs8::xch_read_h0(X, xr, xr + 65536u);
            asm volatile("s_barrier" ::: "memory");
            stamp(4);
            // ---- S' -> L, half 1 || large IFFT of h0 ----
            if constexpr (IL) {
                bs8::ph_w1_lifft0(X, xw, xw + 65536u);
            } else {
                if constexpr (XCH) bs8::xch_write_h1(X, xw, xw + 65536u);
                if constexpr (ARITH) bs8::large_ifft_h<0>(X);
            }
            RSM_LDS_SYNC;
            keep_half<1>(X);
            if constexpr (XCH) bs8::xch_read_h1(X, xr, xr + 65536u);
            asm volatile("s_barrier" ::: "memory");
            stamp(5);
            if constexpr (TRACE) if (threadIdx.x == 0) trace_stamp(p, it_no, 12, (uint32_t)__builtin_amdgcn_s_memtime());
            // large IFFT h1, middle pair, large FFT h0: one block (gen_bs8_small.cpp emit_lmid)
            if constexpr (ARITH) bs8::lmid_all(X);
            if constexpr (TRACE) if (threadIdx.x == 0) trace_stamp(p, it_no, 13, (uint32_t)__builtin_amdgcn_s_memtime());
            stamp(6);
            // publish the row set stored at the end of the previous set: ops issued
            // since its last stores = this set's direct loads (16, if pre)
            if (pend != kNone) {
                if (pre) asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
                if (t0) {
                    release();
                    sig = q_add(&p.ctr[kQRows + pend]);
                    sig_sq = pend;
                }
                pend = kNone;
            }
            // the claim (issued at the top of the set) becomes the next-next item; a Q1
            // item's readiness is loaded now and read after the next exchange
            asm volatile("" : "+v"(cand));
            if (t0) {
                nnsq = 0u;
                nst = 0u;
                uint32_t it = cand;
                if (it != kNone && it != kQExitCheck && !(it & kQ1) && it >= p.nmain) {
                    qc.main_done = 1u;
                    it = qc.res != kNone ? qc.res : kQExitCheck;
                }
                if (it == kQExitCheck) it = q_leave_or_claim(p, G);
                if (it == kNone || ((it & kQ1) && (it & ~kQ1) >= p.nq1)) {
                    nn = kNone;
                } else {
                    nn = it;
                    if (it & kQ1) {
                        nst = 1u;
                        rv = q_load(&p.ctr[kQRows + p.count + (it & ~kQ1) / p.rn]);
                    }
                }
                qc.rc = q_load(&p.ctr[kQReady]);
                qc.qh = q_load(&p.ctr[kQHead1]);
            }
            stamp(7);
            // ---- L -> S', half 0 || large FFT of h1 ----
            if constexpr (IL) {
                bs8::ph_w0_lfft1(X, xw, xw + 65536u);
            } else {
                if constexpr (XCH) bs8::xch_write_h0(X, xw, xw + 65536u);
                if constexpr (ARITH) bs8::large_fft_h<1>(X);
            }
            if (t0) {
                asm volatile("" : "+v"(sig), "+v"(rv));
                if (sig_sq != kNone) {
                    if (sig == p.rn - 1u) q_publish(p, sig_sq);
                    sig_sq = kNone;
                }
                uint32_t r = 1u;
                if (nst == 1u) {
                    if (rv != 0u) {
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                        nnsq = rv - 1u;
                        if (nn == qc.res) qc.res = kNone;
                    } else {
                        // not published yet: keep it in reserve and take a main item
                        qc.res = nn;
                        uint32_t u = p.nmain;
                        if (!qc.main_done) u = q_add(&p.ctr[kQMain]);
                        if (u < p.nmain) {
                            nn = u;
                        } else {
                            qc.main_done = 1u;
                            qc.res = kNone;
                            r = 0u;  // main sequence exhausted: the slow path waits for it
                        }
                    }
                }
                slot[0] = nn;
                slot[1] = nnsq;
                slot[2] = r;
            }
            RSM_LDS_SYNC;
            keep_half<0>(X);
            if constexpr (XCH) bs8::xch_read_h0(X, xr, xr + 65536u);
            asm volatile("s_barrier" ::: "memory");
            stamp(8);
            // ---- L -> S', half 1 || small FFT, bytes and stores of h0 ----
            const SetAddr a = addr(crow, cset);
            const uint32_t k = p.rows.k;
            const uint32_t oo = (uint32_t)(crow ? p.rows.out_offset : p.cols.out_offset);
            const uint32_t es = (uint32_t)(crow ? p.rows.elem_stride : p.cols.elem_stride);
            if constexpr (IL) {
                bs8::small_fft_h0_all(X, A);
#ifdef RSM_DIAG
                if constexpr (OLDTP) bs8::ph_w1_tr0_old(X, xw, xw + 65536u);
                else
#endif
                bs8::ph_w1_tr0(X, xw, xw + 65536u);  // + planes -> bytes of h0
                split_store_h<0, false, true, false, XCDQ, OPQ>(X, a, A, k, oo, es, crow != 0, MEM);
                if constexpr (XLOAD) {
                    if (pre) {
                        issue_x0(nrow, nxt & kQ1, an);
                    } else {
                        bs8::sfor<8>([&](auto J) { bs8::sfor<8>([&](auto I) { X[decltype(J)::value][decltype(I)::value] = 0u; }); });
                    }
                }
            } else {
                if constexpr (XCH) bs8::xch_write_h1(X, xw, xw + 65536u);
                if constexpr (!LATE0) {
                    if constexpr (ARITH) bs8::small_fft_h0_all(X, A);
                    split_store_h<0, ARITH, true, OLDTP, XCDQ, OPQ>(X, a, A, k, oo, es, crow != 0, MEM);
                }
            }
            RSM_LDS_SYNC;
            keep_half<1>(X);
            if constexpr (XCH) bs8::xch_read_h1(X, xr, xr + 65536u);
            asm volatile("s_barrier" ::: "memory");  // R free: the next set's h1 may land
            if constexpr (NODMA) {
                if (pre) {
                    issue_dma(nrow, nxt & kQ1, an);  // into Q
                } else {
                    // defined on every path, so the old Q is dead after the top of the set
                    bs8::sfor<8>([&](auto J) { bs8::sfor<8>([&](auto I) { Q[decltype(J)::value][decltype(I)::value] = 0u; }); });
                }
            } else if constexpr (!XLOAD) {
                if (pre) issue_dma(nrow, nxt & kQ1, an);
            }
            if constexpr (LATE0) {
                if constexpr (ARITH) bs8::small_fft_h0_all(X, A);
                split_store_h<0, ARITH, true, OLDTP, XCDQ, OPQ>(X, a, A, k, oo, es, crow != 0, MEM);
            }
            stamp(9);
            if constexpr (ARITH) bs8::small_fft_h1_all(X, A);
            split_store_h<1, ARITH, true, OLDTP, XCDQ, OPQ>(X, a, A, k, oo, es, crow != 0, MEM);
            stamp(10);
            if constexpr (TRACE) if (threadIdx.x == 0) trace_stamp(p, it_no, 11, (crow ? 1u : 0u) | ((cur & kQ1) ? 2u : 0u) | (pre ? 0u : 4u));
            ++it_no;
            if (crow) pend = cset / p.rn;
            if (!more) break;
            if (!pre) {
                // slow path (main sequence exhausted, next Q1 set not ready): publish our
                // own row set first, wait, then load the next set synchronously
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
                if (t0) {
                    if (pend != kNone) {
                        release();
                        q_signal(p, pend);
                    }
                    slot[3] = q_wait(p, nxt);
                }
                pend = kNone;
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
                nsq = __builtin_amdgcn_readfirstlane(slot[3]);
                if (nsq == kNone) break;  // stuck wait: skip the set, drain
                q_item(p, nxt, nsq, nrow, nset);
                an = addr(nrow, nset);
                if constexpr (XLOAD) issue_x0(nrow, nxt & kQ1, an);
                else issue_dma(nrow, nxt & kQ1, an);
                issue_direct(nrow, nxt & kQ1, an);
                __builtin_amdgcn_s_waitcnt(0x0F70);
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
            }
            cur = nxt;
            crow = nrow;
            cset = nset;
        }
    }
    // drain: every wave's stores, then the last row set's signal and the exit count;
    // the last workgroup out re-zeroes the queue for the next launch on these words
    // (all its threads: 2 * count words)
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (t0) {
        if (pend != kNone) {
            release();
            q_signal(p, pend);
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);
        slot[0] = q_add(&p.ctr[kQExit]) == G - 1u ? 1u : 0u;
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (__builtin_amdgcn_readfirstlane(slot[0])) {
        for (uint32_t s = threadIdx.x; s < 2u * p.count; s += blockDim.x) q_store(&p.ctr[kQRows + s], 0u);
        if (t0) {
            if (q_load(&p.ctr[kQErr])) {
                __hip_atomic_store(p.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                q_store(&p.ctr[kQErr], 0u);
            }
            q_store(&p.ctr[kQMain], 0u);
            q_store(&p.ctr[kQHead1], 0u);
            q_store(&p.ctr[kQReady], 0u);
            q_store(&p.ctr[kQRes], 0u);
            q_store(&p.ctr[kQLeft], 0u);
            q_store(&p.ctr[kQExit], 0u);
        }
    }
}
#undef RSM_LDS_SYNC

template <int MODE>
__global__ __launch_bounds__(512, 1) void extend_gf8_bs128s_kernel(QueuePlan p) {
    __shared__ uint32_t lds[(kDmaBytes + kXchBytes) / 4];
    bs_split_wave<MODE>(p, lds, (uint32_t)(uintptr_t)lds, __builtin_amdgcn_readfirstlane(threadIdx.x >> 6));
}

template <int MODE>
__global__ __launch_bounds__(512, 1) void extend_gf8_bs128q_kernel(QueuePlan p) {
    __shared__ uint32_t lds[(kDmaBytes + kXchBytes) / 4];
    bs_queue_wave<MODE>(p, lds, (uint32_t)(uintptr_t)lds, __builtin_amdgcn_readfirstlane(threadIdx.x >> 6));
}

#ifdef RSM_DIAG
// ---------------------------------------------------------------------------
// Dual launch (DualPlan): bs_uni_wave's persistent pipeline over the union of two
// independent set lists.  Set t maps to (list, index); with nb == 2 na every group
// of three consecutive t is one set of a and two of b.  No cross-workgroup hand-off:
// the lists touch disjoint squares (the caller orders a batch's column pass after
// its row pass with the stream).
__device__ __forceinline__ void dual_item(const DualPlan& p, uint32_t t, uint32_t& isb, uint32_t& idx) {
    if (p.nb == 2u * p.na) {
        const uint32_t g = t / 3u, r = t - 3u * g;
        isb = r != 0u;
        idx = r == 0u ? g : 2u * g + (r - 1u);
    } else {
        isb = t >= p.na;
        idx = isb ? t - p.na : t;
    }
}

template <int MODE>
__device__ __forceinline__ void bs_dual_wave(const DualPlan& p, uint32_t lds_base, uint32_t A) {
    constexpr bool ADDTID = (MODE & 8) != 0, NTL = (MODE & 32) != 0;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t G = gridDim.x, sets = p.na + p.nb;
    const uint32_t dread = lds_base + kXchBytes + A * 16384u + lane * 16u;
    const uint32_t s_small = __builtin_amdgcn_readfirstlane(lds_base + 4096u * A);
    const uint32_t s_large = __builtin_amdgcn_readfirstlane(lds_base + 256u * A);
    const uint32_t e_small = s_small + lane * 4u, e_large = s_large + lane * 4u;
    uint32_t X[16][8];
    uint32_t P[16 - kPre][8];

    auto issue = [&](uint32_t isb, const SetAddr& a) {
        if (isb) {
            issue_dma_rt<NTL>(p.b, a, lds_base, A);
            issue_direct_rt<NTL>(p.b, a, A, P);
        } else {
            issue_dma_rt<NTL>(p.a, a, lds_base, A);
            issue_direct_rt<NTL>(p.a, a, A, P);
        }
    };
    auto addr = [&](uint32_t isb, uint32_t idx) { return set_addr(isb ? p.b : p.a, idx, lane); };

    uint32_t t = blockIdx.x;
    uint32_t cb = 0, ci = 0;
    dual_item(p, t, cb, ci);
    issue(cb, addr(cb, ci));
    __builtin_amdgcn_s_waitcnt(0x0F70);
    asm volatile("s_barrier" ::: "memory");
    for (;;) {
        {
            v4u g[8];
            bs8::sfor<2>([&](auto Hh) {
                constexpr int hh = decltype(Hh)::value;
                ds_r16x8<8192 * hh, 1024>(dread, g);
                bs8::sfor<4>([&](auto J) {
                    constexpr int j = 4 * hh + decltype(J)::value;
                    const v4u x = g[2 * (j & 3)], y = g[2 * (j & 3) + 1];
                    X[j][0] = x.x; X[j][1] = x.y; X[j][2] = x.z; X[j][3] = x.w;
                    X[j][4] = y.x; X[j][5] = y.y; X[j][6] = y.z; X[j][7] = y.w;
                });
            });
        }
        bs8::sfor<16 - kPre>([&](auto J) {
            constexpr int j = decltype(J)::value;
            bs8::sfor<8>([&](auto I) { X[kPre + j][decltype(I)::value] = P[j][decltype(I)::value]; });
        });
        const uint32_t tn = t + G;
        const bool more = tn < sets;
        uint32_t nb = 0, ni = 0;
        if (more) {
            dual_item(p, tn, nb, ni);
            issue(nb, addr(nb, ni));
        }
        bs8::sfor<16>([&](auto J) { bs8::transpose8_dev(X[decltype(J)::value]); });
        bs8::small_ifft_all(X, A);
        bs8::sfor<8>([&](auto Pp) { xch_to_large<decltype(Pp)::value, ADDTID>(X, e_small, s_small, e_large); });
        bs8::large_ifft_fft(X);
        bs8::sfor<8>([&](auto Pp) { xch_to_small<decltype(Pp)::value, ADDTID>(X, e_large, s_large, e_small); });
        bs8::small_fft_all(X, A);
        {
            const SetAddr a = addr(cb, ci);
            const __amdgpu_buffer_rsrc_t ro = as_rsrc(a.ro);
            const uint32_t k = p.a.k;
            const uint32_t oo = (uint32_t)(cb ? p.b.out_offset : p.a.out_offset);
            const uint32_t es = (uint32_t)(cb ? p.b.elem_stride : p.a.elem_stride);
            bs8::sfor<16>([&](auto J) {
                constexpr int j = decltype(J)::value;
                bs8::transpose8_dev(X[j]);
                const uint32_t so = sym_off(16u * A + j, k, oo, es);
                v4u x, y;
                x.x = X[j][0]; x.y = X[j][1]; x.z = X[j][2]; x.w = X[j][3];
                y.x = X[j][4]; y.y = X[j][5]; y.z = X[j][6]; y.w = X[j][7];
                __builtin_amdgcn_raw_buffer_store_b128(x, ro, a.off[0], so, 0);
                __builtin_amdgcn_raw_buffer_store_b128(y, ro, a.off[1], so, 0);
                asm volatile("s_nop 2" ::: "memory");  // store-data hazard, see bs_uni_wave
            });
        }
        if (!more) break;
        t = tn;
        cb = nb;
        ci = ni;
        asm volatile("s_waitcnt vmcnt(32)\n\ts_barrier" ::: "memory");
    }
}

template <int MODE>
__global__ __launch_bounds__(512, 1) void encode_gf8_bs128p_kernel(DualPlan p) {
    __shared__ uint32_t lds[(kDmaBytes + kXchBytes) / 4];
    if (blockIdx.x >= p.na + p.nb) return;
    bs_dual_wave<MODE>(p, (uint32_t)(uintptr_t)lds, __builtin_amdgcn_readfirstlane(threadIdx.x >> 6));
}

#endif  // RSM_DIAG

}  // namespace


// True when every offset the kernel forms stays below the buffer-resource limit
// (2^31): the set's codeword span + the largest symbol offset.
bool bs128_applicable(const CodewordSet& cs) {
    if (cs.indices != nullptr || ceil_pow2(cs.k) != 128) return false;
    if ((uint64_t)cs.count * cs.S + kSetBytes >= kOobBs) return false;  // 32-bit set index math
    const uint64_t cws_per_set = kSetBytes / cs.S + 2;
    const uint64_t span = cws_per_set * (cs.cw_stride > cs.square_stride ? cs.cw_stride : cs.square_stride) + cs.S;
    const uint64_t sym = (uint64_t)cs.out_offset + (uint64_t)cs.k * cs.elem_stride;
    return span + sym < kOobBs;
}

// Production launch: row pass MODE 104 (ds_write_addtid_b32 exchange + non-temporal
// loads, the next set's direct loads issued after the first exchange: its Q1 stores
// keep the default policy), column pass MODE 184 (+ non-temporal stores -- Q2/Q3 are
// final output, never re-read -- and the direct loads after the large layers).
// Measured in the two-stream schedule (profiles/r02d_sched_ab.jsonl): NT stores 3-4 %,
// the spread-out load issue another 3-4 % per step.  The column pass walks its
// sets in reverse order (its first reads are the squares the row pass wrote last).
// The persistent grid is the caller's (the context's CU count or per-pass cap).
#ifdef RSM_DIAG
static std::atomic<int> g_diag_mode{40};
static std::atomic<int> g_diag_rev{1};
static std::atomic<int> g_diag_xcd{0};
static std::atomic<int> g_diag_row_mode{40};
void set_bs128_diag_mode(int mode, int rev_col, int xcd) {
    g_diag_mode.store(mode);
    g_diag_rev.store(rev_col);
    g_diag_xcd.store(xcd);
}
void set_bs128_diag_row_mode(int mode) { g_diag_row_mode.store(mode); }
bool bs128_diag_xcd_queues() {
    const int m = g_diag_mode.load();
    return m == 55000 || m == 55002 || m == 55004;
}
#endif

hipError_t launch_encode_gf8_bs128(const CodewordSet& cs, hipStream_t st) {
    const uint64_t sets = ((uint64_t)cs.count * cs.S + kSetBytes - 1) / kSetBytes;
    if (sets == 0) return hipSuccess;
    const uint32_t cap = cs.grid ? cs.grid : 256u;
    const uint32_t grid = (uint32_t)(sets < cap ? sets : cap);
    const bool row = cs.pass == 0;
#define RSM_BS_LAUNCH(m, p) \
    hipLaunchKernelGGL((encode_gf8_bs128u_kernel<m, p>), dim3(grid), dim3(512), 0, st, cs, (uint32_t)sets, rev)
#ifdef RSM_DIAG
    {
        const int mode = row ? g_diag_row_mode.load() : g_diag_mode.load();
        const uint32_t xcd = (uint32_t)g_diag_xcd.load();
        const uint32_t rev = (row ? 0u : (uint32_t)g_diag_rev.load()) | (((xcd >> (row ? 0 : 1)) & 1u) << 1);
        switch (mode) {
            case 2: RSM_BS_LAUNCH(10, 1); return hipGetLastError();  // no arithmetic (wrong output)
            case 4: RSM_BS_LAUNCH(12, 1); return hipGetLastError();  // no global memory (wrong output)
            case 0: RSM_BS_LAUNCH(0, 1); return hipGetLastError();   // A/B variants
            case 8: RSM_BS_LAUNCH(8, 1); return hipGetLastError();
            case 24: RSM_BS_LAUNCH(24, 1); return hipGetLastError();
            case 56: RSM_BS_LAUNCH(56, 1); return hipGetLastError();
            case 32: RSM_BS_LAUNCH(32, 1); return hipGetLastError();   // NT loads, dword exchange writes
            case 16: RSM_BS_LAUNCH(16, 1); return hipGetLastError();
            case 42: RSM_BS_LAUNCH(42, 1); return hipGetLastError();  // no arithmetic (wrong output)
            case 58: RSM_BS_LAUNCH(58, 1); return hipGetLastError();  // no arithmetic (wrong output)
            case 44: RSM_BS_LAUNCH(44, 1); return hipGetLastError();  // no global memory (wrong output)
            case 104: RSM_BS_LAUNCH(104, 1); return hipGetLastError();  // 40 + late direct loads
            case 120: RSM_BS_LAUNCH(120, 1); return hipGetLastError();  // 56 + late direct loads
            case 184: RSM_BS_LAUNCH(184, 1); return hipGetLastError();  // 56 + later direct loads
            case 376: RSM_BS_LAUNCH(376, 1); return hipGetLastError();  // 56 + late direct + split DMA
            case 440: RSM_BS_LAUNCH(440, 1); return hipGetLastError();  // 56 + later direct + split DMA
            case 168: RSM_BS_LAUNCH(168, 1); return hipGetLastError();  // 40 + later direct loads
            case 360: RSM_BS_LAUNCH(360, 1); return hipGetLastError();  // 40 + late direct + split DMA
            default: break;
        }
        if (row) RSM_BS_LAUNCH(104, 0);
        else RSM_BS_LAUNCH(184, 1);
        return hipGetLastError();
    }
#else
    const uint32_t rev = row ? 0u : 1u;
    if (row) RSM_BS_LAUNCH(104, 0);
    else RSM_BS_LAUNCH(184, 1);
#endif
#undef RSM_BS_LAUNCH
    return hipGetLastError();
}

// The queue launch needs whole sets per square in both passes (k * S a multiple of
// 2 KiB: every k = 128 square) and the plain row/column CodewordSets to qualify.
bool bs128_queue_applicable(const CodewordSet& rows, const CodewordSet& cols) {
    if (rows.k != 128 || ((uint64_t)rows.k * rows.S) % kSetBytes != 0) return false;
    return bs128_applicable(rows) && bs128_applicable(cols);
}

// Production: MODE 18472 (ds_write_addtid_b32 exchange; the direct half of the next
// set's loads after the small IFFT layers for a column set, right after the first
// exchange for a row set).  Measured (profiles/r02g_queue_ab.jsonl, 3 streams, same
// box): 256 squares per step 8.53 us per square against 8.59-8.60 with both after the
// small IFFT layers (MODE 2088), 8.68-8.76 the other way round; 2088 against 104 (both
// right after the first exchange) 8.43 vs 8.57-8.59, 8.73 right after the transposes; at 128 squares 104 gave 8.80-8.89 against 9.08 after the large
// layers and 9.52 at the top of the set; Q0 read non-temporal +3 %, Q1 read with the
// default policy +3 % (the Infinity-Cache re-read of Q0 needs the default policy, the
// last read of Q1 is best non-temporal).
#ifdef RSM_DIAG
static std::atomic<uint32_t*> g_diag_trace{nullptr};
void set_bs128_diag_trace(uint32_t* d) { g_diag_trace.store(d); }
#endif
hipError_t launch_extend_gf8_bs128_queue(const QueuePlan& p0, hipStream_t st) {
    QueuePlan p = p0;
#ifdef RSM_DIAG
    p.trace = g_diag_trace.load();
#endif
    const uint32_t total = p.nmain + p.nq1;
    if (total == 0) return hipSuccess;
    const uint32_t cap = p.rows.grid ? p.rows.grid : 256u;
    const uint32_t grid = total < cap ? total : cap;
    const bool geo = lane_geo_ok(p.rows) && lane_geo_ok(p.cols);
#ifdef RSM_DIAG
    // diagnostic codes: 2 / 4 no arithmetic / no memory (wrong output by design);
    // 104 direct loads right after the first exchange, 140 after the large layers,
    // 168 rows early / columns late, 296 at the top of the set, 616 = 104 + Q0
    // non-temporal, 1064 after the transposes, 2088 after the small IFFT layers,
    // 4200 = 104 + Q1 default policy, 10280 rows after the small IFFT / columns after
    // the exchange
    switch (g_diag_mode.load()) {
        // half-split schedule (production) and its diagnostic variants
        case 40:  // production (as below)
            if (geo) hipLaunchKernelGGL((extend_gf8_bs128s_kernel<16777216>), dim3(grid), dim3(512), 0, st, p);
            else hipLaunchKernelGGL((extend_gf8_bs128s_kernel<0>), dim3(grid), dim3(512), 0, st, p);
            break;
        case 54000: hipLaunchKernelGGL((extend_gf8_bs128s_kernel<0>), dim3(grid), dim3(512), 0, st, p); break;
        case 50002: hipLaunchKernelGGL((extend_gf8_bs128s_kernel<2>), dim3(grid), dim3(512), 0, st, p); break;
        case 50004: hipLaunchKernelGGL((extend_gf8_bs128s_kernel<4>), dim3(grid), dim3(512), 0, st, p); break;
        case 50768: hipLaunchKernelGGL((extend_gf8_bs128s_kernel<32768>), dim3(grid), dim3(512), 0, st, p); break;
        case 50772: hipLaunchKernelGGL((extend_gf8_bs128s_kernel<32772>), dim3(grid), dim3(512), 0, st, p); break;
        case 50770: hipLaunchKernelGGL((extend_gf8_bs128s_kernel<32770>), dim3(grid), dim3(512), 0, st, p); break;
        case 51000: hipLaunchKernelGGL((extend_gf8_bs128s_kernel<65536>), dim3(grid), dim3(512), 0, st, p); break;
        case 51001: hipLaunchKernelGGL((extend_gf8_bs128s_kernel<131072>), dim3(grid), dim3(512), 0, st, p); break;
        case 51002: hipLaunchKernelGGL((extend_gf8_bs128s_kernel<262144>), dim3(grid), dim3(512), 0, st, p); break;
        case 51010: hipLaunchKernelGGL((extend_gf8_bs128s_kernel<1048576 | 524288>), dim3(grid), dim3(512), 0, st, p); break;
        case 51020: hipLaunchKernelGGL((extend_gf8_bs128s_kernel<0>), dim3(grid), dim3(512), 0, st, p); break;
        case 51021: hipLaunchKernelGGL((extend_gf8_bs128s_kernel<1048576>), dim3(grid), dim3(512), 0, st, p); break;
        case 51030: hipLaunchKernelGGL((extend_gf8_bs128s_kernel<524288>), dim3(grid), dim3(512), 0, st, p); break;
        case 51014: hipLaunchKernelGGL((extend_gf8_bs128s_kernel<524292>), dim3(grid), dim3(512), 0, st, p); break;
        case 51012: hipLaunchKernelGGL((extend_gf8_bs128s_kernel<524290>), dim3(grid), dim3(512), 0, st, p); break;
        case 51004: hipLaunchKernelGGL((extend_gf8_bs128s_kernel<262148>), dim3(grid), dim3(512), 0, st, p); break;
        case 52040: hipLaunchKernelGGL((extend_gf8_bs128s_kernel<4194304>), dim3(grid), dim3(512), 0, st, p); break;
        case 53000: hipLaunchKernelGGL((extend_gf8_bs128s_kernel<8388608>), dim3(grid), dim3(512), 0, st, p); break;
        // XCD-affine queues (needs count % 8 == 0 and the host's zeroed 8-XCD queue words)
        case 57000: hipLaunchKernelGGL((extend_gf8_bs128s_kernel<16777216 | 134217728>), dim3(grid), dim3(512), 0, st, p); break;
        case 56000: hipLaunchKernelGGL((extend_gf8_bs128s_kernel<16777216 | 67108864>), dim3(grid), dim3(512), 0, st, p); break;
        case 55000: hipLaunchKernelGGL((extend_gf8_bs128s_kernel<16777216 | 33554432>), dim3(grid), dim3(512), 0, st, p); break;
        case 55002: hipLaunchKernelGGL((extend_gf8_bs128s_kernel<16777216 | 33554432 | 2>), dim3(grid), dim3(512), 0, st, p); break;
        case 55004: hipLaunchKernelGGL((extend_gf8_bs128s_kernel<16777216 | 33554432 | 4>), dim3(grid), dim3(512), 0, st, p); break;
        case 51006: hipLaunchKernelGGL((extend_gf8_bs128s_kernel<262146>), dim3(grid), dim3(512), 0, st, p); break;
        // round-2 schedule (bs_queue_wave) for A/B
        case 18472: hipLaunchKernelGGL((extend_gf8_bs128q_kernel<18472>), dim3(grid), dim3(512), 0, st, p); break;
        case 2: hipLaunchKernelGGL((extend_gf8_bs128q_kernel<18474>), dim3(grid), dim3(512), 0, st, p); break;
        case 4: hipLaunchKernelGGL((extend_gf8_bs128q_kernel<18476>), dim3(grid), dim3(512), 0, st, p); break;
        case 104: hipLaunchKernelGGL((extend_gf8_bs128q_kernel<104>), dim3(grid), dim3(512), 0, st, p); break;
        case 140: hipLaunchKernelGGL((extend_gf8_bs128q_kernel<40>), dim3(grid), dim3(512), 0, st, p); break;
        case 168: hipLaunchKernelGGL((extend_gf8_bs128q_kernel<168>), dim3(grid), dim3(512), 0, st, p); break;
        case 296: hipLaunchKernelGGL((extend_gf8_bs128q_kernel<296>), dim3(grid), dim3(512), 0, st, p); break;
        case 616: hipLaunchKernelGGL((extend_gf8_bs128q_kernel<616>), dim3(grid), dim3(512), 0, st, p); break;
        case 1064: hipLaunchKernelGGL((extend_gf8_bs128q_kernel<1064>), dim3(grid), dim3(512), 0, st, p); break;
        case 4200: hipLaunchKernelGGL((extend_gf8_bs128q_kernel<4200>), dim3(grid), dim3(512), 0, st, p); break;
        case 10280: hipLaunchKernelGGL((extend_gf8_bs128q_kernel<10280>), dim3(grid), dim3(512), 0, st, p); break;
        case 2088: hipLaunchKernelGGL((extend_gf8_bs128q_kernel<2088>), dim3(grid), dim3(512), 0, st, p); break;
        case 32768: hipLaunchKernelGGL((extend_gf8_bs128q_kernel<18472 | 32768>), dim3(grid), dim3(512), 0, st, p); break;
        case 65536: hipLaunchKernelGGL((extend_gf8_bs128q_kernel<18472 | 65536>), dim3(grid), dim3(512), 0, st, p); break;
        case 131072: hipLaunchKernelGGL((extend_gf8_bs128q_kernel<18472 | 131072>), dim3(grid), dim3(512), 0, st, p); break;
        case 98304: hipLaunchKernelGGL((extend_gf8_bs128q_kernel<18472 | 98304>), dim3(grid), dim3(512), 0, st, p); break;
        case 32772: hipLaunchKernelGGL((extend_gf8_bs128q_kernel<18476 | 32768>), dim3(grid), dim3(512), 0, st, p); break;
        default:
            if (geo) hipLaunchKernelGGL((extend_gf8_bs128s_kernel<16777216>), dim3(grid), dim3(512), 0, st, p);
            else hipLaunchKernelGGL((extend_gf8_bs128s_kernel<0>), dim3(grid), dim3(512), 0, st, p);
            break;
    }
#else
    if (geo) hipLaunchKernelGGL((extend_gf8_bs128s_kernel<16777216>), dim3(grid), dim3(512), 0, st, p);
    else hipLaunchKernelGGL((extend_gf8_bs128s_kernel<0>), dim3(grid), dim3(512), 0, st, p);
#endif
    return hipGetLastError();
}

#ifdef RSM_DIAG
hipError_t launch_encode_gf8_bs128_dual(const DualPlan& p, hipStream_t st) {
    const uint32_t sets = p.na + p.nb;
    if (sets == 0) return hipSuccess;
    const uint32_t cap = p.a.grid ? p.a.grid : 256u;
    const uint32_t grid = sets < cap ? sets : cap;
    hipLaunchKernelGGL((encode_gf8_bs128p_kernel<40>), dim3(grid), dim3(512), 0, st, p);
    return hipGetLastError();
}
#endif  // RSM_DIAG

}  // namespace rsm
