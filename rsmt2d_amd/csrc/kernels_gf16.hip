// kernels_gf16.hip -- CDNA4 Leopard GF(2^16) Reed-Solomon kernels (2k > 256).
//
// klauspost/reedsolomon v1.14.1 leopard.go semantics:
// symbol t of every 64-byte block b of a share is lo = share[64b+t], hi =
// share[64b+32+t] (A.6).  A lane holds 4 adjacent symbols as two dwords (4 lo
// bytes, 4 hi bytes), so a wavefront spans 8 blocks = 512 bytes of share width
// and every multiply-by-constant is 12 v_perm_b32 lookups (PermTab16).
//
// Encode (m = ceilPow2(k) in {256, 512}) is ONE pass per codeword: a workgroup owns a
// (codeword, chunk) and keeps its m-point IFFT + FFT on chip (m = 256: 256-byte chunks,
// one element per lane-half, enc16h_kernel; m = 512 as follows) -- a workgroup of
// m/32 waves, each holding E = 32 elements of a 512-byte chunk in registers; one LDS exchange
// buffer ([element][lane] dwords, one plane at a time) switches between
//   group layout   (wave w: elements 32 w .. 32 w + 31):  layers d < 32
//   residue layout (wave w: residues r = (32/R) w + s, elements r + 32 j, j < R =
//                   m/32):                                 layers d = 32 .. m/2
// so the data shares are read once and the parity shares written once.
// The decoder's n = 2m transforms still run as radix-16 passes through a global
// work array ([codeword][element][S]):
//   decode (n = 2m): 1 group: scale by the error locator + IFFT low
//                    2 residue: IFFT high; also H(in) = high-bit half of the formal derivative
//                    3 group: out = in + L(in) + H(in)  (the derivative's closed form)
//                    4 residue: FFT high          5 group: FFT low + reveal
// Every wave works on one (codeword, 512-byte chunk, group|residue) task, so all
// lanes share each twiddle (wave-uniform SGPR table loads).
#include <hip/hip_runtime.h>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <type_traits>
#include <utility>
#include "gf16.hpp"
#include "rsm_kernels.hpp"

namespace rsm {
namespace {

constexpr uint32_t kMod16 = 65535u;
constexpr uint32_t kOob16 = 0x80000000u;
// The single-pass decoders load only the present cells, after the presence ballot.
// RSM_DEC16_EAGER (diagnostic A/B builds) loads every cell right away instead, before the
// ballot, and zeroes the absent ones: slower on MI355X (k = 256 sweep 0.233-0.236 against
// 0.220-0.224 ms, k = 512 1.151-1.177 against 1.134-1.139; profiles/r06c_dec16_eager_ab.jsonl)
// -- the doubled reads of a sweep whose tasks all start together cost more than the
// presence latency they hide.
#ifdef RSM_DEC16_EAGER
constexpr bool kDec16Eager = true;
#else
constexpr bool kDec16Eager = false;
#endif
// dec16h_kernel stages its twiddle tables right where the pool is free.  RSM_DEC16_PREFETCH
// (diagnostic A/B builds) issues their loads before the scale multiplies instead and stores
// them after the barrier that frees the pool: no faster (k = 512 sweep 1.115-1.157 against
// 1.126-1.146 ms, profiles/r06d_dec16_prefetch_ab.jsonl) -- the staging is not on the
// critical path.  (Loading the reveal tables before the group FFT the same way spills 32
// bytes per lane at 128 VGPRs: kDec16PrefetchRv stays off.)
#ifdef RSM_DEC16_PREFETCH
constexpr bool kDec16PrefetchTw = true, kDec16PrefetchRv = false;
#else
constexpr bool kDec16PrefetchTw = false, kDec16PrefetchRv = false;
#endif

template <int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
    [&]<int... I>(std::integer_sequence<int, I...>) {
        (f(std::integral_constant<int, I>{}), ...);
    }(std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t pm(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}

// The six perm selectors of a lane's 4 symbols (lo dword yl, hi dword yh): bits 0-2,
// 3-5 and 6-7 of every byte.  The shifted groups of both dwords come from ONE 64-bit
// shift of the pair (yh:yl) each -- v_lshrrev_b64 issues at the rate of a 32-bit shift
// (profiles/r03_alu64.jsonl), so 2 half-rate shifts instead of 4 per multiply; the bits
// yh pushes into yl's top byte are masked off with the selector bits.  (Written as asm:
// the compiler folds the masked 64-bit shift back into two 32-bit ones.)
struct Sel16 {
    uint32_t a, b, c, d, e, f;
};
__device__ __forceinline__ Sel16 sel16(uint32_t yl, uint32_t yh) {
#ifdef RSM_SEL32  // (diagnostic A/B builds only: the round-5 selectors, four 32-bit shifts)
    return Sel16{yl & 0x07070707u, (yl >> 3) & 0x07070707u, (yl >> 6) & 0x03030303u,
                 yh & 0x07070707u, (yh >> 3) & 0x07070707u, (yh >> 6) & 0x03030303u};
#endif
    const uint64_t y = ((uint64_t)yh << 32) | yl;
    uint64_t y3, y6;
    asm("v_lshrrev_b64 %0, 3, %1" : "=v"(y3) : "v"(y));
    asm("v_lshrrev_b64 %0, 6, %1" : "=v"(y6) : "v"(y));
    return Sel16{yl & 0x07070707u,        (uint32_t)y3 & 0x07070707u, (uint32_t)y6 & 0x03030303u,
                 yh & 0x07070707u, (uint32_t)(y3 >> 32) & 0x07070707u, (uint32_t)(y6 >> 32) & 0x03030303u};
}

// (xl, xh) ^= (yl, yh) * exp(L), tables t = PermTab16[L]
__device__ __forceinline__ void muladd16(uint32_t& xl, uint32_t& xh, uint32_t yl, uint32_t yh, const PermTab16& t) {
    const Sel16 q = sel16(yl, yh);
    const uint32_t sa = q.a, sb = q.b, sc = q.c, sd = q.d, se = q.e, sf = q.f;
    xl = x3(x3(xl, pm(t.w[1], t.w[0], sa), pm(t.w[5], t.w[4], sb)),
            x3(pm(t.w[8], t.w[8], sc), pm(t.w[13], t.w[12], sd), pm(t.w[17], t.w[16], se)), pm(t.w[20], t.w[20], sf));
    xh = x3(x3(xh, pm(t.w[3], t.w[2], sa), pm(t.w[7], t.w[6], sb)),
            x3(pm(t.w[10], t.w[10], sc), pm(t.w[15], t.w[14], sd), pm(t.w[19], t.w[18], se)), pm(t.w[22], t.w[22], sf));
}
__device__ __forceinline__ void mul16(uint32_t& xl, uint32_t& xh, const PermTab16& t) {
    const uint32_t yl = xl, yh = xh;
    xl = 0;
    xh = 0;
    muladd16(xl, xh, yl, yh, t);
}

struct Res {
    const PermTab16* perm;
    const uint16_t* skew;
};

__device__ __forceinline__ uint32_t skew_at(const Res& r, int idx) {
    return __builtin_amdgcn_readfirstlane((uint32_t)r.skew[idx]);
}

// IFFT_DIT2 / FFT_DIT2 over packed symbols with a runtime (wave-uniform) twiddle.
__device__ __forceinline__ void ifft2(uint32_t& xl, uint32_t& xh, uint32_t& yl, uint32_t& yh, uint32_t L, const Res& r) {
    yl ^= xl;
    yh ^= xh;
    if (L != kMod16) muladd16(xl, xh, yl, yh, r.perm[L]);
}
__device__ __forceinline__ void fft2(uint32_t& xl, uint32_t& xh, uint32_t& yl, uint32_t& yh, uint32_t L, const Res& r) {
    if (L != kMod16) muladd16(xl, xh, yl, yh, r.perm[L]);
    yl ^= xl;
    yh ^= xh;
}

// Group layout: 16 consecutive elements 16g..16g+15.  IFFT layers d = 1..8, block b
// uses SKEW[OFF + b + d]; FFT layers d = 8..1 use SKEW[OFF2 + b + d].
__device__ __forceinline__ void group_ifft(uint32_t (&l)[16], uint32_t (&h)[16], uint32_t g, int off, const Res& r) {
    sfor<4>([&](auto LG) {
        constexpr int d = 1 << decltype(LG)::value;
        sfor<8>([&](auto Q) {
            constexpr int q = decltype(Q)::value;
            constexpr int bl = (q / d) * 2 * d;
            constexpr int i = bl + (q % d);
            const uint32_t L = skew_at(r, off + (int)(16 * g) + bl + d);
            ifft2(l[i], h[i], l[i + d], h[i + d], L, r);
        });
    });
}
__device__ __forceinline__ void group_fft(uint32_t (&l)[16], uint32_t (&h)[16], uint32_t g, const Res& r) {
    sfor<4>([&](auto LG) {
        constexpr int d = 8 >> decltype(LG)::value;
        sfor<8>([&](auto Q) {
            constexpr int q = decltype(Q)::value;
            constexpr int bl = (q / d) * 2 * d;
            constexpr int i = bl + (q % d);
            const uint32_t L = skew_at(r, (int)(16 * g) + bl + d - 1);
            fft2(l[i], h[i], l[i + d], h[i + d], L, r);
        });
    });
}
// Residue layout: R elements rho + 16 j.  Element distance D = 16 d', block
// b = 16 * (j-block start).
template <int R>
__device__ __forceinline__ void residue_ifft(uint32_t (&l)[R], uint32_t (&h)[R], int off, const Res& r) {
    sfor<12>([&](auto LG) {
        constexpr int d = 1 << decltype(LG)::value;
        if constexpr (d < R) {
            sfor<R / 2>([&](auto Q) {
                constexpr int q = decltype(Q)::value;
                constexpr int bl = (q / d) * 2 * d;
                constexpr int i = bl + (q % d);
                const uint32_t L = skew_at(r, off + 16 * bl + 16 * d);
                ifft2(l[i], h[i], l[i + d], h[i + d], L, r);
            });
        }
    });
}
template <int R>
__device__ __forceinline__ void residue_fft(uint32_t (&l)[R], uint32_t (&h)[R], const Res& r) {
    sfor<12>([&](auto LG) {
        constexpr int d = 2048 >> decltype(LG)::value;
        if constexpr (d < R) {
            sfor<R / 2>([&](auto Q) {
                constexpr int q = decltype(Q)::value;
                constexpr int bl = (q / d) * 2 * d;
                constexpr int i = bl + (q % d);
                const uint32_t L = skew_at(r, 16 * bl + 16 * d - 1);
                fft2(l[i], h[i], l[i + d], h[i + d], L, r);
            });
        }
    });
}

// closed-form formal derivative restricted to one coordinate:
//   D'(x)[j] = XOR_{t: bit t of j == 0, j + 2^t < N} x[j + 2^t]   (without the x[j] term)
template <int N>
__device__ __forceinline__ void deriv_terms(const uint32_t (&xl)[N], const uint32_t (&xh)[N], uint32_t (&ol)[N],
                                            uint32_t (&oh)[N]) {
    sfor<N>([&](auto J) {
        constexpr int j = decltype(J)::value;
        uint32_t al = 0, ah = 0;
        sfor<12>([&](auto T) {
            constexpr int t = decltype(T)::value;
            if constexpr ((1 << t) < N && ((j >> t) & 1) == 0 && j + (1 << t) < N) {
                al ^= xl[j + (1 << t)];
                ah ^= xh[j + (1 << t)];
            }
        });
        ol[j] = al;
        oh[j] = ah;
    });
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0,
                                             (int)kOob16, 0x00020000);
}
__device__ __forceinline__ uint32_t ld(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0);
}
__device__ __forceinline__ void st(__amdgpu_buffer_rsrc_t r, uint32_t v, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_buffer_store_b32(v, r, voff, soff, 0);
}

// Per-task geometry: lane -> (lo byte offset) within the share; OOB when past S.
struct Lane {
    uint32_t lo;  // byte offset of this lane's 4 lo bytes (hi = lo + 32)
};
__device__ __forceinline__ Lane lane_of(uint32_t chunk, uint32_t S) {
    const uint32_t l = threadIdx.x & 63u;
    const uint32_t block = chunk * 8u + (l >> 3);
    const uint32_t off = block * 64u + (l & 7u) * 4u;
    return Lane{off < S ? off : kOob16};
}

__device__ __forceinline__ uint64_t cw_rel(const CodewordSet& cs, uint32_t q) {
    if (cs.indices != nullptr) return (uint64_t)cs.indices[q] * cs.cw_stride;
    const uint32_t sq = q / cs.per_square;
    const uint32_t t = q - sq * cs.per_square;
    return (uint64_t)sq * cs.square_stride + (uint64_t)t * cs.cw_stride;
}

struct TaskIdx {
    uint32_t q, chunk, g;
    bool valid;
};
__device__ __forceinline__ TaskIdx task_of(uint32_t count, uint32_t chunks, uint32_t groups) {
    const uint32_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    TaskIdx t{};
    t.valid = w < count * chunks * groups;
    if (!t.valid) return t;
    t.g = w % groups;
    const uint32_t r = w / groups;
    t.chunk = r % chunks;
    t.q = r / chunks;
    return t;
}

// ---------------------------------------------------------------------------
// Single-pass encoder
// ---------------------------------------------------------------------------
struct Enc16 {
    CodewordSet cs;
    const PermTab16* tw;  // skewperm: twiddle table by skew index (zero where skipped)
    uint32_t chunks;
    // merged middle pair: the top IFFT layer (SKEW[m - 1 + m/2]) and the top FFT layer
    // (SKEW[m/2 - 1]) join the same pairs, so they run as ONE multiply by the sum of
    // the two twiddles: y ^= x; x ^= y * (t1 + t2); y ^= x (nullptr: the sum is 0 and
    // the pair is the identity).  Table from the host (run_encode).
    const PermTab16* mid;
};

constexpr int ilog2c(int x) { return x <= 1 ? 0 : 1 + ilog2c(x / 2); }

// The 20 PermTab16 words muladd16 reads, in this order (w[9], w[11], w[21] and
// w[23] are unused): a compact twiddle table of 80 bytes.
constexpr int kTabW = 20;
__device__ __forceinline__ int tab_word(int j) { return j < 9 ? j : (j == 9 ? 10 : (j < 18 ? j + 2 : (j == 18 ? 20 : 22))); }

// (xl, xh) ^= (yl, yh) * exp(L) with the compact table c in VGPRs (both v_perm
// sources are VGPRs: no copies through the one-SGPR-per-instruction bus).
__device__ __forceinline__ void muladd16v(uint32_t& xl, uint32_t& xh, uint32_t yl, uint32_t yh, const uint32_t (&c)[kTabW]) {
    const Sel16 q = sel16(yl, yh);
    const uint32_t sa = q.a, sb = q.b, sc = q.c, sd = q.d, se = q.e, sf = q.f;
    // c: 0..7 = w0..w7, 8 = w8, 9 = w10, 10..17 = w12..w19, 18 = w20, 19 = w22
    xl = x3(x3(xl, pm(c[1], c[0], sa), pm(c[5], c[4], sb)),
            x3(pm(c[8], c[8], sc), pm(c[11], c[10], sd), pm(c[15], c[14], se)), pm(c[18], c[18], sf));
    xh = x3(x3(xh, pm(c[3], c[2], sa), pm(c[7], c[6], sb)),
            x3(pm(c[9], c[9], sc), pm(c[13], c[12], sd), pm(c[17], c[16], se)), pm(c[19], c[19], sf));
}
typedef uint32_t v4u16 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void tab_load(const uint32_t* lds, uint32_t (&c)[kTabW]) {
    sfor<kTabW / 4>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        const v4u16 v = *reinterpret_cast<const v4u16*>(lds + 4 * q);
        c[4 * q] = v.x; c[4 * q + 1] = v.y; c[4 * q + 2] = v.z; c[4 * q + 3] = v.w;
    });
}
// The same as ONE asm statement that waits for its own reads: the compiler can
// neither hoist a later block's table above the butterflies nor keep several tables
// live (the 128-register 16-wave kernels spilled ~700 dwords with tab_load).
__device__ __forceinline__ void tab_load_jit(const uint32_t* lds, uint32_t (&c)[kTabW]) {
    v4u16 a, b, e, f, g;
    const uint32_t base = (uint32_t)(uintptr_t)lds;
    asm volatile(
        "ds_read_b128 %0, %5\n\t"
        "ds_read_b128 %1, %5 offset:16\n\t"
        "ds_read_b128 %2, %5 offset:32\n\t"
        "ds_read_b128 %3, %5 offset:48\n\t"
        "ds_read_b128 %4, %5 offset:64\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(a), "=&v"(b), "=&v"(e), "=&v"(f), "=&v"(g)
        : "v"(base)
        : "memory");
    c[0] = a.x; c[1] = a.y; c[2] = a.z; c[3] = a.w;
    c[4] = b.x; c[5] = b.y; c[6] = b.z; c[7] = b.w;
    c[8] = e.x; c[9] = e.y; c[10] = e.z; c[11] = e.w;
    c[12] = f.x; c[13] = f.y; c[14] = f.z; c[15] = f.w;
    c[16] = g.x; c[17] = g.y; c[18] = g.z; c[19] = g.w;
}
// The same at a compile-time byte offset from `lds` (the instruction's offset field):
// a per-lane base (the half-wave forms) then stays ONE address register instead of
// one per table.
template <int OFF>
__device__ __forceinline__ void tab_load_jit_at(const uint32_t* lds, uint32_t (&c)[kTabW]) {
    static_assert(OFF >= 0 && OFF + 64 < 65536, "ds_read offset field");
    v4u16 a, b, e, f, g;
    const uint32_t base = (uint32_t)(uintptr_t)lds;
    asm volatile(
        "ds_read_b128 %0, %5 offset:%6\n\t"
        "ds_read_b128 %1, %5 offset:%7\n\t"
        "ds_read_b128 %2, %5 offset:%8\n\t"
        "ds_read_b128 %3, %5 offset:%9\n\t"
        "ds_read_b128 %4, %5 offset:%10\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(a), "=&v"(b), "=&v"(e), "=&v"(f), "=&v"(g)
        : "v"(base), "i"(OFF), "i"(OFF + 16), "i"(OFF + 32), "i"(OFF + 48), "i"(OFF + 64)
        : "memory");
    c[0] = a.x; c[1] = a.y; c[2] = a.z; c[3] = a.w;
    c[4] = b.x; c[5] = b.y; c[6] = b.z; c[7] = b.w;
    c[8] = e.x; c[9] = e.y; c[10] = e.z; c[11] = e.w;
    c[12] = f.x; c[13] = f.y; c[14] = f.z; c[15] = f.w;
    c[16] = g.x; c[17] = g.y; c[18] = g.z; c[19] = g.w;
}
// Butterflies with the twiddle table given directly (zero table = no multiply).
__device__ __forceinline__ void ifft2t(uint32_t& xl, uint32_t& xh, uint32_t& yl, uint32_t& yh, const PermTab16& t) {
    yl ^= xl;
    yh ^= xh;
    muladd16(xl, xh, yl, yh, t);
}
__device__ __forceinline__ void fft2t(uint32_t& xl, uint32_t& xh, uint32_t& yl, uint32_t& yh, const PermTab16& t) {
    muladd16(xl, xh, yl, yh, t);
    yl ^= xl;
    yh ^= xh;
}
__device__ __forceinline__ void ifft2v(uint32_t& xl, uint32_t& xh, uint32_t& yl, uint32_t& yh, const uint32_t (&c)[kTabW]) {
    yl ^= xl;
    yh ^= xh;
    muladd16v(xl, xh, yl, yh, c);
}
__device__ __forceinline__ void fft2v(uint32_t& xl, uint32_t& xh, uint32_t& yl, uint32_t& yh, const uint32_t (&c)[kTabW]) {
    muladd16v(xl, xh, yl, yh, c);
    yl ^= xl;
    yh ^= xh;
}

// Twiddle tables of a transform stage over n-point runs, one per (layer, block):
// layer d = 2^L has n/(2d) blocks at slots (n - (n >> L)) + block, n - 1 slots.
__device__ __forceinline__ int slot_layer(int slot, int n) {
    int L = 0;
#pragma unroll
    for (int t = 1; t < 12; ++t) L += (n >> t) > 0 && slot >= n - (n >> t) ? 1 : 0;
    return L;
}

template <int WAVES, int E, int THREADS>
constexpr int grp_tab_per() { return (WAVES * (E - 1) * kTabW + THREADS - 1) / THREADS; }
template <int WAVES, int E, bool FFT, int THREADS = WAVES * 64>
__device__ __forceinline__ void load_grp(const PermTab16* tw, int off, uint32_t (&v)[grp_tab_per<WAVES, E, THREADS>()]) {
    constexpr int NT = WAVES * (E - 1), PER = grp_tab_per<WAVES, E, THREADS>();
    // opaque thread index: a second staging later in the kernel (dec16h_kernel) must not
    // reuse this one's index arithmetic, kept alive (spilled) in between
    uint32_t tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
#pragma unroll
    for (int r = 0; r < PER; ++r) {
        const int n = (int)tid + r * THREADS;
        const int T = n / kTabW, j = n - T * kTabW;
        const int w = T / (E - 1), slot = T - w * (E - 1);
        const int L = slot_layer(slot, E);
        const int d = 1 << L, bl = (slot - (E - (E >> L))) * 2 * d;
        const int idx = FFT ? E * w + bl + d - 1 : off + E * w + bl + d;
        v[r] = n < NT * kTabW ? tw[idx].w[tab_word(j)] : 0u;
    }
}
template <int WAVES, int E, int THREADS = WAVES * 64>
__device__ __forceinline__ void store_grp(uint32_t* tab, const uint32_t (&v)[grp_tab_per<WAVES, E, THREADS>()]) {
    constexpr int NT = WAVES * (E - 1), PER = grp_tab_per<WAVES, E, THREADS>();
    uint32_t tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
#pragma unroll
    for (int r = 0; r < PER; ++r) {
        const int n = (int)tid + r * THREADS;
        if (n < NT * kTabW) tab[n] = v[r];
    }
}
// Stage into LDS `tab` the group-layout tables of every wave (wave w: E - 1
// slots, elements E w ..): IFFT SKEW[off + b + d] or FFT SKEW[b + d - 1].  Fixed
// trip count, loads first: every thread's table words are in flight at once.
template <int WAVES, int E, bool FFT, int THREADS = WAVES * 64>
__device__ __forceinline__ void stage_grp(uint32_t* tab, const PermTab16* tw, int off) {
    uint32_t v[grp_tab_per<WAVES, E, THREADS>()];
    load_grp<WAVES, E, FFT, THREADS>(tw, off, v);
    store_grp<WAVES, E, THREADS>(tab, v);
}
// Residue-layout tables (shared by all waves): slots 0..R-2 IFFT, R-1..2R-3 FFT.
template <int R, int E, int THREADS>
__device__ __forceinline__ void stage_res(uint32_t* tab, const PermTab16* tw, int off) {
    constexpr int NW = 2 * (R - 1) * kTabW, PER = (NW + THREADS - 1) / THREADS;
    uint32_t v[PER];
#pragma unroll
    for (int r = 0; r < PER; ++r) {
        const int n = (int)threadIdx.x + r * THREADS;
        const int T = n / kTabW, j = n - T * kTabW;
        const bool fft = T >= R - 1;
        const int slot = fft ? T - (R - 1) : T;
        const int L = slot_layer(slot, R);
        const int dj = 1 << L, bl = (slot - (R - (R >> L))) * 2 * dj;
        const int idx = fft ? E * bl + E * dj - 1 : off + E * bl + E * dj;
        v[r] = n < NW ? tw[idx].w[tab_word(j)] : 0u;
    }
#pragma unroll
    for (int r = 0; r < PER; ++r) {
        const int n = (int)threadIdx.x + r * THREADS;
        if (n < NW) tab[n] = v[r];
    }
}

// Group layout (E elements per wave): IFFT layers d = 1..E/2 ascending / FFT
// d = E/2..1 descending; the table of (layer, block) from this wave's E-1 slots.
template <int E, bool FFT, bool JIT = false>
__device__ __forceinline__ void grp_xform(uint32_t (&l)[E], uint32_t (&h)[E], const uint32_t* wtab) {
    constexpr int LN = ilog2c(E);
    sfor<LN>([&](auto LGi) {
        constexpr int L = FFT ? LN - 1 - decltype(LGi)::value : decltype(LGi)::value;
        constexpr int d = 1 << L;
        sfor<E / 2 / d>([&](auto Bk) {
            constexpr int block = decltype(Bk)::value;
            uint32_t c[kTabW];
            if constexpr (JIT) tab_load_jit_at<(E - (E >> L) + block) * kTabW * 4>(wtab, c);
            else tab_load(wtab + (E - (E >> L) + block) * kTabW, c);
            sfor<d>([&](auto Q) {
                constexpr int i = block * 2 * d + decltype(Q)::value;
                if constexpr (FFT) fft2v(l[i], h[i], l[i + d], h[i + d], c);
                else ifft2v(l[i], h[i], l[i + d], h[i + d], c);
                // JIT: pin the block's butterflies before the next block's table read
                if constexpr (JIT) asm volatile("" : "+v"(l[i]), "+v"(h[i]), "+v"(l[i + d]), "+v"(h[i + d]));
            });
        });
    });
}
// The same with each table read straight from global memory (wave-uniform:
// scalar loads), for the 16-wave m = 512 form whose registers leave no room for
// LDS-staged tables: IFFT SKEW[off + base + b + d], FFT SKEW[base + b + d - 1].
template <int E, bool FFT>
__device__ __forceinline__ void grp_xform_g(uint32_t (&l)[E], uint32_t (&h)[E], const PermTab16* tw, int base, int off) {
    constexpr int LN = ilog2c(E);
    sfor<LN>([&](auto LGi) {
        constexpr int L = FFT ? LN - 1 - decltype(LGi)::value : decltype(LGi)::value;
        constexpr int d = 1 << L;
        sfor<E / 2 / d>([&](auto Bk) {
            constexpr int bl = decltype(Bk)::value * 2 * d;
            const PermTab16& t = tw[FFT ? base + bl + d - 1 : off + base + bl + d];
            sfor<d>([&](auto Q) {
                constexpr int i = bl + decltype(Q)::value;
                if constexpr (FFT) fft2t(l[i], h[i], l[i + d], h[i + d], t);
                else ifft2t(l[i], h[i], l[i + d], h[i + d], t);
            });
        });
    });
}
// Software-pipelined table reads (round 6): the NEXT block's table is read while this
// block's butterflies run, the wait sits after them.  tab_issue_at puts the five
// ds_read_b128 in flight without a wait; tab_wait waits for them and, through its "+v"
// operands, is the point from which the compiler may read them.  The caller pins each
// block's butterfly outputs before the wait (their asm operands), so the wait cannot be
// hoisted above the butterflies it is meant to overlap.  Two table buffers alternate by
// block parity (compile-time), so no table is copied.
typedef uint32_t tab_v4 __attribute__((ext_vector_type(4)));
struct Tab5 {
    tab_v4 q[5];
};
template <int OFF>
__device__ __forceinline__ void tab_issue_at(uint32_t base, Tab5& t) {
    static_assert(OFF >= 0 && OFF + 64 < 65536, "ds_read offset field");
    asm volatile(
        "ds_read_b128 %0, %5 offset:%6\n\t"
        "ds_read_b128 %1, %5 offset:%7\n\t"
        "ds_read_b128 %2, %5 offset:%8\n\t"
        "ds_read_b128 %3, %5 offset:%9\n\t"
        "ds_read_b128 %4, %5 offset:%10"
        : "=&v"(t.q[0]), "=&v"(t.q[1]), "=&v"(t.q[2]), "=&v"(t.q[3]), "=&v"(t.q[4])
        : "v"(base), "i"(OFF), "i"(OFF + 16), "i"(OFF + 32), "i"(OFF + 48), "i"(OFF + 64)
        : "memory");
}
__device__ __forceinline__ void tab_wait(Tab5& t) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(t.q[0]), "+v"(t.q[1]), "+v"(t.q[2]), "+v"(t.q[3]), "+v"(t.q[4]) :: "memory");
}
__device__ __forceinline__ void tab_unpack(const Tab5& t, uint32_t (&c)[kTabW]) {
    sfor<5>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        c[4 * q] = t.q[q].x; c[4 * q + 1] = t.q[q].y; c[4 * q + 2] = t.q[q].z; c[4 * q + 3] = t.q[q].w;
    });
}
// block n (execution order) of the first NLAY layers of a P-point transform (layer L:
// P / 2 / 2^L blocks; IFFT ascending, FFT descending): its layer and its block
template <int P, int NLAY, bool FFT>
constexpr int pipe_layer(int n) {
    for (int k = 0; k < NLAY; ++k) {
        const int L = FFT ? NLAY - 1 - k : k, nb = P / 2 / (1 << L);
        if (n < nb) return L;
        n -= nb;
    }
    return -1;
}
template <int P, int NLAY, bool FFT>
constexpr int pipe_block(int n) {
    for (int k = 0; k < NLAY; ++k) {
        const int L = FFT ? NLAY - 1 - k : k, nb = P / 2 / (1 << L);
        if (n < nb) return n;
        n -= nb;
    }
    return -1;
}
// grp_xform with pipelined table reads (E - 1 blocks, tables at wtab slot E - (E >> L) + block)
template <int E, bool FFT>
__device__ __forceinline__ void grp_xform_pipe(uint32_t (&l)[E], uint32_t (&h)[E], const uint32_t* wtab) {
    constexpr int NB = E - 1, NL = ilog2c(E);
    const uint32_t base = (uint32_t)(uintptr_t)wtab;
    Tab5 ta, tb;
    {
        constexpr int L0 = pipe_layer<E, NL, FFT>(0), B0 = pipe_block<E, NL, FFT>(0);
        tab_issue_at<(E - (E >> L0) + B0) * kTabW * 4>(base, ta);
        tab_wait(ta);
    }
    sfor<NB>([&](auto N) {
        constexpr int n = decltype(N)::value;
        constexpr int L = pipe_layer<E, NL, FFT>(n), bk = pipe_block<E, NL, FFT>(n), d = 1 << L;
        Tab5& cur = (n & 1) ? tb : ta;
        Tab5& nxt = (n & 1) ? ta : tb;
        if constexpr (n + 1 < NB) {
            constexpr int L1 = pipe_layer<E, NL, FFT>(n + 1), B1 = pipe_block<E, NL, FFT>(n + 1);
            tab_issue_at<(E - (E >> L1) + B1) * kTabW * 4>(base, nxt);
        }
        uint32_t c[kTabW];
        tab_unpack(cur, c);
        sfor<d>([&](auto Q) {
            constexpr int i = bk * 2 * d + decltype(Q)::value;
            if constexpr (FFT) fft2v(l[i], h[i], l[i + d], h[i + d], c);
            else ifft2v(l[i], h[i], l[i + d], h[i + d], c);
            asm volatile("" : "+v"(l[i]), "+v"(h[i]), "+v"(l[i + d]), "+v"(h[i + d]));
        });
        if constexpr (n + 1 < NB) tab_wait(nxt);
    });
}
// rtab slot of residue block n: IFFT slots 0..R-2, FFT R-1..2R-3 (stage_res)
template <int R, bool FFT>
constexpr int res_pipe_slot(int n) {
    constexpr int NL = ilog2c(R) - 1;
    const int L = pipe_layer<R, NL, FFT>(n), b = pipe_block<R, NL, FFT>(n);
    return (FFT ? R - 1 : 0) + (R - (R >> L)) + b;
}
// res_xform (one residue per lane group, E == R, MERGED: the top layer is res_mid) with
// pipelined table reads: IFFT slots 0..R-2, FFT slots R-1..2R-3 of rtab
template <int R, bool FFT>
__device__ __forceinline__ void res_xform_pipe(uint32_t (&l)[R], uint32_t (&h)[R], const uint32_t* rtab) {
    constexpr int NL = ilog2c(R) - 1, NB = R - 2;  // layers dj = 1 .. R/4 (the merged top excluded)
    const uint32_t base = (uint32_t)(uintptr_t)rtab;
    Tab5 ta, tb;
    tab_issue_at<res_pipe_slot<R, FFT>(0) * kTabW * 4>(base, ta);
    tab_wait(ta);
    sfor<NB>([&](auto N) {
        constexpr int n = decltype(N)::value;
        constexpr int L = pipe_layer<R, NL, FFT>(n), bk = pipe_block<R, NL, FFT>(n), dj = 1 << L;
        Tab5& cur = (n & 1) ? tb : ta;
        Tab5& nxt = (n & 1) ? ta : tb;
        if constexpr (n + 1 < NB) tab_issue_at<res_pipe_slot<R, FFT>(n + 1) * kTabW * 4>(base, nxt);
        uint32_t c[kTabW];
        tab_unpack(cur, c);
        sfor<dj>([&](auto Q) {
            constexpr int j = bk * 2 * dj + decltype(Q)::value;
            if constexpr (FFT) fft2v(l[j], h[j], l[j + dj], h[j + dj], c);
            else ifft2v(l[j], h[j], l[j + dj], h[j + dj], c);
            asm volatile("" : "+v"(l[j]), "+v"(h[j]), "+v"(l[j + dj]), "+v"(h[j + dj]));
        });
        if constexpr (n + 1 < NB) tab_wait(nxt);
    });
}

// Residue-layout register of (residue s of the wave, j): s R + j (the full-buffer
// exchange), or -- IL, the half-buffer exchange -- (E / R) j + s, so that the
// registers a wave sends in one pass of xch_plane_half are exactly the ones it
// receives into (element bit 0 = s picks the pass in both layouts).
template <int E, int R, bool IL>
constexpr int ridx(int s, int j) { return IL ? (E / R) * j + s : s * R + j; }

template <int E, int R, bool FFT, bool MERGED = false, bool IL = false>
__device__ __forceinline__ void res_xform_g(uint32_t (&l)[E], uint32_t (&h)[E], const PermTab16* tw, int off) {
    constexpr int LN = ilog2c(R), NL = MERGED ? LN - 1 : LN;  // MERGED: the top layer is res_mid
    sfor<NL>([&](auto LGi) {
        constexpr int L = FFT ? NL - 1 - decltype(LGi)::value : decltype(LGi)::value;
        constexpr int dj = 1 << L;
        sfor<R / 2 / dj>([&](auto Bk) {
            constexpr int bl = decltype(Bk)::value * 2 * dj;
            const PermTab16& t = tw[FFT ? E * bl + E * dj - 1 : off + E * bl + E * dj];
            sfor<dj>([&](auto Q) {
                constexpr int j = bl + decltype(Q)::value;
                sfor<E / R>([&](auto Sx) {
                    constexpr int i = ridx<E, R, IL>(decltype(Sx)::value, j), i2 = ridx<E, R, IL>(decltype(Sx)::value, j + dj);
                    if constexpr (FFT) fft2t(l[i], h[i], l[i2], h[i2], t);
                    else ifft2t(l[i], h[i], l[i2], h[i2], t);
                });
            });
        });
    });
}
// The merged top pair of the residue layers (elements E R / 2 = m / 2 apart), see Enc16::mid.
template <int E, int R, bool IL = false>
__device__ __forceinline__ void res_mid(uint32_t (&l)[E], uint32_t (&h)[E], const PermTab16* mid) {
    constexpr int dj = R / 2;
    if (!mid) return;  // y ^= x twice: the identity
    const PermTab16& t = *mid;
    sfor<E / R>([&](auto Sx) {
        sfor<dj>([&](auto Q) {
            constexpr int i = ridx<E, R, IL>(decltype(Sx)::value, decltype(Q)::value);
            constexpr int i2 = ridx<E, R, IL>(decltype(Sx)::value, decltype(Q)::value + dj);
            l[i2] ^= l[i];
            h[i2] ^= h[i];
            muladd16(l[i], h[i], l[i2], h[i2], t);
            l[i2] ^= l[i];
            h[i2] ^= h[i];
        });
    });
}
// The same with the table read from LDS (mtab: kTabW words, staged from Enc16::mid).
template <int E, int R, bool IL, bool JIT>
__device__ __forceinline__ void res_mid_v(uint32_t (&l)[E], uint32_t (&h)[E], const uint32_t* mtab) {
    constexpr int dj = R / 2;
    uint32_t c[kTabW];
    if constexpr (JIT) tab_load_jit(mtab, c);
    else tab_load(mtab, c);
    sfor<E / R>([&](auto Sx) {
        sfor<dj>([&](auto Q) {
            constexpr int i = ridx<E, R, IL>(decltype(Sx)::value, decltype(Q)::value);
            constexpr int i2 = ridx<E, R, IL>(decltype(Sx)::value, decltype(Q)::value + dj);
            l[i2] ^= l[i];
            h[i2] ^= h[i];
            muladd16v(l[i], h[i], l[i2], h[i2], c);
            l[i2] ^= l[i];
            h[i2] ^= h[i];
            if constexpr (JIT) asm volatile("" : "+v"(l[i]), "+v"(h[i]), "+v"(l[i2]), "+v"(h[i2]));
        });
    });
}
// Residue layout: register s*R + j holds element r_s + E j; a layer over j at
// distance dj joins elements E dj apart (block start E bl): one table per
// (layer, block) for every residue of every wave.
template <int E, int R, bool FFT, bool MERGED = true, bool JIT = false, bool IL = false>
__device__ __forceinline__ void res_xform(uint32_t (&l)[E], uint32_t (&h)[E], const uint32_t* rtab) {
    constexpr int LN = ilog2c(R), NL = MERGED ? LN - 1 : LN;
    sfor<NL>([&](auto LGi) {  // MERGED: the top layer (dj = R/2) is res_mid
        constexpr int L = FFT ? NL - 1 - decltype(LGi)::value : decltype(LGi)::value;
        constexpr int dj = 1 << L;
        sfor<R / 2 / dj>([&](auto Bk) {
            constexpr int block = decltype(Bk)::value;
            uint32_t c[kTabW];
            if constexpr (JIT) tab_load_jit(rtab + ((FFT ? R - 1 : 0) + (R - (R >> L)) + block) * kTabW, c);
            else tab_load(rtab + ((FFT ? R - 1 : 0) + (R - (R >> L)) + block) * kTabW, c);
            sfor<dj>([&](auto Q) {
                constexpr int j = block * 2 * dj + decltype(Q)::value;
                sfor<E / R>([&](auto Sx) {
                    constexpr int i = ridx<E, R, IL>(decltype(Sx)::value, j), i2 = ridx<E, R, IL>(decltype(Sx)::value, j + dj);
                    if constexpr (FFT) fft2v(l[i], h[i], l[i2], h[i2], c);
                    else ifft2v(l[i], h[i], l[i2], h[i2], c);
                    if constexpr (JIT) asm volatile("" : "+v"(l[i]), "+v"(h[i]), "+v"(l[i2]), "+v"(h[i2]));
                });
            });
        });
    });
}

// One plane of the layout switch through LDS xch[element][lane].  Residue
// register s*R + j holds element (E/R) w + s + E j.
template <int E, int R, bool TO_RESIDUE>
__device__ __forceinline__ void xch_plane(uint32_t (&v)[E], uint32_t (*xch)[64], uint32_t w, uint32_t lane) {
    constexpr int RPW = E / R;  // residues per wave
    sfor<E>([&](auto I) {
        constexpr int i = decltype(I)::value;
        const uint32_t e = TO_RESIDUE ? E * w + i : (RPW * w + i / R) + E * (i % R);
        xch[e][lane] = v[i];
    });
    __syncthreads();
    sfor<E>([&](auto I) {
        constexpr int i = decltype(I)::value;
        const uint32_t e = TO_RESIDUE ? (RPW * w + i / R) + E * (i % R) : E * w + i;
        v[i] = xch[e][lane];
    });
    __syncthreads();
}

// One plane of the layout switch through HALF an element-indexed buffer xch[N/2][64]
// (the other half of the LDS holds the twiddle tables), in two passes: pass p moves
// the elements with bit 0 = p.  Group layout: register i = element E w + i (bit 0
// = bit 0 of i); residue layout with the IL register order ridx(s, j) = RPW j + s:
// element RPW w + s + E j, bit 0 = s (RPW = 2).  So in each pass a wave sends and
// receives the SAME registers (even ones, then odd ones), and no register is
// overwritten before it has been sent.  Buffer slot = element >> 1.
template <int E, int R, bool TO_RESIDUE>
__device__ __forceinline__ void xch_plane_half(uint32_t (&v)[E], uint32_t (*xch)[64], uint32_t w, uint32_t lane) {
    constexpr int RPW = E / R;
    static_assert(RPW % 2 == 0, "an even number of residues per wave: element bit 0 = bit 0 of s");
    sfor<2>([&](auto Pc) {
        constexpr int pp = decltype(Pc)::value;
        auto grp_slot = [&](int i) { return (E * w + (uint32_t)i) >> 1; };
        auto res_slot = [&](int s, int j) { return (RPW * w + (uint32_t)s + E * (uint32_t)j) >> 1; };
        if constexpr (TO_RESIDUE) {
            sfor<E / 2>([&](auto I) { constexpr int i = 2 * decltype(I)::value + pp; xch[grp_slot(i)][lane] = v[i]; });
        } else {
            sfor<RPW / 2>([&](auto Sx) {
                constexpr int sr = 2 * decltype(Sx)::value + pp;
                sfor<R>([&](auto J) { constexpr int j = decltype(J)::value; xch[res_slot(sr, j)][lane] = v[ridx<E, R, true>(sr, j)]; });
            });
        }
        __syncthreads();
        if constexpr (TO_RESIDUE) {
            sfor<RPW / 2>([&](auto Sx) {
                constexpr int sr = 2 * decltype(Sx)::value + pp;
                sfor<R>([&](auto J) { constexpr int j = decltype(J)::value; v[ridx<E, R, true>(sr, j)] = xch[res_slot(sr, j)][lane]; });
            });
        } else {
            sfor<E / 2>([&](auto I) { constexpr int i = 2 * decltype(I)::value + pp; v[i] = xch[grp_slot(i)][lane]; });
        }
        __syncthreads();
    });
}

// Encoder: parity of codeword q, chunk c (512 bytes) = FFT(IFFT(data)).  The
// encoder's IFFT uses SKEW[m - 1 + b + d] (data occupy the upper half of the
// 2m-point domain), its FFT SKEW[b + d - 1]; every index is < 2m <= kSkewPermN.
// Twiddle tables: staged in LDS per workgroup (the group stages' 31 per wave in
// the exchange buffer, which is idle then; the residue stages' in rtab), read by
// uniform ds_read_b128 -- a table load from L2 per butterfly would leave the waves
// waiting on scalar loads (the tables of one transform exceed the scalar cache).
// m/32 waves of E = 32 elements; residues of R = m/32 elements.
//   m = 256: 8 waves (2 per SIMD, up to 256 registers), persistent (one workgroup
//            per CU), twiddle tables staged once into LDS and read by uniform
//            ds_read_b128 -- one scalar table load from L2 per butterfly left the
//            waves waiting (the tables of a transform exceed the scalar cache);
//   m = 512: 16 waves (128 registers each, no room for LDS-read tables), one
//            workgroup per task, tables by scalar loads (A/B: faster here).
// E = 64 (m = 512 only, round 3q): 8 waves of 64 elements, 256 registers each (the
// 16-wave form is held to 128 registers and spills 44 dwords per lane); the merged
// middle pair is affordable there.
// HX (m = 512, 16 waves; production HX = 3 since round 4): persistent, the twiddle
// tables staged in LDS beside HALF an exchange buffer (two passes per plane,
// xch_plane_half, the IL residue register order); the top residue layer pair is not
// merged (128 registers).  1.5-2.5 % faster than the round-3 form with scalar-loaded
// tables (HX = 0, one workgroup per task) -- the tables were not what held it at ~5.8
// cycles per VALU instruction.
// HX bits: 1 half exchange buffer (persistent), 2 LDS tables, 4 just-in-time table reads,
// 8 the merged middle residue pair (res_mid)
template <int M, int E = 32, int HX = 0>
__global__ __launch_bounds__(M * 64 / E, HX ? 4 : ((M == 256 && E == 32) ? 2 : (E <= 32 ? 4 : 1))) void enc16_kernel(Enc16 p) {
    constexpr int WAVES = M / E, R = M / E;
    constexpr bool LDS_TAB = M == 256 || (HX & 2);
    constexpr bool JIT = (HX & 4) != 0;
    constexpr bool MID = (HX & 8) != 0;  // the merged middle pair (res_mid)
    static_assert(!HX || E == 32, "HX: waves of 32 elements");
    constexpr int GT = WAVES * (E - 1) * kTabW;
    __shared__ uint32_t xch[HX ? M / 2 : M][64];
    __shared__ uint32_t tabs[LDS_TAB ? 2 * GT + (2 * (R - 1) + (MID ? 1 : 0)) * kTabW : 1];
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    uint32_t* gI = tabs;
    uint32_t* gF = tabs + GT;
    uint32_t* rtab = tabs + 2 * GT;
    if constexpr (LDS_TAB) {
        stage_grp<WAVES, E, false>(gI, p.tw, M - 1);
        stage_grp<WAVES, E, true>(gF, p.tw, 0);
        stage_res<R, E, WAVES * 64>(rtab, p.tw, M - 1);
        if constexpr (MID)
            if (p.mid && threadIdx.x < (uint32_t)kTabW) rtab[2 * (R - 1) * kTabW + threadIdx.x] = p.mid->w[tab_word((int)threadIdx.x)];
    }
    const uint32_t es = (uint32_t)p.cs.elem_stride, k = p.cs.k;
    const uint32_t oo = (uint32_t)p.cs.out_offset;
    const uint32_t tasks = p.cs.count * p.chunks;
    auto run = [&](uint32_t task) {
        const uint32_t q = task / p.chunks, chunk = task - q * p.chunks;
        const Lane ln = lane_of(chunk, p.cs.S);
        const uint64_t rel = cw_rel(p.cs, q);
        const auto in = rsrc(p.cs.base + rel);
        uint32_t l[E], h[E];
        sfor<E>([&](auto I) {
            constexpr int i = decltype(I)::value;
            const uint32_t e = E * w + i;
            const uint32_t so = e < k ? e * es : kOob16;
            l[i] = ld(in, ln.lo, so);
            h[i] = ld(in, ln.lo + 32, so);
        });
        if constexpr (HX != 0) {
            __syncthreads();  // tables staged (first task)
            if constexpr (LDS_TAB) grp_xform<E, false, JIT>(l, h, gI + w * (E - 1) * kTabW);
            else grp_xform_g<E, false>(l, h, p.tw, (int)(E * w), M - 1);
            xch_plane_half<E, R, true>(l, xch, w, lane);
            xch_plane_half<E, R, true>(h, xch, w, lane);
            if constexpr (LDS_TAB) {
                res_xform<E, R, false, MID, JIT, true>(l, h, rtab);
                if constexpr (MID)
                    if (p.mid) res_mid_v<E, R, true, JIT>(l, h, rtab + 2 * (R - 1) * kTabW);
                res_xform<E, R, true, MID, JIT, true>(l, h, rtab);
            } else {
                res_xform_g<E, R, false, false, true>(l, h, p.tw, M - 1);
                res_xform_g<E, R, true, false, true>(l, h, p.tw, 0);
            }
            xch_plane_half<E, R, false>(l, xch, w, lane);
            xch_plane_half<E, R, false>(h, xch, w, lane);
            if constexpr (LDS_TAB) grp_xform<E, true, JIT>(l, h, gF + w * (E - 1) * kTabW);
            else grp_xform_g<E, true>(l, h, p.tw, (int)(E * w), 0);
        } else {
        if constexpr (LDS_TAB) {
            __syncthreads();  // tables staged (first task)
            grp_xform<E, false>(l, h, gI + w * (E - 1) * kTabW);
        } else {
            grp_xform_g<E, false>(l, h, p.tw, (int)(E * w), M - 1);
        }
        xch_plane<E, R, true>(l, xch, w, lane);
        xch_plane<E, R, true>(h, xch, w, lane);
        if constexpr (LDS_TAB) {
            res_xform<E, R, false>(l, h, rtab);
            res_mid<E, R>(l, h, p.mid);
            res_xform<E, R, true>(l, h, rtab);
        } else if constexpr (E == 64) {  // m = 512, 256 registers: the merged middle pair
            res_xform_g<E, R, false, true>(l, h, p.tw, M - 1);
            res_mid<E, R>(l, h, p.mid);
            res_xform_g<E, R, true, true>(l, h, p.tw, 0);
        } else {  // m = 512, 16 waves: not merged (its 128-register form spills more with it: c5 0.58 -> 0.70 ms)
            res_xform_g<E, R, false>(l, h, p.tw, M - 1);
            res_xform_g<E, R, true>(l, h, p.tw, 0);
        }
        xch_plane<E, R, false>(l, xch, w, lane);
        xch_plane<E, R, false>(h, xch, w, lane);
        if constexpr (LDS_TAB) grp_xform<E, true>(l, h, gF + w * (E - 1) * kTabW);
        else grp_xform_g<E, true>(l, h, p.tw, (int)(E * w), 0);
        }
        const auto out = rsrc(p.cs.out_base + rel);
        sfor<E>([&](auto I) {
            constexpr int i = decltype(I)::value;
            const uint32_t e = E * w + i;
            const uint32_t so = e < k ? oo + e * es : kOob16;
            st(out, l[i], ln.lo, so);
            st(out, h[i], ln.lo + 32, so);
        });
    };
    if constexpr (LDS_TAB) {
        for (uint32_t task = blockIdx.x; task < tasks; task += gridDim.x) run(task);
    } else {
        run(blockIdx.x);  // grid = tasks
    }
}

// Half-wave form of the m = 256 encoder (round 4): one task per (codeword, 256-byte
// chunk), so each lane-half (32 lanes x 4 symbols = 256 bytes) holds ONE element's
// chunk and every register two elements: half g = 2 w + (lane >> 5) of wave w.
//   group layout   (half g: elements 16 g .. 16 g + 15):  layers d = 1..8, each half
//                  reading its own twiddle tables (per-lane LDS address: one address
//                  per 16-lane LDS group, a broadcast)
//   residue layout (half g: elements g + 16 j, j < 16):  layers d = 16..128, tables
//                  shared by all lanes
// State is 32 registers per lane and the LDS 73 KiB (one plane of a [256][32]
// exchange buffer + the tables), so TWO 8-wave workgroups share a CU: one's loads and
// stores overlap the other's butterflies (the 512-byte-chunk forms hold 128 KiB of
// state per task and run one workgroup per CU, their memory phases exposed).
template <int E>
__device__ __forceinline__ void xch_halfwave(uint32_t (&v)[E], uint32_t (*xch)[32], uint32_t g, uint32_t l32, bool to_res) {
    sfor<E>([&](auto I) {
        constexpr int i = decltype(I)::value;
        xch[to_res ? E * g + i : g + E * i][l32] = v[i];
    });
    __syncthreads();
    sfor<E>([&](auto I) {
        constexpr int i = decltype(I)::value;
        v[i] = xch[to_res ? g + E * i : E * g + i][l32];
    });
    __syncthreads();
}

// The group <-> residue exchange of enc16h_body through an [M][XL] buffer: XL = 32 moves
// a whole half per pass (xch_halfwave), XL = 8 a quarter of its lanes per pass (four
// passes, a quarter of the LDS).
template <int E, int XL>
__device__ __forceinline__ void xch_part(uint32_t (&v)[E], uint32_t (*xch)[XL], uint32_t g, uint32_t l32, bool to_res) {
    const uint32_t ls = l32 % XL, sub = l32 / XL;
    sfor<32 / XL>([&](auto Pc) {
        constexpr uint32_t pp = decltype(Pc)::value;
        if (sub == pp)
            sfor<E>([&](auto I) {
                constexpr int i = decltype(I)::value;
                xch[to_res ? E * g + i : g + E * i][ls] = v[i];
            });
        __syncthreads();
        if (sub == pp)
            sfor<E>([&](auto I) {
                constexpr int i = decltype(I)::value;
                v[i] = xch[to_res ? g + E * i : E * g + i][ls];
            });
        __syncthreads();
    });
}

// PF: the next task's points are loaded while the current one transforms
// XL: lanes per exchange pass (32: production, two workgroups per CU; 8: the 49 KiB form,
// enc16h3_kernel, three workgroups per CU at 80 registers)
// PIPE (production since round 6; PIPE = false is diagnostic form 22): twiddle tables read
// one block ahead (grp_xform_pipe / res_xform_pipe) instead of just in time
// SH (round 6): 0 plain, 1 / 2 the multi-GPU all-to-all's row pass with side output /
// column pass with blocked inputs (CodewordSet::side / blk)
template <bool JIT, bool PF, int XL, bool PIPE = false, int SH = 0>
__device__ __forceinline__ void enc16h_body(const Enc16& p) {
    constexpr int M = 256, E = 16, G = 16, R = 16, THREADS = 512;
    constexpr int GT = G * (E - 1) * kTabW;
    __shared__ uint32_t xch[M][XL];
    __shared__ uint32_t tabs[2 * GT + 2 * (R - 1) * kTabW];
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint32_t hh = lane >> 5, l32 = lane & 31u, g = 2u * w + hh;
    uint32_t* gI = tabs;
    uint32_t* gF = tabs + GT;
    uint32_t* rtab = tabs + 2 * GT;
    stage_grp<G, E, false, THREADS>(gI, p.tw, M - 1);
    stage_grp<G, E, true, THREADS>(gF, p.tw, 0);
    stage_res<R, E, THREADS>(rtab, p.tw, M - 1);
    __syncthreads();
    const uint32_t es = (uint32_t)p.cs.elem_stride, k = p.cs.k, S = p.cs.S;
    const uint32_t oo = (uint32_t)p.cs.out_offset;
    const uint32_t tasks = p.cs.count * p.chunks;
    const uint32_t lim = k > E * g ? k - E * g : 0u;  // registers i < lim hold data / parity
    const uint32_t hoff = hh * (uint32_t)E * es;     // the half's first element, beyond the wave's
    const uint32_t* tI = gI + g * (E - 1) * kTabW;
    const uint32_t* tF = gF + g * (E - 1) * kTabW;
    auto lane_off = [&](uint32_t task) -> uint32_t {
        const uint32_t chunk = task - (task / p.chunks) * p.chunks;
        const uint32_t off = (chunk * 4u + (l32 >> 3)) * 64u + (l32 & 7u) * 4u;
        return off < S ? off + hoff : kOob16;
    };
    // all-to-all, SH = 1 (row pass): the cells of this wave -- data c = e, parity
    // c = k + e -- also go to the send block of the GPU owning their column block
    // (CodewordSet::side; a wave's 2E cells lie in one block: shard_fused_ok)
    auto side_store = [&](uint32_t qq, uint32_t lo, uint32_t lm, const uint32_t (&l)[E], const uint32_t (&h)[E],
                          uint32_t cbase) {
        const uint32_t c0 = cbase + 2u * E * w;  // the wave's first cell
        const uint32_t owner = c0 / p.cs.side_cols;
        if (owner == p.cs.side_self) return;  // (wave-uniform) its own block stays in the square
        const auto sr = rsrc(p.cs.side + (uint64_t)owner * p.cs.side_blk + (uint64_t)qq * p.cs.side_cols * S);
        const uint32_t vs = lo == kOob16 ? kOob16 : lo - hoff + hh * (uint32_t)E * S;
        const uint32_t cb = (c0 - owner * p.cs.side_cols) * S;
        sfor<E>([&](auto I) {
            constexpr int i = decltype(I)::value;
            const uint32_t v = (uint32_t)i < lm ? vs : kOob16;
            const uint32_t so = 2u * E * w + i < k ? cb + (uint32_t)i * S : 0u;
            st(sr, l[i], v, so);
            st(sr, h[i], v + 32u, so);
        });
    };
    auto load_task = [&](uint32_t task, uint32_t (&l)[E], uint32_t (&h)[E]) {
        const uint32_t lo = lane_off(task);
        const uint32_t qq = task / p.chunks;
        auto in = rsrc(p.cs.base + cw_rel(p.cs, qq));
        uint32_t vb = lo, eb = 0u, stv = es;  // symbol e at voffset vb, soffset (e - eb) * stv
        if constexpr (SH == 2) {  // all-to-all column pass: another GPU's rows, read in place
            const uint32_t hb = (2u * E * w) / p.cs.blk_rows;  // (wave-uniform) row block
            if (hb != p.cs.blk_self) {
                in = rsrc(p.cs.blk + (uint64_t)hb * p.cs.blk_size + (uint64_t)qq * S);
                vb = lo == kOob16 ? kOob16 : lo - hoff + hh * (uint32_t)E * p.cs.blk_pitch;
                eb = hb * p.cs.blk_rows;
                stv = p.cs.blk_pitch;
            }
        }
        sfor<E>([&](auto I) {
            constexpr int i = decltype(I)::value;
            const uint32_t v = (uint32_t)i < lim ? vb : kOob16;
            // (0 for padding: an offset past the half would wrap kOob16 + so)
            const uint32_t so = 2u * E * w + i < k ? (2u * E * w + i - eb) * stv : 0u;
            l[i] = ld(in, v, so);
            h[i] = ld(in, v + 32u, so);
        });
        if constexpr (SH == 1) side_store(qq, lo, lim, l, h, 0u);
    };
    uint32_t nl[E], nh[E];
    if constexpr (PF)
        if (blockIdx.x < tasks) load_task(blockIdx.x, nl, nh);
    for (uint32_t task = blockIdx.x; task < tasks; task += gridDim.x) {
        const uint32_t q = task / p.chunks;
        const uint32_t lo = lane_off(task);
        const uint64_t rel = cw_rel(p.cs, q);
        uint32_t l[E], h[E];
        if constexpr (PF) {
            sfor<E>([&](auto I) {
                l[decltype(I)::value] = nl[decltype(I)::value];
                h[decltype(I)::value] = nh[decltype(I)::value];
            });
            if (task + gridDim.x < tasks) load_task(task + gridDim.x, nl, nh);
        } else {
            load_task(task, l, h);
        }
        if constexpr (PIPE) grp_xform_pipe<E, false>(l, h, tI);
        else grp_xform<E, false, JIT>(l, h, tI);
        xch_part<E, XL>(l, xch, g, l32, true);
        xch_part<E, XL>(h, xch, g, l32, true);
        if constexpr (PIPE) res_xform_pipe<R, false>(l, h, rtab);
        else res_xform<E, R, false, true, JIT>(l, h, rtab);
        res_mid<E, R>(l, h, p.mid);
        if constexpr (PIPE) res_xform_pipe<R, true>(l, h, rtab);
        else res_xform<E, R, true, true, JIT>(l, h, rtab);
        xch_part<E, XL>(l, xch, g, l32, false);
        xch_part<E, XL>(h, xch, g, l32, false);
        if constexpr (PIPE) grp_xform_pipe<E, true>(l, h, tF);
        else grp_xform<E, true, JIT>(l, h, tF);
        const auto out = rsrc(p.cs.out_base + rel);
        // the store offsets are recomputed here from opaque copies (the compiler would
        // otherwise keep the load phase's 16 per-lane offsets alive across the transform)
        uint32_t slo = lo, slim = lim;
#ifndef RSM_ENC16_HOISTED_OFFSETS  // (diagnostic A/B builds: the round-5 hoisted offsets)
        asm volatile("" : "+v"(slo), "+v"(slim));
#endif
        sfor<E>([&](auto I) {
            constexpr int i = decltype(I)::value;
            const uint32_t v = (uint32_t)i < slim ? slo : kOob16;
            const uint32_t so = oo + (2u * E * w + i < k ? (2u * E * w + i) * es : 0u);
            st(out, l[i], v, so);
            st(out, h[i], v + 32u, so);
        });
        if constexpr (SH == 1) side_store(q, slo, slim, l, h, k);  // parity cells c = k + e
    }
}

template <bool JIT, bool PF = false, bool PIPE = false, int SH = 0>
__global__ __launch_bounds__(512, 4) void enc16h_kernel(Enc16 p) {
    enc16h_body<JIT, PF, 32, PIPE, SH>(p);
}
// three workgroups per CU: 6 waves per SIMD (80 registers), 49 KiB of LDS each
__global__ __launch_bounds__(512, 6) void enc16h3_kernel(Enc16 p) {
    enc16h_body<true, false, 8>(p);
}

// Half-wave form of the m = 512 encoder (round 4): one task per (codeword, 256-byte
// chunk), 16 waves, half g = 2 w + (lane >> 5) holding elements 16 g .. 16 g + 15 in
// its registers (32 state registers, against 64 for 512-byte chunks):
//   layers d = 1..8   in registers, per-half tables (as enc16h_kernel);
//   layer  d = 16     joins the two halves of a wave: v_permlane32_swap of the register
//                     pairs (i, i + 1) puts elements 32 w + i + hh and 32 w + 16 + i + hh
//                     in one lane each, and the wave's one table serves both halves;
//   layers d = 32..256 in the residue layout (half g: elements g + 32 j, j < 16),
//                     through a [512][32] exchange buffer (one plane at a time).
__device__ __forceinline__ void swap_halves(uint32_t& a, uint32_t& b) {
    const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    a = r[0];
    b = r[1];
}
// element of register r in the swapped group arrangement (after the d = 16 swap)
__device__ __forceinline__ uint32_t swapped_elem(uint32_t w, int r, uint32_t hh) {
    return 32u * w + ((r & 1) ? 16u : 0u) + (uint32_t)(r & ~1) + hh;
}

// PF: the next task's points are loaded while the current one transforms (32 more registers)
// PIPE (production since round 6; PIPE = false is diagnostic form 22): twiddle tables
// read one block ahead
template <bool JIT, bool PF = false, bool PIPE = false, int SH = 0>
__global__ __launch_bounds__(1024, 4) void enc16h512_kernel(Enc16 p) {
    constexpr int M = 512, E = 16, G = 32, R = 16, THREADS = 1024;
    constexpr int GT = G * (E - 1) * kTabW, WT = 16 * kTabW, RT = 2 * (R - 1) * kTabW;
    __shared__ uint32_t xch[M][32];
    __shared__ uint32_t tabs[2 * GT + 2 * WT + RT];
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint32_t hh = lane >> 5, l32 = lane & 31u, g = 2u * w + hh;
    uint32_t* gI = tabs;
    uint32_t* gF = tabs + GT;
    uint32_t* wI = tabs + 2 * GT;
    uint32_t* wF = wI + WT;
    uint32_t* rtab = wF + WT;
    stage_grp<G, E, false, THREADS>(gI, p.tw, M - 1);
    stage_grp<G, E, true, THREADS>(gF, p.tw, 0);
    {  // the d = 16 layer's table of every wave: IFFT SKEW[m - 1 + 32 w + 16], FFT SKEW[32 w + 15]
        uint32_t tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        if (tid < 2u * WT) {
            const bool fft = tid >= (uint32_t)WT;
            const uint32_t n = fft ? tid - WT : tid, ww = n / kTabW, j = n - ww * kTabW;
            const uint32_t idx = fft ? 32u * ww + 15u : M - 1 + 32u * ww + 16u;
            (fft ? wF : wI)[n] = p.tw[idx].w[tab_word((int)j)];
        }
    }
    stage_res<R, 32, THREADS>(rtab, p.tw, M - 1);
    __syncthreads();
    const uint32_t es = (uint32_t)p.cs.elem_stride, k = p.cs.k, S = p.cs.S;
    const uint32_t oo = (uint32_t)p.cs.out_offset;
    const uint32_t tasks = p.cs.count * p.chunks;
    const uint32_t lim = k > E * g ? k - E * g : 0u;  // registers i < lim hold data / parity
    const uint32_t hoff = hh * (uint32_t)E * es;
    const uint32_t* tI = gI + g * (E - 1) * kTabW;
    const uint32_t* tF = gF + g * (E - 1) * kTabW;
    auto lane_off = [&](uint32_t task) -> uint32_t {
        const uint32_t chunk = task - (task / p.chunks) * p.chunks;
        const uint32_t off = (chunk * 4u + (l32 >> 3)) * 64u + (l32 & 7u) * 4u;
        return off < S ? off + hoff : kOob16;
    };
    // all-to-all, SH = 1 (row pass): the cells of this wave -- data c = e, parity
    // c = k + e -- also go to the send block of the GPU owning their column block
    // (CodewordSet::side; a wave's 2E cells lie in one block: shard_fused_ok)
    auto side_store = [&](uint32_t qq, uint32_t lo, uint32_t lm, const uint32_t (&l)[E], const uint32_t (&h)[E],
                          uint32_t cbase) {
        const uint32_t c0 = cbase + 2u * E * w;  // the wave's first cell
        const uint32_t owner = c0 / p.cs.side_cols;
        if (owner == p.cs.side_self) return;  // (wave-uniform) its own block stays in the square
        const auto sr = rsrc(p.cs.side + (uint64_t)owner * p.cs.side_blk + (uint64_t)qq * p.cs.side_cols * S);
        const uint32_t vs = lo == kOob16 ? kOob16 : lo - hoff + hh * (uint32_t)E * S;
        const uint32_t cb = (c0 - owner * p.cs.side_cols) * S;
        sfor<E>([&](auto I) {
            constexpr int i = decltype(I)::value;
            const uint32_t v = (uint32_t)i < lm ? vs : kOob16;
            const uint32_t so = 2u * E * w + i < k ? cb + (uint32_t)i * S : 0u;
            st(sr, l[i], v, so);
            st(sr, h[i], v + 32u, so);
        });
    };
    auto load_task = [&](uint32_t task, uint32_t (&l)[E], uint32_t (&h)[E]) {
        const uint32_t lo = lane_off(task);
        const uint32_t qq = task / p.chunks;
        auto in = rsrc(p.cs.base + cw_rel(p.cs, qq));
        uint32_t vb = lo, eb = 0u, stv = es;  // symbol e at voffset vb, soffset (e - eb) * stv
        if constexpr (SH == 2) {  // all-to-all column pass: another GPU's rows, read in place
            const uint32_t hb = (2u * E * w) / p.cs.blk_rows;  // (wave-uniform) row block
            if (hb != p.cs.blk_self) {
                in = rsrc(p.cs.blk + (uint64_t)hb * p.cs.blk_size + (uint64_t)qq * S);
                vb = lo == kOob16 ? kOob16 : lo - hoff + hh * (uint32_t)E * p.cs.blk_pitch;
                eb = hb * p.cs.blk_rows;
                stv = p.cs.blk_pitch;
            }
        }
        sfor<E>([&](auto I) {
            constexpr int i = decltype(I)::value;
            const uint32_t v = (uint32_t)i < lim ? vb : kOob16;
            // (0 for padding: an offset past the half would wrap kOob16 + so)
            const uint32_t so = 2u * E * w + i < k ? (2u * E * w + i - eb) * stv : 0u;
            l[i] = ld(in, v, so);
            h[i] = ld(in, v + 32u, so);
        });
        if constexpr (SH == 1) side_store(qq, lo, lim, l, h, 0u);
    };
    uint32_t nl[E], nh[E];
    if constexpr (PF)
        if (blockIdx.x < tasks) load_task(blockIdx.x, nl, nh);
    for (uint32_t task = blockIdx.x; task < tasks; task += gridDim.x) {
        const uint32_t q = task / p.chunks;
        const uint32_t lo = lane_off(task);
        const uint64_t rel = cw_rel(p.cs, q);
        uint32_t l[E], h[E];
        if constexpr (PF) {
            sfor<E>([&](auto I) {
                l[decltype(I)::value] = nl[decltype(I)::value];
                h[decltype(I)::value] = nh[decltype(I)::value];
            });
            if (task + gridDim.x < tasks) load_task(task + gridDim.x, nl, nh);
        } else {
            load_task(task, l, h);
        }
        if constexpr (PIPE) grp_xform_pipe<E, false>(l, h, tI);
        else grp_xform<E, false, JIT>(l, h, tI);
        {  // d = 16
            sfor<E / 2>([&](auto P) {
                constexpr int i = 2 * decltype(P)::value;
                swap_halves(l[i], l[i + 1]);
                swap_halves(h[i], h[i + 1]);
            });
            uint32_t c[kTabW];
            if constexpr (JIT) tab_load_jit(wI + w * kTabW, c);
            else tab_load(wI + w * kTabW, c);
            sfor<E / 2>([&](auto P) {
                constexpr int i = 2 * decltype(P)::value;
                ifft2v(l[i], h[i], l[i + 1], h[i + 1], c);
            });
        }
        auto to_res = [&](uint32_t (&v)[E]) {
            sfor<E>([&](auto I) {
                constexpr int r = decltype(I)::value;
                xch[swapped_elem(w, r, hh)][l32] = v[r];
            });
            __syncthreads();
            sfor<R>([&](auto J) {
                constexpr int j = decltype(J)::value;
                v[j] = xch[g + 32u * j][l32];
            });
            __syncthreads();
        };
        auto to_grp = [&](uint32_t (&v)[E]) {
            sfor<R>([&](auto J) {
                constexpr int j = decltype(J)::value;
                xch[g + 32u * j][l32] = v[j];
            });
            __syncthreads();
            sfor<E>([&](auto I) {
                constexpr int r = decltype(I)::value;
                v[r] = xch[swapped_elem(w, r, hh)][l32];
            });
            __syncthreads();
        };
        to_res(l);
        to_res(h);
        if constexpr (PIPE) res_xform_pipe<R, false>(l, h, rtab);
        else res_xform<R, R, false, true, JIT>(l, h, rtab);
        res_mid<R, R>(l, h, p.mid);
        if constexpr (PIPE) res_xform_pipe<R, true>(l, h, rtab);
        else res_xform<R, R, true, true, JIT>(l, h, rtab);
        to_grp(l);
        to_grp(h);
        {  // d = 16, then back to the plain group arrangement
            uint32_t c[kTabW];
            if constexpr (JIT) tab_load_jit(wF + w * kTabW, c);
            else tab_load(wF + w * kTabW, c);
            sfor<E / 2>([&](auto P) {
                constexpr int i = 2 * decltype(P)::value;
                fft2v(l[i], h[i], l[i + 1], h[i + 1], c);
            });
            sfor<E / 2>([&](auto P) {
                constexpr int i = 2 * decltype(P)::value;
                swap_halves(l[i], l[i + 1]);
                swap_halves(h[i], h[i + 1]);
            });
        }
        if constexpr (PIPE) grp_xform_pipe<E, true>(l, h, tF);
        else grp_xform<E, true, JIT>(l, h, tF);
        const auto out = rsrc(p.cs.out_base + rel);
        // the store offsets are recomputed here from opaque copies (the compiler would
        // otherwise keep the load phase's 16 per-lane offsets alive across the transform)
        uint32_t slo = lo, slim = lim;
#ifndef RSM_ENC16_HOISTED_OFFSETS  // (diagnostic A/B builds: the round-5 hoisted offsets)
        asm volatile("" : "+v"(slo), "+v"(slim));
#endif
        sfor<E>([&](auto I) {
            constexpr int i = decltype(I)::value;
            const uint32_t v = (uint32_t)i < slim ? slo : kOob16;
            const uint32_t so = oo + (2u * E * w + i < k ? (2u * E * w + i) * es : 0u);
            st(out, l[i], v, so);
            st(out, h[i], v + 32u, so);
        });
        if constexpr (SH == 1) side_store(q, slo, slim, l, h, k);  // parity cells c = k + e
    }
}

// ---------------------------------------------------------------------------
// Decoder
// ---------------------------------------------------------------------------
struct Dec16 {
    DecodeSet ds;
    Res r;
    const uint16_t* logwalsh;
    uint16_t* errs;     // [count][n]
    uint8_t* scratch;   // [count][2][n][S] (the five-pass form)
    uint32_t q0, count, chunks;
    const PermTab16* tw;  // skewperm (the single-pass form)
    uint32_t diag;        // diagnostic builds: dec16h_kernel A/B bits (rsm_diag_set_dec16_mode), else 0
};

__device__ __forceinline__ uint32_t addm(uint32_t a, uint32_t b) {
    uint32_t s = a + b;
    return (s + (s >> 16)) & kMod16;
}
__device__ __forceinline__ uint32_t subm(uint32_t a, uint32_t b) {
    uint32_t d = a - b;
    return (d + (d >> 16)) & kMod16;
}

// cell of element e (e < 2k: data e < k, parity k <= e < 2k) of listed vector q
__device__ __forceinline__ uint64_t cell_of(const DecodeSet& ds, uint32_t q, uint32_t e) {
    const uint64_t W = 2ull * ds.k;
    const uint64_t vec = ds.indices[q];
    return ds.axis == 0 ? vec * W + e : (uint64_t)e * W + vec;
}

// Error locator of one codeword (klauspost reconstruct, SURVEY A.5: FWHT of the
// erasure indicator over all 65536 entries, times LogWalsh, FWHT again; err[0..N)),
// computed on N = 2M points.  The indicator is zero past N, so the first 65536-point
// FWHT is its N-point FWHT repeated 65536 / N times (the layers d >= N add zeros:
// a + 0, a - 0), and outputs j < N of the second only see i mod N (popcount(i & j) =
// popcount((i mod N) & j)): err = FWHT_N(FWHT_N(ind) * fold_N) with fold_N[r] =
// sum_q LogWalsh[qN + r] (host table, gf16.hpp kLwFoldOff).  The same residues mod
// 65535 as the full transforms; a result of 0 may come out as 65535 (or back), which
// every consumer reads alike (perm[65535] == perm[0]: exp(65535) = exp(0)).
// 2 x log2(N) layers of N / 2 butterflies instead of 2 x 16 x 32768.
template <int M>
__global__ __launch_bounds__(M) void errloc16_kernel(Dec16 p) {
    constexpr int N = 2 * M;
    __shared__ uint32_t err[N];
    const uint32_t q = blockIdx.x;
    const uint32_t k = p.ds.k;
    for (uint32_t i = threadIdx.x; i < (uint32_t)N; i += M) {
        uint32_t v = 0;
        if (i < k) v = p.ds.presence[cell_of(p.ds, p.q0 + q, k + i)] ? 0u : 1u;
        else if (i < (uint32_t)M) v = 1u;
        else if (i < (uint32_t)M + k) v = p.ds.presence[cell_of(p.ds, p.q0 + q, i - M)] ? 0u : 1u;
        err[i] = v;
    }
    __syncthreads();
    const uint16_t* fold = p.logwalsh + kLwFoldOff + (N - 512);
#pragma unroll 1
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
        for (uint32_t d = 1; d < (uint32_t)N; d <<= 1) {
            const uint32_t b = threadIdx.x;  // one butterfly per thread
            const uint32_t i = (b / d) * 2 * d + (b % d);
            const uint32_t a = err[i], c = err[i + d];
            err[i] = addm(a, c);
            err[i + d] = subm(a, c);
            __syncthreads();
        }
        if (pass == 0) {
            for (uint32_t i = threadIdx.x; i < (uint32_t)N; i += M) err[i] = (err[i] * fold[i]) % kMod16;
            __syncthreads();
        }
    }
    for (uint32_t i = threadIdx.x; i < (uint32_t)N; i += M) p.errs[(uint64_t)q * N + i] = (uint16_t)err[i];
}

__device__ __forceinline__ uint32_t err_of(const Dec16& p, uint32_t q, uint32_t i, uint32_t n) {
    return __builtin_amdgcn_readfirstlane((uint32_t)p.errs[(uint64_t)q * n + i]);
}

template <int M>
__global__ __launch_bounds__(256) void dec16_p1(Dec16 p) {  // group: scale + IFFT low
    constexpr int N = 2 * M;
    const TaskIdx t = task_of(p.count, p.chunks, N / 16);
    if (!t.valid) return;
    const Lane ln = lane_of(t.chunk, p.ds.S);
    const uint32_t k = p.ds.k, S = p.ds.S;
    const auto sq = rsrc(p.ds.base);
    const auto wk = rsrc(p.scratch + (uint64_t)t.q * 2 * N * S);
    uint32_t l[16], h[16];
    sfor<16>([&](auto E) {
        constexpr int i = decltype(E)::value;
        const uint32_t e = 16 * t.g + i;
        uint32_t src = 0xFFFFFFFFu;  // share element feeding work slot e
        if (e < k) src = k + e;                                 // recovery (parity)
        else if (e >= (uint32_t)M && e < (uint32_t)M + k) src = e - M;  // original data
        bool have = false;
        uint32_t so = kOob16;
        if (src != 0xFFFFFFFFu) {
            const uint64_t cell = cell_of(p.ds, p.q0 + t.q, src);
            have = p.ds.presence[cell] != 0;
            if (have) so = (uint32_t)(cell * S);
        }
        have = __builtin_amdgcn_readfirstlane(have ? 1u : 0u) != 0;
        l[i] = ld(sq, ln.lo, so);
        h[i] = ld(sq, ln.lo + 32, so);
        if (have) mul16(l[i], h[i], p.r.perm[err_of(p, t.q, e, N)]);
    });
    group_ifft(l, h, t.g, -1, p.r);
    sfor<16>([&](auto E) {
        constexpr int i = decltype(E)::value;
        const uint32_t so = (16 * t.g + i) * S;
        st(wk, l[i], ln.lo, so);
        st(wk, h[i], ln.lo + 32, so);
    });
}

template <int M>
__global__ __launch_bounds__(256) void dec16_p2(Dec16 p) {  // residue: IFFT high, H(in)
    constexpr int N = 2 * M, R = N / 16;
    const TaskIdx t = task_of(p.count, p.chunks, 16);
    if (!t.valid) return;
    const Lane ln = lane_of(t.chunk, p.ds.S);
    const uint32_t S = p.ds.S;
    const auto wk = rsrc(p.scratch + (uint64_t)t.q * 2 * N * S);
    const uint32_t hoff = N * S;  // second array: H(in)
    uint32_t l[R], h[R];
    sfor<R>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t so = (t.g + 16 * j) * S;
        l[j] = ld(wk, ln.lo, so);
        h[j] = ld(wk, ln.lo + 32, so);
    });
    residue_ifft<R>(l, h, -1, p.r);
    sfor<R>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t so = (t.g + 16 * j) * S;
        st(wk, l[j], ln.lo, so);
        st(wk, h[j], ln.lo + 32, so);
        // high-bit half of the formal derivative, H(in)[j] (residue coordinate)
        uint32_t al = 0, ah = 0;
        sfor<12>([&](auto T) {
            constexpr int tb = decltype(T)::value;
            if constexpr ((1 << tb) < R && ((j >> tb) & 1) == 0 && j + (1 << tb) < R) {
                al ^= l[j + (1 << tb)];
                ah ^= h[j + (1 << tb)];
            }
        });
        st(wk, al, ln.lo, hoff + so);
        st(wk, ah, ln.lo + 32, hoff + so);
    });
}

template <int M>
__global__ __launch_bounds__(256) void dec16_p3(Dec16 p) {  // group: out = in + L(in) + H(in)
    constexpr int N = 2 * M;
    const TaskIdx t = task_of(p.count, p.chunks, N / 16);
    if (!t.valid) return;
    const Lane ln = lane_of(t.chunk, p.ds.S);
    const uint32_t S = p.ds.S;
    const auto wk = rsrc(p.scratch + (uint64_t)t.q * 2 * N * S);
    const uint32_t hoff = N * S;
    uint32_t l[16], h[16], ol[16], oh[16];
    sfor<16>([&](auto E) {
        constexpr int i = decltype(E)::value;
        const uint32_t so = (16 * t.g + i) * S;
        l[i] = ld(wk, ln.lo, so);
        h[i] = ld(wk, ln.lo + 32, so);
    });
    deriv_terms<16>(l, h, ol, oh);
    sfor<16>([&](auto E) {
        constexpr int i = decltype(E)::value;
        const uint32_t so = (16 * t.g + i) * S;
        const uint32_t hl = ld(wk, ln.lo, hoff + so), hh = ld(wk, ln.lo + 32, hoff + so);
        st(wk, x3(l[i], ol[i], hl), ln.lo, so);
        st(wk, x3(h[i], oh[i], hh), ln.lo + 32, so);
    });
}

template <int M>
__global__ __launch_bounds__(256) void dec16_p4(Dec16 p) {  // residue: FFT high
    constexpr int N = 2 * M, R = N / 16;
    const TaskIdx t = task_of(p.count, p.chunks, 16);
    if (!t.valid) return;
    const Lane ln = lane_of(t.chunk, p.ds.S);
    const uint32_t S = p.ds.S;
    const auto wk = rsrc(p.scratch + (uint64_t)t.q * 2 * N * S);
    uint32_t l[R], h[R];
    sfor<R>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t so = (t.g + 16 * j) * S;
        l[j] = ld(wk, ln.lo, so);
        h[j] = ld(wk, ln.lo + 32, so);
    });
    residue_fft<R>(l, h, p.r);
    sfor<R>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t so = (t.g + 16 * j) * S;
        st(wk, l[j], ln.lo, so);
        st(wk, h[j], ln.lo + 32, so);
    });
}

template <int M>
__global__ __launch_bounds__(256) void dec16_p5(Dec16 p) {  // group: FFT low + reveal erasures
    constexpr int N = 2 * M;
    const TaskIdx t = task_of(p.count, p.chunks, N / 16);
    if (!t.valid) return;
    const Lane ln = lane_of(t.chunk, p.ds.S);
    const uint32_t k = p.ds.k, S = p.ds.S;
    const auto sq = rsrc(p.ds.base);
    const auto wk = rsrc(p.scratch + (uint64_t)t.q * 2 * N * S);
    uint32_t l[16], h[16];
    sfor<16>([&](auto E) {
        constexpr int i = decltype(E)::value;
        const uint32_t so = (16 * t.g + i) * S;
        l[i] = ld(wk, ln.lo, so);
        h[i] = ld(wk, ln.lo + 32, so);
    });
    group_fft(l, h, t.g, p.r);
    sfor<16>([&](auto E) {
        constexpr int i = decltype(E)::value;
        const uint32_t e = 16 * t.g + i;
        uint32_t dst = 0xFFFFFFFFu;
        if (e < k) dst = k + e;
        else if (e >= (uint32_t)M && e < (uint32_t)M + k) dst = e - M;
        if (dst != 0xFFFFFFFFu) {
            const uint64_t cell = cell_of(p.ds, p.q0 + t.q, dst);
            const bool missing = __builtin_amdgcn_readfirstlane(p.ds.presence[cell] ? 0u : 1u) != 0;
            if (missing) {
                const uint32_t L = kMod16 - err_of(p, t.q, e, N);
                mul16(l[i], h[i], p.r.perm[L]);
                const uint32_t so = (uint32_t)(cell * S);
                st(sq, l[i], ln.lo, so);
                st(sq, h[i], ln.lo + 32, so);
            }
        }
    });
}


// ---------------------------------------------------------------------------
// Single-pass decoder for m = 256 (n = 512 points; 129 <= k <= 256): one workgroup
// of 16 waves per (codeword, 512-byte chunk) keeps the whole n-point transform on
// chip, as enc16_kernel<512> does for the encoder -- the work array of the five
// passes above never touches memory:
//   group layout   (wave w: elements 32 w .. 32 w + 31): scale by the error locator,
//                  IFFT layers d = 1..16;
//   residue layout (wave w: residues 2 w, 2 w + 1; elements r + 32 j, j < 16): IFFT
//                  d = 32..256; the formal derivative out = in + L(in) + H(in) (H:
//                  partners e + 2^t, t >= 5, in registers, updated in ascending j so
//                  every term reads a pre-derivative value; L: partners t < 5, read
//                  from the pre-derivative plane the waves leave in LDS); FFT d =
//                  256..32;
//   group layout   FFT d = 16..1; reveal the missing shares (times exp(-err)).
// The error locators come from errloc16_kernel (one workgroup per codeword).
// ---------------------------------------------------------------------------
// Stage the codeword's per-element multiply tables -- exp(err[e]) (scale) or
// exp(-err[e]) (reveal) -- into LDS dst[e][kTabW]: every thread loads its words at
// once, so the err -> table chain costs one round of latency for the whole codeword
// instead of one per element (a wave-uniform scalar chain per register left the
// single-pass decoders waiting most of the time).
template <int N, int THREADS>
constexpr int elem_tab_per() { return (N * kTabW + THREADS - 1) / THREADS; }
// `mid` runs between the locator loads and the dependent table gathers: loads issued
// there (the decoders' point loads) are in flight behind the locator loads, and the
// gathers wait only for the locator values (vmcnt retires in order).
struct NoMid {
    __device__ void operator()() const {}
};
template <int N, int THREADS, typename F = NoMid>
__device__ __forceinline__ void load_elem_tabs(const Dec16& p, uint32_t q, bool reveal,
                                               uint32_t (&v)[elem_tab_per<N, THREADS>()], F&& mid = F{}) {
    constexpr int W = N * kTabW, PER = elem_tab_per<N, THREADS>();
    uint32_t tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    if constexpr (std::is_same_v<std::decay_t<F>, NoMid>) {  // one chain per word
#pragma unroll
        for (int r = 0; r < PER; ++r) {
            const uint32_t n = tid + (uint32_t)r * THREADS;
            const uint32_t e = n / kTabW, j = n - e * kTabW;
            uint32_t x = 0u;
            if (n < (uint32_t)W) {
                const uint32_t L = p.errs[(uint64_t)q * N + e];
                x = p.r.perm[reveal ? kMod16 - L : L].w[tab_word((int)j)];
            }
            v[r] = x;
        }
        return;
    }
    uint32_t L[PER];
#pragma unroll
    for (int r = 0; r < PER; ++r) {
        const uint32_t n = tid + (uint32_t)r * THREADS;
        const uint32_t e = n / kTabW;
        L[r] = n < (uint32_t)W ? (uint32_t)p.errs[(uint64_t)q * N + e] : 0u;
    }
    mid();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int r = 0; r < PER; ++r) {
        const uint32_t n = tid + (uint32_t)r * THREADS;
        const uint32_t e = n / kTabW, j = n - e * kTabW;
        v[r] = n < (uint32_t)W ? p.r.perm[reveal ? kMod16 - L[r] : L[r]].w[tab_word((int)j)] : 0u;
    }
}
template <int N, int THREADS>
__device__ __forceinline__ void store_elem_tabs(uint32_t* dst, const uint32_t (&v)[elem_tab_per<N, THREADS>()]) {
    constexpr int W = N * kTabW, PER = elem_tab_per<N, THREADS>();
    uint32_t tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
#pragma unroll
    for (int r = 0; r < PER; ++r) {
        const uint32_t n = tid + (uint32_t)r * THREADS;
        if (n < (uint32_t)W) dst[n] = v[r];
    }
}
// Stage the codeword's per-element multiply tables -- exp(err[e]) (scale) or
// exp(-err[e]) (reveal) -- into LDS dst[e][kTabW]: every thread loads its words at
// once, so the err -> table chain costs one round of latency for the whole codeword
// instead of one per element (a wave-uniform scalar chain per register left the
// single-pass decoders waiting most of the time).
template <int N, int THREADS>
__device__ __forceinline__ void stage_elem_tabs(uint32_t* dst, const Dec16& p, uint32_t q, bool reveal) {
    uint32_t v[elem_tab_per<N, THREADS>()];
    load_elem_tabs<N, THREADS>(p, q, reveal, v);
    store_elem_tabs<N, THREADS>(dst, v);
}

// The formal derivative of one plane in the residue layout (see dec16f_kernel), in
// two passes over the element halves (the L partners e + 2^t, t < 5, share e's half):
// each pass publishes that half's pre-derivative values to LDS, then every wave
// updates its registers of that half in ascending j.
template <int E, int R>
__device__ __forceinline__ void deriv_plane(uint32_t (&v)[E], uint32_t (*xch)[64], uint32_t w, uint32_t lane) {
    // residues per wave; register ridx(s, j) = RPW j + s (IL) holds element RPW w + s + E j
    constexpr int RPW = E / R, HJ = R / 2;
    sfor<2>([&](auto Hc) {
        constexpr int hf = decltype(Hc)::value;
        sfor<RPW>([&](auto Sx) {
            sfor<HJ>([&](auto J) {
                constexpr int sx = decltype(Sx)::value, j = hf * HJ + decltype(J)::value;
                xch[(RPW * w + sx) + E * (j - hf * HJ)][lane] = v[ridx<E, R, true>(sx, j)];
            });
        });
        __syncthreads();
        sfor<RPW>([&](auto Sx) {
            constexpr int sx = decltype(Sx)::value;
            const uint32_t r = RPW * w + sx;  // residue = the element's low 5 bits
            sfor<HJ>([&](auto J) {  // ascending j: register (sx, j + 2^t) still holds the pre-derivative value
                constexpr int j = hf * HJ + decltype(J)::value;
                constexpr int i = ridx<E, R, true>(sx, j);
                uint32_t a = v[i];
                sfor<12>([&](auto T) {  // H: the element's high bits (t >= 5) = bits of j
                    constexpr int t = decltype(T)::value;
                    if constexpr ((1 << t) < R && ((j >> t) & 1) == 0) a ^= v[ridx<E, R, true>(sx, j + (1 << t))];
                });
                sfor<5>([&](auto T) {  // L: bits of the residue, from this half's plane in LDS
                    constexpr uint32_t bit = 1u << decltype(T)::value;
                    if ((r & bit) == 0u) a ^= xch[(r + bit) + E * (j - hf * HJ)][lane];
                });
                v[i] = a;
            });
        });
        __syncthreads();
    });
}

// Twiddle tables staged once per workgroup in LDS and read by uniform ds_read_b128
// (enc16_kernel<256>'s scheme; a scalar table load from L2 per butterfly block left
// the 16-wave kernels waiting, ~6.6 cycles per VALU instruction): the exchange
// buffer is half the elements (two passes per plane) so the tables fit beside it.
// ZC: the zero-copy form for Repair (DecodeSet in_base / mirror: present cells read
// from host-mapped memory and stored into the device square too, rebuilt cells written
// to both)
template <int M, bool ZC = false>
__global__ __launch_bounds__(1024, 4) void dec16f_kernel(Dec16 p) {
    constexpr int N = 2 * M, E = 32, R = N / E, WAVES = N / E;
    static_assert(WAVES == 16 && R == 16, "n = 512: 16 waves of 32 elements, residues of 16");
    constexpr int GT = WAVES * (E - 1) * kTabW;  // group tables (words)
    __shared__ uint32_t xch[N / 2][64];
    __shared__ uint32_t tabs[GT + 2 * (R - 1) * kTabW];
    // decoder skews: IFFT SKEW[-1 + b + d], FFT SKEW[b + d - 1] -- the same tables, so
    // one set serves both directions; staged once per workgroup of the persistent grid
    uint32_t* gI = tabs;
    uint32_t* gF = tabs;
    uint32_t* rtab = tabs + GT;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    stage_grp<WAVES, E, false>(gI, p.tw, -1);
    stage_res<R, E, WAVES * 64>(rtab, p.tw, -1);
    const uint32_t tasks = p.count * p.chunks;
    for (uint32_t task = blockIdx.x; task < tasks; task += gridDim.x) {
    const uint32_t q = task / p.chunks, chunk = task - q * p.chunks;
    const Lane ln = lane_of(chunk, p.ds.S);
    const uint32_t k = p.ds.k, S = p.ds.S;
    // work slot e <- share: e < k parity k + e, M <= e < M + k data e - M, else zero
    auto share_of = [&](uint32_t e) -> uint32_t {
        return e < k ? k + e : (e >= (uint32_t)M && e < (uint32_t)M + k) ? e - (uint32_t)M : 0xFFFFFFFFu;
    };
    uint32_t* etab = &xch[0][0];  // per-element tables while the exchange buffer is idle
    // presence: lane j < 32 of wave w asks for slot 32 w + j (one load per lane, a ballot);
    // issued first, the scale tables' err -> table chain beside it
    const uint32_t vec = __builtin_amdgcn_readfirstlane(p.ds.indices[p.q0 + q]);
    const uint32_t Wd = 2u * k;
    auto cell = [&](uint32_t s) -> uint32_t { return p.ds.axis == 0 ? vec * Wd + s : s * Wd + vec; };
    // this wave's half of the codeword (slots e < M: parity shares, waves w < 8; else
    // data) from its own 64-bit base, 32-bit offsets within it (narrow_fits)
    const uint32_t hfirst = w < (uint32_t)WAVES / 2 ? k : 0u, cstep = p.ds.axis == 0 ? 1u : Wd;
    const uint64_t hbase = ((uint64_t)cell(0) + (uint64_t)hfirst * cstep) * S;
    const auto sq = rsrc(p.ds.base + hbase);
    const auto si = rsrc((ZC ? p.ds.in_base : p.ds.base) + hbase);  // present cells
    const bool mirror = p.ds.mirror != nullptr;                       // rebuilt cells also written there
    const auto sm = rsrc((mirror ? p.ds.mirror : p.ds.base) + hbase);
    auto hoff = [&](uint32_t s) -> uint32_t { return (s - hfirst) * cstep * S; };
    const uint32_t my_s = lane < (uint32_t)E ? share_of(E * w + lane) : 0xFFFFFFFFu;
    const uint32_t my_p = my_s != 0xFFFFFFFFu ? (uint32_t)p.ds.presence[cell(my_s)] : 0u;
    uint32_t etv[elem_tab_per<N, 1024>()];
    uint32_t l[E], h[E];
    // device form: every real cell loaded right away (behind the presence byte and the
    // scale tables' locator loads, ahead of the ballot), the absent ones zeroed after it
    // -- the loads do not wait for the presence bytes; zero-copy: only the present
    // cells, after the ballot
    auto load_points = [&](uint32_t m) {
        sfor<E>([&](auto I) {
            constexpr int i = decltype(I)::value;
            const uint32_t src = share_of(E * w + i);
            const uint32_t so = ((m >> i) & 1u) && src != 0xFFFFFFFFu ? hoff(src) : kOob16;
            l[i] = ld(si, ln.lo, so);
            h[i] = ld(si, ln.lo + 32, so);
            if constexpr (ZC) {  // the present cell lands in the device square as well
                st(sq, l[i], ln.lo, so);
                st(sq, h[i], ln.lo + 32, so);
            }
        });
    };
    constexpr bool EAGER = !ZC && kDec16Eager;
    if constexpr (EAGER) load_elem_tabs<N, 1024>(p, q, false, etv, [&] { load_points(~0u); });
    else load_elem_tabs<N, 1024>(p, q, false, etv);
    const uint32_t have = __builtin_amdgcn_readfirstlane((uint32_t)__ballot(my_p != 0u));
    if constexpr (!EAGER) load_points(have);
    if constexpr (EAGER)
        sfor<E>([&](auto I) {
            constexpr int i = decltype(I)::value;
            const bool keep = (have >> i) & 1u;
            l[i] = keep ? l[i] : 0u;
            h[i] = keep ? h[i] : 0u;
        });
    store_elem_tabs<N, 1024>(etab, etv);
    __syncthreads();  // twiddle and scale tables staged
    sfor<E>([&](auto I) {
        constexpr int i = decltype(I)::value;
        if ((have >> i) & 1u) {
            uint32_t c[kTabW];
            tab_load_jit_at<i * kTabW * 4>(etab + E * w * kTabW, c);
            const uint32_t yl = l[i], yh = h[i];
            l[i] = 0u;
            h[i] = 0u;
            muladd16v(l[i], h[i], yl, yh, c);
        }
    });
    __syncthreads();  // the exchange buffer is free again
    grp_xform<E, false, true>(l, h, gI + w * (E - 1) * kTabW);
    xch_plane_half<E, R, true>(l, xch, w, lane);
    xch_plane_half<E, R, true>(h, xch, w, lane);
    res_xform<E, R, false, false, true, true>(l, h, rtab);
    deriv_plane<E, R>(l, xch, w, lane);
    deriv_plane<E, R>(h, xch, w, lane);
    res_xform<E, R, true, false, true, true>(l, h, rtab);
    xch_plane_half<E, R, false>(l, xch, w, lane);
    xch_plane_half<E, R, false>(h, xch, w, lane);
    uint32_t qr = q;
    asm volatile("" : "+s"(qr));
    stage_elem_tabs<N, 1024>(etab, p, qr, true);  // (the exchange's last barrier freed xch)
    grp_xform<E, true, true>(l, h, gF + w * (E - 1) * kTabW);
    __syncthreads();  // reveal tables staged
    sfor<E>([&](auto I) {
        constexpr int i = decltype(I)::value;
        const uint32_t e = E * w + i;
        const uint32_t dst = share_of(e);
        if (dst != 0xFFFFFFFFu && !((have >> i) & 1u)) {
            uint32_t c[kTabW];
            tab_load_jit_at<i * kTabW * 4>(etab + E * w * kTabW, c);
            const uint32_t yl = l[i], yh = h[i];
            l[i] = 0u;
            h[i] = 0u;
            muladd16v(l[i], h[i], yl, yh, c);
            const uint32_t so = hoff(dst);
            st(sq, l[i], ln.lo, so);
            st(sq, h[i], ln.lo + 32, so);
            if (mirror) {
                st(sm, l[i], ln.lo, so);
                st(sm, h[i], ln.lo + 32, so);
            }
        }
    });
    __syncthreads();  // the next task's scale tables reuse the exchange buffer
    }
}

// ---------------------------------------------------------------------------
// Half-wave single-pass decoder for m = 512 (n = 1024 points; 257 <= k <= 512), round
// 4: one workgroup of 16 waves per (codeword, 256-byte chunk); lane-half g = 2 w +
// (lane >> 5) of wave w holds ONE element's 256-byte chunk per register (32 lanes x 4
// symbols), so the n-point state is 64 registers per lane, as in dec16f_kernel<256>:
//   group layout   (half g: elements 32 g .. 32 g + 31): scale by exp(err), IFFT
//                  d = 1..16 (twiddle tables per half: per-lane LDS addresses, one per
//                  16-lane LDS group);
//   residue layout (half g: elements g + 32 j, j < 32): IFFT d = 32..512, the formal
//                  derivative (partners e + 2^t: t >= 5 in registers, t < 5 from the
//                  other halves through LDS, deriv_halfwave), FFT d = 512..32;
//   group layout   FFT d = 16..1; reveal the missing shares (times exp(-err)).
// No element bit is held by the registers in both layouts (group: bits 0-4, residue:
// bits 5-9), so the exchange buffer -- one plane, [1024][16] -- moves half the LANES per
// pass (lanes 0-15 of both halves, then 16-31).  One LDS pool holds in turn the
// per-element scale tables (stage_elem_tabs), the twiddle tables (the group tables, 32
// halves x 31 slots = 79 KiB: the decoder's IFFT and FFT twiddles coincide) and the
// per-element reveal tables.
// ---------------------------------------------------------------------------
// diagnostic phase stamp of the single-pass decoders (RSM_DIAG builds with a decode
// trace set): thread 0, 100 MHz clock, kDec16TraceWords per workgroup
__device__ __forceinline__ void d16_stamp(const Dec16& p, int i) {
#ifdef RSM_DIAG
    if (p.ds.trace && threadIdx.x == 0) {
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(p.ds.trace, (short)0, 0x7FFFFFFF, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32((uint32_t)__builtin_amdgcn_s_memrealtime(), r,
                                              (blockIdx.x * kDec16TraceWords + i) * 4u, 0, 0);
    }
#else
    (void)p;
    (void)i;
#endif
}

template <int E>
__device__ __forceinline__ void xch_lanesplit(uint32_t (&v)[E], uint32_t (*xch)[16], uint32_t g, uint32_t l32,
                                              bool to_res) {
    const uint32_t ls = l32 & 15u, sub = l32 >> 4;
    sfor<2>([&](auto Pc) {
        constexpr uint32_t pp = decltype(Pc)::value;
        if (sub == pp)
            sfor<E>([&](auto I) {
                constexpr int i = decltype(I)::value;
                xch[to_res ? E * g + i : g + E * i][ls] = v[i];
            });
        __syncthreads();
        if (sub == pp)
            sfor<E>([&](auto I) {
                constexpr int i = decltype(I)::value;
                v[i] = xch[to_res ? g + E * i : E * g + i][ls];
            });
        __syncthreads();
    });
}
// Formal derivative of one plane in the half-wave residue layout (element g + E j in
// register j of half g = 2 w + hh): out[e] = in[e] ^ XOR over the 0-bits t of e of
// in[e + 2^t], every term pre-derivative.  Two passes over the register halves (element
// bit 9): the partners across g (t < 5) share j, so a pass publishes only its R/2
// registers of every half to LDS x2[N/2][32]; registers are updated in ascending j, so
// the in-register partners (t >= 5, j + 2^t) are still pre-derivative.  Bits 1-4 of g
// are bits of w (wave-uniform branches), bit 0 is the lane half.
template <int E, int R>
__device__ __forceinline__ void deriv_halfwave(uint32_t (&v)[R], uint32_t (*x2)[32], uint32_t w, uint32_t g, bool hi,
                                               uint32_t l32) {
    constexpr int HJ = R / 2;
    sfor<2>([&](auto Hc) {
        constexpr int hf = decltype(Hc)::value;
        sfor<HJ>([&](auto J) {
            constexpr int j = hf * HJ + decltype(J)::value;
            x2[g + E * (j - hf * HJ)][l32] = v[j];
        });
        __syncthreads();
        sfor<HJ>([&](auto J) {
            constexpr int j = hf * HJ + decltype(J)::value;
            uint32_t a = v[j];
            sfor<12>([&](auto T) {  // t >= log2(E): bits of j
                constexpr int t = decltype(T)::value;
                if constexpr ((1 << t) < R && ((j >> t) & 1) == 0) a ^= v[j + (1 << t)];
            });
            {  // t = 0: the other lane half (g ^ 1) of this wave's register j, when this
               // half's bit is 0 -- a lane swap instead of an LDS read
                const auto sw = __builtin_amdgcn_permlane32_swap(v[j], v[j], false, false);
                a ^= hi ? 0u : sw[1];
            }
            sfor<ilog2c(E) - 1>([&](auto B) {  // t = 1..4: bit t - 1 of w
                constexpr uint32_t bit = 2u << decltype(B)::value;
                if ((w & (bit >> 1)) == 0u) a ^= x2[(g + bit) + E * (j - hf * HJ)][l32];
            });
            v[j] = a;
        });
        __syncthreads();
    });
}

template <int M, bool ZC = false>
__global__ __launch_bounds__(1024, 4) void dec16h_kernel(Dec16 p) {
    constexpr int N = 2 * M, E = 32, G = N / E, R = N / E;
    static_assert(G == 32 && R == 32, "n = 1024: 32 halves of 32 elements, residues of 32");
    constexpr int GT = G * (E - 1) * kTabW;  // group tables of one direction (words)
    constexpr int RT = 2 * (R - 1) * kTabW, ET = N * kTabW;
    __shared__ uint32_t xch[N][16];
    // the pool holds the per-element scale tables, then the twiddle tables, then the
    // per-element reveal tables
    __shared__ uint32_t pool[GT + RT > ET ? GT + RT : ET];
    uint32_t* gtab = pool;
    uint32_t* rtab = pool + GT;
    uint32_t* etab = pool;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint32_t hh = lane >> 5, l32 = lane & 31u, g = 2u * w + hh;
    const bool hi = hh != 0u;
    const uint32_t task = blockIdx.x;
    d16_stamp(p, 0);
    const uint32_t q = task / p.chunks, chunk = task - q * p.chunks;
    const uint32_t k = p.ds.k, S = p.ds.S;
    const uint32_t off = (chunk * 4u + (l32 >> 3)) * 64u + (l32 & 7u) * 4u;
    const bool lane_ok = off < S;
    auto share_of = [&](uint32_t e) -> uint32_t {
        return e < k ? k + e : (e >= (uint32_t)M && e < (uint32_t)M + k) ? e - (uint32_t)M : 0xFFFFFFFFu;
    };
    // presence: lane j of wave w asks for element 64 w + j = register j & 31 of half j >> 5
    // (issued first: the point loads wait for it; the scale tables' err -> table chain
    // runs beside it)
    const uint32_t vec = __builtin_amdgcn_readfirstlane(p.ds.indices[p.q0 + q]);
    const uint32_t Wd = 2u * k;
    auto cell = [&](uint32_t s) -> uint32_t { return p.ds.axis == 0 ? vec * Wd + s : s * Wd + vec; };
    // this wave's half of the codeword (elements < M: parity shares, waves w < 8; else
    // data) from its own 64-bit base, 32-bit offsets within it (narrow_fits)
    const uint32_t hfirst = w < 8u ? k : 0u, cstep = p.ds.axis == 0 ? 1u : Wd;
    const uint64_t hbase = ((uint64_t)cell(0) + (uint64_t)hfirst * cstep) * S;
    const auto sq = rsrc(p.ds.base + hbase);
    const auto si = rsrc((ZC ? p.ds.in_base : p.ds.base) + hbase);  // present cells
    const bool mirror = p.ds.mirror != nullptr;                       // rebuilt cells also written there
    const auto sm = rsrc((mirror ? p.ds.mirror : p.ds.base) + hbase);
    auto hoff = [&](uint32_t s) -> uint32_t { return (s - hfirst) * cstep * S; };
    const uint32_t my_s = share_of(64u * w + lane);
    const uint32_t my_p = my_s != 0xFFFFFFFFu ? (uint32_t)p.ds.presence[cell(my_s)] : 0u;
    uint32_t etv[elem_tab_per<N, 1024>()];
    uint32_t l[E], h[E];
    // Device form: every real cell's points are loaded right away, absent or not (issued
    // behind the presence byte and the scale tables' chain, before the ballot), and the
    // absent ones are zeroed once the ballot is in -- the loads no longer wait for the
    // presence bytes (a whole load latency per task; the absent cells' bytes cost HBM
    // reads, not time).  Zero-copy form: only the present cells cross PCIe, after the ballot.
    auto load_points = [&](uint32_t m0, uint32_t m1) {
        sfor<E>([&](auto I) {  // the two halves' elements of register i: E (2 w) + i, E (2 w + 1) + i
            constexpr int i = decltype(I)::value;
            const uint32_t s0 = share_of(E * 2u * w + i), s1 = share_of(E * (2u * w + 1u) + i);
            const uint32_t c0 = ((m0 >> i) & 1u) && s0 != 0xFFFFFFFFu ? hoff(s0) : kOob16;
            const uint32_t c1 = ((m1 >> i) & 1u) && s1 != 0xFFFFFFFFu ? hoff(s1) : kOob16;
            const uint32_t c = hi ? c1 : c0;
            uint32_t vo = (c == kOob16 || !lane_ok) ? kOob16 : c + off;
#ifdef RSM_DIAG
            if (p.diag & 2u) vo = kOob16;  // A/B bit 1: no point loads (wrong output)
#endif
            l[i] = ld(si, vo, 0u);
            h[i] = ld(si, vo + 32u, 0u);
            if constexpr (ZC) {  // the present cell lands in the device square as well
                st(sq, l[i], vo, 0u);
                st(sq, h[i], vo + 32u, 0u);
            }
        });
    };
    constexpr bool EAGER = !ZC && kDec16Eager;
#ifdef RSM_DIAG
    if (p.diag & 1u) {  // A/B bit 0: no scale / reveal table staging (wrong output)
        if constexpr (EAGER) load_points(~0u, ~0u);
    } else
#endif
    if constexpr (EAGER) load_elem_tabs<N, 1024>(p, q, false, etv, [&] { load_points(~0u, ~0u); });
    else load_elem_tabs<N, 1024>(p, q, false, etv);
    const uint64_t hv = __ballot(my_p != 0u);
    const uint32_t have0 = __builtin_amdgcn_readfirstlane((uint32_t)hv);
    const uint32_t have1 = __builtin_amdgcn_readfirstlane((uint32_t)(hv >> 32));
    d16_stamp(p, 1);
    if constexpr (!EAGER) load_points(have0, have1);
    if constexpr (EAGER) {  // absent points enter the transform as zero
        const uint32_t mine = hi ? have1 : have0;
        sfor<E>([&](auto I) {
            constexpr int i = decltype(I)::value;
            const bool keep = (mine >> i) & 1u;
            l[i] = keep ? l[i] : 0u;
            h[i] = keep ? h[i] : 0u;
        });
    }
#ifdef RSM_DIAG
    if (!(p.diag & 1u))
#endif
    store_elem_tabs<N, 1024>(etab, etv);
    __syncthreads();
    d16_stamp(p, 2);
    // the twiddle tables' loads go out now, beside the scale multiplies (the pool holds
    // the scale tables until every wave is past them)
    constexpr bool PF = kDec16PrefetchTw, PR = kDec16PrefetchRv;
    uint32_t gv[PF ? grp_tab_per<G, E, 1024>() : 1];
    if constexpr (PF) load_grp<G, E, false, 1024>(p.tw, -1, gv);
    sfor<E>([&](auto I) {  // scale by exp(err) (absent points are zero)
        constexpr int i = decltype(I)::value;
        if (((have0 | have1) >> i) & 1u) {
            uint32_t c[kTabW];
            tab_load_jit_at<i * kTabW * 4>(etab + E * g * kTabW, c);
            const uint32_t yl = l[i], yh = h[i];
            l[i] = 0u;
            h[i] = 0u;
            muladd16v(l[i], h[i], yl, yh, c);
        }
    });
    __syncthreads();  // every wave is past the scale tables
    // decoder skews: IFFT SKEW[-1 + b + d], FFT SKEW[b + d - 1]
    if constexpr (PF) store_grp<G, E, 1024>(gtab, gv);
    else stage_grp<G, E, false, 1024>(gtab, p.tw, -1);
    stage_res<R, E, 1024>(rtab, p.tw, -1);
    __syncthreads();  // twiddle tables staged
    d16_stamp(p, 3);
    grp_xform<E, false, true>(l, h, gtab + g * (E - 1) * kTabW);
    d16_stamp(p, 4);
    xch_lanesplit<E>(l, xch, g, l32, true);
    xch_lanesplit<E>(h, xch, g, l32, true);
    // (the decoder's FFT twiddles SKEW[b + d - 1] are its IFFT ones SKEW[-1 + b + d]: the
    // group tables stay)
    d16_stamp(p, 5);
    res_xform<E, R, false, false, true, false>(l, h, rtab);
    d16_stamp(p, 6);
    uint32_t (*x2)[32] = reinterpret_cast<uint32_t (*)[32]>(&xch[0][0]);  // [N/2][32], the same 64 KiB
    deriv_halfwave<E, R>(l, x2, w, g, hi, l32);
    deriv_halfwave<E, R>(h, x2, w, g, hi, l32);
    d16_stamp(p, 7);
    res_xform<E, R, true, false, true, false>(l, h, rtab);
    d16_stamp(p, 8);
    xch_lanesplit<E>(l, xch, g, l32, false);
    xch_lanesplit<E>(h, xch, g, l32, false);
    d16_stamp(p, 9);
    // the reveal recomputes its cell offsets (opaque codeword index: the compiler would
    // otherwise keep the load phase's 64 offsets alive across the transforms); its
    // tables' loads go out before the group FFT, their LDS stores after it
    uint32_t qr = q, wr = w;
    asm volatile("" : "+s"(qr), "+s"(wr));
    uint32_t rv[PR ? elem_tab_per<N, 1024>() : 1];
#ifdef RSM_DIAG
    if (!(p.diag & 1u))
#endif
    if constexpr (PR) load_elem_tabs<N, 1024>(p, qr, true, rv);
    grp_xform<E, true, true>(l, h, gtab + g * (E - 1) * kTabW);
    __syncthreads();  // every wave is past the twiddle tables
    d16_stamp(p, 10);
#ifdef RSM_DIAG
    if (!(p.diag & 1u))
#endif
    {
        if constexpr (PR) store_elem_tabs<N, 1024>(etab, rv);
        else stage_elem_tabs<N, 1024>(etab, p, qr, true);
    }
    __syncthreads();  // reveal tables staged
    d16_stamp(p, 11);
    sfor<E>([&](auto I) {
        constexpr int i = decltype(I)::value;
        const uint32_t e0 = E * 2u * wr + i, e1 = E * (2u * wr + 1u) + i;
        const uint32_t d0 = share_of(e0), d1 = share_of(e1);
        const bool m0 = d0 != 0xFFFFFFFFu && !((have0 >> i) & 1u), m1 = d1 != 0xFFFFFFFFu && !((have1 >> i) & 1u);
        if (m0 || m1) {
            uint32_t c[kTabW];
            tab_load_jit_at<i * kTabW * 4>(etab + E * g * kTabW, c);
            uint32_t xl = 0u, xh = 0u;
            muladd16v(xl, xh, l[i], h[i], c);
            const uint32_t c0 = m0 ? hoff(d0) : kOob16;
            const uint32_t c1 = m1 ? hoff(d1) : kOob16;
            const uint32_t cc = hi ? c1 : c0;
            const uint32_t vo = (cc == kOob16 || !lane_ok) ? kOob16 : cc + off;
            st(sq, xl, vo, 0u);
            st(sq, xh, vo + 32u, 0u);
            if (mirror) {
                st(sm, xl, vo, 0u);
                st(sm, xh, vo + 32u, 0u);
            }
        }
    });
    d16_stamp(p, 12);
}

// ---------------------------------------------------------------------------
// Generic multi-pass transforms for m = ceilPow2(k) >= 1024 (k up to 32768, the
// reference's MaxChunks: leopard.go:76-84).  The m- (encode) or n = 2m- (decode)
// point transforms no longer fit one workgroup, so they run as radix-2^b passes
// through a global work array [codeword][point][S]: a wave owns one group of
// G = 2^b points e = base + j D (j < G) of one 512-byte chunk and applies the
// layers d = D, 2D, .., D G / 2 (IFFT ascending, then -- in the top pass -- FFT
// descending), with the twiddle of (layer, block) read per butterfly (wave-uniform
// scalar loads, as the decoder's passes above).  Bit groups: 4 bits per pass from
// the bottom, the top group takes the remainder.
//   encode: pass(group 0, IFFT) reads the data shares (zero past k), ...,
//           pass(top, IFFT + FFT), ..., pass(group 0, FFT) writes parity e < k.
//   decode: errloc16g_kernel; pass(group 0, IFFT) reads the present shares scaled
//           by the error locator; IFFT passes up to the top -> work A; the formal
//           derivative as one pass per bit group (B = A + sum_g T_g(A), every
//           term from the pre-derivative A: the closed form of the reference's
//           sequential loop); FFT passes on B down to group 0, which reveals the
//           missing shares (times exp(-err)).
// ---------------------------------------------------------------------------
struct G16Pass {
    CodewordSet cs;        // encode: shares (first pass reads data, last writes parity)
    DecodeSet ds;          // decode: shares and presence
    Res r;
    const uint16_t* errs;  // decode: error locators [count][n] (log domain)
    uint16_t* errs_out;    // the same array, written by errloc16g_kernel
    const uint16_t* logwalsh;
    uint8_t* work;         // [count][2][npts][S] (decode) or [count][npts][S] (encode)
    uint64_t cw_bytes;     // bytes of one codeword's work (all arrays)
    uint64_t pitch;        // decode: bytes between consecutive cells (the share size)
    uint32_t npts, m, k, S, chunks;
    uint32_t q0, count;    // codewords [q0, q0 + count) of the set, work slot q - q0
    uint32_t D, bits;      // group stride and size (G = 2^bits <= 16)
    uint32_t nifft, nfft;  // IFFT layers (ascending from d = D), then FFT layers (descending to D)
    int ifft_off;          // encode: m - 1; decode: -1
    uint32_t src, dst;     // 0 work A; 1 work B; 2 shares (first / last pass)
    uint32_t decode;
};

__device__ __forceinline__ uint64_t g16_share(const G16Pass& p, uint32_t q, uint32_t e, bool out) {
    // byte offset of share e (encode: data e, or parity e when out) of codeword q
    const uint64_t rel = cw_rel(p.cs, q);
    return rel + (out ? p.cs.out_offset : 0ull) + (uint64_t)e * p.cs.elem_stride;
}

template <int BITS, int NI, int NF>
__global__ __launch_bounds__(256) void g16_pass_kernel(G16Pass p) {
    constexpr uint32_t G = 1u << BITS;
    const uint32_t groups = p.npts >> BITS;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    if (wv >= p.count * p.chunks * groups) return;
    const uint32_t g = wv % groups, rest = wv / groups;
    const uint32_t chunk = rest % p.chunks, qi = rest / p.chunks, q = p.q0 + qi;
    const Lane ln = lane_of(chunk, p.S);
    const uint32_t D = p.D;
    const uint32_t base = (g / D) * G * D + (g % D);
    uint8_t* const wk = p.work + (uint64_t)qi * p.cw_bytes;
    const uint64_t arr = (uint64_t)p.npts * p.S;  // decode: array B follows A
    uint32_t l[G], h[G];
    // load
    sfor<G>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t e = base + (uint32_t)j * D;
        l[j] = 0u;
        h[j] = 0u;
        if (p.src <= 1u) {
            const auto rs = rsrc(wk + (p.src ? arr : 0ull) + (uint64_t)e * p.S);
            l[j] = ld(rs, ln.lo, 0u);
            h[j] = ld(rs, ln.lo + 32, 0u);
        } else if (!p.decode) {
            if (e < p.k) {
                const auto rs = rsrc(p.cs.base + g16_share(p, q, e, false));
                l[j] = ld(rs, ln.lo, 0u);
                h[j] = ld(rs, ln.lo + 32, 0u);
            }
        } else {
            // decoder input: point e < k <- parity share k + e, m <= e < m + k <- data e - m
            uint32_t srcs = 0xFFFFFFFFu;
            if (e < p.k) srcs = p.k + e;
            else if (e >= p.m && e < p.m + p.k) srcs = e - p.m;
            if (srcs != 0xFFFFFFFFu) {
                const uint64_t cell = cell_of(p.ds, q, srcs);
                const bool have = __builtin_amdgcn_readfirstlane(p.ds.presence[cell] ? 1u : 0u) != 0;
                if (have) {
                    const auto rs = rsrc(p.ds.base + cell * p.pitch);
                    l[j] = ld(rs, ln.lo, 0u);
                    h[j] = ld(rs, ln.lo + 32, 0u);
                    const uint32_t L = __builtin_amdgcn_readfirstlane((uint32_t)p.errs[(uint64_t)qi * p.npts + e]);
                    mul16(l[j], h[j], p.r.perm[L]);
                }
            }
        }
    });
    // IFFT layers d = D 2^t (t < NI ascending), then FFT layers (t = NF-1 .. 0)
    sfor<NI>([&](auto T) {
        constexpr int t = decltype(T)::value, dj = 1 << t;
        const uint32_t d = D << t;
        sfor<G / 2>([&](auto Q) {
            constexpr int qq = decltype(Q)::value;
            constexpr int j = (qq / dj) * 2 * dj + (qq % dj);
            const uint32_t bl = (base + (uint32_t)j * D) & ~(2u * d - 1u);
            ifft2(l[j], h[j], l[j + dj], h[j + dj], skew_at(p.r, p.ifft_off + (int)(bl + d)), p.r);
        });
    });
    sfor<NF>([&](auto T) {
        constexpr int t = NF - 1 - decltype(T)::value, dj = 1 << t;
        const uint32_t d = D << t;
        sfor<G / 2>([&](auto Q) {
            constexpr int qq = decltype(Q)::value;
            constexpr int j = (qq / dj) * 2 * dj + (qq % dj);
            const uint32_t bl = (base + (uint32_t)j * D) & ~(2u * d - 1u);
            fft2(l[j], h[j], l[j + dj], h[j + dj], skew_at(p.r, (int)(bl + d) - 1), p.r);
        });
    });
    // store
    sfor<G>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t e = base + (uint32_t)j * D;
        if (p.dst <= 1u) {
            const auto rs = rsrc(wk + (p.dst ? arr : 0ull) + (uint64_t)e * p.S);
            st(rs, l[j], ln.lo, 0u);
            st(rs, h[j], ln.lo + 32, 0u);
        } else if (!p.decode) {
            if (e < p.k) {
                const auto rs = rsrc(p.cs.out_base + g16_share(p, q, e, true));
                st(rs, l[j], ln.lo, 0u);
                st(rs, h[j], ln.lo + 32, 0u);
            }
        } else {
            uint32_t dsts = 0xFFFFFFFFu;
            if (e < p.k) dsts = p.k + e;
            else if (e >= p.m && e < p.m + p.k) dsts = e - p.m;
            if (dsts != 0xFFFFFFFFu) {
                const uint64_t cell = cell_of(p.ds, q, dsts);
                const bool missing = __builtin_amdgcn_readfirstlane(p.ds.presence[cell] ? 0u : 1u) != 0;
                if (missing) {
                    const uint32_t L = kMod16 - __builtin_amdgcn_readfirstlane((uint32_t)p.errs[(uint64_t)qi * p.npts + e]);
                    mul16(l[j], h[j], p.r.perm[L]);
                    const auto rs = rsrc(p.ds.base + cell * p.pitch);
                    st(rs, l[j], ln.lo, 0u);
                    st(rs, h[j], ln.lo + 32, 0u);
                }
            }
        }
    });
}

// One bit group of the decoder's formal derivative: B[e] (^)= XOR over the group's
// bits t with bit t of e clear of A[e + 2^t]; the first group also adds A[e].
template <int BITS>
__global__ __launch_bounds__(256) void g16_deriv_kernel(G16Pass p) {
    constexpr uint32_t G = 1u << BITS;
    const uint32_t groups = p.npts >> BITS;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    if (wv >= p.count * p.chunks * groups) return;
    const uint32_t g = wv % groups, rest = wv / groups;
    const uint32_t chunk = rest % p.chunks, qi = rest / p.chunks;
    const Lane ln = lane_of(chunk, p.S);
    const uint32_t D = p.D;
    const uint32_t base = (g / D) * G * D + (g % D);
    uint8_t* const wk = p.work + (uint64_t)qi * p.cw_bytes;
    const uint64_t arr = (uint64_t)p.npts * p.S;
    const bool first = p.src != 0u;  // src = 1 marks the first group (B starts as A)
    uint32_t al[G], ah[G];
    sfor<G>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const auto rs = rsrc(wk + (uint64_t)(base + (uint32_t)j * D) * p.S);
        al[j] = ld(rs, ln.lo, 0u);
        ah[j] = ld(rs, ln.lo + 32, 0u);
    });
    sfor<G>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t e = base + (uint32_t)j * D;
        const auto rb = rsrc(wk + arr + (uint64_t)e * p.S);
        uint32_t ol = first ? al[j] : ld(rb, ln.lo, 0u);
        uint32_t oh = first ? ah[j] : ld(rb, ln.lo + 32, 0u);
        sfor<BITS>([&](auto T) {
            constexpr int t = decltype(T)::value;
            if constexpr (((j >> t) & 1) == 0) {
                ol ^= al[j + (1 << t)];
                oh ^= ah[j + (1 << t)];
            }
        });
        st(rb, ol, ln.lo, 0u);
        st(rb, oh, ln.lo + 32, 0u);
    });
}

// Error locator for any m: the m <= 512 kernel with n = npts = 2m a runtime value
// (n <= 65536; n = 65536 folds nothing: the table itself).
__global__ __launch_bounds__(1024) void errloc16g_kernel(G16Pass p) {
    __shared__ uint16_t err[65536];
    const uint32_t qi = blockIdx.x, q = p.q0 + qi;
    const uint32_t k = p.k, M = p.m, n = p.npts;
    const uint16_t* fold = n >= 65536u ? p.logwalsh : p.logwalsh + kLwFoldOff + (n - 512u);
#pragma unroll 2
    for (uint32_t i = threadIdx.x; i < n; i += 1024u) {
        uint32_t v = 0;
        if (i < k) v = p.ds.presence[cell_of(p.ds, q, k + i)] ? 0u : 1u;
        else if (i < M) v = 1u;
        else if (i < M + k) v = p.ds.presence[cell_of(p.ds, q, i - M)] ? 0u : 1u;
        err[i] = (uint16_t)v;
    }
    __syncthreads();
#pragma unroll 1
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll 1
        for (uint32_t d = 1; d < n; d <<= 1) {
#pragma unroll 4
            for (uint32_t b = threadIdx.x; b < n / 2u; b += 1024u) {
                const uint32_t i = (b / d) * 2 * d + (b % d);
                const uint32_t a = err[i], c = err[i + d];
                err[i] = (uint16_t)addm(a, c);
                err[i + d] = (uint16_t)subm(a, c);
            }
            __syncthreads();
        }
        if (pass == 0) {
#pragma unroll 4
            for (uint32_t i = threadIdx.x; i < n; i += 1024u)
                err[i] = (uint16_t)(((uint32_t)err[i] * fold[i]) % kMod16);
            __syncthreads();
        }
    }
    for (uint32_t i = threadIdx.x; i < n; i += 1024u) p.errs_out[(uint64_t)qi * n + i] = err[i];
}

inline uint32_t blocks_for(uint64_t tasks) { return (uint32_t)((tasks + 3) / 4); }

// m = 512 encoder form: 16 waves x 32 elements (production) or 8 x 64 (diagnostic A/B)
// (diagnostic A/B: rsm_diag_set_enc16_e64 1 = 8 waves x 64 elements, 2 = the
// round-3 16-wave form with scalar-loaded tables, one workgroup per task, 3 = that
// form with the half exchange buffer, 5 = production with just-in-time table reads)
#ifdef RSM_DIAG
static std::atomic<int> g_enc16_e64{0};
static bool enc16_e64() { return g_enc16_e64.load() == 1; }
static int enc16_form() { return g_enc16_e64.load(); }
#else
static bool enc16_e64() { return false; }
static int enc16_form() { return 0; }
#endif

template <int M>
hipError_t run_encode(const CodewordSet& cs, const Gf16Dev& g, hipStream_t st) {
    const uint32_t chunks = (cs.S + 511) / 512;
    const uint64_t tasks = (uint64_t)cs.count * chunks;
    if (tasks == 0) return hipSuccess;
    if (tasks >= (1ull << 31)) return hipErrorInvalidValue;
    // the merged middle pair's twiddle: exp(SKEW[m - 1 + m/2]) + exp(SKEW[m/2 - 1])
    const Gf16Host& hst = gf16_host();
    auto elem = [&](uint32_t L) { return L == kMod16 ? 0u : (uint32_t)hst.exp[L]; };
    const uint32_t sum = elem(hst.skew[M - 1 + M / 2]) ^ elem(hst.skew[M / 2 - 1]);
    Enc16 p{cs, g.skewperm, chunks, sum ? g.perm + hst.log[sum] : nullptr};
    // persistent forms: one workgroup per CU (two for the m = 256 half-wave form), the
    // twiddle tables staged once per workgroup; the non-persistent diagnostic forms run
    // one workgroup per task
    const uint32_t pgrid = tasks > g.cus ? g.cus : (uint32_t)tasks;  // persistent forms
    const uint32_t grid = M == 256 ? pgrid : (uint32_t)tasks;
    if (cs.side || cs.blk) {  // multi-GPU all-to-all hooks: the production form with SH = 1 / 2
        Enc16 ph = p;
        ph.chunks = (cs.S + 255) / 256;
        const uint64_t th = (uint64_t)cs.count * ph.chunks;
        if (th >= (1ull << 31)) return hipErrorInvalidValue;
        const uint32_t per_cu = M == 256 ? 2u : 1u;  // workgroups per CU of the half-wave forms
        const uint32_t gh = th > (uint64_t)per_cu * g.cus ? per_cu * g.cus : (uint32_t)th;
        if constexpr (M == 512) {
            if (cs.side) hipLaunchKernelGGL((enc16h512_kernel<true, false, true, 1>), dim3(gh), dim3(1024), 0, st, ph);
            else hipLaunchKernelGGL((enc16h512_kernel<true, false, true, 2>), dim3(gh), dim3(1024), 0, st, ph);
        } else {
            if (cs.side) hipLaunchKernelGGL((enc16h_kernel<true, false, true, 1>), dim3(gh), dim3(512), 0, st, ph);
            else hipLaunchKernelGGL((enc16h_kernel<true, false, true, 2>), dim3(gh), dim3(512), 0, st, ph);
        }
        return hipGetLastError();
    }
    if constexpr (M == 512) {
        if (enc16_e64()) {
            hipLaunchKernelGGL((enc16_kernel<512, 64>), dim3(grid), dim3(512), 0, st, p);
            return hipGetLastError();
        }
        // production since round 4 (form 0): the half-wave form with just-in-time tables
        // (enc16h512_kernel<true>), c5 0.472-0.474 ms per square against 0.587-0.590 for
        // 512-byte chunks (form 4 below; profiles/r04aa_gf16_enc_ab.jsonl).  Diagnostic
        // forms: 1 8 waves x 64 elements (above), 4 persistent 16 waves x 32 elements, LDS
        // tables beside a half exchange buffer (0.568-0.574, production through the
        // round's middle), 2 the round-3 form (0.581-0.583), 3 form 2 with the half
        // buffer, 5 form 4 with just-in-time table reads (0.584), 8 / 9 forms 4 / 5 with
        // the merged middle pair, 16 the half-wave form with compiler-scheduled table
        // reads (0.505-0.510)
        switch (enc16_form()) {
            case 0:      // production since round 6: the half-wave form with tables read one
            case 21: {   // block ahead (form 21 in round 6's A/B: c5 0.451-0.466 against
                         // 0.466-0.469 ms for just-in-time tables, now form 22;
                         // profiles/r06i_gf16_pipe_ab.jsonl)
                Enc16 ph = p;
                ph.chunks = (cs.S + 255) / 256;
                const uint64_t th = (uint64_t)cs.count * ph.chunks;
                if (th >= (1ull << 31)) return hipErrorInvalidValue;
                const uint32_t gh = th > g.cus ? g.cus : (uint32_t)th;
                hipLaunchKernelGGL((enc16h512_kernel<true, false, true>), dim3(gh), dim3(1024), 0, st, ph);
                return hipGetLastError();
            }
            case 22: {  // the round-4/5 production form: just-in-time table reads
                Enc16 ph = p;
                ph.chunks = (cs.S + 255) / 256;
                const uint64_t th = (uint64_t)cs.count * ph.chunks;
                if (th >= (1ull << 31)) return hipErrorInvalidValue;
                const uint32_t gh = th > g.cus ? g.cus : (uint32_t)th;
                hipLaunchKernelGGL(enc16h512_kernel<true>, dim3(gh), dim3(1024), 0, st, ph);
                return hipGetLastError();
            }
            case 4: hipLaunchKernelGGL((enc16_kernel<512, 32, 3>), dim3(pgrid), dim3(1024), 0, st, p); return hipGetLastError();
            case 3: hipLaunchKernelGGL((enc16_kernel<512, 32, 1>), dim3(grid), dim3(1024), 0, st, p); return hipGetLastError();
            case 5: hipLaunchKernelGGL((enc16_kernel<512, 32, 7>), dim3(pgrid), dim3(1024), 0, st, p); return hipGetLastError();
            case 8: hipLaunchKernelGGL((enc16_kernel<512, 32, 11>), dim3(pgrid), dim3(1024), 0, st, p); return hipGetLastError();
            case 9: hipLaunchKernelGGL((enc16_kernel<512, 32, 15>), dim3(pgrid), dim3(1024), 0, st, p); return hipGetLastError();
            case 18: {  // the production form with the next task's points prefetched
                Enc16 ph = p;
                ph.chunks = (cs.S + 255) / 256;
                const uint64_t th = (uint64_t)cs.count * ph.chunks;
                if (th >= (1ull << 31)) return hipErrorInvalidValue;
                const uint32_t gh = th > g.cus ? g.cus : (uint32_t)th;
                hipLaunchKernelGGL((enc16h512_kernel<true, true>), dim3(gh), dim3(1024), 0, st, ph);
                return hipGetLastError();
            }
            case 16: {
                Enc16 ph = p;
                ph.chunks = (cs.S + 255) / 256;
                const uint64_t th = (uint64_t)cs.count * ph.chunks;
                if (th >= (1ull << 31)) return hipErrorInvalidValue;
                const uint32_t gh = th > g.cus ? g.cus : (uint32_t)th;
                hipLaunchKernelGGL(enc16h512_kernel<false>, dim3(gh), dim3(1024), 0, st, ph);
                return hipGetLastError();
            }
            default: break;
        }
    }
    if constexpr (M == 256) {
        // production since round 4: the half-wave form (enc16h_kernel<true>: 256-byte
        // chunks, 32 state registers, two workgroups per CU, just-in-time tables), c4
        // 0.415-0.419 ms per square against 0.427-0.431 for 16 waves x 16 elements over
        // 512-byte chunks (diagnostic form 6) and 0.435-0.450 for 8 waves x 32 elements
        // (form 7, through round 3); form 14: the half-wave form with compiler-scheduled
        // table reads (0.436-0.440).  profiles/r04k_gf16_enc_ab.jsonl, r04q_gf16_enc_ab.jsonl
        const int form = enc16_form();
        if (form == 6) {
            hipLaunchKernelGGL((enc16_kernel<256, 16>), dim3(grid), dim3(1024), 0, st, p);
            return hipGetLastError();
        }
        if (form != 7) {
            Enc16 ph = p;
            ph.chunks = (cs.S + 255) / 256;
            const uint64_t th = (uint64_t)cs.count * ph.chunks;
            if (th >= (1ull << 31)) return hipErrorInvalidValue;
            const uint32_t gh = th > 2ull * g.cus ? 2u * g.cus : (uint32_t)th;
            const uint32_t gh3 = th > 3ull * g.cus ? 3u * g.cus : (uint32_t)th;
            if (form == 20) hipLaunchKernelGGL(enc16h3_kernel, dim3(gh3), dim3(512), 0, st, ph);
            else if (form == 19) hipLaunchKernelGGL((enc16h_kernel<true, true>), dim3(gh), dim3(512), 0, st, ph);
            else if (form == 14) hipLaunchKernelGGL(enc16h_kernel<false>, dim3(gh), dim3(512), 0, st, ph);
            else if (form == 22) hipLaunchKernelGGL(enc16h_kernel<true>, dim3(gh), dim3(512), 0, st, ph);
            // production since round 6 (and form 21): tables read one block ahead; c4
            // 0.400-0.410 against 0.409-0.422 ms for just-in-time tables (form 22,
            // profiles/r06i_gf16_pipe_ab.jsonl)
            else hipLaunchKernelGGL((enc16h_kernel<true, false, true>), dim3(gh), dim3(512), 0, st, ph);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL(enc16_kernel<M>, dim3(grid), dim3(M * 2), 0, st, p);
    return hipGetLastError();
}

#ifdef RSM_DIAG
static std::atomic<bool> g_dec16_five{false};
static bool dec16_five_pass() { return g_dec16_five.load(); }
static std::atomic<uint32_t> g_dec16_mode{0};
static uint32_t dec16_diag_mode() { return g_dec16_mode.load(); }
#else
static bool dec16_five_pass() { return false; }
static uint32_t dec16_diag_mode() { return 0u; }
#endif
// m = 512: the half-wave single pass (dec16h_kernel) since round 4 -- decode sweep
// k = 512 1.43-1.45 ms against 1.84-1.85 for the five passes (diagnostic A/B:
// rsm_diag_set_dec16_five_pass; profiles/r04w_gf16_dec_ab.jsonl)
static bool dec16h_enabled() { return !dec16_five_pass(); }
}  // namespace
bool dec16_needs_work() { return dec16_five_pass(); }
namespace {


template <int M>
hipError_t run_decode(const DecodeSet& ds, const Gf16Dev& g, const uint16_t* logwalsh, hipStream_t st) {
    constexpr int N = 2 * M;
    const uint32_t chunks = (ds.S + 511) / 512;
    // batches: the error locators of a batch (the host sizes them for the whole set);
    // only the five-pass diagnostic form also needs per-codeword work arrays
    uint32_t batch = (uint32_t)(g.errs_bytes / (N * sizeof(uint16_t)));
    if (dec16_needs_work()) {
        const uint32_t wbatch = (uint32_t)(g.scratch_bytes / (2ull * N * ds.S));
        if (wbatch < batch) batch = wbatch;
    }
    if (batch == 0) return hipErrorOutOfMemory;
    if ((ds.in_base || ds.mirror) && dec16_five_pass()) return hipErrorInvalidValue;  // no zero-copy five passes
    for (uint32_t q0 = 0; q0 < ds.count; q0 += batch) {
        Dec16 p{ds, Res{g.perm, g.skew}, logwalsh, g.errs, g.scratch, q0,
                ds.count - q0 < batch ? ds.count - q0 : batch, chunks, g.skewperm};
        p.ds.trace = dec_diag_trace_ptr();
        p.diag = dec16_diag_mode();
        hipLaunchKernelGGL(errloc16_kernel<M>, dim3(p.count), dim3(M), 0, st, p);
        if constexpr (M == 512) {
            if (dec16h_enabled()) {  // the half-wave single pass: 256-byte chunks
                const uint32_t ch = (ds.S + 255) / 256;
                Dec16 ph = p;
                ph.chunks = ch;
                if (ds.in_base) hipLaunchKernelGGL((dec16h_kernel<M, true>), dim3(p.count * ch), dim3(1024), 0, st, ph);
                else hipLaunchKernelGGL((dec16h_kernel<M, false>), dim3(p.count * ch), dim3(1024), 0, st, ph);
                if (hipError_t e = hipGetLastError()) return e;
                continue;
            }
        }
        if constexpr (M == 256) {
            if (!dec16_five_pass()) {  // the single-pass form (diagnostic builds can A/B the five passes)
                const uint32_t tk = p.count * chunks;
                const uint32_t grid = tk > g.cus ? g.cus : tk;
                if (ds.in_base) hipLaunchKernelGGL((dec16f_kernel<M, true>), dim3(grid), dim3(1024), 0, st, p);
                else hipLaunchKernelGGL((dec16f_kernel<M, false>), dim3(grid), dim3(1024), 0, st, p);
                if (hipError_t e = hipGetLastError()) return e;
                continue;
            }
        }
        hipLaunchKernelGGL(dec16_p1<M>, dim3(blocks_for((uint64_t)p.count * chunks * (N / 16))), dim3(256), 0, st, p);
        hipLaunchKernelGGL(dec16_p2<M>, dim3(blocks_for((uint64_t)p.count * chunks * 16)), dim3(256), 0, st, p);
        hipLaunchKernelGGL(dec16_p3<M>, dim3(blocks_for((uint64_t)p.count * chunks * (N / 16))), dim3(256), 0, st, p);
        hipLaunchKernelGGL(dec16_p4<M>, dim3(blocks_for((uint64_t)p.count * chunks * 16)), dim3(256), 0, st, p);
        hipLaunchKernelGGL(dec16_p5<M>, dim3(blocks_for((uint64_t)p.count * chunks * (N / 16))), dim3(256), 0, st, p);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}


// ---- generic multi-pass launchers (m >= 1024) ----
template <int BITS, int NI, int NF>
static void g16_go(const G16Pass& p, hipStream_t st) {
    const uint64_t waves = (uint64_t)p.count * p.chunks * (p.npts >> BITS);
    hipLaunchKernelGGL((g16_pass_kernel<BITS, NI, NF>), dim3(blocks_for(waves)), dim3(256), 0, st, p);
}
// pass shapes: lower groups IFFT-only / FFT-only (4 bits); the top group (1..4
// bits) IFFT + FFT (encode), or IFFT-only and FFT-only around the derivative (decode)
static hipError_t g16_pass(const G16Pass& p, uint32_t bits, uint32_t ni, uint32_t nf, hipStream_t st) {
#define RSM_G16(b)                                          \
    case b:                                                 \
        if (ni == b && nf == b) g16_go<b, b, b>(p, st);     \
        else if (ni == b && nf == 0) g16_go<b, b, 0>(p, st); \
        else if (ni == 0 && nf == b) g16_go<b, 0, b>(p, st); \
        else return hipErrorInvalidValue;                   \
        break;
    switch (bits) {
        RSM_G16(1)
        RSM_G16(2)
        RSM_G16(3)
        RSM_G16(4)
        default: return hipErrorInvalidValue;
    }
#undef RSM_G16
    return hipGetLastError();
}
template <int BITS>
static void g16_deriv_go(const G16Pass& p, hipStream_t st) {
    const uint64_t waves = (uint64_t)p.count * p.chunks * (p.npts >> BITS);
    hipLaunchKernelGGL((g16_deriv_kernel<BITS>), dim3(blocks_for(waves)), dim3(256), 0, st, p);
}
static hipError_t g16_deriv(const G16Pass& p, uint32_t bits, hipStream_t st) {
    switch (bits) {
        case 1: g16_deriv_go<1>(p, st); break;
        case 2: g16_deriv_go<2>(p, st); break;
        case 3: g16_deriv_go<3>(p, st); break;
        case 4: g16_deriv_go<4>(p, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// bit groups of an L-bit transform: 4 bits per group from the bottom, the
// remainder (1..4 bits) on top
struct G16Groups {
    uint32_t n = 0, bits[4] = {}, D[4] = {};
};
static G16Groups g16_groups(uint32_t L) {
    G16Groups g;
    g.n = (L + 3) / 4;
    for (uint32_t i = 0; i < g.n; ++i) {
        g.bits[i] = i + 1 < g.n ? 4u : L - 4u * (g.n - 1);
        g.D[i] = 1u << (4u * i);
    }
    return g;
}
static uint32_t ilog2u(uint32_t x) {
    uint32_t r = 0;
    while ((1u << r) < x) ++r;
    return r;
}

// Byte slabs of the shares: a codeword's work arrays (`per_point` bytes per point and
// byte of share width) must fit the stream's scratch, so wide shares run as slabs of
// whole 64-byte blocks (the GF(2^16) symbol layout never crosses one) -- each slab a
// launch sequence of its own over base + first byte, the strides unchanged.
static uint32_t g16_slab(uint64_t per_point, uint32_t S, uint64_t scratch) {
    if (per_point * S <= scratch) return S;
    return (uint32_t)(scratch / per_point / 64u * 64u);
}

static hipError_t run_encode_generic(const CodewordSet& cs0, const Gf16Dev& g, hipStream_t st) {
    const uint32_t m = ceil_pow2(cs0.k);
    const uint32_t slab = g16_slab(m, cs0.S, g.scratch_bytes);
    if (slab == 0) return hipErrorOutOfMemory;
    const G16Groups gr = g16_groups(ilog2u(m));
    for (uint64_t c0 = 0; c0 < cs0.S; c0 += slab) {
    CodewordSet cs = cs0;
    cs.base = cs0.base + c0;
    cs.out_base = (cs0.out_base ? cs0.out_base : cs0.base) + c0;
    cs.S = (uint32_t)(cs0.S - c0 < slab ? cs0.S - c0 : slab);
    const uint32_t chunks = (cs.S + 511) / 512;
    const uint64_t per_cw = (uint64_t)m * cs.S;
    const uint32_t batch = (uint32_t)(g.scratch_bytes / per_cw);
    if (batch == 0) return hipErrorOutOfMemory;
    for (uint32_t q0 = 0; q0 < cs.count; q0 += batch) {
        G16Pass p{};
        p.cs = cs;
        p.r = Res{g.perm, g.skew};
        p.work = g.scratch;
        p.cw_bytes = per_cw;
        p.npts = m;
        p.m = m;
        p.k = cs.k;
        p.S = cs.S;
        p.chunks = chunks;
        p.q0 = q0;
        p.count = cs.count - q0 < batch ? cs.count - q0 : batch;
        p.ifft_off = (int)m - 1;
        hipError_t e;
        const uint32_t top = gr.n - 1;
        for (uint32_t i = 0; i < top; ++i) {  // IFFT, lower groups (the first reads the data shares)
            p.D = gr.D[i];
            p.src = i == 0 ? 2u : 0u;
            p.dst = 0u;
            if ((e = g16_pass(p, 4, 4, 0, st)) != hipSuccess) return e;
        }
        p.D = gr.D[top];
        p.src = top == 0 ? 2u : 0u;
        p.dst = top == 0 ? 2u : 0u;
        if ((e = g16_pass(p, gr.bits[top], gr.bits[top], gr.bits[top], st)) != hipSuccess) return e;
        for (uint32_t i = top; i-- > 0;) {  // FFT, lower groups (the last writes the parity)
            p.D = gr.D[i];
            p.src = 0u;
            p.dst = i == 0 ? 2u : 0u;
            if ((e = g16_pass(p, 4, 0, 4, st)) != hipSuccess) return e;
        }
    }
    }
    return hipSuccess;
}

static hipError_t run_decode_generic(const DecodeSet& ds0, const Gf16Dev& g, hipStream_t st) {
    const uint32_t m = ceil_pow2(ds0.k), n = 2 * m;
    const uint32_t slab = g16_slab(2ull * n, ds0.S, g.scratch_bytes);
    if (slab == 0) return hipErrorOutOfMemory;
    const G16Groups gr = g16_groups(ilog2u(n));
    const uint32_t top = gr.n - 1;
    for (uint64_t c0 = 0; c0 < ds0.S; c0 += slab) {
    DecodeSet ds = ds0;
    ds.base = ds0.base + c0;
    ds.S = (uint32_t)(ds0.S - c0 < slab ? ds0.S - c0 : slab);
    const uint32_t chunks = (ds.S + 511) / 512;
    const uint64_t per_cw = 2ull * n * ds.S;
    uint32_t batch = (uint32_t)(g.scratch_bytes / per_cw);
    const uint32_t ebatch = (uint32_t)(g.errs_bytes / (n * sizeof(uint16_t)));
    if (ebatch < batch) batch = ebatch;
    if (batch == 0) return hipErrorOutOfMemory;
    for (uint32_t q0 = 0; q0 < ds.count; q0 += batch) {
        G16Pass p{};
        p.ds = ds;
        p.r = Res{g.perm, g.skew};
        p.errs = g.errs;
        p.errs_out = g.errs;
        p.logwalsh = g.logwalsh;
        p.work = g.scratch;
        p.cw_bytes = per_cw;
        p.pitch = ds0.pitch ? ds0.pitch : ds0.S;
        p.npts = n;
        p.m = m;
        p.k = ds.k;
        p.S = ds.S;
        p.chunks = chunks;
        p.q0 = q0;
        p.count = ds.count - q0 < batch ? ds.count - q0 : batch;
        p.ifft_off = -1;
        p.decode = 1u;
        hipLaunchKernelGGL(errloc16g_kernel, dim3(p.count), dim3(1024), 0, st, p);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        for (uint32_t i = 0; i <= top; ++i) {  // IFFT up to the top group -> A
            p.D = gr.D[i];
            p.src = i == 0 ? 2u : 0u;
            p.dst = 0u;
            if ((e = g16_pass(p, gr.bits[i], gr.bits[i], 0, st)) != hipSuccess) return e;
        }
        for (uint32_t i = 0; i <= top; ++i) {  // formal derivative: B = A + sum T_g(A)
            p.D = gr.D[i];
            p.src = i == 0 ? 1u : 0u;
            if ((e = g16_deriv(p, gr.bits[i], st)) != hipSuccess) return e;
        }
        for (uint32_t i = top + 1; i-- > 0;) {  // FFT on B down to group 0, which reveals
            p.D = gr.D[i];
            p.src = 1u;
            p.dst = i == 0 ? 2u : 1u;
            if ((e = g16_pass(p, gr.bits[i], 0, gr.bits[i], st)) != hipSuccess) return e;
        }
    }
    }
    return hipSuccess;
}
}  // namespace

#ifdef RSM_DIAG
void set_enc16_diag_e64(int mode) { g_enc16_e64.store(mode); }
void set_dec16_diag_five_pass(bool on) { g_dec16_five.store(on); }
void set_dec16_diag_mode(uint32_t m) { g_dec16_mode.store(m); }
#endif

hipError_t launch_encode_gf16(const CodewordSet& cs, const Gf16Dev& g, hipStream_t st) {
    if (cs.wide) return cs.k <= 32768u ? run_encode_generic(cs, g, st) : hipErrorNotSupported;
    switch (ceil_pow2(cs.k)) {
        case 256: return run_encode<256>(cs, g, st);
        case 512: return run_encode<512>(cs, g, st);
        default: return cs.k <= 32768u ? run_encode_generic(cs, g, st) : hipErrorNotSupported;
    }
}

hipError_t launch_decode_gf16(const DecodeSet& ds, const Gf16Dev& g, hipStream_t st) {
    if (ds.wide) return ds.k <= 32768u ? run_decode_generic(ds, g, st) : hipErrorNotSupported;
    switch (ceil_pow2(ds.k)) {
        case 256: return run_decode<256>(ds, g, g.logwalsh, st);
        case 512: return run_decode<512>(ds, g, g.logwalsh, st);
        default: return ds.k <= 32768u ? run_decode_generic(ds, g, st) : hipErrorNotSupported;
    }
}

}  // namespace rsm
