// kernels_gf16.hip -- CDNA4 Leopard GF(2^16) Reed-Solomon kernels (2k > 256).
//
// klauspost/reedsolomon v1.14.1 leopard.go semantics:
// symbol t of every 64-byte block b of a share is lo = share[64b+t], hi =
// share[64b+32+t] (A.6).  A lane holds 4 adjacent symbols as two dwords (4 lo
// bytes, 4 hi bytes), so a wavefront spans 8 blocks = 512 bytes of share width
// and every multiply-by-constant is 12 v_perm_b32 lookups (PermTab16).
//
// The m-point transforms (m = ceilPow2(k) in {256, 512}) do not fit in one
// lane's registers, so they run as radix-16 passes through a global scratch
// work array ([codeword][element][S], L2/MALL-resident for the batch sizes the
// launcher picks):
//   encode: A group layout  (16 consecutive elements): IFFT layers 1..8
//           B residue layout (elements r, r+16, ...):  IFFT layers 16..m/2, FFT m/2..16
//           C group layout:                            FFT layers 8..1, parity out
//   decode (n = 2m): 1 group: scale by the error locator + IFFT low
//                    2 residue: IFFT high; also H(in) = high-bit half of the formal derivative
//                    3 group: out = in + L(in) + H(in)  (the derivative's closed form)
//                    4 residue: FFT high          5 group: FFT low + reveal
// Every wave works on one (codeword, 512-byte chunk, group|residue) task, so all
// lanes share each twiddle (wave-uniform SGPR table loads).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>
#include <utility>
#include "gf16.hpp"
#include "rsm_kernels.hpp"

namespace rsm {
namespace {

constexpr uint32_t kMod16 = 65535u;
constexpr uint32_t kOob16 = 0x80000000u;

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

// (xl, xh) ^= (yl, yh) * exp(L), tables t = PermTab16[L]
__device__ __forceinline__ void muladd16(uint32_t& xl, uint32_t& xh, uint32_t yl, uint32_t yh, const PermTab16& t) {
    const uint32_t sa = yl & 0x07070707u, sb = (yl >> 3) & 0x07070707u, sc = (yl >> 6) & 0x03030303u;
    const uint32_t sd = yh & 0x07070707u, se = (yh >> 3) & 0x07070707u, sf = (yh >> 6) & 0x03030303u;
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
// Encoder passes (codewords q0 .. q0 + count of the CodewordSet; scratch row
// (q - q0) holds that codeword's m-element work array)
// ---------------------------------------------------------------------------
struct Enc16 {
    CodewordSet cs;
    Res r;
    uint8_t* scratch;
    uint32_t q0, count, chunks;
};

template <int M>
__global__ __launch_bounds__(256) void enc16_a(Enc16 p) {
    const TaskIdx t = task_of(p.count, p.chunks, M / 16);
    if (!t.valid) return;
    const Lane ln = lane_of(t.chunk, p.cs.S);
    const auto in = rsrc(p.cs.base + cw_rel(p.cs, p.q0 + t.q));
    const auto wk = rsrc(p.scratch + (uint64_t)t.q * M * p.cs.S);
    const uint32_t es = (uint32_t)p.cs.elem_stride, k = p.cs.k, S = p.cs.S;
    uint32_t l[16], h[16];
    sfor<16>([&](auto E) {
        constexpr int i = decltype(E)::value;
        const uint32_t e = 16 * t.g + i;
        const uint32_t so = e < k ? e * es : kOob16;
        l[i] = ld(in, ln.lo, so);
        h[i] = ld(in, ln.lo + 32, so);
    });
    group_ifft(l, h, t.g, M - 1, p.r);
    sfor<16>([&](auto E) {
        constexpr int i = decltype(E)::value;
        const uint32_t so = (16 * t.g + i) * S;
        st(wk, l[i], ln.lo, so);
        st(wk, h[i], ln.lo + 32, so);
    });
}

template <int M>
__global__ __launch_bounds__(256) void enc16_b(Enc16 p) {
    constexpr int R = M / 16;
    const TaskIdx t = task_of(p.count, p.chunks, 16);
    if (!t.valid) return;
    const Lane ln = lane_of(t.chunk, p.cs.S);
    const auto wk = rsrc(p.scratch + (uint64_t)t.q * M * p.cs.S);
    const uint32_t S = p.cs.S;
    uint32_t l[R], h[R];
    sfor<R>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t so = (t.g + 16 * j) * S;
        l[j] = ld(wk, ln.lo, so);
        h[j] = ld(wk, ln.lo + 32, so);
    });
    residue_ifft<R>(l, h, M - 1, p.r);
    residue_fft<R>(l, h, p.r);
    sfor<R>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t so = (t.g + 16 * j) * S;
        st(wk, l[j], ln.lo, so);
        st(wk, h[j], ln.lo + 32, so);
    });
}

template <int M>
__global__ __launch_bounds__(256) void enc16_c(Enc16 p) {
    const TaskIdx t = task_of(p.count, p.chunks, M / 16);
    if (!t.valid) return;
    const Lane ln = lane_of(t.chunk, p.cs.S);
    const uint64_t rel = cw_rel(p.cs, p.q0 + t.q);
    const auto out = rsrc(p.cs.out_base + rel);
    const auto wk = rsrc(p.scratch + (uint64_t)t.q * M * p.cs.S);
    const uint32_t es = (uint32_t)p.cs.elem_stride, k = p.cs.k, S = p.cs.S;
    const uint32_t oo = (uint32_t)p.cs.out_offset;
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
        const uint32_t so = e < k ? oo + e * es : kOob16;
        st(out, l[i], ln.lo, so);
        st(out, h[i], ln.lo + 32, so);
    });
}

// ---------------------------------------------------------------------------
// Decoder
// ---------------------------------------------------------------------------
struct Dec16 {
    DecodeSet ds;
    Res r;
    const uint16_t* logwalsh;
    uint16_t* errs;     // [count][n]
    uint8_t* scratch;   // [count][2][n][S]
    uint32_t q0, count, chunks;
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

// Error locator of one codeword (klauspost reconstruct): FWHT over the
// full 65536-entry table in LDS, times LogWalsh, FWHT again; writes err[0..n).
template <int M>
__global__ __launch_bounds__(1024) void errloc16_kernel(Dec16 p) {
    constexpr int N = 2 * M;
    __shared__ uint16_t err[65536];
    const uint32_t q = blockIdx.x;
    const uint32_t k = p.ds.k;
#pragma unroll 2
    for (uint32_t i = threadIdx.x; i < 65536u; i += 1024u) {
        uint32_t v = 0;
        if (i < k) v = p.ds.presence[cell_of(p.ds, p.q0 + q, k + i)] ? 0u : 1u;
        else if (i < (uint32_t)M) v = 1u;
        else if (i < (uint32_t)M + k) v = p.ds.presence[cell_of(p.ds, p.q0 + q, i - M)] ? 0u : 1u;
        err[i] = (uint16_t)v;
    }
    __syncthreads();
#pragma unroll 1
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll 1
        for (uint32_t d = 1; d < 65536u; d <<= 1) {
#pragma unroll 4
            for (uint32_t b = threadIdx.x; b < 32768u; b += 1024u) {
                const uint32_t i = (b / d) * 2 * d + (b % d);
                const uint32_t a = err[i], c = err[i + d];
                err[i] = (uint16_t)addm(a, c);
                err[i + d] = (uint16_t)subm(a, c);
            }
            __syncthreads();
        }
        if (pass == 0) {
#pragma unroll 4
            for (uint32_t i = threadIdx.x; i < 65536u; i += 1024u)
                err[i] = (uint16_t)(((uint32_t)err[i] * p.logwalsh[i]) % kMod16);
            __syncthreads();
        }
    }
    for (uint32_t i = threadIdx.x; i < (uint32_t)N; i += 1024u) p.errs[(uint64_t)q * N + i] = err[i];
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

inline uint32_t blocks_for(uint64_t tasks) { return (uint32_t)((tasks + 3) / 4); }

// Work-array bytes per encode launch triple (A, B, C).  Measured on config 4 (k=256,
// S=2048) and 5 (k=512, S=512): capping a batch at 64 MiB so that its work arrays
// stay in the Infinity Cache between the passes is SLOWER (175 vs 196 GiB/s, 0.90
// vs 0.77 ms) than one launch triple over up to 1 GiB of work arrays -- the extra
// launches cost more than the HBM round trips they save.  RSM_GF16_BATCH_MB
// overrides it in the diagnostic build only (A/B measurements).
static uint64_t gf16_batch_bytes() {
#ifdef RSM_DIAG
    static const uint64_t b = [] {
        const char* v = getenv("RSM_GF16_BATCH_MB");
        const uint64_t mb = v ? strtoull(v, nullptr, 10) : 0;
        return (mb ? mb : 1024ull) << 20;
    }();
    return b;
#else
    return 1024ull << 20;
#endif
}

template <int M>
hipError_t run_encode(const CodewordSet& cs, const Gf16Dev& g, hipStream_t st) {
    const uint32_t chunks = (cs.S + 511) / 512;
    const uint64_t per_cw = (uint64_t)M * cs.S;
    uint32_t batch = (uint32_t)((g.scratch_bytes < gf16_batch_bytes() ? g.scratch_bytes : gf16_batch_bytes()) / per_cw);
    if (batch == 0) batch = (uint32_t)(g.scratch_bytes / per_cw);
    if (batch == 0) return hipErrorOutOfMemory;
    for (uint32_t q0 = 0; q0 < cs.count; q0 += batch) {
        Enc16 p{cs, Res{g.perm, g.skew}, g.scratch, q0, cs.count - q0 < batch ? cs.count - q0 : batch, chunks};
        hipLaunchKernelGGL(enc16_a<M>, dim3(blocks_for((uint64_t)p.count * chunks * (M / 16))), dim3(256), 0, st, p);
        hipLaunchKernelGGL(enc16_b<M>, dim3(blocks_for((uint64_t)p.count * chunks * 16)), dim3(256), 0, st, p);
        hipLaunchKernelGGL(enc16_c<M>, dim3(blocks_for((uint64_t)p.count * chunks * (M / 16))), dim3(256), 0, st, p);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

template <int M>
hipError_t run_decode(const DecodeSet& ds, const Gf16Dev& g, const uint16_t* logwalsh, hipStream_t st) {
    constexpr int N = 2 * M;
    const uint32_t chunks = (ds.S + 511) / 512;
    const uint64_t per_cw = 2ull * N * ds.S;
    uint32_t batch = (uint32_t)(g.scratch_bytes / per_cw);
    const uint32_t ebatch = (uint32_t)(g.errs_bytes / (N * sizeof(uint16_t)));
    if (ebatch < batch) batch = ebatch;
    if (batch == 0) return hipErrorOutOfMemory;
    for (uint32_t q0 = 0; q0 < ds.count; q0 += batch) {
        Dec16 p{ds, Res{g.perm, g.skew}, logwalsh, g.errs, g.scratch, q0,
                ds.count - q0 < batch ? ds.count - q0 : batch, chunks};
        hipLaunchKernelGGL(errloc16_kernel<M>, dim3(p.count), dim3(1024), 0, st, p);
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

}  // namespace

hipError_t launch_encode_gf16(const CodewordSet& cs, const Gf16Dev& g, hipStream_t st) {
    switch (ceil_pow2(cs.k)) {
        case 256: return run_encode<256>(cs, g, st);
        case 512: return run_encode<512>(cs, g, st);
        default: return hipErrorNotSupported;
    }
}

hipError_t launch_decode_gf16(const DecodeSet& ds, const Gf16Dev& g, hipStream_t st) {
    switch (ceil_pow2(ds.k)) {
        case 256: return run_decode<256>(ds, g, g.logwalsh, st);
        case 512: return run_decode<512>(ds, g, g.logwalsh, st);
        default: return hipErrorNotSupported;
    }
}

}  // namespace rsm
