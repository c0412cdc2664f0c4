// kernels_gf8_bs.hip -- bit-sliced GF(2^8) encode for M = 128 (65 <= k <= 128).
//
// The byte-table kernel (kernels_gf8.hip) spends ~10 VALU per 4 bytes per GF
// multiply and is VALU-bound (SQ counters: ~98% of VALU issue cycles on the
// column pass).  Here 32 bytes of a symbol are 8 bit-planes and a multiply by a
// constant is ~16 VALU per 32 bytes (bs8.hpp): 4.7K VALU per wave-set against
// 9.4K.  A lane can hold 16 symbols x 8 planes (128 VGPRs), not the whole
// 128-symbol codeword, so the transform is split between the 8 wavefronts of a
// workgroup (bs8.hpp):
//
//   set       = 64 lanes x 32 bytes = 2 KiB of share width (e.g. four 512-byte
//               codewords), all 128 symbols of it;
//   wave w    : small layout, symbols e = 16w + j: IFFT layers d = 1,2,4
//   LDS       : 2 rounds x 4 planes, [symbol][lane] x 16 B = 128 KiB
//   wave w    : large layout, symbols e = 8h + w: IFFT d = 8..64, FFT d = 64..8
//   LDS back, FFT layers d = 4,2,1, planes -> bytes, store.
//
// The small layers' twiddles depend on w, so the whole per-wave program is a
// template on w and the kernel branches once, at entry, into one of 8 copies:
// no control-flow merge carries the 128 planes (a merge costs ~250 register
// copies per wave and spills -- measured).
//
// Persistent: one workgroup per CU walks sets t = blockIdx.x, += gridDim.x, and
// loads set t+G while computing set t -- symbols j >= 8 of each wave into 64
// VGPRs (issued once the LDS buffer is released), j < 8 by LDS-DMA into the
// 128 KiB exchange buffer (issued after the second exchange).  Both are waited
// for with an explicit vmcnt that leaves the previous set's 32 stores in flight.
// (With one set per workgroup, memory and compute phases of the CU do not
// overlap: measured 4.2 TB/s for loads + stores with no arithmetic at all.)
//
// Memory: lane l holds bytes [16l, 16l+16) and [1024+16l, +16) of the set's 2 KiB
// (two dwordx4 per symbol; every wave instruction covers 1 KiB contiguous per
// codeword run).  Same CodewordSet contract as encode_gf8_kernel (row pass,
// column pass, slices); callers with an index list use the byte-table kernel.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "bs8.hpp"
#include "rsm_kernels.hpp"

namespace rsm {

namespace {

constexpr uint32_t kOobBs = 0x80000000u;
constexpr uint32_t kSetBytes = 2048;

__device__ __forceinline__ uint64_t cw_rel_bs(const CodewordSet& cs, uint32_t q) {
    const uint32_t sq = q / cs.per_square;
    const uint32_t t = q - sq * cs.per_square;
    return (uint64_t)sq * cs.square_stride + (uint64_t)t * cs.cw_stride;
}

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

__device__ __forceinline__ uint32_t sym_off(uint32_t e, uint32_t k, uint32_t base, uint32_t es) {
    return __builtin_amdgcn_readfirstlane(e < k ? base + e * es : kOobBs);
}

constexpr int kPre = 8;  // symbols j < kPre of each wave arrive by LDS-DMA

// LDS-DMA (buffer_load_dwordx4 ... lds): 16 B per lane to M0 + 16*lane.  Inline
// asm, so the compiler neither tracks nor conservatively drains it; the caller
// waits with an explicit vmcnt.
__device__ __forceinline__ void dma16(uint32_t lds_byte, uint32_t voff, v4u srd, uint32_t soff) {
    uint32_t keep;  // M0 is compiler-reserved: save and restore it around the DMA
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %1\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "s"(lds_byte), "v"(voff), "s"(srd), "s"(soff)
        : "memory");
}

template <int A>
__device__ __forceinline__ void issue_dma(const CodewordSet& cs, const SetAddr& a, uint32_t lds_base) {
    const uint32_t k = cs.k, es = (uint32_t)cs.elem_stride;
    bs8::sfor<kPre>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t so = sym_off(16u * A + j, k, 0, es);
        dma16(lds_base + ((A * kPre + j) * 2 + 0) * 1024u, a.off[0], a.rs, so);
        dma16(lds_base + ((A * kPre + j) * 2 + 1) * 1024u, a.off[1], a.rs, so);
    });
}

template <int A>
__device__ __forceinline__ void issue_direct(const CodewordSet& cs, const SetAddr& a, uint32_t (&P)[16 - kPre][8]) {
    const uint32_t k = cs.k, es = (uint32_t)cs.elem_stride;
    const __amdgpu_buffer_rsrc_t rs = as_rsrc(a.rs);
    bs8::sfor<16 - kPre>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t so = sym_off(16u * A + kPre + j, k, 0, es);
        const v4u x = __builtin_amdgcn_raw_buffer_load_b128(rs, a.off[0], so, 0);
        const v4u y = __builtin_amdgcn_raw_buffer_load_b128(rs, a.off[1], so, 0);
        P[j][0] = x.x; P[j][1] = x.y; P[j][2] = x.z; P[j][3] = x.w;
        P[j][4] = y.x; P[j][5] = y.y; P[j][6] = y.z; P[j][7] = y.w;
    });
}

__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// LDS traffic as inline asm with immediate offsets: left to the compiler, the 32
// loop-invariant per-symbol addresses are hoisted out of the set loop into 16+
// VGPRs and the prefetch registers spill.  A read group waits for its own data
// (lgkmcnt(0) inside the statement), so the compiler never sees stale outputs.
template <uint32_t OFF>
__device__ __forceinline__ void ds_w16(uint32_t base, v4u v) {
    asm volatile("ds_write_b128 %0, %1 offset:%2" : : "v"(base), "v"(v), "i"(OFF) : "memory");
}
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

// Exchange buffer [symbol e][lane] x 16 B: byte e*1024 + 16*lane.  base0 covers
// e < 64, base1 = base0 + 64 KiB covers e >= 64 (ds offsets are 16-bit).
template <int A>
struct XLayout {
    // small layout e = 16A + j (all 16 symbols on one side of 64)
    static constexpr bool small_hi = A >= 4;
    static constexpr uint32_t small_off(int j) { return (uint32_t)((16 * A + j - (small_hi ? 64 : 0)) * 1024); }
    // large layout e = 8j + A: j < 8 on base0, j >= 8 on base1
    static constexpr uint32_t large_off(int j) { return (uint32_t)((8 * (j & 7) + A) * 1024); }
};

// Moves the 16 symbols of wave A between the small layout (e = 16A + j) and
// the large layout (e = 8j + A), 4 planes per round.
template <bool TO_LARGE, int A>
__device__ __forceinline__ void exchange(uint32_t (&X)[16][8], uint32_t base0) {
    using Lx = XLayout<A>;
    const uint32_t base1 = base0 + 65536u;
    const uint32_t bsmall = Lx::small_hi ? base1 : base0;
    bs8::sfor<2>([&](auto R) {
        constexpr int r = decltype(R)::value;
        bs8::sfor<16>([&](auto J) {
            constexpr int j = decltype(J)::value;
            v4u v;
            v.x = X[j][4 * r + 0]; v.y = X[j][4 * r + 1]; v.z = X[j][4 * r + 2]; v.w = X[j][4 * r + 3];
            if constexpr (TO_LARGE) ds_w16<Lx::small_off(j)>(bsmall, v);
            else ds_w16<Lx::large_off(j)>(j < 8 ? base0 : base1, v);
        });
        lds_barrier();
        v4u g[2][8];
        if constexpr (TO_LARGE) {
            ds_r16x8<Lx::large_off(0), 8192>(base0, g[0]);
            ds_r16x8<Lx::large_off(8), 8192>(base1, g[1]);
        } else {
            ds_r16x8<Lx::small_off(0), 1024>(bsmall, g[0]);
            ds_r16x8<Lx::small_off(8), 1024>(bsmall, g[1]);
        }
        bs8::sfor<16>([&](auto J) {
            constexpr int j = decltype(J)::value;
            const v4u v = g[j >> 3][j & 7];
            X[j][4 * r + 0] = v.x; X[j][4 * r + 1] = v.y; X[j][4 * r + 2] = v.z; X[j][4 * r + 3] = v.w;
        });
        lds_barrier();
    });
}

// The whole per-wave program for wave A (compile-time).  The set loop is rotated
// so that a set's direct loads are issued and consumed in one iteration (the
// compiler then counts them exactly: its waits leave the 32 stores of the
// previous set in flight); only the planes X and the LDS-DMA cross iterations.
//   iteration:  [issue direct loads of set t+G] small FFT(t), store(t)
//               | wait vmcnt(32): DMA + direct loads of t+G landed
//               | first half of t+G: read DMA, transpose, small IFFT, exchange,
//                 large layers, exchange back, DMA of t+2G.
template <int A>
__device__ __forceinline__ void bs_wave(const CodewordSet& cs, uint32_t sets, v4u* lds) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t lds_base = (uint32_t)(uintptr_t)lds;
    const uint32_t xbase = lds_base + lane * 16u;
    const uint32_t k = cs.k, es = (uint32_t)cs.elem_stride, oo = (uint32_t)cs.out_offset;
    const uint32_t G = gridDim.x;
    uint32_t X[16][8];
    uint32_t P[16 - kPre][8];

    // symbols of a set whose DMA and direct loads have landed -> planes -> the
    // first half of the transform, then the next-but-one set's DMA.
    auto first_half = [&](uint32_t t) __attribute__((always_inline)) {
        asm volatile("s_barrier" ::: "memory");  // every wave's DMA share has landed
        {
            v4u g[2][8];  // DMA buffer [wave][j][half][lane] x 16 B
            const uint32_t b = xbase + A * (kPre * 2048u);
            ds_r16x8<0, 1024>(b, g[0]);
            ds_r16x8<8192, 1024>(b, g[1]);
            bs8::sfor<kPre>([&](auto J) {
                constexpr int j = decltype(J)::value;
                const v4u x = g[(2 * j) >> 3][(2 * j) & 7], y = g[(2 * j + 1) >> 3][(2 * j + 1) & 7];
                X[j][0] = x.x; X[j][1] = x.y; X[j][2] = x.z; X[j][3] = x.w;
                X[j][4] = y.x; X[j][5] = y.y; X[j][6] = y.z; X[j][7] = y.w;
            });
        }
        bs8::sfor<16 - kPre>([&](auto J) {
            constexpr int j = decltype(J)::value;
            bs8::sfor<8>([&](auto I) { X[kPre + j][decltype(I)::value] = P[j][decltype(I)::value]; });
        });
        lds_barrier();  // DMA buffer consumed by every wave
        bs8::sfor<16>([&](auto J) { bs8::transpose8(X[decltype(J)::value]); });
        bs8::small_ifft<A>(X);
        exchange<true, A>(X, xbase);
        bs8::large_ifft_fft(X);
        exchange<false, A>(X, xbase);
        if (t + G < sets) issue_dma<A>(cs, set_addr(cs, t + G, lane), lds_base);
    };

    uint32_t t = blockIdx.x;
    {
        const SetAddr a = set_addr(cs, t, lane);
        issue_direct<A>(cs, a, P);
        issue_dma<A>(cs, a, lds_base);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    first_half(t);
    for (;;) {
        const uint32_t tn = t + G;
        const bool more = tn < sets;
        if (more) issue_direct<A>(cs, set_addr(cs, tn, lane), P);
        bs8::small_fft<A>(X);
        {
            const SetAddr a = set_addr(cs, t, lane);
            const __amdgpu_buffer_rsrc_t ro = as_rsrc(a.ro);
            bs8::sfor<16>([&](auto J) {
                constexpr int j = decltype(J)::value;
                bs8::transpose8(X[j]);
                const uint32_t so = sym_off(16u * A + j, k, oo, es);
                v4u x, y;
                x.x = X[j][0]; x.y = X[j][1]; x.z = X[j][2]; x.w = X[j][3];
                y.x = X[j][4]; y.y = X[j][5]; y.z = X[j][6]; y.w = X[j][7];
                __builtin_amdgcn_raw_buffer_store_b128(x, ro, a.off[0], so, 0);
                __builtin_amdgcn_raw_buffer_store_b128(y, ro, a.off[1], so, 0);
            });
        }
        if (!more) break;
        t = tn;
        // issue order: DMA(t) [16], direct(t) [16], stores(t - G) [32]
        asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
        first_half(t);
    }
}

}  // namespace

__global__ __launch_bounds__(512, 1) void encode_gf8_bs128_kernel(CodewordSet cs, uint32_t sets) {
    __shared__ v4u lds[128 * 64];
    if (blockIdx.x >= sets) return;
    switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {
        case 0: bs_wave<0>(cs, sets, lds); break;
        case 1: bs_wave<1>(cs, sets, lds); break;
        case 2: bs_wave<2>(cs, sets, lds); break;
        case 3: bs_wave<3>(cs, sets, lds); break;
        case 4: bs_wave<4>(cs, sets, lds); break;
        case 5: bs_wave<5>(cs, sets, lds); break;
        case 6: bs_wave<6>(cs, sets, lds); break;
        default: bs_wave<7>(cs, sets, lds); break;
    }
}

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

static uint32_t device_cus() {
    static const uint32_t n = [] {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        return (uint32_t)cus;
    }();
    return n;
}

hipError_t launch_encode_gf8_bs128(const CodewordSet& cs, hipStream_t st) {
    const uint64_t sets = ((uint64_t)cs.count * cs.S + kSetBytes - 1) / kSetBytes;
    if (sets == 0) return hipSuccess;
    const uint32_t grid = (uint32_t)(sets < device_cus() ? sets : device_cus());
    hipLaunchKernelGGL(encode_gf8_bs128_kernel, dim3(grid), dim3(512), 0, st, cs, (uint32_t)sets);
    return hipGetLastError();
}

}  // namespace rsm
