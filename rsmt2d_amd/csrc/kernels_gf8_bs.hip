// kernels_gf8_bs.hip -- bit-sliced GF(2^8) encode for M = 128 (65 <= k <= 128).
//
// The byte-table kernel (kernels_gf8.hip) spends ~10 VALU per 4 bytes per GF
// multiply and is VALU-bound (SQ counters: ~98% of VALU issue cycles on the
// column pass).  Here 32 bytes of a symbol are 8 bit-planes and a multiply by a
// constant is ~16 VALU per 32 bytes (bs8.hpp).  A lane can hold 16 symbols x 8
// planes (128 VGPRs), not the whole 128-symbol codeword, so the transform is
// split between the 8 wavefronts of a workgroup (bs8.hpp):
//
//   workgroup = one "set": 64 lanes x 32 bytes = 2 KiB of share width (e.g. four
//   512-byte codewords), all 128 symbols of it;
//   wave w, small layout : symbols e = 16w + j (j = 0..15), IFFT layers d = 1,2,4
//                          (code specialised on w: wave-uniform branch, 8 variants)
//   LDS exchange         : 2 rounds x 4 planes, [symbol][lane] x 16 B = 128 KiB
//   wave w, large layout : symbols e = 8h + w (h = 0..15), IFFT d = 8..64 then
//                          FFT d = 64..8 (one code path for all waves)
//   LDS exchange back, FFT layers d = 4,2,1 (specialised), planes -> bytes, store.
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

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc_bs(const void* p) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void* u = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(u, (short)0, (int)kOobBs, 0x00020000);
}

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// Opaque point for all 128 planes: work cannot be hoisted above / sunk below it.
// Each variant brackets its code with fences carrying a distinct tag, so the
// compiler cannot pull the XOR halves the 8 variants have in common out of the
// switch (which makes them all live at once and spills).  The s_nop padding
// separates the hand-scheduled XOR block from the compiler's register copies at
// the switch merge: without it lanes 12-15 of every 16 read stale planes
// (measured on MI355X; the hazard recognizer cannot see into the asm).
template <int TAG>
__device__ __forceinline__ void fence_all(uint32_t (&X)[16][8]) {
#define RSM_BS_F(p)                                                                                         \
    asm volatile("; fence %16"                                                                             \
                 : "+v"(X[p][0]), "+v"(X[p][1]), "+v"(X[p][2]), "+v"(X[p][3]), "+v"(X[p][4]), "+v"(X[p][5]), \
                   "+v"(X[p][6]), "+v"(X[p][7]), "+v"(X[p + 1][0]), "+v"(X[p + 1][1]), "+v"(X[p + 1][2]),   \
                   "+v"(X[p + 1][3]), "+v"(X[p + 1][4]), "+v"(X[p + 1][5]), "+v"(X[p + 1][6]),               \
                   "+v"(X[p + 1][7])                                                                       \
                 : "i"(TAG));
    RSM_BS_F(0) RSM_BS_F(2) RSM_BS_F(4) RSM_BS_F(6) RSM_BS_F(8) RSM_BS_F(10) RSM_BS_F(12) RSM_BS_F(14)
#undef RSM_BS_F
}

template <bool INVERSE>
__device__ __forceinline__ void small_layers(uint32_t wv, uint32_t (&X)[16][8]) {
    switch (wv) {
#define RSM_BS_CASE(A)                                   \
    case A:                                              \
        fence_all<2 * A + 16 * INVERSE>(X); asm volatile("s_nop 7");                    \
        if constexpr (INVERSE) bs8::small_ifft<A>(X);    \
        else bs8::small_fft<A>(X);                       \
        asm volatile("s_nop 7"); fence_all<2 * A + 1 + 16 * INVERSE>(X);                   \
        break;
        RSM_BS_CASE(0) RSM_BS_CASE(1) RSM_BS_CASE(2) RSM_BS_CASE(3)
        RSM_BS_CASE(4) RSM_BS_CASE(5) RSM_BS_CASE(6) RSM_BS_CASE(7)
#undef RSM_BS_CASE
        default: __builtin_unreachable();
    }
}

// Moves the 16 symbols of this wave between the small layout (e = 16w + j) and
// the large layout (e = 8j + w).  lds: [128 symbols][64 lanes] x uint4.
template <bool TO_LARGE>
__device__ __forceinline__ void exchange(uint32_t (&X)[16][8], v4u* lds, uint32_t wv, uint32_t lane) {
    bs8::sfor<2>([&](auto R) {
        constexpr int r = decltype(R)::value;
        bs8::sfor<16>([&](auto J) {
            constexpr int j = decltype(J)::value;
            const uint32_t e = TO_LARGE ? 16u * wv + j : 8u * j + wv;
            v4u v;
            v.x = X[j][4 * r + 0]; v.y = X[j][4 * r + 1]; v.z = X[j][4 * r + 2]; v.w = X[j][4 * r + 3];
            lds[e * 64u + lane] = v;
        });
        __syncthreads();
        bs8::sfor<16>([&](auto J) {
            constexpr int j = decltype(J)::value;
            const uint32_t e = TO_LARGE ? 8u * j + wv : 16u * wv + j;
            const v4u v = lds[e * 64u + lane];
            X[j][4 * r + 0] = v.x; X[j][4 * r + 1] = v.y; X[j][4 * r + 2] = v.z; X[j][4 * r + 3] = v.w;
        });
        __syncthreads();
    });
}

}  // namespace

// Per-set addressing: a set is virtual bytes [2048 t, 2048 t + 2048) of the
// concatenated shares of the CodewordSet; lane l's two 16-byte pieces are at
// set bytes 16l and 1024 + 16l.  off[] are relative to the set's first codeword.
struct SetAddr {
    __amdgpu_buffer_rsrc_t rs, ro;
    uint32_t off[2];
};

__device__ __forceinline__ SetAddr set_addr(const CodewordSet& cs, uint32_t t, uint32_t lane) {
    SetAddr a;
    const uint32_t S = cs.S;
    const uint64_t v0 = (uint64_t)t * kSetBytes;
    const uint32_t q0 = __builtin_amdgcn_readfirstlane((uint32_t)(v0 / S));
    const uint32_t r0 = __builtin_amdgcn_readfirstlane((uint32_t)(v0 - (uint64_t)q0 * S));
    const uint64_t rel0 = cw_rel_bs(cs, q0);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint32_t v = r0 + 1024u * h + 16u * lane;  // < S + 2048
        const uint32_t dq = v / S;
        const uint32_t q = q0 + dq;
        const uint32_t o = v - dq * S;
        a.off[h] = q < cs.count ? (uint32_t)(cw_rel_bs(cs, q) - rel0) + o : kOobBs;
    }
    a.rs = make_rsrc_bs(cs.base + rel0);
    a.ro = make_rsrc_bs(cs.out_base + rel0);
    return a;
}

__device__ __forceinline__ uint32_t sym_off(uint32_t e, uint32_t k, uint32_t base, uint32_t es) {
    return __builtin_amdgcn_readfirstlane(e < k ? base + e * es : kOobBs);
}

// Symbols j < kPre of every wave's small-layout group are prefetched into LDS
// (LDS-DMA, no VGPRs) while the previous set finishes; the rest load to VGPRs.
// P layout: [wave][j][half][lane] x 16 B = 128 KiB, time-shared with the
// exchange buffer (P is consumed before the first exchange and refilled after
// the second).
constexpr int kPre = 8;

__device__ __forceinline__ void prefetch_set(const CodewordSet& cs, uint32_t t, uint32_t wv, uint32_t lane,
                                             v4u* lds) {
    const SetAddr a = set_addr(cs, t, lane);
    const uint32_t k = cs.k, es = (uint32_t)cs.elem_stride;
    bs8::sfor<kPre>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t so = sym_off(16u * wv + j, k, 0, es);
#pragma unroll
        for (int h = 0; h < 2; ++h)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                a.rs, (__attribute__((address_space(3))) void*)&lds[((wv * kPre + j) * 2 + h) * 64], 16, a.off[h],
                so, 0, 0);
    });
}

// Persistent: one workgroup per CU walks sets t = blockIdx.x, += gridDim.x.
__global__ __launch_bounds__(512, 1) void encode_gf8_bs128_kernel(CodewordSet cs, uint32_t sets) {
    __shared__ v4u lds[128 * 64];
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t k = cs.k;
    const uint32_t es = (uint32_t)cs.elem_stride;
    const uint32_t oo = (uint32_t)cs.out_offset;
    uint32_t t = blockIdx.x;
    if (t >= sets) return;
    prefetch_set(cs, t, wv, lane, lds);

    for (; t < sets; t += gridDim.x) {
        const SetAddr a = set_addr(cs, t, lane);
        uint32_t X[16][8];
        bs8::sfor<16 - kPre>([&](auto J) {
            constexpr int j = kPre + decltype(J)::value;
            const uint32_t so = sym_off(16u * wv + j, k, 0, es);
            const v4u x = __builtin_amdgcn_raw_buffer_load_b128(a.rs, a.off[0], so, 0);
            const v4u y = __builtin_amdgcn_raw_buffer_load_b128(a.rs, a.off[1], so, 0);
            X[j][0] = x.x; X[j][1] = x.y; X[j][2] = x.z; X[j][3] = x.w;
            X[j][4] = y.x; X[j][5] = y.y; X[j][6] = y.z; X[j][7] = y.w;
        });
        __syncthreads();  // prefetched symbols landed (waits on the LDS-DMA)
        bs8::sfor<kPre>([&](auto J) {
            constexpr int j = decltype(J)::value;
            const v4u x = lds[((wv * kPre + j) * 2 + 0) * 64 + lane];
            const v4u y = lds[((wv * kPre + j) * 2 + 1) * 64 + lane];
            X[j][0] = x.x; X[j][1] = x.y; X[j][2] = x.z; X[j][3] = x.w;
            X[j][4] = y.x; X[j][5] = y.y; X[j][6] = y.z; X[j][7] = y.w;
        });
        __syncthreads();  // P consumed before the exchange reuses it
        bs8::sfor<16>([&](auto J) { bs8::transpose8(X[decltype(J)::value]); });

        small_layers<true>(wv, X);
        exchange<true>(X, lds, wv, lane);
        bs8::large_ifft_fft(X);
        exchange<false>(X, lds, wv, lane);
        if (t + gridDim.x < sets) prefetch_set(cs, t + gridDim.x, wv, lane, lds);
        small_layers<false>(wv, X);

        bs8::sfor<16>([&](auto J) {
            constexpr int j = decltype(J)::value;
            bs8::transpose8(X[j]);
            const uint32_t so = sym_off(16u * wv + j, k, oo, es);
            v4u x, y;
            x.x = X[j][0]; x.y = X[j][1]; x.z = X[j][2]; x.w = X[j][3];
            y.x = X[j][4]; y.y = X[j][5]; y.z = X[j][6]; y.w = X[j][7];
            __builtin_amdgcn_raw_buffer_store_b128(x, a.ro, a.off[0], so, 0);
            __builtin_amdgcn_raw_buffer_store_b128(y, a.ro, a.off[1], so, 0);
        });
    }
}

// True when every offset the kernel forms stays below the buffer-resource limit
// (2^31): the set's codeword span + the largest symbol offset.
bool bs128_applicable(const CodewordSet& cs) {
    if (cs.indices != nullptr || ceil_pow2(cs.k) != 128) return false;
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
