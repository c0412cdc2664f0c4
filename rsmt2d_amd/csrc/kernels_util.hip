// kernels_util.hip -- small device helpers: Repair fast-path comparisons and the
// synthetic-input generator used by benchmarks.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "rsm_kernels.hpp"

namespace rsm {

// Fills n bytes with the SplitMix64 stream of `seed` (word i = splitmix(seed + (i+1)*golden)),
// byte-identical to oracle.splitmix64_bytes.
__global__ __launch_bounds__(256) void fill_random_kernel(uint64_t* p, uint64_t nwords, uint64_t seed) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nwords; i += (uint64_t)gridDim.x * 256ull) {
        uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

hipError_t launch_fill_random(void* p, uint64_t bytes, uint64_t seed, hipStream_t st) {
    const uint64_t nwords = bytes / 8;
    if (nwords == 0) return hipSuccess;
    uint64_t blocks = (nwords + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(fill_random_kernel, dim3((uint32_t)blocks), dim3(256), 0, st, static_cast<uint64_t*>(p),
                       nwords, seed);
    return hipGetLastError();
}

// *mismatch |= any(a[i] != b[i]) over n bytes (n multiple of 16): the on-device
// form of verifyEncoding's bytes.Equal (extendeddatacrossword.go:496-500).
__global__ __launch_bounds__(256) void compare_kernel(const uint4* a, const uint4* b, uint64_t n16,
                                                      uint32_t* mismatch) {
    uint32_t diff = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256ull) {
        const uint4 x = a[i], y = b[i];
        diff |= (x.x ^ y.x) | (x.y ^ y.y) | (x.z ^ y.z) | (x.w ^ y.w);
    }
    // a plain store of 1 (the flag starts at 0): also valid when `mismatch` is host memory
    if (__any(diff != 0) && (threadIdx.x & 63u) == 0) *mismatch = 1u;
}

// dst = src, 16-byte words (the byte count rounded up): a pinned host buffer, through its
// device mapping, into device memory as a kernel on the caller's stream.  Repair stages
// its presence map and row list this way: a copy-engine transfer put a cross-engine
// wait of 10-16 us in front of the sweep kernel (profiles/r05ap_repair_stage.txt).
__global__ __launch_bounds__(256) void stage_copy_kernel(uint4* dst, const uint4* src, uint64_t n16) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256ull) dst[i] = src[i];
}

hipError_t launch_stage_copy(void* dst, const void* src, uint64_t bytes, hipStream_t st) {
    const uint64_t n16 = (bytes + 15) / 16;
    if (n16 == 0) return hipSuccess;
    uint64_t blocks = (n16 + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(stage_copy_kernel, dim3((uint32_t)blocks), dim3(256), 0, st, static_cast<uint4*>(dst),
                       static_cast<const uint4*>(src), n16);
    return hipGetLastError();
}

hipError_t launch_compare(const uint8_t* a, const uint8_t* b, uint64_t n, uint32_t* mismatch,
                          hipStream_t st) {
    const uint64_t n16 = n / 16;
    if (n16 == 0) return hipSuccess;
    uint64_t blocks = (n16 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(compare_kernel, dim3((uint32_t)blocks), dim3(256), 0, st,
                       reinterpret_cast<const uint4*>(a), reinterpret_cast<const uint4*>(b), n16, mismatch);
    return hipGetLastError();
}

// flags[q] = 1 iff the parity half (cells k..2k-1) of vector indices[q] differs
// between squares a and b (both [W][W][S]); one block per listed vector.
__global__ __launch_bounds__(256) void compare_parity_kernel(const uint8_t* a, const uint8_t* b, uint32_t k,
                                                             uint32_t S, uint32_t axis, const uint32_t* indices,
                                                             uint32_t* flags) {
    const uint32_t q = blockIdx.x;
    const uint64_t W = 2ull * k;
    const uint64_t vec = indices[q];
    const uint32_t per_cell = S / 16;
    uint32_t diff = 0;
    for (uint32_t t = threadIdx.x; t < k * per_cell; t += 256) {
        const uint64_t e = k + t / per_cell;
        const uint64_t cell = axis == 0 ? vec * W + e : e * W + vec;
        const uint64_t off = cell * S + (uint64_t)(t % per_cell) * 16;
        const uint4 x = *reinterpret_cast<const uint4*>(a + off);
        const uint4 y = *reinterpret_cast<const uint4*>(b + off);
        diff |= (x.x ^ y.x) | (x.y ^ y.y) | (x.z ^ y.z) | (x.w ^ y.w);
    }
    __shared__ uint32_t any;
    if (threadIdx.x == 0) any = 0;
    __syncthreads();
    if (diff) atomicOr(&any, 1u);
    __syncthreads();
    if (threadIdx.x == 0) flags[q] = any;
}

hipError_t launch_compare_parity(const uint8_t* a, const uint8_t* b, uint32_t k, uint32_t S, uint32_t axis,
                                 const uint32_t* indices, uint32_t count, uint32_t* flags, hipStream_t st) {
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(compare_parity_kernel, dim3(count), dim3(256), 0, st, a, b, k, S, axis, indices, flags);
    return hipGetLastError();
}

}  // namespace rsm
