// shaprobe.hip -- cycles per SHA-256 compression for one lone wave per SIMD, cold
// and warm instruction cache: what bounds the latency of tree_root_kernel
// (kernels_sha.hip).  Each wave runs `nblk` compressions of sha256_dev.hpp's
// sha_block in a loop (one code copy: the first iteration runs cold, the rest
// warm), then the same count through a second, distinct code copy (a compression
// on a different constant message layout), stamping s_memtime after each.
// usage: shaprobe <blocks> <threads per block> <nblk>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../rsmt2d_amd/csrc/sha256_dev.hpp"

using namespace rsm;

__global__ void probe(uint32_t* __restrict__ stamps, uint32_t* __restrict__ sink, int nblk, uint32_t active,
                      uint32_t distinct) {
    uint32_t h[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = kH0[i] ^ (threadIdx.x % distinct);
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t* st = stamps + (size_t)wave * (2 * nblk + 4);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    for (int b = 0; b < nblk; ++b) {
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = h[i & 7] + i;
        if (lane < active) sha_block(h, w);
        const uint64_t t = __builtin_amdgcn_s_memtime();
        if (lane == 0) st[b] = (uint32_t)(t - t0);
    }
    for (int b = 0; b < nblk; ++b) {  // second copy: half the message constant
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = h[i] ^ 0x5a5a5a5au;
        w[8] = 0x80000000u;
#pragma unroll
        for (int i = 9; i < 15; ++i) w[i] = 0;
        w[15] = 256;
        if (lane < active) sha_block(h, w);
        const uint64_t t = __builtin_amdgcn_s_memtime();
        if (lane == 0) st[nblk + b] = (uint32_t)(t - t0);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        st[2 * nblk] = (uint32_t)(t1 - t0);
        st[2 * nblk + 1] = (uint32_t)(r1 - r0);
        st[2 * nblk + 2] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
        st[2 * nblk + 3] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) x ^= h[i];
    sink[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 1;
    const int threads = argc > 2 ? atoi(argv[2]) : 64;
    const int nblk = argc > 3 ? atoi(argv[3]) : 8;
    const uint32_t active = argc > 4 ? (uint32_t)atoi(argv[4]) : 64u;
    const uint32_t distinct = argc > 5 ? (uint32_t)atoi(argv[5]) : 1024u;  // lanes with distinct data
    if (threads % 64 || threads > 1024 || blocks < 1 || blocks > 4096 || nblk < 1 || nblk > 256) return 2;
    const int waves = blocks * threads / 64;
    uint32_t *d_st, *d_sink;
    if (hipMalloc(&d_st, (size_t)waves * (2 * nblk + 4) * 4) != hipSuccess) return 1;
    if (hipMalloc(&d_sink, (size_t)blocks * threads * 4) != hipSuccess) return 1;
    for (int rep = 0; rep < 3; ++rep) {
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        hipEventRecord(a, 0);
        hipLaunchKernelGGL(probe, dim3(blocks), dim3(threads), 0, 0, d_st, d_sink, nblk, active, distinct ? distinct : 1u);
        hipEventRecord(b, 0);
        if (hipEventSynchronize(b) != hipSuccess) return 1;
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        std::vector<uint32_t> st((size_t)waves * (2 * nblk + 4));
        hipMemcpy(st.data(), d_st, st.size() * 4, hipMemcpyDeviceToHost);
        // per-iteration deltas, averaged over waves
        std::vector<double> d1(nblk, 0), d2(nblk, 0);
        for (int wv = 0; wv < waves; ++wv) {
            const uint32_t* s = &st[(size_t)wv * (2 * nblk + 4)];
            for (int i = 0; i < nblk; ++i) {
                d1[i] += (i ? s[i] - s[i - 1] : s[0]);
                d2[i] += s[nblk + i] - (i ? s[nblk + i - 1] : s[nblk - 1]);
            }
        }
        printf("rep %d blocks %d threads %d nblk %d active lanes %u distinct %u: %.1f us;  copy1 ticks/compression:", rep,
               blocks, threads, nblk, active, distinct, ms * 1e3);
        for (int i = 0; i < nblk && i < 6; ++i) printf(" %.0f", d1[i] / waves);
        printf(" ... %.0f;  copy2:", d1[nblk - 1] / waves);
        for (int i = 0; i < nblk && i < 6; ++i) printf(" %.0f", d2[i] / waves);
        printf(" ... %.0f\n", d2[nblk - 1] / waves);
        if (waves <= 8)
            for (int wv = 0; wv < waves; ++wv) {
                const uint32_t* s = &st[(size_t)wv * (2 * nblk + 4)];
                printf("   wave %2d xcc %u cu %2u simd %u: memtime %u realtime %u (100 MHz) -> %.2f GHz\n", wv,
                       s[2 * nblk + 2] & 15u, (s[2 * nblk + 3] >> 8) & 15u, (s[2 * nblk + 3] >> 4) & 3u, s[2 * nblk],
                       s[2 * nblk + 1], s[2 * nblk + 1] ? 0.1 * s[2 * nblk] / s[2 * nblk + 1] : 0.0);
            }
    }
    return 0;
}
