// lutprobe.hip -- diagnostic: throughput of the GF(2^16) multiply-accumulate forms on one
// CU shape (512-thread workgroups, two per CU = 4 waves per SIMD, as enc16h_kernel):
//   form 0  perm:  12 v_perm_b32 lookups in VGPR tables (production muladd16v, 64-bit
//                  selector shifts)
//   form 1  lds:   split u16 tables in LDS, T_lo[yl byte] ^ T_hi[yh byte]: 8 addresses by
//                  v_add_u32_sdwa (2 * byte), 8 ds_read_u16_d16(_hi) packing two products
//                  per dword, 2 XOR + 2 v_perm to the lo/hi dword layout
//   form 2..7  the first F of every 8 butterflies through LDS, the rest perm
// Each thread runs 8 butterflies (x ^= y c; y ^= x) per iteration over 16 register pairs.
// Prints one JSON line per form: ns per wave-butterfly per CU and the speed-up over perm.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++20 -o scripts/diag/lutprobe scripts/diag/lutprobe.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
__device__ __forceinline__ uint32_t pm(uint32_t hi, uint32_t lo, uint32_t sel) { return __builtin_amdgcn_perm(hi, lo, sel); }

__device__ __forceinline__ void muladd_perm(uint32_t& xl, uint32_t& xh, uint32_t yl, uint32_t yh, const uint32_t (&c)[20]) {
    const uint64_t y = ((uint64_t)yh << 32) | yl;
    uint64_t y3, y6;
    asm("v_lshrrev_b64 %0, 3, %1" : "=v"(y3) : "v"(y));
    asm("v_lshrrev_b64 %0, 6, %1" : "=v"(y6) : "v"(y));
    const uint32_t sa = yl & 0x07070707u, sb = (uint32_t)y3 & 0x07070707u, sc = (uint32_t)y6 & 0x03030303u;
    const uint32_t sd = yh & 0x07070707u, se = (uint32_t)(y3 >> 32) & 0x07070707u, sf = (uint32_t)(y6 >> 32) & 0x03030303u;
    xl = x3(x3(xl, pm(c[1], c[0], sa), pm(c[5], c[4], sb)), x3(pm(c[8], c[8], sc), pm(c[11], c[10], sd), pm(c[15], c[14], se)),
            pm(c[18], c[18], sf));
    xh = x3(x3(xh, pm(c[3], c[2], sa), pm(c[7], c[6], sb)), x3(pm(c[9], c[9], sc), pm(c[13], c[12], sd), pm(c[17], c[16], se)),
            pm(c[19], c[19], sf));
}

// two multiply-accumulates through the LDS split tables at byte offset OFF (T_lo at OFF,
// T_hi at OFF + 512): all 16 reads in flight, one wait
template <int OFF>
__device__ __forceinline__ void muladd_lds2(uint32_t& xl0, uint32_t& xh0, uint32_t yl0, uint32_t yh0, uint32_t& xl1,
                                            uint32_t& xh1, uint32_t yl1, uint32_t yh1) {
    uint32_t a0, a1, a2, a3, b0, b1, b2, b3, c0, c1, c2, c3, d0, d1, d2, d3;
    asm volatile(
        "v_add_u32_sdwa %0, %16, %16 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
        "v_add_u32_sdwa %2, %16, %16 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:BYTE_2\n\t"
        "v_add_u32_sdwa %1, %16, %16 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_1\n\t"
        "v_add_u32_sdwa %3, %16, %16 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:BYTE_3\n\t"
        "ds_read_u16_d16 %0, %0 offset:%20\n\t"
        "ds_read_u16_d16_hi %0, %2 offset:%20\n\t"
        "ds_read_u16_d16 %1, %1 offset:%20\n\t"
        "ds_read_u16_d16_hi %1, %3 offset:%20\n\t"
        "v_add_u32_sdwa %4, %17, %17 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
        "v_add_u32_sdwa %6, %17, %17 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:BYTE_2\n\t"
        "v_add_u32_sdwa %5, %17, %17 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_1\n\t"
        "v_add_u32_sdwa %7, %17, %17 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:BYTE_3\n\t"
        "ds_read_u16_d16 %4, %4 offset:%21\n\t"
        "ds_read_u16_d16_hi %4, %6 offset:%21\n\t"
        "ds_read_u16_d16 %5, %5 offset:%21\n\t"
        "ds_read_u16_d16_hi %5, %7 offset:%21\n\t"
        "v_add_u32_sdwa %8, %18, %18 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
        "v_add_u32_sdwa %10, %18, %18 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:BYTE_2\n\t"
        "v_add_u32_sdwa %9, %18, %18 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_1\n\t"
        "v_add_u32_sdwa %11, %18, %18 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:BYTE_3\n\t"
        "ds_read_u16_d16 %8, %8 offset:%20\n\t"
        "ds_read_u16_d16_hi %8, %10 offset:%20\n\t"
        "ds_read_u16_d16 %9, %9 offset:%20\n\t"
        "ds_read_u16_d16_hi %9, %11 offset:%20\n\t"
        "v_add_u32_sdwa %12, %19, %19 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
        "v_add_u32_sdwa %14, %19, %19 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:BYTE_2\n\t"
        "v_add_u32_sdwa %13, %19, %19 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_1\n\t"
        "v_add_u32_sdwa %15, %19, %19 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:BYTE_3\n\t"
        "ds_read_u16_d16 %12, %12 offset:%21\n\t"
        "ds_read_u16_d16_hi %12, %14 offset:%21\n\t"
        "ds_read_u16_d16 %13, %13 offset:%21\n\t"
        "ds_read_u16_d16_hi %13, %15 offset:%21\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(a0), "=&v"(a1), "=&v"(a2), "=&v"(a3), "=&v"(b0), "=&v"(b1), "=&v"(b2), "=&v"(b3), "=&v"(c0), "=&v"(c1),
          "=&v"(c2), "=&v"(c3), "=&v"(d0), "=&v"(d1), "=&v"(d2), "=&v"(d3)
        : "v"(yl0), "v"(yh0), "v"(yl1), "v"(yh1), "i"(OFF), "i"(OFF + 512)
        : "memory");
    // a0 = [p(b0) | p(b2)], a1 = [p(b1) | p(b3)] from T_lo; b0, b1 likewise from T_hi
    const uint32_t r1 = a0 ^ b0, r2 = a1 ^ b1, s1 = c0 ^ d0, s2 = c1 ^ d1;
    xl0 ^= pm(r2, r1, 0x06020400u);
    xh0 ^= pm(r2, r1, 0x07030501u);
    xl1 ^= pm(s2, s1, 0x06020400u);
    xh1 ^= pm(s2, s1, 0x07030501u);
}

template <int F>  // butterflies of 8 through LDS (F = 8: all)
__global__ __launch_bounds__(512, 4) void probe(uint32_t iters, const uint32_t* tabs, const uint16_t* lut, uint32_t* sink) {
    __shared__ uint16_t T[4096];  // 4 split tables (lo + hi)
    for (uint32_t i = threadIdx.x; i < 4096; i += 512) T[i] = lut[i];
    uint32_t c[20];
    for (int i = 0; i < 20; ++i) c[i] = tabs[i];
    __syncthreads();
    uint32_t l[16], h[16];
    for (int i = 0; i < 16; ++i) {
        l[i] = (threadIdx.x + 1u) * 2654435761u + (uint32_t)i * 0x9E3779B9u;
        h[i] = l[i] * 0x85EBCA6Bu + 0xC2B2AE35u;
    }
    for (uint32_t n = 0; n < iters; ++n) {
#pragma unroll
        for (int b = 0; b < 8; b += 2) {
            if (b < F) {
                muladd_lds2<0>(l[b], h[b], l[b + 8], h[b + 8], l[b + 1], h[b + 1], l[b + 9], h[b + 9]);
            } else {
                muladd_perm(l[b], h[b], l[b + 8], h[b + 8], c);
                muladd_perm(l[b + 1], h[b + 1], l[b + 9], h[b + 9], c);
            }
            l[b + 8] ^= l[b];
            h[b + 8] ^= h[b];
            l[b + 9] ^= l[b + 1];
            h[b + 9] ^= h[b + 1];
        }
#pragma unroll
        for (int b = 0; b < 8; ++b) {  // rotate roles so every register is a multiplier input
            const uint32_t tl = l[b], th = h[b];
            l[b] = l[b + 8];
            h[b] = h[b + 8];
            l[b + 8] = tl;
            h[b + 8] = th;
        }
    }
    uint32_t acc = 0;
    for (int i = 0; i < 16; ++i) acc ^= l[i] ^ h[i];
    sink[blockIdx.x * 512 + threadIdx.x] = acc;
}

template <int F>
static void run(int cus, uint32_t iters, const uint32_t* tabs, const uint16_t* lut, uint32_t* sink, hipEvent_t e0,
                hipEvent_t e1, double* base) {
    std::vector<float> ts;
    for (int r = 0; r < 7; ++r) {
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(probe<F>, dim3(2 * cus), dim3(512), 0, 0, iters, tabs, lut, sink);
        CK(hipGetLastError());
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 2) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const double us = ts[ts.size() / 2] * 1e3;
    // wave-butterflies per CU: 16 waves x iters x 8
    const double ns = us * 1e3 / (16.0 * iters * 8);
    if (F == 0) *base = ns;
    printf("{\"probe\": \"lut16\", \"lds_share\": %.3f, \"us\": %.1f, \"ns_per_wave_butterfly_cu\": %.4f, \"speedup\": %.3f}\n",
           F / 8.0, us, ns, *base / ns);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const uint32_t iters = argc > 1 ? atoi(argv[1]) : 4096;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t *tabs, *sink;
    uint16_t* lut;
    CK(hipMalloc(&tabs, 20 * 4));
    CK(hipMalloc(&lut, 4096 * 2));
    CK(hipMalloc(&sink, (size_t)2 * cus * 512 * 4));
    std::vector<uint32_t> ht(20);
    std::vector<uint16_t> hl(4096);
    uint32_t s = 12345;
    for (auto& v : ht) v = (s = s * 1664525u + 1013904223u);
    for (auto& v : hl) v = (uint16_t)((s = s * 1664525u + 1013904223u) >> 16);
    CK(hipMemcpy(tabs, ht.data(), 80, hipMemcpyHostToDevice));
    CK(hipMemcpy(lut, hl.data(), 8192, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    double base = 0;
    run<0>(cus, iters, tabs, lut, sink, e0, e1, &base);
    run<2>(cus, iters, tabs, lut, sink, e0, e1, &base);
    run<4>(cus, iters, tabs, lut, sink, e0, e1, &base);
    run<6>(cus, iters, tabs, lut, sink, e0, e1, &base);
    run<8>(cus, iters, tabs, lut, sink, e0, e1, &base);
    return 0;
}
