// mixprobe.hip -- diagnostic (NOT part of librsmt2d_hip.so): the HBM ceiling of the
// 2D extension's ALGORITHMIC traffic with no re-reads and no arithmetic.  For every
// row r < k of every square: read the Q0 row (k*S contiguous bytes) and write the
// Q1 row, the Q2 row r and the Q3 row r (3 x k*S): exactly 4k^2 S per square, the
// best any schedule of the extension can move.
// Usage: mixprobe <squares> <wg_per_cu> <mode> [threads] [launches]
//   mode bits: 1 = non-temporal loads, 2 = non-temporal stores, 4 = sc1 stores,
//              8 = read only (no stores), 16 = write only (no loads)
// Prints one JSON line: us per square, algorithmic TB/s and fraction of 8 TB/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr uint32_t K = 128, S = 512, W = 2 * K;
constexpr uint64_t SQ = (uint64_t)W * W * S, ROW = (uint64_t)W * S, HALF = (uint64_t)K * S;
constexpr int U = 8;  // 16-B pieces per thread in flight per row chunk

template <int MODE>
__global__ void mix(uint8_t* base, uint32_t units, uint32_t* sink) {
    const uint32_t nthr = blockDim.x;
    uint32_t acc = 0;
    for (uint32_t u = blockIdx.x; u < units; u += gridDim.x) {
        const uint32_t sq = u / K, r = u % K;
        uint8_t* q0 = base + sq * SQ + r * ROW;  // Q0 row r
        uint8_t* q1 = q0 + HALF;                 // Q1 row r
        uint8_t* q2 = base + sq * SQ + (K + r) * ROW;
        uint8_t* q3 = q2 + HALF;
        for (uint32_t c = threadIdx.x * 16; c < HALF; c += nthr * 16 * U) {
            v4u x[U];
#pragma unroll
            for (int i = 0; i < U; ++i) {
                const uint32_t o = c + i * nthr * 16;
                if (MODE & 16) x[i] = v4u{o, r, sq, 1u};
                else if (MODE & 1) x[i] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(q0 + o));
                else x[i] = *reinterpret_cast<const v4u*>(q0 + o);
            }
            if (MODE & 8) {
#pragma unroll
                for (int i = 0; i < U; ++i) acc ^= x[i].x ^ x[i].w;
                continue;
            }
#pragma unroll
            for (int i = 0; i < U; ++i) {
                const uint32_t o = c + i * nthr * 16;
                uint8_t* dst[3] = {q1 + o, q2 + o, q3 + o};
#pragma unroll
                for (int d = 0; d < 3; ++d) {
                    v4u* p = reinterpret_cast<v4u*>(dst[d]);
                    v4u y = x[i] ^ v4u{(uint32_t)d, 0u, 0u, 0u};
                    if (MODE & 2) __builtin_nontemporal_store(y, p);
                    else if (MODE & 4) __builtin_amdgcn_raw_buffer_store_b128(
                        y, __builtin_amdgcn_make_buffer_rsrc(dst[d], (short)0, 0x7FFFFFFF, 0x00020000), 0, 0, 16);
                    else *p = y;
                }
            }
        }
    }
    if ((MODE & 8) && acc == 0x12345678u) sink[threadIdx.x] = acc;
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: mixprobe squares wg_per_cu mode [threads]\n");
        return 2;
    }
    const uint32_t nsq = atoi(argv[1]);
    const int wgcu = atoi(argv[2]), mode = atoi(argv[3]);
    const int thr = argc > 4 ? atoi(argv[4]) : 512;
    const int reps = argc > 5 ? atoi(argv[5]) : 16;  // launches (the first 3 untimed)
    if (nsq == 0 || nsq > 512 || wgcu < 1 || wgcu > 8 || thr < 64 || thr > 1024 || thr % 64) {
        fprintf(stderr, "bad arguments\n");
        return 2;
    }
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const size_t bytes = (size_t)nsq * SQ;
    uint8_t* buf[3];
    for (auto& b : buf) {
        CK(hipMalloc(&b, bytes));
        CK(hipMemset(b, 1, bytes));
    }
    uint32_t* sink;
    CK(hipMalloc(&sink, 4096 * 4));
    const uint32_t units = nsq * K;
    const uint32_t grid = std::min<uint32_t>(units, cus * wgcu);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto launch = [&](uint8_t* b) {
        switch (mode) {
#define M(m) case m: hipLaunchKernelGGL((mix<m>), dim3(grid), dim3(thr), 0, 0, b, units, sink); break;
            M(0) M(1) M(2) M(3) M(4) M(5) M(8) M(9) M(16) M(18) M(20)
#undef M
            default: fprintf(stderr, "mode %d not built\n", mode); exit(2);
        }
    };
    std::vector<float> ts;
    for (int r = 0; r < (reps > 4 ? reps : 4); ++r) {
        CK(hipEventRecord(e0, 0));
        launch(buf[r % 3]);
        CK(hipGetLastError());
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 3) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const double med = ts[ts.size() / 2] * 1e-3;
    const double moved = (double)nsq * ((mode & 8) ? 1 : (mode & 16) ? 3 : 4) * K * K * S;
    printf("{\"probe\": \"mix\", \"squares\": %u, \"wg_per_cu\": %d, \"threads\": %d, \"mode\": %d, \"grid\": %u, "
           "\"us_per_square\": %.3f, \"TB_s\": %.3f, \"frac_of_8TBs_algorithmic\": %.4f}\n",
           nsq, wgcu, thr, mode, grid, med / nsq * 1e6, moved / med / 1e12, 4.0 * K * K * S * nsq / med / 8e12);
    fflush(stdout);
    for (auto& b : buf) CK(hipFree(b));
    return 0;
}
