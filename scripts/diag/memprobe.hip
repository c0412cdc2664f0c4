// memprobe.hip -- diagnostic (NOT part of librsmt2d_hip.so): HBM rate of the 2D
// extension's access patterns with no arithmetic, to find which shapes and which
// per-CU structure stream at the chip's ~6 TB/s.  A "set" is what one 8-wave
// workgroup of the GF(2^8) M = 128 kernel moves: 128 symbols x 2 KiB in, 128
// symbols x 2 KiB out.  Each symbol's 2 KiB is runs of R bytes:
//   run i of symbol e of set t = base + sq * SQ + e * ES + i * RS + (t % SPS) * TS
// with sq = t / SPS; the output goes to the same offsets + OUT.
// Usage: memprobe <name> R ES RS TS SPS OUT nsets order mode wg_per_cu [square_MiB [J]]
//   order 0: set t = block + i * grid (strided, as the production kernel)
//   order 1: consecutive sets per workgroup (block * n + i)
//   mode bits: 1 = software pipeline (load set t+G before storing set t),
//              2 = non-temporal loads, 4 = non-temporal stores,
//              8 = read only, 16 = write only
// Prints one JSON line per configuration.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

struct P {
    uint8_t* base;
    uint32_t* sink;
    uint64_t SQ, ES, RS, TS, OUT;
    uint32_t R, SPS, nsets, order;
};

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t run_off(const P& p, uint32_t t, uint32_t e, uint32_t byte) {
    const uint32_t i = byte / p.R, o = byte - i * p.R;
    const uint64_t sq = t / p.SPS;
    return sq * p.SQ + (uint64_t)e * p.ES + (uint64_t)i * p.RS + (uint64_t)(t % p.SPS) * p.TS + o;
}

// J symbols per wave, 128 / J waves per workgroup; PRE of the J symbols are
// prefetched one set ahead in software-pipelined modes
template <int MODE, int J, int N>
__device__ __forceinline__ void load_set(const P& p, uint32_t t, uint32_t A, uint32_t lane, v4u (&X)[N][2], int j0) {
#pragma unroll
    for (int j = 0; j < N; ++j)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint64_t off = run_off(p, t, J * A + j0 + j, 1024u * h + 16u * lane);
            const v4u* q = reinterpret_cast<const v4u*>(p.base + off);
            X[j][h] = (MODE & 2) ? __builtin_nontemporal_load(q) : *q;
        }
}
template <int MODE, int J, int N>
__device__ __forceinline__ void store_set(const P& p, uint32_t t, uint32_t A, uint32_t lane, const v4u (&X)[N][2],
                                          int j0) {
#pragma unroll
    for (int j = 0; j < N; ++j)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint64_t off = run_off(p, t, J * A + j0 + j, 1024u * h + 16u * lane) + p.OUT;
            v4u* q = reinterpret_cast<v4u*>(p.base + off);
            if (MODE & 4) __builtin_nontemporal_store(X[j][h], q);
            else *q = X[j][h];
        }
}

template <int MODE, int J>
__global__ __launch_bounds__(64 * (128 / J)) void probe(P p) {
    constexpr int PRE = J == 16 ? 8 : J;
    extern __shared__ uint32_t pad[];
    if (threadIdx.x == 0xFFFF) pad[0] = 0;
    const uint32_t lane = threadIdx.x & 63u, A = threadIdx.x >> 6;
    const uint32_t G = gridDim.x;
    const uint32_t per = (p.nsets + G - 1) / G;
    auto set_of = [&](uint32_t n) -> uint32_t {
        const uint32_t t = p.order ? blockIdx.x * per + n : blockIdx.x + n * G;
        const bool ok = p.order ? (n < per && t < p.nsets) : t < p.nsets;
        return ok ? t : 0xFFFFFFFFu;
    };
    v4u X[J][2], Y[PRE][2];
    uint32_t acc = 0;
    uint32_t t = set_of(0);
    if (t == 0xFFFFFFFFu) return;
    if (!(MODE & 16)) load_set<MODE, J>(p, t, A, lane, X, 0);
    else
        for (int j = 0; j < J; ++j) X[j][0] = X[j][1] = v4u{lane, (uint32_t)j, t, 1u};
    for (uint32_t n = 1;; ++n) {
        const uint32_t tn = set_of(n);
        const bool more = tn != 0xFFFFFFFFu;
        if ((MODE & 1) && more && !(MODE & 16)) load_set<MODE, J>(p, tn, A, lane, Y, 0);
        if (MODE & 8) {
#pragma unroll
            for (int j = 0; j < J; ++j) acc ^= X[j][0].x ^ X[j][1].w;
        } else {
            store_set<MODE, J>(p, t, A, lane, X, 0);
        }
        if (!more) break;
        if (!(MODE & 16)) {
            if (MODE & 1) {
#pragma unroll
                for (int j = 0; j < PRE; ++j) X[j][0] = Y[j][0], X[j][1] = Y[j][1];
                if constexpr (PRE < J) {
                    v4u Z[J - PRE][2];
                    load_set<MODE, J>(p, tn, A, lane, Z, PRE);
#pragma unroll
                    for (int j = 0; j < J - PRE; ++j) X[PRE + j][0] = Z[j][0], X[PRE + j][1] = Z[j][1];
                }
            } else {
                load_set<MODE, J>(p, tn, A, lane, X, 0);
            }
        }
        t = tn;
    }
    if ((MODE & 8) && acc == 0x12345678u) p.sink[threadIdx.x] = acc;
}

int main(int argc, char** argv) {
    if (argc < 12) {
        fprintf(stderr, "usage: memprobe name R ES RS TS SPS OUT nsets order mode wg_per_cu\n");
        return 2;
    }
    P p{};
    const char* name = argv[1];
    p.R = atoi(argv[2]);
    p.ES = strtoull(argv[3], 0, 0);
    p.RS = strtoull(argv[4], 0, 0);
    p.TS = strtoull(argv[5], 0, 0);
    p.SPS = atoi(argv[6]);
    p.OUT = strtoull(argv[7], 0, 0);
    p.nsets = atoi(argv[8]);
    p.order = atoi(argv[9]);
    const int mode = atoi(argv[10]);
    const int wgcu = atoi(argv[11]);
    const int J = argc > 13 ? atoi(argv[13]) : 16;  // symbols per wave (16: 8 waves, 8: 16 waves)
    p.SQ = (argc > 12 ? strtoull(argv[12], 0, 0) : 32ull) << 20;  // square stride (C2: 32 MiB)
    if (p.R == 0 || 2048 % p.R != 0 || p.SPS == 0 || wgcu < 1 || wgcu > 4 || (J != 16 && J != 8)) {
        fprintf(stderr, "bad arguments\n");
        return 2;
    }
    // host-side bound check of every offset the kernel forms (no faulting probes)
    const uint64_t nr = 2048 / p.R;
    const uint64_t maxin = (uint64_t)(p.SPS - 1) * p.TS + 127 * p.ES + (nr - 1) * p.RS + p.R;
    if (maxin + p.OUT > p.SQ) {
        fprintf(stderr, "%s: offsets exceed the square (%llu > %llu)\n", name,
                (unsigned long long)(maxin + p.OUT), (unsigned long long)p.SQ);
        return 2;
    }
    const uint32_t nsq = (p.nsets + p.SPS - 1) / p.SPS;
    const size_t bytes = (size_t)nsq * p.SQ;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint8_t* buf[2];
    for (auto& b : buf) {
        CK(hipMalloc(&b, bytes));
        CK(hipMemset(b, 1, bytes));
    }
    CK(hipMalloc(&p.sink, 4096));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint32_t grid = std::min<uint32_t>(p.nsets, cus * wgcu);
    const size_t lds = (160 * 1024) / wgcu - 1024;
    auto launch = [&]() {
        switch (mode) {
#define M(m)                                                                                            \
    case m:                                                                                             \
        if (J == 16) hipLaunchKernelGGL((probe<m, 16>), dim3(grid), dim3(512), lds, 0, p);              \
        else hipLaunchKernelGGL((probe<m, 8>), dim3(grid), dim3(1024), lds, 0, p);                      \
        break;
            M(0) M(1) M(2) M(3) M(6) M(7) M(8) M(10) M(16) M(20)
#undef M
            default: fprintf(stderr, "mode %d not built\n", mode); exit(2);
        }
    };
    std::vector<float> ts;
    for (int r = 0; r < 24; ++r) {
        p.base = buf[r & 1];
        CK(hipEventRecord(e0, 0));
        launch();
        CK(hipGetLastError());
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 4) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const double med = ts[ts.size() / 2];
    const double moved = (double)p.nsets * ((mode & 24) ? 1 : 2) * 128 * 2048;
    printf("{\"probe\": \"%s\", \"J\": %d, \"mode\": %d, \"wg_per_cu\": %d, \"R\": %u, \"ES\": %llu, \"RS\": %llu, \"TS\": %llu, "
           "\"SPS\": %u, \"nsets\": %u, \"order\": %u, \"grid\": %u, \"us_median\": %.2f, \"us_min\": %.2f, "
           "\"TB_s\": %.3f}\n",
           name, J, mode, wgcu, p.R, (unsigned long long)p.ES, (unsigned long long)p.RS, (unsigned long long)p.TS, p.SPS,
           p.nsets, p.order, grid, med * 1e3, ts[0] * 1e3, moved / (med * 1e-3) / 1e12);
    fflush(stdout);
    for (auto& b : buf) CK(hipFree(b));
    return 0;
}
