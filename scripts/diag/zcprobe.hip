// zcprobe.hip -- diagnostic only (not part of the product): PCIe rates of
// GPU-initiated reads/writes of mapped host memory ("zero-copy") by allocation
// flag and access width, next to copy-engine H2D/D2H, to size the Repair fast
// path's transport (rsmt2d_amd/csrc/eds.cpp).  Prints one JSON line per case.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

typedef unsigned v4u __attribute__((ext_vector_type(4)));

// each wave reads `per_wave` bytes: W = 4 (dword) or 16 (dwordx4) bytes per lane per load
template <int W>
__global__ __launch_bounds__(256) void zc_read(const unsigned char* __restrict__ src, size_t bytes, unsigned* out) {
    const size_t nthreads = (size_t)gridDim.x * blockDim.x;
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned acc = 0;
    if constexpr (W == 4) {
        const unsigned* p = reinterpret_cast<const unsigned*>(src);
        for (size_t i = tid; i < bytes / 4; i += nthreads) acc ^= __builtin_nontemporal_load(p + i);
    } else {
        const v4u* p = reinterpret_cast<const v4u*>(src);
        for (size_t i = tid; i < bytes / 16; i += nthreads) {
            v4u v = p[i];
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int W>
__global__ __launch_bounds__(256) void zc_write(unsigned char* __restrict__ dst, size_t bytes) {
    const size_t nthreads = (size_t)gridDim.x * blockDim.x;
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if constexpr (W == 4) {
        unsigned* p = reinterpret_cast<unsigned*>(dst);
        for (size_t i = tid; i < bytes / 4; i += nthreads) p[i] = (unsigned)i;
    } else {
        v4u* p = reinterpret_cast<v4u*>(dst);
        for (size_t i = tid; i < bytes / 16; i += nthreads) p[i] = v4u{(unsigned)i, 1u, 2u, 3u};
    }
}

// 256 B of every 512 B (one chunk of each 512-B cell, as a decode block reads a row)
__global__ __launch_bounds__(256) void zc_read_strided(const unsigned char* __restrict__ src, size_t bytes, unsigned* out) {
    const size_t nthreads = (size_t)gridDim.x * blockDim.x;
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned* p = reinterpret_cast<const unsigned*>(src);
    unsigned acc = 0;
    for (size_t i = tid; i < bytes / 8; i += nthreads) acc ^= p[(i / 64) * 128 + (i % 64)];
    if (acc == 0x12345678u) out[0] = acc;
}

// The Repair decoder's pattern: workgroup = (row, 256-B chunk), 4 waves x 64 cells
// of 512 B; a wave reads its chunk of the present cells (half, random) and, when
// `write`, stores the chunk of each missing cell.
__global__ __launch_bounds__(256) void zc_row_pattern(unsigned char* __restrict__ sq, const unsigned char* pres,
                                                      int write, unsigned* out) {
    const unsigned row = blockIdx.x >> 1, chunk = blockIdx.x & 1, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const size_t rowb = (size_t)row * 256 * 512;
    unsigned v[64];
#pragma unroll
    for (int j = 0; j < 64; ++j) {
        const unsigned cell = w * 64 + j;
        v[j] = pres[row * 256 + cell] ? *reinterpret_cast<const unsigned*>(sq + rowb + cell * 512 + chunk * 256 + lane * 4) : 0u;
    }
    unsigned acc = 0;
#pragma unroll
    for (int j = 0; j < 64; ++j) acc ^= v[j];
    if (write) {
#pragma unroll
        for (int j = 0; j < 64; ++j) {
            const unsigned cell = w * 64 + j;
            if (!pres[row * 256 + cell]) *reinterpret_cast<unsigned*>(sq + rowb + cell * 512 + chunk * 256 + lane * 4) = acc ^ j;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

static float timed(hipStream_t st, auto&& fn) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    fn();  // warm
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(a, st));
    for (int i = 0; i < 5; ++i) fn();
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms / 5;
}

int main() {
    const size_t bytes = 64ull << 20;
    hipStream_t st;
    CK(hipStreamCreate(&st));
    unsigned* dout;
    unsigned char* dbuf;
    CK(hipMalloc(&dout, 4));
    CK(hipMalloc(&dbuf, bytes));
    struct Flag {
        const char* name;
        unsigned f;
    } flags[] = {{"default", hipHostMallocDefault},
                 {"mapped", hipHostMallocMapped},
                 {"coherent", hipHostMallocCoherent | hipHostMallocMapped},
                 {"noncoherent", hipHostMallocNonCoherent | hipHostMallocMapped}};
    for (auto& fl : flags) {
        unsigned char* h = nullptr;
        CK(hipHostMalloc((void**)&h, bytes, fl.f));
        for (size_t i = 0; i < bytes; ++i) h[i] = (unsigned char)i;
        unsigned char* hd = nullptr;
        CK(hipHostGetDevicePointer((void**)&hd, h, 0));
        for (int grid : {256, 1024, 4096}) {
            float r4 = timed(st, [&] { hipLaunchKernelGGL(zc_read<4>, dim3(grid), dim3(256), 0, st, hd, bytes, dout); });
            float r16 = timed(st, [&] { hipLaunchKernelGGL(zc_read<16>, dim3(grid), dim3(256), 0, st, hd, bytes, dout); });
            float w4 = timed(st, [&] { hipLaunchKernelGGL(zc_write<4>, dim3(grid), dim3(256), 0, st, hd, bytes); });
            float w16 = timed(st, [&] { hipLaunchKernelGGL(zc_write<16>, dim3(grid), dim3(256), 0, st, hd, bytes); });
            printf("{\"alloc\": \"%s\", \"grid\": %d, \"read4_GBs\": %.1f, \"read16_GBs\": %.1f, \"write4_GBs\": %.1f, "
                   "\"write16_GBs\": %.1f}\n",
                   fl.name, grid, bytes / r4 / 1e6, bytes / r16 / 1e6, bytes / w4 / 1e6, bytes / w16 / 1e6);
            fflush(stdout);
        }
        float h2d = timed(st, [&] { CK(hipMemcpyAsync(dbuf, h, bytes, hipMemcpyHostToDevice, st)); });
        float d2h = timed(st, [&] { CK(hipMemcpyAsync(h, dbuf, bytes, hipMemcpyDeviceToHost, st)); });
        // copy engine H2D beside a zero-copy read kernel (two streams)
        hipStream_t s2;
        CK(hipStreamCreate(&s2));
        unsigned char* h2 = nullptr;
        CK(hipHostMalloc((void**)&h2, bytes, fl.f));
        unsigned char* hd2 = nullptr;
        CK(hipHostGetDevicePointer((void**)&hd2, h2, 0));
        float both = timed(st, [&] {
            hipEvent_t e;
            CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            CK(hipEventRecord(e, st));
            CK(hipStreamWaitEvent(s2, e, 0));
            CK(hipMemcpyAsync(dbuf, h, bytes, hipMemcpyHostToDevice, s2));
            hipLaunchKernelGGL(zc_read<16>, dim3(1024), dim3(256), 0, st, hd2, bytes, dout);
            CK(hipEventRecord(e, s2));
            CK(hipStreamWaitEvent(st, e, 0));
            CK(hipEventDestroy(e));
        });
        {
            unsigned char* dpres;
            CK(hipMalloc(&dpres, 256 * 256));
            unsigned char hp[256 * 256];
            unsigned long long x = 0x9E3779B97F4A7C15ull;
            for (int i = 0; i < 256 * 256; ++i) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; hp[i] = (x >> 20) & 1; }
            CK(hipMemcpy(dpres, hp, sizeof hp, hipMemcpyHostToDevice));
            float pr = timed(st, [&] { hipLaunchKernelGGL(zc_row_pattern, dim3(512), dim3(256), 0, st, hd, dpres, 0, dout); });
            float pw = timed(st, [&] { hipLaunchKernelGGL(zc_row_pattern, dim3(512), dim3(256), 0, st, hd, dpres, 1, dout); });
            float dr = timed(st, [&] { hipLaunchKernelGGL(zc_row_pattern, dim3(512), dim3(256), 0, st, dbuf, dpres, 1, dout); });
            const double half = 256.0 * 256 * 512 / 2;
            printf("{\"alloc\": \"%s\", \"row_pattern_read_us\": %.1f, \"read_GBs\": %.1f, \"row_pattern_rw_us\": %.1f, "
                   "\"rw_total_GBs\": %.1f, \"hbm_rw_us\": %.1f}\n",
                   fl.name, pr * 1e3, half / pr / 1e6, pw * 1e3, 2 * half / pw / 1e6, dr * 1e3);
            fflush(stdout);
            CK(hipFree(dpres));
        }
        float strided = timed(st, [&] { hipLaunchKernelGGL(zc_read_strided, dim3(1024), dim3(256), 0, st, hd, bytes, dout); });
        float rw = timed(st, [&] {  // zero-copy read and zero-copy write at once (two streams)
            hipEvent_t e;
            CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            CK(hipEventRecord(e, st));
            CK(hipStreamWaitEvent(s2, e, 0));
            hipLaunchKernelGGL(zc_write<4>, dim3(1024), dim3(256), 0, s2, hd, bytes);
            hipLaunchKernelGGL(zc_read<4>, dim3(1024), dim3(256), 0, st, hd2, bytes, dout);
            CK(hipEventRecord(e, s2));
            CK(hipStreamWaitEvent(st, e, 0));
            CK(hipEventDestroy(e));
        });
        float dup = timed(st, [&] {  // copy engine both directions at once
            hipEvent_t e;
            CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            CK(hipEventRecord(e, st));
            CK(hipStreamWaitEvent(s2, e, 0));
            CK(hipMemcpyAsync(h2, dbuf, bytes, hipMemcpyDeviceToHost, s2));
            CK(hipMemcpyAsync(dbuf, h, bytes / 2, hipMemcpyHostToDevice, st));
            CK(hipMemcpyAsync(dbuf + bytes / 2, h + bytes / 2, bytes / 2, hipMemcpyHostToDevice, st));
            CK(hipEventRecord(e, s2));
            CK(hipStreamWaitEvent(st, e, 0));
            CK(hipEventDestroy(e));
        });
        printf("{\"alloc\": \"%s\", \"zc_read_strided_GBs\": %.1f, \"zc_read_plus_write_total_GBs\": %.1f, \"sdma_duplex_total_GBs\": %.1f}\n",
               fl.name, bytes / 2 / strided / 1e6, 2 * bytes / rw / 1e6, 2 * bytes / dup / 1e6);
        printf("{\"alloc\": \"%s\", \"sdma_h2d_GBs\": %.1f, \"sdma_d2h_GBs\": %.1f, \"sdma_plus_zc_read_total_GBs\": %.1f}\n",
               fl.name, bytes / h2d / 1e6, bytes / d2h / 1e6, 2 * bytes / both / 1e6);
        fflush(stdout);
        CK(hipStreamDestroy(s2));
        CK(hipHostFree(h2));
        CK(hipHostFree(h));
    }
    CK(hipFree(dout));
    CK(hipFree(dbuf));
    return 0;
}
