// calib16.hip -- diagnostic (NOT part of librsmt2d_hip.so): calibrates the PMC
// FETCH_SIZE / WRITE_SIZE counters and the achieved rate for the GF(2^16) kernels'
// access shape against plain 16-B-per-lane streaming of the same bytes.
//   shape 0 ("lohi4"): the enc16/dec16 lane pattern (kernels_gf16.hip lane_of): lane l of a
//            wave owns 64-B block 8c + l/8, dword l%8 of its lo half and the same dword of
//            its hi half (+32 B); one 4-B load / store per half.
//   shape 1 ("x4"):    16 B per lane, a wave covers 1 KiB contiguous (dwordx4).
// Each kernel copies N bytes from `in` to `out` (read once, write once), grid-stride,
// E symbols per wave in flight (the loads of a task issued before its stores, as the
// encoders do).  Usage: calib16 <shape> <MiB> <reps>; prints one JSON line.
// Run under rocprofv3 --pmc FETCH_SIZE (and separately WRITE_SIZE) to read the counters
// for the same launch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr int E = 16;  // symbols (rows of 512 B) per wave-task

// task = (row group of E rows, 512-B chunk): rows are 2048 B apart (S = 2048, as C4)
__global__ __launch_bounds__(256) void lohi4(const uint8_t* in, uint8_t* out, uint64_t nbytes) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (uint64_t)gridDim.x * 4;
    const uint64_t S = 2048, tasks = nbytes / (S * E) * (S / 512);
    for (uint64_t t = wave; t < tasks; t += nw) {
        const uint64_t grp = t / (S / 512), chunk = t % (S / 512);
        const uint64_t off = grp * S * E + chunk * 512 + (lane >> 3) * 64 + (lane & 7u) * 4;
        uint32_t l[E], h[E];
#pragma unroll
        for (int i = 0; i < E; ++i) {
            l[i] = *reinterpret_cast<const uint32_t*>(in + off + i * S);
            h[i] = *reinterpret_cast<const uint32_t*>(in + off + i * S + 32);
        }
#pragma unroll
        for (int i = 0; i < E; ++i) {
            *reinterpret_cast<uint32_t*>(out + off + i * S) = l[i] ^ 1u;
            *reinterpret_cast<uint32_t*>(out + off + i * S + 32) = h[i] ^ 1u;
        }
    }
}
__global__ __launch_bounds__(256) void x4(const uint8_t* in, uint8_t* out, uint64_t nbytes) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (uint64_t)gridDim.x * 4;
    const uint64_t S = 2048, tasks = nbytes / (S * E) * (S / 1024);
    for (uint64_t t = wave; t < tasks; t += nw) {
        const uint64_t grp = t / (S / 1024), chunk = t % (S / 1024);
        const uint64_t off = grp * S * E + chunk * 1024 + lane * 16;
        v4u v[E];
#pragma unroll
        for (int i = 0; i < E; ++i) v[i] = *reinterpret_cast<const v4u*>(in + off + i * S);
#pragma unroll
        for (int i = 0; i < E; ++i) *reinterpret_cast<v4u*>(out + off + i * S) = v[i] ^ 1u;
    }
}

int main(int argc, char** argv) {
    const int shape = argc > 1 ? atoi(argv[1]) : 0;
    const uint64_t mib = argc > 2 ? strtoull(argv[2], 0, 0) : 1024;
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    const uint64_t n = mib << 20;
    uint8_t *in, *out;
    CK(hipMalloc(&in, n));
    CK(hipMalloc(&out, n));
    CK(hipMemset(in, 0x5a, n));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0, 0));
        if (shape == 0) hipLaunchKernelGGL(lohi4, dim3(cus * 8), dim3(256), 0, 0, in, out, n);
        else hipLaunchKernelGGL(x4, dim3(cus * 8), dim3(256), 0, 0, in, out, n);
        CK(hipGetLastError());
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const double ms = ts[ts.size() / 2];
    printf("{\"probe\": \"calib16\", \"shape\": \"%s\", \"bytes_read\": %llu, \"bytes_written\": %llu, \"ms\": %.4f, "
           "\"TBps_rw\": %.3f, \"launches\": %d}\n",
           shape == 0 ? "lohi4" : "x4", (unsigned long long)n, (unsigned long long)n, ms, 2.0 * n / (ms * 1e-3) / 1e12,
           reps);
    return 0;
}
