// rsm_internal.hpp -- host-side internals shared by the runtime and the EDS layer.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>

#include "../../include/rsmt2d_hip.h"
#include "rsm_kernels.hpp"

namespace rsm {

// Bytes of share width one GF(2^16) wave task covers (see kernels_gf16.hip).
constexpr uint32_t kGf16BytesPerWave = 128;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int hip_fail(hipError_t e, const char* what);
const char* last_error();
int validate_chunk_size(int64_t share_size);
int field_bits(uint32_t k);

// Grow-only device / pinned-host scratch buffers owned by a context.
struct DevBuf {
    void* ptr = nullptr;
    size_t cap = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf();
    hipError_t ensure(size_t n);
};
struct HostBuf {
    void* ptr = nullptr;
    size_t cap = 0;
    HostBuf() = default;
    HostBuf(const HostBuf&) = delete;
    HostBuf& operator=(const HostBuf&) = delete;
    ~HostBuf();
    hipError_t ensure(size_t n);
};

int launch_encode(const CodewordSet& cs, hipStream_t st);
int launch_decode(const DecodeSet& ds, hipStream_t st);
int extend_squares(uint8_t* d_eds, uint32_t k, uint32_t S, uint32_t count, hipStream_t st, int phases = 3);

}  // namespace rsm

struct rsm_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::recursive_mutex mu_storage;
    std::mutex mu;
    std::map<int, std::unique_ptr<rsm::DevBuf>> bufs;
    std::map<int, std::unique_ptr<rsm::HostBuf>> hbufs;
    uint32_t* d_zero_index = nullptr;

    rsm::DevBuf& dev_buf(int slot) {
        auto& p = bufs[slot];
        if (!p) p = std::make_unique<rsm::DevBuf>();
        return *p;
    }
    rsm::HostBuf& host_buf(int slot) {
        auto& p = hbufs[slot];
        if (!p) p = std::make_unique<rsm::HostBuf>();
        return *p;
    }
    // Device array holding a single 0 (index list of a one-codeword decode).
    const uint32_t* zero_index() {
        if (!d_zero_index) {
            rsm::DevBuf& b = dev_buf(-1);
            if (b.ensure(64) != hipSuccess) return nullptr;
            if (hipMemsetAsync(b.ptr, 0, 64, stream) != hipSuccess) return nullptr;
            d_zero_index = static_cast<uint32_t*>(b.ptr);
        }
        return d_zero_index;
    }
};
