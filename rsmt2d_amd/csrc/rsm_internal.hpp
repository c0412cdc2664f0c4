// rsm_internal.hpp -- host-side internals shared by the runtime and the EDS layer.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>

#include "../../include/rsmt2d_hip.h"
#include "gf16.hpp"
#include "rsm_kernels.hpp"

namespace rsm {

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

}  // namespace rsm

struct rsm_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;       // serialises API calls that use the context's staging buffers
    std::mutex gf16_mu;  // guards gf16 table upload / scratch growth
    std::map<int, std::unique_ptr<rsm::DevBuf>> bufs;
    std::map<int, std::unique_ptr<rsm::HostBuf>> hbufs;
    // queue/counter words of the fused extension kernel, one buffer per stream (two
    // launches in flight on different streams must not share a queue)
    std::mutex fused_mu;
    std::map<void*, std::unique_ptr<rsm::DevBuf>> fused_ctr;
    uint32_t fused_trace_n = 0;  // items of the last traced fused launch (RSM_FUSED_TRACE)
    uint32_t* d_zero_index = nullptr;
    rsm::Gf16Dev gf16{};
    bool gf16_ready = false;

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

namespace rsm {

// GF(2^16) tables on the context's device (uploaded once) + scratch sized for
// `scratch_bytes` of work arrays.  Returns RSM_OK or an RSM_E* code.
int ensure_gf16(rsm_ctx* ctx, uint64_t scratch_bytes, uint64_t errs_bytes);

int launch_encode(rsm_ctx* ctx, const CodewordSet& cs, hipStream_t st);
int launch_decode(rsm_ctx* ctx, const DecodeSet& ds, hipStream_t st);
int extend_squares(rsm_ctx* ctx, uint8_t* d_eds, uint32_t k, uint32_t S, uint32_t count, hipStream_t st,
                   int phases = 3);
// DefaultTree row + column roots of a device-resident complete [W][W][S] square:
// d_roots receives 2*W*32 bytes (row roots, then column roots).  RSM_EUNSUPPORTED
// when W is outside roots_dev_supported().
int device_roots(rsm_ctx* ctx, const uint8_t* d_eds, uint32_t W, uint32_t S, uint8_t* d_roots, hipStream_t st,
                 uint32_t squares = 1);

}  // namespace rsm
