// hip_stub.cpp -- TEST INFRASTRUCTURE ONLY (tests/test_tsan_cpu.py): a host-memory
// stand-in for the HIP runtime calls and kernel launchers that the product's host
// code (rsm_runtime.cpp, eds.cpp) makes, so that code can be built with
// -fsanitize=thread and hammered from many threads on a machine without a GPU.
// "Kernels" here only touch the bytes a real launch would read and write (so the
// sanitizer sees every buffer access); they compute nothing meaningful, and
// nothing in the product links this file.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../rsmt2d_amd/csrc/gf16.hpp"
#include "../../rsmt2d_amd/csrc/rsm_kernels.hpp"

namespace {
struct FakeStream {
    int id;
};
std::atomic<int> g_streams{0};
}  // namespace

extern "C" {
#ifdef RSM_STUB_ORACLE
static thread_local int t_device = 0;  // G host "devices" for the multi-GPU check
hipError_t hipGetDeviceCount(int* n) { *n = 8; return hipSuccess; }
hipError_t hipSetDevice(int d) { if (d < 0 || d >= 8) return hipErrorInvalidDevice; t_device = d; return hipSuccess; }
hipError_t hipGetDevice(int* d) { *d = t_device; return hipSuccess; }
#else
hipError_t hipGetDeviceCount(int* n) { *n = 1; return hipSuccess; }
hipError_t hipSetDevice(int) { return hipSuccess; }
hipError_t hipGetDevice(int* d) { *d = 0; return hipSuccess; }
#endif
hipError_t hipDeviceGetAttribute(int* v, hipDeviceAttribute_t, int) { *v = 256; return hipSuccess; }
hipError_t hipDeviceSynchronize(void) { return hipSuccess; }
hipError_t hipGetLastError(void) { return hipSuccess; }
hipError_t hipPeekAtLastError(void) { return hipSuccess; }
const char* hipGetErrorString(hipError_t) { return "stub"; }
hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned int) {
    *s = reinterpret_cast<hipStream_t>(new FakeStream{g_streams++});
    return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t s) {
    delete reinterpret_cast<FakeStream*>(s);
    return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipStreamQuery(hipStream_t) { return hipSuccess; }
hipError_t hipMalloc(void** p, size_t n) {
    *p = calloc(1, n ? n : 1);
    return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipFree(void* p) { free(p); return hipSuccess; }
hipError_t hipHostMalloc(void** p, size_t n, unsigned int) { return hipMalloc(p, n); }
hipError_t hipHostFree(void* p) { free(p); return hipSuccess; }
hipError_t hipHostGetDevicePointer(void** d, void* h, unsigned int) { *d = h; return hipSuccess; }
hipError_t hipMemcpy(void* d, const void* s, size_t n, hipMemcpyKind) { memcpy(d, s, n); return hipSuccess; }
hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind, hipStream_t) {
    memcpy(d, s, n);
    return hipSuccess;
}
hipError_t hipMemcpy2DAsync(void* d, size_t dp, const void* s, size_t sp, size_t w, size_t h, hipMemcpyKind,
                            hipStream_t) {
    for (size_t r = 0; r < h; ++r) memcpy(static_cast<char*>(d) + r * dp, static_cast<const char*>(s) + r * sp, w);
    return hipSuccess;
}
hipError_t hipMemset(void* d, int v, size_t n) { memset(d, v, n); return hipSuccess; }
hipError_t hipMemsetAsync(void* d, int v, size_t n, hipStream_t) { memset(d, v, n); return hipSuccess; }
hipError_t hipEventCreate(hipEvent_t* e) { *e = reinterpret_cast<hipEvent_t>(new int(0)); return hipSuccess; }
hipError_t hipEventDestroy(hipEvent_t e) { delete reinterpret_cast<int*>(e); return hipSuccess; }
hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
hipError_t hipEventSynchronize(hipEvent_t) { return hipSuccess; }
hipError_t hipEventElapsedTime(float* ms, hipEvent_t, hipEvent_t) { *ms = 0.f; return hipSuccess; }
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) { return hipEventCreate(e); }
hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t, unsigned int) { return hipSuccess; }
}

namespace rsm {

// A launch reads every data symbol and writes every parity symbol of its codewords.
static void touch_codewords(const CodewordSet& cs, bool gf16) {
    (void)gf16;
    for (uint32_t q = 0; q < cs.count; ++q) {
        const uint64_t rel = cs.indices ? (uint64_t)cs.indices[q] * cs.cw_stride
                                        : (uint64_t)(q / cs.per_square) * cs.square_stride +
                                              (uint64_t)(q % cs.per_square) * cs.cw_stride;
        uint8_t acc = 0;
        for (uint32_t e = 0; e < cs.k; ++e) acc ^= cs.base[rel + (uint64_t)e * cs.elem_stride];
        for (uint32_t e = 0; e < cs.k; ++e)
            memset(cs.out_base + rel + cs.out_offset + (uint64_t)e * cs.elem_stride, acc, cs.S);
    }
}

#ifdef RSM_STUB_ORACLE
// multi_check (tests/test_multi_cpu.py): "kernels" that compute the real parity
// with the C oracle, so the product's host code above them (CodewordSet
// construction, the multi-GPU exchange) is checked bit for bit on the CPU.
}  // namespace rsm
extern "C" int leo_encode(unsigned k, size_t S, const uint8_t* const* data, uint8_t* const* parity);
namespace rsm {
static hipError_t oracle_codewords(const CodewordSet& cs) {
    std::vector<const uint8_t*> d(cs.k);
    std::vector<uint8_t*> p(cs.k);
    for (uint32_t q = 0; q < cs.count; ++q) {
        const uint64_t rel = cs.indices ? (uint64_t)cs.indices[q] * cs.cw_stride
                                        : (uint64_t)(q / cs.per_square) * cs.square_stride +
                                              (uint64_t)(q % cs.per_square) * cs.cw_stride;
        uint8_t* out = cs.out_base ? cs.out_base : cs.base;
        for (uint32_t e = 0; e < cs.k; ++e) {
            d[e] = cs.base + rel + (uint64_t)e * cs.elem_stride;
            // the all-to-all column pass: another GPU's rows from the received block
            if (cs.blk && e / cs.blk_rows != cs.blk_self)
                d[e] = cs.blk + (uint64_t)(e / cs.blk_rows) * cs.blk_size + (uint64_t)(e % cs.blk_rows) * cs.blk_pitch +
                       (uint64_t)q * cs.S;
            p[e] = out + rel + cs.out_offset + (uint64_t)e * cs.elem_stride;
        }
        if (leo_encode(cs.k, cs.S, d.data(), p.data()) != 0) return hipErrorInvalidValue;
        if (cs.side)  // the all-to-all row pass: cells of other GPUs' column blocks into their send blocks
            for (uint32_t c = 0; c < 2 * cs.k; ++c) {
                const uint32_t owner = c / cs.side_cols;
                if (owner == cs.side_self) continue;
                const uint8_t* src = c < cs.k ? d[c] : p[c - cs.k];
                memcpy(cs.side + (uint64_t)owner * cs.side_blk + (uint64_t)q * cs.side_cols * cs.S +
                           (uint64_t)(c % cs.side_cols) * cs.S,
                       src, cs.S);
            }
    }
    return hipSuccess;
}
hipError_t launch_encode_gf8(const CodewordSet& cs, hipStream_t) { return oracle_codewords(cs); }
hipError_t launch_encode_gf16(const CodewordSet& cs, const Gf16Dev&, hipStream_t) { return oracle_codewords(cs); }
#else
hipError_t launch_encode_gf8(const CodewordSet& cs, hipStream_t) {
    touch_codewords(cs, false);
    return hipSuccess;
}
hipError_t launch_encode_gf16(const CodewordSet& cs, const Gf16Dev& g, hipStream_t) {
    if (g.scratch) memset(g.scratch, 0, g.scratch_bytes < 4096 ? g.scratch_bytes : 4096);
    touch_codewords(cs, true);
    return hipSuccess;
}
#endif
static void touch_decode(const DecodeSet& ds) {
    const uint64_t W = 2ull * ds.k;
    for (uint32_t i = 0; i < ds.count; ++i) {
        const uint64_t vec = ds.indices[i];
        for (uint64_t e = 0; e < W; ++e) {
            const uint64_t cell = ds.axis == 0 ? vec * W + e : e * W + vec;
            if (!ds.presence[cell]) memset(ds.base + cell * ds.S, 0, ds.S);
        }
    }
}
hipError_t launch_decode_gf8(const DecodeSet& ds, hipStream_t) {
    touch_decode(ds);
    return hipSuccess;
}
hipError_t launch_decode_gf16(const DecodeSet& ds, const Gf16Dev& g, hipStream_t) {
    if (g.scratch) memset(g.scratch, 0, g.scratch_bytes < 4096 ? g.scratch_bytes : 4096);
    if (g.errs) memset(g.errs, 0, g.errs_bytes < 4096 ? g.errs_bytes : 4096);
    touch_decode(ds);
    return hipSuccess;
}
hipError_t launch_encode_gf8_wide(const CodewordSet& cs, hipStream_t st) { return launch_encode_gf8(cs, st); }
hipError_t launch_decode_gf8_wide(const DecodeSet& ds, hipStream_t st) { return launch_decode_gf8(ds, st); }
bool dec16_needs_work() { return false; }
bool bs128_applicable(const CodewordSet&) { return false; }
hipError_t launch_encode_gf8_bs128(const CodewordSet& cs, hipStream_t st) { return launch_encode_gf8(cs, st); }
bool split_fused_enabled() { return false; }  // the stub runs the two-launch form
hipError_t launch_extend_gf8_split_fused(const CodewordSet&, const CodewordSet&, const CodewordSet&, uint32_t*,
                                         uint32_t*, hipStream_t) {
    return hipErrorInvalidValue;
}
hipError_t launch_encode_gf8_split(const CodewordSet& a, const CodewordSet* b, hipStream_t st, int) {
    if (hipError_t e = launch_encode_gf8(a, st)) return e;
    return b ? launch_encode_gf8(*b, st) : hipSuccess;
}
// the single-launch batch path never qualifies here (batches take the two-launch form)
bool bs128_queue_applicable(const CodewordSet&, const CodewordSet&) { return false; }
hipError_t launch_extend_gf8_bs128_queue(const QueuePlan&, hipStream_t) { return hipErrorInvalidValue; }
bool roots_dev_supported(uint32_t W) { return W >= 1 && W <= 2048; }
hipError_t launch_roots(const uint8_t* d_eds, uint32_t W, uint32_t S, uint32_t squares, uint32_t* d_leaf,
                        uint8_t* d_roots, hipStream_t) {
    for (uint32_t s = 0; s < squares; ++s) {
        for (uint64_t c = 0; c < (uint64_t)W * W; ++c)
            d_leaf[(s * (uint64_t)W * W + c) * 8] = d_eds[(s * (uint64_t)W * W + c) * S];
        memset(d_roots + (uint64_t)s * 2 * W * 32, 0, (size_t)2 * W * 32);
    }
    return hipSuccess;
}
hipError_t launch_leaf_hashes(const uint8_t* d_cells, uint32_t cells, uint32_t S, uint32_t* d_leaf, hipStream_t) {
    for (uint32_t c = 0; c < cells; ++c) d_leaf[(uint64_t)c * 8] = d_cells[(uint64_t)c * S];
    return hipSuccess;
}
hipError_t launch_tree_roots(const uint32_t* d_leaf, uint32_t W, uint32_t first, uint32_t count, uint8_t* d_roots,
                             hipStream_t) {
    for (uint32_t t = first; t < first + count; ++t) d_roots[(uint64_t)t * 32] = (uint8_t)d_leaf[0];
    (void)W;
    return hipSuccess;
}
bool nmt_dev_supported(uint32_t W, uint32_t ns) { return W >= 2 && W <= 1024 && ns >= 1 && ns <= 32; }
hipError_t launch_nmt_roots(const uint8_t* d_eds, uint32_t W, uint32_t S, uint32_t ns, uint32_t, uint32_t,
                            uint32_t* d_leaf, uint8_t* d_roots, uint32_t* d_status, hipStream_t, uint32_t squares) {
    for (uint32_t q = 0; q < squares; ++q) {
        const uint8_t* e = d_eds + (uint64_t)q * W * W * S;
        uint32_t* lf = d_leaf + (uint64_t)q * W * W * 16;
        for (uint64_t c = 0; c < (uint64_t)W * W; ++c) lf[c * 16] = e[c * S];
        memset(d_roots + (uint64_t)q * 2 * W * (2 * ns + 32), 0, (size_t)2 * W * (2 * ns + 32));
        if (d_status) memset(d_status + (uint64_t)q * 2 * W, 0, (size_t)2 * W * 4);
    }
    return hipSuccess;
}
hipError_t launch_fill_random(void* p, uint64_t bytes, uint64_t seed, hipStream_t) {
    memset(p, (int)(seed & 0xFF), bytes);
    return hipSuccess;
}
hipError_t launch_stage_copy(void* dst, const void* src, uint64_t bytes, hipStream_t) {
    memcpy(dst, src, (bytes + 15) / 16 * 16);
    return hipSuccess;
}
hipError_t launch_compare(const uint8_t* a, const uint8_t* b, uint64_t n, uint32_t* mismatch, hipStream_t) {
    *mismatch = memcmp(a, b, n) != 0;
    return hipSuccess;
}
hipError_t launch_compare_parity(const uint8_t*, const uint8_t*, uint32_t, uint32_t, uint32_t, const uint32_t*,
                                 uint32_t count, uint32_t* flags, hipStream_t) {
    memset(flags, 0, count * 4);
    return hipSuccess;
}

}  // namespace rsm
