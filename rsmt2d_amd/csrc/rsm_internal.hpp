// rsm_internal.hpp -- host-side internals shared by the runtime and the EDS layer.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rsmt2d_hip.h"
#include "gf16.hpp"
#include "rsm_kernels.hpp"

namespace rsm {

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int hip_fail(hipError_t e, const char* what);
const char* last_error();
int validate_chunk_size(int64_t share_size);
int field_bits(uint32_t k);

// Grow-only device / pinned-host scratch buffers.  Not synchronised: every
// instance below has exactly one owner (a lane, a stream's scratch under its own
// mutex, or the EDS state under rsm_ctx::eds_mu).
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

// Per-call resources of the Codec / host-memory entry points: rsmt2d calls
// Encode/Decode from up to 2k goroutines at once (extendeddatasquare.go:186-224),
// so each call takes a lane (own stream + pinned staging + device staging) from a
// pool instead of serialising on one context lock.
struct Lane {
    hipStream_t stream = nullptr;
    HostBuf host;
    DevBuf dev, aux;
    hipEvent_t ev[2] = {nullptr, nullptr};  // created on first use (lane_event), kept with the lane
};

// Event i (< 2) of a lane the caller holds, created once (hipEventDisableTiming): Repair
// synchronises its two streams with them instead of creating events per call.
inline hipEvent_t lane_event(Lane& L, int i) {
    if (!L.ev[i] && hipEventCreateWithFlags(&L.ev[i], hipEventDisableTiming) != hipSuccess) L.ev[i] = nullptr;
    return L.ev[i];
}

// Device scratch that belongs to one stream: kernels queued on different streams
// never share it.  `mu` is held while the scratch is grown AND while the launches
// that use it are enqueued.
struct StreamScratch {
    std::mutex mu;
    DevBuf gf16_work, gf16_errs;  // GF(2^16) work arrays / error locators
    DevBuf leaf;                  // DefaultTree leaf digests (device roots)
    DevBuf queue;                 // work-queue words of the single-launch extension
    HostBuf qerr;                 // its stuck-wait report (pinned, written by the device)
};

// Buffers of the ExtendedDataSquare layer (Repair, device roots of an EDS):
// used only under rsm_ctx::eds_mu, on the context stream.
struct EdsBufs {
    DevBuf eds, scratch, pres, idx, flags, roots, status;
};

// A Tree plugin the GPU computes itself: the DefaultTree (tree_fn NULL or
// rsm_default_tree_root) or the namespaced Merkle tree (rsm_nmt_tree_root).
struct DevTree {
    bool nmt = false;
    rsm_nmt_params p{};
    uint32_t root_len = 32;
};

}  // namespace rsm

struct rsm_ctx {
    int device = 0;
    uint32_t cus = 256;          // compute units of `device` (persistent-grid size)
    hipStream_t stream = nullptr;
    std::atomic<uint32_t> pass_grid[2] = {0, 0};  // rsm_ctx_set_pass_grid (0 = all CUs)
    std::atomic<uint32_t> split_max{12};           // rsm_ctx_set_split_max
    // rsm_ctx_set_limits (test hooks; defaults: the kernels' own limits): codeword halves
    // spanning more than offset_limit bytes take the wide forms, and GF(2^16) work
    // arrays get at most work_budget bytes per stream (wider shares run as byte slabs)
    std::atomic<uint64_t> offset_limit{rsm::kOffsetLimit};
    std::atomic<uint64_t> work_budget{1ull << 30};

    // lane pool (Codec calls, host-memory extension)
    static constexpr size_t kMaxLanes = 32;
    std::mutex lane_mu;
    std::condition_variable lane_cv;
    std::vector<std::unique_ptr<rsm::Lane>> lanes;
    std::vector<rsm::Lane*> free_lanes;

    // per-stream scratch
    std::mutex scratch_mu;  // guards the map only
    std::map<hipStream_t, std::unique_ptr<rsm::StreamScratch>> scratch;

    // GF(2^16) tables, uploaded once
    std::mutex gf16_mu;
    bool gf16_ready = false;
    rsm::DevBuf gf16_perm, gf16_skew, gf16_logwalsh, gf16_skewperm;
    rsm::Gf16Dev gf16{};  // table pointers only (scratch comes per stream)

    rsm::DevBuf zero_index;  // one device u32 = 0 (index list of a single-codeword decode)

    std::mutex eds_mu;
    rsm::EdsBufs eds;
};

namespace rsm {

// Lane pool: blocks while all kMaxLanes lanes are busy.
Lane* acquire_lane(rsm_ctx* ctx, int* rc);
void release_lane(rsm_ctx* ctx, Lane* l);
int acquire_lanes(rsm_ctx* ctx, int n, Lane** out);
struct LaneGuard {
    rsm_ctx* ctx;
    Lane* lane;
    int rc = RSM_OK;
    explicit LaneGuard(rsm_ctx* c) : ctx(c), lane(acquire_lane(c, &rc)) {}
    ~LaneGuard() {
        if (lane) release_lane(ctx, lane);
    }
    LaneGuard(const LaneGuard&) = delete;
    LaneGuard& operator=(const LaneGuard&) = delete;
};

StreamScratch& stream_scratch(rsm_ctx* ctx, hipStream_t st);

// GF(2^16) tables on the context's device (uploaded once).  Returns RSM_OK or an RSM_E* code.
int ensure_gf16_tables(rsm_ctx* ctx);

// Selects the context's device on the calling thread (cgo moves goroutines
// between OS threads; the HIP current device is per thread).
int use_device(rsm_ctx* ctx);

// Whether the single-pass kernels address codewords of k symbols es bytes apart
// (narrow_fits under the context's offset limit); otherwise the wide forms run.
bool narrow_ok(const rsm_ctx* ctx, uint64_t k, uint64_t es, uint64_t S);
int launch_encode(rsm_ctx* ctx, const CodewordSet& cs, hipStream_t st);
int launch_decode(rsm_ctx* ctx, const DecodeSet& ds, hipStream_t st);
int extend_squares(rsm_ctx* ctx, uint8_t* d_eds, uint32_t k, uint32_t S, uint32_t count, hipStream_t st,
                   int phases = 3);
// Both passes of `count` k = 128 squares as ONE queue-driven launch
// (extend_gf8_bs128q_kernel); RSM_EUNSUPPORTED when the shape does not qualify.
// `delay`: squares of row sets handed out before the first Q0-column set.
int extend_squares_queue(rsm_ctx* ctx, uint8_t* d_eds, uint32_t k, uint32_t S, uint32_t count, hipStream_t st,
                         uint32_t delay = 2, uint32_t margin = ~0u);
// RSM_EDEVICE (and clears the report) when a completed queue launch on `st` (NULL:
// on any stream of the context) timed out waiting -- its output is invalid.
int check_queue_reports(rsm_ctx* ctx, hipStream_t st);
// DefaultTree row + column roots of a device-resident complete [W][W][S] square:
// d_roots receives 2*W*32 bytes (row roots, then column roots).  RSM_EUNSUPPORTED
// when W is outside roots_dev_supported().
int device_roots(rsm_ctx* ctx, const uint8_t* d_eds, uint32_t W, uint32_t S, uint8_t* d_roots, hipStream_t st,
                 uint32_t squares = 1);
// Whether (tree_fn, user) is a tree the GPU computes for a square of width W.
bool device_tree_for(rsm_tree_root_fn fn, void* user, uint32_t W, DevTree* out);
// Roots of all 2W trees of `squares` complete consecutive device squares: d_roots
// 2W * t.root_len bytes per square (rows, then columns); d_status 2W words per square,
// non-zero where a tree fails (NMT push order; all zero for the DefaultTree).
// Asynchronous on st.
int device_tree_roots(rsm_ctx* ctx, const DevTree& t, const uint8_t* d_eds, uint32_t W, uint32_t S,
                      uint8_t* d_roots, uint32_t* d_status, hipStream_t st, uint32_t squares = 1);

}  // namespace rsm
