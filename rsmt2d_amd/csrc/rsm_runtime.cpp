// rsm_runtime.cpp -- context, device memory and the Codec half of the C ABI.
//
// The HIP kernels are the only compute path: every entry point that needs
// arithmetic fails with RSM_EDEVICE when no GPU/HIP runtime is usable; there is
// no CPU fallback anywhere in the product.
//
// Threading (rsmt2d calls the Codec from up to 2k goroutines at once,
// extendeddatasquare.go:186-224, extendeddatacrossword.go:372-425):
//   * Codec and host-memory entry points take a Lane (own stream, pinned and
//     device staging) from the context's pool -- concurrent calls run
//     concurrently on the GPU;
//   * scratch that kernels use (GF(2^16) work arrays, leaf digests) belongs to the
//     stream the kernels are queued on, so launches on different streams never
//     share it;
//   * every entry point selects the context's device on the calling thread first.
#include "rsm_internal.hpp"

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstring>

namespace rsm {

static thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    return fail(RSM_EDEVICE, "%s: %s", what, hipGetErrorString(e));
}

const char* last_error() { return g_last_error.c_str(); }

DevBuf::~DevBuf() {
    if (ptr) (void)hipFree(ptr);
}
hipError_t DevBuf::ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    if (ptr) {
        (void)hipFree(ptr);
        ptr = nullptr;
        cap = 0;
    }
    hipError_t e = hipMalloc(&ptr, n);
    if (e == hipSuccess) cap = n;
    return e;
}

HostBuf::~HostBuf() {
    if (ptr) (void)hipHostFree(ptr);
}
hipError_t HostBuf::ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    if (ptr) {
        (void)hipHostFree(ptr);
        ptr = nullptr;
        cap = 0;
    }
    hipError_t e = hipHostMalloc(&ptr, n, hipHostMallocDefault);
    if (e == hipSuccess) cap = n;
    return e;
}

int validate_chunk_size(int64_t share_size) {
    if (share_size % 64 != 0)
        return fail(RSM_ESHARESIZE, "shareSize %lld must be a multiple of 64 bytes", (long long)share_size);
    return RSM_OK;
}

int field_bits(uint32_t k) { return 2ull * k > 256ull ? 16 : 8; }

int use_device(rsm_ctx* ctx) {
    hipError_t e = hipSetDevice(ctx->device);
    return e == hipSuccess ? RSM_OK : hip_fail(e, "hipSetDevice");
}

// ---------------------------------------------------------------------------
// Lanes and per-stream scratch
// ---------------------------------------------------------------------------
Lane* acquire_lane(rsm_ctx* ctx, int* rc) {
    std::unique_lock<std::mutex> lk(ctx->lane_mu);
    for (;;) {
        if (!ctx->free_lanes.empty()) {
            Lane* l = ctx->free_lanes.back();
            ctx->free_lanes.pop_back();
            *rc = RSM_OK;
            return l;
        }
        if (ctx->lanes.size() < rsm_ctx::kMaxLanes) {
            auto l = std::make_unique<Lane>();
            hipError_t e = hipStreamCreateWithFlags(&l->stream, hipStreamNonBlocking);
            if (e != hipSuccess) {
                *rc = hip_fail(e, "hipStreamCreate (lane)");
                return nullptr;
            }
            ctx->lanes.push_back(std::move(l));
            *rc = RSM_OK;
            return ctx->lanes.back().get();
        }
        ctx->lane_cv.wait(lk);
    }
}

// n lanes in one step: waits (holding none) until n are free or can be created, so
// callers that each need several lanes never deadlock holding part of a set.
int acquire_lanes(rsm_ctx* ctx, int n, Lane** out) {
    if (n <= 0 || (size_t)n > rsm_ctx::kMaxLanes) return fail(RSM_EINVAL, "acquire_lanes: bad lane count %d", n);
    std::unique_lock<std::mutex> lk(ctx->lane_mu);
    ctx->lane_cv.wait(lk, [&] {
        return ctx->free_lanes.size() + (rsm_ctx::kMaxLanes - ctx->lanes.size()) >= (size_t)n;
    });
    int got = 0;
    while (got < n && !ctx->free_lanes.empty()) {
        out[got++] = ctx->free_lanes.back();
        ctx->free_lanes.pop_back();
    }
    while (got < n) {
        auto l = std::make_unique<Lane>();
        hipError_t e = hipStreamCreateWithFlags(&l->stream, hipStreamNonBlocking);
        if (e != hipSuccess) {
            for (int i = 0; i < got; ++i) ctx->free_lanes.push_back(out[i]);
            lk.unlock();
            ctx->lane_cv.notify_all();
            return hip_fail(e, "hipStreamCreate (lane)");
        }
        ctx->lanes.push_back(std::move(l));
        out[got++] = ctx->lanes.back().get();
    }
    return RSM_OK;
}

void release_lane(rsm_ctx* ctx, Lane* l) {
    {
        std::lock_guard<std::mutex> lk(ctx->lane_mu);
        ctx->free_lanes.push_back(l);
    }
    // notify_all: a multi-lane waiter (acquire_lanes) woken by a single release may
    // still lack lanes and sleep again; it must not swallow a single-lane caller's wakeup
    ctx->lane_cv.notify_all();
}

StreamScratch& stream_scratch(rsm_ctx* ctx, hipStream_t st) {
    std::lock_guard<std::mutex> lk(ctx->scratch_mu);
    auto& p = ctx->scratch[st];
    if (!p) p = std::make_unique<StreamScratch>();
    return *p;
}

// ---------------------------------------------------------------------------
// Launch helpers (device-resident, asynchronous on `st`)
// ---------------------------------------------------------------------------
// GF(2^16): m = ceilPow2(k) in {256, 512} runs the on-chip single-pass kernels
// (every configuration in BASELINE.json); 512 < k <= 32768 (the reference's
// MaxChunks = 32768^2, leopard.go:76-84) the multi-pass generic kernels through
// per-stream work arrays.
static bool gf16_supported(uint32_t k) { return k > 128 && k <= 32768; }
static bool gf16_generic(uint32_t k) { return ceil_pow2(k) > 512; }

int ensure_gf16_tables(rsm_ctx* ctx) {
    std::lock_guard<std::mutex> lk(ctx->gf16_mu);
    if (ctx->gf16_ready) return RSM_OK;
    const Gf16Host& t = gf16_host();
    const size_t pb = t.perm.size() * sizeof(PermTab16), sb = t.skew.size() * 2, lb = (kLwFoldOff + t.lwfold.size()) * 2;
    const size_t kb = t.skewperm.size() * sizeof(PermTab16);
    hipError_t e;
    if ((e = ctx->gf16_perm.ensure(pb)) != hipSuccess || (e = ctx->gf16_skew.ensure(sb)) != hipSuccess ||
        (e = ctx->gf16_logwalsh.ensure(lb)) != hipSuccess || (e = ctx->gf16_skewperm.ensure(kb)) != hipSuccess)
        return hip_fail(e, "hipMalloc (GF16 tables)");
    if ((e = hipMemcpy(ctx->gf16_perm.ptr, t.perm.data(), pb, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(ctx->gf16_skew.ptr, t.skew.data(), sb, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(ctx->gf16_logwalsh.ptr, t.logwalsh.data(), kLwFoldOff * 2, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(static_cast<uint16_t*>(ctx->gf16_logwalsh.ptr) + kLwFoldOff, t.lwfold.data(),
                       t.lwfold.size() * 2, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(ctx->gf16_skewperm.ptr, t.skewperm.data(), kb, hipMemcpyHostToDevice)) != hipSuccess)
        return hip_fail(e, "upload GF16 tables");
    ctx->gf16.skewperm = static_cast<const PermTab16*>(ctx->gf16_skewperm.ptr);
    ctx->gf16.perm = static_cast<const PermTab16*>(ctx->gf16_perm.ptr);
    ctx->gf16.skew = static_cast<const uint16_t*>(ctx->gf16_skew.ptr);
    ctx->gf16.logwalsh = static_cast<const uint16_t*>(ctx->gf16_logwalsh.ptr);
    ctx->gf16_ready = true;
    return RSM_OK;
}

// GF(2^16) work arrays of stream `st` (caller holds ss.mu): grown after the
// stream has drained, since a kernel queued earlier on it may still use them.
static int gf16_for_stream(rsm_ctx* ctx, StreamScratch& ss, hipStream_t st, uint64_t work, uint64_t errs,
                           Gf16Dev* out) {
    if (int rc = ensure_gf16_tables(ctx)) return rc;
    hipError_t e;
    if (work > ss.gf16_work.cap || errs > ss.gf16_errs.cap) {
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
        if ((e = ss.gf16_work.ensure(work)) != hipSuccess) return hip_fail(e, "hipMalloc (GF16 work arrays)");
        if (errs && (e = ss.gf16_errs.ensure(errs)) != hipSuccess)
            return hip_fail(e, "hipMalloc (GF16 error locators)");
    }
    *out = ctx->gf16;
    out->scratch = static_cast<uint8_t*>(ss.gf16_work.ptr);
    out->scratch_bytes = ss.gf16_work.cap;
    out->errs = static_cast<uint16_t*>(ss.gf16_errs.ptr);
    out->errs_bytes = ss.gf16_errs.cap;
    return RSM_OK;
}

// Work arrays for GF(2^16): all codewords of a launch when that fits the budget,
// else a whole number of codewords of the budget per batch (the launcher loops), and
// at least one codeword's worth -- or, for shares too wide for that, one byte slab's
// (the launcher slabs the shares: kernels_gf16.hip g16_slab).
static uint64_t gf16_budget(uint64_t per_cw, uint64_t count, uint64_t cap) {
    const uint64_t want = per_cw * count;
    if (want <= cap) return want;
    return per_cw <= cap ? (cap / per_cw) * per_cw : cap;
}

bool narrow_ok(const rsm_ctx* ctx, uint64_t k, uint64_t es, uint64_t S) {
    return narrow_fits(k, es, S, ctx->offset_limit.load(std::memory_order_relaxed));
}

int launch_encode(rsm_ctx* ctx, const CodewordSet& cs0, hipStream_t st) {
    // parity from its own base (out_base + out_offset): every kernel's symbol offsets
    // then span one half of the codeword, k symbols es bytes apart (narrow_fits)
    CodewordSet cs = rebased(cs0);
    cs.wide = narrow_ok(ctx, cs.k, cs.elem_stride, cs.S) ? 0u : 1u;
    // the all-to-all hooks (rsm_multi.cpp) exist in the single-pass GF(2^16) encoders only
    if ((cs.side || cs.blk) && (field_bits(cs.k) != 16 || gf16_generic(cs.k) || cs.wide))
        return fail(RSM_EUNSUPPORTED, "encode: multi-GPU side output / blocked input need the single-pass GF(2^16) form");
    hipError_t e;
    if (field_bits(cs.k) == 8) {
        if (cs.wide) {
            e = launch_encode_gf8_wide(cs, st);
        } else {
            cs.chunks = (cs.S + 255) / 256;
            const uint32_t cap = ctx->pass_grid[cs.pass == 0 ? 0 : 1].load(std::memory_order_relaxed);
            cs.grid = (cap > 0 && cap < ctx->cus) ? cap : ctx->cus;
            e = launch_encode_gf8(cs, st);
        }
    } else {
        if (!gf16_supported(cs.k)) return fail(RSM_EUNSUPPORTED, "encode: k=%u exceeds 32768", cs.k);
        if (!gf16_generic(cs.k) && !cs.wide) {
            // single pass per codeword: the tables only, no work arrays
            if (int rc = ensure_gf16_tables(ctx)) return rc;
            Gf16Dev g = ctx->gf16;
            g.cus = ctx->cus;
            e = launch_encode_gf16(cs, g, st);
        } else {
            // multi-pass through per-stream work arrays, 64-bit per-symbol bases (the
            // wide form of k <= 512 as well)
            cs.wide = 1u;
            const uint64_t per_cw = (uint64_t)ceil_pow2(cs.k) * cs.S;
            StreamScratch& ss = stream_scratch(ctx, st);
            std::lock_guard<std::mutex> lk(ss.mu);
            Gf16Dev g;
            if (int rc = gf16_for_stream(ctx, ss, st, gf16_budget(per_cw, cs.count, ctx->work_budget.load()), 0, &g))
                return rc;
            g.cus = ctx->cus;
            e = launch_encode_gf16(cs, g, st);
        }
    }
    if (e == hipErrorOutOfMemory) return fail(RSM_ENOMEM, "encode: GF(2^16) scratch too small (work arrays below one byte slab)");
    if (e != hipSuccess) return hip_fail(e, "encode kernel launch");
    return RSM_OK;
}

int launch_decode(rsm_ctx* ctx, const DecodeSet& ds0, hipStream_t st) {
    DecodeSet ds = ds0;
    hipError_t e;
    // each half of a row / column (its k data or k parity cells) from its own base
    const uint64_t es = ds.axis == 0 ? (uint64_t)ds.S : 2ull * ds.k * ds.S;
    ds.wide = narrow_ok(ctx, ds.k, es, ds.S) ? 0u : 1u;
    // (the five-pass diagnostic GF(2^16) form addresses the whole square with 32-bit offsets)
    if (field_bits(ds.k) == 16 && dec16_needs_work() && 4ull * ds.k * ds.k * ds.S >= kOffsetLimit) ds.wide = 1u;
    if (ds.wide && (ds.in_base || ds.mirror))
        return fail(RSM_EUNSUPPORTED, "decode: zero-copy form of a codeword over the offset limit");
    if (ds.wide) ds.pitch = ds.S;
    if (field_bits(ds.k) == 8) {
        if (ds.wide) {
            e = launch_decode_gf8_wide(ds, st);
        } else {
            ds.chunks = (ds.S + 255) / 256;
            e = launch_decode_gf8(ds, st);
        }
    } else {
        if (!gf16_supported(ds.k)) return fail(RSM_EUNSUPPORTED, "decode: k=%u exceeds 32768", ds.k);
        const uint64_t n = 2ull * ceil_pow2(ds.k);
        StreamScratch& ss = stream_scratch(ctx, st);
        std::lock_guard<std::mutex> lk(ss.mu);
        Gf16Dev g;
        if (!gf16_generic(ds.k) && !ds.wide && !dec16_needs_work()) {
            // single pass per codeword: only the error locators of every codeword
            if (int rc = gf16_for_stream(ctx, ss, st, 0, ds.count * n * sizeof(uint16_t), &g)) return rc;
        } else {
            if (gf16_generic(ds.k)) {
                ds.wide = 1u;
                ds.pitch = ds.S;
            }
            const uint64_t per_cw = 2ull * n * ds.S;
            const uint64_t budget = gf16_budget(per_cw, ds.count, ctx->work_budget.load());
            // codewords per batch: of whole shares, or of the byte slab the launcher
            // cuts when one codeword's arrays exceed the budget (kernels_gf16.hip g16_slab)
            const uint64_t slab = per_cw <= budget ? ds.S : budget / (2 * n) / 64 * 64;
            uint64_t cws = slab ? budget / (2 * n * slab) : 1u;
            if (cws > ds.count) cws = ds.count;
            if (int rc = gf16_for_stream(ctx, ss, st, budget, (cws ? cws : 1u) * n * sizeof(uint16_t), &g)) return rc;
        }
        e = launch_decode_gf16(ds, g, st);
    }
    if (e == hipErrorOutOfMemory)
        return fail(RSM_ENOMEM, "decode: GF(2^16) scratch too small (error locators or work arrays below one codeword / byte slab)");
    if (e != hipSuccess) return hip_fail(e, "decode kernel launch");
    return RSM_OK;
}

// Two-phase in-place extension of `count` squares (extendeddatasquare.go:154-227):
//   phase 1: every row r < k: Q0 row -> Q1 row            (erasureExtendRow)
//   phase 2: every column c < 2k: [Q0|Q1] column -> [Q2|Q3] column
// Phase 2 computes Q2 exactly as erasureExtendCol and Q3 by column-encoding Q1,
// which equals the reference's row-encoding of Q2 by linearity of the 2D code
// (extendeddatasquare.go:204-207; asserted in tests against the oracle, which
// runs the reference order).
static CodewordSet rows_set(uint8_t* d_eds, uint32_t k, uint32_t S, uint32_t count) {
    const uint64_t W = 2ull * k;
    CodewordSet rows{};
    rows.base = rows.out_base = d_eds;
    rows.square_stride = W * W * S;
    rows.cw_stride = W * S;
    rows.elem_stride = S;
    rows.out_offset = (uint64_t)k * S;
    rows.per_square = k;
    rows.count = k * count;
    rows.k = k;
    rows.S = S;
    rows.pass = 0;
    return rows;
}

static CodewordSet cols_set(uint8_t* d_eds, uint32_t k, uint32_t S, uint32_t count) {
    const uint64_t W = 2ull * k;
    CodewordSet cols = rows_set(d_eds, k, S, count);
    cols.cw_stride = S;
    cols.elem_stride = W * S;
    cols.out_offset = (uint64_t)k * W * S;
    cols.per_square = (uint32_t)W;
    cols.count = (uint32_t)W * count;
    cols.pass = 1;
    return cols;
}

int check_queue_reports(rsm_ctx* ctx, hipStream_t st) {
    bool stuck = false;
    std::lock_guard<std::mutex> lk(ctx->scratch_mu);
    for (auto& kv : ctx->scratch) {
        if (st && kv.first != st) continue;
        // the stream's lock: extend_squares_queue allocates the word under it (lock
        // order scratch_mu -> StreamScratch::mu, as everywhere else)
        std::lock_guard<std::mutex> lk2(kv.second->mu);
        volatile uint32_t* w = static_cast<volatile uint32_t*>(kv.second->qerr.ptr);
        if (w && *w) {
            *w = 0;
            stuck = true;
            // a timed-out wait may leave the stream's shared hand-off words non-zero (the
            // launch drains without its final re-zeroing): clear them, in stream order
            // behind that launch, before any later launch on this stream reads them
            if (kv.second->queue.ptr) (void)hipMemsetAsync(kv.second->queue.ptr, 0, kv.second->queue.cap, kv.first);
        }
    }
    return stuck ? fail(RSM_EDEVICE, "single-launch extension: a column set timed out waiting for its rows "
                                     "(that launch's output is invalid)")
                 : RSM_OK;
}

// The stream's device-side hand-off words (zeroed once: every launch that uses them
// leaves them zeroed) and its pinned stuck-wait report word; caller holds ss.mu.
static int queue_words(StreamScratch& ss, uint32_t count, hipStream_t st) {
    const size_t bytes = (kQueueFixedWords + 2 * (size_t)count) * 4;
    hipError_t e;
    if (bytes > ss.queue.cap) {
        if ((e = hipStreamSynchronize(st)) != hipSuccess || (e = ss.queue.ensure(bytes)) != hipSuccess ||
            (e = hipMemsetAsync(ss.queue.ptr, 0, ss.queue.cap, st)) != hipSuccess)
            return hip_fail(e, "single-launch extension: queue words");
    }
    if (!ss.qerr.ptr) {
        if ((e = ss.qerr.ensure(64)) != hipSuccess) return hip_fail(e, "single-launch extension: report word");
        *static_cast<volatile uint32_t*>(ss.qerr.ptr) = 0;
    }
    return RSM_OK;
}

int extend_squares_queue(rsm_ctx* ctx, uint8_t* d_eds, uint32_t k, uint32_t S, uint32_t count, hipStream_t st,
                         uint32_t delay, uint32_t margin) {
    if (field_bits(k) != 8 || count == 0) return RSM_EUNSUPPORTED;
    QueuePlan p{};
    // parity from its own base: the symbol offsets span one half (narrow_fits)
    p.rows = rebased(rows_set(d_eds, k, S, count));
    p.cols = rebased(cols_set(d_eds, k, S, count));
    // persistent grid: every CU, or the row-pass cap of rsm_ctx_set_pass_grid
    const uint32_t cap = ctx->pass_grid[0].load(std::memory_order_relaxed);
    p.rows.grid = p.cols.grid = cap && cap < ctx->cus ? cap : ctx->cus;
    p.rows.chunks = p.cols.chunks = (S + 255) / 256;
    if (!bs128_queue_applicable(p.rows, p.cols)) return RSM_EUNSUPPORTED;
    if (int rc = check_queue_reports(ctx, st)) return rc;
    p.count = count;
    p.rn = (uint32_t)((uint64_t)k * S / 2048);
    p.cn = 2 * p.rn;
    p.delay = (delay > count ? count : delay) * p.rn;
    p.nmain = 2 * count * p.rn;
    p.nq1 = count * p.rn;
    p.margin = margin == ~0u ? p.rn / 2 : margin;
    StreamScratch& ss = stream_scratch(ctx, st);
    std::lock_guard<std::mutex> lk(ss.mu);
#ifdef RSM_DIAG
    // XCD-affine queues (diagnostic): 8 blocks of queue words, zeroed before each launch
    const bool xcdq = bs128_diag_xcd_queues();
    if (xcdq && count % 8 != 0) return fail(RSM_EINVAL, "XCD-affine queues need a multiple of 8 squares");
    if (int rc = queue_words(ss, xcdq ? count + 7 * kQueueFixedWords / 2 : count, st)) return rc;
    if (xcdq) {
        if (hipError_t e = hipMemsetAsync(ss.queue.ptr, 0, ss.queue.cap, st)) return hip_fail(e, "queue words");
    }
#else
    if (int rc = queue_words(ss, count, st)) return rc;
#endif
    p.ctr = static_cast<uint32_t*>(ss.queue.ptr);
    p.err = static_cast<uint32_t*>(ss.qerr.ptr);
    if (hipError_t e = launch_extend_gf8_bs128_queue(p, st)) return hip_fail(e, "single-launch extension");
    return RSM_OK;
}

// Latency form for one or a few squares with 65 <= k <= 128 (what a cgo
// ComputeExtendedDataSquare call extends): launch 1 = rows of Q0 -> Q1 together with
// columns of Q0 -> Q2, launch 2 = columns of Q1 -> Q3, both on the split byte-table
// encoder (NW waves per codeword chunk), so each phase spreads over every CU instead
// of the queue kernel's 64 + 32 sets of ~16 us each.
int extend_squares_split(rsm_ctx* ctx, uint8_t* d_eds, uint32_t k, uint32_t S, uint32_t count, hipStream_t st) {
    const uint32_t M = ceil_pow2(k);
    if (field_bits(k) != 8 || count == 0) return RSM_EUNSUPPORTED;
    // M = 32 / 64 (round 6): the split form too (encode_gf8_splitm_kernel) for up to
    // split_max squares; larger batches take the byte-table passes
    if (M != 128 && M != 16 && M != 32 && M != 64) return RSM_EUNSUPPORTED;
    const CodewordSet rows = rows_set(d_eds, k, S, count);
    CodewordSet c0 = cols_set(d_eds, k, S, count);  // columns 0 .. k-1 (Q0 -> Q2)
    c0.per_square = k;
    c0.count = k * count;
    CodewordSet c1 = c0;  // columns k .. 2k-1 (Q1 -> Q3)
    c1.base = c1.out_base = d_eds + (uint64_t)k * S;
    hipError_t e;
    // one square: ONE launch whose Q1-column workgroups wait on the device for the row
    // tasks -- 3 k ceil(S / 256) workgroups of 8 waves, resident at once when they fit
    // 4 per CU (otherwise the two launches below)
    const uint64_t wgs = 3ull * k * ((S + 255) / 256);
    if (M == 128 && count == 1 && wgs <= 4ull * ctx->cus && split_fused_enabled()) {
        if (int rc = check_queue_reports(ctx, st)) return rc;
        StreamScratch& ss = stream_scratch(ctx, st);
        std::lock_guard<std::mutex> lk(ss.mu);
        if (int rc = queue_words(ss, 640, st)) return rc;  // >= 1280 words: counters + 64 done flags
        if ((e = launch_extend_gf8_split_fused(rows, c0, c1, static_cast<uint32_t*>(ss.queue.ptr),
                                               static_cast<uint32_t*>(ss.qerr.ptr), st)) != hipSuccess)
            return hip_fail(e, "split extension (one launch)");
        return RSM_OK;
    }
    // launch 1 = rows + Q0 columns, launch 2 = Q1 columns (moving half of the Q0
    // columns into launch 2 measured 25.9 against 21.9 us per square, r03m)
    // waves per task: 16 for one square (shorter per-wave chains, twice the waves to hide
    // the latencies of a launch that runs one wave of tasks), 8 for batches (issue-bound:
    // the 16-wave form's two extra exchanges cost more than they hide)
    const int nw = count == 1 ? kSplitWavesOne : 8;
    if ((e = launch_encode_gf8_split(rows, &c0, st, nw)) != hipSuccess) return hip_fail(e, "split extension (launch 1)");
    if ((e = launch_encode_gf8_split(c1, nullptr, st, nw)) != hipSuccess) return hip_fail(e, "split extension (launch 2)");
    return RSM_OK;
}

// Two-phase in-place extension; batches of k = 128 squares run both phases as one
// queue-driven launch (extend_squares_queue), which re-reads Q0 and Q1 from the
// Infinity Cache instead of HBM; up to ctx->split_max squares take the latency form
// (rsm_ctx_set_split_max; default 12: the crossover, profiles/r03_single.jsonl).
int extend_squares(rsm_ctx* ctx, uint8_t* d_eds, uint32_t k, uint32_t S, uint32_t count, hipStream_t st,
                   int phases) {
    const uint64_t W = 2ull * k;
    // the latency and queue forms address the column halves with 32-bit offsets; wider
    // squares take the two passes below, whose launches pick the wide forms
    const bool narrow = narrow_ok(ctx, k, W * S, S);
    // (9 <= k <= 64: the split form wins up to 64 squares per call, profiles/r06w_small_ab.jsonl,
    // r06y_small16_ab.jsonl)
    const uint32_t smax = ctx->split_max.load(std::memory_order_relaxed);
    const uint32_t M = ceil_pow2(k);
    const uint32_t split_limit = smax && (M == 16 || M == 32 || M == 64) && smax < kSplitSmallBatch ? kSplitSmallBatch : smax;
    if (phases == 3 && narrow && count <= split_limit) {
        const int rc = extend_squares_split(ctx, d_eds, k, S, count, st);
        if (rc != RSM_EUNSUPPORTED) return rc;
    }
    if (phases == 3 && narrow) {  // k = 128: one queue-driven launch
        const int rc = extend_squares_queue(ctx, d_eds, k, S, count, st);
        if (rc != RSM_EUNSUPPORTED) return rc;
    }
    if (phases & 1) {
        CodewordSet rows{};
        rows.base = d_eds;
        rows.square_stride = W * W * S;
        rows.cw_stride = W * S;
        rows.elem_stride = S;
        rows.out_offset = (uint64_t)k * S;
        rows.per_square = k;
        rows.count = k * count;
        rows.k = k;
        rows.S = S;
        rows.pass = 0;
        if (int rc = launch_encode(ctx, rows, st)) return rc;
    }
    if (!(phases & 2)) return RSM_OK;
    CodewordSet cols{};
    cols.base = d_eds;
    cols.square_stride = W * W * S;
    cols.cw_stride = S;
    cols.elem_stride = W * S;
    cols.out_offset = (uint64_t)k * W * S;
    cols.per_square = (uint32_t)W;
    cols.count = (uint32_t)W * count;
    cols.k = k;
    cols.S = S;
    cols.pass = 1;
    return launch_encode(ctx, cols, st);
}

int device_roots(rsm_ctx* ctx, const uint8_t* d_eds, uint32_t W, uint32_t S, uint8_t* d_roots, hipStream_t st,
                 uint32_t squares) {
    if (!roots_dev_supported(W)) return fail(RSM_EUNSUPPORTED, "device roots: width %u not supported", W);
    if ((uint64_t)W * W * squares >= (1ull << 32) || squares > 65535)
        return fail(RSM_EINVAL, "device roots: %u squares of width %u exceed one launch", squares, W);
    StreamScratch& ss = stream_scratch(ctx, st);
    std::lock_guard<std::mutex> lk(ss.mu);
    const size_t need = (size_t)W * W * 32 * squares;
    hipError_t e;
    if (need > ss.leaf.cap) {
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
        if ((e = ss.leaf.ensure(need)) != hipSuccess) return hip_fail(e, "hipMalloc (leaf digests)");
    }
    if ((e = launch_roots(d_eds, W, S, squares, static_cast<uint32_t*>(ss.leaf.ptr), d_roots, st)) != hipSuccess)
        return hip_fail(e, "roots kernel launch");
    return RSM_OK;
}

bool device_tree_for(rsm_tree_root_fn fn, void* user, uint32_t W, DevTree* out) {
    DevTree t;
    if (fn == nullptr || fn == rsm_default_tree_root) {
        if (!roots_dev_supported(W)) return false;
    } else if (fn == rsm_nmt_tree_root && user) {
        t.nmt = true;
        t.p = *static_cast<const rsm_nmt_params*>(user);
        // the plugin's own errors (past the square, too short) stay on the host path
        if (!nmt_dev_supported(W, t.p.namespace_size) || t.p.square_size == 0 || W > 2 * t.p.square_size)
            return false;
        t.root_len = 2 * t.p.namespace_size + 32;
    } else {
        return false;
    }
    *out = t;
    return true;
}

int device_tree_roots(rsm_ctx* ctx, const DevTree& t, const uint8_t* d_eds, uint32_t W, uint32_t S,
                      uint8_t* d_roots, uint32_t* d_status, hipStream_t st, uint32_t squares) {
    hipError_t e;
    if (!t.nmt) {
        if (d_status && (e = hipMemsetAsync(d_status, 0, (size_t)squares * 2 * W * 4, st)) != hipSuccess)
            return hip_fail(e, "hipMemsetAsync (status)");
        return device_roots(ctx, d_eds, W, S, d_roots, st, squares);
    }
    if (S < t.p.namespace_size) return fail(RSM_ETREE, "data is too short to contain namespace ID");
    StreamScratch& ss = stream_scratch(ctx, st);
    std::lock_guard<std::mutex> lk(ss.mu);
    const size_t need = (size_t)squares * W * W * 64;
    if (need > ss.leaf.cap) {
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
        if ((e = ss.leaf.ensure(need)) != hipSuccess) return hip_fail(e, "hipMalloc (NMT leaves)");
    }
    if ((e = launch_nmt_roots(d_eds, W, S, t.p.namespace_size, t.p.square_size, t.p.ignore_max_namespace,
                              static_cast<uint32_t*>(ss.leaf.ptr), d_roots, d_status, st, squares)) != hipSuccess)
        return hip_fail(e, "NMT roots kernel launch");
    return RSM_OK;
}

// One square host -> device -> host on `st`: the ODS goes straight into the EDS's
// top-left quadrant (the EDS aliases the ODS); only Q1, Q2 and Q3 come back, the
// caller's Q0 quadrant is filled from its own ODS on the host.
static int host_square(rsm_ctx* ctx, const uint8_t* ods, size_t ods_pitch, uint8_t* eds, uint8_t* d, uint32_t k,
                       uint32_t S, hipStream_t st) {
    const size_t W = 2ull * k, row = W * S, half = (size_t)k * S;
    hipError_t e;
    if ((e = hipMemcpy2DAsync(d, row, ods, ods_pitch, half, k, hipMemcpyHostToDevice, st)) != hipSuccess)
        return hip_fail(e, "hipMemcpy2DAsync H2D");
    if (int rc = extend_squares(ctx, d, k, S, 1, st)) return rc;
    if ((e = hipMemcpy2DAsync(eds + half, row, d + half, row, half, k, hipMemcpyDeviceToHost, st)) != hipSuccess)
        return hip_fail(e, "hipMemcpy2DAsync D2H (Q1)");
    if ((e = hipMemcpyAsync(eds + (size_t)k * row, d + (size_t)k * row, (size_t)k * row, hipMemcpyDeviceToHost, st)) !=
        hipSuccess)
        return hip_fail(e, "hipMemcpyAsync D2H (Q2|Q3)");
    return RSM_OK;
}

static void fill_q0(const uint8_t* ods, uint8_t* eds, uint32_t k, uint32_t S) {
    const size_t row = 2ull * k * S, half = (size_t)k * S;
    if (eds == ods) return;
    for (uint32_t r = 0; r < k; ++r) memcpy(eds + r * row, ods + r * half, half);
}

// Completion wait of a Codec call's lane.  Diagnostic builds may spin on
// hipStreamQuery for up to `codec_spin_us` before blocking (A/B of the wake-up
// latency of hipStreamSynchronize for ~20 us calls).
#ifdef RSM_DIAG
static std::atomic<uint32_t> g_codec_spin_us{0};
void set_codec_spin_diag(uint32_t us) { g_codec_spin_us.store(us); }
static uint32_t codec_spin_us() { return g_codec_spin_us.load(); }
#else
static uint32_t codec_spin_us() { return 0; }
#endif
static hipError_t lane_wait(hipStream_t s) {
    if (const uint32_t spin = codec_spin_us()) {
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            const hipError_t q = hipStreamQuery(s);
            if (q != hipErrorNotReady) return q;
            if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin)) break;
        }
    }
    return hipStreamSynchronize(s);
}
}  // namespace rsm

using namespace rsm;

// ---------------------------------------------------------------------------
// C ABI: context
// ---------------------------------------------------------------------------
extern "C" {

const char* rsm_last_error(void) { return last_error(); }
const char* rsm_version(void) { return "rsmt2d-mi355x 0.2.0 (gfx950)"; }

int rsm_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int rsm_ctx_create(int device, rsm_ctx** out) {
    if (!out) return fail(RSM_EINVAL, "rsm_ctx_create: out is NULL");
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0)
        return fail(RSM_EDEVICE, "no HIP device available (%s): the MI355X path has no CPU fallback",
                    e == hipSuccess ? "0 devices" : hipGetErrorString(e));
    if (device < 0 || device >= n) return fail(RSM_EINVAL, "device %d out of range [0,%d)", device, n);
    e = hipSetDevice(device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    auto* c = new (std::nothrow) rsm_ctx();
    if (!c) return fail(RSM_ENOMEM, "rsm_ctx_create: out of memory");
    c->device = device;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
        c->cus = (uint32_t)cus;
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = c->zero_index.ensure(64);
    if (e == hipSuccess) e = hipMemset(c->zero_index.ptr, 0, 64);
    if (e != hipSuccess) {
        if (c->stream) (void)hipStreamDestroy(c->stream);
        delete c;
        return hip_fail(e, "rsm_ctx_create");
    }
    *out = c;
    return RSM_OK;
}

void rsm_ctx_destroy(rsm_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipDeviceSynchronize();
    for (auto& l : ctx->lanes) {
        (void)hipStreamDestroy(l->stream);
        for (hipEvent_t ev : l->ev)
            if (ev) (void)hipEventDestroy(ev);
    }
    ctx->lanes.clear();
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

int rsm_ctx_device(const rsm_ctx* ctx) { return ctx ? ctx->device : -1; }

int rsm_ctx_set_pass_grid(rsm_ctx* ctx, int pass, int cus, int* previous) {
    if (!ctx || (pass != 0 && pass != 1) || cus < 0)
        return fail(RSM_EINVAL, "rsm_ctx_set_pass_grid: pass must be 0 (rows) or 1 (columns), cus >= 0");
    const uint32_t prev = ctx->pass_grid[pass].exchange((uint32_t)cus);
    if (previous) *previous = (int)prev;
    return RSM_OK;
}

int rsm_ctx_set_limits(rsm_ctx* ctx, uint64_t offset_limit, uint64_t work_budget) {
    if (!ctx) return fail(RSM_EINVAL, "rsm_ctx_set_limits: NULL ctx");
    if (offset_limit > kOffsetLimit) return fail(RSM_EINVAL, "rsm_ctx_set_limits: offset limit above 2^31");
    ctx->offset_limit.store(offset_limit ? offset_limit : kOffsetLimit);
    ctx->work_budget.store(work_budget ? work_budget : (1ull << 30));
    return RSM_OK;
}

int rsm_ctx_set_split_max(rsm_ctx* ctx, int squares, int* previous) {
    if (!ctx || squares < 0) return fail(RSM_EINVAL, "rsm_ctx_set_split_max: squares must be >= 0");
    const uint32_t prev = ctx->split_max.exchange((uint32_t)squares);
    if (previous) *previous = (int)prev;
    return RSM_OK;
}

// ---------------------------------------------------------------------------
// C ABI: Codec
// ---------------------------------------------------------------------------
const char* rsm_codec_name(void) { return "Leopard"; }
int64_t rsm_codec_max_chunks(void) { return (int64_t)32768 * 32768; }
int rsm_codec_validate_chunk_size(int64_t share_size) { return validate_chunk_size(share_size); }
int rsm_codec_field_bits(uint32_t k) { return field_bits(k); }

// Device address of a lane's pinned staging: the Codec calls of GF(2^8) codewords with
// 65 <= k <= 128 and of GF(2^16) codewords with k <= 512 (the single-pass kernels) run
// zero-copy -- the kernels read the shares from the pinned buffer over PCIe and write
// their results back there (no DMA copies; the GF(2^16) decoder's intermediate passes
// stay in device scratch); nullptr where the runtime cannot map it (the copy path then).
static void* lane_host_dev(Lane& L) {
    void* p = nullptr;
    if (hipHostGetDevicePointer(&p, L.host.ptr, 0) != hipSuccess) return nullptr;
    return p;
}
static bool codec_zero_copy(uint32_t k) {
    return (field_bits(k) == 8 && ceil_pow2(k) == 128) || (field_bits(k) == 16 && !gf16_generic(k));
}

int rsm_encode(rsm_ctx* ctx, const uint8_t* const* data, uint32_t k, uint32_t share_size,
               uint8_t* const* parity) {
    if (!ctx || !data || !parity || k == 0) return fail(RSM_EINVAL, "rsm_encode: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (share_size == 0) return fail(RSM_ESHAPE, "rsm_encode: zero-length shares");
    if (2ull * k > 65536ull) return fail(RSM_ESHAPE, "rsm_encode: %u shards exceed the Leopard limit", 2 * k);
    for (uint32_t i = 0; i < k; ++i)
        if (!data[i]) return fail(RSM_EINVAL, "rsm_encode: data[%u] is nil", i);
    if (int rc = use_device(ctx)) return rc;
    LaneGuard g(ctx);
    if (!g.lane) return g.rc;
    Lane& L = *g.lane;
    const size_t S = share_size;
    const size_t bytes = 2ull * k * S;
    hipError_t e;
    if ((e = L.host.ensure(bytes)) != hipSuccess) return hip_fail(e, "hipHostMalloc");
    if ((e = L.dev.ensure(bytes)) != hipSuccess) return hip_fail(e, "hipMalloc");
    uint8_t* h = static_cast<uint8_t*>(L.host.ptr);
    for (uint32_t i = 0; i < k; ++i) memcpy(h + i * S, data[i], S);
    if (codec_zero_copy(k))
        if (uint8_t* hd = static_cast<uint8_t*>(lane_host_dev(L))) {
            // GF(2^8): the latency form (the split byte-table encoder: one 8-wave
            // workgroup per 256-B chunk); GF(2^16): the single-pass encoder -- straight on
            // the pinned buffer
            CodewordSet cs{};
            cs.base = cs.out_base = hd;
            cs.elem_stride = S;
            cs.out_offset = (uint64_t)k * S;
            cs.per_square = 1;
            cs.count = 1;
            cs.k = k;
            cs.S = share_size;
            cs.pass = 1;
            if (field_bits(k) == 8) {
                if ((e = launch_encode_gf8_split(cs, nullptr, L.stream, kSplitWavesOne)) != hipSuccess)
                    return hip_fail(e, "encode kernel launch");
            } else if (int rc = launch_encode(ctx, cs, L.stream)) {
                return rc;
            }
            if ((e = lane_wait(L.stream)) != hipSuccess) return hip_fail(e, "encode");
            for (uint32_t i = 0; i < k; ++i) memcpy(parity[i], h + (k + i) * S, S);
            return RSM_OK;
        }
    uint8_t* d = static_cast<uint8_t*>(L.dev.ptr);
    if ((e = hipMemcpyAsync(d, h, k * S, hipMemcpyHostToDevice, L.stream)) != hipSuccess)
        return hip_fail(e, "hipMemcpyAsync H2D");
    CodewordSet cs{};
    cs.base = d;
    cs.elem_stride = S;
    cs.out_offset = (uint64_t)k * S;
    cs.per_square = 1;
    cs.count = 1;
    cs.k = k;
    cs.S = share_size;
    cs.pass = 1;
    if (int rc = launch_encode(ctx, cs, L.stream)) return rc;
    if ((e = hipMemcpyAsync(h + k * S, d + k * S, k * S, hipMemcpyDeviceToHost, L.stream)) != hipSuccess)
        return hip_fail(e, "hipMemcpyAsync D2H");
    if ((e = lane_wait(L.stream)) != hipSuccess) return hip_fail(e, "encode");
    for (uint32_t i = 0; i < k; ++i) memcpy(parity[i], h + (k + i) * S, S);
    return RSM_OK;
}

int rsm_decode(rsm_ctx* ctx, uint8_t* const* shares, const uint8_t* present, uint32_t n,
               uint32_t share_size) {
    if (!ctx || !shares || !present || n == 0 || (n & 1u)) return fail(RSM_EINVAL, "rsm_decode: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    const uint32_t k = n / 2;
    uint32_t np = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (!shares[i]) return fail(RSM_EINVAL, "rsm_decode: shares[%u] buffer is NULL", i);
        np += present[i] ? 1u : 0u;
    }
    if (np == n) return RSM_OK;
    if (np < k) return fail(RSM_ETOOFEW, "too few shards given (%u of %u, need %u)", np, n, k);
    if (int rc = use_device(ctx)) return rc;
    LaneGuard g(ctx);
    if (!g.lane) return g.rc;
    Lane& L = *g.lane;
    const size_t S = share_size;
    const size_t bytes = (size_t)n * S;
    hipError_t e;
    if ((e = L.host.ensure(bytes + n + 16)) != hipSuccess) return hip_fail(e, "hipHostMalloc");
    if ((e = L.dev.ensure(bytes)) != hipSuccess) return hip_fail(e, "hipMalloc");
    if ((e = L.aux.ensure(n + 16)) != hipSuccess) return hip_fail(e, "hipMalloc");
    uint8_t* h = static_cast<uint8_t*>(L.host.ptr);
    // the zero-copy decoders never use an absent share's bytes (the GF(2^8) split decoder
    // scales them by zero, the GF(2^16) ones do not load them), so only the copy path
    // clears them
    uint8_t* const hd = codec_zero_copy(k) ? static_cast<uint8_t*>(lane_host_dev(L)) : nullptr;
    for (uint32_t i = 0; i < n; ++i) {
        if (present[i]) memcpy(h + i * S, shares[i], S);
        else if (!hd) memset(h + i * S, 0, S);
    }
    uint8_t* hp = h + bytes;
    for (uint32_t i = 0; i < n; ++i) hp[i] = present[i] ? 1 : 0;
    if (hd) {
        // the decoder straight on the pinned buffer: it reads the points and the
        // presence bytes over PCIe and writes only the missing shares back
        DecodeSet ds{};
        ds.base = hd;
        ds.presence = hd + bytes;
        ds.indices = static_cast<const uint32_t*>(ctx->zero_index.ptr);
        ds.count = 1;
        ds.axis = 0;
        ds.k = k;
        ds.S = share_size;
        if (int rc = launch_decode(ctx, ds, L.stream)) return rc;
        if ((e = lane_wait(L.stream)) != hipSuccess) return hip_fail(e, "decode");
        for (uint32_t i = 0; i < n; ++i)
            if (!present[i]) memcpy(shares[i], h + i * S, S);
        return RSM_OK;
    }
    uint8_t* d = static_cast<uint8_t*>(L.dev.ptr);
    uint8_t* dpres = static_cast<uint8_t*>(L.aux.ptr);
    if ((e = hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, L.stream)) != hipSuccess)
        return hip_fail(e, "hipMemcpyAsync H2D");
    if ((e = hipMemcpyAsync(dpres, hp, n, hipMemcpyHostToDevice, L.stream)) != hipSuccess)
        return hip_fail(e, "hipMemcpyAsync H2D");
    DecodeSet ds{};
    ds.base = d;
    ds.presence = dpres;
    ds.indices = static_cast<const uint32_t*>(ctx->zero_index.ptr);
    ds.count = 1;
    ds.axis = 0;  // a single codeword is row 0 of a 1 x 2k "square"
    ds.k = k;
    ds.S = share_size;
    if (int rc = launch_decode(ctx, ds, L.stream)) return rc;
    if ((e = hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, L.stream)) != hipSuccess)
        return hip_fail(e, "hipMemcpyAsync D2H");
    if ((e = lane_wait(L.stream)) != hipSuccess) return hip_fail(e, "decode");
    for (uint32_t i = 0; i < n; ++i)
        if (!present[i]) memcpy(shares[i], h + i * S, S);
    return RSM_OK;
}

int rsm_extend_square(rsm_ctx* ctx, const uint8_t* ods, uint32_t k, uint32_t share_size, uint8_t* eds) {
    if (!ctx || !ods || !eds || k == 0) return fail(RSM_EINVAL, "rsm_extend_square: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (int rc = use_device(ctx)) return rc;
    LaneGuard g(ctx);
    if (!g.lane) return g.rc;
    const size_t S = share_size, W = 2ull * k;
    hipError_t e;
    if ((e = g.lane->dev.ensure(W * W * S)) != hipSuccess) return hip_fail(e, "hipMalloc");
    if (int rc = host_square(ctx, ods, (size_t)k * S, eds, static_cast<uint8_t*>(g.lane->dev.ptr), k, share_size,
                             g.lane->stream))
        return rc;
    fill_q0(ods, eds, k, share_size);
    if ((e = hipStreamSynchronize(g.lane->stream)) != hipSuccess) return hip_fail(e, "extend");
    return RSM_OK;
}

// The EDS buffer's top-left quadrant already holds the ODS (the cgo shim gathers
// the [][]byte shares straight into a pinned EDS arena): extend it in place.
int rsm_extend_square_inplace_host(rsm_ctx* ctx, uint8_t* eds, uint32_t k, uint32_t share_size) {
    if (!ctx || !eds || k == 0) return fail(RSM_EINVAL, "rsm_extend_square_inplace_host: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (int rc = use_device(ctx)) return rc;
    LaneGuard g(ctx);
    if (!g.lane) return g.rc;
    const size_t S = share_size, W = 2ull * k;
    hipError_t e;
    if ((e = g.lane->dev.ensure(W * W * S)) != hipSuccess) return hip_fail(e, "hipMalloc");
    if (int rc = host_square(ctx, eds, W * S, eds, static_cast<uint8_t*>(g.lane->dev.ptr), k, share_size,
                             g.lane->stream))
        return rc;
    if ((e = hipStreamSynchronize(g.lane->stream)) != hipSuccess) return hip_fail(e, "extend");
    return RSM_OK;
}

// Host-memory batch (ComputeExtendedDataSquare over many squares from host
// buffers): square i uses lane i % n_lanes, so the H2D of one square, the
// extension of another and the D2H of a third overlap on the copy engines and the
// CUs.  With pinned buffers (rsm_host_alloc) every copy is an async DMA.
int rsm_extend_squares_host(rsm_ctx* ctx, const uint8_t* ods, uint32_t k, uint32_t share_size, uint32_t count,
                            uint8_t* eds) {
    if (!ctx || !ods || !eds || k == 0) return fail(RSM_EINVAL, "rsm_extend_squares_host: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (count == 0) return RSM_OK;
    if (int rc = use_device(ctx)) return rc;
    constexpr int kLanes = 3;
    const int nl = (int)std::min<uint32_t>(count, kLanes);
    Lane* lanes[kLanes] = {};
    // all lanes in one step (a caller holding some while waiting for more could
    // deadlock against other multi-lane callers); released on every return path,
    // after their streams have drained
    if (int rc = acquire_lanes(ctx, nl, lanes)) return rc;
    struct Release {
        rsm_ctx* ctx;
        Lane** l;
        int n;
        ~Release() {
            for (int i = 0; i < n; ++i) {
                (void)hipStreamSynchronize(l[i]->stream);
                release_lane(ctx, l[i]);
            }
        }
    } rel{ctx, lanes, nl};
    const size_t S = share_size, W = 2ull * k, ods_b = (size_t)k * k * S, eds_b = W * W * S;
    hipError_t e;
    for (int i = 0; i < nl; ++i)
        if ((e = lanes[i]->dev.ensure(eds_b)) != hipSuccess) return hip_fail(e, "hipMalloc");
    for (uint32_t i = 0; i < count; ++i) {
        Lane& L = *lanes[i % nl];
        if (int rc = host_square(ctx, ods + i * ods_b, (size_t)k * S, eds + i * eds_b, static_cast<uint8_t*>(L.dev.ptr),
                                 k, share_size, L.stream))
            return rc;
        fill_q0(ods + i * ods_b, eds + i * eds_b, k, share_size);
    }
    for (int i = 0; i < nl; ++i)
        if ((e = hipStreamSynchronize(lanes[i]->stream)) != hipSuccess) return hip_fail(e, "extend (host batch)");
    return RSM_OK;
}

int rsm_host_alloc(rsm_ctx* ctx, uint64_t bytes, void** out) {
    if (!ctx || !out) return fail(RSM_EINVAL, "rsm_host_alloc: bad arguments");
    *out = nullptr;
    if (int rc = use_device(ctx)) return rc;
    hipError_t e = hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault);
    return e == hipSuccess ? RSM_OK : hip_fail(e, "hipHostMalloc");
}

int rsm_host_free(rsm_ctx* ctx, void* p) {
    if (!ctx) return fail(RSM_EINVAL, "rsm_host_free: NULL ctx");
    if (!p) return RSM_OK;
    hipError_t e = hipHostFree(p);
    return e == hipSuccess ? RSM_OK : hip_fail(e, "hipHostFree");
}

static hipStream_t pick(rsm_ctx* ctx, void* stream) {
    return stream ? static_cast<hipStream_t>(stream) : ctx->stream;
}

int rsm_extend_squares_dev(rsm_ctx* ctx, void* d_eds, uint32_t k, uint32_t share_size, uint32_t count,
                           void* stream) {
    if (!ctx || !d_eds || k == 0) return fail(RSM_EINVAL, "rsm_extend_squares_dev: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (count == 0) return RSM_OK;
    if (int rc = use_device(ctx)) return rc;
    return extend_squares(ctx, static_cast<uint8_t*>(d_eds), k, share_size, count, pick(ctx, stream));
}

int rsm_extend_squares_phase_dev(rsm_ctx* ctx, void* d_eds, uint32_t k, uint32_t share_size, uint32_t count,
                                 int phase, void* stream) {
    if (!ctx || !d_eds || k == 0 || phase < 1 || phase > 3)
        return fail(RSM_EINVAL, "rsm_extend_squares_phase_dev: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (count == 0) return RSM_OK;
    if (int rc = use_device(ctx)) return rc;
    return extend_squares(ctx, static_cast<uint8_t*>(d_eds), k, share_size, count, pick(ctx, stream), phase);
}

// Row / column slices of ONE in-place [2k][2k][S] square -- the per-GPU units of the
// row-sharded multi-GPU schedule (erasureExtendRow / erasureExtendCol for a range).
int rsm_extend_rows_dev(rsm_ctx* ctx, void* d_eds, uint32_t k, uint32_t share_size, uint32_t row0, uint32_t nrows,
                        void* stream) {
    if (!ctx || !d_eds || k == 0 || row0 + nrows > 2 * k) return fail(RSM_EINVAL, "rsm_extend_rows_dev: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (nrows == 0) return RSM_OK;
    if (int rc = use_device(ctx)) return rc;
    const uint64_t W = 2ull * k, S = share_size;
    CodewordSet cs{};
    cs.base = static_cast<uint8_t*>(d_eds) + row0 * W * S;
    cs.cw_stride = W * S;
    cs.elem_stride = S;
    cs.out_offset = k * S;
    cs.per_square = nrows;
    cs.count = nrows;
    cs.k = k;
    cs.S = share_size;
    cs.pass = 0;
    return launch_encode(ctx, cs, pick(ctx, stream));
}

int rsm_extend_rows_blocks_dev(rsm_ctx* ctx, void* d_eds, uint32_t k, uint32_t share_size, uint32_t row0,
                               uint32_t nrows, void* d_blocks, uint32_t nblocks, void* stream) {
    if (!ctx || !d_eds || !d_blocks || k == 0 || nblocks == 0 || (2 * k) % nblocks != 0 || row0 + nrows > 2 * k)
        return fail(RSM_EINVAL, "rsm_extend_rows_blocks_dev: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (nrows == 0) return RSM_OK;
    if (int rc = use_device(ctx)) return rc;
    const uint64_t W = 2ull * k, S = share_size;
    const uint32_t cb = (uint32_t)(W / nblocks);
    const uint64_t blk = (uint64_t)nrows * cb * S;
    uint8_t* rows = static_cast<uint8_t*>(d_eds) + row0 * W * S;
    uint8_t* blocks = static_cast<uint8_t*>(d_blocks);
    hipStream_t st = pick(ctx, stream);
    // the single-pass GF(2^16) encoders store every cell a second time into its block (the
    // side output; every wave's 32 cells lie in one block when k and the block width are
    // multiples of 32): no copy pass
    if (field_bits(k) == 16 && !gf16_generic(k) && k % 32u == 0 && cb % 32u == 0 && narrow_ok(ctx, k, S, S)) {
        CodewordSet cs{};
        cs.base = rows;
        cs.cw_stride = W * S;
        cs.elem_stride = S;
        cs.out_offset = k * S;
        cs.per_square = nrows;
        cs.count = nrows;
        cs.k = k;
        cs.S = share_size;
        cs.pass = 0;
        cs.side = blocks;
        cs.side_blk = blk;
        cs.side_cols = cb;
        cs.side_self = ~0u;  // no block stays behind: all of them go to the exchange
        return launch_encode(ctx, cs, st);
    }
    // other shapes: the row pass, then one strided device copy per block
    if (int rc = rsm_extend_rows_dev(ctx, d_eds, k, share_size, row0, nrows, st)) return rc;
    for (uint32_t h = 0; h < nblocks; ++h)
        if (hipError_t e = hipMemcpy2DAsync(blocks + h * blk, (size_t)cb * S, rows + (uint64_t)h * cb * S, W * S,
                                            (size_t)cb * S, nrows, hipMemcpyDeviceToDevice, st))
            return hip_fail(e, "rsm_extend_rows_blocks_dev: block copy");
    return RSM_OK;
}

int rsm_extend_cols_dev(rsm_ctx* ctx, void* d_eds, uint32_t k, uint32_t share_size, uint32_t col0, uint32_t ncols,
                        void* stream) {
    if (!ctx || !d_eds || k == 0 || col0 + ncols > 2 * k) return fail(RSM_EINVAL, "rsm_extend_cols_dev: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (ncols == 0) return RSM_OK;
    if (int rc = use_device(ctx)) return rc;
    const uint64_t W = 2ull * k, S = share_size;
    CodewordSet cs{};
    cs.base = static_cast<uint8_t*>(d_eds) + col0 * S;
    cs.cw_stride = S;
    cs.elem_stride = W * S;
    cs.out_offset = k * W * S;
    cs.per_square = ncols;
    cs.count = ncols;
    cs.k = k;
    cs.S = share_size;
    cs.pass = 1;
    return launch_encode(ctx, cs, pick(ctx, stream));
}

int rsm_roots_dev(rsm_ctx* ctx, const void* d_eds, uint32_t width, uint32_t share_size, void* d_roots,
                  void* stream) {
    if (!ctx || !d_eds || !d_roots || width == 0) return fail(RSM_EINVAL, "rsm_roots_dev: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (int rc = use_device(ctx)) return rc;
    return device_roots(ctx, static_cast<const uint8_t*>(d_eds), width, share_size, static_cast<uint8_t*>(d_roots),
                        pick(ctx, stream));
}

int rsm_nmt_roots_dev(rsm_ctx* ctx, const void* d_eds, uint32_t width, uint32_t share_size,
                      const rsm_nmt_params* params, void* d_roots, void* d_status, void* stream) {
    if (!ctx || !d_eds || !d_roots || !params || width == 0) return fail(RSM_EINVAL, "rsm_nmt_roots_dev: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (int rc = use_device(ctx)) return rc;
    DevTree t;
    if (!device_tree_for(rsm_nmt_tree_root, const_cast<rsm_nmt_params*>(params), width, &t))
        return fail(RSM_EUNSUPPORTED, "device NMT roots: width %u, namespace size %u not supported", width,
                    params->namespace_size);
    return device_tree_roots(ctx, t, static_cast<const uint8_t*>(d_eds), width, share_size,
                             static_cast<uint8_t*>(d_roots), static_cast<uint32_t*>(d_status), pick(ctx, stream));
}

int rsm_nmt_roots_squares_dev(rsm_ctx* ctx, const void* d_eds, uint32_t width, uint32_t share_size, uint32_t count,
                              const rsm_nmt_params* params, void* d_roots, void* d_status, void* stream) {
    if (!ctx || !d_eds || !d_roots || !params || width == 0)
        return fail(RSM_EINVAL, "rsm_nmt_roots_squares_dev: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (count == 0) return RSM_OK;
    if (int rc = use_device(ctx)) return rc;
    DevTree t;
    if (!device_tree_for(rsm_nmt_tree_root, const_cast<rsm_nmt_params*>(params), width, &t))
        return fail(RSM_EUNSUPPORTED, "device NMT roots: width %u, namespace size %u not supported", width,
                    params->namespace_size);
    if ((uint64_t)count * width * width * 64 > (1ull << 34))
        return fail(RSM_EUNSUPPORTED, "rsm_nmt_roots_squares_dev: %u squares need over 16 GiB of leaf records", count);
    return device_tree_roots(ctx, t, static_cast<const uint8_t*>(d_eds), width, share_size,
                             static_cast<uint8_t*>(d_roots), static_cast<uint32_t*>(d_status), pick(ctx, stream), count);
}

int rsm_roots_squares_dev(rsm_ctx* ctx, const void* d_eds, uint32_t width, uint32_t share_size, uint32_t count,
                          void* d_roots, void* stream) {
    if (!ctx || !d_eds || !d_roots || width == 0) return fail(RSM_EINVAL, "rsm_roots_squares_dev: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (count == 0) return RSM_OK;
    if (int rc = use_device(ctx)) return rc;
    return device_roots(ctx, static_cast<const uint8_t*>(d_eds), width, share_size, static_cast<uint8_t*>(d_roots),
                        pick(ctx, stream), count);
}

int rsm_encode_batch_dev(rsm_ctx* ctx, const void* d_in, void* d_out, uint32_t k, uint32_t share_size,
                         uint32_t count, uint64_t cw_stride, uint64_t share_stride, void* stream) {
    if (!ctx || !d_in || !d_out || k == 0 || share_stride < share_size)
        return fail(RSM_EINVAL, "rsm_encode_batch_dev: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (count == 0) return RSM_OK;
    if (int rc = use_device(ctx)) return rc;
    CodewordSet cs{};
    cs.base = static_cast<uint8_t*>(const_cast<void*>(d_in));
    cs.out_base = static_cast<uint8_t*>(d_out);
    cs.cw_stride = cw_stride;
    cs.elem_stride = share_stride;
    cs.out_offset = 0;
    cs.per_square = count;
    cs.count = count;
    cs.k = k;
    cs.S = share_size;
    cs.pass = 1;
    return launch_encode(ctx, cs, pick(ctx, stream));
}

int rsm_decode_vectors_dev(rsm_ctx* ctx, void* d_eds, const uint8_t* d_presence, uint32_t k,
                           uint32_t share_size, int axis, const uint32_t* d_indices, uint32_t count,
                           void* stream) {
    if (!ctx || !d_eds || !d_presence || !d_indices || k == 0 || (axis != 0 && axis != 1))
        return fail(RSM_EINVAL, "rsm_decode_vectors_dev: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (count == 0) return RSM_OK;
    if (int rc = use_device(ctx)) return rc;
    DecodeSet ds{};
    ds.base = static_cast<uint8_t*>(d_eds);
    ds.presence = d_presence;
    ds.indices = d_indices;
    ds.count = count;
    ds.axis = (uint32_t)axis;
    ds.k = k;
    ds.S = share_size;
    return launch_decode(ctx, ds, pick(ctx, stream));
}

}  // extern "C"

// ---------------------------------------------------------------------------
// C ABI: device memory, streams, events and synthetic inputs on the context's own
// HIP runtime.  (A host process embedding a second HIP runtime -- e.g. PyTorch's
// bundled one -- must not hand its stream objects to this library; device
// pointers are shared fine.)
// ---------------------------------------------------------------------------
extern "C" {

void* rsm_ctx_stream(rsm_ctx* ctx) { return ctx ? static_cast<void*>(ctx->stream) : nullptr; }

int rsm_dev_alloc(rsm_ctx* ctx, uint64_t bytes, void** out) {
    if (!ctx || !out) return fail(RSM_EINVAL, "rsm_dev_alloc: bad arguments");
    if (int rc = use_device(ctx)) return rc;
    hipError_t e = hipMalloc(out, bytes ? bytes : 1);
    return e == hipSuccess ? RSM_OK : hip_fail(e, "hipMalloc");
}

int rsm_dev_free(rsm_ctx* ctx, void* p) {
    if (!ctx) return fail(RSM_EINVAL, "rsm_dev_free: NULL ctx");
    if (!p) return RSM_OK;
    if (int rc = use_device(ctx)) return rc;
    hipError_t e = hipFree(p);
    return e == hipSuccess ? RSM_OK : hip_fail(e, "hipFree");
}

int rsm_memcpy(rsm_ctx* ctx, void* dst, const void* src, uint64_t bytes, int kind) {
    if (!ctx || !dst || !src || kind < 0 || kind > 2) return fail(RSM_EINVAL, "rsm_memcpy: bad arguments");
    const hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : kind == 1 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
    if (int rc = use_device(ctx)) return rc;
    hipError_t e;
    if ((e = hipMemcpyAsync(dst, src, bytes, k, ctx->stream)) != hipSuccess) return hip_fail(e, "hipMemcpyAsync");
    if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    return RSM_OK;
}

int rsm_dev_fill_random(rsm_ctx* ctx, void* d, uint64_t bytes, uint64_t seed) {
    if (!ctx || !d) return fail(RSM_EINVAL, "rsm_dev_fill_random: bad arguments");
    if (int rc = use_device(ctx)) return rc;
    hipError_t e = launch_fill_random(d, bytes, seed, ctx->stream);
    return e == hipSuccess ? RSM_OK : hip_fail(e, "fill_random");
}

int rsm_stream_create(rsm_ctx* ctx, void** out) {
    if (!ctx || !out) return fail(RSM_EINVAL, "rsm_stream_create: bad arguments");
    *out = nullptr;
    if (int rc = use_device(ctx)) return rc;
    hipStream_t st = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    if (e != hipSuccess) return hip_fail(e, "hipStreamCreate");
    *out = static_cast<void*>(st);
    return RSM_OK;
}

int rsm_stream_destroy(rsm_ctx* ctx, void* stream) {
    if (!ctx || !stream) return fail(RSM_EINVAL, "rsm_stream_destroy: bad arguments");
    if (int rc = use_device(ctx)) return rc;
    hipStream_t st = static_cast<hipStream_t>(stream);
    (void)hipStreamSynchronize(st);
    // the stream's stuck-wait report is read before its scratch (which holds the
    // report word) is released, so a failed launch is never lost
    const int rep = check_queue_reports(ctx, st);
    {
        std::lock_guard<std::mutex> lk(ctx->scratch_mu);
        ctx->scratch.erase(st);  // its scratch dies with it
    }
    hipError_t e = hipStreamDestroy(st);
    if (rep != RSM_OK) return rep;
    return e == hipSuccess ? RSM_OK : hip_fail(e, "hipStreamDestroy");
}

// Device-side equality of two device buffers (a compare kernel on `stream`, then
// one word back): checks of large device-resident results without downloading them.
int rsm_dev_equal(rsm_ctx* ctx, const void* a, const void* b, uint64_t bytes, void* stream, int* equal) {
    if (!ctx || !a || !b || !equal || bytes % 16 != 0 || (((uintptr_t)a | (uintptr_t)b) & 15u) != 0)
        return fail(RSM_EINVAL, "rsm_dev_equal: bad arguments (bytes and both pointers must be 16-byte multiples)");
    *equal = 0;
    if (int rc = use_device(ctx)) return rc;
    LaneGuard g(ctx);
    if (!g.lane) return g.rc;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    hipError_t e;
    uint32_t word = 1;
    if ((e = g.lane->aux.ensure(64)) != hipSuccess ||
        (e = hipMemsetAsync(g.lane->aux.ptr, 0, 4, st)) != hipSuccess ||
        (e = launch_compare(static_cast<const uint8_t*>(a), static_cast<const uint8_t*>(b), bytes,
                            static_cast<uint32_t*>(g.lane->aux.ptr), st)) != hipSuccess ||
        (e = hipMemcpyAsync(&word, g.lane->aux.ptr, 4, hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipStreamSynchronize(st)) != hipSuccess)
        return hip_fail(e, "rsm_dev_equal");
    *equal = word == 0;
    return RSM_OK;
}

int rsm_stream_check(rsm_ctx* ctx, void* stream) {
    if (!ctx) return fail(RSM_EINVAL, "rsm_stream_check: NULL ctx");
    if (int rc = use_device(ctx)) return rc;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    return check_queue_reports(ctx, st);
}

int rsm_stream_sync(void* stream) {
    if (!stream) return fail(RSM_EINVAL, "rsm_stream_sync: NULL stream");
    hipError_t e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
    return e == hipSuccess ? RSM_OK : hip_fail(e, "hipStreamSynchronize");
}

int rsm_sync(rsm_ctx* ctx) {
    if (!ctx) return fail(RSM_EINVAL, "rsm_sync: NULL ctx");
    if (int rc = use_device(ctx)) return rc;
    hipError_t e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    // only the stream this call has drained: a report word of another stream may
    // belong to a launch still running there (rsm_stream_check reports those)
    return check_queue_reports(ctx, ctx->stream);
}

// Events: in-loop timing of the production launches (bench.py records one per
// phase boundary of every timed step).
int rsm_event_create(rsm_ctx* ctx, void** out) {
    if (!ctx || !out) return fail(RSM_EINVAL, "rsm_event_create: bad arguments");
    if (int rc = use_device(ctx)) return rc;
    hipEvent_t ev = nullptr;
    hipError_t e = hipEventCreate(&ev);
    if (e != hipSuccess) return hip_fail(e, "hipEventCreate");
    *out = static_cast<void*>(ev);
    return RSM_OK;
}

int rsm_event_destroy(void* ev) {
    if (!ev) return RSM_OK;
    hipError_t e = hipEventDestroy(static_cast<hipEvent_t>(ev));
    return e == hipSuccess ? RSM_OK : hip_fail(e, "hipEventDestroy");
}

int rsm_event_record(rsm_ctx* ctx, void* ev, void* stream) {
    if (!ctx || !ev) return fail(RSM_EINVAL, "rsm_event_record: bad arguments");
    hipError_t e = hipEventRecord(static_cast<hipEvent_t>(ev), pick(ctx, stream));
    return e == hipSuccess ? RSM_OK : hip_fail(e, "hipEventRecord");
}

int rsm_event_elapsed_ms(void* start, void* end, float* ms) {
    if (!start || !end || !ms) return fail(RSM_EINVAL, "rsm_event_elapsed_ms: bad arguments");
    hipError_t e = hipEventSynchronize(static_cast<hipEvent_t>(end));
    if (e == hipSuccess) e = hipEventElapsedTime(ms, static_cast<hipEvent_t>(start), static_cast<hipEvent_t>(end));
    return e == hipSuccess ? RSM_OK : hip_fail(e, "hipEventElapsedTime");
}

int rsm_time_extend(rsm_ctx* ctx, void* d_eds, uint32_t k, uint32_t share_size, uint32_t count, uint32_t reps,
                    float* row_ms, float* col_ms, float* step_ms) {
    if (!ctx || !d_eds || reps == 0) return fail(RSM_EINVAL, "rsm_time_extend: bad arguments");
    if (int rc = use_device(ctx)) return rc;
    hipEvent_t ev[3];
    for (auto& x : ev)
        if (hipEventCreate(&x) != hipSuccess) return fail(RSM_EDEVICE, "hipEventCreate");
    float acc[3] = {0, 0, 0};
    int rc = RSM_OK;
    for (uint32_t r = 0; r < reps && rc == RSM_OK; ++r) {
        (void)hipEventRecord(ev[0], ctx->stream);
        rc = extend_squares(ctx, static_cast<uint8_t*>(d_eds), k, share_size, count, ctx->stream, 1);
        (void)hipEventRecord(ev[1], ctx->stream);
        if (rc == RSM_OK) rc = extend_squares(ctx, static_cast<uint8_t*>(d_eds), k, share_size, count, ctx->stream, 2);
        (void)hipEventRecord(ev[2], ctx->stream);
        if (hipEventSynchronize(ev[2]) != hipSuccess) rc = fail(RSM_EDEVICE, "hipEventSynchronize");
        float a = 0, b = 0;
        (void)hipEventElapsedTime(&a, ev[0], ev[1]);
        (void)hipEventElapsedTime(&b, ev[1], ev[2]);
        acc[0] += a;
        acc[1] += b;
        acc[2] += a + b;
    }
    for (auto& x : ev) (void)hipEventDestroy(x);
    if (rc) return rc;
    if (row_ms) *row_ms = acc[0] / reps;
    if (col_ms) *col_ms = acc[1] / reps;
    if (step_ms) *step_ms = acc[2] / reps;
    return RSM_OK;
}

}  // extern "C"
