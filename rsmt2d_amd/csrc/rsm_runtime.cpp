// rsm_runtime.cpp -- context, device memory and the Codec half of the C ABI.
//
// The HIP kernels are the only compute path: every entry point that needs
// arithmetic fails with RSM_EDEVICE when no GPU/HIP runtime is usable; there is
// no CPU fallback anywhere in the product.
#include <atomic>
#include "rsm_internal.hpp"

#include <cstdio>
#include <cstring>
#include <cstdarg>

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

// ---------------------------------------------------------------------------
// Launch helpers (device-resident, asynchronous on `st`)
// ---------------------------------------------------------------------------
// GF(2^16) kernels support m = ceilPow2(k) in {256, 512} (2k <= 1024 shards:
// every configuration in BASELINE.json); larger k returns RSM_EUNSUPPORTED.
static bool gf16_supported(uint32_t k) { return k > 128 && k <= 512; }

int ensure_gf16(rsm_ctx* ctx, uint64_t scratch_bytes, uint64_t errs_bytes) {
    std::lock_guard<std::mutex> lk(ctx->gf16_mu);
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    if (!ctx->gf16_ready) {
        const Gf16Host& t = gf16_host();
        DevBuf& perm = ctx->dev_buf(20);
        DevBuf& skew = ctx->dev_buf(21);
        DevBuf& lw = ctx->dev_buf(22);
        const size_t pb = t.perm.size() * sizeof(PermTab16), sb = t.skew.size() * 2, lb = t.logwalsh.size() * 2;
        if ((e = perm.ensure(pb)) != hipSuccess || (e = skew.ensure(sb)) != hipSuccess || (e = lw.ensure(lb)) != hipSuccess)
            return hip_fail(e, "hipMalloc (GF16 tables)");
        if ((e = hipMemcpy(perm.ptr, t.perm.data(), pb, hipMemcpyHostToDevice)) != hipSuccess ||
            (e = hipMemcpy(skew.ptr, t.skew.data(), sb, hipMemcpyHostToDevice)) != hipSuccess ||
            (e = hipMemcpy(lw.ptr, t.logwalsh.data(), lb, hipMemcpyHostToDevice)) != hipSuccess)
            return hip_fail(e, "upload GF16 tables");
        ctx->gf16.perm = static_cast<const PermTab16*>(perm.ptr);
        ctx->gf16.skew = static_cast<const uint16_t*>(skew.ptr);
        ctx->gf16.logwalsh = static_cast<const uint16_t*>(lw.ptr);
        ctx->gf16_ready = true;
    }
    if (scratch_bytes > ctx->gf16.scratch_bytes) {
        // a kernel may still read the old scratch: drain the device before freeing it
        if ((e = hipDeviceSynchronize()) != hipSuccess) return hip_fail(e, "hipDeviceSynchronize");
        DevBuf& s = ctx->dev_buf(23);
        if ((e = s.ensure(scratch_bytes)) != hipSuccess) return hip_fail(e, "hipMalloc (GF16 scratch)");
        ctx->gf16.scratch = static_cast<uint8_t*>(s.ptr);
        ctx->gf16.scratch_bytes = scratch_bytes;
    }
    if (errs_bytes > ctx->gf16.errs_bytes) {
        if ((e = hipDeviceSynchronize()) != hipSuccess) return hip_fail(e, "hipDeviceSynchronize");
        DevBuf& s = ctx->dev_buf(24);
        if ((e = s.ensure(errs_bytes)) != hipSuccess) return hip_fail(e, "hipMalloc (GF16 error locators)");
        ctx->gf16.errs = static_cast<uint16_t*>(s.ptr);
        ctx->gf16.errs_bytes = errs_bytes;
    }
    return RSM_OK;
}

// Scratch budget for GF16 work arrays: all codewords of a launch when that fits
// in 1 GiB, else 1 GiB worth per batch (the launcher loops).
static uint64_t gf16_budget(uint64_t per_cw, uint64_t count) {
    const uint64_t cap = 1ull << 30;
    const uint64_t want = per_cw * count;
    return want < cap ? want : (cap / per_cw) * per_cw;
}

int launch_encode(rsm_ctx* ctx, const CodewordSet& cs0, hipStream_t st) {
    CodewordSet cs = cs0;
    if (cs.out_base == nullptr) cs.out_base = cs.base;
    hipError_t e;
    if (field_bits(cs.k) == 8) {
        cs.chunks = (cs.S + 255) / 256;
        e = launch_encode_gf8(cs, st);
    } else {
        if (!gf16_supported(cs.k)) return fail(RSM_EUNSUPPORTED, "encode: k=%u (m > 512) not supported in this build", cs.k);
        const uint64_t per_cw = (uint64_t)ceil_pow2(cs.k) * cs.S;
        if (int rc = ensure_gf16(ctx, gf16_budget(per_cw, cs.count), 0)) return rc;
        e = launch_encode_gf16(cs, ctx->gf16, st);
    }
    if (e != hipSuccess) return hip_fail(e, "encode kernel launch");
    return RSM_OK;
}

int launch_decode(rsm_ctx* ctx, const DecodeSet& ds0, hipStream_t st) {
    DecodeSet ds = ds0;
    hipError_t e;
    if (field_bits(ds.k) == 8) {
        ds.chunks = (ds.S + 255) / 256;
        e = launch_decode_gf8(ds, st);
    } else {
        if (!gf16_supported(ds.k)) return fail(RSM_EUNSUPPORTED, "decode: k=%u (m > 512) not supported in this build", ds.k);
        const uint64_t n = 2ull * ceil_pow2(ds.k);
        const uint64_t per_cw = 2ull * n * ds.S;
        const uint64_t budget = gf16_budget(per_cw, ds.count);
        if (int rc = ensure_gf16(ctx, budget, (budget / per_cw) * n * sizeof(uint16_t))) return rc;
        e = launch_decode_gf16(ds, ctx->gf16, st);
    }
    if (e != hipSuccess) return hip_fail(e, "decode kernel launch");
    return RSM_OK;
}

// The fused launch is opt-in (RSM_FUSED=1 or rsm_set_fused): measured no faster
// than the two launches; RSM_FUSED_LAG sets FusedPlan::lag.
std::atomic<int> g_fused{-1};
bool fused_enabled() {
    int v = g_fused.load(std::memory_order_relaxed);
    if (v < 0) {
        const char* e = getenv("RSM_FUSED");
        v = (e != nullptr && atoi(e) != 0) ? 1 : 0;
        g_fused.store(v, std::memory_order_relaxed);
    }
    return v != 0;
}

// Both passes in one launch (FusedPlan): the queue words live in a per-stream
// buffer that the kernel leaves zeroed; a new or grown buffer is zeroed in stream
// order before its first launch.
int extend_fused(rsm_ctx* ctx, const CodewordSet& rows, const CodewordSet& cols, uint32_t count, hipStream_t st) {
    static const uint32_t lag_env = [] {
        const char* v = getenv("RSM_FUSED_LAG");
        return v ? (uint32_t)atoi(v) : 4u;
    }();
    FusedPlan p{};
    p.rows = rows;
    p.cols = cols;
    p.count = count;
    p.lag = lag_env < 1 ? 1 : (lag_env > count ? count : lag_env);
    p.rn = (uint32_t)((uint64_t)rows.k * rows.S / 2048);
    p.cn = 2 * p.rn;
    p.total = count * (p.rn + p.cn);
    static const uint32_t flags_env = [] {
        const char* v = getenv("RSM_FUSED_FLAGS");
        return v ? (uint32_t)atoi(v) : 0u;
    }();
    p.flags = flags_env;
    if (getenv("RSM_FUSED_TRACE")) {
        DevBuf& tb = ctx->dev_buf(41);
        if (tb.ensure((size_t)p.total * 4) != hipSuccess) return fail(RSM_EDEVICE, "fused trace buffer");
        (void)hipMemsetAsync(tb.ptr, 0xFF, (size_t)p.total * 4, st);
        p.trace = static_cast<uint32_t*>(tb.ptr);
        ctx->fused_trace_n = p.total;
    }
    const size_t words = (size_t)count + 3;
    {
        std::lock_guard<std::mutex> g(ctx->fused_mu);
        auto& b = ctx->fused_ctr[(void*)st];
        if (!b) b = std::make_unique<DevBuf>();
        if (b->cap < words * 4) {
            hipError_t e = hipStreamSynchronize(st);  // an older, smaller buffer may still be in use
            if (e == hipSuccess) e = b->ensure(((words * 4 + 4095) / 4096) * 4096);
            if (e == hipSuccess) e = hipMemsetAsync(b->ptr, 0, b->cap, st);
            if (e != hipSuccess) return hip_fail(e, "fused extension: queue buffer");
        }
        p.ctr = static_cast<uint32_t*>(b->ptr);
    }
    hipError_t e = launch_extend_gf8_bs128_fused(p, st);
    if (e != hipSuccess) return hip_fail(e, "fused extension kernel launch");
    return RSM_OK;
}

// Two-phase in-place extension of `count` squares (extendeddatasquare.go:154-227):
//   phase 1: every row r < k: Q0 row -> Q1 row            (erasureExtendRow)
//   phase 2: every column c < 2k: [Q0|Q1] column -> [Q2|Q3] column
// Phase 2 computes Q2 exactly as erasureExtendCol and Q3 by column-encoding Q1,
// which equals the reference's row-encoding of Q2 by linearity of the 2D code
// (extendeddatasquare.go:204-207; asserted in tests against the oracle, which
// runs the reference order).
int extend_squares(rsm_ctx* ctx, uint8_t* d_eds, uint32_t k, uint32_t S, uint32_t count, hipStream_t st,
                   int phases) {
    const uint64_t W = 2ull * k;
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
    if (phases == 3 && fused_enabled() && field_bits(k) == 8) {
        CodewordSet cols = rows;
        cols.cw_stride = S;
        cols.elem_stride = W * S;
        cols.out_offset = (uint64_t)k * W * S;
        cols.per_square = (uint32_t)W;
        cols.count = (uint32_t)W * count;
        rows.out_base = rows.base;
        cols.out_base = cols.base;
        if (bs128_fused_applicable(rows, cols)) return extend_fused(ctx, rows, cols, count, st);
    }
    if (phases & 1) {
        int rc = launch_encode(ctx, rows, st);
        if (rc) return rc;
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
    return launch_encode(ctx, cols, st);
}

int device_roots(rsm_ctx* ctx, const uint8_t* d_eds, uint32_t W, uint32_t S, uint8_t* d_roots, hipStream_t st,
                 uint32_t squares) {
    if (!roots_dev_supported(W)) return fail(RSM_EUNSUPPORTED, "device roots: width %u not supported", W);
    if ((uint64_t)W * W * squares >= (1ull << 32) || squares > 65535)
        return fail(RSM_EINVAL, "device roots: %u squares of width %u exceed one launch", squares, W);
    DevBuf& leaf = ctx->dev_buf(30);
    hipError_t e = leaf.ensure((size_t)W * W * 32 * squares);
    if (e != hipSuccess) return hip_fail(e, "hipMalloc (leaf digests)");
    if ((e = launch_roots(d_eds, W, S, squares, static_cast<uint32_t*>(leaf.ptr), d_roots, st)) != hipSuccess)
        return hip_fail(e, "roots kernel launch");
    return RSM_OK;
}

}  // namespace rsm

using namespace rsm;

// ---------------------------------------------------------------------------
// C ABI: context
// ---------------------------------------------------------------------------
extern "C" {

const char* rsm_last_error(void) { return last_error(); }
const char* rsm_version(void) { return "rsmt2d-mi355x 0.1.0 (gfx950)"; }

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
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return hip_fail(e, "hipStreamCreate");
    }
    *out = c;
    return RSM_OK;
}

void rsm_ctx_destroy(rsm_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    ctx->bufs.clear();
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

// ---------------------------------------------------------------------------
// C ABI: Codec
// ---------------------------------------------------------------------------
const char* rsm_codec_name(void) { return "Leopard"; }
int64_t rsm_codec_max_chunks(void) { return (int64_t)32768 * 32768; }
int rsm_codec_validate_chunk_size(int64_t share_size) { return validate_chunk_size(share_size); }
int rsm_codec_field_bits(uint32_t k) { return field_bits(k); }

int rsm_encode(rsm_ctx* ctx, const uint8_t* const* data, uint32_t k, uint32_t share_size,
               uint8_t* const* parity) {
    if (!ctx || !data || !parity || k == 0) return fail(RSM_EINVAL, "rsm_encode: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (share_size == 0) return fail(RSM_ESHAPE, "rsm_encode: zero-length shares");
    if (2ull * k > 65536ull) return fail(RSM_ESHAPE, "rsm_encode: %u shards exceed the Leopard limit", 2 * k);
    for (uint32_t i = 0; i < k; ++i)
        if (!data[i]) return fail(RSM_EINVAL, "rsm_encode: data[%u] is nil", i);
    std::lock_guard<std::mutex> lk(ctx->mu);
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    const size_t S = share_size;
    const size_t bytes = 2ull * k * S;
    HostBuf& hb = ctx->host_buf(0);
    DevBuf& db = ctx->dev_buf(0);
    if ((e = hb.ensure(bytes)) != hipSuccess) return hip_fail(e, "hipHostMalloc");
    if ((e = db.ensure(bytes)) != hipSuccess) return hip_fail(e, "hipMalloc");
    uint8_t* h = static_cast<uint8_t*>(hb.ptr);
    for (uint32_t i = 0; i < k; ++i) memcpy(h + i * S, data[i], S);
    uint8_t* d = static_cast<uint8_t*>(db.ptr);
    if ((e = hipMemcpyAsync(d, h, k * S, hipMemcpyHostToDevice, ctx->stream)) != hipSuccess)
        return hip_fail(e, "hipMemcpyAsync H2D");
    CodewordSet cs{};
    cs.base = d;
    cs.square_stride = 0;
    cs.cw_stride = 0;
    cs.elem_stride = S;
    cs.out_offset = (uint64_t)k * S;
    cs.per_square = 1;
    cs.count = 1;
    cs.k = k;
    cs.S = share_size;
    if (int rc = launch_encode(ctx, cs, ctx->stream)) return rc;
    if ((e = hipMemcpyAsync(h + k * S, d + k * S, k * S, hipMemcpyDeviceToHost, ctx->stream)) != hipSuccess)
        return hip_fail(e, "hipMemcpyAsync D2H");
    if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess) return hip_fail(e, "encode");
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
    std::lock_guard<std::mutex> lk(ctx->mu);
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    const size_t S = share_size;
    const size_t bytes = (size_t)n * S;
    HostBuf& hb = ctx->host_buf(0);
    DevBuf& db = ctx->dev_buf(0);
    DevBuf& dp = ctx->dev_buf(1);
    if ((e = hb.ensure(bytes + n + 16)) != hipSuccess) return hip_fail(e, "hipHostMalloc");
    if ((e = db.ensure(bytes)) != hipSuccess) return hip_fail(e, "hipMalloc");
    if ((e = dp.ensure(n + 16)) != hipSuccess) return hip_fail(e, "hipMalloc");
    uint8_t* h = static_cast<uint8_t*>(hb.ptr);
    for (uint32_t i = 0; i < n; ++i) {
        if (present[i]) memcpy(h + i * S, shares[i], S);
        else memset(h + i * S, 0, S);
    }
    uint8_t* hp = h + bytes;
    for (uint32_t i = 0; i < n; ++i) hp[i] = present[i] ? 1 : 0;
    uint32_t* hidx = reinterpret_cast<uint32_t*>(hp + ((n + 3) & ~3u));
    (void)hidx;
    uint8_t* d = static_cast<uint8_t*>(db.ptr);
    uint8_t* dpres = static_cast<uint8_t*>(dp.ptr);
    if ((e = hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, ctx->stream)) != hipSuccess)
        return hip_fail(e, "hipMemcpyAsync H2D");
    if ((e = hipMemcpyAsync(dpres, hp, n, hipMemcpyHostToDevice, ctx->stream)) != hipSuccess)
        return hip_fail(e, "hipMemcpyAsync H2D");
    DecodeSet ds{};
    ds.base = d;
    ds.presence = dpres;
    ds.indices = ctx->zero_index();
    ds.count = 1;
    ds.axis = 0;  // a single codeword is row 0 of a 1 x 2k "square"
    ds.k = k;
    ds.S = share_size;
    if (!ds.indices) return fail(RSM_EDEVICE, "rsm_decode: index buffer allocation failed");
    if (int rc = launch_decode(ctx, ds, ctx->stream)) return rc;
    if ((e = hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, ctx->stream)) != hipSuccess)
        return hip_fail(e, "hipMemcpyAsync D2H");
    if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess) return hip_fail(e, "decode");
    for (uint32_t i = 0; i < n; ++i)
        if (!present[i]) memcpy(shares[i], h + i * S, S);
    return RSM_OK;
}

int rsm_extend_square(rsm_ctx* ctx, const uint8_t* ods, uint32_t k, uint32_t share_size, uint8_t* eds) {
    if (!ctx || !ods || !eds || k == 0) return fail(RSM_EINVAL, "rsm_extend_square: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    std::lock_guard<std::mutex> lk(ctx->mu);
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    const size_t S = share_size, W = 2ull * k;
    DevBuf& db = ctx->dev_buf(0);
    if ((e = db.ensure(W * W * S)) != hipSuccess) return hip_fail(e, "hipMalloc");
    uint8_t* d = static_cast<uint8_t*>(db.ptr);
    // Q0 straight into the top-left quadrant: the EDS aliases the ODS.
    if ((e = hipMemcpy2DAsync(d, W * S, ods, k * S, k * S, k, hipMemcpyHostToDevice, ctx->stream)) != hipSuccess)
        return hip_fail(e, "hipMemcpy2DAsync H2D");
    if (int rc = extend_squares(ctx, d, k, share_size, 1, ctx->stream)) return rc;
    if ((e = hipMemcpyAsync(eds, d, W * W * S, hipMemcpyDeviceToHost, ctx->stream)) != hipSuccess)
        return hip_fail(e, "hipMemcpyAsync D2H");
    if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess) return hip_fail(e, "extend");
    return RSM_OK;
}

int rsm_extend_squares_dev(rsm_ctx* ctx, void* d_eds, uint32_t k, uint32_t share_size, uint32_t count,
                           void* stream) {
    if (!ctx || !d_eds || k == 0) return fail(RSM_EINVAL, "rsm_extend_squares_dev: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (count == 0) return RSM_OK;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    return extend_squares(ctx, static_cast<uint8_t*>(d_eds), k, share_size, count, st);
}

int rsm_extend_squares_phase_dev(rsm_ctx* ctx, void* d_eds, uint32_t k, uint32_t share_size, uint32_t count,
                                 int phase, void* stream) {
    if (!ctx || !d_eds || k == 0 || phase < 1 || phase > 3)
        return fail(RSM_EINVAL, "rsm_extend_squares_phase_dev: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (count == 0) return RSM_OK;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    return extend_squares(ctx, static_cast<uint8_t*>(d_eds), k, share_size, count, st, phase);
}

// Row / column slices of ONE in-place [2k][2k][S] square -- the per-GPU units of the
// row-sharded multi-GPU schedule (erasureExtendRow / erasureExtendCol for a range).
int rsm_extend_rows_dev(rsm_ctx* ctx, void* d_eds, uint32_t k, uint32_t share_size, uint32_t row0, uint32_t nrows,
                        void* stream) {
    if (!ctx || !d_eds || k == 0 || row0 + nrows > 2 * k) return fail(RSM_EINVAL, "rsm_extend_rows_dev: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (nrows == 0) return RSM_OK;
    const uint64_t W = 2ull * k, S = share_size;
    CodewordSet cs{};
    cs.base = static_cast<uint8_t*>(d_eds) + row0 * W * S;
    cs.square_stride = 0;
    cs.cw_stride = W * S;
    cs.elem_stride = S;
    cs.out_offset = k * S;
    cs.per_square = nrows;
    cs.count = nrows;
    cs.k = k;
    cs.S = share_size;
    return launch_encode(ctx, cs, stream ? static_cast<hipStream_t>(stream) : ctx->stream);
}

int rsm_extend_cols_dev(rsm_ctx* ctx, void* d_eds, uint32_t k, uint32_t share_size, uint32_t col0, uint32_t ncols,
                        void* stream) {
    if (!ctx || !d_eds || k == 0 || col0 + ncols > 2 * k) return fail(RSM_EINVAL, "rsm_extend_cols_dev: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (ncols == 0) return RSM_OK;
    const uint64_t W = 2ull * k, S = share_size;
    CodewordSet cs{};
    cs.base = static_cast<uint8_t*>(d_eds) + col0 * S;
    cs.square_stride = 0;
    cs.cw_stride = S;
    cs.elem_stride = W * S;
    cs.out_offset = k * W * S;
    cs.per_square = ncols;
    cs.count = ncols;
    cs.k = k;
    cs.S = share_size;
    return launch_encode(ctx, cs, stream ? static_cast<hipStream_t>(stream) : ctx->stream);
}

int rsm_roots_dev(rsm_ctx* ctx, const void* d_eds, uint32_t width, uint32_t share_size, void* d_roots,
                  void* stream) {
    if (!ctx || !d_eds || !d_roots || width == 0) return fail(RSM_EINVAL, "rsm_roots_dev: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    std::lock_guard<std::mutex> lk(ctx->mu);
    return device_roots(ctx, static_cast<const uint8_t*>(d_eds), width, share_size, static_cast<uint8_t*>(d_roots),
                        stream ? static_cast<hipStream_t>(stream) : ctx->stream);
}

int rsm_roots_squares_dev(rsm_ctx* ctx, const void* d_eds, uint32_t width, uint32_t share_size, uint32_t count,
                          void* d_roots, void* stream) {
    if (!ctx || !d_eds || !d_roots || width == 0) return fail(RSM_EINVAL, "rsm_roots_squares_dev: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (count == 0) return RSM_OK;
    std::lock_guard<std::mutex> lk(ctx->mu);
    return device_roots(ctx, static_cast<const uint8_t*>(d_eds), width, share_size, static_cast<uint8_t*>(d_roots),
                        stream ? static_cast<hipStream_t>(stream) : ctx->stream, count);
}

int rsm_encode_batch_dev(rsm_ctx* ctx, const void* d_in, void* d_out, uint32_t k, uint32_t share_size,
                         uint32_t count, uint64_t cw_stride, uint64_t share_stride, void* stream) {
    if (!ctx || !d_in || !d_out || k == 0 || share_stride < share_size)
        return fail(RSM_EINVAL, "rsm_encode_batch_dev: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (count == 0) return RSM_OK;
    CodewordSet cs{};
    cs.base = static_cast<uint8_t*>(const_cast<void*>(d_in));
    cs.out_base = static_cast<uint8_t*>(d_out);
    cs.square_stride = 0;
    cs.cw_stride = cw_stride;
    cs.elem_stride = share_stride;
    cs.out_offset = 0;
    cs.per_square = count;
    cs.count = count;
    cs.k = k;
    cs.S = share_size;
    return launch_encode(ctx, cs, stream ? static_cast<hipStream_t>(stream) : ctx->stream);
}

int rsm_decode_vectors_dev(rsm_ctx* ctx, void* d_eds, const uint8_t* d_presence, uint32_t k,
                           uint32_t share_size, int axis, const uint32_t* d_indices, uint32_t count,
                           void* stream) {
    if (!ctx || !d_eds || !d_presence || !d_indices || k == 0 || (axis != 0 && axis != 1))
        return fail(RSM_EINVAL, "rsm_decode_vectors_dev: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (count == 0) return RSM_OK;
    DecodeSet ds{};
    ds.base = static_cast<uint8_t*>(d_eds);
    ds.presence = d_presence;
    ds.indices = d_indices;
    ds.count = count;
    ds.axis = (uint32_t)axis;
    ds.k = k;
    ds.S = share_size;
    return launch_decode(ctx, ds, stream ? static_cast<hipStream_t>(stream) : ctx->stream);
}

}  // extern "C"

// ---------------------------------------------------------------------------
// C ABI: device memory, synthetic inputs and event timing on the context's own
// HIP runtime/stream.  (A host process embedding a second HIP runtime -- e.g.
// PyTorch's bundled one -- must not hand its stream objects to this library;
// device pointers are shared fine.)
// ---------------------------------------------------------------------------
extern "C" {

void* rsm_ctx_stream(rsm_ctx* ctx) { return ctx ? static_cast<void*>(ctx->stream) : nullptr; }

int rsm_dev_alloc(rsm_ctx* ctx, uint64_t bytes, void** out) {
    if (!ctx || !out) return fail(RSM_EINVAL, "rsm_dev_alloc: bad arguments");
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    if ((e = hipMalloc(out, bytes ? bytes : 1)) != hipSuccess) return hip_fail(e, "hipMalloc");
    return RSM_OK;
}

int rsm_dev_free(rsm_ctx* ctx, void* p) {
    if (!ctx) return fail(RSM_EINVAL, "rsm_dev_free: NULL ctx");
    if (!p) return RSM_OK;
    (void)hipSetDevice(ctx->device);
    hipError_t e = hipFree(p);
    return e == hipSuccess ? RSM_OK : hip_fail(e, "hipFree");
}

int rsm_memcpy(rsm_ctx* ctx, void* dst, const void* src, uint64_t bytes, int kind) {
    if (!ctx || !dst || !src || kind < 0 || kind > 2) return fail(RSM_EINVAL, "rsm_memcpy: bad arguments");
    const hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : kind == 1 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    if ((e = hipMemcpyAsync(dst, src, bytes, k, ctx->stream)) != hipSuccess) return hip_fail(e, "hipMemcpyAsync");
    if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    return RSM_OK;
}

int rsm_dev_fill_random(rsm_ctx* ctx, void* d, uint64_t bytes, uint64_t seed) {
    if (!ctx || !d) return fail(RSM_EINVAL, "rsm_dev_fill_random: bad arguments");
    hipError_t e = launch_fill_random(d, bytes, seed, ctx->stream);
    return e == hipSuccess ? RSM_OK : hip_fail(e, "fill_random");
}

int rsm_stream_create(rsm_ctx* ctx, void** out) {
    if (!ctx || !out) return fail(RSM_EINVAL, "rsm_stream_create: bad arguments");
    *out = nullptr;
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    hipStream_t st = nullptr;
    if ((e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking)) != hipSuccess) return hip_fail(e, "hipStreamCreate");
    *out = static_cast<void*>(st);
    return RSM_OK;
}

int rsm_stream_destroy(rsm_ctx* ctx, void* stream) {
    if (!ctx || !stream) return fail(RSM_EINVAL, "rsm_stream_destroy: bad arguments");
    hipError_t e = hipStreamDestroy(static_cast<hipStream_t>(stream));
    return e == hipSuccess ? RSM_OK : hip_fail(e, "hipStreamDestroy");
}

int rsm_stream_sync(void* stream) {
    if (!stream) return fail(RSM_EINVAL, "rsm_stream_sync: NULL stream");
    hipError_t e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
    return e == hipSuccess ? RSM_OK : hip_fail(e, "hipStreamSynchronize");
}

int rsm_sync(rsm_ctx* ctx) {
    if (!ctx) return fail(RSM_EINVAL, "rsm_sync: NULL ctx");
    hipError_t e = hipStreamSynchronize(ctx->stream);
    return e == hipSuccess ? RSM_OK : hip_fail(e, "hipStreamSynchronize");
}

int rsm_fused_trace(rsm_ctx* ctx, uint32_t* out, uint32_t n, uint32_t* err) {
    if (!ctx || !out) return fail(RSM_EINVAL, "rsm_fused_trace: bad arguments");
    if (hipStreamSynchronize(ctx->stream) != hipSuccess) return fail(RSM_EDEVICE, "hipStreamSynchronize");
    const uint32_t m = n < ctx->fused_trace_n ? n : ctx->fused_trace_n;
    if (m && hipMemcpy(out, ctx->dev_buf(41).ptr, (size_t)m * 4, hipMemcpyDeviceToHost) != hipSuccess)
        return fail(RSM_EDEVICE, "rsm_fused_trace: copy");
    if (err) {
        *err = 0;
        auto it = ctx->fused_ctr.find((void*)ctx->stream);
        if (it != ctx->fused_ctr.end() && it->second->ptr &&
            hipMemcpy(err, static_cast<uint32_t*>(it->second->ptr) + 2, 4, hipMemcpyDeviceToHost) != hipSuccess)
            return fail(RSM_EDEVICE, "rsm_fused_trace: error flag");
    }
    return (int)m;
}

int rsm_extend_pipeline_dev(rsm_ctx* ctx, void* d_rows_eds, void* d_cols_eds, uint32_t k, uint32_t share_size,
                            uint32_t count, void* stream) {
    if (!ctx || k == 0 || (!d_rows_eds && !d_cols_eds)) return fail(RSM_EINVAL, "rsm_extend_pipeline_dev: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (count == 0) return RSM_OK;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    const uint64_t W = 2ull * k, S = share_size;
    CodewordSet rows{}, cols{};
    rows.base = rows.out_base = static_cast<uint8_t*>(d_rows_eds);
    rows.square_stride = W * W * S;
    rows.cw_stride = W * S;
    rows.elem_stride = S;
    rows.out_offset = (uint64_t)k * S;
    rows.per_square = k;
    rows.count = k * count;
    rows.k = k;
    rows.S = share_size;
    cols = rows;
    cols.base = cols.out_base = static_cast<uint8_t*>(d_cols_eds);
    cols.cw_stride = S;
    cols.elem_stride = W * S;
    cols.out_offset = (uint64_t)k * W * S;
    cols.per_square = (uint32_t)W;
    cols.count = (uint32_t)W * count;
    const bool dual = field_bits(k) == 8 && d_rows_eds && d_cols_eds && bs128_applicable(rows) && bs128_applicable(cols);
    if (!dual) {  // separate launches (independent batches: order does not matter)
        if (d_rows_eds)
            if (int rc = extend_squares(ctx, static_cast<uint8_t*>(d_rows_eds), k, share_size, count, st, 1)) return rc;
        if (d_cols_eds)
            if (int rc = extend_squares(ctx, static_cast<uint8_t*>(d_cols_eds), k, share_size, count, st, 2)) return rc;
        return RSM_OK;
    }
    DualPlan p{};
    p.a = rows;
    p.b = cols;
    p.na = (uint32_t)(((uint64_t)rows.count * S + 2047) / 2048);
    p.nb = (uint32_t)(((uint64_t)cols.count * S + 2047) / 2048);
    hipError_t e = launch_encode_gf8_bs128_dual(p, st);
    if (e != hipSuccess) return hip_fail(e, "pipelined extension kernel launch");
    return RSM_OK;
}

int rsm_time_pipeline(rsm_ctx* ctx, void* d_rows_eds, void* d_cols_eds, uint32_t k, uint32_t share_size,
                      uint32_t count, uint32_t reps, float* ms) {
    if (!ctx || !ms || reps == 0) return fail(RSM_EINVAL, "rsm_time_pipeline: bad arguments");
    hipEvent_t ev[2];
    for (auto& x : ev)
        if (hipEventCreate(&x) != hipSuccess) return fail(RSM_EDEVICE, "hipEventCreate");
    int rc = RSM_OK;
    (void)hipEventRecord(ev[0], ctx->stream);
    for (uint32_t r = 0; r < reps && rc == RSM_OK; ++r)
        rc = rsm_extend_pipeline_dev(ctx, d_rows_eds, d_cols_eds, k, share_size, count, nullptr);
    (void)hipEventRecord(ev[1], ctx->stream);
    if (hipEventSynchronize(ev[1]) != hipSuccess && rc == RSM_OK) rc = fail(RSM_EDEVICE, "hipEventSynchronize");
    float t = 0;
    (void)hipEventElapsedTime(&t, ev[0], ev[1]);
    for (auto& x : ev) (void)hipEventDestroy(x);
    if (rc) return rc;
    *ms = t / reps;
    return RSM_OK;
}

int rsm_set_pass_grid(int pass, int cus) {
    if (pass != 0 && pass != 1) return fail(RSM_EINVAL, "rsm_set_pass_grid: pass must be 0 (rows) or 1 (columns)");
    return set_pass_grid_cap(pass, cus);
}

int rsm_set_fused(int on) {
    const int prev = fused_enabled() ? 1 : 0;
    g_fused.store(on ? 1 : 0, std::memory_order_relaxed);
    return prev;
}

int rsm_extend_fused(uint32_t k, uint32_t share_size) {
    if (!fused_enabled() || k != 128 || validate_chunk_size(share_size) != RSM_OK) return 0;
    return ((uint64_t)k * share_size) % 2048 == 0 ? 1 : 0;
}

int rsm_time_extend(rsm_ctx* ctx, void* d_eds, uint32_t k, uint32_t share_size, uint32_t count, uint32_t reps,
                    float* row_ms, float* col_ms, float* step_ms) {
    if (!ctx || !d_eds || reps == 0) return fail(RSM_EINVAL, "rsm_time_extend: bad arguments");
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
        float a = 0, b = 0, c = 0;
        (void)hipEventElapsedTime(&a, ev[0], ev[1]);
        (void)hipEventElapsedTime(&b, ev[1], ev[2]);
        // step: the production form (one fused launch where it applies)
        if (rc == RSM_OK) {
            (void)hipEventRecord(ev[0], ctx->stream);
            rc = extend_squares(ctx, static_cast<uint8_t*>(d_eds), k, share_size, count, ctx->stream, 3);
            (void)hipEventRecord(ev[1], ctx->stream);
            if (hipEventSynchronize(ev[1]) != hipSuccess) rc = fail(RSM_EDEVICE, "hipEventSynchronize");
            (void)hipEventElapsedTime(&c, ev[0], ev[1]);
        }
        acc[0] += a;
        acc[1] += b;
        acc[2] += c;
    }
    for (auto& x : ev) (void)hipEventDestroy(x);
    if (rc) return rc;
    if (row_ms) *row_ms = acc[0] / reps;
    if (col_ms) *col_ms = acc[1] / reps;
    if (step_ms) *step_ms = acc[2] / reps;
    return RSM_OK;
}

}  // extern "C"
