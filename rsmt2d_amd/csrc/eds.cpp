// eds.cpp -- host half of the ExtendedDataSquare API and the crossword Repair.
//
// Mirrors extendeddatasquare.go / datasquare.go / extendeddatacrossword.go of
// celestiaorg/rsmt2d with the same names, argument meaning and error
// behaviour.  All Reed-Solomon arithmetic goes to the HIP kernels:
//   * ComputeExtendedDataSquare -> one H2D of the ODS into the EDS quadrant, the
//     two-phase device extension, one D2H;
//   * Repair -> a device fast path (batched row/column decode sweeps over a
//     device-resident square + full re-encode check + host roots) whose result is
//     provably what the reference returns on success (DESIGN.md "Repair"); any
//     failure of that path (unrepairable, byzantine) falls back to the exact
//     sequential reference order (solveCrossword, :87-282) using the
//     per-codeword device codec, so error identity matches the reference.
#include "rsm_internal.hpp"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

using namespace rsm;

// Host bytes of a square: pinned (hipHostMalloc) whenever a HIP runtime is
// usable, so Repair's square upload and download are direct DMA; plain memory on
// a host without a GPU (Import/New are host-only operations).
struct HostSquare {
    uint8_t* p = nullptr;
    size_t n = 0;
    bool pinned = false;
    HostSquare() = default;
    HostSquare(const HostSquare&) = delete;
    HostSquare& operator=(const HostSquare&) = delete;
    ~HostSquare() { release(); }
    void release() {
        if (p) {
            if (pinned) (void)hipHostFree(p);
            else free(p);
        }
        p = nullptr;
        n = 0;
    }
    bool assign(size_t bytes) {  // zero-filled
        release();
        if (bytes == 0) return true;
        void* q = nullptr;
        if (hipHostMalloc(&q, bytes, hipHostMallocDefault) == hipSuccess) {
            pinned = true;
        } else {
            (void)hipGetLastError();
            q = malloc(bytes);
            pinned = false;
            if (!q) return false;
        }
        p = static_cast<uint8_t*>(q);
        n = bytes;
        memset(p, 0, n);
        return true;
    }
    uint8_t* data() { return p; }
    const uint8_t* data() const { return p; }
    size_t size() const { return n; }
    void swap(HostSquare& o) {
        std::swap(p, o.p);
        std::swap(n, o.n);
        std::swap(pinned, o.pinned);
    }
};

struct rsm_eds {
    rsm_ctx* ctx = nullptr;
    uint32_t width = 0;
    uint32_t odw = 0;  // originalDataWidth
    uint32_t S = 0;    // shareSize
    HostSquare data;               // width*width*S, row-major
    std::vector<uint8_t> present;  // width*width
    std::vector<uint8_t> byz_data;
    std::vector<uint8_t> byz_present;
    rsm_repair_stats stats{};

    uint8_t* cell(uint32_t r, uint32_t c) { return data.data() + ((size_t)r * width + c) * S; }
    const uint8_t* cell(uint32_t r, uint32_t c) const { return data.data() + ((size_t)r * width + c) * S; }
    bool has(uint32_t r, uint32_t c) const { return present[(size_t)r * width + c] != 0; }
    // (axis, index, position) -> cell coordinates
    uint32_t rr(int axis, uint32_t idx, uint32_t pos) const { return axis == RSM_AXIS_ROW ? idx : pos; }
    uint32_t cc(int axis, uint32_t idx, uint32_t pos) const { return axis == RSM_AXIS_ROW ? pos : idx; }
};

// Repair A/B (diagnostic builds): 1 = the zero-copy sweep as two launches, top half then
// bottom half, the column re-encode of the top half overlapping the bottom sweep (the
// form up to r05am); production: one launch, the re-encode behind all of it
#ifdef RSM_DIAG
static std::atomic<uint32_t> g_repair_mode{0};
namespace rsm {
void set_repair_diag_mode(uint32_t m) { g_repair_mode.store(m); }
}  // namespace rsm
static uint32_t repair_mode() { return g_repair_mode.load(); }
#else
static uint32_t repair_mode() { return 0; }
#endif

namespace {

uint32_t get_width(uint64_t n) {  // datasquare.go:35-37
    return (uint32_t)std::ceil(std::sqrt((double)n));
}

// newDataSquare shape checks (datasquare.go:42-64) + getShareSize
// (extendeddatasquare.go:374-381).  Returns width / share size.
int check_square(const uint8_t* const* data, const uint32_t* lens, uint64_t n, uint32_t* width,
                 uint32_t* share_size) {
    uint32_t S = 0;
    for (uint64_t i = 0; i < n; ++i)
        if (data[i]) {
            S = lens[i];
            break;
        }
    if (int rc = validate_chunk_size(S)) return rc;
    uint32_t w = get_width(n);
    if ((uint64_t)w * w != n) return fail(RSM_ESHAPE, "number of chunks must be a square number");
    for (uint64_t i = 0; i < n; ++i)
        if (data[i] && lens[i] != S) return fail(RSM_ESHAPE, "non-nil shares not all of equal size");
    *width = w;
    *share_size = S;
    return RSM_OK;
}

rsm_eds* alloc_eds(rsm_ctx* ctx, uint32_t width, uint32_t S) {
    auto* e = new (std::nothrow) rsm_eds();
    if (!e) return nullptr;
    e->ctx = ctx;
    e->width = width;
    e->S = S;
    try {
        e->present.assign((size_t)width * width, 0);
    } catch (...) {
        delete e;
        return nullptr;
    }
    if (!e->data.assign((size_t)width * width * S)) {
        delete e;
        return nullptr;
    }
    return e;
}

// ---------------------------------------------------------------------------
// Tree plumbing
// ---------------------------------------------------------------------------
struct Tree {
    rsm_tree_root_fn fn;
    void* user;
    bool is_default() const { return fn == nullptr || fn == rsm_default_tree_root; }
    // the library's own trees are pure functions: safe to call from many threads
    bool pure() const { return is_default() || fn == rsm_nmt_tree_root; }
    // Returns 0 and the root, or non-zero on a tree error.
    int root(int axis, uint32_t index, const std::vector<const uint8_t*>& leaves, uint32_t S,
             std::vector<uint8_t>& out) const {
        uint8_t buf[256];
        uint32_t len = sizeof(buf);
        rsm_tree_root_fn f = fn ? fn : rsm_default_tree_root;
        int rc = f(user, axis, index, leaves.data(), (uint32_t)leaves.size(), S, buf, &len);
        if (rc != 0 || len > sizeof(buf)) return rc ? rc : RSM_ETREE;
        out.assign(buf, buf + len);
        return 0;
    }
};

// Computes roots of many vectors; parallel over host threads for the library's
// own (pure, thread-safe) trees, sequential for caller-provided trees.
// jobs: (axis, index, leaves).  ok[i] = root computed; roots[i] = root bytes.
void roots_many(const Tree& tree, const std::vector<int>& axes, const std::vector<uint32_t>& idxs,
                const std::vector<std::vector<const uint8_t*>>& leaves, uint32_t S,
                std::vector<std::vector<uint8_t>>& roots, std::vector<int>& rcs) {
    const size_t n = axes.size();
    roots.assign(n, {});
    rcs.assign(n, 0);
    unsigned nt = tree.pure() ? std::max(1u, std::min(64u, std::thread::hardware_concurrency())) : 1u;
    if (n < 8) nt = 1;
    if (nt == 1) {
        for (size_t i = 0; i < n; ++i) rcs[i] = tree.root(axes[i], idxs[i], leaves[i], S, roots[i]);
        return;
    }
    std::atomic<size_t> next{0};
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&] {
            for (size_t i; (i = next.fetch_add(1)) < n;) rcs[i] = tree.root(axes[i], idxs[i], leaves[i], S, roots[i]);
        });
    for (auto& x : th) x.join();
}

std::vector<const uint8_t*> vector_leaves(const rsm_eds* e, int axis, uint32_t idx) {
    std::vector<const uint8_t*> v(e->width);
    for (uint32_t p = 0; p < e->width; ++p) {
        uint32_t r = e->rr(axis, idx, p), c = e->cc(axis, idx, p);
        v[p] = e->has(r, c) ? e->cell(r, c) : nullptr;
    }
    return v;
}

bool vector_complete(const rsm_eds* e, int axis, uint32_t idx, int skip = -1) {  // noMissingData
    for (uint32_t p = 0; p < e->width; ++p) {
        if ((int)p == skip) continue;
        if (!e->has(e->rr(axis, idx, p), e->cc(axis, idx, p))) return false;
    }
    return true;
}

uint32_t vector_present(const rsm_eds* e, int axis, uint32_t idx) {
    uint32_t n = 0;
    for (uint32_t p = 0; p < e->width; ++p) n += e->has(e->rr(axis, idx, p), e->cc(axis, idx, p)) ? 1 : 0;
    return n;
}

void snapshot_byzantine(rsm_eds* e, int axis, uint32_t idx, int drop_pos = -1) {
    e->byz_data.assign((size_t)e->width * e->S, 0);
    e->byz_present.assign(e->width, 0);
    for (uint32_t p = 0; p < e->width; ++p) {
        uint32_t r = e->rr(axis, idx, p), c = e->cc(axis, idx, p);
        if (e->has(r, c) && (int)p != drop_pos) {
            memcpy(e->byz_data.data() + (size_t)p * e->S, e->cell(r, c), e->S);
            e->byz_present[p] = 1;
        }
    }
}

// ---------------------------------------------------------------------------
// Device square for Repair
// ---------------------------------------------------------------------------
struct DevSquare {
    rsm_ctx* ctx;
    uint32_t k, W, S;
    uint8_t* d_eds = nullptr;
    uint8_t* d_scratch = nullptr;
    uint8_t* d_pres = nullptr;
    uint32_t* d_idx = nullptr;
    uint32_t* d_flags = nullptr;
    hipStream_t st;

    // caller holds c->eds_mu (the buffers and the context stream are the EDS layer's)
    int init(rsm_ctx* c, uint32_t width, uint32_t share_size) {
        ctx = c;
        W = width;
        k = width / 2;
        S = share_size;
        st = c->stream;
        if (int rc = use_device(c)) return rc;
        hipError_t e;
        const size_t sq = (size_t)W * W * S;
        DevBuf& a = c->eds.eds;
        DevBuf& b = c->eds.scratch;
        DevBuf& p = c->eds.pres;
        DevBuf& ix = c->eds.idx;
        DevBuf& fl = c->eds.flags;
        if ((e = a.ensure(sq)) != hipSuccess || (e = b.ensure(sq)) != hipSuccess ||
            // presence map, then (zero-copy fast path) its row list: one staged copy
            (e = p.ensure((size_t)W * W + sizeof(uint32_t) * (2 * W + 16) + 64)) != hipSuccess ||
            (e = ix.ensure(sizeof(uint32_t) * (2 * W + 16))) != hipSuccess ||
            (e = fl.ensure(sizeof(uint32_t) * (2 * W + 16))) != hipSuccess)
            return hip_fail(e, "hipMalloc (repair square)");
        d_eds = static_cast<uint8_t*>(a.ptr);
        d_scratch = static_cast<uint8_t*>(b.ptr);
        d_pres = static_cast<uint8_t*>(p.ptr);
        d_idx = static_cast<uint32_t*>(ix.ptr);
        d_flags = static_cast<uint32_t*>(fl.ptr);
        return RSM_OK;
    }
    int upload(const rsm_eds* e) {
        hipError_t r;
        if ((r = hipMemcpyAsync(d_eds, e->data.data(), e->data.size(), hipMemcpyHostToDevice, st)) != hipSuccess)
            return hip_fail(r, "H2D square");
        return upload_presence(e->present);
    }
    int upload_presence(const std::vector<uint8_t>& pres) {
        hipError_t r = hipMemcpyAsync(d_pres, pres.data(), pres.size(), hipMemcpyHostToDevice, st);
        return r == hipSuccess ? RSM_OK : hip_fail(r, "H2D presence");
    }
    int sync() {
        hipError_t r = hipStreamSynchronize(st);
        return r == hipSuccess ? RSM_OK : hip_fail(r, "repair stream");
    }
    int decode(int axis, const std::vector<uint32_t>& idx) {
        if (idx.empty()) return RSM_OK;
        hipError_t r = hipMemcpyAsync(d_idx, idx.data(), idx.size() * 4, hipMemcpyHostToDevice, st);
        if (r != hipSuccess) return hip_fail(r, "H2D indices");
        DecodeSet ds{};
        ds.base = d_eds;
        ds.presence = d_pres;
        ds.indices = d_idx;
        ds.count = (uint32_t)idx.size();
        ds.axis = (uint32_t)axis;
        ds.k = k;
        ds.S = S;
        return launch_decode(ctx, ds, st);
    }
    // verifyEncoding for many complete vectors at once: re-encode their first
    // half into the scratch square and compare parity halves.  bad[i] = 1 on mismatch.
    int verify_encoding(int axis, const std::vector<uint32_t>& idx, std::vector<uint32_t>& bad) {
        bad.assign(idx.size(), 0);
        if (idx.empty()) return RSM_OK;
        hipError_t r = hipMemcpyAsync(d_idx, idx.data(), idx.size() * 4, hipMemcpyHostToDevice, st);
        if (r != hipSuccess) return hip_fail(r, "H2D indices");
        CodewordSet cs{};
        cs.base = d_eds;
        cs.out_base = d_scratch;
        cs.indices = d_idx;
        cs.cw_stride = axis == RSM_AXIS_ROW ? (uint64_t)W * S : S;
        cs.elem_stride = axis == RSM_AXIS_ROW ? S : (uint64_t)W * S;
        cs.out_offset = axis == RSM_AXIS_ROW ? (uint64_t)k * S : (uint64_t)k * W * S;
        cs.per_square = 1;
        cs.count = (uint32_t)idx.size();
        cs.k = k;
        cs.S = S;
        if (int rc = launch_encode(ctx, cs, st)) return rc;
        if ((r = launch_compare_parity(d_eds, d_scratch, k, S, (uint32_t)axis, d_idx, cs.count, d_flags, st)) != hipSuccess)
            return hip_fail(r, "compare parity");
        if ((r = hipMemcpyAsync(bad.data(), d_flags, idx.size() * 4, hipMemcpyDeviceToHost, st)) != hipSuccess)
            return hip_fail(r, "D2H flags");
        return sync();
    }
};

// Per-codeword device codec calls for the exact sequential path.
int codec_decode_vector(rsm_eds* e, int axis, uint32_t idx, std::vector<uint8_t>& out, bool* decoded) {
    const uint32_t W = e->width;
    *decoded = false;
    if (vector_present(e, axis, idx) < W / 2) return RSM_OK;  // Decode error: swallowed (:292-297)
    out.assign((size_t)W * e->S, 0);
    std::vector<uint8_t*> ptrs(W);
    std::vector<uint8_t> pres(W);
    for (uint32_t p = 0; p < W; ++p) {
        uint32_t r = e->rr(axis, idx, p), c = e->cc(axis, idx, p);
        ptrs[p] = out.data() + (size_t)p * e->S;
        pres[p] = e->has(r, c) ? 1 : 0;
        if (pres[p]) memcpy(ptrs[p], e->cell(r, c), e->S);
    }
    int rc = rsm_decode(e->ctx, ptrs.data(), pres.data(), W, e->S);
    if (rc == RSM_ETOOFEW) return RSM_OK;
    if (rc) return rc;
    *decoded = true;
    return RSM_OK;
}

// verifyEncoding(data, rebuiltIndex, rebuiltShare) (:480-502): vector with an
// optional rebuilt share at `pos`.  *ok = parity equals re-encoded first half.
int codec_verify_encoding(rsm_eds* e, const std::vector<const uint8_t*>& v, bool* ok) {
    const uint32_t W = (uint32_t)v.size(), k = W / 2;
    std::vector<uint8_t> parity((size_t)k * e->S);
    std::vector<uint8_t*> pp(k);
    for (uint32_t i = 0; i < k; ++i) pp[i] = parity.data() + (size_t)i * e->S;
    for (uint32_t i = 0; i < W; ++i)
        if (!v[i]) {
            // Encode of a nil share errors in the reference; bytes.Equal(nil, x) is
            // false for the parity half.  Either way the encoding is rejected.
            *ok = false;
            return RSM_OK;
        }
    int rc = rsm_encode(e->ctx, v.data(), k, e->S, pp.data());
    if (rc) return rc;
    *ok = true;
    for (uint32_t i = 0; i < k && *ok; ++i)
        if (memcmp(v[k + i], pp[i], e->S) != 0) *ok = false;
    return RSM_OK;
}

// ---------------------------------------------------------------------------
// Exact sequential solver (solveCrossword / solveCrosswordRow / solveCrosswordCol)
// ---------------------------------------------------------------------------
int set_byz(rsm_eds* e, rsm_byzantine* byz, int axis, uint32_t idx) {
    if (byz) {
        byz->axis = axis;
        byz->index = idx;
    }
    return fail(RSM_EBYZANTINE, "byzantine %s: %u", axis == RSM_AXIS_ROW ? "row" : "col", idx);
}

// solveCrosswordRow (axis Row) / solveCrosswordCol (axis Col).
int solve_vector(rsm_eds* e, int axis, uint32_t idx, const uint8_t* my_roots, const uint8_t* orth_roots,
                 uint32_t root_len, const Tree& tree, rsm_byzantine* byz, bool* solved, bool* progress) {
    const uint32_t W = e->width;
    *solved = false;
    *progress = false;
    if (vector_complete(e, axis, idx)) {
        *solved = true;
        return RSM_OK;
    }
    std::vector<uint8_t> rebuilt;
    bool decoded = false;
    if (int rc = codec_decode_vector(e, axis, idx, rebuilt, &decoded)) return rc;
    if (!decoded) return RSM_OK;
    auto rb = [&](uint32_t p) { return rebuilt.data() + (size_t)p * e->S; };

    // verifyAgainst{Row,Col}Roots of the rebuilt vector
    {
        std::vector<const uint8_t*> leaves(W);
        for (uint32_t p = 0; p < W; ++p) leaves[p] = rb(p);
        std::vector<uint8_t> root;
        int trc = tree.root(axis, idx, leaves, e->S, root);
        if (trc != 0 || root.size() != root_len || memcmp(root.data(), my_roots + (size_t)idx * root_len, root_len) != 0) {
            snapshot_byzantine(e, axis, idx);  // eds.Row/Col(idx): pre-repair, nil-preserving
            return set_byz(e, byz, axis, idx);
        }
    }
    // newly completed orthogonal vectors
    const int oaxis = axis == RSM_AXIS_ROW ? RSM_AXIS_COL : RSM_AXIS_ROW;
    for (uint32_t o = 0; o < W; ++o) {
        const uint32_t r = e->rr(axis, idx, o), c = e->cc(axis, idx, o);
        if (e->has(r, c)) continue;  // not newly completed
        if (!vector_complete(e, oaxis, o, (int)idx)) continue;
        std::vector<const uint8_t*> leaves = vector_leaves(e, oaxis, o);
        leaves[idx] = rb(o);
        std::vector<uint8_t> root;
        int trc = tree.root(oaxis, o, leaves, e->S, root);
        if (trc != 0 || root.size() != root_len || memcmp(root.data(), orth_roots + (size_t)o * root_len, root_len) != 0) {
            snapshot_byzantine(e, oaxis, o);  // deepCopy(col): the rebuilt position is still nil
            return set_byz(e, byz, oaxis, o);
        }
        bool ok = false;
        if (int rc = codec_verify_encoding(e, leaves, &ok)) return rc;
        if (!ok) {
            snapshot_byzantine(e, oaxis, o);
            return set_byz(e, byz, oaxis, o);
        }
    }
    // insert rebuilt shares
    for (uint32_t p = 0; p < W; ++p) {
        const uint32_t r = e->rr(axis, idx, p), c = e->cc(axis, idx, p);
        if (!e->has(r, c)) {
            memcpy(e->cell(r, c), rb(p), e->S);
            e->present[(size_t)r * W + c] = 1;
        }
    }
    *solved = true;
    *progress = true;
    return RSM_OK;
}

int solve_crossword(rsm_eds* e, const uint8_t* row_roots, const uint8_t* col_roots, uint32_t root_len,
                    const Tree& tree, rsm_byzantine* byz) {
    for (;;) {
        bool solved = true, progress = false;
        for (uint32_t i = 0; i < e->width; ++i) {
            bool s1, p1, s2, p2;
            if (int rc = solve_vector(e, RSM_AXIS_ROW, i, row_roots, col_roots, root_len, tree, byz, &s1, &p1)) return rc;
            if (int rc = solve_vector(e, RSM_AXIS_COL, i, col_roots, row_roots, root_len, tree, byz, &s2, &p2)) return rc;
            solved = solved && s1 && s2;
            progress = progress || p1 || p2;
        }
        if (solved) return RSM_OK;
        if (!progress) return fail(RSM_EUNREPAIRABLE, "failed to solve data square");
    }
}

// preRepairSanityCheck (:366-429): every complete row/column must match its root
// and be a valid codeword.  The reference checks them concurrently and returns
// whichever failure its errgroup sees first; this checks them in index order
// (row i root, row i encoding, col i root, col i encoding).
int pre_repair_sanity_check(rsm_eds* e, DevSquare& dev, const uint8_t* row_roots, const uint8_t* col_roots,
                            uint32_t root_len, const Tree& tree, rsm_byzantine* byz) {
    const uint32_t W = e->width;
    std::vector<int> axes;
    std::vector<uint32_t> idxs;
    std::vector<std::vector<const uint8_t*>> leaves;
    std::vector<uint32_t> rows, cols;
    for (uint32_t i = 0; i < W; ++i) {
        if (vector_complete(e, RSM_AXIS_ROW, i)) rows.push_back(i);
        if (vector_complete(e, RSM_AXIS_COL, i)) cols.push_back(i);
    }
    if (rows.empty() && cols.empty()) return RSM_OK;
    for (uint32_t i : rows) { axes.push_back(RSM_AXIS_ROW); idxs.push_back(i); leaves.push_back(vector_leaves(e, RSM_AXIS_ROW, i)); }
    for (uint32_t i : cols) { axes.push_back(RSM_AXIS_COL); idxs.push_back(i); leaves.push_back(vector_leaves(e, RSM_AXIS_COL, i)); }
    std::vector<std::vector<uint8_t>> roots;
    std::vector<int> rcs;
    roots_many(tree, axes, idxs, leaves, e->S, roots, rcs);
    std::vector<uint32_t> bad_rows, bad_cols;
    if (int rc = dev.upload(e)) return rc;
    if (int rc = dev.verify_encoding(RSM_AXIS_ROW, rows, bad_rows)) return rc;
    if (int rc = dev.verify_encoding(RSM_AXIS_COL, cols, bad_cols)) return rc;
    std::vector<int> row_pos(W, -1), col_pos(W, -1);
    for (size_t j = 0; j < rows.size(); ++j) row_pos[rows[j]] = (int)j;
    for (size_t j = 0; j < cols.size(); ++j) col_pos[cols[j]] = (int)j;
    auto root_ok = [&](size_t j, const uint8_t* want) {
        return rcs[j] == 0 && roots[j].size() == root_len && memcmp(roots[j].data(), want, root_len) == 0;
    };
    for (uint32_t i = 0; i < W; ++i) {
        if (row_pos[i] >= 0) {
            size_t j = (size_t)row_pos[i];
            if (!root_ok(j, row_roots + (size_t)i * root_len) || bad_rows[j]) {
                snapshot_byzantine(e, RSM_AXIS_ROW, i);
                return set_byz(e, byz, RSM_AXIS_ROW, i);
            }
        }
        if (col_pos[i] >= 0) {
            size_t j = rows.size() + (size_t)col_pos[i];
            if (!root_ok(j, col_roots + (size_t)i * root_len) || bad_cols[col_pos[i]]) {
                snapshot_byzantine(e, RSM_AXIS_COL, i);
                return set_byz(e, byz, RSM_AXIS_COL, i);
            }
        }
    }
    return RSM_OK;
}

// Device fast path.  Returns RSM_OK with the square repaired, 1 to request the
// exact sequential path (e is untouched in that case), or an RSM_E* error.
enum { kFallbackStuck = 1, kFallbackEncoding = 2, kFallbackRoots = 3 };

// Zero-copy form of the common first sweep (BenchmarkRepair's shape: every
// incomplete row has >= k shares, so one row sweep completes the square).  The
// EDS's host square is pinned and mapped: the decode kernel reads the present
// cells straight from it over PCIe, stores them into the device square, and writes
// every rebuilt cell both into the device square and straight back into the host
// square -- half the bytes of an upload + download of the whole square, no copy
// engine.  Writing the rebuilt bytes into cells that are still nil is harmless:
// nothing reads a cell whose presence byte is 0 (the exact solver, snapshots and
// Flattened go by presence), and presence flips only after the device verification
// passes.  Returns RSM_OK (repaired), 1 (fall back) or an RSM_E* error.
int fast_repair_rows_zero_copy(rsm_eds* e, DevSquare& dev, const std::vector<uint32_t>& todo,
                               const uint8_t* row_roots, const uint8_t* col_roots, const DevTree& dt) {
    const uint32_t W = e->width, k = W / 2;
    const size_t S = e->S, row = (size_t)W * S;
    // the zero-copy decoders: GF(2^8) 65 <= k <= 128 (decode_gf8_split_zc_kernel) and the
    // GF(2^16) single passes, k <= 512 (dec16f_kernel / dec16h_kernel)
    const bool zc_decoder = field_bits(k) == 8 ? ceil_pow2(k) == 128 : ceil_pow2(k) <= 512;
    // the rows' decoders AND the columns' verification re-encode (elem_stride = row) must
    // take the narrow forms: a wide GF(2^16) column encode runs through sv's work arrays
    // and takes sv's scratch lock, which this function holds for the leaf digests
    if (!e->data.pinned || !zc_decoder || !narrow_ok(dev.ctx, k, S, S) || !narrow_ok(dev.ctx, k, row, S)) return 1;
    void* hmap = nullptr;
    hipError_t r = hipHostGetDevicePointer(&hmap, e->data.data(), 0);
    if (r != hipSuccess || !hmap) {
        (void)hipGetLastError();
        return 1;
    }
    // Zero-copy transport (profiles/r02c_zcprobe.jsonl: GPU reads of mapped host
    // memory reach the copy engine's ~57 GB/s, and reads plus writes together ~73
    // GB/s, more than the copy engine's duplex): only the present cells go up and
    // only the rebuilt cells come back.  The decoder runs on a capped grid so its
    // stores of one task drain while the loads of its next task arrive -- ONE sweep
    // launch over every row (two launches, top half then bottom half so that the
    // verification could start on the top half, were 9 % slower end to end: each
    // launch's tail leaves the link half idle; profiles/r05an_repair_sweep_ab.jsonl).
    // Then, beside each other:
    //   sv: the columns of the top half are re-encoded and compared with the bottom half
    //   (every row is a codeword by construction, so this makes the square a valid 2D
    //   codeword: the reference's verifyEncoding of each completed column,
    //   extendeddatacrossword.go:184);
    //   st: the roots of all 2W vectors (verifyAgainstRowRoots / ColRoots, :153, :173).
    hipStream_t st = dev.st;
    LaneGuard gv(dev.ctx);
    if (!gv.lane) return gv.rc;
    hipStream_t sv = gv.lane->stream;
    StreamScratch& ss = stream_scratch(dev.ctx, sv);
    std::lock_guard<std::mutex> lk(ss.mu);
    if ((r = hipStreamSynchronize(sv)) != hipSuccess) return hip_fail(r, "hipStreamSynchronize");
    if ((r = ss.leaf.ensure((size_t)W * W * (dt.nmt ? 64 : 32))) != hipSuccess)
        return hip_fail(r, "hipMalloc (leaf digests)");
    uint32_t* leaf = static_cast<uint32_t*>(ss.leaf.ptr);
    const uint32_t RL = dt.root_len;
    DevBuf& rb = dev.ctx->eds.roots;
    if ((r = rb.ensure((size_t)2 * W * RL)) != hipSuccess) return hip_fail(r, "hipMalloc (roots)");
    uint8_t* d_roots = static_cast<uint8_t*>(rb.ptr);
    DevBuf& sb = dev.ctx->eds.status;
    if ((r = sb.ensure((size_t)2 * W * 4)) != hipSuccess) return hip_fail(r, "hipMalloc (tree status)");
    uint32_t* d_status = static_cast<uint32_t*>(sb.ptr);
    // the verification lane's own events (created once per lane, not per call)
    hipEvent_t ev_top = lane_event(*gv.lane, 0), ev_bot = lane_event(*gv.lane, 1);
    if (!ev_top || !ev_bot) return hip_fail(hipErrorOutOfMemory, "hipEventCreate (repair)");
    // the presence map and the row list go up from the lane's pinned staging: from the
    // pageable vectors hipMemcpyAsync is a staged, synchronous copy (35 us of host time
    // for k = 128's 64 KiB map)
    HostBuf& hb = gv.lane->host;
    const size_t pres_n = e->present.size();  // W * W: the row list after it stays 4-byte aligned
    // then, 16-byte aligned, the verification results (mismatch flag, roots, NMT tree
    // statuses), written into the same pinned staging by the kernels (flag, DefaultTree
    // roots) or by asynchronous copies (NMT roots and statuses)
    const size_t back = (pres_n + todo.size() * 4 + 15) / 16 * 16;
    const size_t roots_n = (size_t)2 * W * dt.root_len;
    if ((r = hb.ensure(back + 16 + roots_n + (size_t)2 * W * 4)) != hipSuccess)
        return hip_fail(r, "hipHostMalloc (repair staging)");
    uint8_t* hs = static_cast<uint8_t*>(hb.ptr);
    void* hs_map = nullptr;  // the staging's device address: the DefaultTree roots and the
                             // mismatch flag are written there by the kernels themselves
    if ((r = hipHostGetDevicePointer(&hs_map, hs, 0)) != hipSuccess || !hs_map) {
        (void)hipGetLastError();
        return 1;
    }
    memcpy(hs, e->present.data(), pres_n);
    memcpy(hs + pres_n, todo.data(), todo.size() * 4);
    struct DrainSt {  // an early return must not hand the lane's staging back with its DMA in flight
        hipStream_t s[2];
        bool armed = true;
        ~DrainSt() {
            if (armed)
                for (hipStream_t x : s) (void)hipStreamSynchronize(x);
        }
    } drain_st{{st, sv}};
    // presence map and row list in one copy kernel on st, read through the staging's
    // device mapping (a copy-engine transfer put a 10-16 us cross-engine wait in front of
    // the sweep); the row list lands right behind the map in the same device buffer
    if ((r = launch_stage_copy(dev.d_pres, hs_map, pres_n + todo.size() * 4, st)) != hipSuccess)
        return hip_fail(r, "stage presence and rows");
    const uint32_t* const d_rows = reinterpret_cast<const uint32_t*>(dev.d_pres + pres_n);
    // a quarter of the CUs (A/B on MI355X, profiles/r02c_repair_ab.txt: 64 workgroups
    // 0.87 ms, 128 0.89 ms, one per task 0.91 ms)
    const uint32_t zc_grid = dev.ctx->cus / 4 ? dev.ctx->cus / 4 : 1;
    // (A split transport -- a gather kernel reading the present cells on a second lane while
    // the device decoder of the previous chunk writes its rebuilt cells back -- and the two
    // halves' sweeps on two lanes at once both measured no faster: DESIGN.md §5.)
    auto sweep = [&](size_t t0, size_t t1) -> int {
        if (t1 <= t0) return RSM_OK;
        DecodeSet ds{};
        ds.base = dev.d_eds;
        ds.presence = dev.d_pres;
        ds.indices = d_rows + t0;
        ds.count = (uint32_t)(t1 - t0);
        ds.axis = RSM_AXIS_ROW;
        ds.k = k;
        ds.S = e->S;
        ds.in_base = static_cast<const uint8_t*>(hmap);
        ds.mirror = static_cast<uint8_t*>(hmap);
        ds.grid = zc_grid;
        return launch_decode(dev.ctx, ds, st);
    };
    // complete rows (not decoded) go up as they are, top half first
    auto upload_complete = [&](uint32_t lo, uint32_t hi, size_t t) -> int {
        for (uint32_t i = lo; i < hi;) {
            if (t < todo.size() && todo[t] == i) {
                ++i, ++t;
                continue;
            }
            uint32_t j = i;
            while (j < hi && !(t < todo.size() && todo[t] == j)) ++j;
            if ((r = hipMemcpyAsync(dev.d_eds + i * row, e->data.data() + i * row, (j - i) * row,
                                    hipMemcpyHostToDevice, st)) != hipSuccess)
                return hip_fail(r, "H2D complete rows");
            i = j;
        }
        return RSM_OK;
    };
    const bool halves = repair_mode() == 1;  // (diagnostic A/B: the two-launch form)
    size_t split = todo.size();
    if (halves) {
        split = 0;
        while (split < todo.size() && todo[split] < k) ++split;
    }
    if (int rc = upload_complete(0, halves ? k : W, 0)) return rc;
    if (int rc = sweep(0, split)) return rc;
    if (halves) {
        (void)hipEventRecord(ev_top, st);
        if (int rc = upload_complete(k, W, split)) return rc;
        if (int rc = sweep(split, todo.size())) return rc;
    }
    (void)hipEventRecord(ev_bot, st);
    // verification.  sv: the column re-encode of the top half and the encoding compare;
    // st, right behind its own sweep: the leaf digests of the WHOLE square and the
    // trees.  (A cross-queue wait costs 11-12 us on the critical path even when its event
    // has long completed, and one leaf launch is latency-bound -- 9 compressions per
    // cell, one wave per SIMD for the whole square -- so hashing the top half early on sv
    // saved nothing: profiles/r05al_repair_tail.txt.)  The mismatch flag and the
    // DefaultTree roots land in the pinned staging straight from the kernels.
    uint32_t* const h_mismatch = reinterpret_cast<uint32_t*>(hs + back);
    uint8_t* const got = hs + back + 16;
    uint32_t* const status = reinterpret_cast<uint32_t*>(got + roots_n);
    uint8_t* const got_map = static_cast<uint8_t*>(hs_map) + back + 16;
    *h_mismatch = 0;
    memset(status, 0, (size_t)2 * W * 4);
    (void)hipStreamWaitEvent(sv, halves ? ev_top : ev_bot, 0);  // (one event record on st)
    CodewordSet cols{};
    cols.base = dev.d_eds;
    cols.out_base = dev.d_scratch;
    cols.square_stride = (uint64_t)W * row;
    cols.cw_stride = S;
    cols.elem_stride = row;
    cols.out_offset = (uint64_t)k * row;
    cols.per_square = W;
    cols.count = W;
    cols.k = k;
    cols.S = e->S;
    cols.pass = 1;
    if (int rc = launch_encode(dev.ctx, cols, sv)) return rc;
    if (halves) (void)hipStreamWaitEvent(sv, ev_bot, 0);
    e->stats.sweeps++;
    e->stats.decoded_vectors += (uint32_t)todo.size();
    if ((r = launch_compare(dev.d_eds + (size_t)k * row, dev.d_scratch + (size_t)k * row, (uint64_t)k * row,
                            reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(hs_map) + back), sv)) != hipSuccess)
        return hip_fail(r, "verify (encoding)");
    if (dt.nmt) {
        // namespaced trees: leaves and nodes of the whole square in one launch pair
        // (leaf scratch: sv's StreamScratch, held above for the whole call, both streams
        // drained before it is released); the kernel stores roots byte-wise, so they
        // come back by copy
        if ((r = launch_nmt_roots(dev.d_eds, W, e->S, dt.p.namespace_size, dt.p.square_size, dt.p.ignore_max_namespace,
                                  leaf, d_roots, d_status, st)) != hipSuccess)
            return hip_fail(r, "NMT roots");
        if ((r = hipMemcpyAsync(got, d_roots, roots_n, hipMemcpyDeviceToHost, st)) != hipSuccess ||
            (r = hipMemcpyAsync(status, d_status, (size_t)2 * W * 4, hipMemcpyDeviceToHost, st)) != hipSuccess)
            return hip_fail(r, "verify (NMT roots)");
    } else if ((r = launch_leaf_hashes(dev.d_eds, W * W, e->S, leaf, st)) != hipSuccess ||
               (r = launch_tree_roots(leaf, W, 0, 2 * W, got_map, st)) != hipSuccess) {  // latency-bound: one launch
        return hip_fail(r, "verify (roots)");
    }
    if ((r = hipStreamSynchronize(st)) != hipSuccess || (r = hipStreamSynchronize(sv)) != hipSuccess)
        return hip_fail(r, "verify");
    drain_st.armed = false;  // both streams drained
    const bool enc_ok = *h_mismatch == 0;
    const bool roots_ok = std::all_of(status, status + 2 * W, [](uint32_t x) { return x == 0; }) &&
                          memcmp(got, row_roots, (size_t)W * RL) == 0 &&
                          memcmp(got + (size_t)W * RL, col_roots, (size_t)W * RL) == 0;
    if (!enc_ok || !roots_ok) {
        e->stats.fallback_reason = enc_ok ? kFallbackRoots : kFallbackEncoding;
        return 1;
    }
    std::fill(e->present.begin(), e->present.end(), 1);
    e->stats.fast_path = 1;
    return RSM_OK;
}

int fast_repair(rsm_eds* e, DevSquare& dev, const uint8_t* row_roots, const uint8_t* col_roots,
                uint32_t root_len, const Tree& tree) {
    const uint32_t W = e->width, k = W / 2;
    DevTree dt;
    const bool dev_tree = device_tree_for(tree.fn, tree.user, W, &dt) && root_len == dt.root_len;
    if (dev_tree) {
        // one row sweep completes the square?  then the pipelined form
        std::vector<uint32_t> todo;
        bool rows_only = true;
        for (uint32_t i = 0; i < W && rows_only; ++i) {
            const uint8_t* pr = e->present.data() + (size_t)i * W;
            const uint32_t have = W - (uint32_t)std::count(pr, pr + W, uint8_t{0});
            if (have < W) {
                if (have >= k) todo.push_back(i);
                else rows_only = false;
            }
        }
        if (rows_only && !todo.empty()) {
            int rc = fast_repair_rows_zero_copy(e, dev, todo, row_roots, col_roots, dt);
            if (rc <= 0 || e->stats.fallback_reason) return rc;  // repaired / error / byzantine evidence
        }
    }
    std::vector<uint8_t> pres = e->present;
    auto missing_in = [&](int axis, uint32_t idx, uint32_t* have) {
        uint32_t h = 0;
        for (uint32_t p = 0; p < W; ++p) h += pres[(size_t)e->rr(axis, idx, p) * W + e->cc(axis, idx, p)] ? 1 : 0;
        *have = h;
        return W - h;
    };
    if (int rc = dev.upload(e)) return rc;
    for (;;) {
        bool progress = false;
        for (int axis = RSM_AXIS_ROW; axis <= RSM_AXIS_COL; ++axis) {
            std::vector<uint32_t> todo;
            for (uint32_t i = 0; i < W; ++i) {
                uint32_t have;
                if (missing_in(axis, i, &have) > 0 && have >= k) todo.push_back(i);
            }
            if (todo.empty()) continue;
            if (int rc = dev.decode(axis, todo)) return rc;
            for (uint32_t i : todo)
                for (uint32_t p = 0; p < W; ++p) pres[(size_t)e->rr(axis, i, p) * W + e->cc(axis, i, p)] = 1;
            if (int rc = dev.upload_presence(pres)) return rc;
            e->stats.sweeps++;
            e->stats.decoded_vectors += (uint32_t)todo.size();
            progress = true;
        }
        if (!progress) break;
    }
    for (uint8_t p : pres)
        if (!p) {
            e->stats.fallback_reason = kFallbackStuck;
            return 1;
        }
    // The repaired square must be the 2D extension of its own Q0 ...
    const size_t S = e->S;
    hipError_t r = hipMemcpy2DAsync(dev.d_scratch, (size_t)W * S, dev.d_eds, (size_t)W * S, (size_t)k * S, k,
                                    hipMemcpyDeviceToDevice, dev.st);
    if (r != hipSuccess) return hip_fail(r, "D2D Q0");
    if (int rc = extend_squares(dev.ctx, dev.d_scratch, k, e->S, 1, dev.st)) return rc;
    if ((r = hipMemsetAsync(dev.d_flags, 0, 4, dev.st)) != hipSuccess) return hip_fail(r, "memset");
    if ((r = launch_compare(dev.d_eds, dev.d_scratch, (uint64_t)W * W * S, dev.d_flags, dev.st)) != hipSuccess)
        return hip_fail(r, "compare");
    uint32_t mismatch = 0;
    // ... and match every committed row and column root: on the device for the
    // DefaultTree (kernels_sha.hip), through the host Tree plugin otherwise.  The
    // device check runs before any copy back, so an accepted square lands straight
    // in the EDS's own (already resident) buffer and a rejected one costs no D2H.
    if (dev_tree) {
        const uint32_t RL = dt.root_len;
        DevBuf& rb = dev.ctx->eds.roots;
        DevBuf& sb = dev.ctx->eds.status;
        if ((r = rb.ensure((size_t)2 * W * RL)) != hipSuccess) return hip_fail(r, "hipMalloc (roots)");
        if ((r = sb.ensure((size_t)2 * W * 4)) != hipSuccess) return hip_fail(r, "hipMalloc (tree status)");
        if (int rc = device_tree_roots(dev.ctx, dt, dev.d_eds, W, e->S, static_cast<uint8_t*>(rb.ptr),
                                       static_cast<uint32_t*>(sb.ptr), dev.st))
            return rc;
        std::vector<uint8_t> got((size_t)2 * W * RL);
        std::vector<uint32_t> status((size_t)2 * W);
        if ((r = hipMemcpyAsync(&mismatch, dev.d_flags, 4, hipMemcpyDeviceToHost, dev.st)) != hipSuccess)
            return hip_fail(r, "D2H flag");
        if ((r = hipMemcpyAsync(got.data(), rb.ptr, got.size(), hipMemcpyDeviceToHost, dev.st)) != hipSuccess ||
            (r = hipMemcpyAsync(status.data(), sb.ptr, status.size() * 4, hipMemcpyDeviceToHost, dev.st)) != hipSuccess)
            return hip_fail(r, "D2H roots");
        if (int rc = dev.sync()) return rc;
        if (mismatch) {
            e->stats.fallback_reason = kFallbackEncoding;
            return 1;
        }
        if (!std::all_of(status.begin(), status.end(), [](uint32_t x) { return x == 0; }) ||
            memcmp(got.data(), row_roots, (size_t)W * RL) != 0 ||
            memcmp(got.data() + (size_t)W * RL, col_roots, (size_t)W * RL) != 0) {
            e->stats.fallback_reason = kFallbackRoots;
            return 1;
        }
        if ((r = hipMemcpyAsync(e->data.data(), dev.d_eds, e->data.size(), hipMemcpyDeviceToHost, dev.st)) !=
            hipSuccess)
            return hip_fail(r, "D2H square");
        if (int rc = dev.sync()) return rc;
        std::fill(e->present.begin(), e->present.end(), 1);
        e->stats.fast_path = 1;
        return RSM_OK;
    }
    HostSquare repaired;
    if (!repaired.assign((size_t)W * W * S)) return fail(RSM_ENOMEM, "Repair: out of memory");
    if ((r = hipMemcpyAsync(&mismatch, dev.d_flags, 4, hipMemcpyDeviceToHost, dev.st)) != hipSuccess)
        return hip_fail(r, "D2H flag");
    if ((r = hipMemcpyAsync(repaired.data(), dev.d_eds, repaired.size(), hipMemcpyDeviceToHost, dev.st)) != hipSuccess)
        return hip_fail(r, "D2H square");
    if (int rc = dev.sync()) return rc;
    if (mismatch) {
        e->stats.fallback_reason = kFallbackEncoding;
        return 1;
    }
    std::vector<int> axes;
    std::vector<uint32_t> idxs;
    std::vector<std::vector<const uint8_t*>> leaves;
    for (int axis = RSM_AXIS_ROW; axis <= RSM_AXIS_COL; ++axis)
        for (uint32_t i = 0; i < W; ++i) {
            axes.push_back(axis);
            idxs.push_back(i);
            std::vector<const uint8_t*> v(W);
            for (uint32_t p = 0; p < W; ++p)
                v[p] = repaired.data() + ((size_t)e->rr(axis, i, p) * W + e->cc(axis, i, p)) * S;
            leaves.push_back(std::move(v));
        }
    std::vector<std::vector<uint8_t>> roots;
    std::vector<int> rcs;
    roots_many(tree, axes, idxs, leaves, e->S, roots, rcs);
    for (size_t j = 0; j < axes.size(); ++j) {
        const uint8_t* want = (axes[j] == RSM_AXIS_ROW ? row_roots : col_roots) + (size_t)idxs[j] * root_len;
        if (rcs[j] != 0 || roots[j].size() != root_len || memcmp(roots[j].data(), want, root_len) != 0) {
            e->stats.fallback_reason = kFallbackRoots;
            return 1;
        }
    }
    e->data.swap(repaired);
    std::fill(e->present.begin(), e->present.end(), 1);
    e->stats.fast_path = 1;
    return RSM_OK;
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

int rsm_eds_compute(rsm_ctx* ctx, const uint8_t* const* data, const uint32_t* lens, uint64_t n, rsm_eds** out) {
    if (!ctx || !out || (n && (!data || !lens))) return fail(RSM_EINVAL, "rsm_eds_compute: bad arguments");
    *out = nullptr;
    if (n > (uint64_t)rsm_codec_max_chunks()) return fail(RSM_ESHAPE, "number of chunks exceeds the maximum");
    uint32_t k = 0, S = 0;
    if (int rc = check_square(data, lens, n, &k, &S)) return rc;
    for (uint64_t i = 0; i < n; ++i)
        if (!data[i]) return fail(RSM_EINVAL, "ComputeExtendedDataSquare: share %llu is nil", (unsigned long long)i);
    rsm_eds* e = alloc_eds(ctx, 2 * k, S);
    if (!e) return fail(RSM_ENOMEM, "rsm_eds_compute: out of memory");
    e->odw = k;
    if (k > 0) {
        // gather the ODS straight into the (pinned) EDS's Q0 quadrant, then extend
        // in place from there (rsm_extend_square leaves Q0 alone when ods == eds's Q0)
        const size_t row = (size_t)2 * k * S;
        for (uint64_t i = 0; i < n; ++i) memcpy(e->data.data() + (i / k) * row + (i % k) * S, data[i], S);
        int rc = rsm_extend_square_inplace_host(ctx, e->data.data(), k, S);
        if (rc) {
            delete e;
            return rc;
        }
        std::fill(e->present.begin(), e->present.end(), 1);
    }
    *out = e;
    return RSM_OK;
}

int rsm_eds_import(rsm_ctx* ctx, const uint8_t* const* data, const uint32_t* lens, uint64_t n, rsm_eds** out) {
    if (!out || (n && (!data || !lens))) return fail(RSM_EINVAL, "rsm_eds_import: bad arguments");
    *out = nullptr;
    if (n > 4ull * (uint64_t)rsm_codec_max_chunks()) return fail(RSM_ESHAPE, "number of chunks exceeds the maximum");
    uint32_t w = 0, S = 0;
    if (int rc = check_square(data, lens, n, &w, &S)) return rc;
    if (w % 2 != 0) return fail(RSM_ESHAPE, "extended data square width %u must be even", w);
    rsm_eds* e = alloc_eds(ctx, w, S);
    if (!e) return fail(RSM_ENOMEM, "rsm_eds_import: out of memory");
    e->odw = w / 2;
    for (uint64_t i = 0; i < n; ++i)
        if (data[i]) {
            memcpy(e->data.data() + i * S, data[i], S);
            e->present[i] = 1;
        }
    *out = e;
    return RSM_OK;
}

int rsm_eds_new(rsm_ctx* ctx, uint32_t eds_width, uint32_t share_size, rsm_eds** out) {
    if (!out) return fail(RSM_EINVAL, "rsm_eds_new: bad arguments");
    *out = nullptr;
    if (eds_width % 2 != 0) return fail(RSM_ESHAPE, "extended data square width %u must be even", eds_width);
    if (int rc = validate_chunk_size(share_size)) return rc;
    rsm_eds* e = alloc_eds(ctx, eds_width, share_size);
    if (!e) return fail(RSM_ENOMEM, "rsm_eds_new: out of memory");
    e->odw = eds_width / 2;
    *out = e;
    return RSM_OK;
}

void rsm_eds_free(rsm_eds* eds) { delete eds; }

// Attach (or replace) the GPU context of a square built host-only.
int rsm_eds_set_context(rsm_eds* e, rsm_ctx* ctx) {
    if (!e) return fail(RSM_EINVAL, "NULL eds");
    e->ctx = ctx;
    return RSM_OK;
}
uint32_t rsm_eds_width(const rsm_eds* e) { return e ? e->width : 0; }
uint32_t rsm_eds_original_width(const rsm_eds* e) { return e ? e->odw : 0; }
uint32_t rsm_eds_share_size(const rsm_eds* e) { return e ? e->S : 0; }

int rsm_eds_get_cell(const rsm_eds* e, uint32_t row, uint32_t col, uint8_t* out) {
    if (!e || row >= e->width || col >= e->width) return fail(RSM_EINVAL, "GetCell: index out of range");
    if (!e->has(row, col)) return 0;
    if (out) memcpy(out, e->cell(row, col), e->S);
    return 1;
}

int rsm_eds_set_cell(rsm_eds* e, uint32_t row, uint32_t col, const uint8_t* share, uint32_t len) {
    if (!e || row >= e->width || col >= e->width) return fail(RSM_EINVAL, "SetCell: index out of range");
    if (e->has(row, col)) return fail(RSM_ECELL, "cannot set cell (%u, %u) as it already has a value", row, col);
    if (!share || len != e->S)
        return fail(RSM_ECELL, "cannot set cell with chunk size %u because dataSquare chunk size is %u", len, e->S);
    memcpy(e->cell(row, col), share, e->S);
    e->present[(size_t)row * e->width + col] = 1;
    return RSM_OK;
}

int rsm_eds_overwrite_cell(rsm_eds* e, uint32_t row, uint32_t col, const uint8_t* share, uint32_t len) {
    if (!e || row >= e->width || col >= e->width) return fail(RSM_EINVAL, "setCell: index out of range");
    if (!share) {
        e->present[(size_t)row * e->width + col] = 0;
        memset(e->cell(row, col), 0, e->S);
        return RSM_OK;
    }
    if (len != e->S) return fail(RSM_ECELL, "setCell: share of %u bytes in a square of %u-byte shares", len, e->S);
    memcpy(e->cell(row, col), share, e->S);
    e->present[(size_t)row * e->width + col] = 1;
    return RSM_OK;
}

int rsm_eds_flattened(const rsm_eds* e, uint8_t* out, uint8_t* present) {
    if (!e) return fail(RSM_EINVAL, "Flattened: NULL eds");
    if (out) memcpy(out, e->data.data(), e->data.size());
    if (present) memcpy(present, e->present.data(), e->present.size());
    return RSM_OK;
}

int rsm_eds_roots(rsm_eds* e, int axis, rsm_tree_root_fn tree_fn, void* user, uint8_t* roots_out,
                  uint32_t root_cap, uint32_t* root_len) {
    if (!e || !roots_out || !root_len || (axis != RSM_AXIS_ROW && axis != RSM_AXIS_COL))
        return fail(RSM_EINVAL, "roots: bad arguments");
    Tree tree{tree_fn, user};
    DevTree dt;
    if (e->ctx && device_tree_for(tree_fn, user, e->width, &dt) && root_cap >= dt.root_len &&
        std::all_of(e->present.begin(), e->present.end(), [](uint8_t p) { return p != 0; })) {
        // complete square + a tree the GPU computes (DefaultTree, NMT): every leaf
        // and node hash on the device
        const uint32_t W = e->width, RL = dt.root_len;
        std::lock_guard<std::mutex> lk(e->ctx->eds_mu);
        DevSquare dev{};
        if (int rc = dev.init(e->ctx, W, e->S)) return rc;
        hipError_t r = hipMemcpyAsync(dev.d_eds, e->data.data(), e->data.size(), hipMemcpyHostToDevice, dev.st);
        if (r != hipSuccess) return hip_fail(r, "H2D square");
        DevBuf& rb = e->ctx->eds.roots;
        DevBuf& sb = e->ctx->eds.status;
        if ((r = rb.ensure((size_t)2 * W * RL)) != hipSuccess) return hip_fail(r, "hipMalloc (roots)");
        if ((r = sb.ensure((size_t)2 * W * 4)) != hipSuccess) return hip_fail(r, "hipMalloc (tree status)");
        if (int rc = device_tree_roots(e->ctx, dt, dev.d_eds, W, e->S, static_cast<uint8_t*>(rb.ptr),
                                       static_cast<uint32_t*>(sb.ptr), dev.st))
            return rc;
        const size_t ax = axis == RSM_AXIS_COL ? 1 : 0;
        std::vector<uint8_t> got((size_t)W * RL);
        std::vector<uint32_t> status(W);
        if ((r = hipMemcpyAsync(got.data(), static_cast<uint8_t*>(rb.ptr) + ax * W * RL, got.size(),
                                hipMemcpyDeviceToHost, dev.st)) != hipSuccess ||
            (r = hipMemcpyAsync(status.data(), static_cast<uint32_t*>(sb.ptr) + ax * W, status.size() * 4,
                                hipMemcpyDeviceToHost, dev.st)) != hipSuccess)
            return hip_fail(r, "D2H roots");
        if (int rc = dev.sync()) return rc;
        for (uint32_t i = 0; i < W; ++i) {
            if (status[i]) return fail(RSM_ETREE, "tree error computing root %u (namespace push order)", i);
            memcpy(roots_out + (size_t)i * root_cap, got.data() + (size_t)i * RL, RL);
        }
        *root_len = RL;
        return RSM_OK;
    }
    std::vector<int> axes;
    std::vector<uint32_t> idxs;
    std::vector<std::vector<const uint8_t*>> leaves;
    for (uint32_t i = 0; i < e->width; ++i) {
        if (!vector_complete(e, axis, i))
            return fail(RSM_ETREE, "can not compute root of incomplete %s", axis == RSM_AXIS_ROW ? "row" : "column");
        axes.push_back(axis);
        idxs.push_back(i);
        leaves.push_back(vector_leaves(e, axis, i));
    }
    std::vector<std::vector<uint8_t>> roots;
    std::vector<int> rcs;
    roots_many(tree, axes, idxs, leaves, e->S, roots, rcs);
    uint32_t len = 0;
    for (uint32_t i = 0; i < e->width; ++i) {
        if (rcs[i] != 0) return fail(RSM_ETREE, "tree error computing root %u", i);
        len = (uint32_t)roots[i].size();
        if (len > root_cap) return fail(RSM_EINVAL, "root of %u bytes exceeds capacity %u", len, root_cap);
        memcpy(roots_out + (size_t)i * root_cap, roots[i].data(), len);
    }
    *root_len = len;
    return RSM_OK;
}

int rsm_eds_repair(rsm_eds* e, const uint8_t* row_roots, const uint8_t* col_roots, uint32_t root_len,
                   rsm_tree_root_fn tree_fn, void* user, rsm_byzantine* byz) {
    if (!e || !row_roots || !col_roots || root_len == 0) return fail(RSM_EINVAL, "Repair: bad arguments");
    e->stats = rsm_repair_stats{};
    e->byz_data.clear();
    e->byz_present.clear();
    if (byz) {
        byz->axis = -1;
        byz->index = 0;
    }
    if (e->width == 0) return RSM_OK;
    if (!e->ctx) return fail(RSM_EDEVICE, "Repair needs a GPU context (square was built without one)");
    Tree tree{tree_fn, user};
    DevSquare dev{};
    {
        std::lock_guard<std::mutex> lk(e->ctx->eds_mu);
        if (int rc = dev.init(e->ctx, e->width, e->S)) return rc;
        if (int rc = pre_repair_sanity_check(e, dev, row_roots, col_roots, root_len, tree, byz)) return rc;
        const bool complete = memchr(e->present.data(), 0, e->present.size()) == nullptr;
        if (complete) return RSM_OK;  // solveCrossword: solved on the first sweep
        int rc = fast_repair(e, dev, row_roots, col_roots, root_len, tree);
        if (rc <= 0) return rc;
    }
    return solve_crossword(e, row_roots, col_roots, root_len, tree, byz);
}

int rsm_eds_byzantine_shares(const rsm_eds* e, uint8_t* out, uint8_t* present) {
    if (!e) return fail(RSM_EINVAL, "NULL eds");
    if (e->byz_present.empty()) return fail(RSM_EINVAL, "no ErrByzantineData recorded");
    if (out) memcpy(out, e->byz_data.data(), e->byz_data.size());
    if (present) memcpy(present, e->byz_present.data(), e->byz_present.size());
    return RSM_OK;
}

int rsm_eds_repair_stats(const rsm_eds* e, rsm_repair_stats* out) {
    if (!e || !out) return fail(RSM_EINVAL, "NULL argument");
    *out = e->stats;
    return RSM_OK;
}

}  // extern "C"
