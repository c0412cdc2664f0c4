// rsm_multi.cpp -- one square over several GPUs of one node, behind the C ABI
// (configuration 5: k = 512, S = 512, rows sharded over 8 MI355X).
//
// One process drives all GPUs (a cgo ComputeExtendedDataSquare call,
// extendeddatasquare.go:50-77, is one goroutine): one rsm_ctx per device and an
// RCCL clique from ncclCommInitAll.  GPU g owns Q0 rows [g k/G, (g+1) k/G):
//   1. row pass of its rows (erasureExtendRow) -> its rows of the top half [Q0|Q1];
//   2. exchange over xGMI:
//        RSM_SCHED_ALLGATHER (north_star): in-place all-gather of the top half, every
//          GPU receives (G-1) k/G x 2k shares;
//        RSM_SCHED_ALLTOALL: grouped send/recv transpose, GPU g receives only its
//          2k/G columns of every other GPU's rows (G-1 times fewer bytes);
//   3. column pass of its 2k/G columns (erasureExtendCol; Q3 from Q1 columns equals
//      the reference's Q3 from Q2 rows by linearity, extendeddatasquare.go:204-207).
// Every step of a GPU is queued on that GPU's context stream, so the device orders
// kernels and collectives itself: no host synchronisation between the steps.
#include <rccl/rccl.h>

#include <cstring>

#include "rsm_internal.hpp"

using namespace rsm;

struct rsm_multi {
    int n = 0;
    std::vector<rsm_ctx*> ctx;
    std::vector<ncclComm_t> comm;
    std::vector<DevBuf> eds;       // per GPU: a full [2k][2k][S] square (host path)
    std::vector<DevBuf> pack[2];   // per GPU: all-to-all send / receive staging
    std::vector<hipStream_t> side; // per GPU: the host path's Q1 download (overlaps the column pass)
    std::vector<hipEvent_t> rows_done;  // per GPU: recorded after its row pass (host path)
    std::mutex mu;                 // one multi-GPU extension at a time
};

namespace {

int nccl_fail(ncclResult_t r, const char* what) {
    return fail(RSM_EDEVICE, "%s: %s", what, ncclGetErrorString(r));
}

// The all-to-all without copies (round 6): the row pass itself stores the cells of the
// column blocks other GPUs own into the per-peer send blocks (CodewordSet::side), and the
// column pass reads the received blocks in place (CodewordSet::blk) -- no pack and no
// unpack pass.  The hooks exist in the single-pass GF(2^16) encoders (k = 129..512) and
// need every wave's 32 cells (two lane halves of 16 elements) in one block: the row and
// column block sizes and k multiples of 32, and the narrow (32-bit offset) addressing.
// Other shapes (GF(2^8), k > 512, small blocks) keep the copy passes.
bool shard_fused_ok(const rsm_ctx* ctx, uint32_t k, uint32_t S, int G) {
    const uint32_t W = 2u * k, rk = k / (uint32_t)G, ck = W / (uint32_t)G;
    return field_bits(k) == 16 && ceil_pow2(k) <= 512 && k % 32u == 0 && rk % 32u == 0 && ck % 32u == 0 &&
           narrow_ok(ctx, k, (uint64_t)W * S, S) && narrow_ok(ctx, k, S, S);
}

// row pass of rows [row0, row0 + nrows) with the side output into `snd` (block h at
// snd + h * blk: the GPU's rows x GPU h's ck columns, row pitch ck * S)
int rows_with_side(rsm_ctx* ctx, uint8_t* d_eds, uint32_t k, uint32_t S, uint32_t row0, uint32_t nrows, uint8_t* snd,
                   uint64_t blk, uint32_t ck, uint32_t self) {
    const uint64_t W = 2ull * k;
    CodewordSet cs{};
    cs.base = d_eds + row0 * W * S;
    cs.cw_stride = W * S;
    cs.elem_stride = S;
    cs.out_offset = (uint64_t)k * S;
    cs.per_square = nrows;
    cs.count = nrows;
    cs.k = k;
    cs.S = S;
    cs.pass = 0;
    cs.side = snd;
    cs.side_blk = blk;
    cs.side_cols = ck;
    cs.side_self = self;
    return launch_encode(ctx, cs, ctx->stream);
}

// column pass of columns [col0, col0 + ncols) whose rows of other GPUs come from the
// received blocks `rcv` (block h at rcv + h * blk: GPU h's rk rows x these columns)
int cols_with_blocks(rsm_ctx* ctx, uint8_t* d_eds, uint32_t k, uint32_t S, uint32_t col0, uint32_t ncols,
                     const uint8_t* rcv, uint64_t blk, uint32_t rk, uint32_t self) {
    const uint64_t W = 2ull * k;
    CodewordSet cs{};
    cs.base = d_eds + col0 * S;
    cs.cw_stride = S;
    cs.elem_stride = W * S;
    cs.out_offset = (uint64_t)k * W * S;
    cs.per_square = ncols;
    cs.count = ncols;
    cs.k = k;
    cs.S = S;
    cs.pass = 1;
    cs.blk = rcv;
    cs.blk_size = blk;
    cs.blk_rows = rk;
    cs.blk_self = self;
    cs.blk_pitch = ncols * S;
    return launch_encode(ctx, cs, ctx->stream);
}

// Steps 1-3 over device-resident squares d_eds[g] (each a full [2k][2k][S] buffer
// on GPU g whose Q0 rows of shard g are valid).  Leaves on GPU g: its rows of the
// top half and its column slice of the whole square (all-gather: the whole top
// half too).
// rows_done (host path): an event per GPU recorded on its stream right after its row
// pass, so the download of its Q1 rows can start on a side stream while the exchange
// and the column pass run.
int extend_sharded(rsm_multi* m, uint8_t* const* d_eds, uint32_t k, uint32_t S, int schedule,
                   const hipEvent_t* rows_done = nullptr) {
    const int G = m->n;
    const size_t W = 2ull * k, row = W * S;
    const uint32_t rk = k / G, ck = (uint32_t)(W / G);
    const size_t blk = (size_t)rk * ck * S;  // all-to-all block: rk rows x ck columns
    // the all-to-all without copies where the encoders have the hooks (shard_fused_ok)
    bool fused = G > 1 && schedule == RSM_SCHED_ALLTOALL;
    for (int g = 0; g < G && fused; ++g) fused = shard_fused_ok(m->ctx[g], k, S, G);  // (per-context limits)
    if (G > 1 && schedule == RSM_SCHED_ALLTOALL) {
        hipError_t e;
        for (int g = 0; g < G; ++g) {
            if (int rc = use_device(m->ctx[g])) return rc;
            if ((e = m->pack[0][g].ensure(blk * G)) != hipSuccess || (e = m->pack[1][g].ensure(blk * G)) != hipSuccess)
                return hip_fail(e, "hipMalloc (all-to-all staging)");
        }
    }
    // 1. row pass (fused all-to-all: each GPU's crossing column blocks straight into its
    //    send staging)
    for (int g = 0; g < G; ++g) {
        if (int rc = use_device(m->ctx[g])) return rc;
        if (fused) {
            if (int rc = rows_with_side(m->ctx[g], static_cast<uint8_t*>(d_eds[g]), k, S, g * rk, rk,
                                        static_cast<uint8_t*>(m->pack[0][g].ptr), blk, ck, (uint32_t)g))
                return rc;
        } else if (int rc = rsm_extend_rows_dev(m->ctx[g], d_eds[g], k, S, g * rk, rk, nullptr)) {
            return rc;
        }
        if (rows_done) {
            if (hipError_t e = hipEventRecord(rows_done[g], m->ctx[g]->stream)) return hip_fail(e, "hipEventRecord");
        }
    }
    // 2. exchange (one GPU: its rows are the whole top half already)
    ncclResult_t r;
    if (G == 1) {
    } else if (schedule == RSM_SCHED_ALLGATHER) {
        if ((r = ncclGroupStart()) != ncclSuccess) return nccl_fail(r, "ncclGroupStart");
        for (int g = 0; g < G; ++g) {
            uint8_t* top = d_eds[g];
            r = ncclAllGather(top + (size_t)g * rk * row, top, (size_t)rk * row, ncclUint8, m->comm[g],
                              m->ctx[g]->stream);
            if (r != ncclSuccess) {
                (void)ncclGroupEnd();
                return nccl_fail(r, "ncclAllGather");
            }
        }
        if ((r = ncclGroupEnd()) != ncclSuccess) return nccl_fail(r, "ncclGroupEnd");
    } else {
        // block (h rows) x (g columns): rk rows x ck*S bytes, packed contiguously -- by the
        // row pass itself (fused) or by a copy pass here
        hipError_t e;
        for (int g = 0; g < G && !fused; ++g) {
            if (int rc = use_device(m->ctx[g])) return rc;
            uint8_t* snd = static_cast<uint8_t*>(m->pack[0][g].ptr);
            const uint8_t* mine = d_eds[g] + (size_t)g * rk * row;
            for (int h = 0; h < G; ++h) {
                if (h == g) continue;  // GPU g's own block stays where its column pass reads it
                if ((e = hipMemcpy2DAsync(snd + h * blk, (size_t)ck * S, mine + (size_t)h * ck * S, row, (size_t)ck * S, rk,
                                          hipMemcpyDeviceToDevice, m->ctx[g]->stream)) != hipSuccess)
                    return hip_fail(e, "all-to-all pack");
            }
        }
        if ((r = ncclGroupStart()) != ncclSuccess) return nccl_fail(r, "ncclGroupStart");
        for (int g = 0; g < G && r == ncclSuccess; ++g) {
            uint8_t* snd = static_cast<uint8_t*>(m->pack[0][g].ptr);
            uint8_t* rcv = static_cast<uint8_t*>(m->pack[1][g].ptr);
            for (int h = 0; h < G && r == ncclSuccess; ++h) {
                if (h == g) continue;
                r = ncclSend(snd + h * blk, blk, ncclUint8, h, m->comm[g], m->ctx[g]->stream);
                if (r == ncclSuccess) r = ncclRecv(rcv + h * blk, blk, ncclUint8, h, m->comm[g], m->ctx[g]->stream);
            }
        }
        ncclResult_t r2 = ncclGroupEnd();
        if (r != ncclSuccess) return nccl_fail(r, "ncclSend/ncclRecv");
        if (r2 != ncclSuccess) return nccl_fail(r2, "ncclGroupEnd");
        for (int g = 0; g < G && !fused; ++g) {
            if (int rc = use_device(m->ctx[g])) return rc;
            const uint8_t* rcv = static_cast<const uint8_t*>(m->pack[1][g].ptr);
            for (int h = 0; h < G; ++h) {
                if (h == g) continue;
                uint8_t* dst = d_eds[g] + (size_t)h * rk * row + (size_t)g * ck * S;
                if ((e = hipMemcpy2DAsync(dst, row, rcv + h * blk, (size_t)ck * S, (size_t)ck * S, rk,
                                          hipMemcpyDeviceToDevice, m->ctx[g]->stream)) != hipSuccess)
                    return hip_fail(e, "all-to-all unpack");
            }
        }
    }
    // 3. column pass of each GPU's column slice (fused all-to-all: the other GPUs' rows read
    //    in place from the receive staging; the square's top half then holds only this
    //    GPU's rows)
    for (int g = 0; g < G; ++g) {
        if (int rc = use_device(m->ctx[g])) return rc;
        if (fused) {
            if (int rc = cols_with_blocks(m->ctx[g], static_cast<uint8_t*>(d_eds[g]), k, S, g * ck, ck,
                                          static_cast<const uint8_t*>(m->pack[1][g].ptr), blk, rk, (uint32_t)g))
                return rc;
        } else if (int rc = rsm_extend_cols_dev(m->ctx[g], d_eds[g], k, S, g * ck, ck, nullptr)) {
            return rc;
        }
    }
    return RSM_OK;
}

int check_shape(const rsm_multi* m, uint32_t k, uint32_t S, int schedule) {
    if (int rc = validate_chunk_size(S)) return rc;
    if (k == 0 || k % m->n != 0) return fail(RSM_ESHAPE, "k=%u must be a positive multiple of the GPU count %d", k, m->n);
    if (schedule != RSM_SCHED_ALLGATHER && schedule != RSM_SCHED_ALLTOALL)
        return fail(RSM_EINVAL, "unknown multi-GPU schedule %d", schedule);
    return RSM_OK;
}

// One square from host memory over the clique: GPU g uploads its Q0 rows (from `ods`
// with row pitch `opitch`), the sharded extension runs, GPU g downloads its rows of Q1
// (side stream, behind its row pass) and its column slice of the bottom half [Q2|Q3]
// (its stream, behind its column pass) into `eds`.  Q0 of `eds` is not written.  With
// pinned host buffers every copy is a DMA of the GPU's copy engines; caller holds m->mu.
int host_extend(rsm_multi* m, const uint8_t* ods, size_t opitch, uint8_t* eds, uint32_t k, uint32_t share_size,
                int schedule) {
    const int G = m->n;
    const size_t S = share_size, W = 2ull * k, row = W * S, half = (size_t)k * S;
    const uint32_t rk = k / G, ck = (uint32_t)(W / G);
    std::vector<uint8_t*> d(G);
    hipError_t e;
    for (int g = 0; g < G; ++g) {
        if (int rc = use_device(m->ctx[g])) return rc;
        if ((e = m->eds[g].ensure(W * W * S)) != hipSuccess) return hip_fail(e, "hipMalloc (sharded square)");
        d[g] = static_cast<uint8_t*>(m->eds[g].ptr);
        const size_t r0 = (size_t)g * rk;
        if ((e = hipMemcpy2DAsync(d[g] + r0 * row, row, ods + r0 * opitch, opitch, half, rk, hipMemcpyHostToDevice,
                                  m->ctx[g]->stream)) != hipSuccess)
            return hip_fail(e, "H2D (Q0 rows)");
    }
    if (int rc = extend_sharded(m, d.data(), k, share_size, schedule, m->rows_done.data())) return rc;
    for (int g = 0; g < G; ++g) {
        if (int rc = use_device(m->ctx[g])) return rc;
        const size_t r0 = (size_t)g * rk;
        if ((e = hipStreamWaitEvent(m->side[g], m->rows_done[g], 0)) != hipSuccess ||
            (e = hipMemcpy2DAsync(eds + r0 * row + half, row, d[g] + r0 * row + half, row, half, rk,
                                  hipMemcpyDeviceToHost, m->side[g])) != hipSuccess)
            return hip_fail(e, "D2H (Q1 rows)");
        const size_t c0 = (size_t)g * ck * S;
        if ((e = hipMemcpy2DAsync(eds + (size_t)k * row + c0, row, d[g] + (size_t)k * row + c0, row, (size_t)ck * S, k,
                                  hipMemcpyDeviceToHost, m->ctx[g]->stream)) != hipSuccess)
            return hip_fail(e, "D2H (bottom-half columns)");
    }
    return RSM_OK;
}

int sync_all(rsm_multi* m) {
    for (int g = 0; g < m->n; ++g) {
        if (int rc = rsm_sync(m->ctx[g])) return rc;
        if (int rc = use_device(m->ctx[g])) return rc;
        if (hipError_t e = hipStreamSynchronize(m->side[g])) return hip_fail(e, "hipStreamSynchronize (side)");
    }
    return RSM_OK;
}

}  // namespace

extern "C" {

int rsm_multi_create(const int* devices, int n, rsm_multi** out) {
    if (!devices || n <= 0 || !out) return fail(RSM_EINVAL, "rsm_multi_create: bad arguments");
    *out = nullptr;
    auto* m = new (std::nothrow) rsm_multi();
    if (!m) return fail(RSM_ENOMEM, "rsm_multi_create: out of memory");
    m->n = n;
    m->ctx.assign(n, nullptr);
    for (int g = 0; g < n; ++g)
        if (int rc = rsm_ctx_create(devices[g], &m->ctx[g])) {
            rsm_multi_destroy(m);
            return rc;
        }
    m->comm.assign(n, nullptr);
    ncclResult_t r = ncclCommInitAll(m->comm.data(), n, devices);
    if (r != ncclSuccess) {
        m->comm.clear();
        rsm_multi_destroy(m);
        return nccl_fail(r, "ncclCommInitAll");
    }
    m->eds = std::vector<DevBuf>(n);
    m->pack[0] = std::vector<DevBuf>(n);
    m->pack[1] = std::vector<DevBuf>(n);
    m->side.assign(n, nullptr);
    m->rows_done.assign(n, nullptr);
    for (int g = 0; g < n; ++g) {
        hipError_t e;
        if (int rc = use_device(m->ctx[g])) {
            rsm_multi_destroy(m);
            return rc;
        }
        if ((e = hipStreamCreateWithFlags(&m->side[g], hipStreamNonBlocking)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&m->rows_done[g], hipEventDisableTiming)) != hipSuccess) {
            rsm_multi_destroy(m);
            return hip_fail(e, "rsm_multi_create: side stream / event");
        }
    }
    *out = m;
    return RSM_OK;
}

void rsm_multi_destroy(rsm_multi* m) {
    if (!m) return;
    for (auto* c : m->ctx)
        if (c) {
            (void)hipSetDevice(c->device);
            (void)hipDeviceSynchronize();
        }
    for (auto& c : m->comm)
        if (c) (void)ncclCommDestroy(c);
    auto drop = [](DevBuf& b) {
        if (b.ptr) (void)hipFree(b.ptr);
        b.ptr = nullptr;
        b.cap = 0;
    };
    for (size_t g = 0; g < m->eds.size(); ++g) {  // freed with their own device current
        (void)hipSetDevice(m->ctx[g]->device);
        drop(m->eds[g]);
        drop(m->pack[0][g]);
        drop(m->pack[1][g]);
        if (g < m->side.size() && m->side[g]) {
            (void)hipStreamSynchronize(m->side[g]);
            (void)hipStreamDestroy(m->side[g]);
        }
        if (g < m->rows_done.size() && m->rows_done[g]) (void)hipEventDestroy(m->rows_done[g]);
    }
    for (auto* c : m->ctx)
        if (c) rsm_ctx_destroy(c);
    delete m;
}

int rsm_multi_size(const rsm_multi* m) { return m ? m->n : 0; }

rsm_ctx* rsm_multi_context(rsm_multi* m, int i) { return (m && i >= 0 && i < m->n) ? m->ctx[i] : nullptr; }

int rsm_multi_extend_dev(rsm_multi* m, void* const* d_eds, uint32_t k, uint32_t share_size, int schedule) {
    if (!m || !d_eds) return fail(RSM_EINVAL, "rsm_multi_extend_dev: bad arguments");
    if (int rc = check_shape(m, k, share_size, schedule)) return rc;
    std::lock_guard<std::mutex> lk(m->mu);
    std::vector<uint8_t*> p(m->n);
    for (int g = 0; g < m->n; ++g) p[g] = static_cast<uint8_t*>(d_eds[g]);
    return extend_sharded(m, p.data(), k, share_size, schedule);
}

int rsm_multi_sync(rsm_multi* m) {
    if (!m) return fail(RSM_EINVAL, "rsm_multi_sync: NULL");
    return sync_all(m);
}

int rsm_multi_host_alloc(rsm_multi* m, uint64_t bytes, void** out) {
    if (!m || !out) return fail(RSM_EINVAL, "rsm_multi_host_alloc: bad arguments");
    *out = nullptr;
    if (int rc = use_device(m->ctx[0])) return rc;
    // portable: pinned for (and DMA-able by) every GPU of the clique, not just GPU 0
    hipError_t e = hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocPortable);
    return e == hipSuccess ? RSM_OK : hip_fail(e, "hipHostMalloc (portable)");
}

int rsm_multi_host_free(rsm_multi* m, void* p) {
    if (!m) return fail(RSM_EINVAL, "rsm_multi_host_free: NULL");
    if (!p) return RSM_OK;
    hipError_t e = hipHostFree(p);
    return e == hipSuccess ? RSM_OK : hip_fail(e, "hipHostFree");
}

// ComputeExtendedDataSquare of one square from host memory over all GPUs: GPU g
// uploads its Q0 rows, the sharded extension runs, and each GPU downloads its
// rows of Q1 and its column slice of the bottom half [Q2|Q3]; Q0 is filled from
// the host ODS.
int rsm_multi_extend_square(rsm_multi* m, const uint8_t* ods, uint32_t k, uint32_t share_size, uint8_t* eds,
                            int schedule) {
    if (!m || !ods || !eds) return fail(RSM_EINVAL, "rsm_multi_extend_square: bad arguments");
    if (int rc = check_shape(m, k, share_size, schedule)) return rc;
    std::lock_guard<std::mutex> lk(m->mu);
    const size_t S = share_size, row = 2ull * k * S, half = (size_t)k * S;
    if (int rc = host_extend(m, ods, half, eds, k, share_size, schedule)) {
        (void)sync_all(m);  // no copy may still target the caller's buffers
        return rc;
    }
    for (uint32_t r = 0; r < k; ++r) memcpy(eds + r * row, ods + r * half, half);  // Q0 (host, beside the GPUs)
    return sync_all(m);
}

int rsm_multi_extend_square_inplace(rsm_multi* m, uint8_t* eds, uint32_t k, uint32_t share_size, int schedule) {
    if (!m || !eds) return fail(RSM_EINVAL, "rsm_multi_extend_square_inplace: bad arguments");
    if (int rc = check_shape(m, k, share_size, schedule)) return rc;
    std::lock_guard<std::mutex> lk(m->mu);
    int rc = host_extend(m, eds, 2ull * k * share_size, eds, k, share_size, schedule);
    const int rs = sync_all(m);
    return rc ? rc : rs;
}

#ifdef RSM_DIAG
// Diagnostic / test hook: the copy-free all-to-all of extend_sharded with G "GPUs" on ONE
// device (a context), so the encoders' side output and blocked inputs run on the hardware
// without a multi-GPU node: rank g's row pass stores its crossing column blocks into its
// send staging, device copies stand in for the RCCL send/recv, and rank g's column pass
// reads the received blocks in place.  d_eds[g]: rank g's full square buffer (Q0 rows of
// shard g valid).  Synchronous.
int rsm_diag_alltoall_emulated(rsm_ctx* ctx, void* const* d_eds, int G, uint32_t k, uint32_t share_size) {
    if (!ctx || !d_eds || G <= 1 || k == 0 || k % (uint32_t)G != 0)
        return fail(RSM_EINVAL, "rsm_diag_alltoall_emulated: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (!shard_fused_ok(ctx, k, share_size, G)) return fail(RSM_EUNSUPPORTED, "rsm_diag_alltoall_emulated: shape");
    if (int rc = use_device(ctx)) return rc;
    const uint64_t S = share_size, W = 2ull * k;
    const uint32_t rk = k / G, ck = (uint32_t)(W / G);
    const uint64_t blk = (uint64_t)rk * ck * S;
    void *snd = nullptr, *rcv = nullptr;
    hipError_t e;
    if ((e = hipMalloc(&snd, blk * G * G)) != hipSuccess) return hip_fail(e, "hipMalloc (emulated send staging)");
    if ((e = hipMalloc(&rcv, blk * G * G)) != hipSuccess) {
        (void)hipFree(snd);
        return hip_fail(e, "hipMalloc (emulated receive staging)");
    }
    uint8_t* sb = static_cast<uint8_t*>(snd);
    uint8_t* rb = static_cast<uint8_t*>(rcv);
    int rc = RSM_OK;
    for (int g = 0; g < G && rc == RSM_OK; ++g)
        rc = rows_with_side(ctx, static_cast<uint8_t*>(d_eds[g]), k, share_size, g * rk, rk, sb + (uint64_t)g * G * blk, blk, ck,
                            (uint32_t)g);
    for (int g = 0; g < G && rc == RSM_OK; ++g)  // "GPU g sends its block h to GPU h"
        for (int h = 0; h < G && rc == RSM_OK; ++h)
            if (h != g && (e = hipMemcpyAsync(rb + ((uint64_t)h * G + g) * blk, sb + ((uint64_t)g * G + h) * blk, blk,
                                              hipMemcpyDeviceToDevice, ctx->stream)) != hipSuccess)
                rc = hip_fail(e, "emulated exchange");
    for (int g = 0; g < G && rc == RSM_OK; ++g)
        rc = cols_with_blocks(ctx, static_cast<uint8_t*>(d_eds[g]), k, share_size, g * ck, ck, rb + (uint64_t)g * G * blk,
                              blk, rk, (uint32_t)g);
    if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess && rc == RSM_OK) rc = hip_fail(e, "hipStreamSynchronize");
    (void)hipFree(snd);
    (void)hipFree(rcv);
    return rc;
}
#endif

}  // extern "C"
