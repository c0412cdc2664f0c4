// rsm_diag.cpp -- entry points of the DIAGNOSTIC library only (librsmt2d_hip_diag.so,
// `make diag`, compiled with -DRSM_DIAG).  Nothing here is part of the product
// library: the A/B kernel variants (no-arithmetic / no-memory modes give wrong
// output by design), the fused single-launch extension and the software-pipelined
// dual launch were measured no faster than the production two-launch schedule
//  and stay available for measurements.
#ifndef RSM_DIAG
#error "rsm_diag.cpp belongs to the diagnostic build (-DRSM_DIAG)"
#endif
#include "../../include/rsmt2d_hip_diag.h"
#include "rsm_internal.hpp"

using namespace rsm;

namespace {

[[maybe_unused]] CodewordSet rows_of(uint8_t* d_eds, uint32_t k, uint32_t S, uint32_t count, uint32_t grid) {
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
    rows.grid = grid;
    return rows;
}

CodewordSet cols_of(uint8_t* d_eds, uint32_t k, uint32_t S, uint32_t count, uint32_t grid) {
    CodewordSet cols = rows_of(d_eds, k, S, count, grid);
    const uint64_t W = 2ull * k;
    cols.cw_stride = S;
    cols.elem_stride = W * S;
    cols.out_offset = (uint64_t)k * W * S;
    cols.per_square = (uint32_t)W;
    cols.count = (uint32_t)W * count;
    cols.pass = 1;
    return cols;
}

}  // namespace

extern "C" {

int rsm_diag_set_bs_mode(int mode, int rev_col, int xcd) {
    set_bs128_diag_mode(mode, rev_col, xcd);
    return RSM_OK;
}

int rsm_diag_set_trace(void* d_trace) {
    set_bs128_diag_trace(static_cast<uint32_t*>(d_trace));
    return RSM_OK;
}

int rsm_diag_set_split_waves(int first, int second) {
    auto ok = [](int n) { return n == 0 || n == 2 || n == 4 || n == 8 || n == 16; };  // 0: production choice
    if (!ok(first) || !ok(second)) return RSM_EINVAL;
    set_split_diag_waves(first, second);
    return RSM_OK;
}

int rsm_diag_set_split_fused(int on) {
    set_split_diag_fused(on != 0);
    return RSM_OK;
}

int rsm_diag_set_enc16_e64(int mode) {
    set_enc16_diag_e64(mode);
    return RSM_OK;
}

int rsm_diag_set_dec16_five_pass(int on) {
    set_dec16_diag_five_pass(on != 0);
    return RSM_OK;
}

int rsm_diag_set_dec_trace(void* d_trace) {
    set_dec_diag_trace(static_cast<uint32_t*>(d_trace));
    return RSM_OK;
}

int rsm_diag_set_dec16_mode(uint32_t mode) {
    set_dec16_diag_mode(mode);
    return RSM_OK;
}

int rsm_diag_set_dec_delay(uint32_t ticks) {
    set_dec_diag_delay(ticks);
    return RSM_OK;
}

int rsm_diag_set_dec8_mode(uint32_t mode) {
    set_dec8_diag_mode(mode);
    return RSM_OK;
}

int rsm_diag_set_codec_spin(uint32_t us) {
    set_codec_spin_diag(us);
    return RSM_OK;
}

int rsm_diag_set_repair_mode(uint32_t mode) {
    set_repair_diag_mode(mode);
    return RSM_OK;
}

int rsm_diag_set_bs_row_mode(int mode) {
    set_bs128_diag_row_mode(mode);
    return RSM_OK;
}

// Both passes of `count` in-place k = 128 squares as ONE persistent launch
// (extend_gf8_bs128q_kernel, the kernel variant chosen by rsm_diag_set_bs_mode):
// `delay` squares of row sets lead the Q0-column sets.  Asynchronous on `stream`;
// rsm_diag_queue_check reports a stuck wait.
int rsm_diag_extend_fused(rsm_ctx* ctx, void* d_eds, uint32_t k, uint32_t share_size, uint32_t count, uint32_t delay,
                          void* stream) {
    if (!ctx || !d_eds || k != 128 || validate_chunk_size(share_size) != RSM_OK ||
        ((uint64_t)k * share_size) % 2048 != 0)
        return fail(RSM_EINVAL, "rsm_diag_extend_fused: needs k = 128 and k * S a multiple of 2 KiB");
    if (count == 0) return RSM_OK;
    if (int rc = use_device(ctx)) return rc;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    // delay bits 0-7: squares; bits 8-15 (if non-zero): the Q1 claim margin + 1
    const uint32_t m = (delay >> 8) & 0xFFu;
    const int rc = extend_squares_queue(ctx, static_cast<uint8_t*>(d_eds), k, share_size, count, st, delay & 0xFFu,
                                        m ? m - 1 : ~0u);
    return rc == RSM_EUNSUPPORTED ? fail(rc, "queue extension not applicable") : rc;
}

// Waits for `stream` and reports (and clears) a stuck wait of its queue launches.
int rsm_diag_queue_check(rsm_ctx* ctx, void* stream) {
    if (!ctx) return fail(RSM_EINVAL, "rsm_diag_queue_check: bad arguments");
    if (int rc = use_device(ctx)) return rc;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    return check_queue_reports(ctx, st);
}

// ONE launch running the row pass of the squares at d_rows_eds and the column pass
// of the squares at d_cols_eds (either may be NULL; the batches must not overlap).
int rsm_diag_extend_pipeline_dev(rsm_ctx* ctx, void* d_rows_eds, void* d_cols_eds, uint32_t k, uint32_t share_size,
                                 uint32_t count, void* stream) {
    if (!ctx || k == 0 || (!d_rows_eds && !d_cols_eds)) return fail(RSM_EINVAL, "rsm_diag_extend_pipeline_dev: bad arguments");
    if (int rc = validate_chunk_size(share_size)) return rc;
    if (count == 0) return RSM_OK;
    if (int rc = use_device(ctx)) return rc;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    const CodewordSet rows = rows_of(static_cast<uint8_t*>(d_rows_eds), k, share_size, count, ctx->cus);
    const CodewordSet cols = cols_of(static_cast<uint8_t*>(d_cols_eds), k, share_size, count, ctx->cus);
    const bool dual = field_bits(k) == 8 && d_rows_eds && d_cols_eds && bs128_applicable(rows) && bs128_applicable(cols);
    if (!dual) {
        if (d_rows_eds)
            if (int rc = extend_squares(ctx, static_cast<uint8_t*>(d_rows_eds), k, share_size, count, st, 1)) return rc;
        if (d_cols_eds)
            if (int rc = extend_squares(ctx, static_cast<uint8_t*>(d_cols_eds), k, share_size, count, st, 2)) return rc;
        return RSM_OK;
    }
    DualPlan p{};
    p.a = rows;
    p.b = cols;
    p.na = (uint32_t)(((uint64_t)rows.count * share_size + 2047) / 2048);
    p.nb = (uint32_t)(((uint64_t)cols.count * share_size + 2047) / 2048);
    hipError_t e = launch_encode_gf8_bs128_dual(p, st);
    return e == hipSuccess ? RSM_OK : hip_fail(e, "pipelined extension kernel launch");
}

}  // extern "C"
