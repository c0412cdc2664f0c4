/*
 * rsmt2d_hip_diag.h -- entry points of the DIAGNOSTIC library
 * (rsmt2d_amd/librsmt2d_hip_diag.so, built by `make -C rsmt2d_amd/csrc diag` with
 * -DRSM_DIAG).  Measurement tooling only: the product library
 * (librsmt2d_hip.so, include/rsmt2d_hip.h) contains none of these kernels or
 * switches, and no environment variable changes its results.
 */
#ifndef RSMT2D_HIP_DIAG_H
#define RSMT2D_HIP_DIAG_H

#include "rsmt2d_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Kernel variant of the bit-sliced GF(2^8) M = 128 encode, process-wide:
 * 40 = production; 0 / 8 / 24 / 56 = A-B variants (exchange form, cache policy);
 * 2 = no arithmetic, 4 = no global memory (both give WRONG output by design).
 * rev_col: column pass in reverse set order; xcd: bit 0 rows / bit 1 columns in
 * XCD-grouped set order. */
int rsm_diag_set_bs_mode(int mode, int rev_col, int xcd);
/* Kernel variant of the row pass alone (same codes; the setting above then applies
 * to every other launch). */
int rsm_diag_set_bs_row_mode(int mode);
/* Phase timeline of the half-split queue kernel's trace modes (51010/51012/51014):
 * d_trace = device buffer of 256 workgroups x 256 sets x 12 words (NULL: off). */
int rsm_diag_set_trace(void* d_trace);
/* Phase stamps of the M = 128 split decoder: 8 words (s_memrealtime, 100 MHz) per
 * workgroup of every following GF(2^8) decode launch; NULL = off. */
int rsm_diag_set_dec_trace(void* d_trace);
/* Waves per (codeword, 256-B chunk) of the two launches of the latency-form extension
 * (2, 4, 8 or 16 each; 0 = the production choice: 16 for one square, 8 for batches). */
int rsm_diag_set_split_waves(int first, int second);
/* One square in the latency form: 1 = one launch with a device-side wait (A/B only:
 * slower), 0 = two launches (production). */
int rsm_diag_set_split_fused(int on);
/* GF(2^16) encoder form (m = 512): 0 = production (the half-wave form, enc16h512_kernel,
 * just-in-time tables), 1 = 8 waves x 64 elements, 2 = the round-3 16-wave form (scalar
 * tables), 3 = form 2 with the half exchange buffer, 4 = 16 waves x 32 elements,
 * persistent, LDS tables beside a half exchange buffer, 5 = form 4 with just-in-time
 * table reads, 8 / 9 = forms 4 / 5 with the merged middle pair, 16 = the half-wave form
 * with compiler-scheduled table reads.  m = 256: 6 = 16 waves x 16 elements, 7 = 8 waves
 * x 32 elements, 14 = the half-wave form with compiler-scheduled reads, 19 = the half-wave
 * form prefetching the next task's points, 20 = the half-wave form with three workgroups per
 * CU (quarter-lane exchange passes, 49 KiB of LDS, 80 registers), any other value the
 * production half-wave form. */
int rsm_diag_set_enc16_e64(int mode);
/* GF(2^16) m = 256 / 512 decoders: 1 = the five global passes (A/B), 0 = the single-pass kernels
 * (production: dec16f_kernel for m = 256, the half-wave dec16h_kernel for m = 512). */
int rsm_diag_set_dec16_five_pass(int on);
/* GF(2^16) m = 512 half-wave decoder A/B bits (wrong output by design): 1 = no scale /
 * reveal table staging, 2 = no point loads; 0 = production. */
int rsm_diag_set_dec16_mode(uint32_t mode);
/* GF(2^8) split decoder A/B: the upper half of the grid delays its point loads by
 * `ticks` of the 100 MHz s_memrealtime clock (0 = off, production). */
int rsm_diag_set_dec_delay(uint32_t ticks);
/* GF(2^8) split decoder A/B: 1 = the other error-locator form than production (every
 * wave computing the locator itself with scalar-loaded tables, or wave 0 staging the
 * per-point tables in LDS for all waves; production takes the first for launches of at
 * most 64 tasks, the second for larger ones); 2 = the setup-free floor of a pre-pass design
 * (no presence loads and no error locator in the kernel: a zero locator and every other
 * point present -- wrong output, timing only); 0 = production. */
int rsm_diag_set_dec8_mode(uint32_t mode);
/* Codec calls (rsm_encode / rsm_decode) spin on hipStreamQuery for up to `us`
 * microseconds before blocking in hipStreamSynchronize (0: block at once, production). */
int rsm_diag_set_codec_spin(uint32_t us);
/* Zero-copy Repair A/B: 1 = the sweep as two launches (top half, then bottom half; the
 * column re-encode of the top half overlapping the bottom sweep); 0 = production (one
 * sweep launch over all rows, the re-encode behind it). */
int rsm_diag_set_repair_mode(uint32_t mode);
/* Both passes of `count` in-place k = 128 squares in ONE persistent launch
 * (extend_gf8_bs128q_kernel: row and Q0-column sets from one queue, Q1-column sets
 * from a ready list; `delay` squares of row sets lead the Q0-column sets).
 * Asynchronous on `stream`. */
int rsm_diag_extend_fused(rsm_ctx* ctx, void* d_eds, uint32_t k, uint32_t share_size, uint32_t count, uint32_t delay,
                          void* stream);
/* Reads and clears the stuck-wait word of the queue launches on `stream`:
 * RSM_EDEVICE if one timed out since the last check (its output is invalid). */
int rsm_diag_queue_check(rsm_ctx* ctx, void* stream);
/* ONE launch running the row pass of the squares at d_rows_eds and the column pass
 * of the squares at d_cols_eds (encode_gf8_bs128p_kernel); either may be NULL. */
int rsm_diag_extend_pipeline_dev(rsm_ctx* ctx, void* d_rows_eds, void* d_cols_eds, uint32_t k, uint32_t share_size,
                                 uint32_t count, void* stream);

/* The copy-free multi-GPU all-to-all (rsm_multi_extend_dev, RSM_SCHED_ALLTOALL, GF(2^16)
 * shapes whose row and column blocks are multiples of 32) with G "GPUs" emulated on ONE
 * context: rank g's row pass with the encoder's side output into its send staging, device
 * copies in place of the RCCL send/recv, rank g's column pass reading the received blocks
 * in place.  d_eds[g] is rank g's [2k][2k][S] buffer holding the Q0 rows of shard g;
 * afterwards it holds shard g's rows of the top half and the bottom half of its column
 * slice.  Synchronous. */
int rsm_diag_alltoall_emulated(rsm_ctx* ctx, void* const* d_eds, int G, uint32_t k, uint32_t share_size);

#ifdef __cplusplus
}
#endif
#endif /* RSMT2D_HIP_DIAG_H */
