/*
 * rsmt2d_hip.h -- C ABI of the MI355X-native 2D Reed-Solomon EDS engine.
 *
 * Drop-in boundary for celestiaorg/rsmt2d's hot path: the Codec plugin
 * (codecs.go:14-30, implemented by LeoRSCodec in leopard.go:16-103) and the
 * two-dimensional schedule / crossword solver built on it
 * (extendeddatasquare.go:50-243, extendeddatacrossword.go:74-502).
 * Everything is plain pointers and sizes so a cgo shim can bind
 * it directly; no call ever aborts or throws across the ABI.
 *
 * Return codes: 0 on success, a negative RSM_E* code on failure;
 * rsm_last_error() gives a thread-local human-readable message.
 */
#ifndef RSMT2D_HIP_H
#define RSMT2D_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RSM_OK 0
#define RSM_EINVAL (-1)        /* bad argument */
#define RSM_ESHARESIZE (-2)    /* share size not a multiple of 64 (leopard.go:92-99) */
#define RSM_ETOOFEW (-3)       /* Decode: fewer than k of 2k shares present */
#define RSM_ESHAPE (-4)        /* non-square count, uneven shares, odd EDS width, > MaxChunks */
#define RSM_EDEVICE (-5)       /* HIP runtime failure / no GPU: never a silent CPU fallback */
#define RSM_ENOMEM (-6)
#define RSM_EUNSUPPORTED (-7)  /* configuration this build does not implement (2k > 65536,
                                   as klauspost rejects it; device roots beyond their widths) */
#define RSM_EUNREPAIRABLE (-8) /* ErrUnrepairableDataSquare (extendeddatacrossword.go:37) */
#define RSM_EBYZANTINE (-9)    /* ErrByzantineData (extendeddatacrossword.go:42-58) */
#define RSM_ECELL (-10)        /* SetCell on a non-nil cell or wrong size (datasquare.go:341-353) */
#define RSM_ETREE (-11)        /* tree callback error / root of an incomplete vector */

#define RSM_AXIS_ROW 0 /* rsmt2d.Row (extendeddatacrossword.go:15-18) */
#define RSM_AXIS_COL 1 /* rsmt2d.Col */

typedef struct rsm_ctx rsm_ctx;
typedef struct rsm_eds rsm_eds;

/* ---- context --------------------------------------------------------------- */
/* One context per GPU (device ordinal).  Thread-safe: rsmt2d calls the Codec from
 * up to 2k goroutines at once (extendeddatasquare.go:186-224); each Codec /
 * host-memory call takes its own stream and staging buffers from the context's
 * pool (up to 32 in flight, further callers wait), device scratch belongs to the
 * stream it is used on, and every call selects the context's device on the
 * calling thread (cgo moves goroutines between OS threads). */
int rsm_ctx_create(int device, rsm_ctx** out);
void rsm_ctx_destroy(rsm_ctx* ctx);
int rsm_ctx_device(const rsm_ctx* ctx);
/* Throughput tuning for several extensions in flight on different streams: cap the
 * persistent grid (CUs) of this context's GF(2^8) M = 128 row pass (pass 0) or
 * column pass (pass 1); the single-launch queue extension (both passes) takes the
 * pass-0 cap; 0 = all CUs (default).  *previous (may be NULL) receives the old cap.
 * Results never depend on it. */
int rsm_ctx_set_pass_grid(rsm_ctx* ctx, int pass, int cus, int* previous);
/* Latency tuning: GF(2^8) extensions of up to `squares` squares per call with
 * 65 <= k <= 128 run in the latency form (two launches of the split byte-table
 * encoder over every CU) instead of the single queue-driven launch; 0 = always the
 * queue launch.  Default 12.  With 9 <= k <= 64 the latency form takes up to
 * max(squares, 64) squares per call (0: never) instead of the one-wave-per-codeword
 * byte-table passes.  *previous (may be NULL) receives the old value.  Results
 * never depend on it. */
int rsm_ctx_set_split_max(rsm_ctx* ctx, int squares, int* previous);
/* Test hook: the single-pass kernels address each half of a codeword with 32-bit
 * offsets, so codewords whose halves span more than offset_limit bytes (default 2^31:
 * columns of squares over 4 GiB) run on the wide forms (64-bit per-symbol bases), and
 * GF(2^16) work arrays get at most work_budget bytes per stream (default 1 GiB; wider
 * shares run as byte slabs).  Lowering them sends small shapes down those paths so
 * their parity can be tested without 4 GiB squares; 0 restores a default.  Results
 * never depend on them. */
int rsm_ctx_set_limits(rsm_ctx* ctx, uint64_t offset_limit, uint64_t work_budget);
const char* rsm_last_error(void);
const char* rsm_version(void);
int rsm_device_count(void);

/* ---- Codec (codecs.go:14-30; LeoRSCodec leopard.go:16-103) ------------------- */
/* Name() -- "Leopard" (codecs.go:11): EDS.Equals and JSON compare codec names. */
const char* rsm_codec_name(void);
/* MaxChunks() -- 32768 * 32768 (leopard.go:76-84). */
int64_t rsm_codec_max_chunks(void);
/* ValidateChunkSize(shareSize) -- RSM_ESHARESIZE unless a multiple of 64. */
int rsm_codec_validate_chunk_size(int64_t share_size);
/* 8 when 2k <= 256 (GF(2^8)), else 16 (GF(2^16)) -- codecs.go:6-10. */
int rsm_codec_field_bits(uint32_t k);
/* Encode(data) (leopard.go:28-45): k complete shares of share_size bytes in host
 * memory -> k parity shares written to parity[0..k). */
int rsm_encode(rsm_ctx* ctx, const uint8_t* const* data, uint32_t k, uint32_t share_size,
               uint8_t* const* parity);
/* Decode(data) (leopard.go:51-59, klauspost Reconstruct): n = 2k slots; slot i is
 * present iff present[i] != 0; every missing slot's buffer shares[i] (caller
 * allocated, share_size bytes) is filled.  RSM_ETOOFEW if fewer than k present;
 * all present is a no-op. */
int rsm_decode(rsm_ctx* ctx, uint8_t* const* shares, const uint8_t* present, uint32_t n,
               uint32_t share_size);

/* ---- batched 2D extension (erasureExtendSquare, extendeddatasquare.go:154-227) -- */
/* Host memory: ods = k*k shares row-major, eds = (2k)^2 shares row-major.  Only
 * Q1, Q2, Q3 cross PCIe back; Q0 of eds is filled from ods on the host. */
int rsm_extend_square(rsm_ctx* ctx, const uint8_t* ods, uint32_t k, uint32_t share_size,
                      uint8_t* eds);
/* Host memory, in place: the top-left quadrant of eds already holds the ODS (the
 * cgo shim gathers the [][]byte shares straight into a pinned EDS arena from
 * rsm_host_alloc); Q1..Q3 are written around it. */
int rsm_extend_square_inplace_host(rsm_ctx* ctx, uint8_t* eds, uint32_t k, uint32_t share_size);
/* Host memory, `count` consecutive squares (ods: [count][k][k][S], eds:
 * [count][2k][2k][S]): H2D, extension and D2H of different squares overlap on
 * three streams.  Pinned buffers (rsm_host_alloc) make every copy an async DMA. */
int rsm_extend_squares_host(rsm_ctx* ctx, const uint8_t* ods, uint32_t k, uint32_t share_size, uint32_t count,
                            uint8_t* eds);
/* Pinned (page-locked) host memory for the arenas above. */
int rsm_host_alloc(rsm_ctx* ctx, uint64_t bytes, void** out);
int rsm_host_free(rsm_ctx* ctx, void* p);
/* Device-resident, in place: d_eds holds `count` consecutive [2k][2k][S] squares
 * whose top-left quadrant already holds the ODS (the EDS aliases the ODS, as in
 * ComputeExtendedDataSquare).  Enqueued on `stream` (a hipStream_t of this
 * library's HIP runtime; NULL = the context stream); asynchronous.  With
 * 65 <= k <= 128, batches of more than rsm_ctx_set_split_max squares run both passes
 * as ONE queue-driven launch, smaller batches (a single square included) as two
 * latency-form launches over every CU.  The queue launch's bounded waits cannot time
 * out short of a hardware fault, and if one did, the stream's next rsm_stream_check
 * (rsm_sync for the context stream), its rsm_stream_destroy or the next extension on
 * that stream returns RSM_EDEVICE. */
int rsm_extend_squares_dev(rsm_ctx* ctx, void* d_eds, uint32_t k, uint32_t share_size, uint32_t count,
                           void* stream);
/* One phase of the above: phase 1 = row pass (Q0 -> Q1), phase 2 = column pass
 * ([Q0|Q1] -> [Q2|Q3]), 3 = both; for per-kernel timing/profiling.  Asynchronous. */
int rsm_extend_squares_phase_dev(rsm_ctx* ctx, void* d_eds, uint32_t k, uint32_t share_size,
                                 uint32_t count, int phase, void* stream);
/* Rows [row0, row0+nrows) / columns [col0, col0+ncols) of one in-place
 * [2k][2k][S] square: the per-GPU units of the row-sharded multi-GPU schedule
 * (rows of the top half on each GPU, an all-gather of [Q0|Q1], then each GPU's
 * column slice).  Asynchronous on `stream` (NULL = context stream). */
int rsm_extend_rows_dev(rsm_ctx* ctx, void* d_eds, uint32_t k, uint32_t share_size, uint32_t row0,
                        uint32_t nrows, void* stream);
int rsm_extend_cols_dev(rsm_ctx* ctx, void* d_eds, uint32_t k, uint32_t share_size, uint32_t col0,
                        uint32_t ncols, void* stream);
/* The row pass of rows [row0, row0+nrows) (as rsm_extend_rows_dev) that also leaves the
 * extended rows split into `nblocks` column blocks of 2k/nblocks columns each: block h
 * at d_blocks + h*nrows*(2k/nblocks)*S, row pitch (2k/nblocks)*S -- the send buffer of
 * the all-to-all multi-GPU schedule (rank h receives block h), with no copy pass where the
 * encoder stores the blocks itself (GF(2^16), k <= 512, k and the block width multiples
 * of 32; other shapes: the row pass, then strided device copies).  Asynchronous. */
int rsm_extend_rows_blocks_dev(rsm_ctx* ctx, void* d_eds, uint32_t k, uint32_t share_size, uint32_t row0,
                               uint32_t nrows, void* d_blocks, uint32_t nblocks, void* stream);
/* Generic device batch of `count` codewords (k data shares -> k parity shares each,
 * the Encode of leopard.go:28-45 for every codeword): data share e of codeword q is
 * at d_in + q*cw_stride + e*share_stride, its parity share e is written at
 * d_out + q*cw_stride + e*share_stride (byte strides).  Used for the compact
 * column slices of the all-to-all multi-GPU schedule.  Asynchronous. */
int rsm_encode_batch_dev(rsm_ctx* ctx, const void* d_in, void* d_out, uint32_t k, uint32_t share_size,
                         uint32_t count, uint64_t cw_stride, uint64_t share_stride, void* stream);
/* RowRoots()/ColRoots() with DefaultTree (datasquare.go:218-327, tree.go:32-59) of a
 * complete device-resident [width][width][share_size] square, on the GPU:
 * d_roots (device) receives 2*width*32 bytes, the row roots then the column roots.
 * width <= 2048.  Asynchronous on `stream`. */
int rsm_roots_dev(rsm_ctx* ctx, const void* d_eds, uint32_t width, uint32_t share_size, void* d_roots,
                  void* stream);
/* rsm_roots_dev over `count` consecutive squares ([count][width][width][share_size],
 * as rsm_extend_squares_dev lays them out): d_roots receives [count][2][width][32]
 * bytes.  One launch pair for the batch (BenchmarkExtensionWithRoots,
 * extendeddatasquare_test.go:309-334, over many squares). */
int rsm_roots_squares_dev(rsm_ctx* ctx, const void* d_eds, uint32_t width, uint32_t share_size, uint32_t count,
                          void* d_roots, void* stream);
/* Device-resident batched reconstruct of whole rows (axis 0) or columns (axis 1)
 * of one [2k][2k][S] square: d_presence is one byte per cell, d_indices the
 * vectors to rebuild (each must have >= k cells present).  Asynchronous. */
int rsm_decode_vectors_dev(rsm_ctx* ctx, void* d_eds, const uint8_t* d_presence, uint32_t k,
                           uint32_t share_size, int axis, const uint32_t* d_indices, uint32_t count,
                           void* stream);

/* ---- one square over several GPUs of a node (config 5) --------------------------- */
/* One process drives G GPUs: a context per device plus an RCCL clique
 * (ncclCommInitAll).  GPU g owns Q0 rows [g k/G, (g+1) k/G): it row-encodes them,
 * the top half is exchanged over xGMI, and GPU g column-encodes its 2k/G columns
 * (SURVEY.md section 8(e)).  Kernels and collectives of a GPU are ordered on that
 * GPU's context stream -- no host synchronisation between the steps. */
typedef struct rsm_multi rsm_multi;
#define RSM_SCHED_ALLGATHER 0 /* north_star: all-gather of the row-encoded top half */
#define RSM_SCHED_ALLTOALL 1  /* grouped send/recv: each GPU receives only its column slice */
int rsm_multi_create(const int* devices, int n, rsm_multi** out);
void rsm_multi_destroy(rsm_multi* m);
int rsm_multi_size(const rsm_multi* m);
/* The per-GPU context (device memory, streams) of GPU i of the clique. */
rsm_ctx* rsm_multi_context(rsm_multi* m, int i);
/* ComputeExtendedDataSquare (extendeddatasquare.go:50-77) of ONE k x k square from
 * host memory (ods k*k*S row-major -> eds (2k)^2*S row-major) over the clique;
 * k must be a multiple of G.  Synchronous. */
int rsm_multi_extend_square(rsm_multi* m, const uint8_t* ods, uint32_t k, uint32_t share_size, uint8_t* eds,
                            int schedule);
/* Pinned host memory for the multi-GPU host path (hipHostMalloc, portable: every GPU
 * of the clique DMAs it directly). */
int rsm_multi_host_alloc(rsm_multi* m, uint64_t bytes, void** p);
int rsm_multi_host_free(rsm_multi* m, void* p);
/* In-place host form (what the cgo ComputeExtendedDataSquare fast path calls on a
 * pinned arena): eds is (2k)^2*S row-major whose top-left k x k quadrant already
 * holds the ODS (Go's EDS aliases its input); only Q1, Q2, Q3 are written.  From
 * rsm_multi_host_alloc memory every copy is one DMA per GPU (Q0 rows up, Q1 rows and
 * the bottom-half column slice down; the Q1 download overlaps the exchange and the
 * column pass); pageable memory also works (staged by HIP).  Synchronous. */
int rsm_multi_extend_square_inplace(rsm_multi* m, uint8_t* eds, uint32_t k, uint32_t share_size, int schedule);
/* Device-resident form: d_eds[g] is a full [2k][2k][S] buffer on GPU g holding Q0
 * rows of shard g; afterwards it holds shard g's rows of the top half and the bottom
 * half [Q2|Q3] of its column slice [g 2k/G, (g+1) 2k/G) (all-gather: the whole top half
 * as well; all-to-all over the copy passes -- GF(2^8), k > 512 or blocks under 32 rows or
 * columns -- also the other shards' rows of its column slice; the copy-free all-to-all
 * leaves those in the clique's receive staging, where its column pass read them).
 * Asynchronous on the context streams; rsm_multi_sync waits. */
int rsm_multi_extend_dev(rsm_multi* m, void* const* d_eds, uint32_t k, uint32_t share_size, int schedule);
int rsm_multi_sync(rsm_multi* m);

/* ---- device memory / timing on the context's HIP runtime ---------------------- */
/* The context's stream (hipStream_t); the *_dev calls above use it when their
 * stream argument is NULL. */
void* rsm_ctx_stream(rsm_ctx* ctx);
int rsm_dev_alloc(rsm_ctx* ctx, uint64_t bytes, void** out);
int rsm_dev_free(rsm_ctx* ctx, void* p);
/* kind: 0 host->device, 1 device->host, 2 device->device; synchronous. */
int rsm_memcpy(rsm_ctx* ctx, void* dst, const void* src, uint64_t bytes, int kind);
/* SplitMix64 byte stream (seeded synthetic shares), asynchronous on the ctx stream. */
int rsm_dev_fill_random(rsm_ctx* ctx, void* d, uint64_t bytes, uint64_t seed);
int rsm_sync(rsm_ctx* ctx);
/* *equal = 1 iff the device buffers a and b (bytes a multiple of 16, both pointers
 * 16-byte aligned: the kernel reads them as uint4; RSM_EINVAL otherwise) are equal,
 * compared on the device (a kernel on `stream`, NULL = context stream); synchronous. */
int rsm_dev_equal(rsm_ctx* ctx, const void* a, const void* b, uint64_t bytes, void* stream, int* equal);
/* Extra HIP streams on the context's device, for callers that pipeline independent
 * batches (e.g. step n's column pass beside step n+1's row pass on another
 * stream).  Each stream owns its device scratch (GF(2^16) work arrays, leaf
 * digests), released by rsm_stream_destroy. */
int rsm_stream_create(rsm_ctx* ctx, void** out);
int rsm_stream_destroy(rsm_ctx* ctx, void* stream);
int rsm_stream_sync(void* stream);
/* Waits for `stream` (NULL = context stream) and returns RSM_EDEVICE (clearing it)
 * if a queue-driven extension on it reported a stuck wait; rsm_sync does the same
 * for the context stream only. */
int rsm_stream_check(rsm_ctx* ctx, void* stream);
/* HIP events on the context's device, for timing launches inside a caller's loop
 * (NULL stream = context stream).  rsm_event_elapsed_ms waits for `end`. */
int rsm_event_create(rsm_ctx* ctx, void** out);
int rsm_event_destroy(void* ev);
int rsm_event_record(rsm_ctx* ctx, void* ev, void* stream);
int rsm_event_elapsed_ms(void* start, void* end, float* ms);
/* Event-timed extension of `count` in-place squares on the ctx stream, averaged
 * over `reps`: row pass and column pass (the two launches of one extension) and
 * `step` = their sum, in milliseconds. */
int rsm_time_extend(rsm_ctx* ctx, void* d_eds, uint32_t k, uint32_t share_size, uint32_t count,
                    uint32_t reps, float* row_ms, float* col_ms, float* step_ms);

/* ---- Tree plugin (tree.go:11-28) ------------------------------------------------ */
/* Computes the root of one row/column: Push(leaves[0..n)) then Root().  Writes
 * the root to root_out (capacity *root_len on entry), sets *root_len, returns 0;
 * non-zero = tree error (treated as byzantine by Repair, as in the reference). */
typedef int (*rsm_tree_root_fn)(void* user, int axis, uint32_t index, const uint8_t* const* leaves,
                                uint32_t n_leaves, uint32_t leaf_size, uint8_t* root_out,
                                uint32_t* root_len);
/* NewDefaultTree restatement: celestiaorg/merkletree over SHA-256 (leaf
 * H(0x00||d), node H(0x01||l||r)).  Passed as NULL tree_fn below. */
int rsm_default_tree_root(void* user, int axis, uint32_t index, const uint8_t* const* leaves,
                          uint32_t n_leaves, uint32_t leaf_size, uint8_t* root_out,
                          uint32_t* root_len);

/* Namespaced Merkle tree (celestiaorg/nmt v0.24.3) as rsmt2d's erasured-NMT
 * wrappers push it (nmtwrapper_test.go:94-120; the buffered pool tree
 * nmtbuffered_tree_test.go:118-152 pushes identically): leaf i of row/column
 * `index` is pushed as ns || share with ns = share[:namespace_size] when
 * i < square_size and index < square_size (quadrant 0), else the parity namespace
 * 0xFF..; root = minNs || maxNs || SHA-256 digest (2*namespace_size + 32 bytes).
 * Tree errors (push order, too short, past the square) return RSM_ETREE. */
typedef struct {
    uint32_t namespace_size;       /* nmt.NamespaceIDSize (Celestia: 29) */
    uint32_t ignore_max_namespace; /* nmt.IgnoreMaxNamespace (the wrappers force 1) */
    uint32_t square_size;          /* ODS width k the wrapper was built for */
} rsm_nmt_params;
/* Tree plugin form: pass rsm_nmt_tree_root with user = (rsm_nmt_params*) as the
 * tree_fn of rsm_eds_roots / rsm_eds_repair: complete squares then take the
 * device path (kernels_nmt.hip), anything else the host restatement. */
int rsm_nmt_tree_root(void* user, int axis, uint32_t index, const uint8_t* const* leaves, uint32_t n_leaves,
                      uint32_t leaf_size, uint8_t* root_out, uint32_t* root_len);
/* Device NMT roots of a complete device-resident [width][width][share_size]
 * square: d_roots receives 2*width roots of 2*namespace_size + 32 bytes (rows,
 * then columns); d_status (device, may be NULL) 2*width uint32, non-zero where
 * that tree fails (push order).  namespace_size <= 32, width <= 1024.
 * Asynchronous on `stream`. */
int rsm_nmt_roots_dev(rsm_ctx* ctx, const void* d_eds, uint32_t width, uint32_t share_size,
                      const rsm_nmt_params* params, void* d_roots, void* d_status, void* stream);
/* The same for `count` consecutive device squares in one launch pair (a block's
 * worth of squares: the trees of one square alone leave most CUs idle); d_roots and
 * d_status hold 2*width entries per square, square after square. */
int rsm_nmt_roots_squares_dev(rsm_ctx* ctx, const void* d_eds, uint32_t width, uint32_t share_size, uint32_t count,
                              const rsm_nmt_params* params, void* d_roots, void* d_status, void* stream);

/* ---- ExtendedDataSquare (extendeddatasquare.go, datasquare.go) ------------------ */
/* ComputeExtendedDataSquare(data, codec, tree) (:50-77): n shares (lens[i] bytes). */
int rsm_eds_compute(rsm_ctx* ctx, const uint8_t* const* data, const uint32_t* lens, uint64_t n,
                    rsm_eds** out);
/* ImportExtendedDataSquare (:95-124): data[i] == NULL marks a missing share.
 * Import/New are host-only and accept ctx == NULL (a context is then needed,
 * via rsm_eds_set_context, before Repair). */
int rsm_eds_import(rsm_ctx* ctx, const uint8_t* const* data, const uint32_t* lens, uint64_t n,
                   rsm_eds** out);
/* NewExtendedDataSquare(codec, tree, edsWidth, shareSize) (:129-152). */
int rsm_eds_new(rsm_ctx* ctx, uint32_t eds_width, uint32_t share_size, rsm_eds** out);
void rsm_eds_free(rsm_eds* eds);
int rsm_eds_set_context(rsm_eds* eds, rsm_ctx* ctx);
uint32_t rsm_eds_width(const rsm_eds* eds);
uint32_t rsm_eds_original_width(const rsm_eds* eds);
uint32_t rsm_eds_share_size(const rsm_eds* eds);
/* GetCell: copies the share to out and returns 1, or returns 0 for nil. */
int rsm_eds_get_cell(const rsm_eds* eds, uint32_t row, uint32_t col, uint8_t* out);
/* SetCell: RSM_ECELL if the cell is non-nil or len != share size. */
int rsm_eds_set_cell(rsm_eds* eds, uint32_t row, uint32_t col, const uint8_t* share, uint32_t len);
/* Test hook mirroring the reference's unexported setCell (datasquare_test.go:735-739):
 * overwrites a cell without the nil check; share == NULL makes it nil. */
int rsm_eds_overwrite_cell(rsm_eds* eds, uint32_t row, uint32_t col, const uint8_t* share, uint32_t len);
/* Flattened(): width^2 * share_size bytes row-major + width^2 presence bytes. */
int rsm_eds_flattened(const rsm_eds* eds, uint8_t* out, uint8_t* present);
/* RowRoots()/ColRoots() (:258-280): width roots of root_cap bytes each. */
int rsm_eds_roots(rsm_eds* eds, int axis, rsm_tree_root_fn tree_fn, void* user, uint8_t* roots_out,
                  uint32_t root_cap, uint32_t* root_len);

typedef struct {
    int32_t axis;   /* RSM_AXIS_ROW / RSM_AXIS_COL */
    uint32_t index; /* row or column index */
} rsm_byzantine;

/* Repair(rowRoots, colRoots) (extendeddatacrossword.go:74-84): roots are
 * width * root_len bytes each.  Returns 0, RSM_EUNREPAIRABLE, or RSM_EBYZANTINE
 * (then *byz names the axis/index; rsm_eds_byzantine_shares() returns the
 * vector's shares as they were before repair, missing shares absent). */
int rsm_eds_repair(rsm_eds* eds, const uint8_t* row_roots, const uint8_t* col_roots, uint32_t root_len,
                   rsm_tree_root_fn tree_fn, void* user, rsm_byzantine* byz);
int rsm_eds_byzantine_shares(const rsm_eds* eds, uint8_t* out, uint8_t* present);

/* Diagnostics: counters of the last Repair (fast device path taken or not,
 * device decode sweeps, codewords decoded). */
typedef struct {
    int32_t fast_path;
    uint32_t sweeps;
    uint32_t decoded_vectors;
    uint32_t fallback_reason;
} rsm_repair_stats;
int rsm_eds_repair_stats(const rsm_eds* eds, rsm_repair_stats* out);

#ifdef __cplusplus
}
#endif
#endif /* RSMT2D_HIP_H */
