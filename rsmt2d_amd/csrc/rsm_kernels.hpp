// rsm_kernels.hpp -- descriptors shared by the HIP kernels and the host runtime.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace rsm {

__host__ __device__ constexpr uint32_t ceil_pow2(uint32_t x) {
    uint32_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

// A batch of codewords laid out affinely in device memory.  Codeword q lives in
// square q / per_square at offset (q % per_square) * cw_stride; its input
// symbol e (e < k) is the share at + e * elem_stride, its parity symbol e at
// + out_offset + e * elem_stride.  Rows of a [W][W][S] square:
//   cw_stride = W*S, elem_stride = S,   out_offset = k*S
// Columns:
//   cw_stride = S,   elem_stride = W*S, out_offset = k*W*S
struct CodewordSet {
    uint8_t* base;
    uint8_t* out_base;          // parity written at the same relative offsets from here
    const uint32_t* indices;    // optional: codeword q is vector indices[q] of square 0
    uint64_t square_stride;
    uint64_t cw_stride;
    uint64_t elem_stride;
    uint64_t out_offset;
    uint32_t per_square;
    uint32_t count;   // total codewords
    uint32_t k;
    uint32_t S;       // share size in bytes (multiple of 64)
    uint32_t chunks;  // ceil(S / bytes-per-wave)
    uint32_t pass;    // 0 = row pass of a square, 1 = column pass / anything else (launch shape)
    uint32_t grid;    // persistent-grid size (workgroups) of the bit-sliced launch: the
                      // context's CU count or its per-pass cap (rsm_ctx_set_pass_grid)
    uint32_t wide;    // non-zero: symbols addressed with 64-bit per-symbol bases (the
                      // wide forms; the host sets it when narrow_fits() fails)
    // Multi-GPU all-to-all (rsm_multi.cpp, round 6): honoured only by the single-pass
    // GF(2^16) encoders (shard_fused_ok(); the host never sets them otherwise).
    //   side (row pass): every cell c of codeword q -- data c = e, parity c = k + e --
    //     whose column block c / side_cols is not side_self is ALSO stored at
    //     side + (c / side_cols) * side_blk + q * side_cols * S + (c % side_cols) * S:
    //     the per-peer send blocks, packed by the encoder instead of a copy pass;
    //   blk (column pass): data symbol e of codeword (column) q whose row block
    //     h = e / blk_rows is not blk_self is read from
    //     blk + h * blk_size + (e % blk_rows) * blk_pitch + q * S -- the received blocks
    //     in place, instead of an unpack pass.
    uint8_t* side;
    uint64_t side_blk;
    uint32_t side_cols, side_self;
    const uint8_t* blk;
    uint64_t blk_size;
    uint32_t blk_rows, blk_self, blk_pitch;
};

// The single-pass kernels address a codeword's symbols with 32-bit buffer offsets
// from one 64-bit base per codeword half (encoders: the data symbols from the
// codeword's first cell, the parity from out_base + out_offset; decoders: each half
// of the 2k cells from its own first cell).  A half of k symbols e * es + byte must
// stay below kOffsetLimit -- the buffer resources' num_records, also the kernels'
// out-of-range marker -- so a half may span up to 2 GiB and a square up to 4 GiB;
// beyond that the wide forms (64-bit per-symbol bases) run instead.
constexpr uint64_t kOffsetLimit = 1ull << 31;
__host__ __device__ constexpr bool narrow_fits(uint64_t k, uint64_t es, uint64_t S, uint64_t limit = kOffsetLimit) {
    return (k + 1) * es + S <= limit;
}

// Parity addressed from its own base: out_base + out_offset with out_offset = 0
// (same bytes; the symbol offsets then span one half instead of out_offset + k es).
__host__ __device__ inline CodewordSet rebased(CodewordSet cs) {
    if (cs.out_base == nullptr) cs.out_base = cs.base;
    cs.out_base += cs.out_offset;
    cs.out_offset = 0;
    return cs;
}

// A list of row (axis 0) or column (axis 1) vectors of ONE [W][W][S] square to
// reconstruct in place; presence is one byte per cell (non-zero = present).
struct DecodeSet {
    uint8_t* base;
    const uint8_t* presence;
    const uint32_t* indices;
    uint32_t count;
    uint32_t axis;
    uint32_t k;
    uint32_t S;
    uint32_t chunks;
    // Zero-copy forms (the M = 128 split decoder and the GF(2^16) single-pass decoders;
    // both nullable): `in_base` (a host-mapped copy of the square): read the present
    // cells from there instead of `base` and store them into `base` as well; `mirror`:
    // write every rebuilt cell there too.
    const uint8_t* in_base;
    uint8_t* mirror;
    // Workgroups of the M = 128 split decoder (0: one per task).  A smaller grid
    // loops over the tasks, so the zero-copy form streams: a workgroup's stores
    // drain over PCIe while its next loads arrive, instead of every workgroup
    // loading, then computing, then storing in lockstep.
    uint32_t grid;
    // diagnostic builds only: per-workgroup phase stamps of the M = 128 split decoder
    // (kDecTraceWords s_memrealtime values per workgroup; nullptr = off)
    uint32_t* trace;
    // diagnostic builds only: the upper half of the split decoder's grid issues its
    // point loads `delay` s_memrealtime ticks (100 MHz) after it starts (0 = off)
    uint32_t delay;
    // wide forms only (64-bit per-cell bases; the host sets `wide` when narrow_fits()
    // fails): bytes between consecutive cells, 0 = S.  The host runs a share wider
    // than one launch handles as byte slabs: base advanced by the slab's first byte,
    // S = the slab's width, pitch = the share size.
    uint32_t wide;
    uint64_t pitch;
};
constexpr int kDecTraceWords = 8;
// DecodeSet::delay value of the diagnostic setup-free floor (rsm_diag_set_dec8_mode(2))
constexpr uint32_t kDecFloor = 0xFFFFFFFFu;
void set_dec_diag_trace(uint32_t* d);
uint32_t* dec_diag_trace_ptr();  // (diagnostic builds; the GF(2^16) single-pass decoders stamp kDec16TraceWords)
constexpr int kDec16TraceWords = 16;
void set_dec_diag_delay(uint32_t ticks);
void set_dec8_diag_mode(uint32_t mode);  // diagnostic builds only: 1 = the other split-decoder locator form
void set_codec_spin_diag(uint32_t us);  // diagnostic builds only (rsm_runtime.cpp)
void set_repair_diag_mode(uint32_t m);  // diagnostic builds only (eds.cpp)

hipError_t launch_encode_gf8(const CodewordSet& cs, hipStream_t st);
// wide forms of the byte-table GF(2^8) kernels (any k <= 128): 64-bit per-symbol
// bases, a capped grid looping over the (codeword, 256-byte chunk) tasks
hipError_t launch_encode_gf8_wide(const CodewordSet& cs, hipStream_t st);
hipError_t launch_decode_gf8_wide(const DecodeSet& ds, hipStream_t st);
// whether the GF(2^16) m <= 512 decoder in use needs per-stream work arrays (only the
// five-pass diagnostic form does; the single-pass forms keep everything on chip)
bool dec16_needs_work();
// bit-sliced M = 128 encode (kernels_gf8_bs.hip); launch_encode_gf8 picks it when applicable
bool bs128_applicable(const CodewordSet& cs);
hipError_t launch_encode_gf8_bs128(const CodewordSet& cs, hipStream_t st);
hipError_t launch_decode_gf8(const DecodeSet& ds, hipStream_t st);
// Latency form of the M = 128 encode (65 <= k <= 128) for one or a few squares
// (kernels_gf8.hip encode_gf8_split_kernel): NW waves per (codeword, 256-B chunk) on
// byte tables, every CU busy.  Launches the codewords of `a` and, if b != nullptr,
// those of `b` in the same grid.
// nw: waves per (codeword, 256-byte chunk), 8 or 16 (kSplitWavesOne)
hipError_t launch_encode_gf8_split(const CodewordSet& a, const CodewordSet* b, hipStream_t st, int nw);
constexpr int kSplitWavesOne = 16;  // one square / one codeword: the 16-wave latency form
constexpr uint32_t kSplitSmallBatch = 64;  // 9 <= k <= 64: squares per call for the split form (split_max > 0)
void set_split_diag_waves(int first, int second);  // diagnostic builds only
void set_split_diag_fused(bool on);                  // diagnostic builds only
void set_enc16_diag_e64(int mode);                   // diagnostic builds only
void set_dec16_diag_five_pass(bool on);              // diagnostic builds only
void set_dec16_diag_mode(uint32_t mode);            // diagnostic builds only: dec16h_kernel A/B bits
bool bs128_diag_xcd_queues();                        // diagnostic builds only: XCD-affine queue mode set
bool split_fused_enabled();                          // product: always
// One square in ONE launch of the split encoder (rows -> Q1, Q0 columns -> Q2, then
// Q1 columns -> Q3 behind a device-side wait on the row tasks); ctr: >= 33 zeroed
// words it leaves zeroed, err: pinned host word set by a stuck wait.  Every workgroup
// must be able to be resident at once (the caller checks the grid).
hipError_t launch_extend_gf8_split_fused(const CodewordSet& rows, const CodewordSet& c0, const CodewordSet& c1,
                                         uint32_t* ctr, uint32_t* err, hipStream_t st);
struct Gf16Dev;
hipError_t launch_encode_gf16(const CodewordSet& cs, const Gf16Dev& g, hipStream_t st);
hipError_t launch_decode_gf16(const DecodeSet& ds, const Gf16Dev& g, hipStream_t st);
// Merkle roots (kernels_sha.hip): d_leaf scratch of squares*W*W*32 bytes
bool roots_dev_supported(uint32_t W);
// Namespaced Merkle tree roots (kernels_nmt.hip): d_leaf W*W*64 bytes of scratch,
// d_roots 2W roots of 2*ns+32 bytes, d_status (nullable) 2W words.
bool nmt_dev_supported(uint32_t W, uint32_t ns);
hipError_t launch_nmt_roots(const uint8_t* d_eds, uint32_t W, uint32_t S, uint32_t ns, uint32_t k, uint32_t ignore_max,
                            uint32_t* d_leaf, uint8_t* d_roots, uint32_t* d_status, hipStream_t st, uint32_t squares = 1);
hipError_t launch_roots(const uint8_t* d_eds, uint32_t W, uint32_t S, uint32_t squares, uint32_t* d_leaf,
                        uint8_t* d_roots, hipStream_t st);
hipError_t launch_leaf_hashes(const uint8_t* d_cells, uint32_t cells, uint32_t S, uint32_t* d_leaf, hipStream_t st);
hipError_t launch_tree_roots(const uint32_t* d_leaf, uint32_t W, uint32_t first, uint32_t count, uint8_t* d_roots,
                             hipStream_t st);
hipError_t launch_fill_random(void* p, uint64_t bytes, uint64_t seed, hipStream_t st);
hipError_t launch_compare(const uint8_t* a, const uint8_t* b, uint64_t n, uint32_t* mismatch, hipStream_t st);
// dst = src for ceil(bytes / 16) 16-byte words (src: e.g. a pinned buffer's device mapping)
hipError_t launch_stage_copy(void* dst, const void* src, uint64_t bytes, hipStream_t st);
hipError_t launch_compare_parity(const uint8_t* a, const uint8_t* b, uint32_t k, uint32_t S, uint32_t axis,
                                 const uint32_t* indices, uint32_t count, uint32_t* flags, hipStream_t st);

// One launch that runs both passes of the 2D extension over `count` k = 128
// squares (kernels_gf8_bs.hip, extend_gf8_bs128q_kernel): row sets and Q0-column
// sets from one queue head, Q1-column sets from a ready list that the last row set
// of each square appends to, so the column sets re-read Q0 and Q1 while they are
// still in the Infinity Cache.  ctr: 224 + 2 * count zeroed words (the kernel
// leaves them zeroed again); a bounded wait that times out (never, by the
// deadlock-freedom argument in the kernel, short of a hardware fault) sets *err,
// a device-visible pinned host word the host checks after the stream completes.
struct QueuePlan {
    CodewordSet rows, cols;
    uint32_t* ctr;
    uint32_t* err;   // pinned host word (device-visible)
    uint32_t count;  // squares
    uint32_t rn, cn; // sets per square: row pass (= Q0-column sets = Q1-column sets), column pass
    uint32_t delay;  // row sets handed out before the first Q0-column set (<= count * rn)
    uint32_t nmain;  // 2 * count * rn: row sets + Q0-column sets
    uint32_t nq1;    // count * rn: Q1-column sets
    uint32_t margin; // a Q1-column set is claimed while more than this many ready ones are unclaimed
    uint32_t* trace; // diagnostic build only (phase timeline), else nullptr
};
constexpr uint32_t kQueueFixedWords = 224;
bool bs128_queue_applicable(const CodewordSet& rows, const CodewordSet& cols);
hipError_t launch_extend_gf8_bs128_queue(const QueuePlan& p, hipStream_t st);


#ifdef RSM_DIAG
// ---------------------------------------------------------------------------
// Diagnostic / A-B kernels: compiled only into librsmt2d_hip_diag.so (make diag),
// never into the product library.
// ---------------------------------------------------------------------------
// Two independent codeword batches in one persistent launch (kernels_gf8_bs.hip,
// encode_gf8_bs128p_kernel): the row pass of one batch of squares and the column
// pass of another, sets interleaved 1 : 2 when nb == 2 * na so that every CU mixes
// the compute-heavier row sets with the memory-heavier column sets.
struct DualPlan {
    CodewordSet a, b;
    uint32_t na, nb;  // sets of a, of b
};

hipError_t launch_encode_gf8_bs128_dual(const DualPlan& p, hipStream_t st);
// A-B kernel variant of the bit-sliced encode: 40 production, 0/8/24/56 A-B
// variants, 2 = no arithmetic, 4 = no global memory (wrong output by design)
void set_bs128_diag_mode(int mode, int rev_col, int xcd);
// per-set phase timeline of the half-split queue kernel (device buffer of
// grid * kTraceSets * kTraceWords words; nullptr: off)
constexpr uint32_t kTraceSets = 256, kTraceWords = 14;
void set_bs128_diag_trace(uint32_t* d);
void set_bs128_diag_row_mode(int mode);
#endif

}  // namespace rsm
