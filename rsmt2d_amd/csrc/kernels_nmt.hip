// kernels_nmt.hip -- row and column namespaced-Merkle-tree roots of a
// device-resident EDS, as rsmt2d's erasured NMT wrappers build them
// (nmtwrapper_test.go:94-120; the pooled tree nmtbuffered_tree_test.go:118-152
// pushes identically) over celestiaorg/nmt v0.24.3 (go.mod:7, not vendored;
// published algorithm restated in merkle.cpp and oracle/nmt.py):
//   cell (r, c) is pushed as ns || share, ns = share[:NS] when r < k and c < k
//   (quadrant 0; the same for the cell's row tree and its column tree), else the
//   parity namespace 0xFF..;
//   leaf node  = ns || ns || H(0x00 || ns || share);
//   inner node = l.min || max || H(0x01 || l || r), max = l.max when r.min is the
//                parity namespace (IgnoreMaxNamespace), else r.max;
//   root       = RFC 6962 split: pairing level by level and carrying an unpaired
//                last node up unchanged gives the same tree.
// Push order (namespaces non-decreasing along a vector) and sibling order are
// checked; a failing tree reports status 1 (the reference's Push/Root error,
// which Repair turns into ErrByzantineData, extendeddatacrossword.go:316-320).
//
// Two kernels, as for the DefaultTree (kernels_sha.hip):
//   nmt_leaf_kernel : one thread per cell, streams ns || share through SHA-256;
//                     one leaf record (ns, digest) serves the cell's row and column
//                     (nmt_leaf29_kernel: the same for 29-byte namespaces, 16-byte loads);
//   nmt_tree_kernel : one workgroup per tree, levels ping-pong in LDS; each thread
//                     lays its node message out in its own LDS bytes and hashes it.
// Namespace sizes up to 32 bytes (Celestia: 29), widths up to 1024 (LDS permitting).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <utility>

#include "sha256_dev.hpp"

namespace rsm {

namespace {

template <int N, typename F>
__device__ __forceinline__ void sfor_n(F&& f) {
    [&]<int... I>(std::integer_sequence<int, I...>) {
        (f(std::integral_constant<int, I>{}), ...);
    }(std::make_integer_sequence<int, N>{});
}

constexpr uint32_t kMaxNs = 32;
constexpr uint32_t kNsWords = kMaxNs / 4;
constexpr uint32_t kNodeWords = 3 * kNsWords;  // min[8] | max[8] | digest[8] (LDS)
constexpr uint32_t kLeafWords = 16;            // ns[8] | digest[8] (global, per cell)
constexpr uint32_t kMaxWidth = 1024;
constexpr size_t kLdsCap = 160 * 1024 - 256;  // per workgroup, less the static words

// SHA blocks of a node message 0x01 || l || r (nodes of 2 ns + 32 bytes)
__host__ __device__ constexpr uint32_t node_blocks(uint32_t ns) { return (1 + 2 * (2 * ns + 32) + 8) / 64 + 1; }
size_t tree_lds_bytes(uint32_t W, uint32_t ns) {  // two levels, a spare node, 256 message buffers
    return ((size_t)(2 * (W / 2) + 1) * kNodeWords + (size_t)256 * 16 * node_blocks(ns)) * 4;
}

// the first n bytes of a big-endian word (n clamped to 0..4)
__device__ __forceinline__ uint32_t head_mask(int n) {
    return n <= 0 ? 0u : (n >= 4 ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> (8 * n)));
}
__device__ __forceinline__ uint32_t be_word(const uint32_t* p, int i) { return __builtin_bswap32(p[i]); }

// Leaf records: leaf[cell][0..7] = namespace (big-endian words, zero padded),
// leaf[cell][8..15] = SHA256(0x00 || ns || share).
// Batched: blockIdx.y is the square (consecutive [W][W][S] buffers, leaf records
// consecutive per square).
__global__ __launch_bounds__(256) void nmt_leaf_kernel(const uint8_t* __restrict__ eds, uint32_t W, uint32_t S,
                                                       uint32_t ns, uint32_t k, uint32_t* __restrict__ leaf) {
    const uint32_t cell = blockIdx.x * 256u + threadIdx.x;
    if (cell >= W * W) return;
    eds += (uint64_t)blockIdx.y * W * W * S;
    leaf += (uint64_t)blockIdx.y * W * W * kLeafWords;
    const uint32_t r = cell / W, c = cell - r * W;
    const bool q0 = r < k && c < k;
    const uint32_t* dw = reinterpret_cast<const uint32_t*>(eds + (uint64_t)cell * S);
    const int nD = (int)(S / 4u);
    const int off = 1 + (int)ns;           // message bytes before the share
    const int L = off + (int)S;            // message length
    const int m0 = off >> 2;               // first word holding share bytes
    const uint32_t sh = 8u * (uint32_t)(off & 3);
    const int nb = (L + 8) / 64 + 1;       // SHA blocks
    // the namespace prefix words (message words 0..8 at most): 0x00 || ns
    uint32_t d0[kNsWords + 1];
#pragma unroll
    for (int i = 0; i <= (int)kNsWords; ++i) d0[i] = be_word(dw, i < nD ? i : 0);
    uint32_t h[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = kH0[i];
    uint32_t prev = 0;
    for (int b = 0; b < nb; ++b) {
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int m = 16 * b + i;
            const int p = 4 * m;  // byte position of the word
            uint32_t pre = 0;
            if (m <= (int)kNsWords) {  // only block 0 reaches here (m <= 8)
                const uint32_t lo = d0[i <= (int)kNsWords ? i : 0];
                const uint32_t hi = i >= 1 && i <= (int)kNsWords + 1 ? d0[i >= 1 ? i - 1 : 0] : 0u;
                pre = q0 ? __builtin_amdgcn_alignbit(m == 0 ? 0u : hi, lo, 8) : (m == 0 ? 0x00FFFFFFu : 0xFFFFFFFFu);
            }
            const int j = m - m0;  // share word index of this message word
            const uint32_t cur = be_word(dw, j < 0 ? 0 : (j < nD ? j : nD - 1));
            const uint32_t r2 = __builtin_amdgcn_alignbit(j <= 0 ? 0u : prev, cur, sh);
            prev = cur;
            const uint32_t mpre = head_mask(off - p);
            const uint32_t mr2 = head_mask(L - p) & ~mpre;
            uint32_t x = (pre & mpre) | (r2 & mr2);
            if (p <= L && L < p + 4) x |= 0x80u << (8 * (3 - (L - p)));
            if (b == nb - 1 && i == 15) x = 8u * (uint32_t)L;  // bit length (< 2^32), word 14 stays 0
            w[i] = x;
        }
        sha_block(h, w);
    }
    uint32_t* o = leaf + (uint64_t)cell * kLeafWords;
#pragma unroll
    for (int i = 0; i < (int)kNsWords; ++i) o[i] = (q0 ? d0[i] : 0xFFFFFFFFu) & head_mask((int)ns - 4 * i);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[kNsWords + i] = h[i];
}

// The same leaf records for Celestia's 29-byte namespace and shares a multiple of 64
// bytes, streamed like kernels_sha.hip's leaf_hash_kernel: 16-byte loads of 64-byte
// share chunks, big-endian words.  The message 0x00 || ns || share puts share byte j
// at message byte 30 + j, so message word m >= 8 is the funnel shift of share words
// m - 8 and m - 7 by 16 bits; words 0..7 carry the prefix (for a Q0 cell ns is the
// share's first 29 bytes: share words shifted by 8 bits, as the DefaultTree leaf).
// Block b (of S/64 + 1) takes chunk b - 1's upper half and chunk b's first nine
// words; the last block's share word S/4 is the 0x80 pad (at message byte 30 + S, byte
// 2 of word S/4 + 7), word 15 the bit length.  The generic kernel above reads each
// word with its own 4-byte load and runtime masks.
typedef uint32_t nv4u __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void nmt_leaf29_kernel(const uint8_t* __restrict__ eds, uint32_t W, uint32_t S,
                                                         uint32_t k, uint32_t* __restrict__ leaf) {
    const uint32_t cell = blockIdx.x * 256u + threadIdx.x;
    if (cell >= W * W) return;
    eds += (uint64_t)blockIdx.y * W * W * S;
    leaf += (uint64_t)blockIdx.y * W * W * kLeafWords;
    const uint32_t r = cell / W, c = cell - r * W;
    const bool q0 = r < k && c < k;
    const nv4u* p = reinterpret_cast<const nv4u*>(eds + (uint64_t)cell * S);
    const uint32_t chunks = S / 64u, L = 30u + S;
    uint32_t h[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = kH0[i];
    uint32_t hi[8];   // words 8..15 of the previous chunk
    uint32_t nsw[8];  // the namespace words (chunk 0's first eight)
    for (uint32_t b = 0; b <= chunks; ++b) {
        uint32_t cw[16];
        if (b < chunks) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const nv4u v = p[b * 4u + q];
                cw[4 * q + 0] = __builtin_bswap32(v.x);
                cw[4 * q + 1] = __builtin_bswap32(v.y);
                cw[4 * q + 2] = __builtin_bswap32(v.z);
                cw[4 * q + 3] = __builtin_bswap32(v.w);
            }
        } else {
            cw[0] = 0x80000000u;  // the pad byte after the share
#pragma unroll
            for (int i = 1; i < 16; ++i) cw[i] = 0u;
        }
        uint32_t w[16];
        if (b == 0) {
#pragma unroll
            for (int i = 0; i < 8; ++i) nsw[i] = cw[i];
#pragma unroll
            for (int i = 0; i < 7; ++i)
                w[i] = q0 ? __builtin_amdgcn_alignbit(i == 0 ? 0u : cw[i - 1], cw[i], 8)
                          : (i == 0 ? 0x00FFFFFFu : 0xFFFFFFFFu);
            w[7] = (q0 ? (__builtin_amdgcn_alignbit(cw[6], cw[7], 8) & 0xFFFF0000u) : 0xFFFF0000u) | (cw[0] >> 16);
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) w[i] = __builtin_amdgcn_alignbit(hi[i], i < 7 ? hi[i + 1] : cw[0], 16);
        }
        if (b < chunks) {
#pragma unroll
            for (int i = 8; i < 16; ++i) w[i] = __builtin_amdgcn_alignbit(cw[i - 8], cw[i - 7], 16);
#pragma unroll
            for (int i = 0; i < 8; ++i) hi[i] = cw[8 + i];
        } else {
#pragma unroll
            for (int i = 8; i < 15; ++i) w[i] = 0u;
            w[15] = 8u * L;
        }
        sha_block(h, w);
    }
    uint32_t* o = leaf + (uint64_t)cell * kLeafWords;
#pragma unroll
    for (int i = 0; i < (int)kNsWords; ++i) o[i] = (q0 ? nsw[i] : 0xFFFFFFFFu) & head_mask(29 - 4 * i);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[kNsWords + i] = h[i];
}

struct Node {
    uint32_t mn[kNsWords], mx[kNsWords], d[8];
};

// a < b over namespaces held as zero-padded big-endian words
__device__ __forceinline__ bool ns_less(const uint32_t (&a)[kNsWords], const uint32_t (&b)[kNsWords]) {
#pragma unroll
    for (int i = 0; i < (int)kNsWords; ++i)
        if (a[i] != b[i]) return a[i] < b[i];
    return false;
}

// byte i of a big-endian word array (i static after unrolling)
__device__ __forceinline__ uint8_t be_byte(const uint32_t* w, int i) { return (uint8_t)(w[i >> 2] >> (24 - 8 * (i & 3))); }

// HashNode(l, r) (nmt hasher): message 0x01 || l || r laid out in this thread's
// LDS bytes `mb`, then hashed as big-endian words.  Returns false on unordered
// siblings (r.min < l.max).
__device__ __forceinline__ bool hash_node(const Node& l, const Node& r, uint32_t ns, bool ignore_max, uint8_t* mb, Node& out) {
    const int NL = 2 * (int)ns + 32;
    const int len = 1 + 2 * NL;
    const int nb = (int)node_blocks(ns);
    uint32_t* mw = reinterpret_cast<uint32_t*>(mb);
    for (int i = 0; i < 16 * nb; ++i) mw[i] = 0;
    mb[0] = 0x01;
    auto put = [&](const Node& n, int at) {
#pragma unroll
        for (int i = 0; i < (int)kMaxNs; ++i)
            if (i < (int)ns) {
                mb[at + i] = be_byte(n.mn, i);
                mb[at + (int)ns + i] = be_byte(n.mx, i);
            }
#pragma unroll
        for (int i = 0; i < 32; ++i) mb[at + 2 * (int)ns + i] = be_byte(n.d, i);
    };
    put(l, 1);
    put(r, 1 + NL);
    mb[len] = 0x80;
    const uint32_t bits = 8u * (uint32_t)len;
    mb[64 * nb - 2] = (uint8_t)(bits >> 8);
    mb[64 * nb - 1] = (uint8_t)bits;
    uint32_t h[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = kH0[i];
    for (int b = 0; b < nb; ++b) {
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = __builtin_bswap32(mw[16 * b + i]);
        sha_block(h, w);
    }
    bool rmin_is_max = true;
#pragma unroll
    for (int i = 0; i < (int)kNsWords; ++i) rmin_is_max &= r.mn[i] == head_mask((int)ns - 4 * i);
    const bool ok = !ns_less(r.mn, l.mx);
#pragma unroll
    for (int i = 0; i < (int)kNsWords; ++i) {
        out.mn[i] = l.mn[i];
        out.mx[i] = (ignore_max && rmin_is_max) ? l.mx[i] : r.mx[i];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) out.d[i] = h[i];
    return ok;
}

__device__ __forceinline__ void leaf_node(const uint32_t* __restrict__ leaf, uint64_t cell, Node& n) {
    const uint32_t* s = leaf + cell * kLeafWords;
#pragma unroll
    for (int i = 0; i < (int)kNsWords; ++i) n.mn[i] = n.mx[i] = s[i];
#pragma unroll
    for (int i = 0; i < 8; ++i) n.d[i] = s[kNsWords + i];
}
__device__ __forceinline__ void lds_node(const uint32_t* p, Node& n) {
#pragma unroll
    for (int i = 0; i < (int)kNsWords; ++i) n.mn[i] = p[i], n.mx[i] = p[kNsWords + i];
#pragma unroll
    for (int i = 0; i < 8; ++i) n.d[i] = p[2 * kNsWords + i];
}
__device__ __forceinline__ void lds_store(uint32_t* p, const Node& n) {
#pragma unroll
    for (int i = 0; i < (int)kNsWords; ++i) p[i] = n.mn[i], p[kNsWords + i] = n.mx[i];
#pragma unroll
    for (int i = 0; i < 8; ++i) p[2 * kNsWords + i] = n.d[i];
}

// One workgroup per tree (blockIdx.x < W: row tree, else column tree; blockIdx.y the
// square of a batch).  Dynamic LDS: two levels of W/2 nodes (ping-pong) + 256
// per-thread message buffers.
__global__ __launch_bounds__(256) void nmt_tree_kernel(const uint32_t* __restrict__ leaf, uint32_t W, uint32_t ns,
                                                       uint32_t ignore_max, uint8_t* __restrict__ roots,
                                                       uint32_t* __restrict__ status) {
    extern __shared__ uint32_t lds[];
    leaf += (uint64_t)blockIdx.y * W * W * kLeafWords;
    roots += (uint64_t)blockIdx.y * 2 * W * (2 * ns + 32);
    if (status) status += (uint64_t)blockIdx.y * 2 * W;
    const uint32_t half = W / 2;
    auto lvl = [&](uint32_t which) -> uint32_t* { return lds + (size_t)which * half * kNodeWords; };
    // the spare node: lanes past a level's last node store their repeat there (below)
    uint32_t* const spare = lds + (size_t)2 * half * kNodeWords;
    uint8_t* mb = reinterpret_cast<uint8_t*>(spare + kNodeWords) + threadIdx.x * (64u * node_blocks(ns));
    __shared__ uint32_t bad;
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    const uint32_t tree = blockIdx.x;
    const uint32_t axis = tree >= W ? 1u : 0u;
    const uint32_t idx = tree - axis * W;
    auto cell_of = [&](uint32_t pos) -> uint64_t { return axis == 0 ? (uint64_t)idx * W + pos : (uint64_t)pos * W + idx; };
    const bool ig = ignore_max != 0;
    uint32_t my_bad = 0;
    // level 1 from the leaf records: pairs (2j, 2j+1); push order checked on
    // every consecutive leaf pair
    // A level's pass runs every lane of the wave that holds its last node: lanes past
    // it repeat node j0 + tid % rem and store to the spare node (a wave with few lanes
    // active hashes 2-3.5x slower per compression: kernels_sha.hip); whole waves past
    // it stay idle.
    auto pass_lane = [&](uint32_t j0, uint32_t n, uint32_t& j, bool& own) -> bool {
        const uint32_t rem = n - j0;
        own = threadIdx.x < rem;
        if (!own && (threadIdx.x >> 6) != ((rem - 1) >> 6)) return false;
        j = j0 + (own ? threadIdx.x : threadIdx.x % rem);
        return true;
    };
    uint32_t cnt = W;
    uint32_t next = (cnt + 1) / 2;
    for (uint32_t j0 = 0; j0 < next; j0 += 256u) {
        uint32_t j;
        bool own;
        if (!pass_lane(j0, next, j, own)) continue;
        Node a, b, o;
        uint32_t bad_here = 0;
        leaf_node(leaf, cell_of(2 * j), a);
        if (2 * j + 1 < cnt) {
            leaf_node(leaf, cell_of(2 * j + 1), b);
            if (ns_less(b.mn, a.mn)) bad_here = 1;
            if (2 * j + 2 < cnt) {
                Node c;
                leaf_node(leaf, cell_of(2 * j + 2), c);
                if (ns_less(c.mn, b.mn)) bad_here = 1;
            }
            if (!hash_node(a, b, ns, ig, mb, o)) bad_here = 1;
        } else {
            o = a;
        }
        if (own) my_bad |= bad_here;
        lds_store(own ? lvl(0) + (size_t)j * kNodeWords : spare, o);
    }
    __syncthreads();
    uint32_t cur = 0;
    for (cnt = next; cnt > 1; cnt = next) {
        next = (cnt + 1) / 2;
        for (uint32_t j0 = 0; j0 < next; j0 += 256u) {
            uint32_t j;
            bool own;
            if (!pass_lane(j0, next, j, own)) continue;
            Node a, b, o;
            lds_node(lvl(cur) + (size_t)(2 * j) * kNodeWords, a);
            if (2 * j + 1 < cnt) {
                lds_node(lvl(cur) + (size_t)(2 * j + 1) * kNodeWords, b);
                if (!hash_node(a, b, ns, ig, mb, o) && own) my_bad = 1;
            } else {
                o = a;
            }
            lds_store(own ? lvl(cur ^ 1u) + (size_t)j * kNodeWords : spare, o);
        }
        __syncthreads();
        cur ^= 1u;
    }
    if (my_bad) atomicOr(&bad, 1u);
    __syncthreads();
    if (threadIdx.x == 0) {
        Node rt;
        lds_node(lvl(cur), rt);
        uint8_t* o = roots + (uint64_t)tree * (2 * ns + 32);
#pragma unroll
        for (int i = 0; i < (int)kMaxNs; ++i)
            if (i < (int)ns) {
                o[i] = be_byte(rt.mn, i);
                o[ns + i] = be_byte(rt.mx, i);
            }
#pragma unroll
        for (int i = 0; i < 32; ++i) o[2 * ns + i] = be_byte(rt.d, i);
        if (status) status[tree] = bad;
    }
}

// ---------------------------------------------------------------------------
// Wave-per-tree form for a compile-time namespace size (Celestia: 29): TPW trees per
// wave, four waves per workgroup, each tree's levels in place in the wave's own LDS
// (node j of a level reads 2j and 2j + 1 >= j: a level's reads precede its writes),
// no workgroup barrier -- the DefaultTree kernel's structure (kernels_sha.hip), which
// beat the level-by-level workgroup form 3x there.  The node message
// 0x01 || l || r (l, r = min || max || digest) is assembled in registers from
// compile-time byte positions (the backend forms v_perm / v_alignbit from them)
// instead of byte stores to a per-thread LDS buffer.  Same tree, same checks, same
// output as nmt_tree_kernel.
template <int NS>
struct WNode {
    static constexpr int kW = (NS + 3) / 4;
    uint32_t mn[kW], mx[kW], d[8];
};
template <int NS, int B>
__device__ __forceinline__ uint32_t node_byte(const WNode<NS>& n) {  // byte B of min || max || digest
    if constexpr (B < NS) return (n.mn[B >> 2] >> (24 - 8 * (B & 3))) & 0xFFu;
    else if constexpr (B < 2 * NS) return (n.mx[(B - NS) >> 2] >> (24 - 8 * ((B - NS) & 3))) & 0xFFu;
    else return (n.d[(B - 2 * NS) >> 2] >> (24 - 8 * ((B - 2 * NS) & 3))) & 0xFFu;
}
template <int NS, int I>
__device__ __forceinline__ uint32_t msg_byte(const WNode<NS>& l, const WNode<NS>& r) {
    constexpr int NL = 2 * NS + 32, LEN = 1 + 2 * NL, NB = (LEN + 8) / 64 + 1;
    if constexpr (I == 0) return 0x01u;
    else if constexpr (I <= NL) return node_byte<NS, I - 1>(l);
    else if constexpr (I <= 2 * NL) return node_byte<NS, I - 1 - NL>(r);
    else if constexpr (I == LEN) return 0x80u;
    else if constexpr (I == 64 * NB - 2) return ((8u * LEN) >> 8) & 0xFFu;
    else if constexpr (I == 64 * NB - 1) return (8u * LEN) & 0xFFu;
    else return 0u;
}
template <int NS>
__device__ __forceinline__ bool hash_node_w(const WNode<NS>& l, const WNode<NS>& r, bool ignore_max, WNode<NS>& out) {
    constexpr int NL = 2 * NS + 32, LEN = 1 + 2 * NL, NB = (LEN + 8) / 64 + 1;
    uint32_t h[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = kH0[i];
    sfor_n<NB>([&](auto Bc) {
        constexpr int b = decltype(Bc)::value;
        uint32_t w[16];
        sfor_n<16>([&](auto Ic) {
            constexpr int t = 16 * b + decltype(Ic)::value;
            w[decltype(Ic)::value] = (msg_byte<NS, 4 * t>(l, r) << 24) | (msg_byte<NS, 4 * t + 1>(l, r) << 16) |
                                     (msg_byte<NS, 4 * t + 2>(l, r) << 8) | msg_byte<NS, 4 * t + 3>(l, r);
        });
        sha_block(h, w);
    });
    constexpr int kW = WNode<NS>::kW;
    bool rmin_is_max = true;
#pragma unroll
    for (int i = 0; i < kW; ++i) rmin_is_max &= r.mn[i] == head_mask(NS - 4 * i);
    bool less = false, decided = false;  // r.mn < l.mx ?
#pragma unroll
    for (int i = 0; i < kW; ++i)
        if (!decided && r.mn[i] != l.mx[i]) {
            less = r.mn[i] < l.mx[i];
            decided = true;
        }
#pragma unroll
    for (int i = 0; i < kW; ++i) {
        out.mn[i] = l.mn[i];
        out.mx[i] = (ignore_max && rmin_is_max) ? l.mx[i] : r.mx[i];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) out.d[i] = h[i];
    return !less;
}
template <int NS>
__host__ __device__ constexpr uint32_t wnode_words() { return 2 * WNode<NS>::kW + 8; }
template <int NS>
__host__ __device__ constexpr uint32_t wtree_lds_words(uint32_t W, bool f2 = false) {
    return (f2 ? W / 4 : (W + 1) / 2) * wnode_words<NS>();  // f2: levels 1 and 2 in one pass
}
// one wave's LDS: its trees, then a spare node that lanes past a level's last node
// store to (so every lane hashes: see the level loops)
template <int NS>
__host__ __device__ constexpr uint32_t wwave_lds_words(uint32_t W, uint32_t tpw, bool f2 = false) {
    return tpw * wtree_lds_words<NS>(W, f2) + wnode_words<NS>();
}
constexpr uint32_t kNmtTreesPerBlock = 4;  // waves per workgroup of the one-tree-per-wave form

// WPB waves per workgroup, TPW trees per wave.  F2 (W a multiple of 4): the first pass
// hashes leaves 4j .. 4j + 3 into level-1 nodes 2j, 2j + 1 and on into level-2 node j,
// so LDS holds W/4 nodes per tree instead of W/2 (more trees, or more waves, per CU).
// Once a wave's TPW trees have fewer than 64 nodes in a level, the workgroup's WPB TPW
// trees are built together (as kernels_sha.hip's COOP form): node U * next + j of the
// workgroup on lane (U * next + j) mod 64 of wave (U * next + j) / 64, a barrier
// between a level's reads and its in-place writes, waves past the level's last node
// idle.  At W = 256, TPW = 2, WPB = 4: 34 wave-passes of three compressions per
// workgroup of 8 trees instead of 48 (each wave's own top five levels were one pass
// each for 32 .. 2 nodes).
template <int NS, int TPW, int WPB, bool F2>
__global__ __launch_bounds__(64 * WPB) void nmt_tree_wave_kernel(const uint32_t* __restrict__ leaf, uint32_t W,
                                                                 uint32_t ignore_max, uint8_t* __restrict__ roots,
                                                                 uint32_t* __restrict__ status) {
    constexpr int kW = WNode<NS>::kW;
    constexpr uint32_t NW = wnode_words<NS>();
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t tw0 = blockIdx.x * WPB * TPW, count = 2 * W;  // the workgroup's first tree
    const uint32_t t0 = tw0 + wv * TPW;
    // waves without trees stay for the workgroup barriers of the upper levels
    const uint32_t nt = t0 >= count ? 0u : (count - t0 < (uint32_t)TPW ? count - t0 : (uint32_t)TPW);
    const uint32_t ntw = count - tw0 < (uint32_t)(WPB * TPW) ? count - tw0 : (uint32_t)(WPB * TPW);
    __shared__ uint32_t wg_bad;  // bit U: workgroup tree U failed
    if (threadIdx.x == 0) wg_bad = 0;
    __syncthreads();  // before any wave's atomicOr (a W whose levels need no other barrier)
    leaf += (uint64_t)blockIdx.y * W * W * kLeafWords;
    roots += (uint64_t)blockIdx.y * 2 * W * (2 * NS + 32);
    if (status) status += (uint64_t)blockIdx.y * 2 * W;
    extern __shared__ uint32_t lds_raw[];
    // workgroup tree U: wave U / TPW's tree U % TPW
    auto tlvl = [&](uint32_t U) {
        return lds_raw + (size_t)(U / TPW) * wwave_lds_words<NS>(W, TPW, F2) + (size_t)(U % TPW) * wtree_lds_words<NS>(W, F2);
    };
    uint32_t* const base = lds_raw + (size_t)wv * wwave_lds_words<NS>(W, TPW, F2);
    auto lvl = [&](uint32_t u) { return base + (size_t)u * wtree_lds_words<NS>(W, F2); };
    uint32_t* const spare = base + (size_t)TPW * wtree_lds_words<NS>(W, F2);
    const bool ig = ignore_max != 0;
    auto leaf_at = [&](uint32_t tree, uint32_t pos, WNode<NS>& n) {
        const uint32_t axis = tree >= W ? 1u : 0u, idx = tree - axis * W;
        const uint64_t cell = axis == 0 ? (uint64_t)idx * W + pos : (uint64_t)pos * W + idx;
        const uint32_t* sp = leaf + cell * kLeafWords;
#pragma unroll
        for (int i = 0; i < kW; ++i) n.mn[i] = n.mx[i] = sp[i];
#pragma unroll
        for (int i = 0; i < 8; ++i) n.d[i] = sp[kNsWords + i];
    };
    auto ld = [&](const uint32_t* p, WNode<NS>& n) {
#pragma unroll
        for (int i = 0; i < kW; ++i) n.mn[i] = p[i], n.mx[i] = p[kW + i];
#pragma unroll
        for (int i = 0; i < 8; ++i) n.d[i] = p[2 * kW + i];
    };
    auto st = [&](uint32_t* p, const WNode<NS>& n) {
#pragma unroll
        for (int i = 0; i < kW; ++i) p[i] = n.mn[i], p[kW + i] = n.mx[i];
#pragma unroll
        for (int i = 0; i < 8; ++i) p[2 * kW + i] = n.d[i];
    };
    auto ns_lt = [&](const uint32_t* a, const uint32_t* b) {  // a < b
        bool less = false, decided = false;
#pragma unroll
        for (int i = 0; i < kW; ++i)
            if (!decided && a[i] != b[i]) {
                less = a[i] < b[i];
                decided = true;
            }
        return less;
    };
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    uint32_t bad = 0;  // bit U: workgroup tree U failed (push order / sibling order)
    // level 1 from the leaf records (push order checked on every consecutive pair)
    // Every lane hashes in every pass of a level: past the level's last node a lane
    // repeats node v0 + lane % rem and stores it to the wave's spare node (a wave
    // with <= 8 lanes active runs its SHA rounds 2-3.5x slower per compression:
    // kernels_sha.hip; the store keeps the compiler from shrinking the hash to the
    // owning lanes).
    uint32_t cnt = W, next = (W + 1) / 2;
    if constexpr (F2) {
        next = W / 4;
        for (uint32_t v0 = 0; v0 < nt * next; v0 += 64u) {
            const uint32_t rem = nt * next - v0;
            const bool own = lane < rem;
            const uint32_t v = v0 + (own ? lane : lane % rem);
            const uint32_t u = v / next, j = v - u * next;
            WNode<NS> a, b, c, d, l, r, o;
            leaf_at(t0 + u, 4 * j, a);
            leaf_at(t0 + u, 4 * j + 1, b);
            leaf_at(t0 + u, 4 * j + 2, c);
            leaf_at(t0 + u, 4 * j + 3, d);
            bool ok = !ns_lt(b.mn, a.mn) && !ns_lt(c.mn, b.mn) && !ns_lt(d.mn, c.mn);
            if (4 * j + 4 < cnt) {  // push order across the next group's first leaf
                WNode<NS> e;
                leaf_at(t0 + u, 4 * j + 4, e);
                if (ns_lt(e.mn, d.mn)) ok = false;
            }
            if (!hash_node_w<NS>(a, b, ig, l)) ok = false;
            if (!hash_node_w<NS>(c, d, ig, r)) ok = false;
            if (!hash_node_w<NS>(l, r, ig, o)) ok = false;
            st(own ? lvl(u) + (size_t)j * NW : spare, o);
            if (own && !ok) bad |= 1u << (wv * TPW + u);
        }
    } else {
        for (uint32_t v0 = 0; v0 < nt * next; v0 += 64u) {
            const uint32_t rem = nt * next - v0;
            const bool own = lane < rem;
            const uint32_t v = v0 + (own ? lane : lane % rem);
            const uint32_t u = v / next, j = v - u * next;
            WNode<NS> a, b, o;
            leaf_at(t0 + u, 2 * j, a);
            bool ok = true;
            if (2 * j + 1 < cnt) {
                leaf_at(t0 + u, 2 * j + 1, b);
                if (ns_lt(b.mn, a.mn)) ok = false;
                if (2 * j + 2 < cnt) {
                    WNode<NS> c;
                    leaf_at(t0 + u, 2 * j + 2, c);
                    if (ns_lt(c.mn, b.mn)) ok = false;
                }
                if (!hash_node_w<NS>(a, b, ig, o)) ok = false;
            } else {
                o = a;
            }
            st(own ? lvl(u) + (size_t)j * NW : spare, o);
            if (own && !ok) bad |= 1u << (wv * TPW + u);
        }
    }
    wave_sync();
    for (cnt = next; cnt > 1; cnt = next) {
        next = (cnt + 1) / 2;
        if ((uint32_t)TPW * next < 64u) {
            // the workgroup's trees together: at most one pass per wave (WPB TPW next < 64 WPB)
            const uint32_t tot = ntw * next, v0 = wv * 64u;
            __syncthreads();  // the previous level's nodes (any wave's) are written
            uint32_t U = 0, j = 0;
            bool own = false;
            WNode<NS> o;
            if (v0 < tot) {
                const uint32_t rem = tot - v0;  // every lane of a working wave hashes
                own = lane < rem;
                const uint32_t v = v0 + (own ? lane : lane % rem);
                U = v / next;
                j = v - U * next;
                WNode<NS> a, b;
                ld(tlvl(U) + (size_t)(2 * j) * NW, a);
                if (2 * j + 1 < cnt) {
                    ld(tlvl(U) + (size_t)(2 * j + 1) * NW, b);
                    if (!hash_node_w<NS>(a, b, ig, o) && own) bad |= 1u << U;
                } else {
                    o = a;
                }
            }
            __syncthreads();  // every read of this level precedes its in-place writes
            if (v0 < tot) st(own ? tlvl(U) + (size_t)j * NW : spare, o);
            continue;
        }
        for (uint32_t v0 = 0; v0 < nt * next; v0 += 64u) {
            const uint32_t rem = nt * next - v0;
            const bool own = lane < rem;
            const uint32_t v = v0 + (own ? lane : lane % rem);
            const uint32_t u = v / next, j = v - u * next;
            WNode<NS> a, b, o;
            ld(lvl(u) + (size_t)(2 * j) * NW, a);
            if (2 * j + 1 < cnt) {
                ld(lvl(u) + (size_t)(2 * j + 1) * NW, b);
                if (!hash_node_w<NS>(a, b, ig, o) && own) bad |= 1u << (wv * TPW + u);
            } else {
                o = a;
            }
            wave_sync();  // every lane's reads of this level before any write (j < 2j)
            st(own ? lvl(u) + (size_t)j * NW : spare, o);
        }
        wave_sync();
    }
    // OR of every lane's failure bits, per workgroup tree
    uint32_t all = bad;
#pragma unroll
    for (int sft = 1; sft < 64; sft <<= 1) all |= __shfl_xor(all, sft);
    if (lane == 0 && all) atomicOr(&wg_bad, all);
    __syncthreads();  // the roots (written by any wave) and wg_bad
    all = wg_bad >> (wv * TPW);
    if (lane < nt) {
        const uint32_t tree = t0 + lane;
        WNode<NS> rt;
        ld(lvl(lane), rt);
        uint8_t* o = roots + (uint64_t)tree * (2 * NS + 32);
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            o[i] = be_byte(rt.mn, i);
            o[NS + i] = be_byte(rt.mx, i);
        }
#pragma unroll
        for (int i = 0; i < 32; ++i) o[2 * NS + i] = be_byte(rt.d, i);
        if (status) status[tree] = (all >> lane) & 1u;
    }
}

// Trees per wave and waves per workgroup.  A batch packs two trees per wave (the upper
// levels of one tree leave most lanes repeating work, so packing cuts the batch's
// wave-instructions) in four-wave workgroups when their LDS fits a third of the CU,
// else two-wave ones; one square (latency: Repair's checks) takes one tree per wave.
// W = 256, 32 squares (scripts/diag/nmtprobe.hip, profiles/r05aa_nmtprobe.txt): one tree
// per wave 1142 us; two per wave 1012; with levels 1-2 fused (F2) 786 at 2 x 4 or 2 x 2
// waves, 913 at four trees per wave.
template <int NS>
inline void nmt_tree_shape(uint32_t W, bool latency, bool f2, uint32_t* tpw, uint32_t* wpb) {
    *tpw = 1;
    *wpb = kNmtTreesPerBlock;
    if (latency) return;
    for (uint32_t b = 4; b >= 2; b >>= 1)
        if ((size_t)b * wwave_lds_words<NS>(W, 2, f2) * 4u <= 52u * 1024u) {
            *tpw = 2;
            *wpb = b;
            return;
        }
}
template <int NS>
hipError_t launch_nmt_tree_wave(const uint32_t* d_leaf, uint32_t W, uint32_t ignore_max, uint8_t* d_roots,
                                uint32_t* d_status, uint32_t squares, hipStream_t st) {
    const bool f2 = W % 4 == 0;
    uint32_t tpw, wpb;
    nmt_tree_shape<NS>(W, squares == 1, f2, &tpw, &wpb);
    const uint32_t blocks = (2 * W + wpb * tpw - 1) / (wpb * tpw);
    const size_t lds = (size_t)wpb * wwave_lds_words<NS>(W, tpw, f2) * 4u;
    const dim3 grid(blocks, squares);
#define RSM_NMT_WAVE(T, B, F)                                                                                     \
    hipLaunchKernelGGL((nmt_tree_wave_kernel<NS, T, B, F>), grid, dim3(64 * B), lds, st, d_leaf, W, ignore_max,    \
                       d_roots, d_status)
#define RSM_NMT_WAVE_F(T, B)      \
    if (f2) RSM_NMT_WAVE(T, B, true); \
    else RSM_NMT_WAVE(T, B, false)
    if (tpw == 2 && wpb == 4) { RSM_NMT_WAVE_F(2, 4); }
    else if (tpw == 2) { RSM_NMT_WAVE_F(2, 2); }
    else { RSM_NMT_WAVE_F(1, 4); }
#undef RSM_NMT_WAVE_F
#undef RSM_NMT_WAVE
    return hipGetLastError();
}

}  // namespace

bool nmt_dev_supported(uint32_t W, uint32_t ns) {
    return W >= 2 && W <= kMaxWidth && ns >= 1 && ns <= kMaxNs && tree_lds_bytes(W, ns) <= kLdsCap;
}

// d_leaf: squares * W*W*64 bytes of scratch; the squares are consecutive [W][W][S]
// buffers, their 2W roots (and statuses) consecutive per square.
hipError_t launch_nmt_roots(const uint8_t* d_eds, uint32_t W, uint32_t S, uint32_t ns, uint32_t k, uint32_t ignore_max,
                            uint32_t* d_leaf, uint8_t* d_roots, uint32_t* d_status, hipStream_t st, uint32_t squares) {
    if (squares == 0) return hipSuccess;
    const uint32_t cells = W * W;
    // Celestia's namespace: the streaming leaf kernel (16-byte loads at eds + cell*S, so
    // the base must be 16-byte aligned; a caller-supplied unaligned square takes the
    // word-load kernel)
    if (ns == 29 && S % 64 == 0 && S >= 64 && (reinterpret_cast<uintptr_t>(d_eds) & 15u) == 0)
        hipLaunchKernelGGL(nmt_leaf29_kernel, dim3((cells + 255) / 256, squares), dim3(256), 0, st, d_eds, W, S, k, d_leaf);
    else
        hipLaunchKernelGGL(nmt_leaf_kernel, dim3((cells + 255) / 256, squares), dim3(256), 0, st, d_eds, W, S, ns, k, d_leaf);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    // Celestia's namespace size: the wave-per-tree kernel (its LDS permitting)
    if (ns == 29 && (size_t)kNmtTreesPerBlock * wwave_lds_words<29>(W, 1, W % 4 == 0) * 4u <= kLdsCap)
        return launch_nmt_tree_wave<29>(d_leaf, W, ignore_max, d_roots, d_status, squares, st);
    const size_t lds = tree_lds_bytes(W, ns);
    hipLaunchKernelGGL(nmt_tree_kernel, dim3(2 * W, squares), dim3(256), lds, st, d_leaf, W, ns, ignore_max, d_roots,
                       d_status);
    return hipGetLastError();
}

}  // namespace rsm
