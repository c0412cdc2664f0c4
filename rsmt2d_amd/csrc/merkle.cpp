// merkle.cpp -- host restatement of rsmt2d's DefaultTree (tree.go:32-59):
// celestiaorg/merkletree over SHA-256 with leaf = H(0x00 || data) and
// node = H(0x01 || left || right); for a non-power-of-two leaf count the
// subtrees are joined right-to-left exactly as the NebulousLabs-style stack
// (push joins equal-height subtrees; Root folds the stack from the newest).
// The Tree plugin is out of the GPU hot path: it stays on
// the host, and callers may pass their own rsm_tree_root_fn instead.
//
// Also the host form of the namespaced Merkle tree (celestiaorg/nmt v0.24.3, a
// go.mod dependency absent from /root/reference) as rsmt2d's NMT wrappers push it
// (nmtwrapper_test.go:94-120, nmtbuffered_tree_test.go:118-152): see
// rsm_nmt_tree_root below; the device form is kernels_nmt.hip.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#if defined(__x86_64__)
#include <cpuid.h>
#include <immintrin.h>
#endif

#include "../../include/rsmt2d_hip.h"

namespace {

#if defined(__x86_64__)
// SHA-256 compression with the x86 SHA extensions (the GPU box's EPYC and Intel
// hosts since Ice Lake have them): ~5-7x the scalar loop below, which stays as the
// fallback.  The host roots are on the fraud-proof and pre-repair paths.
bool cpu_has_sha_ni() {
    unsigned a = 0, b = 0, c = 0, d = 0;
    if (!__get_cpuid_count(7, 0, &a, &b, &c, &d) || !(b & (1u << 29))) return false;  // SHA
    if (!__get_cpuid(1, &a, &b, &c, &d)) return false;
    return (c & (1u << 19)) && (c & (1u << 9));  // SSE4.1, SSSE3
}

alignas(16) constexpr uint32_t kShaK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__attribute__((target("sha,sse4.1,ssse3"))) void sha256_block_ni(uint32_t h[8], const uint8_t* p) {
    const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bLL, 0x0405060700010203LL);
    __m128i t = _mm_shuffle_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i*>(h)), 0xB1);  // CDAB
    __m128i s1 = _mm_shuffle_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i*>(h + 4)), 0x1B);  // EFGH
    __m128i s0 = _mm_alignr_epi8(t, s1, 8);  // ABEF
    s1 = _mm_blend_epi16(s1, t, 0xF0);        // CDGH
    const __m128i abef = s0, cdgh = s1;
    __m128i w[4];
    for (int g = 0; g < 16; ++g) {  // four rounds per group
        __m128i m;
        if (g < 4) {
            m = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(p + 16 * g)), bswap);
        } else {  // W[t..t+3] from the groups g-4, g-3, g-2, g-1
            m = _mm_sha256msg1_epu32(w[g & 3], w[(g + 1) & 3]);
            m = _mm_add_epi32(m, _mm_alignr_epi8(w[(g + 3) & 3], w[(g + 2) & 3], 4));
            m = _mm_sha256msg2_epu32(m, w[(g + 3) & 3]);
        }
        w[g & 3] = m;
        const __m128i wk = _mm_add_epi32(m, _mm_load_si128(reinterpret_cast<const __m128i*>(kShaK + 4 * g)));
        s1 = _mm_sha256rnds2_epu32(s1, s0, wk);
        s0 = _mm_sha256rnds2_epu32(s0, s1, _mm_shuffle_epi32(wk, 0x0E));
    }
    s0 = _mm_add_epi32(s0, abef);
    s1 = _mm_add_epi32(s1, cdgh);
    t = _mm_shuffle_epi32(s0, 0x1B);      // FEBA
    s1 = _mm_shuffle_epi32(s1, 0xB1);     // DCHG
    s0 = _mm_blend_epi16(t, s1, 0xF0);    // DCBA
    s1 = _mm_alignr_epi8(s1, t, 8);       // HGFE
    _mm_storeu_si128(reinterpret_cast<__m128i*>(h), s0);
    _mm_storeu_si128(reinterpret_cast<__m128i*>(h + 4), s1);
}
const bool kShaNi = cpu_has_sha_ni();

// N independent compressions interleaved (multi-buffer SHA-NI): one message's
// sha256rnds2 chain is latency-bound, N independent chains keep the SHA unit busy.
// Same rounds as sha256_block_ni, per state.
template <int N>
__attribute__((target("sha,sse4.1,ssse3"))) void sha256_blocks_ni(uint32_t (*h)[8], const uint8_t* const* p) {
    const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bLL, 0x0405060700010203LL);
    __m128i s0[N], s1[N], abef[N], cdgh[N], w[N][4];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const __m128i t = _mm_shuffle_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i*>(h[i])), 0xB1);
        const __m128i u = _mm_shuffle_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i*>(h[i] + 4)), 0x1B);
        s0[i] = _mm_alignr_epi8(t, u, 8);
        s1[i] = _mm_blend_epi16(u, t, 0xF0);
        abef[i] = s0[i];
        cdgh[i] = s1[i];
    }
#pragma unroll
    for (int g = 0; g < 16; ++g) {
        const __m128i kg = _mm_load_si128(reinterpret_cast<const __m128i*>(kShaK + 4 * g));
#pragma unroll
        for (int i = 0; i < N; ++i) {
            __m128i m;
            if (g < 4) {
                m = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(p[i] + 16 * g)), bswap);
            } else {
                m = _mm_sha256msg1_epu32(w[i][g & 3], w[i][(g + 1) & 3]);
                m = _mm_add_epi32(m, _mm_alignr_epi8(w[i][(g + 3) & 3], w[i][(g + 2) & 3], 4));
                m = _mm_sha256msg2_epu32(m, w[i][(g + 3) & 3]);
            }
            w[i][g & 3] = m;
            const __m128i wk = _mm_add_epi32(m, kg);
            s1[i] = _mm_sha256rnds2_epu32(s1[i], s0[i], wk);
            s0[i] = _mm_sha256rnds2_epu32(s0[i], s1[i], _mm_shuffle_epi32(wk, 0x0E));
        }
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const __m128i a = _mm_add_epi32(s0[i], abef[i]);
        const __m128i c = _mm_add_epi32(s1[i], cdgh[i]);
        const __m128i t = _mm_shuffle_epi32(a, 0x1B);  // FEBA
        const __m128i u = _mm_shuffle_epi32(c, 0xB1);  // DCHG
        _mm_storeu_si128(reinterpret_cast<__m128i*>(h[i]), _mm_blend_epi16(t, u, 0xF0));      // DCBA
        _mm_storeu_si128(reinterpret_cast<__m128i*>(h[i] + 4), _mm_alignr_epi8(u, t, 8));     // HGFE
    }
}
#endif

struct Sha256 {
    uint32_t h[8];
    uint8_t buf[64];
    uint64_t len = 0;
    size_t blen = 0;

    static constexpr uint32_t K[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
        0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
        0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
        0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
        0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
        0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
        0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
        0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

    Sha256() {
        static constexpr uint32_t H0[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                           0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
        memcpy(h, H0, sizeof(h));
    }
    static inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
    void block(const uint8_t* p) {
#if defined(__x86_64__)
        if (kShaNi) {
            sha256_block_ni(h, p);
            return;
        }
#endif
        uint32_t w[64];
        for (int i = 0; i < 16; ++i)
            w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
        for (int i = 16; i < 64; ++i) {
            uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
            uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
            w[i] = w[i - 16] + s0 + w[i - 7] + s1;
        }
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
        for (int i = 0; i < 64; ++i) {
            uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
            uint32_t ch = (e & f) ^ (~e & g);
            uint32_t t1 = hh + S1 + ch + K[i] + w[i];
            uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
            uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
            uint32_t t2 = S0 + mj;
            hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
    }
    void update(const uint8_t* p, size_t n) {
        len += n;
        if (blen) {
            size_t t = 64 - blen < n ? 64 - blen : n;
            memcpy(buf + blen, p, t);
            blen += t; p += t; n -= t;
            if (blen == 64) { block(buf); blen = 0; }
        }
        while (n >= 64) { block(p); p += 64; n -= 64; }
        if (n) { memcpy(buf, p, n); blen = n; }
    }
    void final(uint8_t out[32]) {
        const uint64_t bits = len * 8;
        uint8_t pad[72] = {0x80};  // 0x80, zeros to 56 mod 64, then the bit length
        const size_t zeros = (blen < 56 ? 56 - blen : 120 - blen) - 1;
        for (int i = 0; i < 8; ++i) pad[1 + zeros + i] = (uint8_t)(bits >> (56 - 8 * i));
        update(pad, 1 + zeros + 8);
        for (int i = 0; i < 8; ++i) {
            out[4 * i] = (uint8_t)(h[i] >> 24); out[4 * i + 1] = (uint8_t)(h[i] >> 16);
            out[4 * i + 2] = (uint8_t)(h[i] >> 8); out[4 * i + 3] = (uint8_t)h[i];
        }
    }
};
constexpr uint32_t Sha256::K[64];

struct Digest { uint8_t b[32]; };

Digest node_hash(const Digest& l, const Digest& r) {
    Sha256 s;
    uint8_t pre = 0x01;
    s.update(&pre, 1);
    s.update(l.b, 32);
    s.update(r.b, 32);
    Digest o;
    s.final(o.b);
    return o;
}

// SHA-256 of prefix || msg[i][0, len) for `count` <= kHashBatch messages of one length,
// compressed side by side (sha256_blocks_ni<kHashBatch>; the scalar Sha256 without the
// SHA extensions).  Block b of a message is assembled in a 64-byte buffer: the 1-byte
// prefix shifts the payload off the block grid.  Eight at a time: one DefaultTree root
// of 256 leaves x 512 B on the GPU box's EPYC 9575F takes 55.8 us against 77 at four
// and 121 one message at a time (profiles/r05p_host_tree.txt).
constexpr int kHashBatch = 8;
void hash_prefixed(uint8_t prefix, const uint8_t* const* msg, int count, uint32_t len, Digest* out) {
#if defined(__x86_64__)
    if (kShaNi) {
        const uint64_t total = 1ull + len, bits = total * 8;
        const uint64_t nblk = (total + 8) / 64 + 1;
        uint32_t h[kHashBatch][8];
        static constexpr uint32_t H0[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                           0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
        for (auto& x : h) memcpy(x, H0, sizeof(H0));
        alignas(16) uint8_t buf[kHashBatch][64];
        const uint8_t* bp[kHashBatch];
        for (int i = 0; i < kHashBatch; ++i) bp[i] = buf[i];
        for (uint64_t b = 0; b < nblk; ++b) {
            const uint64_t t0 = 64 * b;  // message bytes [t0, t0 + 64) of prefix || payload || padding
            for (int i = 0; i < kHashBatch; ++i) {
                const uint8_t* m = msg[i < count ? i : count - 1];
                uint8_t* d = buf[i];
                memset(d, 0, 64);
                // payload byte j sits at message position 1 + j
                const uint64_t lo = t0 > 0 ? t0 - 1 : 0, hi = std::min<uint64_t>(t0 + 63, len);
                if (hi > lo) memcpy(d + (1 + lo - t0), m + lo, hi - lo);
                if (t0 == 0) d[0] = prefix;
                if (total >= t0 && total < t0 + 64) d[total - t0] = 0x80;
                if (b == nblk - 1)
                    for (int q = 0; q < 8; ++q) d[56 + q] = (uint8_t)(bits >> (56 - 8 * q));
            }
            sha256_blocks_ni<kHashBatch>(h, bp);
        }
        for (int i = 0; i < count; ++i)
            for (int q = 0; q < 8; ++q) {
                out[i].b[4 * q] = (uint8_t)(h[i][q] >> 24);
                out[i].b[4 * q + 1] = (uint8_t)(h[i][q] >> 16);
                out[i].b[4 * q + 2] = (uint8_t)(h[i][q] >> 8);
                out[i].b[4 * q + 3] = (uint8_t)h[i][q];
            }
        return;
    }
#endif
    for (int i = 0; i < count; ++i) {
        Sha256 s;
        s.update(&prefix, 1);
        s.update(msg[i], len);
        s.final(out[i].b);
    }
}

// ---- namespaced Merkle tree (celestiaorg/nmt v0.24.3, published algorithm) ----
// A node is minNs || maxNs || digest.  HashLeaf(ndata) = ns || ns || H(0x00 || ndata)
// with ns = ndata[:nsSize]; HashNode(l, r) = l.min || max || H(0x01 || l || r) where
// max = l.max when IgnoreMaxNamespace and r.min is the all-0xFF namespace, else
// r.max; the root over n leaves splits at the largest power of two below n
// (RFC 6962 MTH), i.e. the perfect subtrees of the set bits of n folded from the
// right, as the DefaultTree's stack.  Empty tree: zero namespaces || H("").
// Nodes of a level sit contiguously (2 ns + 32 bytes each), so a pair is already the
// message body 0x01 || l || r; leaves and each level are hashed kHashBatch at a time.
// HashNode's validateSiblingsNamespaceOrder: r.min < l.max is an error.
bool nmt_pair(const uint8_t* l, const uint8_t* r, uint32_t nsz, bool ignore_max, uint8_t* out_ns) {
    const uint8_t *lmin = l, *lmax = l + nsz, *rmin = r, *rmax = r + nsz;
    if (memcmp(lmax, rmin, nsz) > 0) return false;
    bool rmin_is_max = true;
    for (uint32_t i = 0; i < nsz; ++i) rmin_is_max &= rmin[i] == 0xFF;
    memcpy(out_ns, lmin, nsz);
    memcpy(out_ns + nsz, (ignore_max && rmin_is_max) ? lmax : rmax, nsz);
    return true;
}

}  // namespace

extern "C" int rsm_nmt_tree_root(void* user, int /*axis*/, uint32_t index, const uint8_t* const* leaves,
                                 uint32_t n_leaves, uint32_t leaf_size, uint8_t* root_out, uint32_t* root_len) {
    const auto* p = static_cast<const rsm_nmt_params*>(user);
    if (!p || !root_len || !root_out || p->namespace_size == 0 || p->square_size == 0) return RSM_EINVAL;
    const uint32_t nsz = p->namespace_size, k = p->square_size, NB = 2 * nsz + 32;
    const bool ig = p->ignore_max_namespace != 0;
    if (*root_len < NB) return RSM_EINVAL;
    // erasuredNamespacedMerkleTree.Push (nmtwrapper_test.go:94-120)
    if (index + 1 > 2 * k || n_leaves > 2 * k) return RSM_ETREE;  // pushed past predetermined square size
    if (leaf_size < nsz) return RSM_ETREE;                         // data is too short to contain namespace ID
    if (n_leaves == 0) {
        Sha256 s;
        memset(root_out, 0, NB);
        s.final(root_out + 2 * nsz);
        *root_len = NB;
        return RSM_OK;
    }
    std::vector<uint8_t> parity(nsz, 0xFF);
    const size_t ML = (size_t)nsz + leaf_size;  // a leaf's message body: ns || share
    std::vector<uint8_t> msg((size_t)n_leaves * ML), nodes((size_t)n_leaves * NB);
    const uint8_t* prev = nullptr;
    for (uint32_t i = 0; i < n_leaves; ++i) {
        if (!leaves[i]) return RSM_ETREE;
        const uint8_t* ns = (i < k && index < k) ? leaves[i] : parity.data();  // isQuadrantZero
        if (prev && memcmp(ns, prev, nsz) < 0) return RSM_ETREE;           // nmt: ErrInvalidPushOrder
        prev = ns;
        memcpy(&msg[i * ML], ns, nsz);
        memcpy(&msg[i * ML + nsz], leaves[i], leaf_size);
        memcpy(&nodes[(size_t)i * NB], ns, nsz);
        memcpy(&nodes[(size_t)i * NB + nsz], ns, nsz);
    }
    std::vector<Digest> dg(kHashBatch);
    std::vector<uint8_t> nsb((size_t)kHashBatch * 2 * nsz);  // the pairs' new min || max
    for (uint32_t i = 0; i < n_leaves; i += kHashBatch) {
        const int c = (int)std::min<uint32_t>(kHashBatch, n_leaves - i);
        const uint8_t* m[kHashBatch];
        for (int q = 0; q < c; ++q) m[q] = &msg[(size_t)(i + q) * ML];
        hash_prefixed(0x00, m, c, (uint32_t)ML, dg.data());
        for (int q = 0; q < c; ++q) memcpy(&nodes[(size_t)(i + q) * NB + 2 * nsz], dg[q].b, 32);
    }
    std::vector<uint32_t> subs;  // first leaf of each perfect subtree, largest first
    for (uint32_t s0 = 0, bit = 31; s0 < n_leaves; --bit) {
        const uint32_t size = 1u << bit;
        if (!(n_leaves & size)) continue;
        for (uint32_t cnt = size; cnt > 1; cnt /= 2) {  // level by level, in place from node s0
            const uint32_t np = cnt / 2;
            for (uint32_t j = 0; j < np; j += kHashBatch) {
                const int c = (int)std::min<uint32_t>(kHashBatch, np - j);
                const uint8_t* m[kHashBatch];
                for (int q = 0; q < c; ++q) {
                    const uint8_t* l = &nodes[(size_t)(s0 + 2 * (j + q)) * NB];
                    if (!nmt_pair(l, l + NB, nsz, ig, &nsb[(size_t)q * 2 * nsz])) return RSM_ETREE;
                    m[q] = l;
                }
                hash_prefixed(0x01, m, c, 2 * NB, dg.data());  // every pair read before any write
                for (int q = 0; q < c; ++q) {
                    uint8_t* o = &nodes[(size_t)(s0 + j + q) * NB];
                    memcpy(o, &nsb[(size_t)q * 2 * nsz], 2 * nsz);
                    memcpy(o + 2 * nsz, dg[q].b, 32);
                }
            }
        }
        subs.push_back(s0);
        s0 += size;
    }
    std::vector<uint8_t> acc(&nodes[(size_t)subs.back() * NB], &nodes[(size_t)subs.back() * NB] + NB);
    std::vector<uint8_t> pair(2 * NB);
    for (int i = (int)subs.size() - 2; i >= 0; --i) {
        memcpy(pair.data(), &nodes[(size_t)subs[i] * NB], NB);
        memcpy(pair.data() + NB, acc.data(), NB);
        if (!nmt_pair(pair.data(), pair.data() + NB, nsz, ig, acc.data())) return RSM_ETREE;
        const uint8_t* m[1] = {pair.data()};
        hash_prefixed(0x01, m, 1, 2 * NB, dg.data());
        memcpy(acc.data() + 2 * nsz, dg[0].b, 32);
    }
    memcpy(root_out, acc.data(), NB);
    *root_len = NB;
    return RSM_OK;
}

extern "C" int rsm_default_tree_root(void* /*user*/, int /*axis*/, uint32_t /*index*/,
                                     const uint8_t* const* leaves, uint32_t n_leaves, uint32_t leaf_size,
                                     uint8_t* root_out, uint32_t* root_len) {
    if (!root_len || *root_len < 32 || !root_out) return RSM_EINVAL;
    if (n_leaves == 0) {  // merkletree.Root() of an empty tree is nil
        *root_len = 0;
        return RSM_OK;
    }
    for (uint32_t i = 0; i < n_leaves; ++i)
        if (!leaves[i]) return RSM_ETREE;
    // The push/join stack ends as the perfect subtrees of the set bits of n (largest
    // first) folded from the newest: root = node(sub_0, node(sub_1, ... sub_last)).
    // Leaves, then each subtree's levels, are hashed kHashBatch messages at a time.
    std::vector<Digest> d(n_leaves);
    for (uint32_t i = 0; i < n_leaves; i += kHashBatch)
        hash_prefixed(0x00, leaves + i, (int)std::min<uint32_t>(kHashBatch, n_leaves - i), leaf_size, &d[i]);
    std::vector<Digest> subs;
    std::vector<uint8_t> pairs;
    for (uint32_t s0 = 0, bit = 31; s0 < n_leaves; --bit) {
        const uint32_t size = 1u << bit;
        if (!(n_leaves & size)) continue;
        for (uint32_t cnt = size; cnt > 1; cnt /= 2) {  // level by level, in place in d[s0 ..)
            const uint32_t np = cnt / 2;
            pairs.resize((size_t)np * 64);
            for (uint32_t j = 0; j < np; ++j) {
                memcpy(&pairs[(size_t)j * 64], d[s0 + 2 * j].b, 32);
                memcpy(&pairs[(size_t)j * 64 + 32], d[s0 + 2 * j + 1].b, 32);
            }
            for (uint32_t j = 0; j < np; j += kHashBatch) {
                const uint8_t* m[kHashBatch];
                const int c = (int)std::min<uint32_t>(kHashBatch, np - j);
                for (int q = 0; q < c; ++q) m[q] = &pairs[(size_t)(j + q) * 64];
                hash_prefixed(0x01, m, c, 64, &d[s0 + j]);
            }
        }
        subs.push_back(d[s0]);
        s0 += size;
    }
    Digest acc = subs.back();
    for (int i = (int)subs.size() - 2; i >= 0; --i) acc = node_hash(subs[i], acc);
    memcpy(root_out, acc.b, 32);
    *root_len = 32;
    return RSM_OK;
}
