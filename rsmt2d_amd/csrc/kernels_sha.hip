// kernels_sha.hip -- row and column Merkle roots of a device-resident EDS.
//
// computeRoots / getRowRoot / getColRoot (datasquare.go:218-327)
// with rsmt2d's DefaultTree (tree.go:32-59): celestiaorg/merkletree over SHA-256,
//   leaf = SHA256(0x00 || share),  node = SHA256(0x01 || left || right),
// and for a leaf count that is not a power of two the NebulousLabs stack order:
// perfect subtrees for the set bits of n (largest first), folded from the right
//   root = node(sub_hi, node(sub_mid, ... sub_lo)).
// Host restatement: merkle.cpp (rsm_default_tree_root); tests compare both with
// Python hashlib.
//
// Two kernels:
//   leaf_hash_kernel : one thread per cell, streams its share through SHA-256
//                      (S/64 + 1 blocks); the digest of a cell serves both its row
//                      tree and its column tree.
//   tree_root_kernel : a few trees per wave (2W trees), levels in place in LDS.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "sha256_dev.hpp"

namespace rsm {

namespace {

// SHA256(0x01 || L || R) for digests held as 8 big-endian words each.
__device__ __forceinline__ void node_hash(const uint32_t (&L)[8], const uint32_t (&R)[8], uint32_t (&out)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = kH0[i];
    uint32_t w[16];
    w[0] = shift8(0x01u, L[0]);
#pragma unroll
    for (int i = 1; i < 8; ++i) w[i] = shift8(L[i - 1], L[i]);
    w[8] = shift8(L[7], R[0]);
#pragma unroll
    for (int i = 1; i < 8; ++i) w[8 + i] = shift8(R[i - 1], R[i]);
    sha_block(out, w);
    w[0] = (R[7] << 24) | 0x00800000u;
#pragma unroll
    for (int i = 1; i < 15; ++i) w[i] = 0;
    w[15] = 65u * 8u;
    sha_block(out, w);
}

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// leaf[cell][8] = SHA256(0x00 || share(cell)), cell = row * W + col.
__global__ __launch_bounds__(256) void leaf_hash_kernel(const uint8_t* __restrict__ eds, uint32_t cells,
                                                        uint32_t S, uint32_t* __restrict__ leaf) {
    const uint32_t cell = blockIdx.x * 256u + threadIdx.x;
    if (cell >= cells) return;
    const v4u* p = reinterpret_cast<const v4u*>(eds + (uint64_t)cell * S);
    uint32_t h[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = kH0[i];
    uint32_t prev = 0;  // the 0x00 leaf prefix
    for (uint32_t blk = 0; blk < S / 64u; ++blk) {
        uint32_t w[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const v4u v = p[blk * 4u + q];  // plain load: the other half of the 128-B line is the next block
            const uint32_t b0 = __builtin_bswap32(v.x), b1 = __builtin_bswap32(v.y);
            const uint32_t b2 = __builtin_bswap32(v.z), b3 = __builtin_bswap32(v.w);
            w[4 * q + 0] = shift8(prev, b0);
            w[4 * q + 1] = shift8(b0, b1);
            w[4 * q + 2] = shift8(b1, b2);
            w[4 * q + 3] = shift8(b2, b3);
            prev = b3;
        }
        sha_block(h, w);
    }
    uint32_t w[16];
    w[0] = (prev << 24) | 0x00800000u;  // last share byte, then the 0x80 pad byte
#pragma unroll
    for (int i = 1; i < 15; ++i) w[i] = 0;
    w[15] = (S + 1u) * 8u;
    sha_block(h, w);
    v4u* o = reinterpret_cast<v4u*>(leaf + (uint64_t)cell * 8u);
    o[0] = v4u{h[0], h[1], h[2], h[3]};
    o[1] = v4u{h[4], h[5], h[6], h[7]};
}

constexpr uint32_t kMaxLevel1 = 1024;  // W <= 2048
constexpr uint32_t kTreesPerBlock = 4;  // one wave per tree

// LDS bytes of one tree: level-1 digests (W/2) in place, plus the carried
// subtrees of the odd levels (16 digests)
__host__ __device__ constexpr uint32_t tree_lds_words(uint32_t W) { return (W / 2) * 8u + 16u * 8u; }

// TPW trees per WAVE (four waves per 256-thread workgroup): trees
// (blockIdx.x * 4 + wave) * TPW + u (u < TPW) + first (< W: row tree, else column
// tree) of square blockIdx.y.  A wave's trees are built level by level together
// (node (u, j) of a level is lane-slot u * cnt + j), in place in the wave's own LDS
// (a level's reads all precede its writes: node j reads 2j and 2j + 1 >= j), with
// no workgroup barrier: the many waves of a CU interleave their dependent SHA
// rounds, and packing TPW trees keeps the upper levels' lanes busy (the
// level-by-level workgroup form left most lanes idle behind __syncthreads: 3x
// slower).  roots: [squares][2][W][32] bytes (big-endian digest bytes, as
// Tree.Root() returns them).
// COOP (batches): once a wave's TPW trees have fewer than 64 nodes in a level, the
// workgroup's 4 TPW trees are built together instead -- node U * cnt + j of the
// workgroup (tree U, whose LDS is U tree-slots from the workgroup's first) on lane
// (U * cnt + j) mod 64 of wave (U * cnt + j) / 64, a barrier between a level's reads
// and its writes, waves past the level's last node idle.  At W = 256 and TPW = 2 the
// workgroup then issues 34 wave-passes of two compressions for its 8 trees instead
// of 48 (each wave's own top five levels were one pass each for 32 .. 2 nodes), and
// a SIMD's SHA throughput is its issued wave-passes (kernels_sha.hip above).  The
// launcher uses COOP for every form (one square's depth is the same either way).
template <int TPW, bool COOP>
__global__ __launch_bounds__(256) void tree_root_kernel(const uint32_t* __restrict__ leaf, uint32_t W,
                                                        uint8_t* __restrict__ roots, uint32_t first, uint32_t count) {
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t tw0 = blockIdx.x * kTreesPerBlock * TPW;  // the workgroup's first tree
    const uint32_t t0 = tw0 + wv * TPW;
    if (!COOP && t0 >= count) return;  // whole wave (no workgroup barrier without COOP)
    const uint32_t nt = t0 >= count ? 0u : (count - t0 < (uint32_t)TPW ? count - t0 : (uint32_t)TPW);
    const uint32_t ntw = count - tw0 < kTreesPerBlock * TPW ? count - tw0 : kTreesPerBlock * TPW;
    leaf += (uint64_t)blockIdx.y * W * W * 8u;
    roots += (uint64_t)blockIdx.y * 2u * W * 32u;
    extern __shared__ uint32_t lds_raw[];
    // tree U of the workgroup (wave U / TPW, its tree U % TPW)
    auto tlvl = [&](uint32_t U) { return lds_raw + (size_t)U * tree_lds_words(W); };
    auto tsub = [&](uint32_t U) { return tlvl(U) + (W / 2) * 8u; };
    auto sub = [&](uint32_t u) { return tsub(wv * TPW + u); };
    const uint32_t n = W;
    auto leaf_at = [&](uint32_t tree, uint32_t pos, uint32_t (&d)[8]) {
        const uint32_t axis = tree >= W ? 1u : 0u, idx = tree - axis * W;
        const uint64_t cell = axis == 0 ? (uint64_t)idx * W + pos : (uint64_t)pos * W + idx;
        const v4u* s = reinterpret_cast<const v4u*>(leaf + cell * 8u);
        const v4u a = s[0], b = s[1];
        d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w; d[4] = b.x; d[5] = b.y; d[6] = b.z; d[7] = b.w;
    };
    // children 2j, 2j + 1 of node j of workgroup tree U at height hgt
    auto children = [&](uint32_t U, uint32_t j, uint32_t hgt, uint32_t (&L)[8], uint32_t (&R)[8]) {
        if (hgt == 1) {
            leaf_at(tw0 + first + U, 2 * j, L);
            leaf_at(tw0 + first + U, 2 * j + 1, R);
        } else {
            const uint32_t* lv = tlvl(U);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                L[i] = lv[(2 * j) * 8u + i];
                R[i] = lv[(2 * j + 1) * 8u + i];
            }
        }
    };
    // node j of workgroup tree U (own: this lane's node; else a repeat, to the spare
    // slot); the last node of an odd level is also the carried subtree of its height
    auto put = [&](uint32_t U, uint32_t j, uint32_t hgt, uint32_t cnt, bool own, const uint32_t (&o)[8]) {
        uint32_t* dst = own ? tlvl(U) + j * 8u : tsub(U) + 15u * 8u;
#pragma unroll
        for (int i = 0; i < 8; ++i) dst[i] = o[i];
        if (own && (cnt & 1u) && j == cnt - 1) {
#pragma unroll
            for (int i = 0; i < 8; ++i) tsub(U)[hgt * 8u + i] = o[i];
        }
    };
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    if ((n & 1u) && lane < nt) {  // height-0 subtree: the last leaf
        uint32_t d[8];
        leaf_at(t0 + first + lane, n - 1, d);
#pragma unroll
        for (int i = 0; i < 8; ++i) sub(lane)[i] = d[i];
    }
    for (uint32_t hgt = 1; (n >> hgt) > 0; ++hgt) {
        const uint32_t cnt = n >> hgt;
        if (COOP && (uint32_t)TPW * cnt < 64u) {
            // the workgroup's trees together: at most one pass per wave (4 TPW cnt < 256)
            const uint32_t tot = ntw * cnt, v0 = wv * 64u;
            __syncthreads();  // the previous level's nodes (any wave's) are written
            uint32_t U = 0, j = 0, o[8];
            bool own = false;
            if (v0 < tot) {
                const uint32_t rem = tot - v0;  // every lane of a working wave hashes, as below
                own = lane < rem;
                const uint32_t v = v0 + (own ? lane : lane % rem);
                U = v / cnt;
                j = v - U * cnt;
                uint32_t L[8], R[8];
                children(U, j, hgt, L, R);
                node_hash(L, R, o);
            }
            __syncthreads();  // every read of this level precedes its in-place writes
            if (v0 < tot) put(U, j, hgt, cnt, own, o);
            continue;
        }
        const uint32_t tot = nt * cnt;
        for (uint32_t v0 = 0; v0 < tot; v0 += 64u) {
            // Every lane hashes: past the level's last node a lane repeats node
            // v0 + lane % rem and stores it to the tree's spare slot (sub slot 15:
            // heights stay below 12), so the compiler cannot shrink the hash to the
            // owning lanes.  A wave with <= 8 of its lanes active runs its SHA
            // rounds 2-3.5x slower per compression than a full wave
            // (profiles/r05j_sha_lanes.txt), and a tree's upper levels have 1-8
            // nodes.
            const uint32_t rem = tot - v0;
            const bool own = lane < rem;
            const uint32_t v = v0 + (own ? lane : lane % rem);
            const uint32_t u = v / cnt, j = v - u * cnt;
            uint32_t L[8], R[8], o[8];
            children(wv * TPW + u, j, hgt, L, R);
            node_hash(L, R, o);
            put(wv * TPW + u, j, hgt, cnt, own, o);
        }
        wave_sync();
    }
    if constexpr (COOP) {
        __syncthreads();  // the top levels' nodes and carried subtrees, from any wave
        if (nt == 0) return;
    }
    {  // fold the carried subtrees (a W that is not a power of two); all lanes, as above
        const uint32_t ul = lane % nt;
        const uint32_t tree = t0 + first + ul;
        const uint32_t axis = tree >= W ? 1u : 0u, idx = tree - axis * W;
        const uint32_t* sb = sub(ul);
        uint32_t acc[8];
        const int lo = __builtin_ctz(n);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = sb[lo * 8 + i];
        for (int hgt = lo + 1; hgt < 16; ++hgt) {
            if (!((n >> hgt) & 1u)) continue;
            uint32_t L[8], o[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) L[i] = sb[hgt * 8 + i];
            node_hash(L, acc, o);
#pragma unroll
            for (int i = 0; i < 8; ++i) acc[i] = o[i];
        }
        // lane ul + nt i writes word i of its tree's root: one store instruction covers the
        // wave's nt consecutive roots (coalesced -- also when `roots` is host memory, as
        // Repair's checks pass it)
        const uint32_t wi = lane / nt;
        if (wi < 8u) {
            uint32_t x = acc[0];
#pragma unroll
            for (int i = 1; i < 8; ++i) x = wi == (uint32_t)i ? acc[i] : x;
            uint32_t* r = reinterpret_cast<uint32_t*>(roots + ((uint64_t)axis * W + idx) * 32u);
            r[wi] = __builtin_bswap32(x);
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) sub(ul)[15u * 8u + i] = acc[i];  // keeps every lane hashing
        }
    }
}

// trees per wave: as many as keep four waves' LDS within a third of the CU (so
// three workgroups share it), at least one.  A latency launch (one square's 2W
// trees, too few waves to fill the chip) takes one tree per wave: a lone wave's
// compressions run back to back, so the launch time is the tree depth in
// compressions per lane -- at W = 256, 18 (two level-1 nodes per lane, then one
// per level) against 24 at two trees per wave.
inline uint32_t trees_per_wave(uint32_t W) {
    for (uint32_t t = 4; t > 1; t >>= 1)
        if ((size_t)kTreesPerBlock * t * tree_lds_words(W) * 4u <= 52u * 1024u) return t;
    return 1;
}
hipError_t launch_tree_kernel(const uint32_t* d_leaf, uint32_t W, uint8_t* d_roots, uint32_t first, uint32_t count,
                              uint32_t squares, bool latency, hipStream_t st) {
    const uint32_t tpw = latency ? 1u : trees_per_wave(W);
    const uint32_t blocks = (count + kTreesPerBlock * tpw - 1) / (kTreesPerBlock * tpw);
    const size_t lds = (size_t)kTreesPerBlock * tpw * tree_lds_words(W) * 4u;
    const dim3 grid(blocks, squares);
    // (the cooperative upper levels in every form: one square's depth is the same either
    // way -- W = 256: 53.6 against 54.6 us -- and a wide square's many trees, W = 1024:
    // 2048 waves on 1024 SIMDs, need fewer wave-passes; profiles/r05av_eds_roots.json)
    if (tpw == 4)
        hipLaunchKernelGGL((tree_root_kernel<4, true>), grid, dim3(256), lds, st, d_leaf, W, d_roots, first, count);
    else if (tpw == 2)
        hipLaunchKernelGGL((tree_root_kernel<2, true>), grid, dim3(256), lds, st, d_leaf, W, d_roots, first, count);
    else
        hipLaunchKernelGGL((tree_root_kernel<1, true>), grid, dim3(256), lds, st, d_leaf, W, d_roots, first, count);
    return hipGetLastError();
}

}  // namespace

bool roots_dev_supported(uint32_t W) { return W >= 2 && W <= 2 * kMaxLevel1 && W < (1u << 16); }

// `squares` consecutive [W][W][S] squares; d_leaf: scratch of squares*W*W*32 bytes.
// The cells of all squares are one leaf launch (a single square is only W*W
// threads: one wave per SIMD on a 256-CU chip, latency-bound SHA rounds).
hipError_t launch_roots(const uint8_t* d_eds, uint32_t W, uint32_t S, uint32_t squares, uint32_t* d_leaf,
                        uint8_t* d_roots, hipStream_t st) {
    const uint32_t cells = W * W * squares;
    hipLaunchKernelGGL(leaf_hash_kernel, dim3((cells + 255) / 256), dim3(256), 0, st, d_eds, cells, S, d_leaf);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_tree_kernel(d_leaf, W, d_roots, 0u, 2 * W, squares, squares == 1, st);
}

// Pieces of launch_roots for one square, so a caller can hash rows as they become
// final: leaf digests of `cells` consecutive cells (d_cells -> d_leaf, both already
// offset to the first cell), and the trees [first, first + count) (row trees 0..W-1,
// column trees W..2W-1) over a complete leaf array.
hipError_t launch_leaf_hashes(const uint8_t* d_cells, uint32_t cells, uint32_t S, uint32_t* d_leaf, hipStream_t st) {
    if (cells == 0) return hipSuccess;
    hipLaunchKernelGGL(leaf_hash_kernel, dim3((cells + 255) / 256), dim3(256), 0, st, d_cells, cells, S, d_leaf);
    return hipGetLastError();
}
hipError_t launch_tree_roots(const uint32_t* d_leaf, uint32_t W, uint32_t first, uint32_t count, uint8_t* d_roots,
                             hipStream_t st) {
    if (count == 0) return hipSuccess;
    return launch_tree_kernel(d_leaf, W, d_roots, first, count, 1, true, st);
}

}  // namespace rsm
