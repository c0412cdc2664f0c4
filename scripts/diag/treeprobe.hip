// treeprobe.hip -- kernels_sha.hip's DefaultTree tree kernel at one, two and four
// trees per wave, on one square (a latency launch: the Repair tail, one square's
// roots) and on a batch (rsm_roots_squares_dev).  Times are hip-event averages
// over back-to-back launches; the first lines check that the forms agree.
// Round-5 finding behind it (shaprobe.hip, profiles/r05j_sha_lanes.txt): a wave
// with <= 8 of its 64 lanes active runs SHA compressions 2-3.5x slower than a full
// wave, and the upper levels of a tree had 1-32 active lanes.  C = 1: the
// workgroup-cooperative top levels (COOP, the batch form since r05aj).
// usage: treeprobe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#include "../../rsmt2d_amd/csrc/kernels_sha.hip"

using namespace rsm;

template <typename F>
static float timed(F&& launch, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 2; ++i) launch();
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i) launch();
    (void)hipEventRecord(b, 0);
    if (hipEventSynchronize(b) != hipSuccess) return -1;
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return ms * 1e3f / reps;
}

template <int TPW, bool C = false>
static float tree(const uint32_t* d_leaf, uint32_t W, uint32_t squares, uint8_t* d_roots, int reps) {
    const uint32_t count = 2 * W;
    const uint32_t blocks = (count + kTreesPerBlock * TPW - 1) / (kTreesPerBlock * TPW);
    const size_t lds = (size_t)kTreesPerBlock * TPW * tree_lds_words(W) * 4u;
    if (lds > 52u * 1024u) return 0.f;  // the production launcher's LDS cap
    return timed([&] {
        hipLaunchKernelGGL((tree_root_kernel<TPW, C>), dim3(blocks, squares), dim3(256), lds, 0, d_leaf, W, d_roots, 0u,
                           count);
    }, reps);
}

int main() {
    const uint32_t W = 256, batch = 16;
    uint32_t* d_leaf;
    uint8_t* d_roots;
    const size_t cells = (size_t)W * W * batch;
    if (hipMalloc(&d_leaf, cells * 32) != hipSuccess) return 1;
    if (hipMalloc(&d_roots, (size_t)batch * 2 * W * 32) != hipSuccess) return 1;
    std::vector<uint32_t> h(cells * 8);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (uint32_t)(i * 2654435761u);
    (void)hipMemcpy(d_leaf, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    // one and two trees per wave, plain and cooperative, agree
    for (uint32_t w : {2u, 6u, 8u, 10u, 200u, 256u}) {
        std::vector<uint8_t> r0(2 * w * 32), r1(2 * w * 32), r2(2 * w * 32), r3(2 * w * 32);
        tree<2>(d_leaf, w, 1, d_roots, 1);
        (void)hipMemcpy(r0.data(), d_roots, r0.size(), hipMemcpyDeviceToHost);
        tree<1>(d_leaf, w, 1, d_roots, 1);
        (void)hipMemcpy(r1.data(), d_roots, r1.size(), hipMemcpyDeviceToHost);
        tree<2, true>(d_leaf, w, 1, d_roots, 1);
        (void)hipMemcpy(r2.data(), d_roots, r2.size(), hipMemcpyDeviceToHost);
        tree<4, true>(d_leaf, w, 1, d_roots, 1);
        (void)hipMemcpy(r3.data(), d_roots, r3.size(), hipMemcpyDeviceToHost);
        printf("W %u: tpw1 == tpw2 == coop2 == coop4 roots: %s\n", w, r0 == r1 && r1 == r2 && r2 == r3 ? "yes" : "NO");
    }
    for (uint32_t w : {8u, 64u, 256u, 512u})
        printf("tree, one square, W %3u: tpw1 %.1f tpw2 %.1f tpw4 %.1f | coop tpw1 %.1f tpw2 %.1f us\n", w,
               tree<1>(d_leaf, w, 1, d_roots, 20), tree<2>(d_leaf, w, 1, d_roots, 20), tree<4>(d_leaf, w, 1, d_roots, 20),
               tree<1, true>(d_leaf, w, 1, d_roots, 20), tree<2, true>(d_leaf, w, 1, d_roots, 20));
    printf("tree, %u squares, W 256: tpw2 %.2f tpw1 %.2f | coop tpw2 %.2f tpw1 %.2f us per square\n", batch,
           tree<2>(d_leaf, W, batch, d_roots, 10) / batch, tree<1>(d_leaf, W, batch, d_roots, 10) / batch,
           tree<2, true>(d_leaf, W, batch, d_roots, 10) / batch, tree<1, true>(d_leaf, W, batch, d_roots, 10) / batch);
    return 0;
}
