// nmtprobe.hip -- kernels_nmt.hip's nmt_tree_wave_kernel<29, TPW, WPB, F2> over a batch of
// 32 squares' leaf records (W = 256, random leaves: push-order statuses are set, the
// hashing is the same), per shape: trees per wave, waves per workgroup, levels 1-2 fused.
// hip-event averages over back-to-back launches (the upper levels workgroup-cooperative
// since r05aj, so every shape differs from its r05aa figure).  usage: nmtprobe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#include "../../rsmt2d_amd/csrc/kernels_nmt.hip"

using namespace rsm;

template <int T, int B, bool F>
static float run(const uint32_t* d_leaf, uint32_t W, uint32_t squares, uint8_t* d_roots, uint32_t* d_status) {
    const uint32_t blocks = (2 * W + B * T - 1) / (B * T);
    const size_t lds = (size_t)B * wwave_lds_words<29>(W, T, F) * 4u;
    if (lds > 64u * 1024u) return 0.f;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    auto launch = [&] {
        hipLaunchKernelGGL((nmt_tree_wave_kernel<29, T, B, F>), dim3(blocks, squares), dim3(64 * B), lds, 0, d_leaf, W,
                           1u, d_roots, d_status);
    };
    launch();
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < 10; ++i) launch();
    (void)hipEventRecord(b, 0);
    if (hipEventSynchronize(b) != hipSuccess) return -1;
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms * 1e3f / 10;
}

int main() {
    const uint32_t W = 256, squares = 32;
    const size_t cells = (size_t)W * W * squares;
    uint32_t *d_leaf, *d_status;
    uint8_t* d_roots;
    if (hipMalloc(&d_leaf, cells * kLeafWords * 4) != hipSuccess) return 1;
    if (hipMalloc(&d_roots, (size_t)squares * 2 * W * 90) != hipSuccess) return 1;
    if (hipMalloc(&d_status, (size_t)squares * 2 * W * 4) != hipSuccess) return 1;
    std::vector<uint32_t> h(cells * kLeafWords);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (uint32_t)(i * 2654435761u);
    (void)hipMemcpy(d_leaf, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    // every shape gives the same roots
    std::vector<uint8_t> r0((size_t)squares * 2 * W * 90), r1(r0.size());
    run<1, 4, false>(d_leaf, W, squares, d_roots, d_status);
    (void)hipMemcpy(r0.data(), d_roots, r0.size(), hipMemcpyDeviceToHost);
    run<4, 2, true>(d_leaf, W, squares, d_roots, d_status);
    (void)hipMemcpy(r1.data(), d_roots, r1.size(), hipMemcpyDeviceToHost);
    printf("roots (1,4,plain) == (4,2,fused): %s\n", r0 == r1 ? "yes" : "NO");
    printf("us per 32-square launch: (1,4) %.1f  (2,2) %.1f | fused: (1,4) %.1f  (2,2) %.1f  (2,4) %.1f  (4,2) %.1f\n",
           run<1, 4, false>(d_leaf, W, squares, d_roots, d_status), run<2, 2, false>(d_leaf, W, squares, d_roots, d_status),
           run<1, 4, true>(d_leaf, W, squares, d_roots, d_status), run<2, 2, true>(d_leaf, W, squares, d_roots, d_status),
           run<2, 4, true>(d_leaf, W, squares, d_roots, d_status), run<4, 2, true>(d_leaf, W, squares, d_roots, d_status));
    return 0;
}
