"""Generate scratch/treestamp.hip: a copy of kernels_sha.hip's tree_root_kernel with an
s_memtime stamp per level per wave (and the wave's XCC / HW_ID), plus a driver that
launches it on one square (W = 8, 64, 256) and prints per-level tick deltas (median
and max over waves).  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o
scripts/diag/treestamp scratch/treestamp.hip.  The kernel text is read from the
product source at generation time, so the stamps measure the current kernel."""
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
src = open(os.path.join(ROOT, "rsmt2d_amd/csrc/kernels_sha.hip")).read()
a = src.index("template <int TPW>\n__global__ __launch_bounds__(256) void tree_root_kernel")
b = src.index("// trees per wave:")
body = src[a:b]
body = body.replace("void tree_root_kernel(", "void tree_stamp_kernel(uint32_t* __restrict__ stamps, ")
body = body.replace("    extern __shared__ uint32_t lds_raw[];", """    extern __shared__ uint32_t lds_raw[];
    const uint64_t ts0 = __builtin_amdgcn_s_memtime();
    uint32_t* stp = stamps + (size_t)(blockIdx.x * 4 + wv) * 20;
    if (lane == 0) {
        stp[17] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
        stp[18] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    }""", 1)
n = body.count("        wave_sync();\n    }")
assert n == 1, n
body = body.replace("        wave_sync();\n    }", """        wave_sync();
        if (lane == 0) stp[hgt] = (uint32_t)(__builtin_amdgcn_s_memtime() - ts0);
    }""")
assert body.rstrip().endswith("}")
body = body.rstrip()[:-1] + "    if (lane == 0) stp[16] = (uint32_t)(__builtin_amdgcn_s_memtime() - ts0);\n}\n"

driver = r'''
#include <algorithm>
#include <cstdio>
#include <vector>
int main() {
    const uint32_t Wmax = 256;
    uint32_t *d_leaf, *d_st;
    uint8_t* d_roots;
    if (hipMalloc(&d_leaf, (size_t)Wmax * Wmax * 32) != hipSuccess) return 1;
    if (hipMalloc(&d_roots, (size_t)2 * Wmax * 32) != hipSuccess) return 1;
    if (hipMalloc(&d_st, (size_t)2 * Wmax * 20 * 4) != hipSuccess) return 1;
    std::vector<uint32_t> h((size_t)Wmax * Wmax * 8);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (uint32_t)(i * 2654435761u);
    (void)hipMemcpy(d_leaf, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    for (uint32_t W : {8u, 64u, 256u}) {
        const uint32_t count = 2 * W, blocks = (count + 3) / 4, waves = blocks * 4;
        const size_t lds = 4 * rsm::tree_lds_words(W) * 4u;
        int levels = 0;
        while ((W >> (levels + 1)) > 0) ++levels;
        for (int rep = 0; rep < 4; ++rep) {
            (void)hipMemset(d_st, 0, (size_t)2 * Wmax * 20 * 4);
            hipEvent_t a, b;
            (void)hipEventCreate(&a);
            (void)hipEventCreate(&b);
            (void)hipEventRecord(a, 0);
            hipLaunchKernelGGL(rsm::tree_stamp_kernel<1>, dim3(blocks, 1), dim3(256), lds, 0, d_st, d_leaf, W, d_roots,
                               0u, count);
            (void)hipEventRecord(b, 0);
            if (hipEventSynchronize(b) != hipSuccess) return 1;
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            std::vector<uint32_t> st((size_t)waves * 20);
            (void)hipMemcpy(st.data(), d_st, st.size() * 4, hipMemcpyDeviceToHost);
            printf("W %u rep %d: %.1f us; per-level ticks (median / max over %u waves):", W, rep, ms * 1e3, waves);
            for (int l = 1; l <= levels + 1; ++l) {
                std::vector<uint32_t> d;
                for (uint32_t w = 0; w < waves; ++w) {
                    const uint32_t* s = &st[(size_t)w * 20];
                    const uint32_t cur = l <= levels ? s[l] : s[16];
                    d.push_back(cur - (l > 1 ? s[l - 1] : 0));
                }
                std::sort(d.begin(), d.end());
                printf(" %s%u/%u", l <= levels ? "" : "fold ", d[d.size() / 2], d.back());
            }
            printf("\n");
        }
    }
    return 0;
}
'''
out = os.path.join(ROOT, "scratch", "treestamp.hip")
os.makedirs(os.path.dirname(out), exist_ok=True)
with open(out, "w") as f:
    f.write('#include "%s"\n' % os.path.join(ROOT, "rsmt2d_amd/csrc/kernels_sha.hip"))
    f.write("namespace rsm {\nnamespace {\n" + body + "}\n}\n" + driver)
print(out)
