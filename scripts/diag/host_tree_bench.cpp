// host_tree_bench.cpp -- diagnostic: time rsm_default_tree_root (merkle.cpp) over 256 leaves x
// 512 B.  Build: g++ -O2 -std=c++20 -I/opt/rocm/include -D__HIP_PLATFORM_AMD__
//   scripts/diag/host_tree_bench.cpp rsmt2d_amd/csrc/merkle.cpp -o scripts/diag/host_tree_bench
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <cstring>
extern "C" int rsm_default_tree_root(void*, int, uint32_t, const uint8_t* const*, uint32_t, uint32_t, uint8_t*, uint32_t*);
extern "C" int rsm_nmt_tree_root(void*, int, uint32_t, const uint8_t* const*, uint32_t, uint32_t, uint8_t*, uint32_t*);
struct NmtP { uint32_t namespace_size, ignore_max_namespace, square_size; };  // rsm_nmt_params
int main() {
    const int n = 256, S = 512;
    std::vector<uint8_t> buf(n * S);
    for (size_t i = 0; i < buf.size(); ++i) buf[i] = (uint8_t)(i * 131 + 7);
    std::vector<const uint8_t*> p(n);
    for (int i = 0; i < n; ++i) p[i] = &buf[i * S];
    uint8_t out[64]; uint32_t len = 64;
    for (int r = 0; r < 50; ++r) { len = 64; rsm_default_tree_root(nullptr, 0, 0, p.data(), n, S, out, &len); }
    auto t0 = std::chrono::steady_clock::now();
    const int R = 2000;
    for (int r = 0; r < R; ++r) { len = 64; rsm_default_tree_root(nullptr, 0, 0, p.data(), n, S, out, &len); }
    double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / R;
    printf("%.1f us per root; root %02x%02x%02x%02x\n", us, out[0], out[1], out[2], out[3]);
    // NMT (29-byte namespaces, k = 128, row 7: the first 128 leaves Q0 with ascending namespaces)
    for (int i = 0; i < n; ++i)
        for (int b = 0; b < 29; ++b) buf[i * S + b] = b == 28 ? (uint8_t)i : 0;
    NmtP np{29, 1, 128};
    uint8_t nout[128];
    for (int r = 0; r < 50; ++r) { len = 128; rsm_nmt_tree_root(&np, 0, 7, p.data(), n, S, nout, &len); }
    t0 = std::chrono::steady_clock::now();
    int rc = 0;
    for (int r = 0; r < R; ++r) { len = 128; rc |= rsm_nmt_tree_root(&np, 0, 7, p.data(), n, S, nout, &len); }
    us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / R;
    printf("NMT: %.1f us per root (rc %d, len %u); digest %02x%02x%02x%02x\n", us, rc, len, nout[58], nout[59], nout[60], nout[61]);
}
