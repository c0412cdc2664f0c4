// multi_check.cpp -- TEST INFRASTRUCTURE ONLY (tests/test_multi_cpu.py): the C-ABI
// multi-GPU extension (rsm_multi.cpp, product code) at G = 2, 4, 8 host "devices"
// over the RCCL stub (rccl_stub.cpp) and oracle-backed encode launches
// (hip_stub.cpp built with RSM_STUB_ORACLE), against the oracle's whole-square
// extension (oracle/leopard_oracle.c, the reference 2D schedule).
//   1. rsm_multi_extend_square (host memory in and out) and the in-place pinned form
//      rsm_multi_extend_square_inplace (an rsm_multi_host_alloc EDS whose Q0 quadrant
//      holds the ODS), both schedules: the whole EDS bit-exact;
//   2. rsm_multi_extend_dev (per-GPU buffers holding only their Q0 rows), both
//      schedules: on GPU g its rows of the top half, its column slice of the
//      whole square and (all-gather) the whole top half, bit-exact -- the
//      all-to-all pack/unpack offsets, the copy-free all-to-all (GF(2^16) k = 256 /
//      512: the encoders' side output and blocked inputs, emulated by the stub's
//      oracle launches) and the in-place all-gather layout;
//   3. concurrency (run under ThreadSanitizer by the test): threads extending
//      through one shared clique and through cliques of their own.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/rsmt2d_hip.h"

extern "C" int leo_extend_square(unsigned k, size_t S, const uint8_t* ods, uint8_t* eds, int nthreads);

namespace {
int g_fail = 0;
#define CHECK(c, ...)                                \
    do {                                             \
        if (!(c)) {                                  \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);            \
            fprintf(stderr, "\n");                   \
            ++g_fail;                                \
        }                                            \
    } while (0)

uint64_t g_seed = 0x9E3779B97F4A7C15ull;
uint8_t next_byte(uint64_t& s) {
    s += 0x9E3779B97F4A7C15ull;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return (uint8_t)(z ^ (z >> 31));
}

bool same_rect(const uint8_t* a, const uint8_t* b, size_t row, size_t r0, size_t r1, size_t c0, size_t c1) {
    for (size_t r = r0; r < r1; ++r)
        if (memcmp(a + r * row + c0, b + r * row + c0, c1 - c0) != 0) return false;
    return true;
}

void check_case(int G, uint32_t k, uint32_t S, uint64_t seed) {
    const size_t W = 2ull * k, row = W * S, half = (size_t)k * S;
    std::vector<uint8_t> ods((size_t)k * k * S), want(W * W * S), got(W * W * S);
    uint64_t s = seed;
    for (auto& b : ods) b = next_byte(s);
    CHECK(leo_extend_square(k, S, ods.data(), want.data(), 1) == 0, "oracle");
    std::vector<int> devs(G);
    for (int g = 0; g < G; ++g) devs[g] = g;
    rsm_multi* m = nullptr;
    CHECK(rsm_multi_create(devs.data(), G, &m) == RSM_OK && m, "rsm_multi_create G=%d", G);
    if (!m) return;
    CHECK(rsm_multi_size(m) == G, "size");
    const uint32_t rk = k / G, ck = (uint32_t)(W / G);
    for (int sched : {RSM_SCHED_ALLGATHER, RSM_SCHED_ALLTOALL}) {
        // 1. host memory in and out
        memset(got.data(), 0xA5, got.size());
        int rc = rsm_multi_extend_square(m, ods.data(), k, S, got.data(), sched);
        CHECK(rc == RSM_OK, "extend_square G=%d k=%u sched=%d rc=%d (%s)", G, k, sched, rc, rsm_last_error());
        CHECK(got == want, "host EDS differs G=%d k=%u S=%u sched=%d", G, k, S, sched);
        // 1b. in place, pinned arena
        void* pin = nullptr;
        CHECK(rsm_multi_host_alloc(m, W * W * S, &pin) == RSM_OK && pin, "rsm_multi_host_alloc");
        if (pin) {
            uint8_t* e = static_cast<uint8_t*>(pin);
            memset(e, 0xA5, W * W * S);
            for (uint32_t r = 0; r < k; ++r) memcpy(e + r * row, ods.data() + r * half, half);
            rc = rsm_multi_extend_square_inplace(m, e, k, S, sched);
            CHECK(rc == RSM_OK, "extend_square_inplace G=%d k=%u sched=%d rc=%d (%s)", G, k, sched, rc, rsm_last_error());
            CHECK(memcmp(e, want.data(), W * W * S) == 0, "in-place pinned EDS differs G=%d k=%u S=%u sched=%d", G, k,
                  S, sched);
            CHECK(rsm_multi_host_free(m, pin) == RSM_OK, "rsm_multi_host_free");
        }
        // 2. device-resident: buffer g holds only the Q0 rows of shard g
        std::vector<void*> d(G);
        for (int g = 0; g < G; ++g) {
            CHECK(rsm_dev_alloc(rsm_multi_context(m, g), W * W * S, &d[g]) == RSM_OK, "alloc");
            uint8_t* p = static_cast<uint8_t*>(d[g]);
            memset(p, 0x5A, W * W * S);
            for (uint32_t r = g * rk; r < (g + 1) * rk; ++r) memcpy(p + r * row, ods.data() + r * half, half);
        }
        rc = rsm_multi_extend_dev(m, d.data(), k, S, sched);
        CHECK(rc == RSM_OK, "extend_dev rc=%d (%s)", rc, rsm_last_error());
        CHECK(rsm_multi_sync(m) == RSM_OK, "sync");
        for (int g = 0; g < G; ++g) {
            const uint8_t* p = static_cast<const uint8_t*>(d[g]);
            CHECK(same_rect(p, want.data(), row, (size_t)g * rk, (size_t)(g + 1) * rk, 0, row),
                  "G=%d k=%u sched=%d gpu %d: its rows of the top half", G, k, sched, g);
            // the bottom half of its column slice; the top half's other rows too unless the
            // copy-free all-to-all left them in the receive staging (GF(2^16), blocks >= 32)
            const bool fused = G > 1 && sched == RSM_SCHED_ALLTOALL && k > 128 && k <= 512 && k % 32 == 0 &&
                               rk % 32 == 0 && ck % 32 == 0;
            CHECK(same_rect(p, want.data(), row, fused ? k : 0, W, (size_t)g * ck * S, (size_t)(g + 1) * ck * S),
                  "G=%d k=%u sched=%d gpu %d: its column slice", G, k, sched, g);
            if (sched == RSM_SCHED_ALLGATHER)
                CHECK(same_rect(p, want.data(), row, 0, k, 0, row), "G=%d k=%u gpu %d: all-gathered top half", G, k, g);
            CHECK(rsm_dev_free(rsm_multi_context(m, g), d[g]) == RSM_OK, "free");
        }
    }
    // contract: k not a multiple of G, unknown schedule
    if (G > 1) CHECK(rsm_multi_extend_square(m, ods.data(), k + 1, S, got.data(), 0) == RSM_ESHAPE, "k %% G check");
    CHECK(rsm_multi_extend_square(m, ods.data(), k, S, got.data(), 7) == RSM_EINVAL, "schedule check");
    if (G > 1) CHECK(rsm_multi_extend_square_inplace(m, got.data(), k + 1, S, 0) == RSM_ESHAPE, "in-place k %% G check");
    CHECK(rsm_multi_extend_square_inplace(m, nullptr, k, S, 0) == RSM_EINVAL, "in-place NULL check");
    rsm_multi_destroy(m);
}

void hammer() {
    const uint32_t k = 16, S = 64;
    const size_t W = 2ull * k;
    std::vector<uint8_t> ods((size_t)k * k * S), want(W * W * S);
    uint64_t s = 77;
    for (auto& b : ods) b = next_byte(s);
    leo_extend_square(k, S, ods.data(), want.data(), 1);
    int devs[4] = {0, 1, 2, 3};
    rsm_multi* shared = nullptr;
    CHECK(rsm_multi_create(devs, 4, &shared) == RSM_OK, "shared clique");
    std::vector<std::thread> th;
    std::vector<int> bad(8, 0);
    for (int t = 0; t < 8; ++t)
        th.emplace_back([&, t] {
            rsm_multi* own = nullptr;
            if (t % 2 == 0 && rsm_multi_create(devs, 2, &own) != RSM_OK) {
                bad[t] = 1;
                return;
            }
            std::vector<uint8_t> out(W * W * S);
            for (int i = 0; i < 6; ++i) {
                rsm_multi* m = own ? own : shared;
                if (i % 3 == 2) {  // the in-place form on a buffer holding only the ODS
                    std::fill(out.begin(), out.end(), 0);
                    for (uint32_t r = 0; r < k; ++r) memcpy(out.data() + r * W * S, ods.data() + r * k * S, k * S);
                    if (rsm_multi_extend_square_inplace(m, out.data(), k, S, i & 1) != RSM_OK || out != want) bad[t] = 1;
                } else if (rsm_multi_extend_square(m, ods.data(), k, S, out.data(), i & 1) != RSM_OK || out != want) {
                    bad[t] = 1;
                }
            }
            rsm_multi_destroy(own);
        });
    for (auto& x : th) x.join();
    for (int t = 0; t < 8; ++t) CHECK(!bad[t], "hammer thread %d", t);
    rsm_multi_destroy(shared);
}
}  // namespace

int main(int argc, char** argv) {
    const bool quick = argc > 1 && strcmp(argv[1], "quick") == 0;  // (the TSan run: small shapes only)
    for (int G : {2, 4, 8})
        for (uint32_t k : {8u, 64u}) check_case(G, k, 64, g_seed + G * 131 + k);
    check_case(2, 256, 64, 4242);  // GF(2^16) (2k > 256) through the same exchange
    // the all-to-all without copies (shard_fused_ok: GF(2^16), blocks of >= 32 rows / columns):
    // the row pass's side output and the column pass's blocked inputs
    check_case(4, 256, 64, 4343);
    if (!quick) {
        check_case(8, 256, 128, 4444);
        check_case(8, 512, 64, 4545);  // config 5's shape over 8 GPUs
    }
    check_case(1, 8, 64, 99);      // the clique of one (what the GPU test runs)
    hammer();
    if (g_fail) {
        fprintf(stderr, "multi_check: %d failures\n", g_fail);
        return 1;
    }
    printf("multi_check: ok\n");
    return 0;
}
