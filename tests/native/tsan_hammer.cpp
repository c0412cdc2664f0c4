// tsan_hammer.cpp -- TEST INFRASTRUCTURE ONLY (tests/test_tsan_cpu.py): many host
// threads on ONE context, as rsmt2d's goroutines use the Codec
// (extendeddatasquare.go:186-224, extendeddatacrossword.go:372-425): Encode and
// Decode of GF(2^8) and GF(2^16) codewords, host-memory extensions, device-resident
// extensions and device roots on caller streams, stream create/destroy and a Repair,
// all at once.  Built with -fsanitize=thread against tests/native/hip_stub.cpp;
// the sanitizer's report (none expected) is the result.
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/rsmt2d_hip.h"

#define CHECK(x)                                                                   \
    do {                                                                           \
        int rc_ = (x);                                                             \
        if (rc_ != 0) {                                                            \
            fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #x, rc_, \
                    rsm_last_error());                                             \
            failed = 1;                                                            \
        }                                                                          \
    } while (0)

static int failed = 0;

int main() {
    rsm_ctx* ctx = nullptr;
    CHECK(rsm_ctx_create(0, &ctx));
    if (!ctx) return 1;
    std::vector<std::thread> th;
    for (int t = 0; t < 64; ++t)
        th.emplace_back([ctx, t] {
            const uint32_t k = (t % 3 == 0) ? 200 : (t % 3 == 1 ? 128 : 16), S = 64;
            std::vector<uint8_t> data((size_t)2 * k * S, (uint8_t)t), par((size_t)k * S);
            std::vector<const uint8_t*> dp(k);
            std::vector<uint8_t*> pp(k), sh(2 * k);
            std::vector<uint8_t> pres(2 * k, 1);
            for (uint32_t i = 0; i < k; ++i) dp[i] = data.data() + (size_t)i * S, pp[i] = par.data() + (size_t)i * S;
            for (uint32_t i = 0; i < 2 * k; ++i) sh[i] = data.data() + (size_t)i * S;
            for (uint32_t i = 0; i < k; i += 2) pres[i] = 0;
            for (int it = 0; it < 8; ++it) {
                CHECK(rsm_encode(ctx, dp.data(), k, S, pp.data()));
                CHECK(rsm_decode(ctx, sh.data(), pres.data(), 2 * k, S));
            }
        });
    for (int t = 0; t < 4; ++t)
        th.emplace_back([ctx, t] {
            const uint32_t k = t % 2 ? 8 : 130, S = 64, W = 2 * k;
            void* st = nullptr;
            CHECK(rsm_stream_create(ctx, &st));
            void *d = nullptr, *roots = nullptr;
            CHECK(rsm_dev_alloc(ctx, (uint64_t)W * W * S, &d));
            CHECK(rsm_dev_alloc(ctx, (uint64_t)2 * W * 32, &roots));
            std::vector<uint8_t> ods((size_t)k * k * S, 3), eds((size_t)W * W * S);
            for (int it = 0; it < 4; ++it) {
                CHECK(rsm_extend_squares_dev(ctx, d, k, S, 1, st));
                CHECK(rsm_roots_dev(ctx, d, W, S, roots, st));
                CHECK(rsm_extend_square(ctx, ods.data(), k, S, eds.data()));
                CHECK(rsm_extend_squares_host(ctx, ods.data(), k, S, 1, eds.data()));
            }
            CHECK(rsm_stream_sync(st));
            CHECK(rsm_dev_free(ctx, d));
            CHECK(rsm_dev_free(ctx, roots));
            CHECK(rsm_stream_destroy(ctx, st));
        });
    // multi-lane host extensions (count = 3 takes 3 lanes at once) from 16 threads while
    // the 64 Codec threads above hold lanes too: with lanes taken one at a time, 11+
    // such callers could each hold some lanes and wait forever for the rest (ADVICE
    // round 2); acquire_lanes takes all of a call's lanes in one step
    for (int t = 0; t < 16; ++t)
        th.emplace_back([ctx, t] {
            const uint32_t k = 8, S = 64, W = 2 * k, n = 3;
            std::vector<uint8_t> ods((size_t)n * k * k * S, (uint8_t)(t + 1)), eds((size_t)n * W * W * S);
            for (int it = 0; it < 6; ++it) CHECK(rsm_extend_squares_host(ctx, ods.data(), k, S, n, eds.data()));
        });
    th.emplace_back([ctx] {  // EDS layer: compute, roots, import with holes, Repair
        const uint32_t k = 4, S = 64, W = 2 * k;
        std::vector<std::vector<uint8_t>> shares(k * k, std::vector<uint8_t>(S));
        std::vector<const uint8_t*> ptr(k * k);
        std::vector<uint32_t> len(k * k, S);
        for (uint32_t i = 0; i < k * k; ++i) memset(shares[i].data(), (int)i, S), ptr[i] = shares[i].data();
        for (int it = 0; it < 3; ++it) {
            rsm_eds* e = nullptr;
            CHECK(rsm_eds_compute(ctx, ptr.data(), len.data(), k * k, &e));
            if (!e) return;
            std::vector<uint8_t> rr(W * 32), cr(W * 32), flat((size_t)W * W * S), pres(W * W);
            uint32_t rl = 0;
            CHECK(rsm_eds_roots(e, RSM_AXIS_ROW, nullptr, nullptr, rr.data(), 32, &rl));
            CHECK(rsm_eds_roots(e, RSM_AXIS_COL, nullptr, nullptr, cr.data(), 32, &rl));
            rsm_nmt_params np{29, 1, k};  // namespaced trees: device path for the complete square
            std::vector<uint8_t> nr(W * 90);
            CHECK(rsm_eds_roots(e, RSM_AXIS_ROW, rsm_nmt_tree_root, &np, nr.data(), 90, &rl));
            CHECK(rsm_eds_flattened(e, flat.data(), pres.data()));
            std::vector<const uint8_t*> fp(W * W);
            std::vector<uint32_t> fl(W * W, S);
            for (uint32_t i = 0; i < W * W; ++i) fp[i] = (i % 3) ? flat.data() + (size_t)i * S : nullptr;
            rsm_eds* h = nullptr;
            CHECK(rsm_eds_import(ctx, fp.data(), fl.data(), W * W, &h));
            rsm_byzantine byz;
            (void)rsm_eds_repair(h, rr.data(), cr.data(), 32, nullptr, nullptr, &byz);  // stubbed math: any outcome
            rsm_eds_free(h);
            rsm_eds_free(e);
        }
    });
    for (auto& x : th) x.join();
    rsm_ctx_destroy(ctx);
    printf(failed ? "hammer: FAILED\n" : "hammer: ok\n");
    return failed;
}
