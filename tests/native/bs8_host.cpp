// Host run of the bit-sliced GF(2^8) M=128 encode arithmetic (rsmt2d_amd/csrc/bs8.hpp)
// against the oracle's leo_encode (test infrastructure: links oracle/).
// Emulates the kernel's data flow for every 32-byte slot of the share width:
//   bytes -> planes, small IFFT per a-group, exchange to the strided layout,
//   large IFFT+FFT, exchange back, small FFT, planes -> bytes.
// usage: bs8_host k S seed   (exit 0 = parity identical to the oracle)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../../rsmt2d_amd/csrc/bs8.hpp"

extern "C" int leo_encode(unsigned k, size_t S, const uint8_t* const* data, uint8_t* const* parity);

using namespace rsm::bs8;

static uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

template <int A>
static void small_ifft_rt(uint32_t (&X)[16][8]) { small_ifft<A>(X); }
template <int A>
static void small_fft_rt(uint32_t (&X)[16][8]) { small_fft<A>(X); }

static void dispatch_small(int a, bool inverse, uint32_t (&X)[16][8]) {
    sfor<8>([&](auto A) {
        if (a == decltype(A)::value) {
            if (inverse) small_ifft_rt<decltype(A)::value>(X);
            else small_fft_rt<decltype(A)::value>(X);
        }
    });
}

template <int A, int G>
static void small_h_rt(bool inverse, uint32_t (&X)[16][8]) {
    if (inverse) small_ifft_h<A, G>(X);
    else small_fft_h<A, G>(X);
}
static void dispatch_small_h(int a, int g, bool inverse, uint32_t (&X)[16][8]) {
    sfor<8>([&](auto A) {
        if (a == decltype(A)::value) {
            if (g == 0) small_h_rt<decltype(A)::value, 0>(inverse, X);
            else small_h_rt<decltype(A)::value, 1>(inverse, X);
        }
    });
}
// symbol of register j of wave a in the half-split small layout S'
static unsigned e_split(int a, int j) { return (unsigned)((j & 7) + 8 * a + 64 * (j >> 3)); }

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    const int split = argc > 4 ? atoi(argv[4]) : 0;  // 1: the half-split schedule (production)
    const unsigned k = (unsigned)atoi(argv[1]);
    const size_t S = (size_t)atoi(argv[2]);
    uint64_t seed = strtoull(argv[3], nullptr, 0);
    if (k < 65 || k > 128 || S % 64) return 2;
    std::vector<std::vector<uint8_t>> data(k, std::vector<uint8_t>(S)), want(k, std::vector<uint8_t>(S)),
        got(k, std::vector<uint8_t>(S));
    for (auto& d : data)
        for (auto& b : d) b = (uint8_t)splitmix(seed);
    std::vector<const uint8_t*> dp(k);
    std::vector<uint8_t*> wp(k);
    for (unsigned i = 0; i < k; ++i) dp[i] = data[i].data(), wp[i] = want[i].data();
    if (leo_encode(k, S, dp.data(), wp.data()) != 0) return 3;

    static uint32_t X[8][16][8];  // [wave][register][plane]
    for (size_t o = 0; split && o < S; o += 32) {
        for (int a = 0; a < 8; ++a)
            for (int j = 0; j < 16; ++j) {
                const unsigned e = e_split(a, j);
                for (int q = 0; q < 8; ++q) {
                    uint32_t v = 0;
                    if (e < k) memcpy(&v, &data[e][o + 4 * q], 4);
                    X[a][j][q] = v;
                }
                transpose8(X[a][j]);
            }
        for (int g = 0; g < 2; ++g)
            for (int a = 0; a < 8; ++a) dispatch_small_h(a, g, true, X[a]);
        static uint32_t Y[8][16][8];
        for (int g = 0; g < 2; ++g)  // wave u's register 8g + v -> wave v's register 8g + u
            for (int u = 0; u < 8; ++u)
                for (int v = 0; v < 8; ++v) memcpy(Y[v][8 * g + u], X[u][8 * g + v], 32);
        for (int w = 0; w < 8; ++w) {
            large_ifft_h<0>(Y[w]);
            large_ifft_h<1>(Y[w]);
            large_mid(Y[w]);
            large_fft_h<0>(Y[w]);
            large_fft_h<1>(Y[w]);
        }
        for (int g = 0; g < 2; ++g)
            for (int u = 0; u < 8; ++u)
                for (int v = 0; v < 8; ++v) memcpy(X[v][8 * g + u], Y[u][8 * g + v], 32);
        for (int g = 0; g < 2; ++g)
            for (int a = 0; a < 8; ++a) dispatch_small_h(a, g, false, X[a]);
        for (int a = 0; a < 8; ++a)
            for (int j = 0; j < 16; ++j) {
                const unsigned e = e_split(a, j);
                transpose8(X[a][j]);
                if (e < k)
                    for (int q = 0; q < 8; ++q) memcpy(&got[e][o + 4 * q], &X[a][j][q], 4);
            }
    }
    for (size_t o = 0; !split && o < S; o += 32) {
        for (int a = 0; a < 8; ++a)
            for (int j = 0; j < 16; ++j) {
                const unsigned e = 16 * a + j;
                for (int q = 0; q < 8; ++q) {
                    uint32_t v = 0;
                    if (e < k) memcpy(&v, &data[e][o + 4 * q], 4);
                    X[a][j][q] = v;
                }
                transpose8(X[a][j]);
            }
        for (int a = 0; a < 8; ++a) dispatch_small(a, true, X[a]);
        static uint32_t Y[8][16][8];
        for (int g = 0; g < 8; ++g)
            for (int h = 0; h < 16; ++h) memcpy(Y[g][h], X[(8 * h + g) / 16][(8 * h + g) % 16], 32);
        for (int g = 0; g < 8; ++g) large_ifft_fft(Y[g]);
        for (int g = 0; g < 8; ++g)
            for (int h = 0; h < 16; ++h) memcpy(X[(8 * h + g) / 16][(8 * h + g) % 16], Y[g][h], 32);
        for (int a = 0; a < 8; ++a) dispatch_small(a, false, X[a]);
        for (int a = 0; a < 8; ++a)
            for (int j = 0; j < 16; ++j) {
                const unsigned e = 16 * a + j;
                transpose8(X[a][j]);
                if (e < k)
                    for (int q = 0; q < 8; ++q) memcpy(&got[e][o + 4 * q], &X[a][j][q], 4);
            }
    }
    for (unsigned i = 0; i < k; ++i)
        if (got[i] != want[i]) {
            size_t b = 0;
            while (got[i][b] == want[i][b]) ++b;
            fprintf(stderr, "parity %u differs at byte %zu: got %u want %u\n", i, b, got[i][b], want[i][b]);
            return 1;
        }
    printf("ok k=%u S=%zu split=%d\n", k, S, split);
    return 0;
}
