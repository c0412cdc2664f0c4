/*
 * leopard_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * CPU restatement of the Reed-Solomon arithmetic that rsmt2d's LeoRSCodec
 * delegates to: github.com/klauspost/reedsolomon v1.14.1 (go.mod:8), built with
 * reedsolomon.New(k, k, WithLeopardGF(true)) (leopard.go:65 of the reference),
 * i.e. the Leopard-RS additive-FFT codec (catid/leopard algorithm):
 *   - GF(2^8)  ("leopard8.go")  when the total shard count 2k <= 256
 *   - GF(2^16) ("leopard.go")   when 2k > 256     (codecs.go:6-10)
 * That module is NOT present in /root/reference and there is no Go toolchain
 * here, so this is a restatement of its published algorithm (SURVEY.md
 * Appendix A).  Parity is pinned only by the reference's own known-answer
 * tests (extendeddatasquare_test.go:39-59, the 1x1 and 2x2 grids); every other
 * size is "parity unpinned vs LeoRSCodec" (see DESIGN.md / tests/golden).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library.  It is deliberately simple scalar C (one 256-entry
 * multiply table per constant for GF8, split lo/hi tables for GF16).
 *
 * Exported (C ABI, see oracle/__init__.py):
 *   int  leo_field_bits(unsigned k)                       -> 8 or 16
 *   int  leo_encode(k, S, data[k], parity[k])            codec.Encode   (leopard.go:28-45)
 *   int  leo_decode(k, S, shards[2k], present[2k])        codec.Decode   (leopard.go:51-59)
 *   int  leo_extend_square(k, S, ods, eds, nthreads)      erasureExtendSquare
 *                                                         (extendeddatasquare.go:154-227)
 *   void leo_tables8/16(...)                              table self-check exports
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

/* ------------------------------------------------------------------------- */
/* GF(2^8): klauspost leopard8.go / catid LeopardFF8.cpp     */
/* ------------------------------------------------------------------------- */
#define B8 8
#define ORD8 256
#define MOD8 255
static const unsigned kBasis8[B8] = {1, 214, 152, 146, 86, 200, 88, 230};
static const unsigned kPoly8 = 0x11D;

static uint8_t exp8[ORD8], log8[ORD8], skew8[MOD8], logwalsh8[ORD8];
static uint8_t mul8[ORD8][ORD8]; /* mul8[logm][x] = mulLog8(x, logm) */
#ifdef LEO_SIMD
static uint8_t nib8[ORD8][2][16];
#endif
#ifdef LEO_GFNI
static uint64_t aff8[ORD8]; /* GF2P8AFFINEQB matrix of x -> mulLog8(x, logm) */
#endif

/* ------------------------------------------------------------------------- */
/* GF(2^16): klauspost leopard.go / catid LeopardFF16.cpp                      */
/* ------------------------------------------------------------------------- */
#define B16 16
#define ORD16 65536
#define MOD16 65535
static const unsigned kBasis16[B16] = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E,
                                       0x914C, 0x4012, 0x6C98, 0x10D8, 0x6A72, 0xB900,
                                       0xFDB8, 0xFB34, 0xFF38, 0x991E};
static const unsigned kPoly16 = 0x1002D;

static uint16_t *exp16, *log16, *skew16, *logwalsh16;

static inline unsigned add_mod8(unsigned a, unsigned b) {
    unsigned s = a + b;
    return (s + (s >> B8)) & MOD8; /* may return MOD8 (== 0 mod 255) like the reference */
}
static inline unsigned sub_mod8(unsigned a, unsigned b) {
    unsigned d = a - b; /* unsigned wrap, as in catid SubMod / klauspost subMod8 */
    return (d + (d >> B8)) & MOD8;
}
static inline unsigned mul_log8(unsigned a, unsigned logb) {
    return a == 0 ? 0 : exp8[add_mod8(log8[a], logb)];
}
static inline unsigned add_mod16(unsigned a, unsigned b) {
    unsigned s = a + b;
    return (s + (s >> B16)) & MOD16;
}
static inline unsigned sub_mod16(unsigned a, unsigned b) {
    unsigned d = a - b;
    return (d + (d >> B16)) & MOD16;
}
static inline unsigned mul_log16(unsigned a, unsigned logb) {
    return a == 0 ? 0 : exp16[add_mod16(log16[a], logb)];
}

/* FWHT over the log domain (catid FWHT / klauspost fwht): SURVEY A.5 last lines. */
static void fwht8(uint8_t *data, unsigned m, unsigned mtrunc) {
    unsigned dist = 1, dist4 = 4;
    for (; dist4 <= m; dist = dist4, dist4 <<= 2)
        for (unsigned r = 0; r < mtrunc; r += dist4)
            for (unsigned i = r; i < r + dist; ++i) {
                unsigned t0 = data[i], t1 = data[i + dist], t2 = data[i + 2 * dist],
                         t3 = data[i + 3 * dist];
                unsigned a;
                a = add_mod8(t0, t1); t1 = sub_mod8(t0, t1); t0 = a;
                a = add_mod8(t2, t3); t3 = sub_mod8(t2, t3); t2 = a;
                a = add_mod8(t0, t2); t2 = sub_mod8(t0, t2); t0 = a;
                a = add_mod8(t1, t3); t3 = sub_mod8(t1, t3); t1 = a;
                data[i] = t0; data[i + dist] = t1; data[i + 2 * dist] = t2; data[i + 3 * dist] = t3;
            }
    if (dist < m)
        for (unsigned i = 0; i < dist; ++i) {
            unsigned a = add_mod8(data[i], data[i + dist]);
            unsigned b = sub_mod8(data[i], data[i + dist]);
            data[i] = a; data[i + dist] = b;
        }
}
static void fwht16(uint16_t *data, unsigned m, unsigned mtrunc) {
    unsigned dist = 1, dist4 = 4;
    for (; dist4 <= m; dist = dist4, dist4 <<= 2)
        for (unsigned r = 0; r < mtrunc; r += dist4)
            for (unsigned i = r; i < r + dist; ++i) {
                unsigned t0 = data[i], t1 = data[i + dist], t2 = data[i + 2 * dist],
                         t3 = data[i + 3 * dist];
                unsigned a;
                a = add_mod16(t0, t1); t1 = sub_mod16(t0, t1); t0 = a;
                a = add_mod16(t2, t3); t3 = sub_mod16(t2, t3); t2 = a;
                a = add_mod16(t0, t2); t2 = sub_mod16(t0, t2); t0 = a;
                a = add_mod16(t1, t3); t3 = sub_mod16(t1, t3); t1 = a;
                data[i] = t0; data[i + dist] = t1; data[i + 2 * dist] = t2; data[i + 3 * dist] = t3;
            }
    if (dist < m)
        for (unsigned i = 0; i < dist; ++i) {
            unsigned a = add_mod16(data[i], data[i + dist]);
            unsigned b = sub_mod16(data[i], data[i + dist]);
            data[i] = a; data[i + dist] = b;
        }
}

static void init8(void) {
    /* A.2 tables */
    unsigned state = 1;
    for (unsigned i = 0; i < MOD8; ++i) {
        exp8[state] = (uint8_t)i;
        state <<= 1;
        if (state >= ORD8) state ^= kPoly8;
    }
    exp8[0] = MOD8;
    log8[0] = 0;
    for (unsigned i = 0; i < B8; ++i) {
        unsigned w = 1u << i;
        for (unsigned j = 0; j < w; ++j) log8[j + w] = log8[j] ^ kBasis8[i];
    }
    for (unsigned i = 0; i < ORD8; ++i) log8[i] = exp8[log8[i]];
    for (unsigned i = 0; i < ORD8; ++i) exp8[log8[i]] = (uint8_t)i;
    exp8[MOD8] = exp8[0];
    /* A.3 FFT skew + LogWalsh */
    unsigned temp[B8 - 1];
    for (unsigned i = 1; i < B8; ++i) temp[i - 1] = 1u << i;
    for (unsigned m = 0; m < B8 - 1; ++m) {
        unsigned step = 1u << (m + 1);
        skew8[(1u << m) - 1] = 0;
        for (unsigned i = m; i < B8 - 1; ++i) {
            unsigned s = 1u << (i + 1);
            for (unsigned j = (1u << m) - 1; j < s; j += step) skew8[j + s] = skew8[j] ^ temp[i];
        }
        temp[m] = MOD8 - log8[mul_log8(temp[m], log8[temp[m] ^ 1])];
        for (unsigned i = m + 1; i < B8 - 1; ++i)
            temp[i] = mul_log8(temp[i], add_mod8(log8[temp[i] ^ 1], temp[m]));
    }
    for (unsigned i = 0; i < MOD8; ++i) skew8[i] = log8[skew8[i]];
    for (unsigned i = 0; i < ORD8; ++i) logwalsh8[i] = log8[i];
    logwalsh8[0] = 0;
    fwht8(logwalsh8, ORD8, ORD8);
    /* per-constant multiply tables (klauspost mul8LUTs equivalent) */
    for (unsigned lm = 0; lm < ORD8; ++lm)
        for (unsigned x = 0; x < ORD8; ++x) mul8[lm][x] = (uint8_t)mul_log8(x, lm);
}

static void init16(void) {
    exp16 = (uint16_t *)malloc(sizeof(uint16_t) * ORD16);
    log16 = (uint16_t *)malloc(sizeof(uint16_t) * ORD16);
    skew16 = (uint16_t *)malloc(sizeof(uint16_t) * MOD16);
    logwalsh16 = (uint16_t *)malloc(sizeof(uint16_t) * ORD16);
    unsigned state = 1;
    for (unsigned i = 0; i < MOD16; ++i) {
        exp16[state] = (uint16_t)i;
        state <<= 1;
        if (state >= ORD16) state ^= kPoly16;
    }
    exp16[0] = MOD16;
    log16[0] = 0;
    for (unsigned i = 0; i < B16; ++i) {
        unsigned w = 1u << i;
        for (unsigned j = 0; j < w; ++j) log16[j + w] = log16[j] ^ kBasis16[i];
    }
    for (unsigned i = 0; i < ORD16; ++i) log16[i] = exp16[log16[i]];
    for (unsigned i = 0; i < ORD16; ++i) exp16[log16[i]] = (uint16_t)i;
    exp16[MOD16] = exp16[0];
    unsigned temp[B16 - 1];
    for (unsigned i = 1; i < B16; ++i) temp[i - 1] = 1u << i;
    for (unsigned m = 0; m < B16 - 1; ++m) {
        unsigned step = 1u << (m + 1);
        skew16[(1u << m) - 1] = 0;
        for (unsigned i = m; i < B16 - 1; ++i) {
            unsigned s = 1u << (i + 1);
            for (unsigned j = (1u << m) - 1; j < s; j += step) skew16[j + s] = skew16[j] ^ temp[i];
        }
        temp[m] = MOD16 - log16[mul_log16(temp[m], log16[temp[m] ^ 1])];
        for (unsigned i = m + 1; i < B16 - 1; ++i)
            temp[i] = mul_log16(temp[i], add_mod16(log16[temp[i] ^ 1], temp[m]));
    }
    for (unsigned i = 0; i < MOD16; ++i) skew16[i] = log16[skew16[i]];
    for (unsigned i = 0; i < ORD16; ++i) logwalsh16[i] = log16[i];
    logwalsh16[0] = 0;
    fwht16(logwalsh16, ORD16, ORD16);
}

static pthread_once_t g_once = PTHREAD_ONCE_INIT;
#ifdef LEO_SIMD
static void init_nib8(void) {
    for (unsigned lm = 0; lm < ORD8; ++lm)
        for (unsigned v = 0; v < 16; ++v) {
            nib8[lm][0][v] = mul8[lm][v];
            nib8[lm][1][v] = mul8[lm][v << 4];
        }
}
static void init_all(void) { init8(); init16(); init_nib8(); }
#elif defined(LEO_GFNI)
/* row i of the bit matrix (byte 7 - i of the qword): input bit j feeds output bit i
 * iff bit i of mulLog8(1 << j, logm) is set */
static void init_aff8(void) {
    for (unsigned lm = 0; lm < ORD8; ++lm) {
        uint64_t a = 0;
        for (unsigned i = 0; i < 8; ++i) {
            unsigned row = 0;
            for (unsigned j = 0; j < 8; ++j) row |= ((mul8[lm][1u << j] >> i) & 1u) << j;
            a |= (uint64_t)row << (8 * (7 - i));
        }
        aff8[lm] = a;
    }
}
static void init_all(void) { init8(); init16(); init_aff8(); }
#else
static void init_all(void) { init8(); init16(); }
#endif
static void ensure_init(void) { pthread_once(&g_once, init_all); }

/* ------------------------------------------------------------------------- */
/* Vector ops on "symbols".  A GF8 work row is S bytes, each byte a symbol.   */
/* A GF16 work row is S bytes; per 64-byte block, symbol t (t<32) is          */
/* lo = row[64b+t], hi = row[64b+32+t]  (klauspost refMulAdd layout, A.6).   */
/* ------------------------------------------------------------------------- */
#if defined(LEO_GFNI)
/* LEO_GFNI (libleopard_gfni.so, the bench's cpu_baseline only): AVX-512 rows with
 * GF(2^8) multiply-by-constant as one GF2P8AFFINEQB per 64 bytes -- the instruction
 * klauspost/reedsolomon's AVX-512 GFNI leopard8 path uses -- and the butterflies
 * fused into one pass over x and y (a restatement, not the reference). */
#include <immintrin.h>
static inline void xor_row(uint8_t *restrict dst, const uint8_t *restrict src, size_t n) {
    for (size_t i = 0; i < n; i += 64)
        _mm512_storeu_si512(dst + i, _mm512_xor_si512(_mm512_loadu_si512(dst + i), _mm512_loadu_si512(src + i)));
}
static inline void muladd8(uint8_t *restrict dst, const uint8_t *restrict src, unsigned lm, size_t n) {
    const __m512i a = _mm512_set1_epi64((long long)aff8[lm]);
    for (size_t i = 0; i < n; i += 64)
        _mm512_storeu_si512(dst + i, _mm512_xor_si512(_mm512_loadu_si512(dst + i),
                                                      _mm512_gf2p8affine_epi64_epi8(_mm512_loadu_si512(src + i), a, 0)));
}
static inline void mul8_row(uint8_t *restrict dst, const uint8_t *restrict src, unsigned lm, size_t n) {
    const __m512i a = _mm512_set1_epi64((long long)aff8[lm]);
    for (size_t i = 0; i < n; i += 64)
        _mm512_storeu_si512(dst + i, _mm512_gf2p8affine_epi64_epi8(_mm512_loadu_si512(src + i), a, 0));
}
/* fused GF(2^8) butterflies: IFFT_DIT2 y ^= x; x ^= y*L -- FFT_DIT2 x ^= y*L; y ^= x */
static inline void ifft2_8(uint8_t *restrict x, uint8_t *restrict y, unsigned lm, size_t n) {
    const __m512i a = _mm512_set1_epi64((long long)aff8[lm]);
    for (size_t i = 0; i < n; i += 64) {
        const __m512i xv = _mm512_loadu_si512(x + i);
        const __m512i yv = _mm512_xor_si512(_mm512_loadu_si512(y + i), xv);
        _mm512_storeu_si512(y + i, yv);
        _mm512_storeu_si512(x + i, _mm512_xor_si512(xv, _mm512_gf2p8affine_epi64_epi8(yv, a, 0)));
    }
}
static inline void fft2_8(uint8_t *restrict x, uint8_t *restrict y, unsigned lm, size_t n) {
    const __m512i a = _mm512_set1_epi64((long long)aff8[lm]);
    for (size_t i = 0; i < n; i += 64) {
        const __m512i yv = _mm512_loadu_si512(y + i);
        const __m512i xv = _mm512_xor_si512(_mm512_loadu_si512(x + i), _mm512_gf2p8affine_epi64_epi8(yv, a, 0));
        _mm512_storeu_si512(x + i, xv);
        _mm512_storeu_si512(y + i, _mm512_xor_si512(yv, xv));
    }
}
#define LEO_FUSED8 1
#elif !defined(LEO_SIMD)
static inline void xor_row(uint8_t *restrict dst, const uint8_t *restrict src, size_t n) {
    for (size_t i = 0; i < n; ++i) dst[i] ^= src[i];
}
/* dst ^= src * log_m (GF8) */
static inline void muladd8(uint8_t *restrict dst, const uint8_t *restrict src, unsigned lm, size_t n) {
    const uint8_t *t = mul8[lm];
    for (size_t i = 0; i < n; ++i) dst[i] ^= t[src[i]];
}
static inline void mul8_row(uint8_t *restrict dst, const uint8_t *restrict src, unsigned lm, size_t n) {
    const uint8_t *t = mul8[lm];
    for (size_t i = 0; i < n; ++i) dst[i] = t[src[i]];
}
#else
/* LEO_SIMD (libleopard_simd.so, the bench's cpu_baseline only): the same rows with
 * AVX2, GF(2^8) multiply-by-constant as two 16-entry pshufb nibble tables -- the
 * technique klauspost/reedsolomon's AVX2 leopard8 path uses (a restatement, not
 * the reference, which cannot run here).  S % 64 == 0, so rows are whole 32-byte
 * vectors. */
#include <immintrin.h>
/* nib8[logm][lo/hi][nibble] = mulLog8(nibble << 4*hi, logm): see init_nib8 */
static inline void xor_row(uint8_t *restrict dst, const uint8_t *restrict src, size_t n) {
    for (size_t i = 0; i < n; i += 32) {
        __m256i d = _mm256_loadu_si256((const __m256i *)(dst + i));
        __m256i s = _mm256_loadu_si256((const __m256i *)(src + i));
        _mm256_storeu_si256((__m256i *)(dst + i), _mm256_xor_si256(d, s));
    }
}
static inline __m256i mul8_v(__m256i x, __m256i tlo, __m256i thi, __m256i m) {
    __m256i lo = _mm256_and_si256(x, m);
    __m256i hi = _mm256_and_si256(_mm256_srli_epi64(x, 4), m);
    return _mm256_xor_si256(_mm256_shuffle_epi8(tlo, lo), _mm256_shuffle_epi8(thi, hi));
}
static inline void muladd8(uint8_t *restrict dst, const uint8_t *restrict src, unsigned lm, size_t n) {
    const __m256i tlo = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)nib8[lm][0]));
    const __m256i thi = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)nib8[lm][1]));
    const __m256i m = _mm256_set1_epi8(0x0F);
    for (size_t i = 0; i < n; i += 32) {
        __m256i x = _mm256_loadu_si256((const __m256i *)(src + i));
        __m256i d = _mm256_loadu_si256((const __m256i *)(dst + i));
        _mm256_storeu_si256((__m256i *)(dst + i), _mm256_xor_si256(d, mul8_v(x, tlo, thi, m)));
    }
}
static inline void mul8_row(uint8_t *restrict dst, const uint8_t *restrict src, unsigned lm, size_t n) {
    const __m256i tlo = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)nib8[lm][0]));
    const __m256i thi = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)nib8[lm][1]));
    const __m256i m = _mm256_set1_epi8(0x0F);
    for (size_t i = 0; i < n; i += 32)
        _mm256_storeu_si256((__m256i *)(dst + i), mul8_v(_mm256_loadu_si256((const __m256i *)(src + i)), tlo, thi, m));
}
#endif
static inline void muladd16(uint8_t *restrict dst, const uint8_t *restrict src, unsigned lm, size_t n) {
    for (size_t b = 0; b < n; b += 64)
        for (unsigned t = 0; t < 32; ++t) {
            unsigned v = src[b + t] | ((unsigned)src[b + 32 + t] << 8);
            unsigned p = mul_log16(v, lm);
            dst[b + t] ^= (uint8_t)p;
            dst[b + 32 + t] ^= (uint8_t)(p >> 8);
        }
}
static inline void mul16_row(uint8_t *restrict dst, const uint8_t *restrict src, unsigned lm, size_t n) {
    for (size_t b = 0; b < n; b += 64)
        for (unsigned t = 0; t < 32; ++t) {
            unsigned v = src[b + t] | ((unsigned)src[b + 32 + t] << 8);
            unsigned p = mul_log16(v, lm);
            dst[b + t] = (uint8_t)p;
            dst[b + 32 + t] = (uint8_t)(p >> 8);
        }
}

typedef struct {
    int gf16;
    unsigned mod;
    size_t n; /* bytes per row */
} field_t;

static inline void muladd(const field_t *f, uint8_t *d, const uint8_t *s, unsigned lm) {
    if (f->gf16) muladd16(d, s, lm, f->n); else muladd8(d, s, lm, f->n);
}
static inline void mulrow(const field_t *f, uint8_t *d, const uint8_t *s, unsigned lm) {
    if (f->gf16) mul16_row(d, s, lm, f->n); else mul8_row(d, s, lm, f->n);
}
static inline unsigned skew_at(const field_t *f, long idx) {
    return f->gf16 ? skew16[idx] : skew8[idx];
}

/* IFFT_DIT2: y ^= x; x ^= y*L   (L == MOD => zero multiplier: XOR half only) */
static inline void ifft2(const field_t *f, uint8_t *x, uint8_t *y, unsigned L) {
#ifdef LEO_FUSED8
    if (!f->gf16 && L != f->mod) { ifft2_8(x, y, L, f->n); return; }
#endif
    xor_row(y, x, f->n);
    if (L != f->mod) muladd(f, x, y, L);
}
/* FFT_DIT2: x ^= y*L; y ^= x */
static inline void fft2(const field_t *f, uint8_t *x, uint8_t *y, unsigned L) {
#ifdef LEO_FUSED8
    if (!f->gf16 && L != f->mod) { fft2_8(x, y, L, f->n); return; }
#endif
    if (L != f->mod) muladd(f, x, y, L);
    xor_row(y, x, f->n);
}

/* klauspost ifftDITEncoder / catid IFFT_DIT_Encoder.
 * skew_off: skewLUT = &SKEW[skew_off] (encoder passes m-1). */
static void ifft_dit_encoder(const field_t *f, uint8_t *const *data, unsigned mtrunc, uint8_t **work,
                             unsigned m, long skew_off) {
    for (unsigned i = 0; i < mtrunc; ++i) memcpy(work[i], data[i], f->n);
    for (unsigned i = mtrunc; i < m; ++i) memset(work[i], 0, f->n);
    unsigned dist = 1, dist4 = 4;
    for (; dist4 <= m; dist = dist4, dist4 <<= 2)
        for (unsigned r = 0; r < mtrunc; r += dist4) {
            unsigned iend = r + dist;
            unsigned L01 = skew_at(f, skew_off + iend);
            unsigned L02 = skew_at(f, skew_off + iend + dist);
            unsigned L23 = skew_at(f, skew_off + iend + 2 * dist);
            for (unsigned i = r; i < iend; ++i) {
                uint8_t **w = work + i;
                ifft2(f, w[0], w[dist], L01);
                ifft2(f, w[2 * dist], w[3 * dist], L23);
                ifft2(f, w[0], w[2 * dist], L02);
                ifft2(f, w[dist], w[3 * dist], L02);
            }
        }
    if (dist < m) {
        unsigned L = skew_at(f, skew_off + dist);
        for (unsigned i = 0; i < dist; ++i) ifft2(f, work[i], work[i + dist], L);
    }
}

/* klauspost ifftDITDecoder: skewLUT = SKEW (index j -> SKEW[j-1]). */
static void ifft_dit_decoder(const field_t *f, unsigned mtrunc, uint8_t **work, unsigned m) {
    unsigned dist = 1, dist4 = 4;
    for (; dist4 <= m; dist = dist4, dist4 <<= 2)
        for (unsigned r = 0; r < mtrunc; r += dist4) {
            unsigned iend = r + dist;
            unsigned L01 = skew_at(f, (long)iend - 1);
            unsigned L02 = skew_at(f, (long)iend + dist - 1);
            unsigned L23 = skew_at(f, (long)iend + 2 * dist - 1);
            for (unsigned i = r; i < iend; ++i) {
                uint8_t **w = work + i;
                ifft2(f, w[0], w[dist], L01);
                ifft2(f, w[2 * dist], w[3 * dist], L23);
                ifft2(f, w[0], w[2 * dist], L02);
                ifft2(f, w[dist], w[3 * dist], L02);
            }
        }
    if (dist < m) {
        unsigned L = skew_at(f, (long)dist - 1);
        for (unsigned i = 0; i < dist; ++i) ifft2(f, work[i], work[i + dist], L);
    }
}

/* klauspost fftDIT / catid FFT_DIT: skewLUT = SKEW (index j -> SKEW[j-1]). */
static void fft_dit(const field_t *f, uint8_t **work, unsigned mtrunc, unsigned m) {
    unsigned dist4 = m, dist = m >> 2;
    for (; dist != 0; dist4 = dist, dist >>= 2)
        for (unsigned r = 0; r < mtrunc; r += dist4) {
            unsigned iend = r + dist;
            unsigned L01 = skew_at(f, (long)iend - 1);
            unsigned L02 = skew_at(f, (long)iend + dist - 1);
            unsigned L23 = skew_at(f, (long)iend + 2 * dist - 1);
            for (unsigned i = r; i < iend; ++i) {
                uint8_t **w = work + i;
                fft2(f, w[0], w[2 * dist], L02);
                fft2(f, w[dist], w[3 * dist], L02);
                fft2(f, w[0], w[dist], L01);
                fft2(f, w[2 * dist], w[3 * dist], L23);
            }
        }
    if (dist4 == 2)
        for (unsigned r = 0; r < mtrunc; r += 2) {
            unsigned L = skew_at(f, (long)r);
            fft2(f, work[r], work[r + 1], L);
        }
}

static unsigned ceil_pow2(unsigned x) {
    unsigned p = 1;
    while (p < x) p <<= 1;
    return p;
}

int leo_field_bits(unsigned k) { return (2 * k > 256) ? 16 : 8; }

/* Encode: k data rows of S bytes -> k parity rows (klauspost leopard encode,
 * called from LeoRSCodec.Encode, leopard.go:28-45).  Returns 0 or negative. */
int leo_encode(unsigned k, size_t S, const uint8_t *const *data, uint8_t *const *parity) {
    ensure_init();
    if (k == 0 || S == 0 || (S % 64) != 0) return -1;
    if (2ul * k > 65536ul) return -2;
    field_t f = {leo_field_bits(k) == 16, leo_field_bits(k) == 16 ? MOD16 : MOD8, S};
    unsigned m = ceil_pow2(k);
    unsigned mtrunc = k < m ? k : m;
    /* per-thread grow-only work rows: a fresh 2m*S allocation per codeword is an
     * mmap/munmap pair (page faults, a process-wide lock) at k=128, S=512 */
    static __thread uint8_t *tbuf = NULL;
    static __thread size_t tcap = 0;
    static __thread uint8_t **twork = NULL;
    static __thread unsigned twcap = 0;
    if (tcap < S * 2 * (size_t)m) {
        free(tbuf);
        tcap = S * 2 * (size_t)m;
        tbuf = (uint8_t *)malloc(tcap);
    }
    if (twcap < 2 * m) {
        free(twork);
        twcap = 2 * m;
        twork = (uint8_t **)malloc(sizeof(uint8_t *) * twcap);
    }
    uint8_t **work = twork;
    uint8_t *buf = tbuf;
    for (unsigned i = 0; i < 2 * m; ++i) work[i] = buf + (size_t)i * S;
    ifft_dit_encoder(&f, (uint8_t *const *)data, mtrunc, work, m, (long)m - 1);
    /* k <= m always for square codes (parity count == data count), so the
     * "further blocks of m data" loop of the reference never runs. */
    fft_dit(&f, work, k, m);
    for (unsigned i = 0; i < k; ++i) memcpy(parity[i], work[i], S);
    return 0;
}

/* Decode / Reconstruct: shards[0..k) data, [k..2k) parity; present[i]==0 means
 * missing (its buffer is filled on success).  klauspost reconstruct with
 * recoverAll=true.  Returns 0, -3 (too few shards). */
int leo_decode(unsigned k, size_t S, uint8_t *const *shards, const uint8_t *present) {
    ensure_init();
    if (k == 0 || S == 0 || (S % 64) != 0) return -1;
    unsigned npresent = 0;
    for (unsigned i = 0; i < 2 * k; ++i) npresent += present[i] ? 1 : 0;
    if (npresent == 2 * k) return 0;
    if (npresent < k) return -3;
    int gf16 = leo_field_bits(k) == 16;
    field_t f = {gf16, gf16 ? MOD16 : MOD8, S};
    unsigned order = gf16 ? ORD16 : ORD8;
    unsigned mod = f.mod;
    unsigned m = ceil_pow2(k);
    unsigned n = ceil_pow2(m + k);
    /* error locator, in the log domain */
    uint16_t *err16 = NULL;
    uint8_t err8[ORD8];
    if (gf16) err16 = (uint16_t *)calloc(order, sizeof(uint16_t));
    else memset(err8, 0, sizeof(err8));
#define ERR_SET(i, v) do { if (gf16) err16[i] = (uint16_t)(v); else err8[i] = (uint8_t)(v); } while (0)
#define ERR_GET(i) (gf16 ? (unsigned)err16[i] : (unsigned)err8[i])
    for (unsigned i = 0; i < k; ++i)
        if (!present[k + i]) ERR_SET(i, 1);
    for (unsigned i = k; i < m; ++i) ERR_SET(i, 1);
    for (unsigned i = 0; i < k; ++i)
        if (!present[i]) ERR_SET(i + m, 1);
    if (gf16) fwht16(err16, order, m + k); else fwht8(err8, order, m + k);
    for (unsigned i = 0; i < order; ++i) {
        unsigned lw = gf16 ? logwalsh16[i] : logwalsh8[i];
        ERR_SET(i, ((unsigned long)ERR_GET(i) * lw) % mod);
    }
    if (gf16) fwht16(err16, order, order); else fwht8(err8, order, order);

    uint8_t **work = (uint8_t **)malloc(sizeof(uint8_t *) * n);
    uint8_t *buf = (uint8_t *)calloc((size_t)n, S);
    for (unsigned i = 0; i < n; ++i) work[i] = buf + (size_t)i * S;
    for (unsigned i = 0; i < k; ++i)
        if (present[k + i]) mulrow(&f, work[i], shards[k + i], ERR_GET(i));
    for (unsigned i = 0; i < k; ++i)
        if (present[i]) mulrow(&f, work[m + i], shards[i], ERR_GET(m + i));
    ifft_dit_decoder(&f, m + k, work, n);
    /* formal derivative */
    for (unsigned i = 1; i < n; ++i) {
        unsigned width = ((i ^ (i - 1)) + 1) >> 1;
        for (unsigned j = 0; j < width; ++j) xor_row(work[i - width + j], work[i + j], S);
    }
    fft_dit(&f, work, m + k, n);
    for (unsigned i = 0; i < 2 * k; ++i) {
        if (present[i]) continue;
        if (i >= k) mulrow(&f, shards[i], work[i - k], mod - ERR_GET(i - k));
        else mulrow(&f, shards[i], work[i + m], mod - ERR_GET(i + m));
    }
#undef ERR_SET
#undef ERR_GET
    free(buf);
    free(work);
    free(err16);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* 2D extension, reference schedule (extendeddatasquare.go:154-227):          */
/*   phase 1: Q1 = RS(rows of Q0), Q2 = RS(cols of Q0)                        */
/*   phase 2: Q3 = RS(rows of Q2)                                             */
/* eds is row-major [2k][2k][S]; ods row-major [k][k][S].                     */
/* ------------------------------------------------------------------------- */
typedef struct {
    unsigned k;
    size_t S;
    uint8_t *eds;
    int phase;
    unsigned next;
    pthread_mutex_t mu;
} ext_job_t;

static void encode_vector(unsigned k, size_t S, uint8_t *eds, int is_col, unsigned idx) {
    size_t W = 2 * (size_t)k;
    const uint8_t *in[32768];
    uint8_t *out[32768];
    if (k > 32768) return;
    for (unsigned i = 0; i < k; ++i) {
        if (is_col) {
            in[i] = eds + ((size_t)i * W + idx) * S;
            out[i] = eds + ((size_t)(k + i) * W + idx) * S;
        } else {
            in[i] = eds + ((size_t)idx * W + i) * S;
            out[i] = eds + ((size_t)idx * W + k + i) * S;
        }
    }
    leo_encode(k, S, in, out);
}

static void *ext_worker(void *arg) {
    ext_job_t *j = (ext_job_t *)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        unsigned t = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (j->phase == 1) {
            if (t >= 2 * j->k) break;
            if (t < j->k) encode_vector(j->k, j->S, j->eds, 0, t);      /* erasureExtendRow(i) */
            else encode_vector(j->k, j->S, j->eds, 1, t - j->k);         /* erasureExtendCol(i) */
        } else {
            if (t >= j->k) break;
            encode_vector(j->k, j->S, j->eds, 0, j->k + t);              /* Q3 from Q2 rows */
        }
    }
    return NULL;
}

int leo_extend_square(unsigned k, size_t S, const uint8_t *ods, uint8_t *eds, int nthreads) {
    ensure_init();
    if (k == 0 || S == 0 || (S % 64) != 0) return -1;
    size_t W = 2 * (size_t)k;
    /* every cell outside Q0 is written by the encodes below */
    for (unsigned r = 0; r < k; ++r)
        memcpy(eds + (size_t)r * W * S, ods + (size_t)r * k * S, (size_t)k * S);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    ext_job_t job;
    job.k = k; job.S = S; job.eds = eds;
    pthread_mutex_init(&job.mu, NULL);
    pthread_t th[256];
    for (int phase = 1; phase <= 2; ++phase) {
        job.phase = phase;
        job.next = 0;
        if (nthreads == 1) {
            ext_worker(&job);
        } else {
            for (int i = 0; i < nthreads; ++i) pthread_create(&th[i], NULL, ext_worker, &job);
            for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
        }
    }
    pthread_mutex_destroy(&job.mu);
    return 0;
}

/* Table exports for self-checks against SURVEY A.2/A.3 values. */
void leo_tables8(uint8_t *exp_out, uint8_t *log_out, uint8_t *skew_out, uint8_t *logwalsh_out) {
    ensure_init();
    if (exp_out) memcpy(exp_out, exp8, ORD8);
    if (log_out) memcpy(log_out, log8, ORD8);
    if (skew_out) memcpy(skew_out, skew8, MOD8);
    if (logwalsh_out) memcpy(logwalsh_out, logwalsh8, ORD8);
}
void leo_tables16(uint16_t *exp_out, uint16_t *log_out, uint16_t *skew_out, uint16_t *logwalsh_out) {
    ensure_init();
    if (exp_out) memcpy(exp_out, exp16, sizeof(uint16_t) * ORD16);
    if (log_out) memcpy(log_out, log16, sizeof(uint16_t) * ORD16);
    if (skew_out) memcpy(skew_out, skew16, sizeof(uint16_t) * MOD16);
    if (logwalsh_out) memcpy(logwalsh_out, logwalsh16, sizeof(uint16_t) * ORD16);
}
