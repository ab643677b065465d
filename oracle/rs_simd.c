/*
 * rs_simd.c -- vectorised CPU encode, the strong CPU baseline.
 *
 * TEST INFRASTRUCTURE ONLY, like rs_oracle.c: bench.py's cpu_baseline leg
 * times it and tests/ check it against the scalar oracle.  The product path
 * (libmemo_ec.so) never links or calls it.
 *
 * Same arithmetic as memo_oracle_encode (rs_oracle.c), i.e. ISA-L
 * ec_encode_data semantics with the gf_gen_cauchy1_matrix generator, computed
 * the way ISA-L's published x86 kernels do (ISA-L is not in the reference nor
 * in this image; this is a restatement of its published techniques, not its
 * code):
 *   - GFNI + AVX-512: multiplication by a constant c is GF(2)-linear in the
 *     bits of x, so one vgf2p8affineqb per 64 bytes applies the 8x8 bit
 *     matrix of "x -> c*x" (poly 0x11D);
 *   - AVX2: split-nibble lookup, c*x = T_lo[c][x & 15] ^ T_hi[c][x >> 4],
 *     two vpshufb per 32 bytes;
 *   - scalar: the 256x256 product table of the oracle.
 * The ISA is chosen at run time (__builtin_cpu_supports).  Work is
 * partitioned by block index over `threads` threads, like
 * memo_oracle_encode_mt.
 */
#include <immintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

int memo_oracle_cauchy(int k, int m, uint8_t *a);
uint8_t memo_oracle_gf_mul(uint8_t a, uint8_t b);
int memo_oracle_decode_matrix(int k, int m, const uint8_t *surv, const uint8_t *lost, int e,
                              uint8_t *out);

enum { ISA_SCALAR = 0, ISA_AVX2 = 1, ISA_GFNI512 = 2 };

int memo_oracle_simd_isa(void)
{
    __builtin_cpu_init();
    if (__builtin_cpu_supports("gfni") && __builtin_cpu_supports("avx512f") &&
        __builtin_cpu_supports("avx512bw"))
        return ISA_GFNI512;
    if (__builtin_cpu_supports("avx2")) return ISA_AVX2;
    return ISA_SCALAR;
}

/* 8x8 GF(2) matrix of x -> c*x in vgf2p8affineqb layout: output bit i is the
 * parity of (byte 7-i of the qword) AND x. */
static uint64_t affine_matrix(uint8_t c)
{
    uint8_t col[8];
    for (int k = 0; k < 8; ++k) col[k] = memo_oracle_gf_mul(c, (uint8_t)(1u << k));
    uint64_t q = 0;
    for (int i = 0; i < 8; ++i) {
        uint8_t row = 0;
        for (int k = 0; k < 8; ++k)
            if ((col[k] >> i) & 1) row |= (uint8_t)(1u << k);
        q |= (uint64_t)row << (8 * (7 - i));
    }
    return q;
}

typedef struct {
    int isa, k, m;
    size_t S, b0, b1;
    const uint8_t *data;
    uint8_t *parity;
    const uint8_t *coef;       /* m x k */
    const uint64_t *aff;       /* m x k affine matrices */
    const uint8_t *nib;        /* m x k x 32: T_lo | T_hi */
} simd_job;

static void scalar_cols(const simd_job *j, const uint8_t *d, uint8_t *p, size_t x0)
{
    for (int r = 0; r < j->m; ++r) {
        uint8_t *o = p + (size_t)r * j->S;
        for (size_t x = x0; x < j->S; ++x) {
            uint8_t acc = 0;
            for (int c = 0; c < j->k; ++c)
                acc ^= memo_oracle_gf_mul(j->coef[r * j->k + c], d[(size_t)c * j->S + x]);
            o[x] = acc;
        }
    }
}

__attribute__((target("avx512f,avx512bw,gfni")))
static void block_gfni(const simd_job *j, const uint8_t *d, uint8_t *p)
{
    const int k = j->k, m = j->m;
    const size_t S = j->S, S64 = S & ~(size_t)63;
    const int nt = ((uintptr_t)p % 64) == 0 && (S % 64) == 0;
    for (int r0 = 0; r0 < m; r0 += 4) {
        const int nr = m - r0 < 4 ? m - r0 : 4;
        for (size_t x = 0; x < S64; x += 64) {
            __m512i a0 = _mm512_setzero_si512(), a1 = a0, a2 = a0, a3 = a0;
            for (int c = 0; c < k; ++c) {
                const __m512i v = _mm512_loadu_si512((const void *)(d + (size_t)c * S + x));
                const uint64_t *A = j->aff + (size_t)r0 * k + c;
                a0 = _mm512_xor_si512(a0, _mm512_gf2p8affine_epi64_epi8(v, _mm512_set1_epi64((long long)A[0]), 0));
                if (nr > 1) a1 = _mm512_xor_si512(a1, _mm512_gf2p8affine_epi64_epi8(v, _mm512_set1_epi64((long long)A[k]), 0));
                if (nr > 2) a2 = _mm512_xor_si512(a2, _mm512_gf2p8affine_epi64_epi8(v, _mm512_set1_epi64((long long)A[2 * k]), 0));
                if (nr > 3) a3 = _mm512_xor_si512(a3, _mm512_gf2p8affine_epi64_epi8(v, _mm512_set1_epi64((long long)A[3 * k]), 0));
            }
            if (nt) {  /* streaming stores: no read-for-ownership of parity lines */
                _mm512_stream_si512((void *)(p + (size_t)r0 * S + x), a0);
                if (nr > 1) _mm512_stream_si512((void *)(p + (size_t)(r0 + 1) * S + x), a1);
                if (nr > 2) _mm512_stream_si512((void *)(p + (size_t)(r0 + 2) * S + x), a2);
                if (nr > 3) _mm512_stream_si512((void *)(p + (size_t)(r0 + 3) * S + x), a3);
            } else {
                _mm512_storeu_si512((void *)(p + (size_t)r0 * S + x), a0);
                if (nr > 1) _mm512_storeu_si512((void *)(p + (size_t)(r0 + 1) * S + x), a1);
                if (nr > 2) _mm512_storeu_si512((void *)(p + (size_t)(r0 + 2) * S + x), a2);
                if (nr > 3) _mm512_storeu_si512((void *)(p + (size_t)(r0 + 3) * S + x), a3);
            }
        }
    }
    if (S64 < S) scalar_cols(j, d, p, S64);
}

__attribute__((target("avx2")))
static void block_avx2(const simd_job *j, const uint8_t *d, uint8_t *p)
{
    const int k = j->k, m = j->m;
    const size_t S = j->S, S32 = S & ~(size_t)31;
    const __m256i low4 = _mm256_set1_epi8(0x0f);
    for (int r0 = 0; r0 < m; r0 += 2) {
        const int nr = m - r0 < 2 ? m - r0 : 2;
        for (size_t x = 0; x < S32; x += 32) {
            __m256i a0 = _mm256_setzero_si256(), a1 = a0;
            for (int c = 0; c < k; ++c) {
                const __m256i v = _mm256_loadu_si256((const __m256i *)(d + (size_t)c * S + x));
                const __m256i lo = _mm256_and_si256(v, low4);
                const __m256i hi = _mm256_and_si256(_mm256_srli_epi64(v, 4), low4);
                const uint8_t *t0 = j->nib + ((size_t)r0 * k + c) * 32;
                const __m256i tl0 = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)t0));
                const __m256i th0 = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)(t0 + 16)));
                a0 = _mm256_xor_si256(a0, _mm256_xor_si256(_mm256_shuffle_epi8(tl0, lo), _mm256_shuffle_epi8(th0, hi)));
                if (nr > 1) {
                    const uint8_t *t1 = t0 + (size_t)k * 32;
                    const __m256i tl1 = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)t1));
                    const __m256i th1 = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)(t1 + 16)));
                    a1 = _mm256_xor_si256(a1, _mm256_xor_si256(_mm256_shuffle_epi8(tl1, lo), _mm256_shuffle_epi8(th1, hi)));
                }
            }
            _mm256_storeu_si256((__m256i *)(p + (size_t)r0 * S + x), a0);
            if (nr > 1) _mm256_storeu_si256((__m256i *)(p + (size_t)(r0 + 1) * S + x), a1);
        }
    }
    if (S32 < S) scalar_cols(j, d, p, S32);
}

__attribute__((target("sse2"))) static void sfence_all(void) { _mm_sfence(); }

static void *simd_thread(void *arg)
{
    const simd_job *j = (const simd_job *)arg;
    for (size_t b = j->b0; b < j->b1; ++b) {
        const uint8_t *d = j->data + b * (size_t)j->k * j->S;
        uint8_t *p = j->parity + b * (size_t)j->m * j->S;
        if (j->isa == ISA_GFNI512) block_gfni(j, d, p);
        else if (j->isa == ISA_AVX2) block_avx2(j, d, p);
        else scalar_cols(j, d, p, 0);
    }
    if (j->isa == ISA_GFNI512) sfence_all();  /* order this thread's streaming stores */
    return NULL;
}

/* Encode n blocks (layout of memo_ec_encode_batch) with `isa` (< 0: best
 * available; a request above what the CPU has is clamped) on `threads`
 * threads.  Returns the ISA used (0 scalar, 1 AVX2, 2 GFNI+AVX-512) or -1. */
int memo_oracle_encode_simd_mt(int k, int m, size_t S, size_t n, const uint8_t *data,
                               uint8_t *parity, int threads, int isa)
{
    if (k < 1 || m < 1 || k + m > 256) return -1;
    const int best = memo_oracle_simd_isa();
    if (isa < 0 || isa > best) isa = best;
    uint8_t *C = (uint8_t *)malloc((size_t)(k + m) * k);
    uint64_t *aff = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)m * k);
    uint8_t *nib = (uint8_t *)malloc((size_t)m * k * 32);
    memo_oracle_cauchy(k, m, C);
    const uint8_t *coef = C + (size_t)k * k;
    for (int i = 0; i < m * k; ++i) {
        aff[i] = affine_matrix(coef[i]);
        for (int v = 0; v < 16; ++v) {
            nib[(size_t)i * 32 + v] = memo_oracle_gf_mul(coef[i], (uint8_t)v);
            nib[(size_t)i * 32 + 16 + v] = memo_oracle_gf_mul(coef[i], (uint8_t)(v << 4));
        }
    }
    if (threads < 1) threads = 1;
    if ((size_t)threads > n && n > 0) threads = (int)n;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    simd_job *jobs = (simd_job *)malloc(sizeof(simd_job) * (size_t)threads);
    for (int t = 0; t < threads; ++t) {
        jobs[t] = (simd_job){isa, k, m, S, n * (size_t)t / (size_t)threads,
                             n * (size_t)(t + 1) / (size_t)threads, data, parity, coef, aff, nib};
        pthread_create(&th[t], NULL, simd_thread, &jobs[t]);
    }
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    if (isa == ISA_GFNI512) sfence_all();
    free(th); free(jobs); free(C); free(aff); free(nib);
    return isa;
}

/* Rebuild with the same vectorised kernels (the CPU baseline of the rebuild
 * configs): per block, the decode rows C[lost] * inv(C[surv]) of the scalar
 * oracle (Gauss-Jordan), their affine matrices / nibble tables, then the MAC
 * of block_gfni / block_avx2 over the k survivors.  Layout of
 * memo_ec_rebuild_batch.  Returns the ISA used, or -1 (bad pattern).
 *
 * A thread with at least 1024 blocks memoises the rows and tables of the
 * erasure patterns it has decoded (a direct-mapped cache keyed by the
 * surv_idx || lost_idx bytes): a batch of a million 4 KiB blocks holds only
 * C(k+m, e) patterns, and re-deriving 8x8 bit matrices per block would cost
 * 20x the MAC.  The bytes are the same either way (the cache holds exactly
 * what a miss computes); shorter calls (the CPU baseline's timed sample)
 * decode every block. */
typedef struct {
    int isa, k, m, e;
    size_t S, b0, b1;
    const uint8_t *sidx, *surv, *lidx;
    uint8_t *out;
    int rc;
} rebuild_job;

enum { PAT_CACHE = 8192 };

static void *rebuild_thread(void *arg)
{
    rebuild_job *r = (rebuild_job *)arg;
    const int k = r->k, e = r->e, ek = e * k, klen = k + e;
    /* entry: key (k + e bytes) | valid | rows (e*k) | aff (e*k u64) | nib (e*k*32) */
    const size_t aff_off = ((size_t)klen + 1 + (size_t)ek + 7) & ~(size_t)7;
    const size_t ent = aff_off + (size_t)ek * 8 + (r->isa == ISA_AVX2 ? (size_t)ek * 32 : 0);
    /* the memo pays off over many blocks per thread (the whole-batch checks);
     * a short call (the CPU baseline's sample) decodes every block, as the
     * GPU does, and allocates no cache */
    size_t slots = 1;
    if (ek <= 256 && r->b1 - r->b0 >= 1024) {
        /* no more slots than erasure patterns (C(k+m, e)), rounded up to a
         * power of two: RS(3,2) needs 16, not 8192 entries per thread */
        double pats = 1.0;
        for (int i = 0; i < e; ++i) pats = pats * (double)(k + r->m - i) / (double)(i + 1);
        while (slots < PAT_CACHE && (double)slots < pats) slots <<= 1;
    }
    uint8_t *cache = (uint8_t *)calloc(slots, ent);
    if (!cache && slots > 1) cache = (uint8_t *)calloc(slots = 1, ent);  /* no memo, same bytes */
    for (size_t b = r->b0; b < r->b1 && cache; ++b) {
        const uint8_t *sv = r->sidx + b * k, *lv = r->lidx + b * e;
        uint32_t h = 2166136261u;
        for (int i = 0; i < k; ++i) h = (h ^ sv[i]) * 16777619u;
        for (int i = 0; i < e; ++i) h = (h ^ lv[i]) * 16777619u;
        uint8_t *c = cache + (size_t)(h & (uint32_t)(slots - 1)) * ent;
        uint8_t *rows = c + klen + 1;
        uint64_t *aff = (uint64_t *)(c + aff_off);
        uint8_t *nib = c + aff_off + (size_t)ek * 8;
        if (!(c[klen] && memcmp(c, sv, (size_t)k) == 0 && memcmp(c + k, lv, (size_t)e) == 0)) {
            if (memo_oracle_decode_matrix(k, r->m, sv, lv, e, rows)) {
                r->rc = -1;
                break;
            }
            for (int i = 0; i < ek; ++i) {
                if (r->isa == ISA_GFNI512) aff[i] = affine_matrix(rows[i]);
                else if (r->isa == ISA_AVX2)
                    for (int v = 0; v < 16; ++v) {
                        nib[(size_t)i * 32 + v] = memo_oracle_gf_mul(rows[i], (uint8_t)v);
                        nib[(size_t)i * 32 + 16 + v] = memo_oracle_gf_mul(rows[i], (uint8_t)(v << 4));
                    }
            }
            memcpy(c, sv, (size_t)k);
            memcpy(c + k, lv, (size_t)e);
            c[klen] = 1;
        }
        const simd_job j = {r->isa, k, e, r->S, 0, 0, NULL, NULL, rows, aff, nib};
        const uint8_t *d = r->surv + b * (size_t)k * r->S;
        uint8_t *o = r->out + b * (size_t)e * r->S;
        if (r->isa == ISA_GFNI512) block_gfni(&j, d, o);
        else if (r->isa == ISA_AVX2) block_avx2(&j, d, o);
        else scalar_cols(&j, d, o, 0);
    }
    if (!cache) r->rc = -1;
    if (r->isa == ISA_GFNI512) sfence_all();
    free(cache);
    return NULL;
}

int memo_oracle_rebuild_simd_mt(int k, int m, size_t S, size_t n, const uint8_t *surv_idx,
                                const uint8_t *surv, const uint8_t *lost_idx, int e,
                                uint8_t *out, int threads, int isa)
{
    if (k < 1 || m < 1 || k + m > 256 || e < 1 || e > m) return -1;
    const int best = memo_oracle_simd_isa();
    if (isa < 0 || isa > best) isa = best;
    if (threads < 1) threads = 1;
    if ((size_t)threads > n && n > 0) threads = (int)n;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    rebuild_job *jobs = (rebuild_job *)malloc(sizeof(rebuild_job) * (size_t)threads);
    for (int t = 0; t < threads; ++t) {
        jobs[t] = (rebuild_job){isa, k, m, e, S, n * (size_t)t / (size_t)threads,
                                n * (size_t)(t + 1) / (size_t)threads, surv_idx, surv, lost_idx, out, 0};
        pthread_create(&th[t], NULL, rebuild_thread, &jobs[t]);
    }
    int rc = isa;
    for (int t = 0; t < threads; ++t) {
        pthread_join(th[t], NULL);
        if (jobs[t].rc) rc = -1;
    }
    free(th); free(jobs);
    return rc;
}
