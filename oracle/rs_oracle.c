/*
 * rs_oracle.c -- CPU restatement of the block erasure-coding path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker and the CPU
 * baseline ("cpu_baseline.kind" = "port").  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product path
 * (memo_amd/csrc, libmemo_ec.so) never links or calls it.
 *
 * PARITY UNPINNED BY THE REFERENCE: infinit/memo contains no erasure code and
 * no GF(2^8) arithmetic.  Its redundancy path is whole-
 * block N-way replication:
 *   - store:   Paxos::_store immutable branch -> Details::send_immutable_block
 *              (src/memo/model/doughnut/consensus/Paxos.cc:1713-1732,1815-1817,
 *               315-391): the same B bytes go to `factor` owners;
 *   - fetch:   Details::_fetch immutable branch (Paxos.cc:486-519): any one
 *              replica returns the B bytes;
 *   - repair:  _disappeared_evict/_rebalance (Paxos.cc:1012-1246): copy a
 *              surviving replica to a new owner.
 * The codec below replaces those byte movements with "k data + m parity
 * shards, any k rebuild the block".  Because the reference has no codec, the
 * byte convention is fixed here and pinned by:
 *   (1) the field: GF(2^8) with polynomial 0x11D and generator 2, the field of
 *       ISO/IEC 18004 (QR code) Reed-Solomon; tests/test_oracle.py checks the
 *       published QR log/antilog values and the published "HELLO WORLD" 1-M
 *       EC codewords against gf_mul/gf_exp here;
 *   (2) the generator matrix: Intel ISA-L's gf_gen_cauchy1_matrix (ISA-L
 *       erasure_code, all 2.x releases; not vendored in the reference nor
 *       installed in this image) -- rows 0..k-1 identity, row i>=k col j =
 *       gf_inv(i ^ j);  encode = ISA-L ec_encode_data semantics
 *       (parity_i[x] = XOR_j C[k+i][j] * D_j[x]);
 *   (3) an independent numpy restatement (oracle/rs_numpy.py, carry-less
 *       Russian-peasant multiply, no tables) whose outputs are the golden
 *       fixtures under tests/golden/ (generator: tests/golden/make_golden.py).
 *
 * Shard convention: S = round_up(ceil(B/k), 64);
 * a block is zero-padded to k*S bytes; data shard j = bytes [j*S, (j+1)*S).
 *
 * Synthetic inputs: block bytes are a splitmix64
 * stream keyed by (seed, block_index); erasure patterns are drawn from a
 * splitmix64 stream keyed by (seed + 1, block_index).
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdlib.h>
#include <pthread.h>

#define GF_POLY 0x11D

static uint8_t gf_exp_t[512];
static uint8_t gf_log_t[256];
static uint8_t gf_mul_t[256][256]; /* scalar codec product table */
static int gf_ready = 0;
static pthread_once_t gf_once = PTHREAD_ONCE_INIT;

static void gf_init_impl(void)
{
    unsigned x = 1;
    for (int i = 0; i < 255; ++i) {
        gf_exp_t[i] = (uint8_t)x;
        gf_log_t[x] = (uint8_t)i;
        x <<= 1;
        if (x & 0x100) x ^= GF_POLY;
    }
    for (int i = 255; i < 512; ++i) gf_exp_t[i] = gf_exp_t[i - 255];
    gf_log_t[0] = 0; /* unused: callers test for zero */
    for (int a = 0; a < 256; ++a)
        for (int b = 0; b < 256; ++b)
            gf_mul_t[a][b] = (a && b) ? gf_exp_t[gf_log_t[a] + gf_log_t[b]] : 0;
    gf_ready = 1;
}

static void gf_init(void) { if (!gf_ready) pthread_once(&gf_once, gf_init_impl); }

uint8_t memo_oracle_gf_mul(uint8_t a, uint8_t b) { gf_init(); return gf_mul_t[a][b]; }
uint8_t memo_oracle_gf_exp(int i) { gf_init(); return gf_exp_t[((i % 255) + 255) % 255]; }
uint8_t memo_oracle_gf_log(uint8_t a) { gf_init(); return gf_log_t[a]; }

uint8_t memo_oracle_gf_inv(uint8_t a)
{
    gf_init();
    if (!a) return 0;
    return gf_exp_t[255 - gf_log_t[a]];
}

size_t memo_oracle_shard_size(size_t B, int k)
{
    size_t per = (B + (size_t)k - 1) / (size_t)k;
    if (per == 0) per = 1;
    return (per + 63) & ~(size_t)63;
}

/* ISA-L gf_gen_cauchy1_matrix restated: a is (k+m) x k row-major. */
int memo_oracle_cauchy(int k, int m, uint8_t *a)
{
    if (k < 1 || m < 0 || k + m > 256) return -1;
    gf_init();
    memset(a, 0, (size_t)(k + m) * k);
    for (int i = 0; i < k; ++i) a[(size_t)i * k + i] = 1;
    for (int i = k; i < k + m; ++i)
        for (int j = 0; j < k; ++j)
            a[(size_t)i * k + j] = memo_oracle_gf_inv((uint8_t)(i ^ j));
    return 0;
}

/* Gauss-Jordan inversion of an n x n matrix over GF(2^8) (ISA-L
 * gf_invert_matrix semantics).  Returns 0, or -1 if singular. */
int memo_oracle_invert(int n, const uint8_t *in, uint8_t *out)
{
    gf_init();
    uint8_t *w = (uint8_t *)malloc((size_t)n * n);
    if (!w) return -2;
    memcpy(w, in, (size_t)n * n);
    memset(out, 0, (size_t)n * n);
    for (int i = 0; i < n; ++i) out[(size_t)i * n + i] = 1;
    for (int c = 0; c < n; ++c) {
        int p = c;
        while (p < n && w[(size_t)p * n + c] == 0) ++p;
        if (p == n) { free(w); return -1; }
        if (p != c) {
            for (int j = 0; j < n; ++j) {
                uint8_t t = w[(size_t)c * n + j]; w[(size_t)c * n + j] = w[(size_t)p * n + j]; w[(size_t)p * n + j] = t;
                t = out[(size_t)c * n + j]; out[(size_t)c * n + j] = out[(size_t)p * n + j]; out[(size_t)p * n + j] = t;
            }
        }
        uint8_t iv = memo_oracle_gf_inv(w[(size_t)c * n + c]);
        for (int j = 0; j < n; ++j) {
            w[(size_t)c * n + j] = gf_mul_t[iv][w[(size_t)c * n + j]];
            out[(size_t)c * n + j] = gf_mul_t[iv][out[(size_t)c * n + j]];
        }
        for (int r = 0; r < n; ++r) {
            if (r == c) continue;
            uint8_t f = w[(size_t)r * n + c];
            if (!f) continue;
            for (int j = 0; j < n; ++j) {
                w[(size_t)r * n + j] ^= gf_mul_t[f][w[(size_t)c * n + j]];
                out[(size_t)r * n + j] ^= gf_mul_t[f][out[(size_t)c * n + j]];
            }
        }
    }
    free(w);
    return 0;
}

/* Decode rows for one erasure pattern: out (e x k) such that
 * shard[lost[r]] = XOR_j out[r][j] * shard[surv[j]].
 * Row for a lost data shard d: row d of inv(C_surv).
 * Row for a lost parity shard p: C[p] * inv(C_surv).  */
int memo_oracle_decode_matrix(int k, int m, const uint8_t *surv, const uint8_t *lost,
                              int e, uint8_t *out)
{
    gf_init();
    if (k < 1 || m < 0 || k + m > 256 || e < 0 || e > m) return -1;
    uint8_t *C = (uint8_t *)malloc((size_t)(k + m) * k);
    uint8_t *A = (uint8_t *)malloc((size_t)k * k);
    uint8_t *I = (uint8_t *)malloc((size_t)k * k);
    int rc = 0;
    memo_oracle_cauchy(k, m, C);
    for (int r = 0; r < k; ++r) {
        if (surv[r] >= k + m) { rc = -1; goto done; }
        memcpy(A + (size_t)r * k, C + (size_t)surv[r] * k, (size_t)k);
    }
    if (memo_oracle_invert(k, A, I)) { rc = -3; goto done; }
    for (int r = 0; r < e; ++r) {
        int l = lost[r];
        if (l >= k + m) { rc = -1; goto done; }
        for (int j = 0; j < k; ++j) {
            uint8_t acc = 0;
            for (int t = 0; t < k; ++t) acc ^= gf_mul_t[C[(size_t)l * k + t]][I[(size_t)t * k + j]];
            out[(size_t)r * k + j] = acc;
        }
    }
done:
    free(C); free(A); free(I);
    return rc;
}

/* out[b][r] = XOR_j M[r][j] * in[b][j]; blocks are contiguous shards. */
static void mac_blocks(int kin, int rout, size_t S, size_t b0, size_t b1,
                       const uint8_t *in, size_t in_bstride,
                       const uint8_t *M, size_t m_bstride,
                       uint8_t *out, size_t out_bstride)
{
    for (size_t b = b0; b < b1; ++b) {
        const uint8_t *ib = in + b * in_bstride;
        const uint8_t *Mb = M + b * m_bstride;
        uint8_t *ob = out + b * out_bstride;
        for (int r = 0; r < rout; ++r) {
            uint8_t *o = ob + (size_t)r * S;
            memset(o, 0, S);
            for (int j = 0; j < kin; ++j) {
                const uint8_t *row = gf_mul_t[Mb[(size_t)r * kin + j]];
                const uint8_t *d = ib + (size_t)j * S;
                for (size_t x = 0; x < S; ++x) o[x] ^= row[d[x]];
            }
        }
    }
}

int memo_oracle_encode(int k, int m, size_t S, size_t n, const uint8_t *data, uint8_t *parity)
{
    gf_init();
    if (k < 1 || m < 1 || k + m > 256) return -1;
    uint8_t *C = (uint8_t *)malloc((size_t)(k + m) * k);
    memo_oracle_cauchy(k, m, C);
    mac_blocks(k, m, S, 0, n, data, (size_t)k * S, C + (size_t)k * k, 0, parity, (size_t)m * S);
    free(C);
    return 0;
}

/* surv_idx: n x k, surv: n x k x S, lost_idx: n x e, out: n x e x S */
int memo_oracle_rebuild(int k, int m, size_t S, size_t n, const uint8_t *surv_idx,
                        const uint8_t *surv, const uint8_t *lost_idx, int e, uint8_t *out)
{
    gf_init();
    if (e == 0) return 0;
    uint8_t *D = (uint8_t *)malloc((size_t)e * k);
    for (size_t b = 0; b < n; ++b) {
        int rc = memo_oracle_decode_matrix(k, m, surv_idx + b * k, lost_idx + b * e, e, D);
        if (rc) { free(D); return rc; }
        mac_blocks(k, e, S, 0, 1, surv + b * k * S, 0, D, 0, out + b * e * S, 0);
    }
    free(D);
    return 0;
}

/* ---------------------------------------------------------------- threads */
typedef struct {
    int kin, rout; size_t S, b0, b1;
    const uint8_t *in; size_t in_bs;
    const uint8_t *M; size_t m_bs;
    uint8_t *out; size_t out_bs;
} mac_job;

static void *mac_thread(void *p)
{
    mac_job *j = (mac_job *)p;
    mac_blocks(j->kin, j->rout, j->S, j->b0, j->b1, j->in, j->in_bs, j->M, j->m_bs, j->out, j->out_bs);
    return NULL;
}

static int run_mt(int threads, int kin, int rout, size_t S, size_t n, const uint8_t *in,
                  size_t in_bs, const uint8_t *M, size_t m_bs, uint8_t *out, size_t out_bs)
{
    if (threads < 1) threads = 1;
    if ((size_t)threads > n && n > 0) threads = (int)n;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    mac_job *jobs = (mac_job *)malloc(sizeof(mac_job) * (size_t)threads);
    for (int t = 0; t < threads; ++t) {
        size_t b0 = n * (size_t)t / (size_t)threads, b1 = n * (size_t)(t + 1) / (size_t)threads;
        jobs[t] = (mac_job){kin, rout, S, b0, b1, in, in_bs, M, m_bs, out, out_bs};
        pthread_create(&th[t], NULL, mac_thread, &jobs[t]);
    }
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    free(th); free(jobs);
    return 0;
}

/* CPU baseline: encode partitioned by block index over `threads` threads. */
int memo_oracle_encode_mt(int k, int m, size_t S, size_t n, const uint8_t *data,
                          uint8_t *parity, int threads)
{
    gf_init();
    if (k < 1 || m < 1 || k + m > 256) return -1;
    uint8_t *C = (uint8_t *)malloc((size_t)(k + m) * k);
    memo_oracle_cauchy(k, m, C);
    run_mt(threads, k, m, S, n, data, (size_t)k * S, C + (size_t)k * k, 0, parity, (size_t)m * S);
    free(C);
    return 0;
}

/* CPU baseline: rebuild; decode matrices per block first (cheap), then the
 * MAC partitioned by block index. */
int memo_oracle_rebuild_mt(int k, int m, size_t S, size_t n, const uint8_t *surv_idx,
                           const uint8_t *surv, const uint8_t *lost_idx, int e,
                           uint8_t *out, int threads)
{
    gf_init();
    if (e == 0) return 0;
    uint8_t *D = (uint8_t *)malloc((size_t)e * k * (n ? n : 1));
    for (size_t b = 0; b < n; ++b) {
        int rc = memo_oracle_decode_matrix(k, m, surv_idx + b * k, lost_idx + b * e, e, D + b * e * k);
        if (rc) { free(D); return rc; }
    }
    run_mt(threads, k, e, S, n, surv, (size_t)k * S, D, (size_t)e * k, out, (size_t)e * S);
    free(D);
    return 0;
}

/* ------------------------------------------------------- synthetic inputs */
static inline uint64_t sm64_mix(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
#define SM64_GAMMA 0x9E3779B97F4A7C15ULL

/* Key of the splitmix64 stream of (seed, block). */
uint64_t memo_oracle_block_key(uint64_t seed, uint64_t block)
{
    return sm64_mix(sm64_mix(seed) ^ (block * SM64_GAMMA));
}

/* Fill n padded blocks: block b (global index first_block + b) occupies
 * k*S bytes at out + b*k*S; bytes [0,B) are the little-endian bytes of
 * splitmix64 outputs w_i = mix(key + (i+1)*GAMMA), the rest are zero. */
void memo_oracle_fill_blocks(uint64_t seed, uint64_t first_block, size_t n, size_t B,
                             int k, size_t S, uint8_t *out)
{
    size_t stride = (size_t)k * S;
    for (size_t b = 0; b < n; ++b) {
        uint8_t *p = out + b * stride;
        uint64_t key = memo_oracle_block_key(seed, first_block + b);
        size_t t = 0;
        for (uint64_t i = 0; t < B; ++i) {
            uint64_t w = sm64_mix(key + (i + 1) * SM64_GAMMA);
            for (int q = 0; q < 8 && t < B; ++q, ++t) p[t] = (uint8_t)(w >> (8 * q));
        }
        memset(p + B, 0, stride - B);
    }
}

/* Erasure pattern of block b: partial Fisher-Yates over [0, k+m) with the
 * stream keyed by (seed + 1, b); lost = first e picks sorted ascending;
 * survivors = the k lowest remaining indices (systematic shards first). */
void memo_oracle_erasures(uint64_t seed, uint64_t first_block, size_t n, int k, int m, int e,
                          uint8_t *surv_idx, uint8_t *lost_idx)
{
    int total = k + m;
    uint8_t perm[256], isl[256];
    for (size_t b = 0; b < n; ++b) {
        uint64_t key = memo_oracle_block_key(seed + 1, first_block + b);
        for (int i = 0; i < total; ++i) { perm[i] = (uint8_t)i; isl[i] = 0; }
        for (int i = 0; i < e; ++i) {
            uint64_t w = sm64_mix(key + (uint64_t)(i + 1) * SM64_GAMMA);
            int r = i + (int)(w % (uint64_t)(total - i));
            uint8_t t = perm[i]; perm[i] = perm[r]; perm[r] = t;
            isl[perm[i]] = 1;
        }
        int li = 0, si = 0;
        for (int i = 0; i < total; ++i) {
            if (isl[i]) lost_idx[b * e + li++] = (uint8_t)i;
            else if (si < k) surv_idx[b * k + si++] = (uint8_t)i;
        }
    }
}

/* Gather survivor shards of n encoded blocks (data n x k x S, parity n x m x S)
 * into surv (n x k x S) by surv_idx, and the expected lost shards into lost. */
void memo_oracle_gather(int k, int m, size_t S, size_t n, const uint8_t *data,
                        const uint8_t *parity, const uint8_t *idx, int cnt, uint8_t *out)
{
    for (size_t b = 0; b < n; ++b)
        for (int r = 0; r < cnt; ++r) {
            int s = idx[b * cnt + r];
            const uint8_t *src = s < k ? data + (b * k + s) * S : parity + (b * m + (s - k)) * S;
            memcpy(out + (b * cnt + r) * S, src, S);
        }
}
