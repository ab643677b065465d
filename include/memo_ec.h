/*
 * memo_ec.h -- C ABI of the MI355X (gfx950) block erasure codec.
 *
 * Drop-in point in infinit/memo (reference, read-only):
 *   The codec replaces the byte movement of the immutable-block redundancy
 *   path, which in the reference is N-way replication:
 *     store  : Paxos::_store immutable branch + Details::send_immutable_block
 *              src/memo/model/doughnut/consensus/Paxos.cc:1713-1732, 1815-1817,
 *              315-391 (same B bytes sent to `factor` owners)
 *              -> memo_ec_encode_batch (k data + m parity shards, one per owner)
 *     fetch  : Paxos::Details::_fetch immutable branch, Paxos.cc:486-519
 *              (first replica that answers) -> any k shards +
 *              memo_ec_rebuild_batch when a data shard is missing
 *     repair : LocalPeer::_disappeared_evict / _rebalance, Paxos.cc:1012-1246
 *              (copy a surviving replica) -> memo_ec_rebuild_batch of the lost
 *              shards, batched over all under-sharded blocks
 *   The plugin surface it sits behind is unchanged:
 *     consensus::Configuration / Consensus virtuals
 *     src/memo/model/doughnut/Consensus.hh:24-174 (see host/ in this repo for
 *     the ErasureConsensus plugin built on this ABI), payload = the
 *     elle::Buffer of Block::data() (src/memo/model/blocks/Block.hh:142,
 *     elle/src/elle/Buffer.hh:34) handed over as plain pointer + size.
 *
 * Convention: GF(2^8), polynomial 0x11D, generator 2;
 * systematic ISA-L "cauchy1" generator: rows 0..k-1 identity, row i >= k,
 * column j = 1 / (i XOR j).  Shard size S = memo_ec_shard_size(B, k) =
 * round_up(ceil(B / k), 64); a block is zero-padded to k*S bytes and data
 * shard j is bytes [j*S, (j+1)*S) of the padded block.
 *
 * Memory layout of a batch (all pointers are caller-owned):
 *   data   : n blocks x k shards x S bytes, contiguous (block b at b*k*S)
 *   parity : n blocks x m shards x S bytes (parity i of block b at (b*m+i)*S)
 *   rebuild: surv_idx n x k (shard indices in [0,k+m)), surv n x k x S
 *            (the survivors' bytes, in surv_idx order), lost_idx n x e,
 *            out n x e x S (the rebuilt shards, in lost_idx order).
 *
 * Threading (mirrors elle::reactor::background, elle/src/elle/reactor/
 * scheduler.cc:562-602, which runs CPU work on <= 16 pool threads): a ctx is
 * used by one thread at a time; distinct ctxs are independent, so each pool
 * thread owns one.  The library owns only device scratch and streams.
 *
 * Errors are returned as negative codes (memo_ec_strerror); the C++ plugin
 * maps them to elle::Error-style exceptions (host/erasure_consensus.hh).
 */
#ifndef MEMO_EC_H
#define MEMO_EC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MEMO_EC_VERSION 2

/* Limits of this implementation. */
#define MEMO_EC_MAX_K 64
#define MEMO_EC_MAX_M 16
#define MEMO_EC_MAX_SEGMENTS 12          /* memo_ec_encode_segments  */
#define MEMO_EC_MAX_REBUILD_SEGMENTS 256 /* memo_ec_rebuild_segments */
/* Shards are shorter than 4 GiB (S < 2^32), and a call's buffers hold less
 * than 2^50 bytes (n * (k + m) * S, n * (k + e) * S; MEMO_EC_ERANGE
 * otherwise, before anything is sized from them). */

typedef struct memo_ec_ctx memo_ec_ctx;

/* Where the buffers of a call live. */
enum memo_ec_where {
    MEMO_EC_HOST = 0,        /* pageable host memory: synchronous call      */
    MEMO_EC_HOST_PINNED = 1, /* page-locked host memory: synchronous call   */
    MEMO_EC_DEVICE = 2       /* device memory of the ctx's GPU: the call is
                                enqueued on the ctx stream and returns; use
                                memo_ec_synchronize for completion/errors   */
};

enum memo_ec_status {
    MEMO_EC_OK = 0,
    MEMO_EC_EINVAL = -1,    /* bad argument (k, m, S, e, pointer, where)    */
    MEMO_EC_ENOMEM = -2,    /* device or pinned allocation failed           */
    MEMO_EC_EHIP = -3,      /* HIP runtime error                            */
    MEMO_EC_ESINGULAR = -4, /* survivor set cannot rebuild (duplicate or
                               out-of-range shard indices)                  */
    MEMO_EC_ENODEV = -5,    /* no such GPU                                  */
    MEMO_EC_ERANGE = -6     /* k or m beyond MEMO_EC_MAX_K / MEMO_EC_MAX_M  */
};

/* One (k, m, S) group of blocks for the fused mixed-geometry encode. */
typedef struct memo_ec_segment {
    int k, m;
    size_t S, n;
    const uint8_t *data; /* device: n x k x S */
    uint8_t *parity;     /* device: n x m x S */
} memo_ec_segment;

/* One (k, m, S) group of blocks of a mixed-geometry rebuild
 * (memo_ec_rebuild_segments).  Per-block patterns (uniform == 0): surv_idx
 * n x k and lost_idx n x e, in the memory `where` names.  One pattern for
 * the group (uniform != 0, the repair of one lost node): surv_idx k and
 * lost_idx e bytes in host memory, as for memo_ec_rebuild_uniform. */
typedef struct memo_ec_rebuild_segment {
    int k, m;
    size_t S, n;
    const uint8_t *surv_idx;
    const uint8_t *surv;     /* n x k x S, in surv_idx order     */
    const uint8_t *lost_idx;
    int e;                   /* lost shards per block, 0..m     */
    int uniform;
    uint8_t *out;            /* n x e x S, in lost_idx order     */
} memo_ec_rebuild_segment;

/* Per-context tuning (memo_ec_ctx_set_option).  Each starts from the
 * environment variable named beside it, read once by memo_ec_ctx_create;
 * a value the option refuses is ignored with a warning on stderr. */
enum memo_ec_option {
    MEMO_EC_OPT_REBUILD_PATH = 1,       /* MEMO_EC_REBUILD_FUSED: -1 auto (default),
                                           0 decode rows + MAC, 1 fused kernel
                                           (the variable: any value > 0 is 1,
                                           any value < 0 is auto)                */
    MEMO_EC_OPT_FUSED_MAX_BYTES = 2,    /* MEMO_EC_FUSED_MAX_MB: auto takes the fused
                                           kernel up to this many survivor bytes
                                           per call (256 MiB)                    */
    MEMO_EC_OPT_ZERO_COPY_BYTES = 3,    /* MEMO_EC_ZC_KB: host calls moving at most
                                           this many bytes run their kernels on
                                           pinned host memory (4 MiB; 0: off)    */
    MEMO_EC_OPT_PIPE_BYTES = 4,         /* MEMO_EC_PIPE_MB: host pipeline batch
                                           (64 MiB)                              */
    MEMO_EC_OPT_COPY_THREADS = 5,       /* MEMO_EC_COPY_THREADS: threads per pageable
                                           bounce copy (0: the shared pool's all;
                                           the variable set to 0 means 1, the
                                           calling thread only)                  */
    MEMO_EC_OPT_MAX_LAUNCH_TILES = 6,   /* MEMO_EC_MAX_LAUNCH_TILES: tiles per MAC
                                           launch (0: the 31-bit grid limit)     */
    MEMO_EC_OPT_XCD_MIN_TILES = 7,      /* MEMO_EC_XCD_MIN_TILES: smallest segment
                                           given the XCD-contiguous tile order   */
    MEMO_EC_OPT_DECODE_WIDE_MAX = 8,    /* MEMO_EC_DECODE_WIDE_MAX: decode-row batches
                                           up to this many blocks take the
                                           column-per-lane kernel (65536)        */
    MEMO_EC_OPT_DECODE_EXACT = 9,       /* MEMO_EC_DECODE_EXACT: exact-k decode
                                           kernels (1)                           */
    MEMO_EC_OPT_DECODE_STAGE = 10,      /* MEMO_EC_DECODE_STAGE: decode rows staged
                                           through LDS (0)                       */
    MEMO_EC_OPT_IMAGE_MIN_TILES = 11,   /* MEMO_EC_IMAGE_MIN_TILES: the decode rows +
                                           MAC rebuild forms per-block product-
                                           table images in HBM for shards of at
                                           least this many whole 4 KiB tiles
                                           (S / 4096) and runs the encode body
                                           over them (1; 0: never, tables built
                                           in LDS)                               */
    MEMO_EC_OPT_IMAGE_MIN_COEFS = 12,   /* MEMO_EC_IMAGE_MIN_COEFS: ... and at least
                                           this many coefficients per block
                                           (padded rows x columns; 40) or a k
                                           without a straight-line MAC body      */
    MEMO_EC_OPT_DECODE_OVERLAP = 13     /* MEMO_EC_DECODE_OVERLAP: a mixed rebuild runs
                                           the decode rows of its later launch
                                           classes on a side stream, overlapping
                                           the earlier MACs (1; 0: all decodes
                                           first, on the call's stream)          */
};

/* Number of GPUs the library can use (0 without a GPU).  A node process
 * spreads its batches over them, one ctx per device per host thread
 * (block-index partition, no collective). */
int memo_ec_device_count(void);

/* Identity of GPU `device`: its PCI bus id ("0000:c1:00.0", pci_len >= 13)
 * and UUID (32 hex digits, uuid_len >= 33), NUL-terminated into the caller's
 * buffers.  A node process that spreads batches over the GPUs records these
 * so a run can prove which physical devices did the work (two ranks naming
 * the same device is a placement error, not a scaling result). */
int memo_ec_device_identity(int device, char *pci_bus_id, size_t pci_len,
                            char *uuid, size_t uuid_len);

/* Context on GPU `device` (its own HIP stream, device scratch). */
int memo_ec_ctx_create(int device, memo_ec_ctx **out);
int memo_ec_ctx_destroy(memo_ec_ctx *ctx);

/* Set / read one memo_ec_option of a ctx (the ctx's owner thread only).
 * MEMO_EC_EINVAL for an unknown option or a value out of its range. */
int memo_ec_ctx_set_option(memo_ec_ctx *ctx, int option, int64_t value);
int memo_ec_ctx_get_option(memo_ec_ctx *ctx, int option, int64_t *value);

/* Enqueue MEMO_EC_DEVICE work on `hip_stream` (a hipStream_t; NULL restores
 * the ctx's own stream).  Lets a caller time kernels with its own events. */
int memo_ec_set_stream(memo_ec_ctx *ctx, void *hip_stream);
void *memo_ec_get_stream(memo_ec_ctx *ctx);

/* Wait for the ctx's enqueued work; returns the first deferred error
 * (e.g. MEMO_EC_ESINGULAR from a device-resident rebuild) and clears it. */
int memo_ec_synchronize(memo_ec_ctx *ctx);

/* round_up(ceil(B / k), 64) */
size_t memo_ec_shard_size(size_t block_bytes, int k);

/* Generator matrix (k+m) x k, row-major, into `out` (host memory). */
int memo_ec_generator(int k, int m, uint8_t *out);

/* parity_i = XOR_j C[k+i][j] * data_j for every block of the batch. */
int memo_ec_encode_batch(memo_ec_ctx *ctx, int k, int m, size_t S, size_t n,
                         const uint8_t *data, uint8_t *parity, int where);

/* Rebuild the e lost shards of each block from its k survivors.  A lost
 * index may name a data or a parity shard.  e == 0 is a no-op. */
int memo_ec_rebuild_batch(memo_ec_ctx *ctx, int k, int m, size_t S, size_t n,
                          const uint8_t *surv_idx, const uint8_t *surv,
                          const uint8_t *lost_idx, int e, uint8_t *out,
                          int where);

/* Diagnostic: the memory system's rate for an encode's own traffic.  Runs
 * the tiles, tile order and non-temporal 16-byte loads / stores that
 * memo_ec_encode_batch(k = kin, m = r) runs, with the GF arithmetic
 * replaced by XOR.  mode MEMO_EC_PROBE_COPY: out shard i of block b = XOR
 * of its kin input shards, every byte XOR i; MEMO_EC_PROBE_READ: the loads
 * alone (out unspecified); MEMO_EC_PROBE_WRITE: the stores alone (out
 * unspecified).  Device pointers only (in n x kin x S, out n x r x S);
 * asynchronous on the ctx stream.  The read and write launches' times
 * added give the "achievable" rate of the codec's roofline: this mix of
 * read and write streams without the cost of interleaving them (bench.py:
 * roofline.achievable, frac_of_achievable). */
enum memo_ec_probe_mode {
    MEMO_EC_PROBE_COPY = 0,
    MEMO_EC_PROBE_READ = 1,
    MEMO_EC_PROBE_WRITE = 2
};
int memo_ec_stream_probe(memo_ec_ctx *ctx, int kin, int r, size_t S, size_t n,
                         const uint8_t *in, uint8_t *out, int mode);

/* Page-locked host memory for MEMO_EC_HOST_PINNED calls (hipHostMalloc):
 * batch buffers the caller reuses, so its host-memory calls skip the
 * library's bounce copies.  NULL on failure.  Free with memo_ec_host_free. */
void *memo_ec_host_alloc(size_t bytes);
int memo_ec_host_free(void *p);

/* Rebuild with ONE erasure pattern for the whole batch: every block lost the
 * shards lost_idx[0..e) and is rebuilt from the survivors surv_idx[0..k)
 * (host pointers: k and e bytes), surv n x k x S in surv_idx order, out
 * n x e x S.  This is the repair of one lost node, where every block that
 * node held shard i of shares a pattern (Paxos::LocalPeer::_disappeared_evict,
 * src/memo/model/doughnut/consensus/Paxos.cc:1012-1087): the decode rows are
 * formed once on the host and their product tables are shared by all
 * blocks, as the encode's parity rows are, so the call runs at encode
 * speed.  An invalid pattern (duplicate or out-of-range index) returns
 * MEMO_EC_ESINGULAR before anything is enqueued.  `where` as for
 * memo_ec_rebuild_batch (surv/out memory only).  The ctx caches the tables
 * of its last 64 patterns; a pattern's first call uploads them
 * synchronously, so make that call before capturing a HIP graph. */
int memo_ec_rebuild_uniform(memo_ec_ctx *ctx, int k, int m, size_t S, size_t n,
                            const uint8_t *surv_idx, const uint8_t *surv,
                            const uint8_t *lost_idx, int e, uint8_t *out,
                            int where);

/* Per-block decode rows (n x e x k bytes, device): row r of block b holds the
 * coefficients of lost_idx[b][r] over the survivors in surv_idx[b] order,
 * i.e. C[lost] * inv(C[surv]) -- computed in closed form (one lane per block,
 * no matrix inversion), as memo_ec_rebuild_batch does before its
 * multiply-accumulate.  Device pointers only; asynchronous on the ctx
 * stream; invalid survivor sets give zero rows and MEMO_EC_ESINGULAR at
 * memo_ec_synchronize. */
int memo_ec_decode_rows(memo_ec_ctx *ctx, int k, int m, size_t n,
                        const uint8_t *surv_idx, const uint8_t *lost_idx,
                        int e, uint8_t *rows);

/* Batched encode of up to MEMO_EC_MAX_SEGMENTS device-resident segments
 * with different (k, m, S): segments of one shard-chunk class (same
 * specialised k) share one launch, classes run back to back.  Asynchronous
 * on the ctx stream. */
int memo_ec_encode_segments(memo_ec_ctx *ctx, int nseg,
                            const memo_ec_segment *segs);

/* Rebuild of up to MEMO_EC_MAX_REBUILD_SEGMENTS groups with different
 * (k, m, S, e) and per-block or shared erasure patterns in ONE call: the
 * read side of the multi-address fetch, which hands a whole batch of blocks
 * over at once (Consensus::_fetch(vector<AddressVersion>, ReceiveBlock),
 * src/memo/model/doughnut/Consensus.cc:101-124; Paxos::_fetch,
 * src/memo/model/doughnut/consensus/Paxos.cc:1857-1890).  Segments of one
 * shard-chunk class and kind share a launch (per-block patterns: the fused
 * kernel or decode rows + MAC; shared patterns: product tables formed once
 * on the host), classes run back to back.  Every segment is validated, and
 * every shared pattern decoded, before anything is enqueued (a bad shared
 * pattern: MEMO_EC_ESINGULAR).  MEMO_EC_DEVICE: asynchronous on the ctx
 * stream, per-block faults at memo_ec_synchronize; host memory: synchronous
 * through the copy pipeline, per-block faults returned (the other blocks
 * are still rebuilt). */
int memo_ec_rebuild_segments(memo_ec_ctx *ctx, int nseg,
                             const memo_ec_rebuild_segment *segs, int where);

/* Batched SHA-256 (FIPS 180-4): digest_i = SHA-256(prefix_i || msg_i) for
 * i < n, with prefix_i = prefix + i*prefix_stride (prefix_len bytes; 0 for
 * none) and msg_i = msg + i*msg_stride of msg_len[i] bytes (msg_len == NULL:
 * uniform_len for all).  digest: n x 32 bytes.  This is the CHB address hash
 * SHA-256(salt || owner || data) of CHB::_hash_address
 * (src/memo/model/doughnut/CHB.cc:264-289) and of CHB::_validate
 * (CHB.cc:79-99) for a whole batch; the caller sets address byte 31 to the
 * immutable flag (model/Address.hh: flag_byte).  Device pointers only;
 * asynchronous on the ctx stream. */
int memo_ec_sha256_batch(memo_ec_ctx *ctx, size_t n, const uint8_t *prefix,
                         size_t prefix_len, size_t prefix_stride,
                         const uint8_t *msg, size_t msg_stride,
                         const uint64_t *msg_len, size_t uniform_len,
                         uint8_t *digest);

/* Synthetic workload helpers (device memory; asynchronous on the ctx
 * stream).  Bytes and erasure patterns follow DESIGN.md section 6. */
int memo_ec_fill_blocks(memo_ec_ctx *ctx, uint64_t seed, uint64_t first_block,
                        size_t n, size_t B, int k, size_t S, uint8_t *out);
int memo_ec_erasures(uint64_t seed, uint64_t first_block, size_t n, int k,
                     int m, int e, uint8_t *surv_idx, uint8_t *lost_idx);
/* out[b][r] = shard idx[b][r] of block b, shards drawn from data (index < k)
 * or parity (index >= k).  Device memory; asynchronous. */
int memo_ec_gather_shards(memo_ec_ctx *ctx, int k, int m, size_t S, size_t n,
                          const uint8_t *data, const uint8_t *parity,
                          const uint8_t *idx, int cnt, uint8_t *out);

const char *memo_ec_strerror(int code);
int memo_ec_version(void);
/* SHA-256 (hex) of the sources this library was built from: include/
 * memo_ec.h, memo_amd/csrc/ec_kernels.h, ec_kernels.hip and memo_ec.cpp,
 * concatenated in that order (memo_amd/csrc/Makefile).  Callers compare it
 * with the sources they ship to prove the loaded kernels are theirs. */
const char *memo_ec_build_id(void);

#ifdef __cplusplus
}
#endif
#endif /* MEMO_EC_H */
