// ec_kernels.h -- launch-side interface of the gfx950 codec kernels
// (internal to libmemo_ec.so; the public ABI is include/memo_ec.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/memo_ec.h"

namespace memo_ec {

// Design choices fixed by measurement (DESIGN.md 4.1 and profiles/HISTORY.md
// 4.1 hold the rejected alternatives and their numbers; their code is gone):
//  - streamed shard loads and output stores are non-temporal (read/written
//    once; plain: 5% slower);
//  - shards fold pairwise, three 3-input XORs per 2 coefficients, also for
//    k = 16 (unpaired: 1-3 points slower);
//  - rebuild tables are built 4 coefficients per lane at once (packed
//    doublings) into split q / lo LDS regions with one pad slot per set
//    (the interleaved 8-dword images cost 2/3 of the 4 KiB RS(16,4)
//    rebuild's LDS cycles in bank conflicts);
//  - straight-line bodies for k = 6, 12, 14 (R <= 4) besides 2, 3, 4, 10, 16.
constexpr bool MAC_NT = true;
// Table dwords per lane staged through registers ahead of the shard loads:
// two sets of R x kpad <= 64 images (a tile across two blocks' per-block
// images); the encode's one shared set needs two.
constexpr int MAC_TAB_REGS = 4;
// Coefficients per lane staged through registers (rebuild tables built in
// LDS): 256 * 6 = 1536 slots, the most a flat-mapped rebuild tile builds
// (launch planning in memo_ec.cpp keeps to it).
constexpr int MAC_COEF_REGS = 6;
// A tile = 256 16-byte columns = one workgroup of gf_mac_kernel.
constexpr uint32_t MAC_TILE = 256;
// Shard-index bytes per lane staged through registers by the fused rebuild
// (the rest of a tile's indices, if any, are loaded after the shards).
constexpr int DEC_IDX_REGS = 2;

// What a MAC launch multiplies with: a precomputed table image (encode), a
// per-block coefficient row from decode_coef_kernel (two-kernel rebuild), or
// rows the tile derives from the shard indices itself (fused rebuild).
// MAC_PROBE: the same traffic without the GF arithmetic (stream_probe_kernel).
// MAC_IMAGES: a rebuild over per-block table images -- the encode's code
// under a kernel name of its own (gf_mac_images_kernel), so traces tell a
// rebuild MAC from an encode.
enum MacMode : int { MAC_ENCODE = 0, MAC_ROWS = 1, MAC_FUSED = 2, MAC_PROBE = 3, MAC_IMAGES = 4,
                     MAC_PERM = 5 /* MEMO_EC_PERM_PROBE builds only (tools/perm_probe.py) */ };

// LDS bytes of the fused rebuild's decode workspace for a tile of ns blocks:
// GF log/antilog (1 KiB), LW0 (128 B), per block 3 survivor-mask words + a
// fault word, the survivor and lost indices, log W_t and log Lam_l.
// Per-wave LDS copy of the GF log/antilog tables + LW0 (wave-local decode).
constexpr uint32_t DEC_WAVE_BYTES = 1152;
__host__ __device__ constexpr uint32_t dec_r4(uint32_t x) { return (x + 3u) & ~3u; }
__host__ __device__ constexpr uint32_t dec_ws_bytes(uint32_t ns, uint32_t k, uint32_t e) {
  return 1024u + 128u + 16u * ns + 2u * dec_r4(ns * k) + 2u * dec_r4(ns * e);
}

// One (kin -> r) multiply-accumulate over n blocks.
struct MacSeg {
  const uint8_t* in;      // block b, input shard j at in + b*in_bstride + j*in_sstride
  uint8_t* out;           // block b, output shard i at out + b*out_bstride + i*out_sstride
  const uint32_t* tab;    // product-table image(s): R x kpad coefficients x 8 dwords
  uint64_t in_bstride, in_sstride;
  uint64_t out_bstride, out_sstride;
  uint64_t tab_bstride;   // dwords between blocks' images; 0 = one image for all
  const uint8_t* coef;    // rebuild: block b's coefficient rows at coef + b*coef_bstride,
  uint64_t coef_bstride;  //   coef_rows x kin bytes (tables built in LDS; tab unused);
                          //   coef_bstride 0: one set of rows for every block
  uint32_t coef_rows;
  uint32_t coef_dense;    // 1: per-block rows are exactly R x kpad (kin == kpad, R ==
                          //   coef_rows, coef_bstride == R * kin): slot ci of a tile is
                          //   byte ci of its range
  uint32_t lo_dw;         // per-coefficient tables: LDS dword offset of the lo region
  uint64_t n;             // blocks
  uint64_t tiles;         // tiles (= workgroups) of this segment
  uint64_t tiles_per_block;  // aligned mapping only
  uint32_t chunks;        // C = S / 16
  uint32_t kin, r, kpad;
  uint32_t flat;          // 1: flattened (block, column) units; 0: tile inside one block
  uint32_t wg_begin;      // first workgroup of this segment
  // fused rebuild (gf_rebuild_kernel): the tile derives its blocks' decode
  // rows from the shard indices itself (coef unused)
  const uint8_t* sidx;    // n x kin survivor indices (surv_idx order)
  const uint8_t* lidx;    // n x r lost indices (lost_idx order)
  const uint32_t* lw0;    // LW0(i) = log sigma(i) - log Pall(i), i < kin + m (bytes, per code)
  uint32_t* status;       // set to 1 on an invalid survivor / lost index set
  uint32_t m;             // parity shards of the code (kin + m = shard count)
  uint32_t ws_dw;         // LDS dword offset of the decode workspace
  uint32_t probe;         // stream_probe_kernel: a memo_ec_probe_mode
};

struct MacLaunch {
  uint32_t nseg;
  uint32_t xcd;  // 1: XCD-contiguous tile order inside each segment (see gf_mac_kernel)
  MacSeg seg[MEMO_EC_MAX_SEGMENTS];
};

struct DecodeArgs {
  const uint8_t* surv_idx;
  const uint8_t* lost_idx;
  uint8_t* rows;          // n x e x k decode rows
  uint32_t* status;       // set to 1 on an invalid survivor set (device or pinned host word)
  uint64_t n;
  uint32_t k, m, e;
  uint32_t pitch;         // decode_coef_kernel: LDS row-staging pitch (set by the launcher)
  const uint32_t* lw0;    // LW0 table of (k, m) (lw0_host; 128 bytes); null: computed per workgroup
  // kernel choice (the ctx's MEMO_EC_OPT_DECODE_* options)
  uint64_t wide_max;      // batches up to this many blocks: column-per-lane kernel
  uint32_t exact;         // 1: exact-k kernels for k in {2,3,4,6,8,10,12,14,16}
  uint32_t stage;         // 1: exact-k rows staged through LDS
  // optional: per-block product-table images of the rows, block b's R x kpad
  // slots of 8 dwords (table_dword's layout) at img + b * R * kpad * 8, so
  // gf_mac_kernel runs its encode body over them (tab_bstride = R * kpad * 8);
  // written by the column-per-lane kernel, which every segment with images
  // takes (kpad <= its lanes per block)
  uint32_t* img;
  uint32_t R, kpad;
};

// Decode rows of up to MEMO_EC_MAX_SEGMENTS segments in one launch: the
// workgroups of segment s start at wg_begin[s].
struct DecodeLaunch {
  uint32_t nseg;
  uint32_t wg_begin[MEMO_EC_MAX_SEGMENTS];
  DecodeArgs seg[MEMO_EC_MAX_SEGMENTS];
};

struct Sha256Args {
  const uint8_t* prefix;  // message i = prefix + i*prefix_stride (prefix_len B) || msg_i
  const uint8_t* msg;     // msg_i = msg + i*msg_stride, msg_len[i] (or uniform_len) bytes
  const uint64_t* msg_len;
  uint8_t* digest;        // n x 32
  uint64_t n, prefix_len, prefix_stride, msg_stride, uniform_len;
};

struct FillArgs {
  uint8_t* out;
  uint64_t seed, first_block, n, B, stride;
};

struct GatherArgs {
  const uint8_t* data;
  const uint8_t* parity;
  const uint8_t* idx;
  uint8_t* out;
  uint64_t S, n;
  uint32_t k, m, cnt;
};

// Compile-time output bound R >= r (rows r..R-1 are zero) and shard chunk KC
// (shards beyond kin inside the last chunk are zero) used for (kin, R).
int mac_rbound(int r);
int mac_kchunk(int kin, int R);
void table_image_host(const uint8_t* coef, uint32_t r, uint32_t kin, uint32_t R, uint32_t kpad,
                      uint32_t* out);
hipError_t launch_mac(int KC, int R, int mode, const MacLaunch& L, uint32_t grid, size_t lds,
                      hipStream_t st);
// LW0 table of (k, m) for the fused rebuild: 128 bytes (entries i < k + m).
void lw0_host(int k, int m, uint8_t* out);
hipError_t launch_decode_coef(const DecodeArgs& a, hipStream_t st);  // closed-form decode rows
hipError_t launch_decode_multi(const DecodeArgs* a, int n, hipStream_t st);  // several segments
hipError_t launch_fill(const FillArgs& a, hipStream_t st);
hipError_t launch_sha256(const Sha256Args& a, hipStream_t st);
hipError_t launch_gather(const GatherArgs& a, hipStream_t st);
const uint8_t* host_gf_log();
const uint8_t* host_gf_exp();

}  // namespace memo_ec
