// ec_kernels.h -- launch-side interface of the gfx950 codec kernels
// (internal to libmemo_ec.so; the public ABI is include/memo_ec.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/memo_ec.h"

namespace memo_ec {

// Columns (16-byte units) per lane per tile; a tile is 256 * MAC_V units.
constexpr int MAC_V = 1;
constexpr uint32_t MAC_UNITS = 256 * MAC_V;
// Streamed shard loads / parity stores bypass cache retention (read once).
constexpr bool MAC_NT = true;

// One (kin -> r) multiply-accumulate over n blocks.
struct MacSeg {
  const uint8_t* in;      // block b, input shard j at in + b*in_bstride + j*in_sstride
  uint8_t* out;           // block b, output shard i at out + b*out_bstride + i*out_sstride
  const uint8_t* coef;    // r x kin per block (coef_bstride apart); nullptr = Cauchy parity rows
  uint64_t in_bstride, in_sstride;
  uint64_t out_bstride, out_sstride;
  uint64_t coef_bstride;
  uint64_t n;             // blocks
  uint64_t tiles;         // work tiles of this segment
  uint64_t tiles_per_block;  // aligned mapping only
  uint32_t chunks;        // C = S / 16
  uint32_t kin, r;
  uint32_t flat;          // 1: flattened (block, column) units; 0: tile inside one block
  uint32_t wg_begin;      // first workgroup of this segment
  uint32_t wgs;           // workgroups of this segment (contiguous tile ranges)
};

struct MacLaunch {
  uint32_t nseg;
  uint32_t pad_;
  MacSeg seg[MEMO_EC_MAX_SEGMENTS];
};

struct DecodeArgs {
  const uint8_t* surv_idx;
  const uint8_t* lost_idx;
  uint8_t* rows;
  uint32_t* status;
  uint64_t n;
  uint32_t k, m, e;
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
// (shards beyond kin inside the last chunk are zero) used for (kin, r).
int mac_rbound(int r);
int mac_kchunk(int kin);
hipError_t launch_mac(int KC, int R, bool shared, const MacLaunch& L, uint32_t grid, size_t lds,
                      hipStream_t st);
hipError_t launch_decode_rows(const DecodeArgs& a, hipStream_t st);
hipError_t launch_fill(const FillArgs& a, hipStream_t st);
hipError_t launch_gather(const GatherArgs& a, hipStream_t st);
const uint8_t* host_gf_log();
const uint8_t* host_gf_exp();

}  // namespace memo_ec
