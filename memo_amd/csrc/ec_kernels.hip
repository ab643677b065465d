// ec_kernels.hip -- gfx950 kernels of the block erasure codec.
//
// Hot path: gf_mac_kernel, the batched GF(2^8) multiply-accumulate
//   out[b][i][x] = XOR_j coef_b[i][j] * in[b][j][x]
// which is RS encode (coef = the Cauchy parity rows, shared by every block)
// and RS rebuild (coef = per-block decode rows from decode_coef_kernel).
// It replaces the replication byte movement of Paxos::Details::
// send_immutable_block / _fetch / _rebalance (src/memo/model/doughnut/
// consensus/Paxos.cc:315-391, 486-519, 1012-1246); see DESIGN.md.
//
// Design, measured on MI355X (tools/hbm_probe.hip):
//  * HBM-bound streaming.  One workgroup = one tile of 256 16-byte columns;
//    each lane loads the same 16 bytes of every input shard (dwordx4: a wave
//    reads 1 KiB of one shard per instruction, fully coalesced) and stores
//    16 bytes of every output shard, non-temporal.  One tile per workgroup
//    and a grid of all tiles beat persistent/grid-stride loops (the shard
//    pattern probe: 5.69 TB/s at 1 unit/lane vs 5.26 at 8).
//  * The kin loads are issued before anything else; the workgroup copies its
//    product tables (global image -> LDS) while they are in flight.
//  * Byte-field GF multiply on the VALU, no MFMA: a data byte x is split into
//    3+3+2-bit fields (x>>5, (x>>2)&7, x&3); c*x = T_hi[x>>5] ^ T_mid[(x>>2)&7]
//    ^ T_lo[x&3].  Each table has <= 8 byte entries, so one v_perm_b32 looks
//    up 4 bytes at once: 3 perms + 1.5 v_bitop3_b32 (3-input XOR) per
//    coefficient per dword; the field selectors are shared by all outputs.
//  * Rebuild coefficients come from decode_coef_kernel: a closed-form
//    (Cauchy/Lagrange) decode, one lane per block, with the GF log/antilog
//    tables in LDS.  The MAC builds each block's product tables in LDS from
//    its coefficient row (gf_xtime doublings), so per-block tables never
//    travel through HBM.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "ec_kernels.h"

namespace memo_ec {

// ----------------------------------------------------------------- GF tables
struct GfTables {
  uint8_t log[256];
  uint8_t exp[768];  // exp[i] = 2^(i mod 255): sums of three logs index it unreduced
};

constexpr GfTables make_gf() {
  GfTables t{};
  unsigned x = 1;
  for (int i = 0; i < 255; ++i) {
    t.exp[i] = (uint8_t)x;
    t.log[x] = (uint8_t)i;
    x <<= 1;
    if (x & 0x100) x ^= 0x11D;
  }
  for (int i = 255; i < 768; ++i) t.exp[i] = t.exp[i - 255];
  t.log[0] = 0;
  return t;
}

__constant__ GfTables kGf = make_gf();
constexpr int kGfDwords = sizeof(GfTables) / 4;
const GfTables kGfHost = make_gf();

__host__ __device__ __forceinline__ uint32_t gf_mul_t(const uint8_t* lg, const uint8_t* ex,
                                                      uint32_t a, uint32_t b) {
  return (a && b) ? ex[lg[a] + lg[b]] : 0u;
}

// Copy the 1024-byte log/antilog image into LDS (256 dwords).
__device__ __forceinline__ void stage_gf(uint32_t* s_gf) {
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&kGf);
  for (int i = threadIdx.x; i < kGfDwords; i += blockDim.x) s_gf[i] = src[i];
}

// Product-table dword q of coefficient c.  Image per coefficient: 8 dwords
// [mid0 mid1 hi0 hi1 lo 0 0 0], each dword packing 4 byte entries:
//   mid0/mid1: c*(v<<2), v = 0..3 / 4..7;  hi0/hi1: c*(v<<5);  lo: c*v, v<4.
__host__ __device__ __forceinline__ uint32_t table_dword(const uint8_t* lg, const uint8_t* ex,
                                                         uint32_t c, uint32_t q) {
  uint32_t r = 0;
  for (uint32_t e = 0; e < 4; ++e) {
    uint32_t x;
    switch (q) {
      case 0: x = e << 2; break;
      case 1: x = (e + 4) << 2; break;
      case 2: x = e << 5; break;
      case 3: x = (e + 4) << 5; break;
      case 4: x = e; break;
      default: return 0;
    }
    r |= gf_mul_t(lg, ex, c, x) << (8 * e);
  }
  return r;
}

// Host: table image (R x kpad coefficients, 8 dwords each) of an r x kin
// coefficient matrix; rows >= r and columns >= kin are zero coefficients.
void table_image_host(const uint8_t* coef, uint32_t r, uint32_t kin, uint32_t R, uint32_t kpad,
                      uint32_t* out) {
  for (uint32_t i = 0; i < R; ++i)
    for (uint32_t j = 0; j < kpad; ++j) {
      const uint32_t c = (i < r && j < kin) ? coef[i * kin + j] : 0u;
      for (uint32_t q = 0; q < 8; ++q)
        out[(i * kpad + j) * 8 + q] = table_dword(kGfHost.log, kGfHost.exp, c, q);
    }
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ uint4 ld16(const uint8_t* p) {
  const u32x4* q = reinterpret_cast<const u32x4*>(p);
  u32x4 v;
  if constexpr (NT) v = __builtin_nontemporal_load(q);
  else v = *q;
  return make_uint4(v.x, v.y, v.z, v.w);
}
template <bool NT>
__device__ __forceinline__ void st16(uint8_t* p, uint4 v) {
  u32x4* q = reinterpret_cast<u32x4*>(p);
  const u32x4 w = {v.x, v.y, v.z, v.w};
  if constexpr (NT) __builtin_nontemporal_store(w, q);
  else *q = w;
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Field selectors of 4 data bytes (shared by every output row).
struct Sel {
  uint32_t lo, mid, hi;
};
__device__ __forceinline__ Sel make_sel(uint32_t x) {
  Sel s;
  s.lo = x & 0x03030303u;
  s.mid = (x >> 2) & 0x07070707u;
  s.hi = (x >> 5) & 0x07070707u;
  return s;
}

struct Tab {
  uint32_t lo, m0, m1, h0, h1;
};
// The LDS tables of one set: interleaved 8-dword images (q + 8s; encode) or
// split q / lo regions (q + 4s, l + s; rebuild, see put_image).
template <bool SOA>
struct TabRef {
  const uint32_t* q;
  const uint32_t* l;
};
template <bool SOA>
__device__ __forceinline__ Tab read_tab(const TabRef<SOA>& t, uint32_t s) {
  if constexpr (SOA) {
    const uint4 q = *reinterpret_cast<const uint4*>(t.q + 4 * s);
    return Tab{t.l[s], q.x, q.y, q.z, q.w};
  } else {
    const uint32_t* tp = t.q + 8 * s;
    const uint4 q = *reinterpret_cast<const uint4*>(tp);
    return Tab{tp[4], q.x, q.y, q.z, q.w};
  }
}
__device__ __forceinline__ void lookups(const Sel& s, const Tab& t, uint32_t& pl, uint32_t& pm,
                                        uint32_t& ph) {
  pl = __builtin_amdgcn_perm(t.lo, t.lo, s.lo);
  pm = __builtin_amdgcn_perm(t.m1, t.m0, s.mid);
  ph = __builtin_amdgcn_perm(t.h1, t.h0, s.hi);
}

// acc[i] ^= coef(i, j0 + g) * d[g] for the KC shards of one chunk.  Shards
// are taken in pairs so that 6 partial products + the accumulator fold with
// three 3-input XORs.  Branch-free: padded rows/shards have all-zero tables.
template <int KC, int R, bool SOA>
__device__ __forceinline__ void mac_chunk(uint32_t (&acc)[R][4], const uint4 (&d)[KC],
                                          const TabRef<SOA>& tab, uint32_t kpad, uint32_t j0) {
  // Pairing costs 12 selector VGPRs (the k = 16 bodies: 3 waves per SIMD
  // instead of 4) and still wins (profiles/r02_w16_occupancy_ab.jsonl).
#pragma unroll
  for (int g = 0; g < KC; g += 2) {
    const bool two = g + 1 < KC;
    Sel sa[4], sb[4];
    sa[0] = make_sel(d[g].x);
    sa[1] = make_sel(d[g].y);
    sa[2] = make_sel(d[g].z);
    sa[3] = make_sel(d[g].w);
    if (two) {
      sb[0] = make_sel(d[g + 1].x);
      sb[1] = make_sel(d[g + 1].y);
      sb[2] = make_sel(d[g + 1].z);
      sb[3] = make_sel(d[g + 1].w);
    }
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const uint32_t sl = i * kpad + j0 + g;
      const Tab ta = read_tab(tab, sl);
      if (two) {
        const Tab tb = read_tab(tab, sl + 1);
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          uint32_t al, am, ah, bl, bm, bh;
          lookups(sa[w], ta, al, am, ah);
          lookups(sb[w], tb, bl, bm, bh);
          const uint32_t x = xor3(acc[i][w], al, am);
          const uint32_t y = xor3(ah, bl, bm);
          acc[i][w] = xor3(x, y, bh);
        }
      } else {
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          uint32_t al, am, ah;
          lookups(sa[w], ta, al, am, ah);
          acc[i][w] = xor3(acc[i][w], al, am) ^ ah;
        }
      }
    }
  }
}

// Block/column of this lane in tile `tile` of segment `sg`.
struct Unit {
  uint64_t b_first;  // first block of the tile (table set 0)
  uint32_t nsets;    // blocks touched by the tile
  uint32_t set;      // this lane's block - b_first
  bool valid;
  const uint8_t* pin;
  uint8_t* pout;
  __device__ __forceinline__ const uint8_t* in(const MacSeg& sg, uint32_t j) const {
    return pin + (uint64_t)j * sg.in_sstride;
  }
  __device__ __forceinline__ uint8_t* out(const MacSeg& sg, uint32_t i) const {
    return pout + (uint64_t)i * sg.out_sstride;
  }
};

__device__ __forceinline__ Unit locate(const MacSeg& sg, uint64_t tile) {
  Unit u;
  const uint32_t tid = threadIdx.x;
  const uint32_t C = sg.chunks;
  uint64_t c0;
  uint64_t b_last;
  if (sg.flat) {
    // units numbered across blocks: u = b*C + c; uniform part in scalars
    const uint64_t total = sg.n * (uint64_t)C;
    const uint64_t u0 = tile * 256ull;
    uint64_t u1 = u0 + 255;
    if (u1 >= total) u1 = total - 1;
    u.b_first = u0 / C;
    b_last = u1 / C;
    c0 = u0 - u.b_first * C;
  } else {
    // a tile lies inside one block
    u.b_first = b_last = tile / sg.tiles_per_block;
    c0 = (tile - u.b_first * sg.tiles_per_block) * 256ull;
  }
  u.nsets = (uint32_t)(b_last - u.b_first) + 1;
  uint32_t cc = (uint32_t)c0 + tid;  // < C + 256
  uint32_t bo = 0;
  if (sg.flat) {
    bo = cc / C;
    cc -= bo * C;
    u.valid = bo < u.nsets;
  } else {
    u.valid = cc < C;
  }
  if (!u.valid) {  // clamp to a real column; nothing is stored
    bo = 0;
    cc = (uint32_t)c0 < C ? (uint32_t)c0 : C - 1;
  }
  u.set = bo;
  const uint64_t b = u.b_first + bo;
  u.pin = sg.in + b * sg.in_bstride + (uint64_t)cc * 16;
  u.pout = sg.out + b * sg.out_bstride + (uint64_t)cc * 16;
  return u;
}

// Copy nsets table images (set s = block b_first + s) into LDS.
__device__ __forceinline__ void stage_tables(const MacSeg& sg, const Unit& u, uint32_t set_dw,
                                             uint32_t* s_tab) {
  // shared image (tab_bstride == 0): one set serves every block
  const uint32_t total = (sg.tab_bstride ? u.nsets : 1u) * set_dw;
  const uint32_t* src = sg.tab + (sg.tab_bstride ? u.b_first * sg.tab_bstride : 0);
  for (uint32_t t = threadIdx.x; t < total; t += 256) s_tab[t] = src[t];
}

// Register-staged table copy for the hot path: up to MAC_TAB_REGS dwords
// per lane (R*kpad*8*nsets <= 256*MAC_TAB_REGS), the rest copied directly.
__device__ __forceinline__ void load_tables(const MacSeg& sg, const Unit& u, uint32_t set_dw,
                                            uint32_t (&tv)[MAC_TAB_REGS]) {
  const uint32_t total = (sg.tab_bstride ? u.nsets : 1u) * set_dw;
  const uint32_t* src = sg.tab + (sg.tab_bstride ? u.b_first * sg.tab_bstride : 0);
#pragma unroll
  for (int q = 0; q < MAC_TAB_REGS; ++q) {
    const uint32_t t = threadIdx.x + 256u * q;
    tv[q] = t < total ? src[t] : 0u;
  }
}
__device__ __forceinline__ void store_tables(const MacSeg& sg, const Unit& u, uint32_t set_dw,
                                             const uint32_t (&tv)[MAC_TAB_REGS],
                                             uint32_t* s_tab) {
  const uint32_t total = (sg.tab_bstride ? u.nsets : 1u) * set_dw;
  const uint32_t* src = sg.tab + (sg.tab_bstride ? u.b_first * sg.tab_bstride : 0);
#pragma unroll
  for (int q = 0; q < MAC_TAB_REGS; ++q) {
    const uint32_t t = threadIdx.x + 256u * q;
    if (t < total) s_tab[t] = tv[q];
  }
  for (uint32_t t = threadIdx.x + 256u * MAC_TAB_REGS; t < total; t += 256) s_tab[t] = src[t];
}

// Segment of workgroup blockIdx.x and its tile (XCD-aware order); false for
// the alignment padding past a segment's tiles.
__device__ __forceinline__ bool seg_tile(const MacLaunch& L, uint32_t& sid, uint64_t& tile) {
  const uint32_t wg = blockIdx.x;
  sid = 0;
  for (uint32_t s = 1; s < L.nseg; ++s)
    if (wg >= L.seg[s].wg_begin) sid = s;
  const MacSeg& sg = L.seg[sid];
  // Segments start on a multiple of 8 (launch_plans); workgroups past a
  // segment's tiles are alignment padding.
  const uint32_t lw = wg - sg.wg_begin;
  if (lw >= sg.tiles) return false;
  tile = lw;
  if (L.xcd) {
    // XCD-aware order: the hardware deals workgroups round-robin over the 8
    // XCDs, so give XCD x a contiguous range of each segment's tiles
    // (bijective for any size): neighbouring tiles, which share the 128-byte
    // lines at their edges when S is not a multiple of 128, then meet in the
    // same L2, and every XCD gets 1/8 of every segment.  Speed only.
    const uint32_t st = (uint32_t)sg.tiles, sq = st / 8, sr = st % 8, sx = lw % 8;
    tile = sx * sq + (sx < sr ? sx : sr) + lw / 8;
  }
  return true;
}

// ---- Rebuild tables built in LDS from per-block decode coefficients.
// Layout: the images of a tile's table sets are split into a
// q region (mid0 mid1 hi0 hi1: 16 B per slot) and a lo region (4 B per
// slot), each set followed by one pad slot.  Consecutive slots' image stores
// are then bank-conflict-free (16-B / 4-B strides), and the 2-4 sets one
// wave reads (one per block its 64 columns touch) fall in distinct banks.
// The interleaved 32-B image of the encode tables cost the 4 KiB RS(16,4)
// rebuild 2/3 of its LDS cycles in bank conflicts (SQ_LDS_BANK_CONFLICT,
// DESIGN.md 4.1).  Slot x of the padded numbering (x = ci + set): q at
// s_tab + 4x, lo at s_tab + lo_dw + x.
__device__ __forceinline__ uint32_t gf_xtime(uint32_t x) { return (x << 1) ^ ((x >> 7) * 0x11Du); }
__device__ __forceinline__ uint32_t pack4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return a | (b << 8) | (c << 16) | (d << 24);
}
// Product-table image of coefficient c (the layout of table_dword), from its
// doublings d_i = c * 2^i: lo = c*{0,1,2,3}, mid = c*{0..7}<<2,
// hi = c*{0..7}<<5.
__device__ __forceinline__ void coef_image(uint32_t c, uint4& q, uint32_t& lo) {
  const uint32_t d0 = c, d1 = gf_xtime(d0), d2 = gf_xtime(d1), d3 = gf_xtime(d2);
  const uint32_t d4 = gf_xtime(d3), d5 = gf_xtime(d4), d6 = gf_xtime(d5), d7 = gf_xtime(d6);
  q = make_uint4(pack4(0, d2, d3, d2 ^ d3), pack4(d4, d4 ^ d2, d4 ^ d3, d4 ^ d3 ^ d2),
                 pack4(0, d5, d6, d5 ^ d6), pack4(d7, d7 ^ d5, d7 ^ d6, d7 ^ d6 ^ d5));
  lo = pack4(0, d0, d1, d0 ^ d1);
}
// Four images at once (byte a of c4 = coefficient a): the doublings run on 4
// bytes per dword and v_perm transposes them into per-coefficient dwords,
// about half the VALU work of four coef_image calls.
__device__ __forceinline__ uint32_t gf_xtime4(uint32_t x) {
  // the reduction byte (0x1d where a byte's top bit was set) by one
  // v_perm_b32 over {0x00, 0x1d} instead of a quarter-rate v_mul_lo_u32
  const uint32_t r = __builtin_amdgcn_perm(0u, 0x1d00u, (x >> 7) & 0x01010101u);
  return ((x & 0x7f7f7f7fu) << 1) ^ r;
}
// Coefficient a's [0, A_a, B_a, A_a ^ B_a] for packed A, B; one v_perm
// interleaves two coefficients: u = [A_a, B_a, A_a+1, B_a+1].
__device__ __forceinline__ void pair_dwords(uint32_t A, uint32_t B, uint32_t (&q)[4]) {
  const uint32_t u01 = __builtin_amdgcn_perm(B, A, 0x05010400u);
  const uint32_t u23 = __builtin_amdgcn_perm(B, A, 0x07030602u);
  const uint32_t y01 = u01 ^ (u01 >> 8), y23 = u23 ^ (u23 >> 8);
  q[0] = __builtin_amdgcn_perm(y01, u01, 0x0401000cu);
  q[1] = __builtin_amdgcn_perm(y01, u01, 0x0603020cu);
  q[2] = __builtin_amdgcn_perm(y23, u23, 0x0401000cu);
  q[3] = __builtin_amdgcn_perm(y23, u23, 0x0603020cu);
}
__device__ __forceinline__ uint32_t bcast_byte(uint32_t x, uint32_t a) {
  return __builtin_amdgcn_perm(x, x, a * 0x01010101u);
}
__device__ __forceinline__ void coef_image4(uint32_t c4, uint4 (&q)[4], uint32_t (&lo)[4]) {
  const uint32_t d0 = c4, d1 = gf_xtime4(d0), d2 = gf_xtime4(d1), d3 = gf_xtime4(d2);
  const uint32_t d4 = gf_xtime4(d3), d5 = gf_xtime4(d4), d6 = gf_xtime4(d5), d7 = gf_xtime4(d6);
  uint32_t mid[4], hi[4];
  pair_dwords(d2, d3, mid);
  pair_dwords(d5, d6, hi);
  pair_dwords(d0, d1, lo);
#pragma unroll
  for (uint32_t a = 0; a < 4; ++a)
    q[a] = make_uint4(mid[a], mid[a] ^ bcast_byte(d4, a), hi[a], hi[a] ^ bcast_byte(d7, a));
}

// Store the image of slot ci (per = R * kpad slots per set).
__device__ __forceinline__ void put_image(uint32_t* s_tab, const MacSeg& sg, uint32_t per,
                                          uint32_t ci, const uint4& q, uint32_t lo) {
  const uint32_t x = ci + ci / per;  // one pad slot per set
  *reinterpret_cast<uint4*>(s_tab + 4 * x) = q;
  s_tab[sg.lo_dw + x] = lo;
}

// Coefficient of table-image slot ci (set, row i, column j; kpad columns per
// row, R rows per set): rows[b_first + set][i][j] for i < coef_rows, j < kin,
// else 0 (padding).  coef_dense: the rows are exactly R x kpad, so slot ci is
// byte ci of the tile's range.
template <int R>
__device__ __forceinline__ uint32_t coef_at(const MacSeg& sg, const Unit& u, uint32_t ci,
                                            uint32_t kpad) {
  if (sg.coef_dense) return sg.coef[u.b_first * sg.coef_bstride + ci];
  const uint32_t set = ci / (R * kpad), rem = ci - set * (R * kpad);
  const uint32_t i = rem / kpad, j = rem - i * kpad;
  if (i >= sg.coef_rows || j >= sg.kin) return 0u;
  return sg.coef[(u.b_first + set) * sg.coef_bstride + i * sg.kin + j];
}

// Table sets a tile builds: one per block, or one for all when the
// coefficients are shared (coef_bstride 0: encode's parity rows).
__device__ __forceinline__ uint32_t coef_sets(const MacSeg& sg, const Unit& u) {
  return sg.coef_bstride ? u.nsets : 1u;
}

// Register-staged coefficient loads for the hot path (issued before the
// shard loads; vmcnt retires in order), then the images into LDS.  Lane t
// owns slots t + 256q, so each image store instruction covers consecutive
// slots.  The loads are unconditional, at a clamped (dense rows) or dummy
// (padding slot) offset: a load under a divergent branch whose other side
// writes the same register makes the compiler wait for it right there
// (vmcnt(0)), which serialised these loads, one memory latency each, in
// front of the shard loads.  Padding slots are zeroed in store_images,
// after the shard loads are out.
template <int R, int KP>
__device__ __forceinline__ bool coef_slot_ok(const MacSeg& sg, uint32_t ci, uint32_t total) {
  if (sg.coef_dense) return ci < total;
  const uint32_t rem = ci % (R * KP), i = rem / KP, j = rem - i * KP;
  return ci < total && i < sg.coef_rows && j < sg.kin;
}
template <int R, int KP>
__device__ __forceinline__ void load_coefs(const MacSeg& sg, const Unit& u,
                                           uint32_t (&cv)[MAC_COEF_REGS]) {
  const uint32_t total = coef_sets(sg, u) * (R * KP);
  const uint32_t tid = threadIdx.x;
  if (sg.coef_dense) {  // uniform: the tile's rows are one contiguous range
    const uint8_t* base = sg.coef + u.b_first * sg.coef_bstride;
#pragma unroll
    for (int q = 0; q < MAC_COEF_REGS; ++q) {
      const uint32_t ci = tid + 256u * q;
      cv[q] = base[ci < total ? ci : total - 1u];
    }
  } else {
#pragma unroll
    for (int q = 0; q < MAC_COEF_REGS; ++q) {
      const uint32_t ci = tid + 256u * q;
      const uint32_t set = ci / (R * KP), rem = ci - set * (R * KP);
      const uint32_t i = rem / KP, j = rem - i * KP;
      const uint64_t off = coef_slot_ok<R, KP>(sg, ci, total)
                               ? (u.b_first + set) * sg.coef_bstride + i * sg.kin + j
                               : 0u;
      cv[q] = sg.coef[off];
    }
  }
}
template <int R, int KP>
__device__ __forceinline__ void store_images(const MacSeg& sg, const Unit& u,
                                             const uint32_t (&cv0)[MAC_COEF_REGS], uint32_t* s_tab) {
  const uint32_t total = coef_sets(sg, u) * (R * KP);
  const uint32_t t = threadIdx.x;
  uint32_t cv[MAC_COEF_REGS];
#pragma unroll
  for (int q = 0; q < MAC_COEF_REGS; ++q)
    cv[q] = coef_slot_ok<R, KP>(sg, t + 256u * q, total) ? cv0[q] : 0u;
  static_assert(MAC_COEF_REGS == 6, "two packed groups: slots t + 256 * (0..3), (4..5)");
  if (t < total) {  // waves past the tile's slots skip the build
    uint4 q[4];
    uint32_t lo[4];
    coef_image4(pack4(cv[0], cv[1], cv[2], cv[3]), q, lo);
#pragma unroll
    for (uint32_t a = 0; a < 4; ++a)
      if (t + 256u * a < total) put_image(s_tab, sg, R * KP, t + 256u * a, q[a], lo[a]);
  }
  if (t + 1024u < total) {
    uint4 q[4];
    uint32_t lo[4];
    coef_image4(pack4(cv[4], cv[5], 0, 0), q, lo);
#pragma unroll
    for (uint32_t a = 0; a < 2; ++a)
      if (t + 256u * (4 + a) < total) put_image(s_tab, sg, R * KP, t + 256u * (4 + a), q[a], lo[a]);
  }
}

// Unstaged variant (generic chunk loop, runtime kpad).
template <int R>
__device__ __forceinline__ void stage_images(const MacSeg& sg, const Unit& u, uint32_t* s_tab) {
  const uint32_t per = R * sg.kpad;
  const uint32_t total = coef_sets(sg, u) * per;
  for (uint32_t ci = threadIdx.x; ci < total; ci += 256) {
    uint4 q;
    uint32_t lo;
    coef_image(coef_at<R>(sg, u, ci, sg.kpad), q, lo);
    put_image(s_tab, sg, per, ci, q, lo);
  }
}

// x mod 255 for x < 2^16 (sums of GF logs).
__device__ __forceinline__ uint32_t mod255(uint32_t x) {
  x = (x & 0xFFu) + (x >> 8);
  x = (x & 0xFFu) + (x >> 8);
  return x >= 255u ? x - 255u : x;
}

// ---- Fused rebuild: a tile derives its blocks' decode rows itself.
// The closed form of decode_coef_kernel (below) per tile, in LDS, while the
// tile's shard loads are in flight: the survivor and lost indices of the
// tile's blocks (contiguous ranges of surv_idx / lost_idx) and the GF tables
// are loaded ahead of the shard loads (vmcnt retires in order), then
//   (a) indices, GF log/antilog and LW0 into LDS, survivor masks zeroed;
//   (b) survivor bit set per block by LDS atomic OR (duplicates and
//       out-of-range indices mark the block faulty);
//   (c) log W_t per (block, survivor) and log Lam_l per (block, lost shard),
//       each a sum over the block's m non-survivors (set bits of the mask
//       complement);
//   (d) the coefficients row_l[t] = W_t Lam_l / (l ^ s_t) of the tile's
//       table slots, then their product-table images, as the two-kernel
//       rebuild builds them from rows read back from HBM.
// No decode rows travel through HBM and no second kernel runs: the step is
// one launch (gf_rebuild_kernel).
struct DecWs {
  uint8_t* lg;     // log[256] exp[768] (the kGf image)
  uint8_t* ex;
  uint8_t* lw0;    // LW0(i), i < k + m
  uint32_t* mask;  // per block: survivor bits 0..95 in 3 words, word 3 = fault
  uint8_t* sv;     // ns x k survivor indices
  uint8_t* lv;     // ns x e lost indices
  uint8_t* lw;     // ns x k log W_t
  uint8_t* llam;   // ns x e log Lam_l (mod 255), DEC_UNIT when l survived
};
constexpr uint32_t DEC_UNIT = 0xFFu;

__device__ __forceinline__ DecWs dec_ws(uint32_t* base, uint32_t ns, uint32_t k, uint32_t e) {
  DecWs w;
  uint8_t* p = reinterpret_cast<uint8_t*>(base);
  w.lg = p;
  w.ex = p + 256;
  w.lw0 = p + 1024;
  w.mask = reinterpret_cast<uint32_t*>(p + 1152);
  p += 1152 + 16 * ns;
  w.sv = p;
  p += dec_r4(ns * k);
  w.lv = p;
  p += dec_r4(ns * e);
  w.lw = p;
  p += dec_r4(ns * k);
  w.llam = p;
  return w;
}

// Registers staged ahead of the shard loads: index bytes z = tid + 256q of
// the tile's [survivors ns*k | lost ns*e] range, one GF-table dword, one LW0
// dword.
struct DecRegs {
  uint32_t v[DEC_IDX_REGS];
  uint32_t gf, lw0;
};
__device__ __forceinline__ uint32_t dec_idx_byte(const MacSeg& sg, const Unit& u, uint32_t z,
                                                 uint32_t nk) {
  return z < nk ? sg.sidx[u.b_first * sg.kin + z] : sg.lidx[u.b_first * sg.r + (z - nk)];
}
__device__ __forceinline__ void dec_load(const MacSeg& sg, const Unit& u, DecRegs& x) {
  const uint32_t tid = threadIdx.x;
  const uint32_t nk = u.nsets * sg.kin, total = nk + u.nsets * sg.r;
#pragma unroll
  for (int q = 0; q < DEC_IDX_REGS; ++q) {
    const uint32_t z = tid + 256u * q;
    x.v[q] = z < total ? dec_idx_byte(sg, u, z, nk) : 0u;
  }
  x.gf = reinterpret_cast<const uint32_t*>(&kGf)[tid];  // 256 dwords: log + exp
  x.lw0 = tid < 32 ? sg.lw0[tid] : 0u;
}

__device__ __forceinline__ void dec_phase_a(const MacSeg& sg, const Unit& u, const DecWs& w,
                                            const DecRegs& x) {
  const uint32_t tid = threadIdx.x;
  const uint32_t nk = u.nsets * sg.kin, total = nk + u.nsets * sg.r;
  reinterpret_cast<uint32_t*>(w.lg)[tid] = x.gf;
  if (tid < 32) reinterpret_cast<uint32_t*>(w.lw0)[tid] = x.lw0;
  for (uint32_t t = tid; t < 4 * u.nsets; t += 256) w.mask[t] = 0u;
#pragma unroll
  for (int q = 0; q < DEC_IDX_REGS; ++q) {
    const uint32_t z = tid + 256u * q;
    if (z < total) (z < nk ? w.sv[z] : w.lv[z - nk]) = (uint8_t)x.v[q];
  }
  for (uint32_t z = tid + 256u * DEC_IDX_REGS; z < total; z += 256)
    (z < nk ? w.sv[z] : w.lv[z - nk]) = (uint8_t)dec_idx_byte(sg, u, z, nk);
}

// (b) survivor masks; k is the compile-time chunk on the hot path.
__device__ __forceinline__ void dec_phase_b(const Unit& u, const DecWs& w, uint32_t k,
                                            uint32_t nt) {
  for (uint32_t x = threadIdx.x; x < u.nsets * k; x += 256) {
    const uint32_t set = x / k, s = w.sv[x];
    uint32_t* mk = w.mask + 4 * set;
    if (s >= nt) {
      atomicOr(mk + 3, 1u);
    } else {
      const uint32_t bit = 1u << (s & 31);
      if (atomicOr(mk + (s >> 5), bit) & bit) atomicOr(mk + 3, 1u);  // duplicate
    }
  }
}

// Sum of log(v ^ c) over the block's non-survivors c (set bits of the
// complement of its mask inside [0, nt)): m lookups for a valid block.
__device__ __forceinline__ uint32_t dec_comp_sum(const DecWs& w, const uint32_t* mk, uint32_t v,
                                                 uint32_t nt) {
  uint32_t acc = 0;
#pragma unroll
  for (uint32_t q = 0; q < 3; ++q) {
    const uint32_t lo = 32u * q;
    uint32_t valid = nt <= lo ? 0u : (nt - lo >= 32u ? ~0u : (1u << (nt - lo)) - 1u);
    uint32_t c = ~mk[q] & valid;
    while (c) {
      const uint32_t b = __builtin_ctz(c);
      c &= c - 1;
      acc += w.lg[v ^ (lo + b)];
    }
  }
  return acc;
}

// (c) log W_t per survivor slot, log Lam_l per lost slot.
template <int R>
__device__ __forceinline__ void dec_phase_c(const Unit& u, const DecWs& w, uint32_t k, uint32_t e,
                                            uint32_t nt) {
  const uint32_t tid = threadIdx.x;
  for (uint32_t x = tid; x < u.nsets * k; x += 256) {
    const uint32_t set = x / k;
    const uint32_t* mk = w.mask + 4 * set;
    if (mk[3]) continue;  // faulty block: its coefficients are zero
    const uint32_t s = w.sv[x];
    w.lw[x] = (uint8_t)mod255(w.lw0[s] + dec_comp_sum(w, mk, s, nt));
  }
  for (uint32_t y = tid; y < u.nsets * R; y += 256) {
    const uint32_t set = y / R, i = y - set * R;
    if (i >= e) continue;
    uint32_t* mk = w.mask + 4 * set;
    const uint32_t l = w.lv[set * e + i];
    if (l >= nt) {
      atomicOr(mk + 3, 1u);
      continue;
    }
    const bool surv = (mk[l >> 5] >> (l & 31)) & 1u;
    // log Lam_l = -(LW0(l) + sum_c log(l ^ c)); c == l adds log[0] = 0
    w.llam[set * e + i] =
        (uint8_t)(surv ? DEC_UNIT : mod255(255u - mod255(w.lw0[l] + dec_comp_sum(w, mk, l, nt))));
  }
}

// (d) coefficient of table slot ci = (set, row i, column j), kp columns per
// row, R rows per set.  Faulty blocks report through the status word.
template <int R>
__device__ __forceinline__ uint32_t dec_coef(const Unit& u, const DecWs& w, uint32_t ci,
                                             uint32_t kp, uint32_t k, uint32_t e) {
  const uint32_t per = R * kp;
  const uint32_t set = ci / per, rem = ci - set * per;
  const uint32_t i = rem / kp, j = rem - i * kp;
  if (set >= u.nsets || i >= e || j >= k || w.mask[4 * set + 3]) return 0u;
  const uint32_t l = w.lv[set * e + i], s = w.sv[set * k + j], ll = w.llam[set * e + i];
  if (ll == DEC_UNIT) return s == l ? 1u : 0u;
  return w.ex[w.lw[set * k + j] + ll + 255u - w.lg[l ^ s]];  // < 765
}
__device__ __forceinline__ void dec_report(const MacSeg& sg, const Unit& u, const DecWs& w) {
  for (uint32_t set = threadIdx.x; set < u.nsets; set += 256)
    if (w.mask[4 * set + 3] && sg.status) *sg.status = 1u;  // plain store: every writer stores 1
}

// ---- Fused rebuild, hot path (kin == KC): wave-local decode.
// Each of the tile's blocks is decoded by a group of L lanes (L = the power
// of two >= KC) inside one wave, so no workgroup barrier separates the
// decode steps: lane t holds survivor s_t and lost index l_t; the block's
// survivor bit set is OR-reduced across the group with __shfl_xor; lane t
// forms log W_t and log Lam_{l_t} from the m non-survivors; the l_r and
// log Lam_r are broadcast in the group, and lane t builds column t of the
// block's R product-table rows straight into the tile's LDS tables.  Each
// wave has its own copy of the GF log/antilog tables and LW0 (1152 bytes),
// so the tile's only barrier is the one before the MAC, as in encode.
template <int KC>
constexpr int dec_lanes() {
  return KC <= 4 ? 4 : KC <= 8 ? 8 : 16;
}
template <int KC, int R>
constexpr bool dec_wave_ok() {
  return R <= dec_lanes<KC>();  // lost index r lives in lane r of the group
}
// The first DEC_PASSES passes (sets g, g + G) have their indices loaded
// ahead of the shard loads; later passes (tiles of > 2G blocks) load theirs
// when they run.
constexpr int DEC_PASSES = 2;

struct DecWaveRegs {
  uint32_t sv[DEC_PASSES], lv[DEC_PASSES];
  uint32_t gf[4], lw0;
};

template <int KC>
__device__ __forceinline__ void dec_wave_idx(const MacSeg& sg, const Unit& u, uint32_t set,
                                             uint32_t t, uint32_t& sv, uint32_t& lv) {
  const bool live = set < u.nsets;
  const uint64_t b = u.b_first + set;
  sv = (live && t < (uint32_t)KC) ? sg.sidx[b * KC + t] : 0u;
  lv = (live && t < sg.r) ? sg.lidx[b * sg.r + t] : 0u;
}

template <int KC>
__device__ __forceinline__ void dec_wave_load(const MacSeg& sg, const Unit& u, DecWaveRegs& x) {
  constexpr uint32_t L = dec_lanes<KC>(), G = 256 / L;
  const uint32_t tid = threadIdx.x, t = tid % L, g = tid / L;
#pragma unroll
  for (int p = 0; p < DEC_PASSES; ++p) dec_wave_idx<KC>(sg, u, g + G * p, t, x.sv[p], x.lv[p]);
  const uint32_t lane = tid % 64;
  const uint32_t* gf = reinterpret_cast<const uint32_t*>(&kGf);
#pragma unroll
  for (int q = 0; q < 4; ++q) x.gf[q] = gf[lane + 64 * q];
  x.lw0 = lane < 32 ? sg.lw0[lane] : 0u;
}

// One block (set) decoded by its L-lane group; column t of its rows built
// into the set's table images.  sv / lv: this lane's survivor / lost index.
template <int KC, int R>
__device__ __forceinline__ void dec_wave_set(const MacSeg& sg, const Unit& u, uint32_t set,
                                             uint32_t sv, uint32_t lv, const uint8_t* lg,
                                             const uint8_t* ex, const uint8_t* lw0,
                                             uint32_t* s_tab) {
  constexpr uint32_t L = dec_lanes<KC>();
  const uint32_t t = threadIdx.x % L;
  const uint32_t nt = KC + sg.m, e = sg.r;
  const bool col = t < (uint32_t)KC, lost = t < e;
  // survivor bit set (3 words: nt <= 80) and the faults, over the group
  bool bad = (col && sv >= nt) || (lost && lv >= nt);
  uint32_t mk0 = 0, mk1 = 0, mk2 = 0;
  if (col && sv < nt) {
    const uint32_t w = sv >> 5, bit = 1u << (sv & 31);
    mk0 = w == 0 ? bit : 0u;
    mk1 = w == 1 ? bit : 0u;
    mk2 = w == 2 ? bit : 0u;
  }
  uint32_t badw = bad ? 1u : 0u;
#pragma unroll
  for (uint32_t off = 1; off < L; off <<= 1) {
    mk0 |= __shfl_xor(mk0, off, L);
    mk1 |= __shfl_xor(mk1, off, L);
    mk2 |= __shfl_xor(mk2, off, L);
    badw |= __shfl_xor(badw, off, L);
  }
  // out of range anywhere, or duplicate survivors (fewer than k distinct)
  bad = badw != 0 || (uint32_t)(__popc(mk0) + __popc(mk1) + __popc(mk2)) != (uint32_t)KC;
  const uint32_t mk[3] = {mk0, mk1, mk2};
  auto comp_sum = [&](uint32_t v) {  // sum of log(v ^ c) over the non-survivors c
    uint32_t acc = 0;
#pragma unroll
    for (uint32_t q = 0; q < 3; ++q) {
      const uint32_t lo = 32u * q;
      const uint32_t valid = nt <= lo ? 0u : (nt - lo >= 32u ? ~0u : (1u << (nt - lo)) - 1u);
      uint32_t c = ~mk[q] & valid;
      while (c) {
        const uint32_t b = __builtin_ctz(c);
        c &= c - 1;
        acc += lg[v ^ (lo + b)];
      }
    }
    return acc;
  };
  uint32_t lw = 0, llam = 0;  // log W_t; log Lam_{l_t} (DEC_UNIT: l_t survived)
  if (!bad) {
    if (col) lw = mod255(lw0[sv] + comp_sum(sv));
    if (lost) {
      const bool surv = (mk[lv >> 5] >> (lv & 31)) & 1u;
      llam = surv ? DEC_UNIT : mod255(255u - mod255(lw0[lv] + comp_sum(lv)));
    }
  }
  // coefficients row_r[t] for r < e (rows >= e and columns >= k are zero)
  uint32_t cf[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t l = __shfl(lv, r, L), ll = __shfl(llam, r, L);
    uint32_t c = 0;
    if (!bad && col && (uint32_t)r < e)
      c = ll == DEC_UNIT ? (sv == l ? 1u : 0u) : ex[lw + ll + 255u - lg[l ^ sv]];  // < 765
    cf[r] = c;
  }
  if (bad && t == 0 && sg.status) *sg.status = 1u;  // plain store: every writer stores 1
  if (!col) return;  // lanes past KC: no column (kpad == KC on the hot path)
  constexpr uint32_t per = R * KC;
  const uint32_t base = set * per + t;  // slot of (set, row 0, column t)
#pragma unroll
  for (int r0 = 0; r0 < R; r0 += 4) {
    uint4 q[4];
    uint32_t lo[4];
    coef_image4(pack4(cf[r0], r0 + 1 < R ? cf[r0 + 1] : 0u, r0 + 2 < R ? cf[r0 + 2] : 0u,
                      r0 + 3 < R ? cf[r0 + 3] : 0u),
                q, lo);
#pragma unroll
    for (int a = 0; a < 4; ++a)
      if (r0 + a < R) put_image(s_tab, sg, per, base + (uint32_t)(r0 + a) * KC, q[a], lo[a]);
  }
}

template <int KC, int R>
__device__ __forceinline__ void dec_wave_tile(const MacSeg& sg, const Unit& u, const DecWaveRegs& x,
                                              uint32_t* s_tab) {
  constexpr uint32_t L = dec_lanes<KC>(), G = 256 / L;
  const uint32_t tid = threadIdx.x, t = tid % L, g = tid / L, lane = tid % 64;
  // this wave's GF tables + LW0 (written and read by this wave only: LDS
  // operations of one wave complete in order)
  uint32_t* wv = s_tab + sg.ws_dw + (tid / 64) * (DEC_WAVE_BYTES / 4);
#pragma unroll
  for (int q = 0; q < 4; ++q) wv[lane + 64 * q] = x.gf[q];
  if (lane < 32) wv[256 + lane] = x.lw0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint8_t* lg = reinterpret_cast<const uint8_t*>(wv);
  const uint8_t* ex = lg + 256;
  const uint8_t* lw0 = lg + 1024;
#pragma unroll
  for (int p = 0; p < DEC_PASSES; ++p) {
    const uint32_t set = g + G * p;
    if (set < u.nsets) dec_wave_set<KC, R>(sg, u, set, x.sv[p], x.lv[p], lg, ex, lw0, s_tab);
  }
  for (uint32_t set = g + G * DEC_PASSES; set < u.nsets; set += G) {
    uint32_t sv, lv;
    dec_wave_idx<KC>(sg, u, set, t, sv, lv);
    dec_wave_set<KC, R>(sg, u, set, sv, lv, lg, ex, lw0, s_tab);
  }
}

// One tile of segment sg: KC is the straight-line shard chunk (kin == KC is
// the hot path; other kin loop over chunks of KC shards).  MODE: the tables
// are copied from a precomputed image (MAC_ENCODE), built from per-block
// coefficient rows in HBM (MAC_ROWS) or from rows the tile decodes itself
// (MAC_FUSED).
template <int KC, int R, bool NT, int MODE>
__device__ __forceinline__ void mac_tile(const MacSeg& sg, uint64_t tile, uint32_t* s_tab) {
  constexpr bool COEF = MODE != MAC_ENCODE;  // tables built in LDS from coefficients
  constexpr bool FUSED = MODE == MAC_FUSED;
  const uint32_t kin = sg.kin, kpad = sg.kpad;
  const uint32_t set_dw = R * kpad * 8;

  const Unit u = locate(sg, tile);
  constexpr bool SOA = COEF;  // per-coefficient tables: split q / lo regions
  TabRef<SOA> tab;
  if constexpr (SOA) {
    const uint32_t x0 = sg.coef_bstride ? u.set * (R * kpad + 1) : 0u;  // padded slot of set
    tab.q = s_tab + 4 * x0;
    tab.l = s_tab + sg.lo_dw + x0;
  } else {
    const bool per_block = COEF ? sg.coef_bstride != 0 : sg.tab_bstride != 0;
    tab.q = s_tab + (per_block ? u.set * set_dw : 0u);
    tab.l = nullptr;
  }
  uint32_t acc[R][4];
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int w = 0; w < 4; ++w) acc[i][w] = 0;

  if constexpr (FUSED) {
    const uint32_t nt = kin + sg.m, e = sg.r;
    if (kin == KC && dec_wave_ok<KC, R>()) {
      // hot path: wave-local decode, one barrier (before the MAC)
      DecWaveRegs xw;
      dec_wave_load<KC>(sg, u, xw);  // ahead of the shard loads
      uint4 d[KC];
#pragma unroll
      for (int g = 0; g < KC; ++g) d[g] = ld16<NT>(u.in(sg, g));
      dec_wave_tile<KC, R>(sg, u, xw, s_tab);
      __syncthreads();
      mac_chunk<KC, R>(acc, d, tab, kpad, 0);
    } else if (kin == KC) {
      const DecWs ws = dec_ws(s_tab + sg.ws_dw, u.nsets, kin, e);
      DecRegs xr;
      dec_load(sg, u, xr);  // ahead of the shard loads
      uint4 d[KC];
#pragma unroll
      for (int g = 0; g < KC; ++g) d[g] = ld16<NT>(u.in(sg, g));
      dec_phase_a(sg, u, ws, xr);
      __syncthreads();
      dec_phase_b(u, ws, KC, nt);
      __syncthreads();
      dec_phase_c<R>(u, ws, KC, e, nt);
      __syncthreads();
      uint32_t cv[MAC_COEF_REGS];
#pragma unroll
      for (int q = 0; q < MAC_COEF_REGS; ++q)
        cv[q] = dec_coef<R>(u, ws, threadIdx.x + 256u * q, KC, KC, e);
      dec_report(sg, u, ws);
      store_images<R, KC>(sg, u, cv, s_tab);
      __syncthreads();
      mac_chunk<KC, R>(acc, d, tab, kpad, 0);
    } else {
      const DecWs ws = dec_ws(s_tab + sg.ws_dw, u.nsets, kin, e);
      DecRegs xr;
      dec_load(sg, u, xr);
      dec_phase_a(sg, u, ws, xr);
      __syncthreads();
      dec_phase_b(u, ws, kin, nt);
      __syncthreads();
      dec_phase_c<R>(u, ws, kin, e, nt);
      __syncthreads();
      {
        const uint32_t per = R * kpad, total = u.nsets * per;
        for (uint32_t ci = threadIdx.x; ci < total; ci += 256) {
          uint4 q;
          uint32_t lo;
          coef_image(dec_coef<R>(u, ws, ci, kpad, kin, e), q, lo);
          put_image(s_tab, sg, per, ci, q, lo);
        }
      }
      dec_report(sg, u, ws);
      __syncthreads();
      for (uint32_t j0 = 0; j0 < kin; j0 += KC) {
        uint4 d[KC];
#pragma unroll
        for (int g = 0; g < KC; ++g)
          if (j0 + g < kin) d[g] = ld16<NT>(u.in(sg, j0 + g));
        mac_chunk<KC, R>(acc, d, tab, kpad, j0);
      }
    }
#ifdef MEMO_EC_PERM_PROBE
  } else if constexpr (MODE == MAC_PERM) {
    // Probe only (tools/perm_probe.py): each block's
    // images come from a per-code table of every erasure pattern's product
    // images (q: 16 B, lo: 4 B per slot), indexed by the block's pattern
    // rank (sg.coef: one u16 per block), instead of being built from decode
    // rows.  Ranks first, the shard loads, then the image loads.
    const uint32_t per = R * KC, total = u.nsets * per, t = threadIdx.x;
    const uint16_t* prank = reinterpret_cast<const uint16_t*>(sg.coef);
    uint32_t pr[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const uint32_t ci = t + 256u * q, set = ci < total ? ci / per : 0u;
      pr[q] = prank[u.b_first + set];
    }
    uint4 d[KC];
#pragma unroll
    for (int g = 0; g < KC; ++g) d[g] = ld16<NT>(u.in(sg, g));
    const uint4* qt = reinterpret_cast<const uint4*>(sg.tab);
    const uint32_t* lt = reinterpret_cast<const uint32_t*>(sg.sidx);
    uint4 qv[6];
    uint32_t lv[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const uint32_t ci = t + 256u * q;
      const uint64_t off = (uint64_t)pr[q] * per + (ci < total ? ci % per : 0u);
      qv[q] = qt[off];
      lv[q] = lt[off];
    }
#pragma unroll
    for (int q = 0; q < 6; ++q)
      if (t + 256u * q < total) put_image(s_tab, sg, per, t + 256u * q, qv[q], lv[q]);
    __syncthreads();
    mac_chunk<KC, R>(acc, d, tab, kpad, 0);
#endif
  } else if (kin == KC) {
    // Hot path.  The table image loads go out first (vmcnt retires in issue
    // order, so the LDS copy then waits only for them), the KC shard loads
    // right behind; the barrier and table copy overlap the shard loads.
    uint32_t tv[COEF ? MAC_COEF_REGS : MAC_TAB_REGS];
    if constexpr (COEF) load_coefs<R, KC>(sg, u, tv);
    else load_tables(sg, u, set_dw, tv);
    uint4 d[KC];
#pragma unroll
    for (int g = 0; g < KC; ++g) d[g] = ld16<NT>(u.in(sg, g));
    if constexpr (COEF) store_images<R, KC>(sg, u, tv, s_tab);
    else store_tables(sg, u, set_dw, tv, s_tab);
    __syncthreads();
    mac_chunk<KC, R>(acc, d, tab, kpad, 0);
  } else {
    if constexpr (COEF) stage_images<R>(sg, u, s_tab);
    else stage_tables(sg, u, set_dw, s_tab);
    __syncthreads();
    for (uint32_t j0 = 0; j0 < kin; j0 += KC) {
      uint4 d[KC];
#pragma unroll
      for (int g = 0; g < KC; ++g)
        if (j0 + g < kin) d[g] = ld16<NT>(u.in(sg, j0 + g));
      mac_chunk<KC, R>(acc, d, tab, kpad, j0);
    }
  }

  if (u.valid) {
#pragma unroll
    for (int i = 0; i < R; ++i)
      if ((uint32_t)i < sg.r)
        st16<NT>(u.out(sg, i),
                 make_uint4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]));
  }
}

// Encode (MAC_ENCODE) and the two-kernel rebuild's MAC (MAC_ROWS).  The
// rebuild instance also takes segments with table images instead of
// coefficient rows (coef null: a shared pattern's image, or per-block images
// the decode formed), so a mixed rebuild's pieces of one shard chunk and row
// bound share one launch whichever way their tables come (the branch is
// uniform per workgroup: one segment per tile).
template <int KC, int R, bool NT, bool COEF>
__global__ void __launch_bounds__(256) gf_mac_kernel(const MacLaunch L) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_tab[];
  uint32_t sid;
  uint64_t tile;
  if (!seg_tile(L, sid, tile)) return;
  if constexpr (COEF) {
    if (L.seg[sid].coef) {
      mac_tile<KC, R, NT, MAC_ROWS>(L.seg[sid], tile, s_tab);
      return;
    }
  }
  mac_tile<KC, R, NT, MAC_ENCODE>(L.seg[sid], tile, s_tab);
}

// The two-kernel rebuild's MAC over per-block table images (the decode
// formed them in HBM): gf_mac_kernel's encode instance under its own name.
template <int KC, int R, bool NT>
__global__ void __launch_bounds__(256) gf_mac_images_kernel(const MacLaunch L) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_tab[];
  uint32_t sid;
  uint64_t tile;
  if (!seg_tile(L, sid, tile)) return;
  mac_tile<KC, R, NT, MAC_ENCODE>(L.seg[sid], tile, s_tab);
}

#ifdef MEMO_EC_PERM_PROBE
template <int KC, int R, bool NT>
__global__ void __launch_bounds__(256) gf_mac_perm_kernel(const MacLaunch L) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_tab[];
  uint32_t sid;
  uint64_t tile;
  if (!seg_tile(L, sid, tile)) return;
  mac_tile<KC, R, NT, MAC_PERM>(L.seg[sid], tile, s_tab);
}
#endif

// Rebuild in one launch: decode rows derived per tile, then the MAC.
template <int KC, int R, bool NT>
__global__ void __launch_bounds__(256) gf_rebuild_kernel(const MacLaunch L) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_tab[];
  uint32_t sid;
  uint64_t tile;
  if (!seg_tile(L, sid, tile)) return;
  mac_tile<KC, R, NT, MAC_FUSED>(L.seg[sid], tile, s_tab);
}

// The memory system's rate for the MAC's own traffic: the tiles, tile
// order, lane -> column map and non-temporal dwordx4 loads / stores of
// gf_mac_kernel, with the GF arithmetic replaced by one XOR per shard
// (output i = XOR of the block's kin inputs, each byte ^ i).  sg.probe
// picks the traffic: MEMO_EC_PROBE_COPY both, MEMO_EC_PROBE_READ the loads
// alone (the XOR kept live by a store that practically never happens),
// MEMO_EC_PROBE_WRITE the stores alone (a per-lane pattern).  bench.py's
// roofline.achievable is the read and write launches' times added: the
// rate this mix of read and write streams gets when they do not interleave
// (memo_ec_stream_probe).
template <int KC, int R, bool NT>
__global__ void __launch_bounds__(256) stream_probe_kernel(const MacLaunch L) {
  uint32_t sid;
  uint64_t tile;
  if (!seg_tile(L, sid, tile)) return;
  const MacSeg& sg = L.seg[sid];
  const Unit u = locate(sg, tile);
  uint4 a = make_uint4((uint32_t)tile, threadIdx.x, 0x9e3779b9u, 0x7f4a7c15u);
  if (sg.probe != MEMO_EC_PROBE_WRITE) {
    a = make_uint4(0, 0, 0, 0);
    for (uint32_t j0 = 0; j0 < sg.kin; j0 += KC) {
      uint4 d[KC];
#pragma unroll
      for (int g = 0; g < KC; ++g)
        d[g] = j0 + g < sg.kin ? ld16<NT>(u.in(sg, j0 + g)) : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int g = 0; g < KC; ++g) {
        a.x ^= d[g].x;
        a.y ^= d[g].y;
        a.z ^= d[g].z;
        a.w ^= d[g].w;
      }
    }
  }
  if (!u.valid) return;
  if (sg.probe == MEMO_EC_PROBE_READ) {
    if (a.x == 0x2545f491u && a.y == ~a.z && a.w == 0x6c078965u) st16<NT>(u.out(sg, 0), a);
    return;
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const uint32_t b = (uint32_t)i * 0x01010101u;
    if ((uint32_t)i < sg.r) st16<NT>(u.out(sg, i), make_uint4(a.x ^ b, a.y ^ b, a.z ^ b, a.w ^ b));
  }
}

// ---- Per-block product-table images through HBM (rows path, multi-tile
// blocks).  The column-per-lane decode (decode_coef_wide_kernel) writes, for
// each slot (block b, row i, column j), the 8-dword image of rows[b][i][j]
// (zero for the padding rows i >= e and columns j >= k) in table_dword's
// layout [mid0 mid1 hi0 hi1 lo 0 0 0], two 16-byte stores per slot.  The MAC
// then copies a block's image set like the encode's shared one instead of
// building it in LDS per tile: for a block of T tiles the build runs once
// instead of T times, at R * kpad * 32 bytes of HBM per block (RS(16,4):
// 2 KiB, 0.15% of a 1 MiB block's traffic).
__device__ __forceinline__ void put_slot_image(uint32_t* img, uint32_t slot, uint32_t c) {
  uint4 q;
  uint32_t lo;
  coef_image(c, q, lo);
  uint4* dst = reinterpret_cast<uint4*>(img + (uint64_t)slot * 8);
  dst[0] = q;
  dst[1] = make_uint4(lo, 0u, 0u, 0u);
}

// ------------------------------------------------- closed-form decode rows
// One LANE per block.  Every shard of the code is a scaled evaluation of
// one polynomial: with f(z) = sum_j D_j / (z ^ j) over the k data indices
// and F(z) = f(z) * prod_{j<k} (z ^ j) (degree < k), data shard j is
// F(j) / sigma(j) and parity shard x is f(x) = F(x) / sigma(x), where
// sigma(i) = prod_{j<k, j != i} (i ^ j) -- the Cauchy rows 1/(x ^ j) of the
// generator.  The k survivors s_t are k evaluations of F, so Lagrange
// interpolation gives every lost shard l directly:
//   row_l[t] = W_t * Lam_l / (l ^ s_t),
//   W_t   = sigma(s_t) / prod_{u != t} (s_t ^ s_u),
//   Lam_l = prod_u (l ^ s_u) / sigma(l),
// and row_l = unit vector when l is itself a survivor.  With
// Pall(i) = prod_{j < k+m, j != i} (i ^ j) the survivor products become
// products over the m non-survivors c (the complement):
//   log W_t   = LW0(s_t) + sum_c log(s_t ^ c),
//   log Lam_l = -LW0(l) - sum_{c != l} log(l ^ c),
//   LW0(i)    = log sigma(i) - log Pall(i)   (per (k, m): LDS, per workgroup).
// O(k*m + e*k) table lookups per block instead of a k x k Gauss-Jordan
// elimination (round 1's decode_rows_reg_kernel: DESIGN.md 4.2).  Checked
// against the oracle's
// Gauss-Jordan rows (tests/test_gpu_parity.py).

// The segment of a multi-segment decode launch workgroup blockIdx.x works
// on, and its workgroup index within that segment.
__device__ __forceinline__ DecodeArgs dec_seg(const DecodeLaunch& L, uint32_t& bid) {
  uint32_t sid = 0;
  for (uint32_t i = 1; i < L.nseg; ++i)
    if (blockIdx.x >= L.wg_begin[i]) sid = i;
  bid = blockIdx.x - L.wg_begin[sid];
  return L.seg[sid];
}

// LW0(i) = log sigma(i) - log Pall(i) for i < k + m, into LDS.
__device__ __forceinline__ void stage_lw0(const uint8_t* lg, uint32_t k, uint32_t nt,
                                          uint32_t* s_lw0) {
  // j == i adds log[0] = 0; the lookups are branch-free so that the unrolled
  // loop keeps several LDS reads in flight
  for (uint32_t i = threadIdx.x; i < nt; i += blockDim.x) {
    uint32_t ls = 0, lp = 0;
#pragma unroll 8
    for (uint32_t j = 0; j < nt; ++j) {
      const uint32_t v = lg[i ^ j];
      lp += v;
      ls += j < k ? v : 0u;
    }
    s_lw0[i] = mod255(mod255(ls) + 255u - mod255(lp));
  }
}

template <int KMAX>
__global__ void __launch_bounds__(256) decode_coef_kernel(const DecodeLaunch DL) {
  uint32_t bid;
  const DecodeArgs a = dec_seg(DL, bid);
  __shared__ __attribute__((aligned(16))) uint32_t s_gf[kGfDwords];
  __shared__ uint32_t s_lw0[MEMO_EC_MAX_K + MEMO_EC_MAX_M];
  __shared__ uint8_t s_comp[MEMO_EC_MAX_M][256];
  extern __shared__ __attribute__((aligned(16))) uint8_t s_out[];  // 256 x pitch (staged rows)
  const uint8_t* lg = reinterpret_cast<const uint8_t*>(s_gf);
  const uint8_t* ex = lg + 256;
  const uint32_t k = a.k, m = a.m, e = a.e, nt = a.k + a.m;
  const uint32_t tid = threadIdx.x;
  const uint64_t b0 = (uint64_t)bid * 256;
  const uint64_t b = b0 + tid;
  const bool live = b < a.n;
  // The block's indices are loaded first, so their latency overlaps the
  // table staging.
  uint32_t sv[KMAX];
  {
    const uint8_t* sidx = a.surv_idx + b * k;
    const bool dw = (k & 3) == 0 && (reinterpret_cast<uintptr_t>(a.surv_idx) & 3) == 0;
#pragma unroll
    for (int t = 0; t < KMAX; ++t) {
      sv[t] = 0;
      if (live && (uint32_t)t < k) {
        if (dw) sv[t] = (reinterpret_cast<const uint32_t*>(sidx)[t >> 2] >> (8 * (t & 3))) & 0xFFu;
        else sv[t] = sidx[t];
      }
    }
  }
  uint32_t lv[MEMO_EC_MAX_M];
#pragma unroll
  for (int r = 0; r < MEMO_EC_MAX_M; ++r) lv[r] = (live && (uint32_t)r < e) ? a.lost_idx[b * e + r] : 0u;
  stage_gf(s_gf);
  __syncthreads();
  stage_lw0(lg, k, nt, s_lw0);
  __syncthreads();
  const uint32_t ek = e * k;
  // Rows are staged in LDS (pitch: an odd number of dwords, so the lanes'
  // byte writes hit distinct banks) and leave as coalesced stores; rows too
  // large for LDS go straight out.
  const uint32_t pitch = a.pitch;
  uint8_t* gout = a.rows + b * (uint64_t)ek;
  uint8_t* out = pitch ? s_out + tid * pitch : gout;

  if (live) {
    // survivors: distinctness / range (bit set over k + m <= 80)
    uint32_t mask[3] = {0u, 0u, 0u};
    bool bad = false;
#pragma unroll
    for (int t = 0; t < KMAX; ++t) {
      if ((uint32_t)t < k) {
        const uint32_t v = sv[t];
        bad |= v >= nt;
        const uint32_t w = (v >> 5) < 3 ? (v >> 5) : 2u, bit = 1u << (v & 31);
        const uint32_t cur = w == 0 ? mask[0] : (w == 1 ? mask[1] : mask[2]);
        bad |= (cur & bit) != 0;
        if (w == 0) mask[0] |= bit;
        else if (w == 1) mask[1] |= bit;
        else mask[2] |= bit;
      }
    }
    auto is_surv = [&](uint32_t v) {
      const uint32_t w = v >> 5, bit = 1u << (v & 31);
      return ((w == 0 ? mask[0] : (w == 1 ? mask[1] : mask[2])) & bit) != 0;
    };
    // the m non-survivors
    uint32_t cnt = 0;
    for (uint32_t i = 0; i < nt; ++i)
      if (!is_surv(i)) {
        if (cnt < MEMO_EC_MAX_M) s_comp[cnt][tid] = (uint8_t)i;
        ++cnt;
      }
    bad |= cnt != m;

    // log W_t
    uint32_t lw[KMAX];
#pragma unroll
    for (int t = 0; t < KMAX; ++t) lw[t] = ((uint32_t)t < k && !bad) ? s_lw0[sv[t]] : 0u;
    if (!bad)
      for (uint32_t c = 0; c < m; ++c) {
        const uint32_t ci = s_comp[c][tid];
#pragma unroll
        for (int t = 0; t < KMAX; ++t)
          if ((uint32_t)t < k) lw[t] += lg[sv[t] ^ ci];
      }
#pragma unroll
    for (int t = 0; t < KMAX; ++t) lw[t] = mod255(lw[t]);

    for (uint32_t r = 0; r < e; ++r) {
      uint32_t l = 0;
#pragma unroll
      for (int q = 0; q < MEMO_EC_MAX_M; ++q)
        if ((uint32_t)q == r) l = lv[q];
      bad |= l >= nt;
      const bool unit = !bad && is_surv(l);
      uint32_t llam = 0;  // log Lam_l
      if (!bad && !unit) {
        uint32_t acc = s_lw0[l];
        for (uint32_t c = 0; c < m; ++c) {
          const uint32_t ci = s_comp[c][tid];
          acc += lg[l ^ ci];  // ci == l adds log[0] = 0
        }
        llam = 255u - mod255(acc);
      }
#pragma unroll
      for (int t = 0; t < KMAX; ++t) {
        if ((uint32_t)t < k) {
          uint32_t v;
          if (bad) v = 0;
          else if (unit) v = sv[t] == l ? 1u : 0u;
          else v = ex[lw[t] + llam + 255u - lg[l ^ sv[t]]]  /* < 765 */;
          out[r * k + t] = (uint8_t)v;
        }
      }
    }
    if (bad) {
      for (uint32_t t = 0; t < ek; ++t) out[t] = 0;  // rows written before the fault
      if (a.status) *a.status = 1u;  // plain store: every writer stores 1
    }
  }
  if (pitch) {
    __syncthreads();
    // this workgroup's rows are one contiguous range of nb * ek bytes
    const uint64_t nb = a.n - b0 < 256 ? a.n - b0 : 256;
    uint8_t* dst = a.rows + b0 * ek;
    const uint32_t total = (uint32_t)nb * ek;
    if ((ek & 3) == 0 && (reinterpret_cast<uintptr_t>(a.rows) & 3) == 0) {
      const uint32_t ekw = ek >> 2;
      for (uint32_t w = tid; w < (total >> 2); w += 256) {
        const uint32_t lb = w / ekw, off = w - lb * ekw;
        reinterpret_cast<uint32_t*>(dst)[w] =
            *reinterpret_cast<const uint32_t*>(s_out + lb * pitch + off * 4);
      }
    } else {
      for (uint32_t x = tid; x < total; x += 256) {
        const uint32_t lb = x / ek, off = x - lb * ek;
        dst[x] = s_out[lb * pitch + off];
      }
    }
  }
}

// Per-block decode for an exact k = K <= 16 (the common codes): K + m <= 32,
// so a block's survivor set is one 32-bit mask; its m non-survivors are
// extracted once into registers (ctz), every loop is unrolled at compile
// time (rows r < e by uniform predicates), the rows are packed into dwords
// and stored from registers (rows of whole dwords: each row as soon as it is
// done; others through LDS when e*K is not a dword multiple), and LW0 comes
// from the host's per-code table.  The coefficient of (lost l, survivor s) costs one XOR, two LDS
// lookups and one v_add3_u32:
//   row_l[t] = EX[lw_t + llam_l + NLG[l ^ s_t]]
// with NLG = 255 - log (so no subtraction), and log sums kept unreduced
// but folded once ((x & 255) + (x >> 8) == x mod 255, 2 ops): lw_t <= 271,
// llam_l = 510 - fold(...) in [239, 510], so the index stays below 1040 and
// EX is 2^(i mod 255) over 1280 entries.  Duplicate and out-of-range
// indices are found from the mask and an OR of all indices (no per-index
// tests); a faulty block's rows are zeroed once at the end.  Same results
// as decode_coef_kernel (tests/test_gpu_parity.py).  MM bounds m (4 or
// MEMO_EC_MAX_M): the per-lane lists of lost and non-survivor indices are MM
// long, so the m <= 4 codes keep fewer registers live.
struct DecTables {
  uint8_t lg[256];    // log
  uint8_t nlg[256];   // 255 - log (nlg[0]: 0, never used for a non-unit row)
  uint8_t ex[1280];   // 2^(i mod 255)
  uint8_t none[256];  // zeros: lg[x ^ kDecNone] for an absent non-survivor
};
// index offset that turns lg[x ^ c] into 0 (x < 256): fills the unused
// slots of the non-survivor list so lookups run in unpredicated groups
constexpr uint32_t kDecNone = 1792;
constexpr DecTables make_dec_tables() {
  DecTables t{};
  const GfTables g = make_gf();
  for (int i = 0; i < 256; ++i) {
    t.lg[i] = g.log[i];
    t.nlg[i] = i ? (uint8_t)(255 - g.log[i]) : 0;
    t.none[i] = 0;
  }
  for (int i = 0; i < 1280; ++i) t.ex[i] = g.exp[i % 255];
  return t;
}
__constant__ DecTables kDec = make_dec_tables();
constexpr int kDecDwords = sizeof(DecTables) / 4;

__device__ __forceinline__ uint32_t fold255(uint32_t x) { return (x & 0xFFu) + (x >> 8); }

template <int K, int MM>
__global__ void __launch_bounds__(256) decode_rows_k_kernel(const DecodeLaunch DL) {
  uint32_t bid;
  const DecodeArgs a = dec_seg(DL, bid);
  static_assert(K <= 16, "one 32-bit survivor mask: K + MEMO_EC_MAX_M <= 32");
  static_assert(MM % 4 == 0 && MM <= MEMO_EC_MAX_M, "m bound in groups of 4");
  __shared__ __attribute__((aligned(16))) uint32_t s_tab[kDecDwords];
  __shared__ uint32_t s_lw0[32];
  extern __shared__ __attribute__((aligned(16))) uint8_t s_out[];  // 256 x pitch
  const uint8_t* lg = reinterpret_cast<const uint8_t*>(s_tab);
  const uint8_t* nlg = lg + 256;
  const uint8_t* ex = lg + 512;
  const uint8_t* lw0 = reinterpret_cast<const uint8_t*>(s_lw0);
  const uint32_t m = a.m, e = a.e, nt = K + a.m;
  const uint32_t tid = threadIdx.x;
  const uint64_t b0 = (uint64_t)bid * 256;
  const uint64_t b = b0 + tid;
  const bool live = b < a.n;
  // The block's indices, with the widest loads their alignment allows (the
  // kernel is short: its first loads are a visible part of it).
  uint32_t sv[K], lv[MM];
  const uintptr_t sa = reinterpret_cast<uintptr_t>(a.surv_idx);
  if (K % 4 == 0 && (sa & 3) == 0) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(a.surv_idx + b * K);
#pragma unroll
    for (int w = 0; w < K / 4; ++w) {
      const uint32_t x = live ? p[w] : 0u;
#pragma unroll
      for (int j = 0; j < 4; ++j) sv[4 * w + j] = (x >> (8 * j)) & 0xFFu;
    }
  } else if (K % 2 == 0 && (sa & 1) == 0) {
    const uint16_t* p = reinterpret_cast<const uint16_t*>(a.surv_idx + b * K);
#pragma unroll
    for (int w = 0; w < K / 2; ++w) {
      const uint32_t x = live ? p[w] : 0u;
      sv[2 * w] = x & 0xFFu;
      sv[2 * w + 1] = x >> 8;
    }
  } else {
#pragma unroll
    for (int t = 0; t < K; ++t) sv[t] = live ? a.surv_idx[b * K + t] : 0u;
  }
  if ((e & 3) == 0 && (reinterpret_cast<uintptr_t>(a.lost_idx) & 3) == 0) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(a.lost_idx + b * e);
#pragma unroll
    for (int w = 0; w < MM / 4; ++w) {
      const uint32_t x = (live && (uint32_t)(4 * w) < e) ? p[w] : 0u;
#pragma unroll
      for (int j = 0; j < 4; ++j) lv[4 * w + j] = (x >> (8 * j)) & 0xFFu;
    }
  } else {
#pragma unroll
    for (int r = 0; r < MM; ++r) lv[r] = (live && (uint32_t)r < e) ? a.lost_idx[b * e + r] : 0u;
  }
  {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(&kDec);
    for (uint32_t i = tid; i < kDecDwords; i += 256) s_tab[i] = src[i];
    if (tid < 32) s_lw0[tid] = a.lw0[tid];
  }
  __syncthreads();
  const uint32_t ek = e * K;
  // the rows go to global memory straight from registers when they are
  // whole dwords (pitch 0, set by the launcher), else through LDS
  const bool direct = a.pitch == 0;
  constexpr int kW = (MM * K + 3) / 4;
  uint32_t wd[kW];
  if (live) {
    // survivor set: a duplicate leaves fewer than K bits, an index >= nt a
    // bit at or past nt (or past 31: caught by the OR of all indices)
    uint32_t mask = 0, any = 0;
#pragma unroll
    for (int t = 0; t < K; ++t) {
      mask |= 1u << (sv[t] & 31);
      any |= sv[t];
    }
    uint32_t lany = 0;
#pragma unroll
    for (int r = 0; r < MM; ++r)
      if ((uint32_t)r < e) lany |= lv[r] >= nt ? 1u : 0u;
    const uint32_t valid = nt >= 32 ? ~0u : (1u << nt) - 1u;
    const bool bad = (uint32_t)__popc(mask) != (uint32_t)K || (mask & ~valid) != 0 || (any >> 5) != 0 ||
                     lany != 0;
    // the m non-survivors, in registers
    uint32_t comp = ~mask & valid;
    uint32_t cl[MM];
#pragma unroll
    for (int q = 0; q < MM; ++q) {
      cl[q] = kDecNone;
      if ((uint32_t)q < m) {
        cl[q] = __builtin_ctz(comp | 0x80000000u);  // a faulty set may run out: 31
        comp &= comp - 1;
      }
    }
    // log W_t = LW0(s_t) + sum_c log(s_t ^ c), folded once (<= 271); the
    // lookups go in groups of 4 (or 2) independent reads per branch
    uint32_t lw[K];
#pragma unroll
    for (int t = 0; t < K; ++t) lw[t] = lw0[sv[t] & 31];
#pragma unroll
    for (int q = 0; q < MM; q += 4) {
      if ((uint32_t)q + 2 < m) {
#pragma unroll
        for (int t = 0; t < K; ++t)
          lw[t] += (lg[sv[t] ^ cl[q]] + lg[sv[t] ^ cl[q + 1]]) + (lg[sv[t] ^ cl[q + 2]] + lg[sv[t] ^ cl[q + 3]]);
      } else if ((uint32_t)q < m) {
#pragma unroll
        for (int t = 0; t < K; ++t) lw[t] += lg[sv[t] ^ cl[q]] + lg[sv[t] ^ cl[q + 1]];
      }
    }
#pragma unroll
    for (int t = 0; t < K; ++t) lw[t] = fold255(lw[t]);
    // rows, packed 4 bytes per register (compile-time positions); a faulty
    // block's rows are zero
    const uint32_t keep = bad ? 0u : ~0u;
    const bool vec16 = (ek & 15) == 0 && (reinterpret_cast<uintptr_t>(a.rows) & 15) == 0;
    const bool vec8 = (ek & 7) == 0 && (reinterpret_cast<uintptr_t>(a.rows) & 7) == 0;
    uint32_t word = 0;
#pragma unroll
    for (int r = 0; r < MM; ++r) {
      if ((uint32_t)r < e) {
        const uint32_t l = lv[r] & 0xFFu;
        const bool unit = (mask >> (l & 31)) & 1u;
        uint32_t acc = lw0[l & 31];
#pragma unroll
        for (int q = 0; q < MM; q += 4)  // c == l adds log[0] = 0
          if ((uint32_t)q < m)
            acc += (lg[l ^ cl[q]] + lg[l ^ cl[q + 1]]) + (lg[l ^ cl[q + 2]] + lg[l ^ cl[q + 3]]);
        uint32_t llam = 510u - fold255(acc);  // == -log(Lam_l) mod 255, in [239, 510]
        asm volatile("" : "+v"(llam));  // keep one v_add3_u32 per coefficient
        uint32_t v[K];
        if (!unit) {
#pragma unroll
          for (int t = 0; t < K; ++t) v[t] = ex[lw[t] + llam + nlg[l ^ sv[t]]];  // < 1040
        } else {  // l itself survived: a unit row (rare: callers name lost shards)
#pragma unroll
          for (int t = 0; t < K; ++t) v[t] = sv[t] == l ? 1u : 0u;
        }
        if constexpr (K % 4 == 0) {
          // whole dwords per row (3 byte permutes per 4 bytes), stored as
          // soon as the row is done: no row buffer in registers
          uint32_t rw[K / 4 + (K < 4)];
#pragma unroll
          for (int t = 0; t < K; t += 4) {
            const uint32_t lo = __builtin_amdgcn_perm(v[t + 1], v[t], 0x0c0c0400u);
            const uint32_t hi = __builtin_amdgcn_perm(v[t + 3], v[t + 2], 0x0c0c0400u);
            rw[t / 4] = __builtin_amdgcn_perm(hi, lo, 0x05040100u) & keep;
          }
          if (direct) {
            uint8_t* dst = a.rows + b * ek + (uint32_t)(r * K);
            if (K % 16 == 0 && vec16) {
#pragma unroll
              for (int w = 0; w < K / 4; w += 4)
                reinterpret_cast<uint4*>(dst)[w / 4] = make_uint4(rw[w], rw[w + 1], rw[w + 2], rw[w + 3]);
            } else if (K % 8 == 0 && vec8) {
#pragma unroll
              for (int w = 0; w < K / 4; w += 2) reinterpret_cast<uint2*>(dst)[w / 2] = make_uint2(rw[w], rw[w + 1]);
            } else {
#pragma unroll
              for (int w = 0; w < K / 4; ++w) reinterpret_cast<uint32_t*>(dst)[w] = rw[w];
            }
          } else {
            uint32_t* out = reinterpret_cast<uint32_t*>(s_out + tid * a.pitch) + r * (K / 4);
#pragma unroll
            for (int w = 0; w < K / 4; ++w) out[w] = rw[w];
          }
          continue;
        }
#pragma unroll
        for (int t = 0; t < K; ++t) {
          const int q = r * K + t;  // compile-time byte position
          word |= v[t] << (8 * (q & 3));
          if ((q & 3) == 3) {
            wd[q >> 2] = word & keep;
            word = 0;
          } else if (t == K - 1 && (uint32_t)r + 1 == e) {
            wd[q >> 2] = word & keep;  // the partial last dword
          }
        }
      }
    }
    if (bad && a.status) *a.status = 1u;  // plain store: every writer stores 1
    if (K % 4 == 0) {
      // rows already stored
    } else if (direct) {
      // ek % 4 == 0 and a 4-aligned base (launcher); widest stores that fit
      uint8_t* dst = a.rows + b * ek;
      if (vec16) {
#pragma unroll
        for (int w = 0; w + 3 < kW; w += 4)
          if ((uint32_t)w * 4 < ek)
            reinterpret_cast<uint4*>(dst)[w >> 2] = make_uint4(wd[w], wd[w + 1], wd[w + 2], wd[w + 3]);
      } else if (vec8) {
#pragma unroll
        for (int w = 0; w + 1 < kW; w += 2)
          if ((uint32_t)w * 4 < ek) reinterpret_cast<uint2*>(dst)[w >> 1] = make_uint2(wd[w], wd[w + 1]);
      } else {
#pragma unroll
        for (int w = 0; w < kW; ++w)
          if ((uint32_t)w * 4 < ek) reinterpret_cast<uint32_t*>(dst)[w] = wd[w];
      }
    } else {
      uint32_t* out = reinterpret_cast<uint32_t*>(s_out + tid * a.pitch);
#pragma unroll
      for (int w = 0; w < kW; ++w)
        if ((uint32_t)w * 4 < ek) out[w] = wd[w];
    }
  }
  if (direct) return;
  __syncthreads();
  // this workgroup's rows are one contiguous range of nb * ek bytes
  const uint64_t nb = a.n - b0 < 256 ? a.n - b0 : 256;
  uint8_t* dst = a.rows + b0 * ek;
  const uint32_t total = (uint32_t)nb * ek;
  if ((ek & 3) == 0 && (reinterpret_cast<uintptr_t>(a.rows) & 3) == 0) {
    const uint32_t ekw = ek >> 2;
    for (uint32_t w = tid; w < (total >> 2); w += 256) {
      const uint32_t lb = w / ekw, off = w - lb * ekw;
      reinterpret_cast<uint32_t*>(dst)[w] = *reinterpret_cast<const uint32_t*>(s_out + lb * a.pitch + off * 4);
    }
  } else {
    for (uint32_t x = tid; x < total; x += 256) {
      const uint32_t lb = x / ek, off = x - lb * ek;
      dst[x] = s_out[lb * a.pitch + off];
    }
  }
}

// Latency variant for small batches: L lanes per block (L = the power of two
// >= k), lane t owns survivor column t.  The block's survivor bit set is
// OR-reduced across its L lanes and its m non-survivors c are extracted into
// registers (as in the exact-k kernel); each lane then needs only its own
// W_t (m lookups) and, per lost shard, Lam_l (m lookups) and one
// coefficient: about (e + 1) * (m + 1) + e lookups per lane.  A C3-sized
// batch takes a few microseconds.  (Round 1-4 looped every lane over all
// k + m indices with a survivor mask, 3-4x the lookups: 36 us for 65,536
// RS(16,4) blocks, profiles/r05_decode_probe.jsonl.)
template <int L>
__global__ void __launch_bounds__(256) decode_coef_wide_kernel(const DecodeLaunch DL) {
  uint32_t bid;
  const DecodeArgs a = dec_seg(DL, bid);
  __shared__ __attribute__((aligned(16))) uint32_t s_gf[kGfDwords];
  __shared__ uint32_t s_lw0[MEMO_EC_MAX_K + MEMO_EC_MAX_M];
  const uint8_t* lg = reinterpret_cast<const uint8_t*>(s_gf);
  const uint8_t* ex = lg + 256;
  const uint32_t k = a.k, m = a.m, e = a.e, nt = a.k + a.m, ek = a.e * a.k;
  const uint32_t t = threadIdx.x % L;
  const uint64_t b = (uint64_t)bid * (256 / L) + threadIdx.x / L;
  const bool live = b < a.n;  // whole groups
  const bool col = t < k;
  // The block's indices are loaded first, so their latency overlaps the
  // table staging: survivor t in lane t, lost shard r in lane r % L.
  constexpr int NS = (MEMO_EC_MAX_M + L - 1) / L;
  const uint32_t sv = (live && col) ? a.surv_idx[b * k + t] : 0u;
  uint32_t lv[NS];
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    const uint32_t r = t + q * L;
    lv[q] = (live && r < e) ? a.lost_idx[b * e + r] : 0u;
  }
  stage_gf(s_gf);
  if (a.lw0)  // LW0 of (k, m) from the host (lw0_host), one byte per index
    for (uint32_t i = threadIdx.x; i < nt; i += 256) s_lw0[i] = reinterpret_cast<const uint8_t*>(a.lw0)[i];
  __syncthreads();
  if (!a.lw0) {
    stage_lw0(lg, k, nt, s_lw0);
    __syncthreads();
  }
  if (!live) return;  // no barrier below
  bool bad = col && sv >= nt;
  uint32_t mk[3] = {0u, 0u, 0u};
  if (col && sv < nt) {
    const uint32_t w = sv >> 5, bit = 1u << (sv & 31);
    if (w == 0) mk[0] = bit;
    else if (w == 1) mk[1] = bit;
    else mk[2] = bit;
  }
  uint32_t badw = bad ? 1u : 0u;
#pragma unroll
  for (int off = 1; off < L; off <<= 1) {
    mk[0] |= __shfl_xor(mk[0], off, L);
    mk[1] |= __shfl_xor(mk[1], off, L);
    mk[2] |= __shfl_xor(mk[2], off, L);
    badw |= __shfl_xor(badw, off, L);
  }
  // out of range anywhere, or duplicates (fewer than k distinct bits)
  bad = badw != 0 || (uint32_t)(__popc(mk[0]) + __popc(mk[1]) + __popc(mk[2])) != k;
  auto is_surv = [&](uint32_t v) {
    const uint32_t w = v >> 5, bit = 1u << (v & 31);
    return ((w == 0 ? mk[0] : (w == 1 ? mk[1] : mk[2])) & bit) != 0;
  };
  // the m non-survivors (indices < nt outside the survivor set), in
  // registers; a faulty set may run out (its rows are zero anyway)
  uint32_t cl[MEMO_EC_MAX_M];
  {
    uint32_t c0 = ~mk[0] & (nt >= 32 ? ~0u : (1u << nt) - 1u);
    uint32_t c1 = nt <= 32 ? 0u : ~mk[1] & (nt >= 64 ? ~0u : (1u << (nt - 32)) - 1u);
    uint32_t c2 = nt <= 64 ? 0u : ~mk[2] & ((1u << (nt - 64)) - 1u);
#pragma unroll
    for (int q = 0; q < MEMO_EC_MAX_M; ++q) {
      cl[q] = 0u;
      if ((uint32_t)q < m) {
        if (c0) {
          cl[q] = __builtin_ctz(c0);
          c0 &= c0 - 1;
        } else if (c1) {
          cl[q] = 32u + __builtin_ctz(c1);
          c1 &= c1 - 1;
        } else if (c2) {
          cl[q] = 64u + __builtin_ctz(c2);
          c2 &= c2 - 1;
        }
      }
    }
  }
  uint32_t lw = 0;  // log W_t = LW0(s_t) + sum_c log(s_t ^ c)
  if (col && !bad) {
    lw = s_lw0[sv];
#pragma unroll
    for (int q = 0; q < MEMO_EC_MAX_M; ++q)
      if ((uint32_t)q < m) lw += lg[sv ^ cl[q]];
    lw = mod255(lw);
  }
  uint8_t* out = a.rows + b * (uint64_t)ek;
  uint32_t* img = a.img ? a.img + b * (uint64_t)(a.R * a.kpad * 8) : nullptr;
  for (uint32_t r = 0; r < e; ++r) {
    uint32_t mine = 0;
#pragma unroll
    for (int q = 0; q < NS; ++q)
      if ((uint32_t)q == r / L) mine = lv[q];
    const uint32_t l = __shfl(mine, r % L, L);  // the same for the whole group
    bad |= l >= nt;
    const bool unit = !bad && is_surv(l);
    uint32_t llam = 0;  // log Lam_l = -(LW0(l) + sum_{c != l} log(l ^ c))
    if (!bad && !unit) {
      uint32_t acc = s_lw0[l];  // c == l adds log[0] = 0
#pragma unroll
      for (int q = 0; q < MEMO_EC_MAX_M; ++q)
        if ((uint32_t)q < m) acc += lg[l ^ cl[q]];
      llam = 255u - mod255(acc);
    }
    uint32_t v = 0;
    if (col) {
      if (bad) v = 0;
      else if (unit) v = sv == l ? 1u : 0u;
      else v = ex[lw + llam + 255u - lg[l ^ sv]]  /* < 765 */;
      out[r * k + t] = (uint8_t)v;
    }
    if (img && t < a.kpad) put_slot_image(img, r * a.kpad + t, bad ? 0u : v);
  }
  if (img)  // padding rows e..R-1: zero images
    for (uint32_t x = e * a.kpad + t; x < a.R * a.kpad; x += L) put_slot_image(img, x, 0u);
  if (bad) {  // the group's lanes share one wave: these stores follow the row stores
    for (uint32_t x = t; x < ek; x += L) out[x] = 0;
    if (img)
      for (uint32_t x = t; x < e * a.kpad; x += L) put_slot_image(img, x, 0u);
    if (t == 0 && a.status) *a.status = 1u;  // plain store: every writer stores 1
  }
}

// ------------------------------------------------------------- synthetic fill
__device__ __forceinline__ uint64_t sm64_mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
constexpr uint64_t kGamma = 0x9E3779B97F4A7C15ull;

__global__ void __launch_bounds__(256) fill_kernel(FillArgs a) {
  const uint64_t per_block = a.stride / 16;  // 16-byte chunks per padded block
  const uint64_t total = a.n * per_block;
  const uint64_t mseed = sm64_mix(a.seed);
  for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total;
       q += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t b = q / per_block;
    const uint64_t off = (q - b * per_block) * 16;
    uint64_t w0 = 0, w1 = 0;
    if (off < a.B) {
      const uint64_t key = sm64_mix(mseed ^ ((a.first_block + b) * kGamma));
      const uint64_t i = off / 8;
      w0 = sm64_mix(key + (i + 1) * kGamma);
      w1 = sm64_mix(key + (i + 2) * kGamma);
      const uint64_t rem = a.B - off;  // bytes of this chunk inside the block
      if (rem < 16) {
        if (rem <= 8) {
          w1 = 0;
          if (rem < 8) w0 &= (1ull << (8 * rem)) - 1;
        } else {
          w1 &= (1ull << (8 * (rem - 8))) - 1;
        }
      }
    }
    uint4 v = make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32));
    *reinterpret_cast<uint4*>(a.out + b * a.stride + off) = v;
  }
}

// ------------------------------------------------------------- shard gather
__global__ void __launch_bounds__(256) gather_kernel(GatherArgs a) {
  const uint64_t per = a.S / 16;
  const uint64_t total = a.n * a.cnt * per;
  for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total;
       q += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t br = q / per;  // (block, slot)
    const uint64_t off = (q - br * per) * 16;
    const uint64_t b = br / a.cnt;
    const uint32_t s = a.idx[br];
    uint4 v = make_uint4(0, 0, 0, 0);  // an out-of-range index yields zeros
    if (s < a.k + a.m) {
      const uint8_t* src = s < a.k ? a.data + (b * a.k + s) * a.S
                                   : a.parity + (b * a.m + (s - a.k)) * a.S;
      v = *reinterpret_cast<const uint4*>(src + off);
    }
    *reinterpret_cast<uint4*>(a.out + br * a.S + off) = v;
  }
}

// ------------------------------------------------------------- SHA-256
// Batched SHA-256 (FIPS 180-4) of n messages prefix_b || msg_b: the CHB
// address hash SHA-256(salt || owner || data) of CHB::_hash_address
// (src/memo/model/doughnut/CHB.cc:264-289) for a whole batch of blocks.  One
// lane per message (SHA-256 is sequential within a message); interior
// 64-byte chunks are read with 4 dwordx4 loads, edge chunks byte-wise.
__constant__ uint32_t kSha256K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }

// One SHA-256 compression.  Sigma/sigma are 3-input XORs and Ch/Maj single
// v_bitop3_b32 truth tables (0xCA, 0xE8), sums v_add3_u32: a short
// dependency chain per round, which bounds large blocks (one lane each).
__device__ __forceinline__ void sha256_compress(uint32_t (&h)[8], uint32_t (&w)[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int t = 0; t < 64; ++t) {
    uint32_t wt;
    if (t < 16) {
      wt = w[t];
    } else {
      const uint32_t w15 = w[(t + 1) & 15], w2 = w[(t + 14) & 15];
      const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
      const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
      wt = w[t & 15] + s0 + w[(t + 9) & 15] + s1;
      w[t & 15] = wt;
    }
    const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
    const uint32_t ch = __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
    const uint32_t t1 = hh + S1 + ch + (kSha256K[t] + wt);
    const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
    const uint32_t mj = __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
    hh = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + S0 + mj;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// Byte o of the padded virtual message prefix || body || 0x80 0.. || len64.
__device__ __forceinline__ uint32_t sha_byte(const uint8_t* pre, uint64_t P, const uint8_t* body,
                                             uint64_t L, uint64_t total_bits, uint64_t padded,
                                             uint64_t o) {
  if (o < P) return pre[o];
  if (o < P + L) return body[o - P];
  if (o == P + L) return 0x80;
  if (o >= padded - 8) return (uint32_t)(total_bits >> (8 * (padded - 1 - o))) & 0xff;
  return 0;
}

__global__ void __launch_bounds__(256) sha256_kernel(Sha256Args a) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  const uint8_t* pre = a.prefix + i * a.prefix_stride;
  const uint8_t* body = a.msg + i * a.msg_stride;
  const uint64_t P = a.prefix_len;
  const uint64_t L = a.msg_len ? a.msg_len[i] : a.uniform_len;
  const uint64_t total = P + L;
  const uint64_t padded = (total + 9 + 63) / 64 * 64;
  const uint64_t bits = total * 8;
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  // body chunks [c_lo, c_hi) are whole 64-byte chunks inside the body whose
  // body offset is 16-byte aligned (fast path)
  const bool fast = (P % 16) == 0 && (((uintptr_t)body) % 16) == 0;
  const uint64_t c_lo = (P + 63) / 64;
  const uint64_t c_hi = (P + L) / 64;
  const uint64_t nchunks = padded / 64;
  const uint64_t f_lo = fast ? c_lo : nchunks, f_hi = fast && c_hi > c_lo ? c_hi : f_lo;
  auto slow_chunk = [&](uint64_t c) {
    uint32_t w[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const uint64_t o = c * 64 + 4 * t;
      w[t] = (sha_byte(pre, P, body, L, bits, padded, o) << 24) |
             (sha_byte(pre, P, body, L, bits, padded, o + 1) << 16) |
             (sha_byte(pre, P, body, L, bits, padded, o + 2) << 8) |
             sha_byte(pre, P, body, L, bits, padded, o + 3);
    }
    sha256_compress(h, w);
  };
  for (uint64_t c = 0; c < f_lo && c < nchunks; ++c) slow_chunk(c);
  if (f_lo < f_hi) {
    // Interior chunks: the next chunk's four dwordx4 loads are issued before
    // this chunk's 64 rounds, so their latency hides behind the round chain.
    const u32x4* q = reinterpret_cast<const u32x4*>(body + (f_lo * 64 - P));
    u32x4 x[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) x[v] = __builtin_nontemporal_load(q + v);
    for (uint64_t c = f_lo; c < f_hi; ++c) {
      uint32_t w[16];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        w[4 * v + 0] = __builtin_bswap32(x[v].x);
        w[4 * v + 1] = __builtin_bswap32(x[v].y);
        w[4 * v + 2] = __builtin_bswap32(x[v].z);
        w[4 * v + 3] = __builtin_bswap32(x[v].w);
      }
      q += 4;
      if (c + 1 < f_hi) {
#pragma unroll
        for (int v = 0; v < 4; ++v) x[v] = __builtin_nontemporal_load(q + v);
      }
      sha256_compress(h, w);
    }
  }
  for (uint64_t c = f_hi; c < nchunks; ++c) slow_chunk(c);
  uint32_t* out = reinterpret_cast<uint32_t*>(a.digest + i * 32);
#pragma unroll
  for (int t = 0; t < 8; ++t) out[t] = __builtin_bswap32(h[t]);
}

hipError_t launch_sha256(const Sha256Args& a, hipStream_t st) {
  if (a.n == 0) return hipSuccess;
  const uint64_t grid = (a.n + 255) / 256;
  hipLaunchKernelGGL(sha256_kernel, dim3((uint32_t)grid), dim3(256), 0, st, a);
  return hipGetLastError();
}

// ------------------------------------------------------------- launchers
template <int KC, int R>
static hipError_t launch_mac_t(int mode, const MacLaunch& L, uint32_t grid, size_t lds,
                               hipStream_t st) {
  if (mode == MAC_PROBE)
    hipLaunchKernelGGL((stream_probe_kernel<KC, R, MAC_NT>), dim3(grid), dim3(256), 0, st, L);
  else if (mode == MAC_FUSED)
    hipLaunchKernelGGL((gf_rebuild_kernel<KC, R, MAC_NT>), dim3(grid), dim3(256), lds, st, L);
  else if (mode == MAC_ROWS)
    hipLaunchKernelGGL((gf_mac_kernel<KC, R, MAC_NT, true>), dim3(grid), dim3(256), lds, st, L);
  else if (mode == MAC_IMAGES)
    hipLaunchKernelGGL((gf_mac_images_kernel<KC, R, MAC_NT>), dim3(grid), dim3(256), lds, st, L);
#ifdef MEMO_EC_PERM_PROBE
  else if (mode == MAC_PERM)
    hipLaunchKernelGGL((gf_mac_perm_kernel<KC, R, MAC_NT>), dim3(grid), dim3(256), lds, st, L);
#endif
  else
    hipLaunchKernelGGL((gf_mac_kernel<KC, R, MAC_NT, false>), dim3(grid), dim3(256), lds, st, L);
  return hipGetLastError();
}

template <int KC>
static hipError_t launch_mac_r(int R, int mode, const MacLaunch& L, uint32_t grid, size_t lds,
                               hipStream_t st) {
  switch (R) {
#define MEMO_EC_R(x) \
  case x: return launch_mac_t<KC, x>(mode, L, grid, lds, st);
    MEMO_EC_R(1) MEMO_EC_R(2) MEMO_EC_R(3) MEMO_EC_R(4) MEMO_EC_R(6) MEMO_EC_R(8)
    MEMO_EC_R(12) MEMO_EC_R(16)
#undef MEMO_EC_R
    default: return hipErrorInvalidValue;
  }
}

int mac_rbound(int r) {
  if (r <= 4) return r;
  if (r <= 6) return 6;
  if (r <= 8) return 8;
  if (r <= 12) return 12;
  return 16;
}

int mac_kchunk(int kin, int R) {
  switch (kin) {
    case 2: case 3: case 4: case 10: case 16: return kin;
    case 6: case 12: case 14: return R <= 4 ? kin : 4;  // instantiated for R <= 4 only
    default: return 4;
  }
}

// Shard chunks instantiated only for R <= 4 (common codes: RS(6,3),
// RS(12,4), RS(14,4)); larger R takes the 4-shard chunk loop.
template <int KC>
static hipError_t launch_mac_r4(int R, int mode, const MacLaunch& L, uint32_t grid, size_t lds,
                                hipStream_t st) {
  switch (R) {
    case 1: return launch_mac_t<KC, 1>(mode, L, grid, lds, st);
    case 2: return launch_mac_t<KC, 2>(mode, L, grid, lds, st);
    case 3: return launch_mac_t<KC, 3>(mode, L, grid, lds, st);
    case 4: return launch_mac_t<KC, 4>(mode, L, grid, lds, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_mac(int KC, int R, int mode, const MacLaunch& L, uint32_t grid, size_t lds,
                      hipStream_t st) {
  switch (KC) {
    case 2: return launch_mac_r<2>(R, mode, L, grid, lds, st);
    case 3: return launch_mac_r<3>(R, mode, L, grid, lds, st);
    case 4: return launch_mac_r<4>(R, mode, L, grid, lds, st);
    case 10: return launch_mac_r<10>(R, mode, L, grid, lds, st);
    case 6: return launch_mac_r4<6>(R, mode, L, grid, lds, st);
    case 12: return launch_mac_r4<12>(R, mode, L, grid, lds, st);
    case 14: return launch_mac_r4<14>(R, mode, L, grid, lds, st);
    case 16: return launch_mac_r<16>(R, mode, L, grid, lds, st);
    default: return hipErrorInvalidValue;
  }
}

// Kernel choice for one decode segment: kind (0 column-per-lane, 1 exact-k,
// 2 generic), its template parameter, workgroups, and the args as the
// kernel takes them (row-staging pitch set).
struct DecodePick {
  int kind = 0, param = 0;
  uint32_t grid = 0;
  size_t lds = 0;
  DecodeArgs a{};
};

static DecodePick decode_pick(const DecodeArgs& a0) {
  DecodePick p;
  p.a = a0;
  DecodeArgs& a = p.a;
  // LDS staging of the rows: pitch = e*k rounded up to an odd dword count
  const uint32_t ek = a.e * a.k;
  uint32_t pw = (ek + 3) / 4;
  pw |= 1u;
  a.pitch = 256u * pw * 4 <= 64 * 1024 ? pw * 4 : 0u;
  const size_t lds = a.pitch ? 256u * a.pitch : 0;
  // 1. the exact-k kernels for the common codes, k in {2, 3, 4, 6, 8, 10,
  // 12, 14, 16} (a.exact), storing whole-dword rows straight from registers
  // unless a.stage asks for the LDS staging (A/B runs and tests): one lane
  // per block is the fastest form at every batch size, 256 blocks to
  // 64 Ki (6.3-7.9 us, against 7.8-17.7 for the column-per-lane kernel;
  // profiles/r05_decode_probe.jsonl).  Not for table images (below).
  DecodeArgs ax = a;
  if (!a.stage && (ek & 3) == 0 && (reinterpret_cast<uintptr_t>(a.rows) & 3) == 0) ax.pitch = 0;
  const bool exact_k = a.k == 2 || a.k == 3 || a.k == 4 || a.k == 6 || a.k == 8 || a.k == 10 ||
                       a.k == 12 || a.k == 14 || a.k == 16;
  if (!a.img && a.exact && (a.pitch || !ax.pitch) && a.lw0 && a.k + a.m <= 32 && exact_k) {
    p.kind = 1;
    p.param = (int)a.k + (a.m <= 4 ? 0 : 100);  // m bound 4 or MEMO_EC_MAX_M
    p.grid = (uint32_t)((a.n + 255) / 256);
    p.lds = ax.pitch ? lds : 0;
    p.a = ax;
    return p;
  }
  // 2. the column-per-lane kernel: other k up to a.wide_max blocks (the
  // ctx's MEMO_EC_OPT_DECODE_WIDE_MAX; the generic one-lane kernel takes
  // 1.6-4x longer there), and any batch whose table images it writes beside
  // the rows, lane t the slots of column t (images go with blocks of whole
  // tiles: few blocks per byte)
  if (a.n <= a.wide_max || a.img) {
    const uint32_t L = a.k <= 4 ? 4 : a.k <= 8 ? 8 : a.k <= 16 ? 16 : a.k <= 32 ? 32 : 64;
    p.kind = 0;
    p.param = (int)L;
    p.grid = (uint32_t)((a.n + 256 / L - 1) / (256 / L));
    p.a.pitch = 0;
    return p;
  }
  // 3. the generic one-lane-per-block kernel
  p.kind = 2;
  p.param = a.k <= 4 ? 4 : a.k <= 10 ? 10 : a.k <= 16 ? 16 : a.k <= 32 ? 32 : 64;
  p.grid = (uint32_t)((a.n + 255) / 256);
  p.lds = lds;
  return p;
}

static hipError_t decode_launch(int kind, int param, const DecodeLaunch& L, uint32_t grid, size_t lds,
                                hipStream_t st) {
  if (kind == 0) {
    switch (param) {
      case 4: hipLaunchKernelGGL(decode_coef_wide_kernel<4>, dim3(grid), dim3(256), 0, st, L); break;
      case 8: hipLaunchKernelGGL(decode_coef_wide_kernel<8>, dim3(grid), dim3(256), 0, st, L); break;
      case 16: hipLaunchKernelGGL(decode_coef_wide_kernel<16>, dim3(grid), dim3(256), 0, st, L); break;
      case 32: hipLaunchKernelGGL(decode_coef_wide_kernel<32>, dim3(grid), dim3(256), 0, st, L); break;
      default: hipLaunchKernelGGL(decode_coef_wide_kernel<64>, dim3(grid), dim3(256), 0, st, L); break;
    }
  } else if (kind == 1) {
    switch (param) {
#define MEMO_EC_DK(x)                                                                            \
  case x: hipLaunchKernelGGL((decode_rows_k_kernel<x, 4>), dim3(grid), dim3(256), lds, st, L); break; \
  case 100 + x:                                                                                   \
    hipLaunchKernelGGL((decode_rows_k_kernel<x, MEMO_EC_MAX_M>), dim3(grid), dim3(256), lds, st, L); \
    break;
      MEMO_EC_DK(2) MEMO_EC_DK(3) MEMO_EC_DK(4) MEMO_EC_DK(6) MEMO_EC_DK(8) MEMO_EC_DK(10)
      MEMO_EC_DK(12) MEMO_EC_DK(14) MEMO_EC_DK(16)
#undef MEMO_EC_DK
      default: return hipErrorInvalidValue;
    }
  } else {
    switch (param) {
      case 4: hipLaunchKernelGGL(decode_coef_kernel<4>, dim3(grid), dim3(256), lds, st, L); break;
      case 10: hipLaunchKernelGGL(decode_coef_kernel<10>, dim3(grid), dim3(256), lds, st, L); break;
      case 16: hipLaunchKernelGGL(decode_coef_kernel<16>, dim3(grid), dim3(256), lds, st, L); break;
      case 32: hipLaunchKernelGGL(decode_coef_kernel<32>, dim3(grid), dim3(256), lds, st, L); break;
      default: hipLaunchKernelGGL(decode_coef_kernel<64>, dim3(grid), dim3(256), lds, st, L); break;
    }
  }
  return hipGetLastError();
}

// Decode rows of several segments: segments that take the same kernel share
// a launch (up to MEMO_EC_MAX_SEGMENTS each), so a mixed rebuild's many
// small decodes fill the chip together instead of one after another.
hipError_t launch_decode_multi(const DecodeArgs* as, int na, hipStream_t st) {
  std::vector<DecodePick> picks;
  for (int i = 0; i < na; ++i)
    if (as[i].n) picks.push_back(decode_pick(as[i]));
  for (const auto& p : picks)  // images: lane t < kpad writes column t's slots
    if (p.a.img && (p.kind != 0 || p.a.kpad > (uint32_t)p.param)) return hipErrorInvalidValue;
  std::vector<bool> done(picks.size(), false);
  for (size_t i = 0; i < picks.size(); ++i) {
    if (done[i]) continue;
    DecodeLaunch L{};
    uint64_t wg = 0;
    size_t lds = 0;
    for (size_t j = i; j < picks.size() && L.nseg < MEMO_EC_MAX_SEGMENTS; ++j) {
      const DecodePick& p = picks[j];
      if (done[j] || p.kind != picks[i].kind || p.param != picks[i].param) continue;
      if (L.nseg && wg + p.grid > 0x7fffffffull) break;
      done[j] = true;
      L.wg_begin[L.nseg] = (uint32_t)wg;
      L.seg[L.nseg++] = p.a;
      wg += p.grid;
      lds = std::max(lds, p.lds);
    }
    if (wg > 0x7fffffffull) return hipErrorInvalidValue;
    if (hipError_t e = decode_launch(picks[i].kind, picks[i].param, L, (uint32_t)wg, lds, st)) return e;
  }
  return hipSuccess;
}

hipError_t launch_decode_coef(const DecodeArgs& a, hipStream_t st) { return launch_decode_multi(&a, 1, st); }

hipError_t launch_fill(const FillArgs& a, hipStream_t st) {
  const uint64_t total = a.n * (a.stride / 16);
  if (total == 0) return hipSuccess;
  uint64_t grid = (total + 255) / 256;
  if (grid > 65536) grid = 65536;
  hipLaunchKernelGGL(fill_kernel, dim3((uint32_t)grid), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_gather(const GatherArgs& a, hipStream_t st) {
  const uint64_t total = a.n * a.cnt * (a.S / 16);
  if (total == 0) return hipSuccess;
  uint64_t grid = (total + 255) / 256;
  if (grid > 65536) grid = 65536;
  hipLaunchKernelGGL(gather_kernel, dim3((uint32_t)grid), dim3(256), 0, st, a);
  return hipGetLastError();
}

// LW0(i) = log sigma(i) - log Pall(i) mod 255 (decode_coef_kernel's
// stage_lw0), i < k + m, for the fused rebuild; zero past k + m.
void lw0_host(int k, int m, uint8_t* out) {
  const int nt = k + m;
  for (int i = 0; i < 128; ++i) out[i] = 0;
  for (int i = 0; i < nt && i < 128; ++i) {
    uint32_t ls = 0, lp = 0;
    for (int j = 0; j < nt; ++j) {
      if (j == i) continue;
      const uint32_t v = kGfHost.log[i ^ j];
      lp += v;
      if (j < k) ls += v;
    }
    out[i] = (uint8_t)((ls % 255 + 255 - lp % 255) % 255);
  }
}

const uint8_t* host_gf_log() { return kGfHost.log; }
const uint8_t* host_gf_exp() { return kGfHost.exp; }

}  // namespace memo_ec
