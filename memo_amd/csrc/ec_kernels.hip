// ec_kernels.hip -- gfx950 kernels of the block erasure codec.
//
// Hot path: gf_mac_kernel, the batched GF(2^8) multiply-accumulate
//   out[b][i][x] = XOR_j coef_b[i][j] * in[b][j][x]
// which is RS encode (coef = the Cauchy parity rows, shared by every block)
// and RS rebuild (coef = per-block decode rows from decode_rows_kernel).
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
//  * The GF log/antilog tables live in LDS in decode_rows_kernel (batched
//    Gauss-Jordan inversion), which also emits the per-block product-table
//    images the rebuild MAC consumes.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ec_kernels.h"

namespace memo_ec {

// ----------------------------------------------------------------- GF tables
struct GfTables {
  uint8_t log[256];
  uint8_t exp[512];
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
  for (int i = 255; i < 512; ++i) t.exp[i] = t.exp[i - 255];
  t.log[0] = 0;
  return t;
}

__constant__ GfTables kGf = make_gf();
const GfTables kGfHost = make_gf();

__host__ __device__ __forceinline__ uint32_t gf_mul_t(const uint8_t* lg, const uint8_t* ex,
                                                      uint32_t a, uint32_t b) {
  return (a && b) ? ex[lg[a] + lg[b]] : 0u;
}
__host__ __device__ __forceinline__ uint32_t gf_inv_t(const uint8_t* lg, const uint8_t* ex,
                                                      uint32_t a) {
  return a ? ex[255 - lg[a]] : 0u;
}

// Copy the 768-byte log/antilog image into LDS (192 dwords).
__device__ __forceinline__ void stage_gf(uint32_t* s_gf) {
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&kGf);
  for (int i = threadIdx.x; i < 192; i += blockDim.x) s_gf[i] = src[i];
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

// Buffer-resource access (uniform base in SGPRs, 32-bit lane offset, shard
// offset as the scalar soffset) with an explicit cache policy (gfx950 cpol
// bits: sc0 = 1, nt = 2, sc1 = 16).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0xffffffff, 0x00020000);
}
__device__ __forceinline__ uint4 bld16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, MEMO_EC_MAC_LDAUX);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void bst16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff,
                                      uint4 v) {
  const u32x4 w = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(w, r, voff, soff, MEMO_EC_MAC_STAUX);
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
__device__ __forceinline__ Tab read_tab(const uint32_t* tp) {
  const uint4 q = *reinterpret_cast<const uint4*>(tp);
  return Tab{tp[4], q.x, q.y, q.z, q.w};
}
__device__ __forceinline__ void lookups(const Sel& s, const Tab& t, uint32_t& pl, uint32_t& pm,
                                        uint32_t& ph) {
#ifdef MEMO_EC_MAC_XORONLY  // diagnostic build: no GF math (wrong results)
  pl = s.lo ^ t.lo; pm = s.mid; ph = s.hi;
#else
  pl = __builtin_amdgcn_perm(t.lo, t.lo, s.lo);
  pm = __builtin_amdgcn_perm(t.m1, t.m0, s.mid);
  ph = __builtin_amdgcn_perm(t.h1, t.h0, s.hi);
#endif
}

// acc[i] ^= coef(i, j0 + g) * d[g] for the KC shards of one chunk.  Shards
// are taken in pairs so that 6 partial products + the accumulator fold with
// three 3-input XORs.  Branch-free: padded rows/shards have all-zero tables.
template <int KC, int R>
__device__ __forceinline__ void mac_chunk(uint32_t (&acc)[R][4], const uint4 (&d)[KC],
                                          const uint32_t* tab, uint32_t kpad, uint32_t j0) {
#pragma unroll
  for (int g = 0; g < KC; g += MAC_PAIR ? 2 : 1) {
    const bool two = MAC_PAIR && g + 1 < KC;
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
      const uint32_t* tp = tab + (i * kpad + j0 + g) * 8;
      const Tab ta = read_tab(tp);
      if (two) {
        const Tab tb = read_tab(tp + 8);
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
  uint32_t voff_in, voff_out;  // byte offsets from the tile's first block (buffer path)
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
  u.voff_in = (uint32_t)(bo * sg.in_bstride + (uint64_t)cc * 16);
  u.voff_out = (uint32_t)(bo * sg.out_bstride + (uint64_t)cc * 16);
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

// One tile of segment sg: KC is the straight-line shard chunk (kin == KC is
// the hot path; other kin loop over chunks of KC shards).
template <int KC, int R, bool NT>
__device__ __forceinline__ void mac_tile(const MacSeg& sg, uint64_t tile, uint32_t* s_tab) {
  const uint32_t kin = sg.kin, kpad = sg.kpad;
  const uint32_t set_dw = R * kpad * 8;

  const Unit u = locate(sg, tile);
  const uint32_t* tab = s_tab + (sg.tab_bstride ? u.set * set_dw : 0u);
  uint32_t acc[R][4];
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int w = 0; w < 4; ++w) acc[i][w] = 0;

  if (kin == KC) {
    // Hot path.  The table image loads go out first (vmcnt retires in issue
    // order, so the LDS copy then waits only for them), the KC shard loads
    // right behind; the barrier and table copy overlap the shard loads.
#if MEMO_EC_MAC_TABFIRST
    uint32_t tv[MAC_TAB_REGS];
    load_tables(sg, u, set_dw, tv);
    uint4 d[KC];
#if MEMO_EC_MAC_BUF
    const __amdgpu_buffer_rsrc_t rin = rsrc_of(sg.in + u.b_first * sg.in_bstride);
#pragma unroll
    for (int g = 0; g < KC; ++g) d[g] = bld16(rin, u.voff_in, (uint32_t)(g * sg.in_sstride));
#else
#pragma unroll
    for (int g = 0; g < KC; ++g) d[g] = ld16<NT>(u.pin + (uint64_t)g * sg.in_sstride);
#endif
    store_tables(sg, u, set_dw, tv, s_tab);
#else
    uint4 d[KC];
#pragma unroll
    for (int g = 0; g < KC; ++g) d[g] = ld16<NT>(u.pin + (uint64_t)g * sg.in_sstride);
    stage_tables(sg, u, set_dw, s_tab);
#endif
    __syncthreads();
    mac_chunk<KC, R>(acc, d, tab, kpad, 0);
  } else {
    stage_tables(sg, u, set_dw, s_tab);
    __syncthreads();
    for (uint32_t j0 = 0; j0 < kin; j0 += KC) {
      uint4 d[KC];
#pragma unroll
      for (int g = 0; g < KC; ++g)
        if (j0 + g < kin) d[g] = ld16<NT>(u.pin + (uint64_t)(j0 + g) * sg.in_sstride);
      mac_chunk<KC, R>(acc, d, tab, kpad, j0);
    }
  }

  if (u.valid) {
#if MEMO_EC_MAC_BUF
    const __amdgpu_buffer_rsrc_t rout = rsrc_of(sg.out + u.b_first * sg.out_bstride);
#pragma unroll
    for (int i = 0; i < R; ++i)
      if ((uint32_t)i < sg.r)
        bst16(rout, u.voff_out, (uint32_t)(i * sg.out_sstride),
              make_uint4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]));
#else
#pragma unroll
    for (int i = 0; i < R; ++i)
      if ((uint32_t)i < sg.r)
        st16<NT>(u.pout + (uint64_t)i * sg.out_sstride,
                 make_uint4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]));
#endif
  }
}

template <int KC, int R, bool NT>
__global__ void __launch_bounds__(256, MEMO_EC_MAC_WAVES) gf_mac_kernel(const MacLaunch L) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_tab[];
  uint32_t sid;
  uint64_t tile;
  if (!seg_tile(L, sid, tile)) return;
  mac_tile<KC, R, NT>(L.seg[sid], tile, s_tab);
}

// ------------------------------------------------------------- decode rows
// One wave per block: Gauss-Jordan on [A | I] in LDS, A = generator rows of
// the k survivors; then rows_b[r] = C[lost[r]] * A^-1.  Lane l owns columns
// l and l+64 of the augmented k x 2k matrix.  The field arithmetic uses the
// LDS log/antilog image.  Optionally emits the block's product-table image
// (R x kpad coefficients) for gf_mac_kernel.
__device__ __forceinline__ uint32_t gen_entry(const uint8_t* lg, const uint8_t* ex, uint32_t k,
                                              uint32_t s, uint32_t j) {
  if (s < k) return s == j ? 1u : 0u;
  return gf_inv_t(lg, ex, s ^ j);
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

__global__ void __launch_bounds__(256) decode_rows_kernel(DecodeArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint32_t* s_gf = smem;
  const uint8_t* lg = reinterpret_cast<const uint8_t*>(s_gf);
  const uint8_t* ex = lg + 256;
  stage_gf(s_gf);
  __syncthreads();

  const uint32_t wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const uint64_t b = (uint64_t)blockIdx.x * 4 + wave;
  if (b >= a.n) return;
  const uint32_t k = a.k, e = a.e, total = a.k + a.m;
  const uint32_t W = 2 * k;  // row width
  uint8_t* base = reinterpret_cast<uint8_t*>(smem + 192);
  uint8_t* M = base + wave * (MEMO_EC_MAX_K * 2 * MEMO_EC_MAX_K);
  uint8_t* Rw = base + 4 * (MEMO_EC_MAX_K * 2 * MEMO_EC_MAX_K) + wave * (MEMO_EC_MAX_M * MEMO_EC_MAX_K);
  const uint8_t* sidx = a.surv_idx + b * k;
  const uint8_t* lidx = a.lost_idx + b * e;

  bool bad = false;
  // [A | I]
  for (uint32_t r = 0; r < k; ++r) {
    const uint32_t s = sidx[r];
    bad |= s >= total;
    for (uint32_t col = lane; col < W; col += 64) {
      uint32_t v;
      if (col < k) v = s < total ? gen_entry(lg, ex, k, s, col) : 0u;
      else v = (col - k) == r ? 1u : 0u;
      M[r * W + col] = (uint8_t)v;
    }
  }
  wave_sync();

  for (uint32_t c = 0; c < k && !bad; ++c) {
    // pivot: first row >= c with a nonzero entry in column c
    const uint32_t pv = (lane < k && lane >= c) ? M[lane * W + c] : 0u;
    const uint64_t mask = __ballot(pv != 0);
    if (mask == 0) {
      bad = true;
      break;
    }
    const uint32_t p = (uint32_t)__builtin_ctzll(mask);
    if (p != c) {
      for (uint32_t col = lane; col < W; col += 64) {
        const uint8_t t = M[c * W + col];
        M[c * W + col] = M[p * W + col];
        M[p * W + col] = t;
      }
      wave_sync();
    }
    const uint32_t iv = gf_inv_t(lg, ex, M[c * W + c]);
    __builtin_amdgcn_wave_barrier();
    for (uint32_t col = lane; col < W; col += 64)
      M[c * W + col] = (uint8_t)gf_mul_t(lg, ex, iv, M[c * W + col]);
    wave_sync();
    for (uint32_t rr = 0; rr < k; ++rr) {
      if (rr == c) continue;
      const uint32_t f = M[rr * W + c];
      wave_sync();
      if (f) {
        for (uint32_t col = lane; col < W; col += 64)
          M[rr * W + col] ^= (uint8_t)gf_mul_t(lg, ex, f, M[c * W + col]);
      }
      wave_sync();
    }
  }

  // rows[r][j] = XOR_t C[lost[r]][t] * Inv[t][j]; lane j (< k).
  for (uint32_t r = 0; r < e; ++r) {
    const uint32_t l = lidx[r];
    const bool lbad = bad || l >= total;
    if (lane < k) {
      uint32_t acc = 0;
      if (!lbad)
        for (uint32_t t = 0; t < k; ++t)
          acc ^= gf_mul_t(lg, ex, gen_entry(lg, ex, k, l, t), M[t * W + k + lane]);
      Rw[r * k + lane] = (uint8_t)acc;
    }
    if (lbad) bad = true;
  }
  wave_sync();
  if (bad) {  // invalid pattern: zero rows (zero output) + deferred error
    for (uint32_t t = lane; t < e * k; t += 64) Rw[t] = 0;
    wave_sync();
    if (lane == 0 && a.status) atomicOr(a.status, 1u);
  }
  if (a.rows)
    for (uint32_t t = lane; t < e * k; t += 64) a.rows[b * (uint64_t)e * k + t] = Rw[t];
  if (a.tab) {
    uint32_t* dst = a.tab + b * (uint64_t)a.R * a.kpad * 8;
    const uint32_t n = a.R * a.kpad * 8;
    for (uint32_t t = lane; t < n; t += 64) {
      const uint32_t q = t & 7, cidx = t >> 3;
      const uint32_t i = cidx / a.kpad, j = cidx - i * a.kpad;
      const uint32_t c = (i < e && j < k) ? Rw[i * k + j] : 0u;
      dst[t] = table_dword(lg, ex, c, q);
    }
  }
}

// Register-resident variant for k <= K (K in {4, 8, 10, 12, 16, 32}): lane l holds
// column l of the K x 2K matrix [A | I] in VGPRs (A padded to K x K with an
// identity block, whose inverse is the identity, so rows/columns >= k never
// mix with the real ones).  Pivot rows and row factors are broadcast with
// v_readlane; each elimination is one independent log/antilog LDS lookup per
// row and lane (no LDS round trip of the matrix, no wave barriers).
template <int K>
__global__ void __launch_bounds__(256) decode_rows_reg_kernel(DecodeArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint32_t* s_gf = smem;
  const uint8_t* lg = reinterpret_cast<const uint8_t*>(s_gf);
  const uint8_t* ex = lg + 256;
  stage_gf(s_gf);
  __syncthreads();

  const uint32_t wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const uint64_t b = (uint64_t)blockIdx.x * 4 + wave;
  if (b >= a.n) return;
  const uint32_t k = a.k, e = a.e, total = a.k + a.m;
  uint8_t* Rw = reinterpret_cast<uint8_t*>(smem + 192) + wave * (MEMO_EC_MAX_M * MEMO_EC_MAX_K);
  const uint8_t* sidx = a.surv_idx + b * k;
  const uint8_t* lidx = a.lost_idx + b * e;

  const bool left = lane < K;
  const uint32_t col = left ? lane : lane - K;  // lanes >= 2K carry copies, unused
  uint32_t m[K];
  bool bad = false;
#pragma unroll
  for (int r = 0; r < K; ++r) {
    if ((uint32_t)r < k) {
      const uint32_t sv = sidx[r];
      bad |= sv >= total;
      if (left) m[r] = (col < k && sv < total) ? gen_entry(lg, ex, k, sv, col) : 0u;
      else m[r] = col == (uint32_t)r ? 1u : 0u;
    } else {
      m[r] = col == (uint32_t)r ? 1u : 0u;  // identity padding, both halves
    }
  }

#ifndef MEMO_EC_DECODE_DIAG_NOGJ  // diagnostic build: skip the elimination (wrong rows)
#pragma unroll
  for (int c = 0; c < K; ++c) {
    if (bad) break;
    // pivot: first row >= c with a nonzero entry in column c (lane c)
    uint32_t pl = K;
#pragma unroll
    for (int r = K - 1; r >= c; --r)
      if (m[r]) pl = r;
    const uint32_t p = __builtin_amdgcn_readlane(pl, c);
    if (p >= (uint32_t)K) {
      bad = true;
      break;
    }
    if (p != (uint32_t)c) {
#pragma unroll
      for (int r = c + 1; r < K; ++r)
        if (p == (uint32_t)r) {
          const uint32_t t = m[c];
          m[c] = m[r];
          m[r] = t;
        }
    }
    const uint32_t piv = __builtin_amdgcn_readlane(m[c], c);
    const uint32_t ilog = 255u - lg[piv];  // log of the pivot's inverse
    const bool nz = m[c] != 0;
    uint32_t lc = lg[m[c]] + ilog;          // log of the normalised entry
    if (lc >= 255) lc -= 255;
    m[c] = nz ? (uint32_t)ex[lc] : 0u;
#pragma unroll
    for (int r = 0; r < K; ++r) {
      if (r == c) continue;
      const uint32_t f = __builtin_amdgcn_readlane(m[r], c);
      if (f) m[r] ^= nz ? (uint32_t)ex[lc + lg[f]] : 0u;
    }
  }
#endif

  // Right half, lane K+j, now holds column j of A^-1: inv[t][j] = m[t].
  for (uint32_t r = 0; r < e; ++r) {
    const uint32_t l = lidx[r];
    const bool lbad = bad || l >= total;
    if (!left && col < k) {
      uint32_t acc = 0;
      if (!lbad) {
        if (l < k) {
#pragma unroll
          for (int t = 0; t < K; ++t)
            if ((uint32_t)t == l) acc = m[t];
        } else {
#pragma unroll
          for (int t = 0; t < K; ++t)
            if ((uint32_t)t < k) acc ^= gf_mul_t(lg, ex, gf_inv_t(lg, ex, l ^ (uint32_t)t), m[t]);
        }
      }
      Rw[r * k + col] = (uint8_t)acc;
    }
    if (lbad) bad = true;
  }
  wave_sync();
  if (bad) {
    for (uint32_t t = lane; t < e * k; t += 64) Rw[t] = 0;
    wave_sync();
    if (lane == 0 && a.status) atomicOr(a.status, 1u);
  }
  if (a.rows)
    for (uint32_t t = lane; t < e * k; t += 64) a.rows[b * (uint64_t)e * k + t] = Rw[t];
  if (a.tab) {
    uint32_t* dst = a.tab + b * (uint64_t)a.R * a.kpad * 8;
    const uint32_t n = a.R * a.kpad * 8;
    for (uint32_t t = lane; t < n; t += 64) {
      const uint32_t q = t & 7, cidx = t >> 3;
      const uint32_t i = cidx / a.kpad, j = cidx - i * a.kpad;
      const uint32_t c = (i < e && j < k) ? Rw[i * k + j] : 0u;
      dst[t] = table_dword(lg, ex, c, q);
    }
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
static hipError_t launch_mac_t(const MacLaunch& L, uint32_t grid, size_t lds, hipStream_t st) {
  hipLaunchKernelGGL((gf_mac_kernel<KC, R, MAC_NT>), dim3(grid), dim3(256), lds, st, L);
  return hipGetLastError();
}

template <int KC>
static hipError_t launch_mac_r(int R, const MacLaunch& L, uint32_t grid, size_t lds,
                               hipStream_t st) {
  switch (R) {
#define MEMO_EC_R(x) \
  case x: return launch_mac_t<KC, x>(L, grid, lds, st);
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

int mac_kchunk(int kin) {
  switch (kin) {
    case 2: case 3: case 4: case 10: case 16: return kin;
    default: return 4;
  }
}

hipError_t launch_mac(int KC, int R, const MacLaunch& L, uint32_t grid, size_t lds,
                      hipStream_t st) {
  switch (KC) {
    case 2: return launch_mac_r<2>(R, L, grid, lds, st);
    case 3: return launch_mac_r<3>(R, L, grid, lds, st);
    case 4: return launch_mac_r<4>(R, L, grid, lds, st);
    case 10: return launch_mac_r<10>(R, L, grid, lds, st);
    case 16: return launch_mac_r<16>(R, L, grid, lds, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_decode_rows(const DecodeArgs& a, hipStream_t st) {
  const uint32_t grid = (uint32_t)((a.n + 3) / 4);
  if (grid == 0) return hipSuccess;
  const size_t lds_reg = 768 + 4 * (size_t)MEMO_EC_MAX_M * MEMO_EC_MAX_K;
  if (a.k <= 4 && !MEMO_EC_DECODE_LDS) {
    hipLaunchKernelGGL(decode_rows_reg_kernel<4>, dim3(grid), dim3(256), lds_reg, st, a);
  } else if (a.k <= 8 && !MEMO_EC_DECODE_LDS) {
    hipLaunchKernelGGL(decode_rows_reg_kernel<8>, dim3(grid), dim3(256), lds_reg, st, a);
  } else if (a.k <= 10 && !MEMO_EC_DECODE_LDS) {  // RS(10,m): no padding steps
    hipLaunchKernelGGL(decode_rows_reg_kernel<10>, dim3(grid), dim3(256), lds_reg, st, a);
  } else if (a.k <= 12 && !MEMO_EC_DECODE_LDS) {
    hipLaunchKernelGGL(decode_rows_reg_kernel<12>, dim3(grid), dim3(256), lds_reg, st, a);
  } else if (a.k <= 16 && !MEMO_EC_DECODE_LDS) {
    hipLaunchKernelGGL(decode_rows_reg_kernel<16>, dim3(grid), dim3(256), lds_reg, st, a);
  } else if (a.k <= 32 && !MEMO_EC_DECODE_LDS) {
    hipLaunchKernelGGL(decode_rows_reg_kernel<32>, dim3(grid), dim3(256), lds_reg, st, a);
  } else {
    const size_t lds = 768 + 4 * (size_t)MEMO_EC_MAX_K * 2 * MEMO_EC_MAX_K +
                       4 * (size_t)MEMO_EC_MAX_M * MEMO_EC_MAX_K;
    hipLaunchKernelGGL(decode_rows_kernel, dim3(grid), dim3(256), lds, st, a);
  }
  return hipGetLastError();
}

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

const uint8_t* host_gf_log() { return kGfHost.log; }
const uint8_t* host_gf_exp() { return kGfHost.exp; }

}  // namespace memo_ec
