// ec_kernels.hip -- gfx950 kernels of the block erasure codec.
//
// Hot path: gf_mac_kernel, the batched GF(2^8) multiply-accumulate
//   out[b][i][x] = XOR_j coef_b[i][j] * in[b][j][x]
// that is RS encode (coef = the Cauchy parity rows, shared by every block)
// and RS rebuild (coef = per-block decode rows from decode_rows_kernel).
// It replaces the replication byte movement of Paxos::Details::
// send_immutable_block / _fetch / _rebalance (src/memo/model/doughnut/
// consensus/Paxos.cc:315-391, 486-519, 1012-1246); see DESIGN.md.
//
// Design:
//  * HBM-bound streaming: each lane owns 16-byte columns of a block and loads
//    the same 16 bytes of every input shard (dwordx4, a wave reads 1 KiB of
//    one shard per instruction, fully coalesced), G shards x V columns in
//    flight per lane, double-buffered.
//  * Byte-field GF multiply on the VALU, no MFMA: a data byte x is split into
//    3+3+2-bit fields (x>>5, (x>>2)&7, x&3); c*x = T_hi[x>>5] ^ T_mid[(x>>2)&7]
//    ^ T_lo[x&3].  Each table has <= 8 byte entries, so one v_perm_b32 looks
//    up 4 bytes at once; 3 perms + 3-input XORs (v_bitop3_b32) per
//    coefficient per dword.  The field selectors are shared by all outputs.
//  * The GF log/antilog tables and the per-coefficient product tables are
//    staged in LDS at workgroup start (tables read back as wave-broadcast
//    ds_read_b128/b32).
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

__device__ __forceinline__ uint32_t gf_mul_lds(const uint8_t* lg, const uint8_t* ex,
                                               uint32_t a, uint32_t b) {
  return (a && b) ? ex[lg[a] + lg[b]] : 0u;
}
__device__ __forceinline__ uint32_t gf_inv_lds(const uint8_t* lg, const uint8_t* ex,
                                               uint32_t a) {
  return a ? ex[255 - lg[a]] : 0u;
}

// Copy the 768-byte log/antilog image into LDS (192 dwords).
__device__ __forceinline__ void stage_gf(uint32_t* s_gf) {
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&kGf);
  for (int i = threadIdx.x; i < 192; i += blockDim.x) s_gf[i] = src[i];
}

// Coefficient of output row i, input column j of segment `sg` for block b.
__device__ __forceinline__ uint32_t seg_coef(const MacSeg& sg, const uint8_t* lg,
                                             const uint8_t* ex, uint64_t b, uint32_t i,
                                             uint32_t j) {
  if (sg.coef == nullptr)  // systematic Cauchy parity rows: 1 / ((kin+i) ^ j)
    return gf_inv_lds(lg, ex, (sg.kin + i) ^ j);
  return sg.coef[b * sg.coef_bstride + (uint64_t)i * sg.kin + j];
}

// Product-table dword q of coefficient c (layout per coefficient: 8 dwords,
// [mid0 mid1 hi0 hi1 lo - - -]; each dword packs 4 byte entries).
__device__ __forceinline__ uint32_t table_dword(const uint8_t* lg, const uint8_t* ex,
                                                uint32_t c, uint32_t q) {
  uint32_t r = 0;
#pragma unroll
  for (uint32_t e = 0; e < 4; ++e) {
    uint32_t x;
    switch (q) {
      case 0: x = e << 2; break;        // mid entries 0..3
      case 1: x = (e + 4) << 2; break;  // mid entries 4..7
      case 2: x = e << 5; break;        // hi entries 0..3
      case 3: x = (e + 4) << 5; break;  // hi entries 4..7
      default: x = e; break;            // lo entries 0..3
    }
    r |= gf_mul_lds(lg, ex, c, x) << (8 * e);
  }
  return r;
}

// Build nsets x R x kpad coefficient tables for blocks [b_first, b_first+nsets).
// Rows i >= r and columns j >= kin get coefficient 0, i.e. all-zero tables,
// so padded shards contribute nothing whatever bytes their registers hold.
__device__ __forceinline__ void build_tables(const MacSeg& sg, uint32_t* s_tab, const uint8_t* lg,
                                             const uint8_t* ex, uint64_t b_first, uint32_t nsets,
                                             uint32_t R, uint32_t kpad) {
  const uint32_t per_set = R * kpad;
  const uint32_t total = nsets * per_set * 5;
  for (uint32_t t = threadIdx.x; t < total; t += blockDim.x) {
    const uint32_t q = t % 5;
    const uint32_t cidx = t / 5;
    const uint32_t set = cidx / per_set;
    const uint32_t rem = cidx - set * per_set;
    const uint32_t i = rem / kpad, j = rem - i * kpad;
    const uint32_t c = (i < sg.r && j < sg.kin) ? seg_coef(sg, lg, ex, b_first + set, i, j) : 0u;
    s_tab[cidx * 8 + q] = table_dword(lg, ex, c, q);
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

// acc ^= coef * x for 4 dwords (16 bytes).
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
  pl = __builtin_amdgcn_perm(t.lo, t.lo, s.lo);
  pm = __builtin_amdgcn_perm(t.m1, t.m0, s.mid);
  ph = __builtin_amdgcn_perm(t.h1, t.h0, s.hi);
}

// acc[i] ^= coef(i, j0 + g) * d[g] for the KC shards of one chunk.  Shards
// are taken in pairs so that 6 partial products + the accumulator fold with
// three 3-input XORs (v_bitop3_b32: 1.5 per coefficient).  Branch-free:
// padded rows/shards have all-zero tables.
template <int KC, int R, int V>
__device__ __forceinline__ void mac_chunk(uint32_t (&acc)[R][V][4], const uint4 (&d)[KC][V],
                                          const uint32_t* const (&tabv)[V], uint32_t kpad,
                                          uint32_t j0) {
#pragma unroll
  for (int g = 0; g < KC; g += 2) {
    constexpr int dummy = 0;
    (void)dummy;
    const bool two = g + 1 < KC;
    Sel sa[V][4], sb[V][4];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      sa[v][0] = make_sel(d[g][v].x);
      sa[v][1] = make_sel(d[g][v].y);
      sa[v][2] = make_sel(d[g][v].z);
      sa[v][3] = make_sel(d[g][v].w);
      if (two) {
        sb[v][0] = make_sel(d[g + 1][v].x);
        sb[v][1] = make_sel(d[g + 1][v].y);
        sb[v][2] = make_sel(d[g + 1][v].z);
        sb[v][3] = make_sel(d[g + 1][v].w);
      }
    }
#pragma unroll
    for (int i = 0; i < R; ++i) {
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const uint32_t* tp = tabv[v] + (i * kpad + j0 + g) * 8;
        const Tab ta = read_tab(tp);
        if (two) {
          const Tab tb = read_tab(tp + 8);
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            uint32_t al, am, ah, bl, bm, bh;
            lookups(sa[v][w], ta, al, am, ah);
            lookups(sb[v][w], tb, bl, bm, bh);
            const uint32_t x = xor3(acc[i][v][w], al, am);
            const uint32_t y = xor3(ah, bl, bm);
            acc[i][v][w] = xor3(x, y, bh);
          }
        } else {
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            uint32_t al, am, ah;
            lookups(sa[v][w], ta, al, am, ah);
            acc[i][v][w] = xor3(acc[i][v][w], al, am) ^ ah;
          }
        }
      }
    }
  }
}

// One work tile of 256*V column-units; unit = one 16-byte column of one
// block.  `flat`: units numbered across blocks (u = b*C + c); otherwise a
// tile lies inside one block (tiles_per_block tiles per block).
template <int KC, int R, int V, bool SHARED, bool NT>
__device__ __forceinline__ void mac_tile(const MacSeg& sg, uint64_t tile, const uint32_t* s_tab,
                                         uint64_t b_first, uint32_t kpad) {
  const uint32_t tid = threadIdx.x;
  const uint32_t C = sg.chunks;
  const uint32_t kin = sg.kin;
  const uint64_t total = sg.n * (uint64_t)C;

  const uint8_t* pin[V];
  uint8_t* pout[V];
  bool valid[V];
  const uint32_t* tabv[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    uint64_t b, c;
    if (sg.flat) {
      uint64_t u = tile * (uint64_t)(256 * V) + (uint64_t)v * 256 + tid;
      valid[v] = u < total;
      if (!valid[v]) u = total - 1;
      b = u / C;
      c = u - b * C;
    } else {
      const uint64_t bt = tile / sg.tiles_per_block;
      const uint64_t t = tile - bt * sg.tiles_per_block;
      c = t * (uint64_t)(256 * V) + (uint64_t)v * 256 + tid;
      b = bt;
      valid[v] = c < C;
      if (!valid[v]) c = C - 1;
    }
    pin[v] = sg.in + b * sg.in_bstride + c * 16;
    pout[v] = sg.out + b * sg.out_bstride + c * 16;
    tabv[v] = SHARED ? s_tab : s_tab + (uint32_t)(b - b_first) * (R * kpad * 8);
  }

  uint32_t acc[R][V][4];
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int v = 0; v < V; ++v)
#pragma unroll
      for (int w = 0; w < 4; ++w) acc[i][v][w] = 0;

  if (kin == KC) {
    // Hot path (kin specialised): every load unconditional, so the compiler
    // issues all KC loads up front and waits with counted vmcnt per pair.
    uint4 d[KC][V];
#pragma unroll
    for (int g = 0; g < KC; ++g)
#pragma unroll
      for (int v = 0; v < V; ++v) d[g][v] = ld16<NT>(pin[v] + (uint64_t)g * sg.in_sstride);
    mac_chunk<KC, R, V>(acc, d, tabv, kpad, 0);
  } else {
    for (uint32_t j0 = 0; j0 < kin; j0 += KC) {
      uint4 d[KC][V];
#pragma unroll
      for (int g = 0; g < KC; ++g)
        if (j0 + g < kin)
#pragma unroll
          for (int v = 0; v < V; ++v)
            d[g][v] = ld16<NT>(pin[v] + (uint64_t)(j0 + g) * sg.in_sstride);
      mac_chunk<KC, R, V>(acc, d, tabv, kpad, j0);
    }
  }

#pragma unroll
  for (int i = 0; i < R; ++i) {
    if ((uint32_t)i < sg.r) {
#pragma unroll
      for (int v = 0; v < V; ++v)
        if (valid[v])
          st16<NT>(pout[v] + (uint64_t)i * sg.out_sstride,
                   make_uint4(acc[i][v][0], acc[i][v][1], acc[i][v][2], acc[i][v][3]));
    }
  }
}

template <int KC, int R, int V, bool SHARED, bool NT>
__global__ void __launch_bounds__(256) gf_mac_kernel(const MacLaunch L) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint32_t* s_gf = smem;          // 768 B log/antilog
  uint32_t* s_tab = smem + 192;   // product tables
  const uint8_t* lg = reinterpret_cast<const uint8_t*>(s_gf);
  const uint8_t* ex = lg + 256;

  // Segment of this workgroup (uniform).
  const uint32_t wg = blockIdx.x;
  uint32_t sid = 0;
  for (uint32_t s = 1; s < L.nseg; ++s)
    if (wg >= L.seg[s].wg_begin) sid = s;
  const MacSeg& sg = L.seg[sid];
  const uint32_t wg_local = wg - sg.wg_begin;
  const uint32_t kpad = (sg.kin + KC - 1) / KC * KC;

  stage_gf(s_gf);
  __syncthreads();

  // Contiguous tile range per workgroup: neighbouring tiles share blocks,
  // so per-block tables are rebuilt only when the block set changes.
  const uint64_t per = (sg.tiles + sg.wgs - 1) / sg.wgs;
  const uint64_t t0 = (uint64_t)wg_local * per;
  uint64_t t1 = t0 + per;
  if (t1 > sg.tiles) t1 = sg.tiles;

  if constexpr (SHARED) {
    build_tables(sg, s_tab, lg, ex, 0, 1, R, kpad);
    __syncthreads();
    for (uint64_t tile = t0; tile < t1; ++tile)
      mac_tile<KC, R, V, true, NT>(sg, tile, s_tab, 0, kpad);
  } else {
    uint64_t have_first = ~0ull, have_last = 0;
    for (uint64_t tile = t0; tile < t1; ++tile) {
      uint64_t b_first, b_last;
      if (sg.flat) {
        const uint64_t u0 = tile * (uint64_t)(256 * V);
        uint64_t u1 = u0 + 256 * V - 1;
        const uint64_t total = sg.n * (uint64_t)sg.chunks;
        if (u1 >= total) u1 = total - 1;
        b_first = u0 / sg.chunks;
        b_last = u1 / sg.chunks;
      } else {
        b_first = b_last = tile / sg.tiles_per_block;
      }
      if (b_first != have_first || b_last != have_last) {
        __syncthreads();  // previous tiles' table reads are done
        build_tables(sg, s_tab, lg, ex, b_first, (uint32_t)(b_last - b_first + 1), R, kpad);
        __syncthreads();
        have_first = b_first;
        have_last = b_last;
      }
      mac_tile<KC, R, V, false, NT>(sg, tile, s_tab, b_first, kpad);
    }
  }
}

// ------------------------------------------------------------- decode rows
// One wave per block: Gauss-Jordan on [A | I] in LDS, A = generator rows of
// the k survivors; then rows_b[r] = C[lost[r]] * A^-1.  Lane l owns columns
// l and l+64 of the augmented k x 2k matrix.  The field arithmetic uses the
// LDS log/antilog image.
__device__ __forceinline__ uint32_t gen_entry(const uint8_t* lg, const uint8_t* ex, uint32_t k,
                                              uint32_t s, uint32_t j) {
  if (s < k) return s == j ? 1u : 0u;
  return gf_inv_lds(lg, ex, s ^ j);
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
  uint8_t* M = reinterpret_cast<uint8_t*>(smem + 192) + wave * (MEMO_EC_MAX_K * 2 * MEMO_EC_MAX_K);
  const uint8_t* sidx = a.surv_idx + b * k;
  const uint8_t* lidx = a.lost_idx + b * e;
  uint8_t* rows = a.rows + b * (uint64_t)e * k;

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
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");

  for (uint32_t c = 0; c < k && !bad; ++c) {
    // pivot: first row >= c with a nonzero entry in column c
    const uint32_t pv = (lane < k && lane >= c) ? M[lane * W + c] : 0u;
    const uint64_t mask = __ballot(pv != 0);
    if (mask == 0) { bad = true; break; }
    const uint32_t p = (uint32_t)__builtin_ctzll(mask);
    if (p != c) {
      for (uint32_t col = lane; col < W; col += 64) {
        const uint8_t t = M[c * W + col];
        M[c * W + col] = M[p * W + col];
        M[p * W + col] = t;
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    const uint32_t iv = gf_inv_lds(lg, ex, M[c * W + c]);
    __builtin_amdgcn_wave_barrier();
    for (uint32_t col = lane; col < W; col += 64)
      M[c * W + col] = (uint8_t)gf_mul_lds(lg, ex, iv, M[c * W + col]);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    for (uint32_t rr = 0; rr < k; ++rr) {
      if (rr == c) continue;
      const uint32_t f = M[rr * W + c];
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      if (f) {
        for (uint32_t col = lane; col < W; col += 64)
          M[rr * W + col] ^= (uint8_t)gf_mul_lds(lg, ex, f, M[c * W + col]);
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
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
          acc ^= gf_mul_lds(lg, ex, gen_entry(lg, ex, k, l, t), M[t * W + k + lane]);
      rows[r * k + lane] = (uint8_t)acc;
    }
    if (lbad) bad = true;
  }
  if (bad && lane == 0 && a.status) atomicOr(a.status, 1u);
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

// ------------------------------------------------------------- launchers
template <int KC, int R, bool SHARED>
static hipError_t launch_mac_t(const MacLaunch& L, uint32_t grid, size_t lds, hipStream_t st) {
  hipLaunchKernelGGL((gf_mac_kernel<KC, R, MAC_V, SHARED, MAC_NT>), dim3(grid), dim3(256), lds, st,
                     L);
  return hipGetLastError();
}

template <int KC, bool SHARED>
static hipError_t launch_mac_r(int R, const MacLaunch& L, uint32_t grid, size_t lds,
                               hipStream_t st) {
  switch (R) {
#define MEMO_EC_R(x) \
  case x: return launch_mac_t<KC, x, SHARED>(L, grid, lds, st);
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

template <bool SHARED>
static hipError_t launch_mac_k(int KC, int R, const MacLaunch& L, uint32_t grid, size_t lds,
                               hipStream_t st) {
  switch (KC) {
    case 2: return launch_mac_r<2, SHARED>(R, L, grid, lds, st);
    case 3: return launch_mac_r<3, SHARED>(R, L, grid, lds, st);
    case 4: return launch_mac_r<4, SHARED>(R, L, grid, lds, st);
    case 10: return launch_mac_r<10, SHARED>(R, L, grid, lds, st);
    case 16: return launch_mac_r<16, SHARED>(R, L, grid, lds, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_mac(int KC, int R, bool shared, const MacLaunch& L, uint32_t grid, size_t lds,
                      hipStream_t st) {
  return shared ? launch_mac_k<true>(KC, R, L, grid, lds, st)
                : launch_mac_k<false>(KC, R, L, grid, lds, st);
}

hipError_t launch_decode_rows(const DecodeArgs& a, hipStream_t st) {
  const uint32_t grid = (uint32_t)((a.n + 3) / 4);
  if (grid == 0) return hipSuccess;
  const size_t lds = 768 + 4 * (size_t)MEMO_EC_MAX_K * 2 * MEMO_EC_MAX_K;
  hipLaunchKernelGGL(decode_rows_kernel, dim3(grid), dim3(256), lds, st, a);
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
