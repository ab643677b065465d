// memo_ec.cpp -- C ABI of the gfx950 erasure codec (include/memo_ec.h).
//
// Host side of the drop-in boundary: validates arguments, plans the
// multiply-accumulate launch (ec_kernels.hip), runs device-resident calls
// asynchronously on the ctx stream and host-memory calls through a 3-slot
// HtoD -> kernel -> DtoH stream pipeline.  No CPU fallback exists:
// every byte of parity/rebuild output is produced by the HIP kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/memo_ec.h"
#include "ec_kernels.h"

using namespace memo_ec;

// Tuning of one ctx (memo_ec_option; defaults from the environment, read
// once at memo_ec_ctx_create, so no call reads the environment).
struct memo_ec_opts {
  int rebuild_path = -1;                  // -1 auto, 0 decode rows + MAC, 1 fused
  size_t fused_max_bytes = 256ull << 20;  // auto: fused up to this many survivor bytes
  size_t zc_max_bytes = 4ull << 20;       // host calls up to this many bytes: zero-copy
  size_t pipe_bytes = 64ull << 20;        // host pipeline batch
  int copy_threads = 0;                   // pageable bounce copy threads (0: all)
  uint64_t max_launch_tiles = 0;          // tiles per MAC launch (0: 31-bit grid)
  uint64_t xcd_min_tiles = 65536;         // XCD-contiguous order from this many tiles
  uint64_t decode_wide_max = 65536;       // column-per-lane decode up to this many blocks
  int decode_exact = 1;
  int decode_stage = 0;
  uint64_t image_min_tiles = 1;           // rows path: HBM table images from this many whole tiles
  uint64_t image_min_coefs = 40;          //   per shard and this many coefficients (R x kpad)
  int decode_overlap = 1;                 // mixed rebuilds: later decodes on a side stream
};

struct memo_ec_ctx {
  int device = 0;
  memo_ec_opts opt;
  hipStream_t own = nullptr;      // ctx stream
  hipStream_t stream = nullptr;   // stream MEMO_EC_DEVICE work goes to
  // host pipeline: copy-in / compute / copy-out streams, a ring of kSlots
  // batch slots, and per-slot events chaining the three stages
  hipStream_t sh = nullptr, sk = nullptr, sd = nullptr;
  hipEvent_t ev_h[3] = {}, ev_k[3] = {}, ev_d[3] = {};
  // orders work after what is pending on `stream` (stream switches; host
  // rebuilds, whose decode rows share d_tabs with device rebuilds)
  hipEvent_t ev_order = nullptr;
  uint32_t* d_status = nullptr;   // deferred device errors (bit 0: singular)
  uint32_t* h_status = nullptr;   // pinned copy of d_status for host-memory calls
  // side stream for a mixed rebuild's later decodes (overlapping earlier
  // MACs) and its events, created on first use
  hipStream_t side = nullptr;
  std::vector<hipEvent_t> side_ev;
  uint32_t* d_tabs = nullptr;     // rebuild scratch: per-block decode rows
  size_t tabs_cap = 0;            // bytes
  struct TabEntry {
    int k, m, R, kpad;
    uint32_t* dev;
  };
  std::vector<TabEntry> enc_tabs;  // cached encode images per (k, m, R, kpad)
  struct Lw0Entry {
    int k, m;
    uint32_t* dev;
  };
  std::vector<Lw0Entry> lw0_tabs;  // cached LW0 tables per (k, m) (decode kernels)
  struct PatEntry {
    int k, m, R, kpad;
    std::vector<uint8_t> key;  // surv_idx (k) || lost_idx (e)
    uint32_t* dev;
    uint64_t used;
    uint64_t call;             // API call that last used it (never evicted within it)
  };
  std::vector<PatEntry> pat_tabs;  // cached uniform-rebuild table images
  uint64_t pat_clock = 0;
  uint64_t call_seq = 0;           // API calls that form pattern tables
  // host pipeline: device slots and pinned bounce buffers
  uint8_t* d_slot[3] = {nullptr, nullptr, nullptr};
  size_t slot_cap = 0;
  uint8_t* h_slot[3] = {nullptr, nullptr, nullptr};
  size_t hslot_cap = 0;
  int deferred = 0;
};

namespace {

constexpr size_t kLdsBudget = 48 * 1024;  // table LDS per workgroup (flat mapping)
// Largest shard (a documented limit: 2^32 bytes, far above any block memo
// stores; the kernels' column indices are 32-bit).
constexpr size_t kMaxShard = (size_t)1 << 32;

int hip_rc(hipError_t e) {
  if (e == hipSuccess) return MEMO_EC_OK;
  if (e == hipErrorOutOfMemory) return MEMO_EC_ENOMEM;
  return MEMO_EC_EHIP;
}
#define HIPCHK(x)                       \
  do {                                  \
    hipError_t _e = (x);                \
    if (_e != hipSuccess) return hip_rc(_e); \
  } while (0)

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != d) (void)hipSetDevice(d);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// Bounds of each memo_ec_option (set_option refuses values outside them).
bool set_opt(memo_ec_opts& o, int opt, int64_t v) {
  switch (opt) {
    case MEMO_EC_OPT_REBUILD_PATH:
      if (v < -1 || v > 1) return false;
      o.rebuild_path = (int)v;
      return true;
    case MEMO_EC_OPT_FUSED_MAX_BYTES:
      if (v < 0) return false;
      o.fused_max_bytes = (size_t)v;
      return true;
    case MEMO_EC_OPT_ZERO_COPY_BYTES:
      if (v < 0) return false;
      o.zc_max_bytes = (size_t)v;
      return true;
    case MEMO_EC_OPT_PIPE_BYTES:
      if (v < (1 << 20) || v > (int64_t(4096) << 20)) return false;
      o.pipe_bytes = (size_t)v;
      return true;
    case MEMO_EC_OPT_COPY_THREADS:
      if (v < 0 || v > 256) return false;
      o.copy_threads = (int)v;
      return true;
    case MEMO_EC_OPT_MAX_LAUNCH_TILES:
      if (v < 0) return false;
      o.max_launch_tiles = (uint64_t)v;
      return true;
    case MEMO_EC_OPT_XCD_MIN_TILES:
      if (v < 0) return false;
      o.xcd_min_tiles = (uint64_t)v;
      return true;
    case MEMO_EC_OPT_DECODE_WIDE_MAX:
      if (v < 0) return false;
      o.decode_wide_max = (uint64_t)v;
      return true;
    case MEMO_EC_OPT_DECODE_EXACT:
      if (v < 0 || v > 1) return false;
      o.decode_exact = (int)v;
      return true;
    case MEMO_EC_OPT_DECODE_STAGE:
      if (v < 0 || v > 1) return false;
      o.decode_stage = (int)v;
      return true;
    case MEMO_EC_OPT_IMAGE_MIN_TILES:
      if (v < 0) return false;
      o.image_min_tiles = (uint64_t)v;
      return true;
    case MEMO_EC_OPT_IMAGE_MIN_COEFS:
      if (v < 0) return false;
      o.image_min_coefs = (uint64_t)v;
      return true;
    case MEMO_EC_OPT_DECODE_OVERLAP:
      if (v < 0 || v > 1) return false;
      o.decode_overlap = (int)v;
      return true;
    default:
      return false;
  }
}

bool get_opt(const memo_ec_opts& o, int opt, int64_t* v) {
  switch (opt) {
    case MEMO_EC_OPT_REBUILD_PATH: *v = o.rebuild_path; return true;
    case MEMO_EC_OPT_FUSED_MAX_BYTES: *v = (int64_t)o.fused_max_bytes; return true;
    case MEMO_EC_OPT_ZERO_COPY_BYTES: *v = (int64_t)o.zc_max_bytes; return true;
    case MEMO_EC_OPT_PIPE_BYTES: *v = (int64_t)o.pipe_bytes; return true;
    case MEMO_EC_OPT_COPY_THREADS: *v = o.copy_threads; return true;
    case MEMO_EC_OPT_MAX_LAUNCH_TILES: *v = (int64_t)o.max_launch_tiles; return true;
    case MEMO_EC_OPT_XCD_MIN_TILES: *v = (int64_t)o.xcd_min_tiles; return true;
    case MEMO_EC_OPT_DECODE_WIDE_MAX: *v = (int64_t)o.decode_wide_max; return true;
    case MEMO_EC_OPT_DECODE_EXACT: *v = o.decode_exact; return true;
    case MEMO_EC_OPT_DECODE_STAGE: *v = o.decode_stage; return true;
    case MEMO_EC_OPT_IMAGE_MIN_TILES: *v = (int64_t)o.image_min_tiles; return true;
    case MEMO_EC_OPT_IMAGE_MIN_COEFS: *v = (int64_t)o.image_min_coefs; return true;
    case MEMO_EC_OPT_DECODE_OVERLAP: *v = o.decode_overlap; return true;
    default: return false;
  }
}

// Defaults of a new ctx from the environment (once per memo_ec_ctx_create).
// The variables keep the meanings they had when each call read them:
// MEMO_EC_REBUILD_FUSED any nonzero value forces the fused path (negative:
// auto), MEMO_EC_COPY_THREADS=0 copies on the calling thread only.
// Unparsable or out-of-range values are ignored with a warning on stderr.
void read_env_options(memo_ec_opts& o) {
  struct Env {
    const char* name;
    int opt;
    int shift;  // value << shift (MB / KB variables)
  };
  static const Env kEnv[] = {
      {"MEMO_EC_REBUILD_FUSED", MEMO_EC_OPT_REBUILD_PATH, 0},
      {"MEMO_EC_FUSED_MAX_MB", MEMO_EC_OPT_FUSED_MAX_BYTES, 20},
      {"MEMO_EC_ZC_KB", MEMO_EC_OPT_ZERO_COPY_BYTES, 10},
      {"MEMO_EC_PIPE_MB", MEMO_EC_OPT_PIPE_BYTES, 20},
      {"MEMO_EC_COPY_THREADS", MEMO_EC_OPT_COPY_THREADS, 0},
      {"MEMO_EC_MAX_LAUNCH_TILES", MEMO_EC_OPT_MAX_LAUNCH_TILES, 0},
      {"MEMO_EC_XCD_MIN_TILES", MEMO_EC_OPT_XCD_MIN_TILES, 0},
      {"MEMO_EC_DECODE_WIDE_MAX", MEMO_EC_OPT_DECODE_WIDE_MAX, 0},
      {"MEMO_EC_DECODE_EXACT", MEMO_EC_OPT_DECODE_EXACT, 0},
      {"MEMO_EC_DECODE_STAGE", MEMO_EC_OPT_DECODE_STAGE, 0},
      {"MEMO_EC_IMAGE_MIN_TILES", MEMO_EC_OPT_IMAGE_MIN_TILES, 0},
      {"MEMO_EC_IMAGE_MIN_COEFS", MEMO_EC_OPT_IMAGE_MIN_COEFS, 0},
      {"MEMO_EC_DECODE_OVERLAP", MEMO_EC_OPT_DECODE_OVERLAP, 0},
  };
  for (const Env& e : kEnv) {
    const char* p = std::getenv(e.name);
    if (!p || !*p) continue;
    char* end = nullptr;
    long long v = std::strtoll(p, &end, 10);
    bool ok = end != p && v <= (LLONG_MAX >> e.shift) && v >= -(LLONG_MAX >> e.shift);
    if (ok) {
      if (e.opt == MEMO_EC_OPT_REBUILD_PATH) v = v < 0 ? -1 : v != 0 ? 1 : 0;
      if (e.opt == MEMO_EC_OPT_COPY_THREADS && v == 0) v = 1;
      ok = set_opt(o, e.opt, (int64_t)v * ((int64_t)1 << e.shift));
    }
    if (!ok) std::fprintf(stderr, "libmemo_ec: ignoring %s=%s (not a valid value)\n", e.name, p);
  }
}

// A call moves n * per bytes of caller buffers.  Products that overflow, or
// pass 2^50 bytes (1 PiB: beyond any device or host memory), are refused
// with MEMO_EC_ERANGE before scratch or grids are sized from them.
constexpr uint64_t kMaxCallBytes = 1ull << 50;
bool too_big(size_t n, size_t per) {
  uint64_t b = 0;
  return __builtin_mul_overflow((uint64_t)n, (uint64_t)per, &b) || b > kMaxCallBytes;
}

int check_km(int k, int m) {
  if (k < 1 || m < 0) return MEMO_EC_EINVAL;
  if (k > MEMO_EC_MAX_K || m > MEMO_EC_MAX_M) return MEMO_EC_ERANGE;
  if (k + m > 256) return MEMO_EC_EINVAL;
  return MEMO_EC_OK;
}

// One segment of a MAC launch plus the compile-time bounds it needs.
struct Plan {
  MacSeg seg{};
  int KC = 4, R = 1;
  int mode = MAC_ENCODE;  // MacMode: encode image / decode rows in HBM / fused decode
  size_t lds = 0;         // LDS bytes of this segment's table sets (+ decode workspace)
};

uint32_t kpad_of(uint32_t kin, int KC) { return (kin + KC - 1) / KC * KC; }

// Blocks a 256-column tile can touch (flat mapping).
uint64_t sets_per_tile(uint64_t C) { return (MAC_TILE - 1 + C - 1) / C + 1; }

Plan plan_segment(uint32_t kin, uint32_t r, size_t S, size_t n, const uint8_t* in,
                  uint64_t in_bs, uint64_t in_ss, uint8_t* out, uint64_t out_bs, uint64_t out_ss,
                  const uint32_t* tab, uint64_t tab_bs_dw, int KC, int R,
                  const uint8_t* coef = nullptr, uint64_t coef_bs = 0, uint32_t coef_rows = 0,
                  bool fused = false) {
  Plan p;
  p.KC = KC;
  p.R = R;
  // fused: per-block coefficients (coef_bs = e * k) the tile decodes itself
  p.mode = fused ? MAC_FUSED : coef ? MAC_ROWS : MAC_ENCODE;
  const bool per_coef = p.mode != MAC_ENCODE;
  MacSeg& s = p.seg;
  s.in = in; s.out = out; s.tab = tab;
  s.in_bstride = in_bs; s.in_sstride = in_ss;
  s.out_bstride = out_bs; s.out_sstride = out_ss;
  s.tab_bstride = tab_bs_dw;
  s.coef = coef; s.coef_bstride = coef_bs; s.coef_rows = coef_rows;
  s.coef_dense = coef && !fused && coef_bs != 0 && coef_rows == (uint32_t)R &&
                 kin == kpad_of(kin, KC) && coef_bs == (uint64_t)R * kin;
  s.n = n; s.kin = kin; s.r = r;
  s.kpad = kpad_of(kin, KC);
  s.chunks = (uint32_t)(S / 16);
  // LDS per table set: 8-dword images, or (per-coefficient tables: rebuild)
  // 16-B q + 4-B lo per slot plus one pad slot (ec_kernels.hip: put_image)
  const size_t per = (size_t)R * s.kpad;
  const bool soa = per_coef;
  const size_t set_bytes = soa ? (per + 1) * 20 : per * 32;
  const uint64_t C = s.chunks;
  uint64_t sets;
  if (per_coef ? coef_bs == 0 : tab_bs_dw == 0) {  // one table set for every block
    s.flat = 1;
    sets = 1;
  } else if (!per_coef && C >= MAC_TILE && sets_per_tile(C) * per * 8 > 256u * MAC_TAB_REGS) {
    // per-block table images too large for a tile across two blocks to stage
    // both sets in registers ahead of its shard loads (R x kpad > 64): tiles
    // inside one block
    s.flat = 0;
    sets = 1;
  } else if (sets_per_tile(C) * set_bytes <= kLdsBudget &&
             (!per_coef || sets_per_tile(C) * per <= 256u * MAC_COEF_REGS)) {
    // (the hot path stages at most MAC_COEF_REGS coefficients per lane)
    s.flat = 1;
    sets = sets_per_tile(C);
  } else {
    s.flat = 0;
    sets = 1;
  }
  p.lds = sets * set_bytes;
  s.lo_dw = soa ? (uint32_t)(sets * (per + 1) * 4) : 0u;
  if (fused) {
    // decode workspace: the LDS phases' (chunk loop) or 4 waves' GF copies
    // (wave-local decode on the hot path), whichever the kernel takes
    s.ws_dw = (uint32_t)(p.lds / 4);
    p.lds += std::max<size_t>(dec_ws_bytes((uint32_t)sets, kin, r),
                                 (MAC_TILE / 64) * DEC_WAVE_BYTES);
  }
  if (s.flat) {
    s.tiles = (n * C + MAC_TILE - 1) / MAC_TILE;
    s.tiles_per_block = 0;
  } else {
    s.tiles_per_block = (C + MAC_TILE - 1) / MAC_TILE;
    s.tiles = n * s.tiles_per_block;
  }
  return p;
}

// Largest table LDS of a launch's segments.
size_t lds_of(const std::vector<Plan>& plans) {
  size_t lds = 0;
  for (const auto& p : plans) lds = std::max(lds, p.lds);
  return lds;
}

// Launch planned segments that share KC, R and mode, one tile per
// workgroup: MEMO_EC_MAX_SEGMENTS segments (and < 2^31 workgroups) per
// kernel launch, more segments in further launches back to back.
int launch_plans(const memo_ec_ctx* c, std::vector<Plan>& plans, hipStream_t st) {
  if (plans.empty()) return MEMO_EC_OK;
  const int KC = plans[0].KC, R = plans[0].R, mode = plans[0].mode;
  for (const auto& p : plans)
    if (p.KC != KC || p.R != R || p.mode != mode) return MEMO_EC_EINVAL;
  if (lds_of(plans) > 160 * 1024) return MEMO_EC_ERANGE;
  size_t i = 0;
  while (i < plans.size()) {
    MacLaunch L{};
    L.nseg = 0;
    uint64_t wg = 0;
    size_t lds = 0;
    for (; i < plans.size() && L.nseg < MEMO_EC_MAX_SEGMENTS; ++i) {
      Plan& p = plans[i];
      if (p.seg.tiles == 0) continue;
      const uint64_t begin = (wg + 7) / 8 * 8;  // segments start on an XCD-round boundary
      if (L.nseg && begin + p.seg.tiles > 0x7fffffffull) break;  // next launch
      p.seg.wg_begin = (uint32_t)begin;
      wg = begin + p.seg.tiles;
      lds = std::max(lds, p.lds);
      L.seg[L.nseg++] = p.seg;
    }
    if (wg == 0) continue;
    if (wg > 0x7fffffffull) return MEMO_EC_ERANGE;
    // The XCD-contiguous tile order pays on large grids (C2, 105k
    // workgroups: +4%) and costs a few % on grids of a few 10k.
    uint64_t min_tiles = ~0ull;
    for (uint32_t s = 0; s < L.nseg; ++s) min_tiles = std::min<uint64_t>(min_tiles, L.seg[s].tiles);
    L.xcd = min_tiles >= c->opt.xcd_min_tiles ? 1u : 0u;
    if (int rc = hip_rc(launch_mac(KC, R, mode, L, (uint32_t)wg, lds, st))) return rc;
  }
  return MEMO_EC_OK;
}

// Cached device table image of the Cauchy parity rows of (k, m).
int encode_tables(memo_ec_ctx* ctx, int k, int m, int R, int KC, const uint32_t** out) {
  const int kpad = (int)kpad_of((uint32_t)k, KC);
  for (auto& e : ctx->enc_tabs)
    if (e.k == k && e.m == m && e.R == R && e.kpad == kpad) {
      *out = e.dev;
      return MEMO_EC_OK;
    }
  std::vector<uint8_t> gen((size_t)(k + m) * k);
  if (int rc = memo_ec_generator(k, m, gen.data())) return rc;
  std::vector<uint32_t> img((size_t)R * kpad * 8);
  table_image_host(gen.data() + (size_t)k * k, (uint32_t)m, (uint32_t)k, (uint32_t)R,
                   (uint32_t)kpad, img.data());
  uint32_t* dev = nullptr;
  HIPCHK(hipMalloc(&dev, img.size() * 4));
  hipError_t e = hipMemcpy(dev, img.data(), img.size() * 4, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(dev);
    return hip_rc(e);
  }
  ctx->enc_tabs.push_back({k, m, R, kpad, dev});
  *out = dev;
  return MEMO_EC_OK;
}

// Cached device LW0 table of (k, m) (fused rebuild).
int lw0_table(memo_ec_ctx* ctx, int k, int m, const uint32_t** out) {
  for (auto& e : ctx->lw0_tabs)
    if (e.k == k && e.m == m) {
      *out = e.dev;
      return MEMO_EC_OK;
    }
  uint8_t img[128];
  lw0_host(k, m, img);
  uint32_t* dev = nullptr;
  HIPCHK(hipMalloc(&dev, sizeof img));
  hipError_t e = hipMemcpy(dev, img, sizeof img, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(dev);
    return hip_rc(e);
  }
  ctx->lw0_tabs.push_back({k, m, dev});
  *out = dev;
  return MEMO_EC_OK;
}

// The device rebuild path of a call moving `in_bytes` of survivors:
//  - fused (gf_rebuild_kernel: each tile derives its blocks' decode rows, one
//    launch) for calls up to MEMO_EC_FUSED_MAX_MB (256) MiB: a chip that
//    is not filled twice over wins by the saved launch and rows round trip
//    (one-block degraded reads: 4 KiB 27-30 -> 23 us, 1 MiB 78-88 -> 62-72
//    us, profiles/r02_host_latency_fused_ab.jsonl; 16-256 MiB calls of 4 KiB
//    or 1 MiB blocks 10-30% faster fused, equal at 420 MiB - 1 GiB,
//    profiles/r03_fused_bound_probe.jsonl);
//  - two kernels (decode_coef*/decode_rows_k rows through HBM, then
//    gf_mac_kernel) above: the MAC is ~75% VALU-busy and the fused decode's
//    VALU/LDS work costs more than the decode kernel it removes (C3 1054 vs
//    1012 us, 4 KiB RS(10,4) 1239 vs 1186 us, profiles/r02_rebuild_pmc.md).
// MEMO_EC_OPT_REBUILD_PATH 0/1 forces one path (A/B runs and tests).
bool rebuild_fused(const memo_ec_ctx* c, size_t in_bytes) {
  if (c->opt.rebuild_path >= 0) return c->opt.rebuild_path != 0;
  return in_bytes <= c->opt.fused_max_bytes;
}

int sync_pipeline(memo_ec_ctx* ctx);

// Grows the per-block table scratch.  Earlier rebuilds of this ctx (on its
// current stream or the host pipeline) may still read the old buffer, so
// those streams drain first; other contexts on the device are not waited for.
int ensure_tabs(memo_ec_ctx* ctx, size_t bytes) {
  if (bytes <= ctx->tabs_cap) return MEMO_EC_OK;
  if (ctx->d_tabs) {
    HIPCHK(hipStreamSynchronize(ctx->stream));
    if (int rc = sync_pipeline(ctx)) return rc;
    HIPCHK(hipFree(ctx->d_tabs));
    ctx->d_tabs = nullptr;
    ctx->tabs_cap = 0;
  }
  const size_t cap = std::max<size_t>(bytes, 1 << 20);
  HIPCHK(hipMalloc(&ctx->d_tabs, cap));
  ctx->tabs_cap = cap;
  return MEMO_EC_OK;
}

// The ctx's side stream and at least n events on it (created on first use,
// kept for the ctx's life).
int side_events(memo_ec_ctx* ctx, size_t n) {
  if (!ctx->side) HIPCHK(hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking));
  while (ctx->side_ev.size() < n) {
    hipEvent_t e = nullptr;
    HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ctx->side_ev.push_back(e);
  }
  return MEMO_EC_OK;
}

constexpr int kSlots = 3;

// Pageable <-> pinned bounce copies run on several host threads: one thread
// moves ~10-20 GB/s, below the ~50 GB/s a PCIe Gen5 x16 direction carries.
// The workers are shared by every ctx of the process and started once; the
// calling thread copies a chunk too and helps with queued chunks while it
// waits.  `threads` (the ctx's MEMO_EC_OPT_COPY_THREADS; 0: no cap) caps the
// threads per copy; 1 copies on the calling thread only.
class CopyPool {
 public:
  static CopyPool& get() {
    static CopyPool* p = new CopyPool();  // never destroyed: workers may be blocked at exit
    return *p;
  }
  void copy(void* dst, const void* src, size_t n, int threads) {
    constexpr size_t kChunkMin = 128u << 10;
    size_t nt = std::min<size_t>(workers_ + 1, n / kChunkMin);
    if (threads > 0) nt = std::min<size_t>(nt, (size_t)threads);
    if (nt <= 1) {
      std::memcpy(dst, src, n);
      return;
    }
    const size_t per = (n / nt + 63) & ~(size_t)63;
    Job job;
    std::vector<Chunk> mine;
    for (size_t lo = per; lo < n; lo += per)
      mine.push_back({(char*)dst + lo, (const char*)src + lo, std::min(per, n - lo), &job});
    job.left = mine.size();
    {
      std::lock_guard<std::mutex> g(mu_);
      for (auto& c : mine) q_.push_back(c);
    }
    cv_.notify_all();
    std::memcpy(dst, src, std::min(per, n));
    // help with queued chunks (this copy's or another's) until ours are done
    for (;;) {
      Chunk c;
      {
        std::lock_guard<std::mutex> g(mu_);
        if (q_.empty()) break;
        c = q_.back();
        q_.pop_back();
      }
      run(c);
    }
    std::unique_lock<std::mutex> l(job.m);
    job.cv.wait(l, [&] { return job.left == 0; });
  }

 private:
  struct Job {
    std::mutex m;
    std::condition_variable cv;
    size_t left = 0;
  };
  struct Chunk {
    char* d;
    const char* s;
    size_t n;
    Job* job;
  };
  CopyPool() {
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    workers_ = std::min<unsigned>(7, hw > 1 ? hw - 1 : 0);
    for (unsigned i = 0; i < workers_; ++i) std::thread([this] { worker(); }).detach();
  }
  // The job's owner returns only after taking job->m, which the last runner
  // holds until it has notified: the job outlives every access to it.
  static void run(const Chunk& c) {
    std::memcpy(c.d, c.s, c.n);
    std::lock_guard<std::mutex> g(c.job->m);
    if (--c.job->left == 0) c.job->cv.notify_all();
  }
  void worker() {
    for (;;) {
      Chunk c;
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return !q_.empty(); });
        c = q_.back();
        q_.pop_back();
      }
      run(c);
    }
  }
  unsigned workers_ = 0;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<Chunk> q_;
};

void par_memcpy(const memo_ec_ctx* c, void* dst, const void* src, size_t n) {
  CopyPool::get().copy(dst, src, n, c->opt.copy_threads);
}

int sync_pipeline(memo_ec_ctx* ctx) {
  for (auto st : {ctx->sh, ctx->sk, ctx->sd}) HIPCHK(hipStreamSynchronize(st));
  return MEMO_EC_OK;
}

int ensure_slots(memo_ec_ctx* ctx, size_t dev_bytes, size_t host_bytes) {
  // capacities drop to 0 before reallocating, so a failed allocation is
  // retried by the next call instead of leaving null slots behind a cap
  if (dev_bytes > ctx->slot_cap) {
    if (int rc = sync_pipeline(ctx)) return rc;
    ctx->slot_cap = 0;
    for (auto& p : ctx->d_slot) {
      if (p) HIPCHK(hipFree(p));
      p = nullptr;
    }
    for (auto& p : ctx->d_slot) HIPCHK(hipMalloc(&p, dev_bytes));
    ctx->slot_cap = dev_bytes;
  }
  if (host_bytes > ctx->hslot_cap) {
    if (int rc = sync_pipeline(ctx)) return rc;
    ctx->hslot_cap = 0;
    for (auto& p : ctx->h_slot) {
      if (p) HIPCHK(hipHostFree(p));
      p = nullptr;
    }
    for (auto& p : ctx->h_slot) HIPCHK(hipHostMalloc(&p, host_bytes, hipHostMallocDefault));
    ctx->hslot_cap = host_bytes;
  }
  return MEMO_EC_OK;
}

// Host-memory calls moving at most this many bytes (in + out) run their
// kernels on pinned host memory directly, with no DMA copies: 5-40% less
// time than the copy pipeline up to ~8 MiB of input, more beyond, where the
// pipeline's copy overlap and threaded bounce copies win
// (profiles/r01_zero_copy_probe.jsonl).  The ctx's MEMO_EC_OPT_ZERO_COPY_BYTES
// (0 disables).
size_t zc_max_bytes(const memo_ec_ctx* c) { return c->opt.zc_max_bytes; }

// Largest batch (blocks) one MAC launch takes: tiles must fit a 31-bit grid.
// MEMO_EC_OPT_MAX_LAUNCH_TILES lowers the bound so tests can reach the split
// path without a 2^31-tile batch.
size_t max_blocks_per_launch(const memo_ec_ctx* c, size_t S) {
  uint64_t limit = 0x7fffffffull - MAC_TILE;
  if (c->opt.max_launch_tiles >= 1 && c->opt.max_launch_tiles < limit) limit = c->opt.max_launch_tiles;
  const uint64_t per = (S / 16 + MAC_TILE - 1) / MAC_TILE + 1;
  return (size_t)std::max<uint64_t>(1, limit / per);
}

// Device-resident encode on stream st.
int encode_device(memo_ec_ctx* ctx, int k, int m, size_t S, size_t n, const uint8_t* data,
                  uint8_t* parity, hipStream_t st) {
  const int R = mac_rbound(m), KC = mac_kchunk(k, R);
  const uint32_t* tab = nullptr;
  if (int rc = encode_tables(ctx, k, m, R, KC, &tab)) return rc;
  const size_t step = max_blocks_per_launch(ctx, S);
  for (size_t b0 = 0; b0 < n; b0 += step) {
    const size_t cnt = std::min(step, n - b0);
    std::vector<Plan> plans{plan_segment((uint32_t)k, (uint32_t)m, S, cnt,
                                         data + b0 * (size_t)k * S, (uint64_t)k * S, S,
                                         parity + b0 * (size_t)m * S, (uint64_t)m * S, S, tab, 0,
                                         KC, R)};
    if (int rc = launch_plans(ctx, plans, st)) return rc;
  }
  return MEMO_EC_OK;
}

DecodeArgs decode_args(const memo_ec_ctx* c, int k, int m, int e, size_t n, const uint8_t* surv_idx,
                       const uint8_t* lost_idx, uint8_t* rows, uint32_t* status, const uint32_t* lw0) {
  DecodeArgs a{};
  a.surv_idx = surv_idx;
  a.lost_idx = lost_idx;
  a.rows = rows;
  a.status = status;
  a.n = n;
  a.k = (uint32_t)k;
  a.m = (uint32_t)m;
  a.e = (uint32_t)e;
  a.pitch = 0;
  a.lw0 = lw0;
  a.wide_max = c->opt.decode_wide_max;
  a.exact = c->opt.decode_exact ? 1u : 0u;
  a.stage = c->opt.decode_stage ? 1u : 0u;
  return a;
}

// Rows path: per-block product-table images through HBM (formed by the
// column-per-lane decode beside the rows, then the encode's code over them:
// gf_mac_images_kernel) when a shard holds at least the ctx's
// MEMO_EC_OPT_IMAGE_MIN_TILES whole tiles and its tables are costly to build
// per tile: R x kpad >= MEMO_EC_OPT_IMAGE_MIN_COEFS, or k off the
// straight-line bodies (the chunk loop builds its images one per lane,
// after the barrier).  A block of T tiles builds the same images T times in
// LDS, against one build and R * kpad * 32 bytes of HBM per block here; below
// one tile per shard the images cost more traffic than the build saves
// (4 KiB RS(16,4): a 2 KiB image per 5 KiB of traffic).  Measured with
// tools/image_ab.py: RS(16,4) 128 KiB-4 MiB +2 to +3.6
// points, RS(10,4) / RS(12,4) 40 KiB-4 MiB -0.3 to +2.9 by box, the
// chunk-loop codes +4 to +7; RS(4,2) and RS(6,3) (8 and 18 coefficients)
// -0.6 to +0.1, so they keep their LDS tables.
bool rows_images(const memo_ec_ctx* c, size_t S, int k, int R, int KC) {
  const uint64_t t = c->opt.image_min_tiles;
  if (t == 0 || S / 16 / MAC_TILE < t) return false;  // whole tiles per shard
  return KC != k || (uint64_t)R * kpad_of((uint32_t)k, KC) >= c->opt.image_min_coefs;
}
size_t round256(size_t b) { return (b + 255) & ~(size_t)255; }
// The decode of `a` also forms its rows' table images (R x kpad slots per
// block) at img.
void with_images(DecodeArgs& a, uint32_t* img, int R, int KC) {
  a.img = img;
  a.R = (uint32_t)R;
  a.kpad = kpad_of(a.k, KC);
}
size_t image_bytes(size_t n, int k, int R, int KC) {
  return n * (size_t)R * kpad_of((uint32_t)k, KC) * 32;
}

// Device-resident rebuild on stream st.  Fused (default): one launch of
// gf_rebuild_kernel, whose tiles derive their blocks' decode rows from the
// indices.  Two-kernel: closed-form decode rows (one lane per block) into
// `scratch` (room for rebuild_scratch(...)), then the MAC, which builds each
// block's product tables in LDS from its rows, or (rows_images) reads the
// table images the decode formed beside the rows.  Faults go to `status`.
int rebuild_device(memo_ec_ctx* ctx, int k, int m, size_t S, size_t n, const uint8_t* surv_idx,
                   const uint8_t* surv, const uint8_t* lost_idx, int e, uint8_t* out,
                   bool fused, void* scratch, hipStream_t st, uint32_t* status) {
  const int R = mac_rbound(e), KC = mac_kchunk(k, R);
  const size_t step = max_blocks_per_launch(ctx, S);
  if (fused) {
    const uint32_t* lw0 = nullptr;
    if (int rc = lw0_table(ctx, k, m, &lw0)) return rc;
    for (size_t b0 = 0; b0 < n; b0 += step) {
      const size_t cnt = std::min(step, n - b0);
      Plan p = plan_segment((uint32_t)k, (uint32_t)e, S, cnt, surv + b0 * (size_t)k * S,
                            (uint64_t)k * S, S, out + b0 * (size_t)e * S, (uint64_t)e * S, S,
                            nullptr, 0, KC, R, nullptr, (uint64_t)e * k, (uint32_t)e, true);
      p.seg.sidx = surv_idx + b0 * (size_t)k;
      p.seg.lidx = lost_idx + b0 * (size_t)e;
      p.seg.lw0 = lw0;
      p.seg.status = status;
      p.seg.m = (uint32_t)m;
      std::vector<Plan> plans{p};
      if (int rc = launch_plans(ctx, plans, st)) return rc;
    }
    return MEMO_EC_OK;
  }
  uint8_t* rows = static_cast<uint8_t*>(scratch);
  const uint64_t row_b = (uint64_t)e * k;
  const uint32_t* lw0 = nullptr;
  if (int rc = lw0_table(ctx, k, m, &lw0)) return rc;
  DecodeArgs a = decode_args(ctx, k, m, e, n, surv_idx, lost_idx, rows, status, lw0);
  const bool images = rows_images(ctx, S, k, R, KC);
  uint32_t* img = reinterpret_cast<uint32_t*>(rows + round256(n * row_b));
  const uint64_t img_dw = (uint64_t)R * kpad_of((uint32_t)k, KC) * 8;  // per block
  if (images) with_images(a, img, R, KC);
  HIPCHK(launch_decode_coef(a, st));
  for (size_t b0 = 0; b0 < n; b0 += step) {
    const size_t cnt = std::min(step, n - b0);
    std::vector<Plan> plans{
        images ? plan_segment((uint32_t)k, (uint32_t)e, S, cnt, surv + b0 * (size_t)k * S,
                              (uint64_t)k * S, S, out + b0 * (size_t)e * S, (uint64_t)e * S, S,
                              img + b0 * img_dw, img_dw, KC, R)
               : plan_segment((uint32_t)k, (uint32_t)e, S, cnt, surv + b0 * (size_t)k * S,
                              (uint64_t)k * S, S, out + b0 * (size_t)e * S, (uint64_t)e * S, S,
                              nullptr, 0, KC, R, rows + b0 * row_b, row_b, (uint32_t)e)};
    if (images) plans[0].mode = MAC_IMAGES;  // the encode's code under a rebuild name
    if (int rc = launch_plans(ctx, plans, st)) return rc;
  }
  return MEMO_EC_OK;
}

// Rebuild scratch for n blocks (a multiple of 256 bytes): their decode rows,
// e x k bytes each, and behind them (rows_images) their table images (the
// two-kernel path; the fused one needs none).
size_t rebuild_scratch(const memo_ec_ctx* c, int k, int e, size_t S, size_t n, bool fused) {
  if (fused) return 0;
  const int R = mac_rbound(e), KC = mac_kchunk(k, R);
  return round256(n * (size_t)e * k) + (rows_images(c, S, k, R, KC) ? image_bytes(n, k, R, KC) : 0);
}

// Deferred-error words in ctx->d_status: device-resident calls (reported by
// memo_ec_synchronize) and the host-memory copy pipeline (reported by the
// call itself) each have their own, so neither consumes the other's fault.
constexpr size_t kStatusDevice = 0, kStatusPipeline = 16;

// Host-memory pipeline over nw waves.  Wave w uses slot w % 3:
//   in(slot, w, st)    host staging + HtoD copies on st
//   run(slot, w, st)   kernels on st, after the slot's HtoD
//   out(slot, w, st)   DtoH copies on st, after the kernels
//   done(slot, w)      host side after the DtoH (pageable copy-out)
// With several waves the three stages run on the copy-in, compute and
// copy-out streams chained by events, so the HtoD of wave i+1 runs under
// the DtoH of wave i (PCIe duplex).  A single wave has nothing to overlap
// and runs on one stream, without the cross-stream event hops (latency).
template <class In, class Run, class Out, class Done>
int run_waves(memo_ec_ctx* c, size_t nw, In in, Run run, Out out, Done done) {
  size_t wave[kSlots] = {};
  bool busy[kSlots] = {};
  const bool one = nw == 1;
  hipStream_t s_in = one ? c->sk : c->sh, s_out = one ? c->sk : c->sd;
  auto finish = [&](int s) -> int {
    if (!busy[s]) return MEMO_EC_OK;
    HIPCHK(hipEventSynchronize(c->ev_d[s]));
    done(s, wave[s]);
    busy[s] = false;
    return MEMO_EC_OK;
  };
  for (size_t w = 0; w < nw; ++w) {
    const int s = (int)(w % kSlots);
    if (int rc = finish(s)) return rc;
    if (int rc = in(s, w, s_in)) return rc;
    if (!one) {
      HIPCHK(hipEventRecord(c->ev_h[s], c->sh));
      HIPCHK(hipStreamWaitEvent(c->sk, c->ev_h[s], 0));
    }
    if (int rc = run(s, w, c->sk)) return rc;
    if (!one) {
      HIPCHK(hipEventRecord(c->ev_k[s], c->sk));
      HIPCHK(hipStreamWaitEvent(c->sd, c->ev_k[s], 0));
    }
    if (int rc = out(s, w, s_out)) return rc;
    HIPCHK(hipEventRecord(c->ev_d[s], s_out));
    wave[s] = w;
    busy[s] = true;
  }
  for (size_t w = nw > kSlots ? nw - kSlots : 0; w < nw; ++w)
    if (int rc = finish((int)(w % kSlots))) return rc;
  return MEMO_EC_OK;
}

// run_waves over batches of nb of n blocks: the callbacks get (slot, first
// block, blocks[, stream]).
template <class In, class Run, class Out, class Done>
int run_pipeline(memo_ec_ctx* c, size_t n, size_t nb, In in, Run run, Out out, Done done) {
  auto span = [&](size_t w, size_t& b0, size_t& cn) {
    b0 = w * nb;
    cn = std::min(nb, n - b0);
  };
  size_t b0, cn;
  return run_waves(
      c, (n + nb - 1) / nb,
      [&](int s, size_t w, hipStream_t st) { span(w, b0, cn); return in(s, b0, cn, st); },
      [&](int s, size_t w, hipStream_t st) { span(w, b0, cn); return run(s, b0, cn, st); },
      [&](int s, size_t w, hipStream_t st) { span(w, b0, cn); return out(s, b0, cn, st); },
      [&](int s, size_t w) {
        size_t x0, xn;
        span(w, x0, xn);
        done(s, x0, xn);
      });
}

// A host-memory call of one multiply-accumulate over n blocks of in_b bytes
// in and out_b bytes out (encode, uniform rebuild): `run(src, dst, cnt, st)`
// enqueues the kernels for cnt blocks of device- or pinned-memory src/dst.
// Small calls run zero-copy on pinned memory; larger ones through the
// 3-stage copy pipeline.
template <class Run>
int host_mac(memo_ec_ctx* c, size_t n, size_t in_b, size_t out_b, const uint8_t* data,
             uint8_t* out, bool pinned, Run run) {
  if (n * (in_b + out_b) <= zc_max_bytes(c)) {
    // Small call: the kernel reads the blocks from, and writes its output
    // to, pinned host memory over PCIe -- no DMA copies to wait for.
    if (int rc = ensure_slots(c, 0, pinned ? 0 : n * (in_b + out_b))) return rc;
    const uint8_t* src = data;
    uint8_t* dst = out;
    if (!pinned) {
      par_memcpy(c, c->h_slot[0], data, n * in_b);
      src = c->h_slot[0];
      dst = c->h_slot[0] + n * in_b;
    }
    if (int rc = run(src, dst, n, c->sk)) return rc;
    HIPCHK(hipStreamSynchronize(c->sk));
    if (!pinned) par_memcpy(c, out, dst, n * out_b);
    return MEMO_EC_OK;
  }
  size_t nb = std::max<size_t>(1, c->opt.pipe_bytes / in_b);
  nb = std::min(nb, n);
  if (int rc = ensure_slots(c, nb * (in_b + out_b), pinned ? 0 : nb * (in_b + out_b))) return rc;
  // slot layout (device and pageable bounce): [in nb*in_b | out nb*out_b]
  return run_pipeline(
      c, n, nb,
      [&](int s, size_t b0, size_t cnt, hipStream_t st) -> int {
        const uint8_t* src = data + b0 * in_b;
        if (!pinned) {
          par_memcpy(c, c->h_slot[s], src, cnt * in_b);
          src = c->h_slot[s];
        }
        return hip_rc(hipMemcpyAsync(c->d_slot[s], src, cnt * in_b, hipMemcpyHostToDevice, st));
      },
      [&](int s, size_t, size_t cnt, hipStream_t st) -> int {
        return run(c->d_slot[s], c->d_slot[s] + nb * in_b, cnt, st);
      },
      [&](int s, size_t b0, size_t cnt, hipStream_t st) -> int {
        uint8_t* dst = pinned ? out + b0 * out_b : c->h_slot[s] + nb * in_b;
        return hip_rc(hipMemcpyAsync(dst, c->d_slot[s] + nb * in_b, cnt * out_b,
                                     hipMemcpyDeviceToHost, st));
      },
      [&](int s, size_t b0, size_t cnt) {
        if (!pinned) par_memcpy(c, out + b0 * out_b, c->h_slot[s] + nb * in_b, cnt * out_b);
      });
}

// Decode rows of one erasure pattern on the host: row r = C[lost_r] *
// inv(C[surv]) by Gauss-Jordan over GF(2^8) (k <= 64: microseconds).  False
// for an invalid pattern (index >= k+m, duplicate survivors).
bool host_decode_rows(int k, int m, const uint8_t* sidx, const uint8_t* lidx, int e, uint8_t* rows) {
  const uint8_t* lg = host_gf_log();
  const uint8_t* ex = host_gf_exp();
  auto mul = [&](uint32_t a, uint32_t b) -> uint32_t { return (a && b) ? ex[lg[a] + lg[b]] : 0u; };
  auto inv = [&](uint32_t a) -> uint32_t { return ex[255 - lg[a]]; };
  const int nt = k + m;
  std::vector<uint8_t> gen((size_t)nt * k);
  memo_ec_generator(k, m, gen.data());
  std::vector<int> seen(nt, 0);
  for (int t = 0; t < k; ++t) {
    if (sidx[t] >= nt || seen[sidx[t]]++) return false;
  }
  for (int r = 0; r < e; ++r)
    if (lidx[r] >= nt) return false;
  // A = C[surv] (k x k) | I, reduced to I | inv(A)
  std::vector<uint8_t> A((size_t)k * 2 * k, 0);
  for (int t = 0; t < k; ++t) {
    std::memcpy(&A[(size_t)t * 2 * k], &gen[(size_t)sidx[t] * k], k);
    A[(size_t)t * 2 * k + k + t] = 1;
  }
  for (int c = 0; c < k; ++c) {
    int p = c;
    while (p < k && !A[(size_t)p * 2 * k + c]) ++p;
    if (p == k) return false;  // cannot happen for a Cauchy code
    if (p != c)
      for (int j = 0; j < 2 * k; ++j) std::swap(A[(size_t)p * 2 * k + j], A[(size_t)c * 2 * k + j]);
    const uint32_t iv = inv(A[(size_t)c * 2 * k + c]);
    for (int j = 0; j < 2 * k; ++j) A[(size_t)c * 2 * k + j] = (uint8_t)mul(A[(size_t)c * 2 * k + j], iv);
    for (int r = 0; r < k; ++r) {
      const uint32_t f = A[(size_t)r * 2 * k + c];
      if (r == c || !f) continue;
      for (int j = 0; j < 2 * k; ++j) A[(size_t)r * 2 * k + j] ^= (uint8_t)mul(f, A[(size_t)c * 2 * k + j]);
    }
  }
  for (int r = 0; r < e; ++r)
    for (int t = 0; t < k; ++t) {
      uint32_t acc = 0;
      for (int j = 0; j < k; ++j) acc ^= mul(gen[(size_t)lidx[r] * k + j], A[(size_t)j * 2 * k + k + t]);
      rows[(size_t)r * k + t] = (uint8_t)acc;
    }
  return true;
}

// Cached device table image of one erasure pattern's decode rows (uniform
// rebuild).  Repairs repeat a few patterns (one per shard index a lost node
// held), so images are kept, least recently used evicted past 64.
int pattern_tables(memo_ec_ctx* ctx, int k, int m, const uint8_t* sidx, const uint8_t* lidx, int e,
                   int R, int KC, const uint32_t** out) {
  const int kpad = (int)kpad_of((uint32_t)k, KC);
  std::vector<uint8_t> key(sidx, sidx + k);
  key.insert(key.end(), lidx, lidx + e);
  ++ctx->pat_clock;
  for (auto& p : ctx->pat_tabs)
    if (p.k == k && p.m == m && p.R == R && p.kpad == kpad && p.key == key) {
      p.used = ctx->pat_clock;
      p.call = ctx->call_seq;
      *out = p.dev;
      return MEMO_EC_OK;
    }
  std::vector<uint8_t> rows((size_t)e * k);
  if (!host_decode_rows(k, m, sidx, lidx, e, rows.data())) return MEMO_EC_ESINGULAR;
  std::vector<uint32_t> img((size_t)R * kpad * 8);
  table_image_host(rows.data(), (uint32_t)e, (uint32_t)k, (uint32_t)R, (uint32_t)kpad, img.data());
  // past 64 images the least recently used goes, unless the current call
  // (a rebuild_segments call with many patterns) still needs it
  auto lru = ctx->pat_tabs.end();
  if (ctx->pat_tabs.size() >= 64)
    for (auto it = ctx->pat_tabs.begin(); it != ctx->pat_tabs.end(); ++it)
      if (it->call != ctx->call_seq && (lru == ctx->pat_tabs.end() || it->used < lru->used)) lru = it;
  if (lru != ctx->pat_tabs.end()) {
    // the evicted image may still be read by enqueued work on this ctx
    HIPCHK(hipStreamSynchronize(ctx->stream));
    if (int rc = sync_pipeline(ctx)) return rc;
    HIPCHK(hipFree(lru->dev));
    ctx->pat_tabs.erase(lru);
  }
  uint32_t* dev = nullptr;
  HIPCHK(hipMalloc(&dev, img.size() * 4));
  hipError_t err = hipMemcpy(dev, img.data(), img.size() * 4, hipMemcpyHostToDevice);
  if (err != hipSuccess) {
    (void)hipFree(dev);
    return hip_rc(err);
  }
  ctx->pat_tabs.push_back({k, m, R, kpad, std::move(key), dev, ctx->pat_clock, ctx->call_seq});
  *out = dev;
  return MEMO_EC_OK;
}

// ---- Mixed-geometry rebuild (memo_ec_rebuild_segments).
// A piece: blocks [b0, b0 + n) of one segment, with the pointers the
// kernels read (device memory, or pinned host memory for a zero-copy call)
// and its launch class, fixed once per call: shard chunk KC, row bound R
// (the class's largest), mode (MAC_ENCODE for a shared pattern, whose
// product tables `tab` were formed on the host; MAC_FUSED or MAC_ROWS for
// per-block patterns).
struct RPiece {
  int seg = 0;
  int k = 0, m = 0, e = 0;
  size_t S = 0, n = 0, b0 = 0;
  const uint8_t* sidx = nullptr;  // per-block: n x k
  const uint8_t* surv = nullptr;  // n x k x S
  const uint8_t* lidx = nullptr;  // per-block: n x e
  uint8_t* out = nullptr;         // n x e x S
  int mode = MAC_ENCODE, KC = 4, R = 1;
  bool img = false;               // MAC_ROWS: table images through HBM (rows_images)
  const uint32_t* tab = nullptr;  // shared pattern: table image
  // the MAC launch this piece takes (MAC_ROWS with images: the encode body)
  int mac_mode() const { return img ? MAC_ENCODE : mode; }
};

// Scratch bytes (a multiple of 256) the MAC_ROWS pieces of `ps` need: the
// decode rows of every piece, then the table images of the pieces with img.
template <class Pieces>
size_t rows_scratch(const Pieces& ps) {
  size_t rows = 0, img = 0;
  for (const RPiece& p : ps) {
    if (p.mode != MAC_ROWS) continue;
    rows += p.n * (size_t)p.e * p.k;
    if (p.img) img += image_bytes(p.n, p.k, p.R, p.KC);
  }
  return round256(rows) + img;
}

// Validates the segments and assigns each non-empty one its class:
// pieces[i] describes segment i whole (pointers as the caller gave them).
// Shared patterns are decoded (and their tables cached) here, before
// anything is enqueued.
int plan_rebuild_segments(memo_ec_ctx* c, int nseg, const memo_ec_rebuild_segment* segs,
                          std::vector<RPiece>& pieces) {
  pieces.clear();
  for (int i = 0; i < nseg; ++i) {
    const auto& s = segs[i];
    if (int rc = check_km(s.k, s.m)) return rc;
    if (s.e < 0 || s.e > s.m) return MEMO_EC_EINVAL;
    if (s.e == 0 || s.n == 0) continue;
    if (s.S == 0 || s.S % 64 || !s.surv_idx || !s.surv || !s.lost_idx || !s.out) return MEMO_EC_EINVAL;
    if (s.S >= kMaxShard || too_big(s.n, (size_t)(s.k + s.e) * s.S + s.k + s.e)) return MEMO_EC_ERANGE;
    RPiece p;
    p.seg = i;
    p.k = s.k;
    p.m = s.m;
    p.e = s.e;
    p.S = s.S;
    p.n = s.n;
    p.sidx = s.surv_idx;
    p.surv = s.surv;
    p.lidx = s.lost_idx;
    p.out = s.out;
    p.R = mac_rbound(s.e);
    p.KC = mac_kchunk(s.k, p.R);
    p.mode = s.uniform ? MAC_ENCODE : MAC_ROWS;  // per-block: fused or rows, below
    pieces.push_back(p);
  }
  // classes (kind, KC): R = the class's largest bound.  KC = 6, 12, 14 are
  // only chosen for R <= 4, so their classes stay within the instantiated
  // bodies.  Per-block classes take the fused kernel up to the ctx's fused
  // bound of survivor bytes (as memo_ec_rebuild_batch does per call).
  struct Cls {
    bool uniform;
    int KC, R;
    size_t in_bytes;
  };
  std::vector<Cls> cls;
  std::vector<size_t> of(pieces.size());
  for (size_t i = 0; i < pieces.size(); ++i) {
    const auto& p = pieces[i];
    const bool u = p.mode == MAC_ENCODE;
    size_t ci = 0;
    while (ci < cls.size() && !(cls[ci].uniform == u && cls[ci].KC == p.KC)) ++ci;
    if (ci == cls.size()) cls.push_back({u, p.KC, 1, 0});
    cls[ci].R = std::max(cls[ci].R, p.R);
    cls[ci].in_bytes += p.n * (size_t)p.k * p.S;
    of[i] = ci;
  }
  ++c->call_seq;
  for (size_t i = 0; i < pieces.size(); ++i) {
    auto& p = pieces[i];
    const Cls& k = cls[of[i]];
    p.R = k.R;
    if (p.mode == MAC_ENCODE) {
      if (int rc = pattern_tables(c, p.k, p.m, p.sidx, p.lidx, p.e, p.R, p.KC, &p.tab)) return rc;
    } else {
      p.mode = rebuild_fused(c, k.in_bytes) ? MAC_FUSED : MAC_ROWS;
      p.img = p.mode == MAC_ROWS && rows_images(c, p.S, p.k, p.R, p.KC);
    }
  }
  return MEMO_EC_OK;
}

// Enqueue the kernels of `ps` on st: decode rows of MAC_ROWS pieces into
// `rows` (rows_scratch(ps) bytes: the rows, then the table images of the
// pieces with img), then one launch set per (MAC mode, KC, R) class, pieces
// longer than one launch's grid split by blocks.
int launch_rebuild_pieces(memo_ec_ctx* c, const std::vector<RPiece>& ps, uint8_t* rows,
                          hipStream_t st, uint32_t* status) {
  std::vector<const uint8_t*> prow(ps.size(), nullptr);
  std::vector<const uint32_t*> pimg(ps.size(), nullptr);
  std::vector<DecodeArgs> dec_of(ps.size());  // per MAC_ROWS piece
  size_t off = 0, rows_total = 0;
  for (const auto& p : ps)
    if (p.mode == MAC_ROWS) rows_total += p.n * (size_t)p.e * p.k;
  uint8_t* img_base = rows + round256(rows_total);
  size_t ioff = 0;
  for (size_t i = 0; i < ps.size(); ++i) {
    const auto& p = ps[i];
    if (p.mode != MAC_ROWS) continue;
    const uint32_t* lw0 = nullptr;
    if (int rc = lw0_table(c, p.k, p.m, &lw0)) return rc;
    dec_of[i] = decode_args(c, p.k, p.m, p.e, p.n, p.sidx, p.lidx, rows + off, status, lw0);
    prow[i] = rows + off;
    if (p.img) {
      uint32_t* img = reinterpret_cast<uint32_t*>(img_base + ioff);
      pimg[i] = img;
      with_images(dec_of[i], img, p.R, p.KC);
      ioff += image_bytes(p.n, p.k, p.R, p.KC);
    }
    off += p.n * (size_t)p.e * p.k;
  }
  // The launch class of a piece: (mode, KC, R).  Pieces that multiply with
  // table images -- per-block images, or a shared pattern's -- join the
  // rows launch of their (KC, R) when the call has one (gf_mac_kernel's
  // rows instance runs both bodies: no extra launch tail); otherwise
  // per-block images take gf_mac_images_kernel (the encode's code under a
  // rebuild name: kernel traces tell it from the encode), and a shared
  // pattern joins that launch, or the encode kernel.
  auto has = [&](const RPiece& p, bool images) {
    for (const auto& q : ps)
      if (q.KC == p.KC && q.R == p.R && (images ? q.img : q.mac_mode() == MAC_ROWS)) return true;
    return false;
  };
  auto launch_mode = [&](const RPiece& p) {
    if (p.mac_mode() != MAC_ENCODE) return p.mac_mode();  // rows, fused
    if (has(p, false)) return (int)MAC_ROWS;
    if (p.img || has(p, true)) return (int)MAC_IMAGES;
    return (int)MAC_ENCODE;
  };
  struct Cls {
    int mode, KC, R;
    std::vector<size_t> pieces;
    std::vector<DecodeArgs> dec;  // the decode rows (and images) its pieces need
  };
  std::vector<Cls> cls;
  {
    std::vector<bool> done(ps.size(), false);
    for (size_t i = 0; i < ps.size(); ++i) {
      if (done[i]) continue;
      Cls k{launch_mode(ps[i]), ps[i].KC, ps[i].R, {}, {}};
      for (size_t j = i; j < ps.size(); ++j)
        if (!done[j] && launch_mode(ps[j]) == k.mode && ps[j].KC == k.KC && ps[j].R == k.R) {
          done[j] = true;
          k.pieces.push_back(j);
          if (ps[j].mode == MAC_ROWS) k.dec.push_back(dec_of[j]);
        }
      cls.push_back(std::move(k));
    }
  }
  // Decode rows.  A call with several classes to decode (a mixed rebuild)
  // runs the decodes of all but the first such class on the ctx's side
  // stream, behind an event of the call's stream, so they overlap the MACs
  // before them instead of running one after another in front of the first
  // MAC; each class's MAC waits for its own decodes' event.  Otherwise every
  // decode goes first on the call's stream, segments of one decode kernel
  // per launch.
  std::vector<int> waits(cls.size(), -1);  // class -> side-stream event
  // On an early return st still waits for the side stream's last decode,
  // so a later call cannot reuse the scratch while that decode runs.
  struct SideJoin {
    memo_ec_ctx* c;
    hipStream_t st;
    int last = -1;  // side event st has not waited for yet
    ~SideJoin() {
      if (last >= 0) (void)hipStreamWaitEvent(st, c->side_ev[last], 0);
    }
  } join{c, st};
  size_t ndec = 0;
  for (const auto& k : cls) ndec += !k.dec.empty();
  if (ndec > 1 && c->opt.decode_overlap) {
    if (int rc = side_events(c, (int)ndec + 1)) return rc;
    // the side stream starts after the call's stream's earlier work, and
    // beside the first class's decode (recorded before it: the side decodes
    // do not depend on it)
    HIPCHK(hipEventRecord(c->side_ev[0], st));
    HIPCHK(hipStreamWaitEvent(c->side, c->side_ev[0], 0));
    bool first = true;
    int ne = 0;
    for (size_t x = 0; x < cls.size(); ++x) {
      if (cls[x].dec.empty()) continue;
      if (first) {  // on the call's stream, before its own MAC
        HIPCHK(launch_decode_multi(cls[x].dec.data(), (int)cls[x].dec.size(), st));
        first = false;
        continue;
      }
      HIPCHK(launch_decode_multi(cls[x].dec.data(), (int)cls[x].dec.size(), c->side));
      HIPCHK(hipEventRecord(c->side_ev[ne + 1], c->side));
      waits[x] = join.last = ne + 1;
      ++ne;
    }
  } else {
    std::vector<DecodeArgs> dec;
    for (const auto& k : cls) dec.insert(dec.end(), k.dec.begin(), k.dec.end());
    if (!dec.empty()) HIPCHK(launch_decode_multi(dec.data(), (int)dec.size(), st));
  }
  for (size_t x = 0; x < cls.size(); ++x) {
    const int mode = cls[x].mode, KC = cls[x].KC, R = cls[x].R;
    std::vector<Plan> plans;
    for (size_t j : cls[x].pieces) {
      const auto& p = ps[j];
      const size_t step = max_blocks_per_launch(c, p.S);
      const uint32_t* lw0 = nullptr;
      if (mode == MAC_FUSED)
        if (int rc = lw0_table(c, p.k, p.m, &lw0)) return rc;
      for (size_t b0 = 0; b0 < p.n; b0 += step) {
        const size_t cnt = std::min(step, p.n - b0);
        const uint64_t in_bs = (uint64_t)p.k * p.S, out_bs = (uint64_t)p.e * p.S;
        const uint8_t* in = p.surv + b0 * in_bs;
        uint8_t* out = p.out + b0 * out_bs;
        if (p.img || p.mode == MAC_ENCODE) {
          const uint64_t per_dw = p.img ? (uint64_t)R * kpad_of((uint32_t)p.k, KC) * 8 : 0;
          Plan q = plan_segment((uint32_t)p.k, (uint32_t)p.e, p.S, cnt, in, in_bs, p.S, out, out_bs,
                                p.S, p.img ? pimg[j] + b0 * per_dw : p.tab, per_dw, KC, R);
          q.mode = mode;  // encode body; in the rows launch when it joins one
          plans.push_back(q);
        } else if (mode == MAC_ROWS) {
          const uint64_t row_b = (uint64_t)p.e * p.k;
          plans.push_back(plan_segment((uint32_t)p.k, (uint32_t)p.e, p.S, cnt, in, in_bs, p.S, out, out_bs,
                                       p.S, nullptr, 0, KC, R, prow[j] + b0 * row_b, row_b, (uint32_t)p.e));
        } else {
          Plan q = plan_segment((uint32_t)p.k, (uint32_t)p.e, p.S, cnt, in, in_bs, p.S, out, out_bs, p.S,
                                nullptr, 0, KC, R, nullptr, (uint64_t)p.e * p.k, (uint32_t)p.e, true);
          q.seg.sidx = p.sidx + b0 * (size_t)p.k;
          q.seg.lidx = p.lidx + b0 * (size_t)p.e;
          q.seg.lw0 = lw0;
          q.seg.status = status;
          q.seg.m = (uint32_t)p.m;
          plans.push_back(q);
        }
      }
    }
    if (waits[x] >= 0) {
      HIPCHK(hipStreamWaitEvent(st, c->side_ev[waits[x]], 0));
      if (waits[x] == join.last) join.last = -1;
    }
    if (int rc = launch_plans(c, plans, st)) return rc;
  }
  return MEMO_EC_OK;
}

int take_deferred(memo_ec_ctx* ctx) {
  uint32_t st = 0;
  HIPCHK(hipMemcpy(&st, ctx->d_status, sizeof st, hipMemcpyDeviceToHost));
  if (st) {
    const uint32_t z = 0;
    HIPCHK(hipMemcpy(ctx->d_status, &z, sizeof z, hipMemcpyHostToDevice));
  }
  int rc = ctx->deferred;
  ctx->deferred = 0;
  if (rc == MEMO_EC_OK && (st & 1u)) rc = MEMO_EC_ESINGULAR;
  return rc;
}

}  // namespace

extern "C" {

int memo_ec_version(void) { return MEMO_EC_VERSION; }

#ifndef MEMO_EC_BUILD_ID
#define MEMO_EC_BUILD_ID "unknown"
#endif
const char* memo_ec_build_id(void) { return MEMO_EC_BUILD_ID; }

int memo_ec_ctx_set_option(memo_ec_ctx* c, int option, int64_t value) {
  if (!c) return MEMO_EC_EINVAL;
  return set_opt(c->opt, option, value) ? MEMO_EC_OK : MEMO_EC_EINVAL;
}

int memo_ec_ctx_get_option(memo_ec_ctx* c, int option, int64_t* value) {
  if (!c || !value) return MEMO_EC_EINVAL;
  return get_opt(c->opt, option, value) ? MEMO_EC_OK : MEMO_EC_EINVAL;
}

int memo_ec_device_count(void) {
  int n = 0;
  return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

int memo_ec_device_identity(int device, char* pci_bus_id, size_t pci_len, char* uuid,
                            size_t uuid_len) {
  if (!pci_bus_id || pci_len < 13 || !uuid || uuid_len < 33) return MEMO_EC_EINVAL;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count)
    return MEMO_EC_ENODEV;
  const int len = (int)std::min<size_t>(pci_len, 64);
  HIPCHK(hipDeviceGetPCIBusId(pci_bus_id, len, device));
  pci_bus_id[len - 1] = '\0';
  hipDevice_t dev;
  HIPCHK(hipDeviceGet(&dev, device));
  hipUUID id{};
  HIPCHK(hipDeviceGetUuid(&id, dev));
  static const char kHex[] = "0123456789abcdef";
  for (int i = 0; i < 16; ++i) {
    const uint8_t b = (uint8_t)id.bytes[i];
    uuid[2 * i] = kHex[b >> 4];
    uuid[2 * i + 1] = kHex[b & 15];
  }
  uuid[32] = '\0';
  return MEMO_EC_OK;
}

const char* memo_ec_strerror(int code) {
  switch (code) {
    case MEMO_EC_OK: return "ok";
    case MEMO_EC_EINVAL: return "invalid argument";
    case MEMO_EC_ENOMEM: return "out of memory";
    case MEMO_EC_EHIP: return "HIP runtime error";
    case MEMO_EC_ESINGULAR: return "survivor shards cannot rebuild the block";
    case MEMO_EC_ENODEV: return "no such GPU";
    case MEMO_EC_ERANGE: return "k, m, shard or call size beyond this build's limits";
    default: return "unknown error";
  }
}

size_t memo_ec_shard_size(size_t B, int k) {
  if (k < 1) return 0;
  size_t per = (B + (size_t)k - 1) / (size_t)k;
  if (per == 0) per = 1;
  return (per + 63) & ~(size_t)63;
}

int memo_ec_generator(int k, int m, uint8_t* out) {
  if (int rc = check_km(k, m)) return rc;
  if (!out) return MEMO_EC_EINVAL;
  const uint8_t* lg = host_gf_log();
  const uint8_t* ex = host_gf_exp();
  std::memset(out, 0, (size_t)(k + m) * k);
  for (int i = 0; i < k; ++i) out[(size_t)i * k + i] = 1;
  for (int i = k; i < k + m; ++i)
    for (int j = 0; j < k; ++j) out[(size_t)i * k + j] = ex[255 - lg[i ^ j]];
  return MEMO_EC_OK;
}

int memo_ec_ctx_create(int device, memo_ec_ctx** out) {
  if (!out) return MEMO_EC_EINVAL;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count)
    return MEMO_EC_ENODEV;
  DeviceGuard g(device);
  auto* c = new (std::nothrow) memo_ec_ctx;
  if (!c) return MEMO_EC_ENOMEM;
  c->device = device;
  int rc = MEMO_EC_OK;
  if ((rc = hip_rc(hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking))) ||
      (rc = hip_rc(hipStreamCreateWithFlags(&c->sh, hipStreamNonBlocking))) ||
      (rc = hip_rc(hipStreamCreateWithFlags(&c->sk, hipStreamNonBlocking))) ||
      (rc = hip_rc(hipStreamCreateWithFlags(&c->sd, hipStreamNonBlocking))) ||
      (rc = hip_rc(hipMalloc(&c->d_status, 256))) ||
      (rc = hip_rc(hipHostMalloc(&c->h_status, 64, hipHostMallocDefault))) ||
      (rc = hip_rc(hipMemset(c->d_status, 0, 256)))) {
    memo_ec_ctx_destroy(c);
    return rc;
  }
  if ((rc = hip_rc(hipEventCreateWithFlags(&c->ev_order, hipEventDisableTiming)))) {
    memo_ec_ctx_destroy(c);
    return rc;
  }
  for (int i = 0; i < kSlots; ++i) {
    if ((rc = hip_rc(hipEventCreateWithFlags(&c->ev_h[i], hipEventDisableTiming))) ||
        (rc = hip_rc(hipEventCreateWithFlags(&c->ev_k[i], hipEventDisableTiming))) ||
        (rc = hip_rc(hipEventCreateWithFlags(&c->ev_d[i], hipEventDisableTiming)))) {
      memo_ec_ctx_destroy(c);
      return rc;
    }
  }
  read_env_options(c->opt);
  c->stream = c->own;
  *out = c;
  return MEMO_EC_OK;
}

int memo_ec_ctx_destroy(memo_ec_ctx* c) {
  if (!c) return MEMO_EC_EINVAL;
  DeviceGuard g(c->device);
  if (c->own) (void)hipStreamSynchronize(c->own);
  if (c->stream && c->stream != c->own) (void)hipStreamSynchronize(c->stream);
  for (auto st : {c->sh, c->sk, c->sd})
    if (st) (void)hipStreamSynchronize(st);
  for (auto& p : c->d_slot)
    if (p) (void)hipFree(p);
  for (auto& p : c->h_slot)
    if (p) (void)hipHostFree(p);
  if (c->d_tabs) (void)hipFree(c->d_tabs);
  for (auto& e : c->enc_tabs) (void)hipFree(e.dev);
  for (auto& e : c->lw0_tabs) (void)hipFree(e.dev);
  for (auto& e : c->pat_tabs) (void)hipFree(e.dev);
  if (c->d_status) (void)hipFree(c->d_status);
  if (c->h_status) (void)hipHostFree(c->h_status);
  for (int i = 0; i < kSlots; ++i)
    for (auto ev : {c->ev_h[i], c->ev_k[i], c->ev_d[i]})
      if (ev) (void)hipEventDestroy(ev);
  if (c->ev_order) (void)hipEventDestroy(c->ev_order);
  if (c->side) (void)hipStreamSynchronize(c->side);
  for (auto ev : c->side_ev) (void)hipEventDestroy(ev);
  if (c->side) (void)hipStreamDestroy(c->side);
  for (auto st : {c->sh, c->sk, c->sd})
    if (st) (void)hipStreamDestroy(st);
  if (c->own) (void)hipStreamDestroy(c->own);
  delete c;
  return MEMO_EC_OK;
}

int memo_ec_set_stream(memo_ec_ctx* c, void* s) {
  if (!c) return MEMO_EC_EINVAL;
  hipStream_t ns = s ? reinterpret_cast<hipStream_t>(s) : c->own;
  if (ns != c->stream) {
    // work on the new stream starts after the old stream's: both reuse the
    // ctx's scratch (decode rows)
    DeviceGuard g(c->device);
    HIPCHK(hipEventRecord(c->ev_order, c->stream));
    HIPCHK(hipStreamWaitEvent(ns, c->ev_order, 0));
  }
  c->stream = ns;
  return MEMO_EC_OK;
}

void* memo_ec_get_stream(memo_ec_ctx* c) { return c ? reinterpret_cast<void*>(c->stream) : nullptr; }

int memo_ec_synchronize(memo_ec_ctx* c) {
  if (!c) return MEMO_EC_EINVAL;
  DeviceGuard g(c->device);
  HIPCHK(hipStreamSynchronize(c->stream));
  return take_deferred(c);
}

int memo_ec_encode_batch(memo_ec_ctx* c, int k, int m, size_t S, size_t n, const uint8_t* data,
                         uint8_t* parity, int where) {
  if (!c) return MEMO_EC_EINVAL;
  if (int rc = check_km(k, m)) return rc;
  if (m == 0 || n == 0) return MEMO_EC_OK;
  if (S == 0 || S % 64 != 0 || !data || !parity) return MEMO_EC_EINVAL;
  if (S >= kMaxShard || too_big(n, (size_t)(k + m) * S)) return MEMO_EC_ERANGE;
  DeviceGuard g(c->device);
  if (where == MEMO_EC_DEVICE) return encode_device(c, k, m, S, n, data, parity, c->stream);
  if (where != MEMO_EC_HOST && where != MEMO_EC_HOST_PINNED) return MEMO_EC_EINVAL;

  return host_mac(c, n, (size_t)k * S, (size_t)m * S, data, parity,
                  where == MEMO_EC_HOST_PINNED,
                  [&](const uint8_t* src, uint8_t* dst, size_t cnt, hipStream_t st) {
                    return encode_device(c, k, m, S, cnt, src, dst, st);
                  });
}

int memo_ec_stream_probe(memo_ec_ctx* c, int kin, int r, size_t S, size_t n, const uint8_t* in,
                         uint8_t* out, int mode) {
  if (!c || mode < MEMO_EC_PROBE_COPY || mode > MEMO_EC_PROBE_WRITE) return MEMO_EC_EINVAL;
  if (int rc = check_km(kin, r)) return rc;
  if (r == 0 || n == 0) return MEMO_EC_OK;
  if (S == 0 || S % 64 != 0 || !in || !out) return MEMO_EC_EINVAL;
  if (S >= kMaxShard || too_big(n, (size_t)(kin + r) * S)) return MEMO_EC_ERANGE;
  DeviceGuard g(c->device);
  // the encode's geometry for (k, m) = (kin, r), launched as the probe
  const int R = mac_rbound(r), KC = mac_kchunk(kin, R);
  const size_t step = max_blocks_per_launch(c, S);
  for (size_t b0 = 0; b0 < n; b0 += step) {
    const size_t cnt = std::min(step, n - b0);
    Plan p = plan_segment((uint32_t)kin, (uint32_t)r, S, cnt, in + b0 * (size_t)kin * S,
                          (uint64_t)kin * S, S, out + b0 * (size_t)r * S, (uint64_t)r * S, S,
                          nullptr, 0, KC, R);
    p.mode = MAC_PROBE;
    p.lds = 0;
    p.seg.probe = (uint32_t)mode;
    std::vector<Plan> plans{p};
    if (int rc = launch_plans(c, plans, c->stream)) return rc;
  }
  return MEMO_EC_OK;
}

#ifdef MEMO_EC_PERM_PROBE
// Probe only (tools/perm_probe.py; not in include/memo_ec.h): the rows MAC
// of n per-block-pattern blocks (e = m lost, survivors and lost shards in
// ascending order) with each block's product images read from a per-code
// table of every pattern's images (qtab: uint4, lotab: dword, R x k slots
// per pattern) at the block's pattern rank (prank[b], u16), instead of
// built from decode rows.  Device pointers; asynchronous on the ctx stream.
extern "C" int memo_ec_probe_perm_mac(memo_ec_ctx* c, int k, int m, size_t S, size_t n,
                                      const uint8_t* surv, uint8_t* out, const uint16_t* prank,
                                      const uint32_t* qtab, const uint32_t* lotab) {
  if (!c || !surv || !out || !prank || !qtab || !lotab) return MEMO_EC_EINVAL;
  if (int rc = check_km(k, m)) return rc;
  DeviceGuard g(c->device);
  const int e = m, R = mac_rbound(e), KC = mac_kchunk(k, R);
  if (KC != k || R != e) return MEMO_EC_EINVAL;  // the straight-line bodies only
  Plan p = plan_segment((uint32_t)k, (uint32_t)e, S, n, surv, (uint64_t)k * S, S, out, (uint64_t)e * S, S,
                        nullptr, 0, KC, R, reinterpret_cast<const uint8_t*>(prank), 1, (uint32_t)e);
  if (!p.seg.flat || sets_per_tile(p.seg.chunks) * (uint64_t)R * k > 6 * 256) return MEMO_EC_ERANGE;
  p.mode = MAC_PERM;
  p.seg.coef_dense = 0;
  p.seg.tab = qtab;
  p.seg.sidx = reinterpret_cast<const uint8_t*>(lotab);
  std::vector<Plan> plans{p};
  return launch_plans(c, plans, c->stream);
}
#endif

void* memo_ec_host_alloc(size_t bytes) {
  void* p = nullptr;
  if (bytes == 0 || hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
  return p;
}

int memo_ec_host_free(void* p) {
  if (!p) return MEMO_EC_OK;
  return hip_rc(hipHostFree(p));
}

int memo_ec_rebuild_uniform(memo_ec_ctx* c, int k, int m, size_t S, size_t n,
                            const uint8_t* surv_idx, const uint8_t* surv, const uint8_t* lost_idx,
                            int e, uint8_t* out, int where) {
  if (!c) return MEMO_EC_EINVAL;
  if (int rc = check_km(k, m)) return rc;
  if (e < 0 || e > m) return MEMO_EC_EINVAL;
  if (e == 0 || n == 0) return MEMO_EC_OK;
  if (S == 0 || S % 64 != 0 || !surv_idx || !surv || !lost_idx || !out) return MEMO_EC_EINVAL;
  if (S >= kMaxShard || too_big(n, (size_t)(k + e) * S + k + e)) return MEMO_EC_ERANGE;
  DeviceGuard g(c->device);
  const int R = mac_rbound(e), KC = mac_kchunk(k, R);
  const uint32_t* tab = nullptr;
  ++c->call_seq;
  if (int rc = pattern_tables(c, k, m, surv_idx, lost_idx, e, R, KC, &tab)) return rc;
  auto run = [&](const uint8_t* src, uint8_t* dst, size_t cnt, hipStream_t st) -> int {
    const size_t step = max_blocks_per_launch(c, S);
    for (size_t b0 = 0; b0 < cnt; b0 += step) {
      const size_t bc = std::min(step, cnt - b0);
      std::vector<Plan> plans{plan_segment((uint32_t)k, (uint32_t)e, S, bc, src + b0 * (size_t)k * S,
                                           (uint64_t)k * S, S, dst + b0 * (size_t)e * S,
                                           (uint64_t)e * S, S, tab, 0, KC, R)};
      if (int rc = launch_plans(c, plans, st)) return rc;
    }
    return MEMO_EC_OK;
  };
  if (where == MEMO_EC_DEVICE) return run(surv, out, n, c->stream);
  if (where != MEMO_EC_HOST && where != MEMO_EC_HOST_PINNED) return MEMO_EC_EINVAL;
  return host_mac(c, n, (size_t)k * S, (size_t)e * S, surv, out, where == MEMO_EC_HOST_PINNED, run);
}

int memo_ec_decode_rows(memo_ec_ctx* c, int k, int m, size_t n, const uint8_t* surv_idx,
                        const uint8_t* lost_idx, int e, uint8_t* rows) {
  if (!c) return MEMO_EC_EINVAL;
  if (int rc = check_km(k, m)) return rc;
  if (e < 0 || e > m) return MEMO_EC_EINVAL;
  if (n == 0 || e == 0) return MEMO_EC_OK;
  if (!surv_idx || !lost_idx || !rows) return MEMO_EC_EINVAL;
  if (too_big(n, (size_t)e * k + k + e)) return MEMO_EC_ERANGE;
  DeviceGuard g(c->device);
  const uint32_t* lw0 = nullptr;
  if (int rc = lw0_table(c, k, m, &lw0)) return rc;
  const DecodeArgs a = decode_args(c, k, m, e, n, surv_idx, lost_idx, rows, c->d_status + kStatusDevice,
                                   lw0);
  return hip_rc(launch_decode_coef(a, c->stream));
}

int memo_ec_rebuild_batch(memo_ec_ctx* c, int k, int m, size_t S, size_t n,
                          const uint8_t* surv_idx, const uint8_t* surv, const uint8_t* lost_idx,
                          int e, uint8_t* out, int where) {
  if (!c) return MEMO_EC_EINVAL;
  if (int rc = check_km(k, m)) return rc;
  if (e < 0 || e > m) return MEMO_EC_EINVAL;
  if (e == 0 || n == 0) return MEMO_EC_OK;
  if (S == 0 || S % 64 != 0 || !surv_idx || !surv || !lost_idx || !out) return MEMO_EC_EINVAL;
  if (S >= kMaxShard || too_big(n, (size_t)(k + e) * S + k + e)) return MEMO_EC_ERANGE;
  DeviceGuard g(c->device);
  const bool fused = rebuild_fused(c, n * (size_t)k * S);
  if (where == MEMO_EC_DEVICE) {
    if (int rc = ensure_tabs(c, rebuild_scratch(c, k, e, S, n, fused))) return rc;
    if (int rc = rebuild_device(c, k, m, S, n, surv_idx, surv, lost_idx, e, out, fused, c->d_tabs,
                                c->stream, c->d_status + kStatusDevice))
      return rc;
    // marks the scratch busy until this rebuild is done (host calls check it)
    return hip_rc(hipEventRecord(c->ev_order, c->stream));
  }
  if (where != MEMO_EC_HOST && where != MEMO_EC_HOST_PINNED) return MEMO_EC_EINVAL;

  const size_t in_b = (size_t)k * S, out_b = (size_t)e * S;
  const size_t idx_b = (size_t)k + e;
  const bool pinned = where == MEMO_EC_HOST_PINNED;
  // device rebuilds still pending on the ctx stream read the same scratch
  const hipError_t q = hipEventQuery(c->ev_order);
  if (q == hipErrorNotReady) {
    HIPCHK(hipStreamWaitEvent(c->sk, c->ev_order, 0));
  } else if (q != hipSuccess) {
    return hip_rc(q);
  }
  if (n * (in_b + out_b + idx_b) + 4 <= zc_max_bytes(c)) {
    // Small call: decode and MAC run on pinned host memory directly (the
    // survivors, indices and output in the bounce slot, or the caller's
    // pinned buffers); the status word rides in the slot too.
    const size_t slot = n * (in_b + out_b + idx_b) + 64;
    if (int rc = ensure_slots(c, 0, slot)) return rc;
    if (int rc = ensure_tabs(c, rebuild_scratch(c, k, e, S, n, fused))) return rc;
    uint8_t* h = c->h_slot[0];
    uint8_t* h_sidx = h + n * (in_b + out_b);
    uint8_t* h_lidx = h_sidx + n * k;
    uint32_t* h_st = reinterpret_cast<uint32_t*>(h + ((n * (in_b + out_b + idx_b) + 3) & ~(size_t)3));
    std::memcpy(h_sidx, surv_idx, n * k);
    std::memcpy(h_lidx, lost_idx, n * e);
    *h_st = 0;
    const uint8_t* sv = surv;
    uint8_t* ov = out;
    if (!pinned) {
      par_memcpy(c, h, surv, n * in_b);
      sv = h;
      ov = h + n * in_b;
    }
    if (int rc = rebuild_device(c, k, m, S, n, h_sidx, sv, h_lidx, e, ov, fused, c->d_tabs, c->sk,
                                h_st))
      return rc;
    HIPCHK(hipStreamSynchronize(c->sk));
    if (!pinned) par_memcpy(c, out, ov, n * out_b);
    int drc = c->deferred;
    c->deferred = 0;
    if (drc == MEMO_EC_OK && (__atomic_load_n(h_st, __ATOMIC_ACQUIRE) & 1u)) drc = MEMO_EC_ESINGULAR;
    return drc;
  }
  size_t nb = std::max<size_t>(1, c->opt.pipe_bytes / in_b);
  nb = std::min(nb, n);
  // slot layout: [surv nb*in_b | out nb*out_b | surv_idx nb*k | lost_idx nb*e];
  // pinned callers' data moves by DMA from their own buffers, so their host
  // slot holds the indices only (no pinned bounce buffers of the batch size)
  const size_t slot = nb * (in_b + out_b + idx_b);
  const size_t hshift = pinned ? nb * (in_b + out_b) : 0;  // host slot offset of the device layout
  if (int rc = ensure_slots(c, slot, slot - hshift)) return rc;
  const size_t tabs = rebuild_scratch(c, k, e, S, nb, fused);
  if (int rc = ensure_tabs(c, kSlots * tabs)) return rc;
  const size_t o_out = nb * in_b, o_sidx = o_out + nb * out_b, o_lidx = o_sidx + nb * k;
  const int rc = run_pipeline(
      c, n, nb,
      [&](int s, size_t b0, size_t cnt, hipStream_t st) -> int {
        uint8_t* h = c->h_slot[s];
        uint8_t* d = c->d_slot[s];
        std::memcpy(h + o_sidx - hshift, surv_idx + b0 * k, cnt * k);  // indices: always bounced
        std::memcpy(h + o_lidx - hshift, lost_idx + b0 * e, cnt * e);
        HIPCHK(hipMemcpyAsync(d + o_sidx, h + o_sidx - hshift, nb * idx_b, hipMemcpyHostToDevice, st));
        const uint8_t* src = surv + b0 * in_b;
        if (!pinned) {
          par_memcpy(c, h, src, cnt * in_b);
          src = h;
        }
        return hip_rc(hipMemcpyAsync(d, src, cnt * in_b, hipMemcpyHostToDevice, st));
      },
      [&](int s, size_t, size_t cnt, hipStream_t st) -> int {
        uint8_t* d = c->d_slot[s];
        return rebuild_device(c, k, m, S, cnt, d + o_sidx, d, d + o_lidx, e, d + o_out, fused,
                              reinterpret_cast<uint8_t*>(c->d_tabs) + (size_t)s * tabs, st,
                              c->d_status + kStatusPipeline);
      },
      [&](int s, size_t b0, size_t cnt, hipStream_t st) -> int {
        uint8_t* dst = pinned ? out + b0 * out_b : c->h_slot[s] + o_out;
        HIPCHK(hipMemcpyAsync(dst, c->d_slot[s] + o_out, cnt * out_b, hipMemcpyDeviceToHost, st));
        // the deferred-error word rides behind the last batch's output, so
        // reading it costs no extra round trip
        if (b0 + cnt == n)
          HIPCHK(hipMemcpyAsync(c->h_status, c->d_status + kStatusPipeline, sizeof(uint32_t),
                                hipMemcpyDeviceToHost,
                                st));
        return MEMO_EC_OK;
      },
      [&](int s, size_t b0, size_t cnt) {
        if (!pinned) par_memcpy(c, out + b0 * out_b, c->h_slot[s] + o_out, cnt * out_b);
      });
  if (rc) return rc;
  const uint32_t st = *c->h_status;
  if (st) {
    HIPCHK(hipMemsetAsync(c->d_status + kStatusPipeline, 0, sizeof(uint32_t), c->sd));
    HIPCHK(hipStreamSynchronize(c->sd));
  }
  int drc = c->deferred;
  c->deferred = 0;
  if (drc == MEMO_EC_OK && (st & 1u)) drc = MEMO_EC_ESINGULAR;
  return drc;
}

int memo_ec_encode_segments(memo_ec_ctx* c, int nseg, const memo_ec_segment* segs) {
  if (!c || nseg < 0 || nseg > MEMO_EC_MAX_SEGMENTS || (nseg && !segs)) return MEMO_EC_EINVAL;
  // Segments are grouped by shard-chunk class (mac_kchunk): each class is
  // one launch of its own straight-line body, with R = the class's largest
  // m bound (smaller m's rows are zero tables); the launches go back to back
  // on the ctx stream.  One launch across classes would force every segment
  // onto the 4-shard chunk loop: 72% of 8 TB/s on the C5 mix against 77% for
  // per-class launches.  Everything is validated
  // before anything is enqueued.
  std::vector<int> classes;  // KC of each class, in order of first appearance
  std::vector<int> cls_R;
  for (int i = 0; i < nseg; ++i) {
    if (int rc = check_km(segs[i].k, segs[i].m)) return rc;
    if (segs[i].m == 0 || segs[i].n == 0) continue;
    if (segs[i].S == 0 || segs[i].S % 64 || !segs[i].data || !segs[i].parity)
      return MEMO_EC_EINVAL;
    if (segs[i].S >= kMaxShard) return MEMO_EC_ERANGE;
    if (segs[i].n > max_blocks_per_launch(c, segs[i].S)) return MEMO_EC_ERANGE;
    if (too_big(segs[i].n, (size_t)(segs[i].k + segs[i].m) * segs[i].S)) return MEMO_EC_ERANGE;
    const int kc = mac_kchunk(segs[i].k, mac_rbound(segs[i].m));
    size_t ci = 0;
    while (ci < classes.size() && classes[ci] != kc) ++ci;
    if (ci == classes.size()) {
      classes.push_back(kc);
      cls_R.push_back(1);
    }
    cls_R[ci] = std::max(cls_R[ci], mac_rbound(segs[i].m));
  }
  if (classes.empty()) return MEMO_EC_OK;
  DeviceGuard g(c->device);
  std::vector<std::vector<Plan>> launches(classes.size());
  for (size_t ci = 0; ci < classes.size(); ++ci) {
    const int KC = classes[ci], R = cls_R[ci];
    for (int i = 0; i < nseg; ++i) {
      const auto& s = segs[i];
      if (s.m == 0 || s.n == 0 || mac_kchunk(s.k, mac_rbound(s.m)) != KC) continue;
      const uint32_t* tab = nullptr;
      if (int rc = encode_tables(c, s.k, s.m, R, KC, &tab)) return rc;
      launches[ci].push_back(plan_segment((uint32_t)s.k, (uint32_t)s.m, s.S, s.n, s.data,
                                          (uint64_t)s.k * s.S, s.S, s.parity,
                                          (uint64_t)s.m * s.S, s.S, tab, 0, KC, R));
    }
    if (lds_of(launches[ci]) > 160 * 1024) return MEMO_EC_ERANGE;
  }
  for (auto& plans : launches)
    if (int rc = launch_plans(c, plans, c->stream)) return rc;
  return MEMO_EC_OK;
}

int memo_ec_rebuild_segments(memo_ec_ctx* c, int nseg, const memo_ec_rebuild_segment* segs, int where) {
  if (!c || nseg < 0 || nseg > MEMO_EC_MAX_REBUILD_SEGMENTS || (nseg && !segs)) return MEMO_EC_EINVAL;
  if (where != MEMO_EC_DEVICE && where != MEMO_EC_HOST && where != MEMO_EC_HOST_PINNED)
    return MEMO_EC_EINVAL;
  DeviceGuard g(c->device);
  std::vector<RPiece> ps;
  if (int rc = plan_rebuild_segments(c, nseg, segs, ps)) return rc;
  if (ps.empty()) return MEMO_EC_OK;
  if (where == MEMO_EC_DEVICE) {
    if (int rc = ensure_tabs(c, rows_scratch(ps))) return rc;
    if (int rc = launch_rebuild_pieces(c, ps, reinterpret_cast<uint8_t*>(c->d_tabs), c->stream,
                                       c->d_status + kStatusDevice))
      return rc;
    // marks the scratch busy until these rebuilds are done (host calls check it)
    return hip_rc(hipEventRecord(c->ev_order, c->stream));
  }
  const bool pinned = where == MEMO_EC_HOST_PINNED;
  // device rebuilds still pending on the ctx stream read the same scratch
  const hipError_t q = hipEventQuery(c->ev_order);
  if (q == hipErrorNotReady) {
    HIPCHK(hipStreamWaitEvent(c->sk, c->ev_order, 0));
  } else if (q != hipSuccess) {
    return hip_rc(q);
  }
  // Chunks of at most one pipeline batch of survivors, packed in order into
  // waves of at most one batch; a wave's slot holds [survivors | outputs |
  // per-block indices].
  struct Chunk {
    RPiece p;  // host pointers
    size_t in, out, idx;
    size_t o_in = 0, o_out = 0, o_idx = 0;
  };
  std::vector<Chunk> ch;
  const size_t pipe = c->opt.pipe_bytes;
  size_t total = 0;
  for (const RPiece& p : ps) {
    const size_t in_b = (size_t)p.k * p.S, out_b = (size_t)p.e * p.S;
    const bool uni = p.mode == MAC_ENCODE;
    const size_t per = std::max<size_t>(1, pipe / in_b);
    for (size_t b0 = 0; b0 < p.n; b0 += per) {
      Chunk x;
      x.p = p;
      x.p.b0 = b0;
      x.p.n = std::min(per, p.n - b0);
      x.p.surv = p.surv + b0 * in_b;
      x.p.out = p.out + b0 * out_b;
      if (!uni) {
        x.p.sidx = p.sidx + b0 * (size_t)p.k;
        x.p.lidx = p.lidx + b0 * (size_t)p.e;
      }
      x.in = x.p.n * in_b;
      x.out = x.p.n * out_b;
      x.idx = uni ? 0 : x.p.n * (size_t)(p.k + p.e);
      total += x.in + x.out + x.idx;
      ch.push_back(x);
    }
  }
  struct Wave {
    std::vector<size_t> ids;
    size_t in = 0, out = 0, idx = 0;
  };
  std::vector<Wave> waves;
  const bool zc = total + 64 <= zc_max_bytes(c);
  for (size_t i = 0; i < ch.size(); ++i) {
    if (waves.empty() || (!zc && waves.back().in + ch[i].in > pipe)) waves.emplace_back();
    Wave& w = waves.back();
    w.ids.push_back(i);
    w.in += ch[i].in;
    w.out += ch[i].out;
    w.idx += ch[i].idx;
  }
  size_t slot = 0, rows = 0;
  for (Wave& w : waves) {
    size_t oi = 0, oo = w.in, ox = w.in + w.out;
    for (size_t i : w.ids) {
      ch[i].o_in = oi;
      ch[i].o_out = oo;
      ch[i].o_idx = ox;
      oi += ch[i].in;
      oo += ch[i].out;
      ox += ch[i].idx;
    }
    slot = std::max(slot, w.in + w.out + w.idx);
    std::vector<RPiece> wp;
    for (size_t i : w.ids) wp.push_back(ch[i].p);
    rows = std::max(rows, rows_scratch(wp));  // decode rows + table images (256-byte multiple)
  }
  // the pieces as the kernels see them, in slot memory at base (surv / out
  // at the caller's pinned buffers when pinned_io)
  auto staged = [&](const Wave& w, uint8_t* base, bool pinned_io) {
    std::vector<RPiece> dp;
    for (size_t i : w.ids) {
      RPiece p = ch[i].p;
      if (!pinned_io) {
        p.surv = base + ch[i].o_in;
        p.out = base + ch[i].o_out;
      }
      if (p.mode != MAC_ENCODE) {
        p.sidx = base + ch[i].o_idx;
        p.lidx = base + ch[i].o_idx + p.n * (size_t)p.k;
      }
      dp.push_back(p);
    }
    return dp;
  };
  // indices staged at their slot offsets less `shift` (pinned pipeline
  // calls keep only the indices in their host slot)
  auto stage_idx = [&](const Wave& w, uint8_t* h, size_t shift = 0) {
    for (size_t i : w.ids) {
      const RPiece& p = ch[i].p;
      if (p.mode == MAC_ENCODE) continue;
      std::memcpy(h + ch[i].o_idx - shift, p.sidx, p.n * (size_t)p.k);
      std::memcpy(h + ch[i].o_idx - shift + p.n * (size_t)p.k, p.lidx, p.n * (size_t)p.e);
    }
  };
  if (zc) {
    // Small call: the kernels read the survivors and indices from, and
    // write their output to, pinned host memory (no DMA copies); the status
    // word rides in the slot.
    const Wave& w = waves[0];
    if (int rc = ensure_slots(c, 0, slot + 64)) return rc;
    if (int rc = ensure_tabs(c, rows)) return rc;
    uint8_t* h = c->h_slot[0];
    uint32_t* h_st = reinterpret_cast<uint32_t*>(h + ((slot + 3) & ~(size_t)3));
    *h_st = 0;
    stage_idx(w, h);
    if (!pinned)
      for (size_t i : w.ids) par_memcpy(c, h + ch[i].o_in, ch[i].p.surv, ch[i].in);
    if (int rc = launch_rebuild_pieces(c, staged(w, h, pinned), reinterpret_cast<uint8_t*>(c->d_tabs),
                                       c->sk, h_st))
      return rc;
    HIPCHK(hipStreamSynchronize(c->sk));
    if (!pinned)
      for (size_t i : w.ids) par_memcpy(c, ch[i].p.out, h + ch[i].o_out, ch[i].out);
    int drc = c->deferred;
    c->deferred = 0;
    if (drc == MEMO_EC_OK && (__atomic_load_n(h_st, __ATOMIC_ACQUIRE) & 1u)) drc = MEMO_EC_ESINGULAR;
    return drc;
  }
  // pinned: the survivors and outputs move by DMA from the caller's
  // buffers, and the host slot holds a wave's indices only
  size_t hslot = slot;
  if (pinned) {
    hslot = 64;
    for (const Wave& w : waves) hslot = std::max(hslot, w.idx);
  }
  if (int rc = ensure_slots(c, slot, hslot)) return rc;
  if (int rc = ensure_tabs(c, kSlots * rows)) return rc;
  const int rc = run_waves(
      c, waves.size(),
      [&](int s, size_t wi, hipStream_t st) -> int {
        const Wave& w = waves[wi];
        uint8_t* h = c->h_slot[s];
        uint8_t* d = c->d_slot[s];
        const size_t shift = pinned ? w.in + w.out : 0;
        stage_idx(w, h, shift);
        if (w.idx)
          HIPCHK(hipMemcpyAsync(d + w.in + w.out, h + w.in + w.out - shift, w.idx, hipMemcpyHostToDevice, st));
        for (size_t i : w.ids) {
          if (pinned) {
            HIPCHK(hipMemcpyAsync(d + ch[i].o_in, ch[i].p.surv, ch[i].in, hipMemcpyHostToDevice, st));
          } else {
            par_memcpy(c, h + ch[i].o_in, ch[i].p.surv, ch[i].in);
          }
        }
        if (!pinned) HIPCHK(hipMemcpyAsync(d, h, w.in, hipMemcpyHostToDevice, st));
        return MEMO_EC_OK;
      },
      [&](int s, size_t wi, hipStream_t st) -> int {
        return launch_rebuild_pieces(c, staged(waves[wi], c->d_slot[s], false),
                                     reinterpret_cast<uint8_t*>(c->d_tabs) + (size_t)s * rows, st,
                                     c->d_status + kStatusPipeline);
      },
      [&](int s, size_t wi, hipStream_t st) -> int {
        const Wave& w = waves[wi];
        uint8_t* d = c->d_slot[s];
        if (pinned) {
          for (size_t i : w.ids)
            HIPCHK(hipMemcpyAsync(ch[i].p.out, d + ch[i].o_out, ch[i].out, hipMemcpyDeviceToHost, st));
        } else {
          HIPCHK(hipMemcpyAsync(c->h_slot[s] + w.in, d + w.in, w.out, hipMemcpyDeviceToHost, st));
        }
        // the deferred-error word rides behind the last wave's output
        if (wi + 1 == waves.size())
          HIPCHK(hipMemcpyAsync(c->h_status, c->d_status + kStatusPipeline, sizeof(uint32_t),
                                hipMemcpyDeviceToHost, st));
        return MEMO_EC_OK;
      },
      [&](int s, size_t wi) {
        if (pinned) return;
        for (size_t i : waves[wi].ids) par_memcpy(c, ch[i].p.out, c->h_slot[s] + ch[i].o_out, ch[i].out);
      });
  if (rc) return rc;
  const uint32_t st = *c->h_status;
  if (st) {
    HIPCHK(hipMemsetAsync(c->d_status + kStatusPipeline, 0, sizeof(uint32_t), c->sd));
    HIPCHK(hipStreamSynchronize(c->sd));
  }
  int drc = c->deferred;
  c->deferred = 0;
  if (drc == MEMO_EC_OK && (st & 1u)) drc = MEMO_EC_ESINGULAR;
  return drc;
}

int memo_ec_sha256_batch(memo_ec_ctx* c, size_t n, const uint8_t* prefix, size_t prefix_len,
                         size_t prefix_stride, const uint8_t* msg, size_t msg_stride,
                         const uint64_t* msg_len, size_t uniform_len, uint8_t* digest) {
  if (!c || (n && (!digest || !msg || (prefix_len && !prefix)))) return MEMO_EC_EINVAL;
  if (n == 0) return MEMO_EC_OK;
  if (n > 0x7fffffffull * 256) return MEMO_EC_ERANGE;
  DeviceGuard g(c->device);
  Sha256Args a{prefix, msg, msg_len, digest, n, prefix_len, prefix_stride, msg_stride, uniform_len};
  return hip_rc(launch_sha256(a, c->stream));
}

int memo_ec_fill_blocks(memo_ec_ctx* c, uint64_t seed, uint64_t first_block, size_t n, size_t B,
                        int k, size_t S, uint8_t* out) {
  if (!c || k < 1 || S % 16 || (size_t)k * S < B || (n && !out)) return MEMO_EC_EINVAL;
  if (S >= kMaxShard || too_big(n, (size_t)k * S)) return MEMO_EC_ERANGE;
  DeviceGuard g(c->device);
  FillArgs a{out, seed, first_block, n, B, (uint64_t)k * S};
  return hip_rc(launch_fill(a, c->stream));
}

int memo_ec_gather_shards(memo_ec_ctx* c, int k, int m, size_t S, size_t n, const uint8_t* data,
                          const uint8_t* parity, const uint8_t* idx, int cnt, uint8_t* out) {
  if (!c || check_km(k, m) || S % 16 || cnt < 0 || (n && cnt && (!data || !idx || !out)))
    return MEMO_EC_EINVAL;
  if (S >= kMaxShard || too_big(n, (size_t)cnt * S + cnt)) return MEMO_EC_ERANGE;
  DeviceGuard g(c->device);
  GatherArgs a{data, parity, idx, out, S, n, (uint32_t)k, (uint32_t)m, (uint32_t)cnt};
  return hip_rc(launch_gather(a, c->stream));
}

static inline uint64_t sm64_mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int memo_ec_erasures(uint64_t seed, uint64_t first_block, size_t n, int k, int m, int e,
                     uint8_t* surv_idx, uint8_t* lost_idx) {
  if (check_km(k, m) || e < 0 || e > m || (n && (!surv_idx || (e && !lost_idx))))
    return MEMO_EC_EINVAL;
  const int total = k + m;
  const uint64_t gamma = 0x9E3779B97F4A7C15ull;
  for (size_t b = 0; b < n; ++b) {
    const uint64_t key = sm64_mix(sm64_mix(seed + 1) ^ ((first_block + b) * gamma));
    uint8_t perm[256], lost[256] = {0};
    for (int i = 0; i < total; ++i) perm[i] = (uint8_t)i;
    for (int i = 0; i < e; ++i) {
      const uint64_t w = sm64_mix(key + (uint64_t)(i + 1) * gamma);
      const int r = i + (int)(w % (uint64_t)(total - i));
      std::swap(perm[i], perm[r]);
      lost[perm[i]] = 1;
    }
    int li = 0, si = 0;
    for (int i = 0; i < total; ++i) {
      if (lost[i]) lost_idx[b * e + li++] = (uint8_t)i;
      else if (si < k) surv_idx[b * k + si++] = (uint8_t)i;
    }
  }
  return MEMO_EC_OK;
}

}  // extern "C"
