// erasure_consensus.cc -- see erasure_consensus.hh.
#include "erasure_consensus.hh"

#include <nmmintrin.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <optional>
#include <random>
#include <set>
#include <unordered_map>

namespace memo_host {

namespace {

// MEMO_EC_PLUGIN_TIMING=1: per-phase wall times of the batched paths on
// stderr (profiling the host side; off by default).
struct PhaseTimer {
  const char* what;
  bool on;
  std::chrono::steady_clock::time_point t;
  std::string line;
  explicit PhaseTimer(const char* w) : what(w) {
    static const bool env = [] {
      const char* p = std::getenv("MEMO_EC_PLUGIN_TIMING");
      return p && *p == '1';
    }();
    on = env;
    t = std::chrono::steady_clock::now();
  }
  void lap(const char* phase) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    line += std::string(" ") + phase + "=" +
            std::to_string(std::chrono::duration<double, std::milli>(now - t).count()) + "ms";
    t = now;
  }
  ~PhaseTimer() {
    if (on) std::fprintf(stderr, "[timing] %s%s\n", what, line.c_str());
  }
};

// Block payload d as k shards of Sb bytes into k slots of S >= Sb bytes at
// dst (memo_ec_shard_size padding and the slot tails zeroed).
void copy_padded(const Buffer& d, int k, size_t Sb, uint8_t* dst, size_t S) {
  for (int j = 0; j < k; ++j) {
    const size_t lo = std::min(d.size(), (size_t)j * Sb), hi = std::min(d.size(), (size_t)(j + 1) * Sb);
    uint8_t* slot = dst + (size_t)j * S;
    if (hi > lo) std::memcpy(slot, d.data() + lo, hi - lo);
    std::memset(slot + (hi - lo), 0, S - (hi - lo));
  }
}
// Batches mix shard sizes within a power-of-two bucket: every byte column is
// coded independently, so a shard zero-padded to the batch's largest S codes
// exactly (the tail codes to zero and is dropped); padding stays below 2x.
int size_bucket(size_t S) {
  int b = 0;
  while (S > 64) {
    S >>= 1;
    ++b;
  }
  return b;
}

void check(int rc, const char* what) {
  if (rc != MEMO_EC_OK) throw Error(std::string("memo_ec ") + what + ": " + memo_ec_strerror(rc));
}
}  // namespace

// ------------------------------------------------------------------ codec
Codec::Codec(int device, int contexts) {
  std::vector<int> devs;
  if (device >= 0) {
    devs.push_back(device);
  } else {
    const int nd = memo_ec_device_count();
    for (int d = 0; d < nd; ++d) devs.push_back(d);
    if (devs.empty()) devs.push_back(0);  // ctx_create reports the missing GPU
  }
  init(devs, contexts);
}

Codec::Codec(const std::vector<int>& devices, int contexts_per_device) {
  init(devices, contexts_per_device);
}

void Codec::init(const std::vector<int>& devices, int contexts) {
  if (devices.empty() || contexts < 1) throw Error("memo_ec: no device / context");
  for (int id : devices) {
    Dev d{id, {}};
    for (int i = 0; i < contexts; ++i) {
      memo_ec_ctx* c = nullptr;
      const int rc = memo_ec_ctx_create(id, &c);
      if (rc != MEMO_EC_OK) {
        for (auto* p : all_) memo_ec_ctx_destroy(p);
        all_.clear();
        throw Error(std::string("memo_ec ctx_create: ") + memo_ec_strerror(rc));
      }
      all_.push_back(c);
      d.free.push_back(c);
    }
    dev_.push_back(std::move(d));
  }
}

Codec::~Codec() {
  for (auto* c : all_) memo_ec_ctx_destroy(c);
}

memo_ec_ctx* Codec::acquire(size_t d) {
  std::unique_lock<std::mutex> l(mu_);
  cv_.wait(l, [&] { return !dev_[d].free.empty(); });
  auto* c = dev_[d].free.back();
  dev_[d].free.pop_back();
  return c;
}

void Codec::release(size_t d, memo_ec_ctx* c) {
  {
    std::lock_guard<std::mutex> g(mu_);
    dev_[d].free.push_back(c);
  }
  cv_.notify_all();
}

void Codec::split(size_t n, const std::function<int(size_t, size_t, size_t)>& fn,
                  const char* what) {
  const size_t D = dev_.size();
  if (D == 1 || n < 2 * D) {
    // one device: rotate over them so concurrent small calls spread out
    const size_t d = D == 1 ? 0 : rr_++ % D;
    check(fn(d, 0, n), what);
    return;
  }
  std::vector<int> rc(D, MEMO_EC_OK);
  std::vector<std::thread> ts;
  const size_t per = (n + D - 1) / D;
  for (size_t d = 0; d < D; ++d) {
    const size_t b0 = d * per;
    if (b0 >= n) break;
    const size_t cnt = std::min(per, n - b0);
    ts.emplace_back([&, d, b0, cnt] { rc[d] = fn(d, b0, cnt); });
  }
  for (auto& t : ts) t.join();
  for (int r : rc) check(r, what);
}

void Codec::encode(int k, int m, size_t S, size_t n, const uint8_t* data, uint8_t* parity,
                   bool pinned) {
  split(n, [&](size_t d, size_t b0, size_t cnt) {
    auto* c = acquire(d);
    const int rc = memo_ec_encode_batch(c, k, m, S, cnt, data + b0 * k * S, parity + b0 * m * S,
                                        pinned ? MEMO_EC_HOST_PINNED : MEMO_EC_HOST);
    release(d, c);
    return rc;
  }, "encode");
  ++encode_calls_;
}

void Codec::rebuild(int k, int m, size_t S, size_t n, const uint8_t* surv_idx,
                    const uint8_t* surv, const uint8_t* lost_idx, int e, uint8_t* out, bool pinned) {
  split(n, [&](size_t d, size_t b0, size_t cnt) {
    auto* c = acquire(d);
    const int rc = memo_ec_rebuild_batch(c, k, m, S, cnt, surv_idx + b0 * k, surv + b0 * k * S,
                                         lost_idx + b0 * e, e, out + b0 * e * S,
                                         pinned ? MEMO_EC_HOST_PINNED : MEMO_EC_HOST);
    release(d, c);
    return rc;
  }, "rebuild");
  ++rebuild_calls_;
}

void Codec::rebuild_uniform(int k, int m, size_t S, size_t n, const uint8_t* surv_idx,
                            const uint8_t* surv, const uint8_t* lost_idx, int e, uint8_t* out,
                            bool pinned) {
  split(n, [&](size_t d, size_t b0, size_t cnt) {
    auto* c = acquire(d);
    const int rc = memo_ec_rebuild_uniform(c, k, m, S, cnt, surv_idx, surv + b0 * k * S, lost_idx, e,
                                           out + b0 * e * S,
                                           pinned ? MEMO_EC_HOST_PINNED : MEMO_EC_HOST);
    release(d, c);
    return rc;
  }, "rebuild_uniform");
  ++uniform_calls_;
}

void Codec::rebuild_segments(const std::vector<memo_ec_rebuild_segment>& segs, bool pinned) {
  const int where = pinned ? MEMO_EC_HOST_PINNED : MEMO_EC_HOST;
  size_t maxn = 0;
  for (const auto& sg : segs) maxn = std::max(maxn, sg.n);
  // device d rebuilds blocks [d * per, (d + 1) * per) of every segment
  const size_t D = (dev_.size() > 1 && maxn >= 2 * dev_.size()) ? dev_.size() : 1;
  auto part = [&](size_t d) {
    std::vector<memo_ec_rebuild_segment> mine;
    for (const auto& sg : segs) {
      const size_t per = (sg.n + D - 1) / D, b0 = std::min(sg.n, d * per), cnt = std::min(per, sg.n - b0);
      if (cnt == 0) continue;
      memo_ec_rebuild_segment x = sg;
      x.n = cnt;
      x.surv = sg.surv + b0 * sg.k * sg.S;
      x.out = sg.out + b0 * (size_t)sg.e * sg.S;
      if (!sg.uniform) {
        x.surv_idx = sg.surv_idx + b0 * sg.k;
        x.lost_idx = sg.lost_idx + b0 * (size_t)sg.e;
      }
      mine.push_back(x);
    }
    return mine;
  };
  auto run = [&](size_t dslot, const std::vector<memo_ec_rebuild_segment>& mine) {
    auto* c = acquire(dslot);
    int rc = MEMO_EC_OK;
    for (size_t i = 0; i < mine.size() && rc == MEMO_EC_OK; i += MEMO_EC_MAX_REBUILD_SEGMENTS) {
      const int cnt = (int)std::min<size_t>(MEMO_EC_MAX_REBUILD_SEGMENTS, mine.size() - i);
      rc = memo_ec_rebuild_segments(c, cnt, mine.data() + i, where);
    }
    release(dslot, c);
    return rc;
  };
  if (D == 1) {
    const size_t d = dev_.size() == 1 ? 0 : rr_++ % dev_.size();
    check(run(d, part(0)), "rebuild_segments");
  } else {
    std::vector<int> rc(D, MEMO_EC_OK);
    std::vector<std::thread> ts;
    for (size_t d = 0; d < D; ++d) ts.emplace_back([&, d] { rc[d] = run(d, part(d)); });
    for (auto& t : ts) t.join();
    for (int r : rc) check(r, "rebuild_segments");
  }
  ++segments_calls_;
  for (const auto& sg : segs) uniform_segments_ += sg.uniform ? 1 : 0;
}

// ------------------------------------------------------- pinned arena
PinnedArena::Lease& PinnedArena::Lease::operator=(Lease&& o) noexcept {
  if (this != &o) {
    if (a_ && p_) a_->put(p_, cap_, pinned_);
    a_ = o.a_;
    p_ = o.p_;
    cap_ = o.cap_;
    pinned_ = o.pinned_;
    o.a_ = nullptr;
    o.p_ = nullptr;
  }
  return *this;
}

PinnedArena::Lease::~Lease() {
  if (a_ && p_) a_->put(p_, cap_, pinned_);
}

void PinnedArena::release(const Buf& b) {
  if (b.pinned) memo_ec_host_free(b.p);
  else std::free(b.p);
}

PinnedArena::~PinnedArena() {
  for (auto& b : free_) release(b);
}

PinnedArena::Lease PinnedArena::lease(size_t bytes) {
  ++leases_;
  bytes = std::max<size_t>(bytes, 64);
  {
    std::lock_guard<std::mutex> g(mu_);
    size_t best = free_.size();
    for (size_t i = 0; i < free_.size(); ++i)
      if (free_[i].cap >= bytes && (best == free_.size() || free_[i].cap < free_[best].cap)) best = i;
    if (best != free_.size()) {
      const Buf b = free_[best];
      free_.erase(free_.begin() + best);
      return Lease(this, b.p, b.cap, b.pinned);
    }
  }
  // round up (fewer distinct sizes to keep) and pin; ordinary memory if the
  // pinned allocation fails
  const size_t cap = bytes <= (1u << 20) ? (size_t)1 << 20 : (bytes + (16u << 20) - 1) & ~(size_t)((16u << 20) - 1);
  if (void* p = memo_ec_host_alloc(cap)) return Lease(this, static_cast<uint8_t*>(p), cap, true);
  void* p = std::malloc(cap);
  if (!p) throw Error("erasure: out of host memory");
  return Lease(this, static_cast<uint8_t*>(p), cap, false);
}

size_t PinnedArena::kept_bytes() const {
  std::lock_guard<std::mutex> g(mu_);
  size_t n = 0;
  for (auto& b : free_) n += b.cap;
  return n;
}

void PinnedArena::put(uint8_t* p, size_t cap, bool pinned) {
  Buf drop{nullptr, 0, false};
  if (cap > kKeepMaxBytes) {  // an outsized lease is not worth holding pinned
    release({p, cap, pinned});
    return;
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    free_.push_back({p, cap, pinned});
    if (free_.size() > keep_) {  // keep the largest buffers
      auto small = std::min_element(free_.begin(), free_.end(),
                                    [](const Buf& a, const Buf& b) { return a.cap < b.cap; });
      drop = *small;
      free_.erase(small);
    }
  }
  if (drop.p) release(drop);
}

// ---------------------------------------------------------- shard format
uint32_t crc32c(const uint8_t* p, size_t n, uint32_t crc) {
  uint64_t c = crc ^ 0xFFFFFFFFu;
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t v;
    std::memcpy(&v, p + i, 8);
    c = _mm_crc32_u64(c, v);
  }
  uint32_t c32 = (uint32_t)c;
  for (; i < n; ++i) c32 = _mm_crc32_u8(c32, p[i]);
  return c32 ^ 0xFFFFFFFFu;
}

namespace {
constexpr size_t kCrcAt = 124;
uint32_t shard_crc(const uint8_t* wire, size_t S) {
  return crc32c(wire + ShardHeader::kSize, S, crc32c(wire, kCrcAt));
}
}  // namespace

Buffer encode_shard(const ShardHeader& h, const uint8_t* payload) { return encode_shard(h, payload, h.index); }

Buffer encode_shard(const ShardHeader& h, const uint8_t* payload, int index) {
  Buffer w(ShardHeader::kSize + h.shard_size);
  frame_shard(h, payload, index, w.data());
  return w;
}

void frame_shard(const ShardHeader& h, const uint8_t* payload, int index, uint8_t* w) {
  if (h.salt.size() > 32) throw Error("shard: salt longer than 32 bytes");
  std::memset(w, 0, ShardHeader::kSize);
  std::memcpy(w + ShardHeader::kSize, payload, h.shard_size);
  std::memcpy(w, "MECS", 4);
  w[4] = ShardHeader::kVersion;
  w[5] = h.k;
  w[6] = h.m;
  w[7] = (uint8_t)index;
  std::memcpy(w + 8, &h.block_size, 8);
  std::memcpy(w + 16, &h.shard_size, 8);
  std::memcpy(w + 24, h.address.value.data(), 32);
  const uint32_t sl = (uint32_t)h.salt.size();
  std::memcpy(w + 56, &sl, 4);
  if (sl) std::memcpy(w + 60, h.salt.data(), sl);
  std::memcpy(w + 92, h.owner.value.data(), 32);
  const uint32_t crc = shard_crc(w, h.shard_size);
  std::memcpy(w + kCrcAt, &crc, 4);
}

ShardHeader decode_shard_header(const uint8_t* w, size_t n) {
  if (n < ShardHeader::kSize || std::memcmp(w, "MECS", 4) != 0) throw ValidationFailed("shard: bad magic");
  ShardHeader h;
  h.version = w[4];
  h.k = w[5];
  h.m = w[6];
  h.index = w[7];
  std::memcpy(&h.block_size, w + 8, 8);
  std::memcpy(&h.shard_size, w + 16, 8);
  h.address = Address(w + 24, 0, false);
  uint32_t sl;
  std::memcpy(&sl, w + 56, 4);
  if (h.version != ShardHeader::kVersion) throw ValidationFailed("shard: unknown version");
  if (sl > 32) throw ValidationFailed("shard: bad salt length");
  h.salt.assign(w + 60, w + 60 + sl);
  h.owner = Address(w + 92, 0, false);
  std::memcpy(&h.crc, w + kCrcAt, 4);
  if (h.k < 1 || h.index >= h.k + h.m) throw ValidationFailed("shard: bad geometry");
  if (h.shard_size != memo_ec_shard_size(h.block_size, h.k))
    throw ValidationFailed("shard: size does not match block size");
  return h;
}

ShardHeader decode_shard_view(const uint8_t* w, size_t n, const uint8_t** payload) {
  ShardHeader h = decode_shard_header(w, n);
  if (n != ShardHeader::kSize + h.shard_size) throw ValidationFailed("shard: truncated");
  if (shard_crc(w, h.shard_size) != h.crc) throw ValidationFailed("shard: checksum mismatch");
  if (payload) *payload = w + ShardHeader::kSize;
  return h;
}

ShardHeader decode_shard(const Buffer& w, const uint8_t** payload) {
  return decode_shard_view(w.data(), w.size(), payload);
}

ShardKeys::ShardKeys(const Address& a) {
  static const uint8_t tag[16] = {'m', 'e', 'm', 'o', '-', 'e', 'c', '-', 's', 'h', 'a', 'r', 'd', 0, 0, 0};
  base = sha256(a.value.data(), 32, tag, sizeof tag);
}

Key ShardKeys::operator()(int index) const {
  std::array<uint8_t, 32> v = base;
  v[0] ^= (uint8_t)index;
  return Address(v.data(), flags::immutable_block, true);
}

Key shard_key(const Address& a, int index) { return ShardKeys(a)(index); }

// ------------------------------------------------------------ thread pool
ThreadPool::ThreadPool(int n) {
  for (int i = 0; i < std::max(1, n); ++i) ts_.emplace_back([this] { worker(); });
}

ThreadPool::~ThreadPool() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : ts_) t.join();
}

void ThreadPool::worker() {
  for (;;) {
    std::function<void()> f;
    {
      std::unique_lock<std::mutex> l(mu_);
      cv_.wait(l, [&] { return stop_ || !q_.empty(); });
      if (stop_ && q_.empty()) return;
      f = std::move(q_.front());
      q_.pop_front();
    }
    f();
  }
}

// Items are claimed from a shared counter by up to `threads` pool tasks and
// by the calling thread itself, so n tiny items cost a few atomic increments
// per thread, not n queue round trips.  The caller returns once every item has run; tasks
// that start late find no item left and only drop their reference to the
// shared state.
void ThreadPool::parallel_for(size_t n, const std::function<void(size_t)>& fn) {
  if (n == 0) return;
  struct State {
    std::atomic<size_t> next{0};
    std::mutex dm;
    std::condition_variable dcv;
    size_t done = 0;
    std::exception_ptr err;
  };
  auto st = std::make_shared<State>();
  const std::function<void(size_t)>* f = &fn;
  // items are claimed `grain` at a time: about 8 claims per thread, so that
  // thousands of small items do not all meet on the shared counter's line
  const size_t grain = std::max<size_t>(1, n / (8 * (ts_.size() + 1)));
  auto work = [st, f, n, grain] {
    size_t mine = 0;
    for (;;) {
      const size_t i0 = st->next.fetch_add(grain);
      if (i0 >= n) break;
      for (size_t i = i0; i < std::min(n, i0 + grain); ++i) {
        try {
          (*f)(i);
        } catch (...) {
          std::lock_guard<std::mutex> g(st->dm);
          if (!st->err) st->err = std::current_exception();
        }
        ++mine;
      }
    }
    if (mine) {
      std::lock_guard<std::mutex> g(st->dm);
      st->done += mine;
      if (st->done == n) st->dcv.notify_all();
    }
  };
  const size_t helpers = std::min(n, ts_.size()) - (n <= ts_.size() ? 1 : 0);
  {
    std::lock_guard<std::mutex> g(mu_);
    for (size_t t = 0; t < helpers; ++t) q_.push_back(work);
  }
  cv_.notify_all();
  work();
  std::unique_lock<std::mutex> l(st->dm);
  st->dcv.wait(l, [&] { return st->done == n; });
  if (st->err) std::rethrow_exception(st->err);
}

// --------------------------------------------------------------- plugin
namespace {
enum MemberEvent { kDiscovered = 0, kDisappeared = 1, kAppeared = 2, kUnderPlaced = 3 };
}

ErasureConsensus::ErasureConsensus(std::unique_ptr<Consensus> backend, Overlay& overlay,
                                   ErasureOptions o)
    : StackedConsensus(std::move(backend)),
      overlay_(overlay),
      o_(o),
      codec_(o.device, 4),
      pool_(o.threads) {
  if (o_.k < 1 || o_.m < 1 || o_.k > MEMO_EC_MAX_K || o_.m > MEMO_EC_MAX_M)
    throw Error("erasure: bad (k, m)");
  if (o_.fetch_hedge < 0 || o_.verify_subsets < 0) throw Error("erasure: bad fetch-hedge / verify-subsets");
  // elle::os::getenv("INFINIT_DISABLE_BALANCED_TRANSFERS", false) (Paxos.cc:488-489)
  if (const char* v = std::getenv("INFINIT_DISABLE_BALANCED_TRANSFERS"))
    if (*v && std::string(v) != "0" && std::string(v) != "false") o_.balanced_transfers = false;
  // the index first: rescan() may throw (silo listing), and must do so before
  // any thread of this object exists
  if (o_.rescan) rescan();
  bthread_ = std::thread([this] { batcher_loop(); });
  mthread_ = std::thread([this] { membership_loop(); });
  Overlay::Handlers h;
  h.discovered = [this](const Address& id) { post(kDiscovered, id); };
  h.disappeared = [this](const Address& id) { post(kDisappeared, id); };
  h.appeared = [this](const Address& id) { post(kAppeared, id); };
  sub_token_ = overlay_.subscribe(std::move(h));
  // blocks the rescan found under-placed go to the nodes present now, as
  // they would to a newcomer
  if (o_.rescan && o_.auto_expand) post(kDiscovered, Address());
}

ErasureConsensus::~ErasureConsensus() {
  overlay_.unsubscribe(sub_token_);
  {
    std::lock_guard<std::mutex> g(mmu_);
    mstop_ = true;
  }
  mcv_.notify_all();
  mthread_.join();
  {
    std::lock_guard<std::mutex> g(bmu_);
    bstop_ = true;
  }
  bcv_.notify_all();
  bthread_.join();
}

// ------------------------------------------------------------ shard peer
ShardLocal::ShardLocal(std::unique_ptr<Local> backend) : Local(*backend), backend_(std::move(backend)) {}

void ShardLocal::validate(const Key& k, const uint8_t* v, size_t n) const {
  if (n < 4 || std::memcmp(v, "MECS", 4) != 0) return backend_->validate(k, v, n);
  const ShardHeader h = decode_shard_view(v, n, nullptr);  // geometry, size, CRC32C
  if (shard_key(h.address, h.index) != k) throw ValidationFailed("shard: stored under a foreign key");
  // validate with the previous value, if any: a shard replaces a shard only
  // (a repair rewriting a damaged copy), never another kind of value
  bool other = false;
  auto prev = [&](const uint8_t* p, size_t pn) { other = pn < 4 || std::memcmp(p, "MECS", 4) != 0; };
  if (storage().read_prefix(k, 4, prev) && other) throw ValidationFailed("shard: key holds another kind of value");
}

std::unique_ptr<Local> make_shard_local(std::unique_ptr<Silo> storage) {
  return std::make_unique<ShardLocal>(make_replica_local(std::move(storage)));
}

std::unique_ptr<Local> ErasureConsensus::make_local(std::optional<int> port,
                                                    std::optional<IpAddress> listen_address,
                                                    std::unique_ptr<Silo> storage) {
  return std::make_unique<ShardLocal>(backend_->make_local(port, std::move(listen_address), std::move(storage)));
}

namespace {
struct ErasureStat : Consensus::Stat {
  std::string text;
  std::string json() const override { return text; }
};
}  // namespace

std::unique_ptr<Consensus::Stat> ErasureConsensus::stat(const Address& a) {
  auto st = std::make_unique<ErasureStat>();
  if (a.mutable_block()) {
    auto b = backend_->stat(a);
    st->text = b->json();
    return st;
  }
  Placement pl;
  bool placed = false;
  {
    std::shared_lock<std::shared_mutex> g(index_mu_);
    auto it = index_.find(a);
    if (it != index_.end()) {
      pl = it->second;
      placed = true;
    }
  }
  std::string holders;
  int reachable = 0;
  for (size_t i = 0; i < pl.holder.size(); ++i) {
    holders += std::string(i ? " " : "") + (pl.holder[i] ? pl.holder[i].hex() : "-");
    if (pl.holder[i])
      if (auto nd = overlay_.node(pl.holder[i]))
        reachable += nd->up && !nd->evicted;
  }
  st->text = to_json({{"placed", placed ? "1" : "0"},
                      {"k", std::to_string(o_.k)},
                      {"m", std::to_string(o_.m)},
                      {"block_size", std::to_string(pl.B)},
                      {"holders", holders},
                      {"reachable", std::to_string(reachable)}});
  return st;
}

std::string ErasureConsensus::redundancy() {
  char f[32];
  std::snprintf(f, sizeof f, "%.4g", double(o_.k + o_.m) / o_.k);
  return to_json({{"type", "erasure"},
                  {"k", std::to_string(o_.k)},
                  {"m", std::to_string(o_.m)},
                  {"desired_factor", f}});
}

size_t ErasureConsensus::under_placed() const {
  std::shared_lock<std::shared_mutex> g(index_mu_);
  size_t n = 0;
  for (auto& kv : index_)
    n += std::any_of(kv.second.holder.begin(), kv.second.holder.end(), [](const Address& h) { return !h; });
  return n;
}

std::string ErasureConsensus::stats() { return stats_text(); }

std::string ErasureConsensus::stats_text() const {
  size_t blocks, under = 0;
  std::string sample;
  {
    std::shared_lock<std::shared_mutex> g(index_mu_);
    blocks = index_.size();
    size_t ns = 0;
    for (auto& kv : index_)
      if (std::any_of(kv.second.holder.begin(), kv.second.holder.end(), [](const Address& h) { return !h; })) {
        ++under;
        if (ns++ < 10) sample += (sample.empty() ? "" : " ") + kv.first.hex();
      }
  }
  return to_json({{"blocks", std::to_string(blocks)},
                  {"under_placed", std::to_string(under)},
                  {"sample_under_placed", sample},
                  {"segments_calls", std::to_string(codec_.segments_calls())},
                  {"stored", std::to_string(stored_.load())},
                  {"fetched", std::to_string(fetched_.load())},
                  {"decoded", std::to_string(decoded_.load())},
                  {"repaired", std::to_string(repaired_)},
                  {"evictions", std::to_string(evictions_)},
                  {"subset_recoveries", std::to_string(subset_recoveries_)},
                  {"corrupt_shards_rewritten", std::to_string(corrupt_rewritten_)},
                  {"pending_evictions", std::to_string(pending_evictions())},
                  {"encode_calls", std::to_string(codec_.encode_calls())},
                  {"rebuild_calls", std::to_string(codec_.rebuild_calls())}});
}

Buffer ErasureConsensus::padded(const Block& b, size_t S) const {
  Buffer p((size_t)o_.k * S, 0);
  std::copy(b.data.begin(), b.data.end(), p.begin());
  return p;
}

ShardHeader ErasureConsensus::header_of(const Address& a, const Placement& pl, int index) const {
  ShardHeader h;
  h.k = (uint8_t)o_.k;
  h.m = (uint8_t)o_.m;
  h.index = (uint8_t)index;
  h.block_size = pl.B;
  h.shard_size = memo_ec_shard_size(pl.B, o_.k);
  h.address = a;
  h.salt = pl.salt;
  h.owner = pl.owner;
  return h;
}

std::vector<Address> ErasureConsensus::swap_placement_locked(const Address& a, Placement pl) {
  std::vector<Address> old;
  auto it = index_.find(a);
  if (it != index_.end()) {
    old = std::move(it->second.holder);
    it->second = std::move(pl);
  } else {
    index_.emplace(a, std::move(pl));
  }
  return old;
}

std::vector<Address> ErasureConsensus::erase_placement_locked(const Address& a) {
  std::vector<Address> old;
  auto it = index_.find(a);
  if (it == index_.end()) return old;
  old = std::move(it->second.holder);
  index_.erase(it);
  return old;
}

size_t ErasureConsensus::node_blocks(const Address& node) const { return nodes_.count(node); }

// ------------------------------------------------------------ node index
NodeIndex::Stripe& NodeIndex::stripe(const Address& node) const {
  return st_[AddressHash()(node) % kStripes];
}

void NodeIndex::update(const Address& block, const std::vector<Address>& old_h,
                       const std::vector<Address>& new_h) {
  auto has = [](const std::vector<Address>& v, const Address& x) {
    return std::find(v.begin(), v.end(), x) != v.end();
  };
  for (size_t i = 0; i < old_h.size(); ++i) {
    const Address& h = old_h[i];
    if (!h || has(new_h, h) || std::find(old_h.begin(), old_h.begin() + i, h) != old_h.begin() + i)
      continue;
    Stripe& s = stripe(h);
    std::lock_guard<std::mutex> g(s.mu);
    auto it = s.m.find(h);
    if (it == s.m.end()) continue;
    it->second.erase(block);
    if (it->second.empty()) s.m.erase(it);
  }
  for (const Address& h : new_h) {
    if (!h || has(old_h, h)) continue;
    Stripe& s = stripe(h);
    std::lock_guard<std::mutex> g(s.mu);
    s.m[h].insert(block);
  }
}

void NodeIndex::update_many(const std::vector<Change>& changes, ThreadPool* pool) {
  auto has = [](const std::vector<Address>& v, const Address& x) {
    return std::find(v.begin(), v.end(), x) != v.end();
  };
  // (holder, block, add?) per stripe, built per part of `changes` (in
  // parallel for a large batch) and applied stripe by stripe, parts in order
  using Op = std::tuple<const Address*, const Address*, bool>;
  const size_t nc = changes.size();
  const size_t parts = pool && nc >= 2048 ? std::min<size_t>(pool->size() + 1, nc / 1024) : 1;
  std::vector<std::array<std::vector<Op>, kStripes>> ops(parts);
  auto build = [&](size_t p) {
    for (size_t ci = p * nc / parts; ci < (p + 1) * nc / parts; ++ci) {
      const Change& c = changes[ci];
      // holders that stayed in place need no membership test (a repair
      // moves e of k + m)
      auto same_at = [&](const std::vector<Address>& v, size_t i, const Address& h) {
        return i < v.size() && v[i] == h;
      };
      for (size_t i = 0; i < c.old_h.size(); ++i) {
        const Address& h = c.old_h[i];
        if (!h || same_at(c.new_h, i, h) || has(c.new_h, h) ||
            std::find(c.old_h.begin(), c.old_h.begin() + i, h) != c.old_h.begin() + i)
          continue;
        ops[p][AddressHash()(h) % kStripes].emplace_back(&h, &c.block, false);
      }
      for (size_t i = 0; i < c.new_h.size(); ++i) {
        const Address& h = c.new_h[i];
        if (h && !same_at(c.old_h, i, h) && !has(c.old_h, h))
          ops[p][AddressHash()(h) % kStripes].emplace_back(&h, &c.block, true);
      }
    }
  };
  if (parts > 1) pool->parallel_for(parts, build);
  else build(0);
  std::vector<size_t> busy;
  size_t nops = 0;
  for (size_t si = 0; si < kStripes; ++si) {
    size_t here = 0;
    for (auto& op : ops) here += op[si].size();
    if (here) busy.push_back(si);
    nops += here;
  }
  auto apply = [&](size_t t) {
    const size_t si = busy[t];
    Stripe& s = st_[si];
    std::lock_guard<std::mutex> g(s.mu);
    for (auto& part : ops)
      for (auto& [h, b, add] : part[si]) {
        if (add) {
          s.m[*h].insert(*b);
        } else {
          auto it = s.m.find(*h);
          if (it == s.m.end()) continue;
          it->second.erase(*b);
          if (it->second.empty()) s.m.erase(it);
        }
      }
  };
  if (pool && busy.size() > 1 && nops >= 256) pool->parallel_for(busy.size(), apply);
  else
    for (size_t t = 0; t < busy.size(); ++t) apply(t);
}

std::vector<Address> NodeIndex::blocks(const Address& node) const {
  Stripe& s = stripe(node);
  std::lock_guard<std::mutex> g(s.mu);
  auto it = s.m.find(node);
  return it == s.m.end() ? std::vector<Address>() : std::vector<Address>(it->second.begin(), it->second.end());
}

size_t NodeIndex::count(const Address& node) const {
  Stripe& s = stripe(node);
  std::lock_guard<std::mutex> g(s.mu);
  auto it = s.m.find(node);
  return it == s.m.end() ? 0 : it->second.size();
}

void ErasureConsensus::on_rebalanced(std::function<void(const Address&)> f) {
  std::lock_guard<std::mutex> g(repair_mu_);
  rebalanced_ = std::move(f);
}

void ErasureConsensus::on_under_placed(std::function<void(const Address&, int)> f) {
  std::lock_guard<std::mutex> g(repair_mu_);
  under_placed_ = std::move(f);
}

void ErasureConsensus::notify_under_placed(const std::vector<std::pair<Address, int>>& v) {
  if (v.empty()) return;
  std::lock_guard<std::mutex> g(repair_mu_);
  if (under_placed_)
    for (auto& x : v) under_placed_(x.first, x.second);
}

// The batcher thread: gathers concurrent store() calls (up to batch_max
// blocks or batch_window_us) and encodes each same-shard-size group with one
// GPU call -- the GPU needs many blocks per launch to stream at HBM speed.
void ErasureConsensus::batcher_loop() {
  for (;;) {
    std::vector<EncodeJob*> jobs;
    {
      std::unique_lock<std::mutex> l(bmu_);
      bcv_.wait(l, [&] { return bstop_ || !bq_.empty(); });
      if (bstop_ && bq_.empty()) return;
      const auto deadline =
          std::chrono::steady_clock::now() + std::chrono::microseconds(o_.batch_window_us);
      while ((int)bq_.size() < o_.batch_max && !bstop_ &&
             bcv_.wait_until(l, deadline) != std::cv_status::timeout) {
      }
      while (!bq_.empty() && (int)jobs.size() < o_.batch_max) {
        jobs.push_back(bq_.front());
        bq_.pop_front();
      }
    }
    std::map<int, std::vector<EncodeJob*>> by_s;
    for (auto* j : jobs) by_s[size_bucket(memo_ec_shard_size(j->block->data.size(), o_.k))].push_back(j);
    for (auto& g : by_s) {
      const size_t n = g.second.size();
      size_t S = 0;
      for (auto* j : g.second) S = std::max(S, memo_ec_shard_size(j->block->data.size(), o_.k));
      try {
        auto data = arena_.lease(n * o_.k * S), parity = arena_.lease(n * o_.m * S);
        for (size_t i = 0; i < n; ++i) {
          const auto& d = g.second[i]->block->data;
          copy_padded(d, o_.k, memo_ec_shard_size(d.size(), o_.k), data.data() + i * o_.k * S, S);
        }
        codec_.encode(o_.k, o_.m, S, n, data.data(), parity.data(), data.pinned() && parity.pinned());
        for (size_t i = 0; i < n; ++i) {
          const size_t Sb = memo_ec_shard_size(g.second[i]->block->data.size(), o_.k);
          Buffer p((size_t)o_.m * Sb);
          for (int r = 0; r < o_.m; ++r)
            std::copy(parity.data() + (i * o_.m + r) * S, parity.data() + (i * o_.m + r) * S + Sb,
                      p.begin() + (size_t)r * Sb);
          g.second[i]->parity.set_value(std::move(p));
        }
      } catch (...) {
        for (auto* j : g.second) j->parity.set_exception(std::current_exception());
      }
    }
  }
}

// Send shard i to owner i (send_immutable_block's fan-out, Paxos.cc:324-360):
// a batch of one, recorded at once.
void ErasureConsensus::place(const Block& b, const uint8_t* parity) {
  const size_t S = memo_ec_shard_size(b.data.size(), o_.k);
  const Buffer own = padded(b, S);  // the block's own shards, zero-padded
  std::vector<Placed> placed(1);
  const std::exception_ptr err = place_batch({&b}, own.data(), parity, S, placed);
  commit_placements(placed);
  if (err) std::rethrow_exception(err);
}

std::exception_ptr ErasureConsensus::place_batch(const std::vector<const Block*>& bs, const uint8_t* data,
                                                 const uint8_t* parity, size_t S,
                                                 std::vector<Placed>& placed) {
  const int k = o_.k, m = o_.m, total = k + m;
  const size_t n = bs.size();
  PhaseTimer tm("place_batch");
  std::vector<std::vector<std::shared_ptr<Node>>> owners(n);
  std::vector<std::optional<ShardKeys>> keys(n);
  std::vector<ShardHeader> hdr(n);
  pool_.parallel_for(n, [&](size_t i) {
    const Block& b = *bs[i];
    owners[i] = overlay_.allocate(b.address, total);
    keys[i].emplace(b.address);
    Placement pl;
    pl.B = b.data.size();
    pl.salt = b.salt;
    pl.owner = b.owner;
    hdr[i] = header_of(b.address, pl, 0);
  });
  tm.lap("owners");
  // an owner's shards as runs of at most `run` (a few tasks per owner keep
  // every pool thread busy; each run still meets its node alone)
  std::unordered_map<Node*, std::vector<uint32_t>> by_node;
  size_t entries = 0;
  for (size_t i = 0; i < n; ++i)
    if ((int)owners[i].size() >= k)
      for (size_t j = 0; j < owners[i].size(); ++j) {
        by_node[owners[i][j].get()].push_back((uint32_t)(i * total + j));
        ++entries;
      }
  const size_t run = std::max<size_t>(32, entries / (4 * std::max<size_t>(1, pool_.size())) + 1);
  std::vector<std::pair<Node*, std::pair<const uint32_t*, size_t>>> tasks;
  for (auto& [nd, v] : by_node)
    for (size_t o = 0; o < v.size(); o += run) tasks.push_back({nd, {v.data() + o, std::min(run, v.size() - o)}});
  std::vector<uint8_t> ok(n * total, 0);
  tm.lap("group");
  // Small shards are framed a run at a time into one buffer (up to
  // kFrameRunBytes) that the run's silo values share: one allocation per
  // run instead of one per shard.  Large shards keep a buffer each (a
  // shared run would stay allocated until its last shard is erased).
  const size_t W = ShardHeader::kSize + S;
  const size_t per_frame = W <= kFrameShardMax ? std::max<size_t>(1, kFrameRunBytes / W) : 0;
  pool_.parallel_for(tasks.size(), [&](size_t t) {
    Node* nd = tasks[t].first;
    const auto [e0, ne] = tasks[t].second;
    auto payload = [&](uint32_t e) {
      const size_t i = e / total;
      const int j = (int)(e % total);
      return j < k ? data + (i * k + j) * S : parity + (i * m + (j - k)) * S;
    };
    for (size_t x0 = 0; x0 < ne;) {
      const size_t cnt = per_frame ? std::min(per_frame, ne - x0) : 1;
      std::shared_ptr<uint8_t> run;
      if (per_frame) {
        run.reset(new uint8_t[cnt * W], std::default_delete<uint8_t[]>());
        for (size_t x = 0; x < cnt; ++x) {
          const uint32_t e = e0[x0 + x];
          frame_shard(hdr[e / total], payload(e), (int)(e % total), run.get() + x * W);
        }
      }
      for (size_t x = 0; x < cnt; ++x) {
        const uint32_t e = e0[x0 + x];
        const size_t i = e / total;
        const int j = (int)(e % total);
        try {
          // a slot is W bytes; the block's own shard may be smaller (a batch
          // mixes shard sizes within one bucket)
          if (per_frame)
            nd->store_shared((*keys[i])(j), std::shared_ptr<const uint8_t>(run, run.get() + x * W),
                             ShardHeader::kSize + hdr[i].shard_size);
          else nd->store((*keys[i])(j), encode_shard(hdr[i], payload(e), j));
          ok[e] = 1;
        } catch (Error&) {
          // unreachable (Unavailable) or refused (silo::InsufficientSpace, ...):
          // a shard not placed, so the placement below records what did land
        }
      }
      x0 += cnt;
    }
  });
  tm.lap("stores");
  std::exception_ptr err;
  size_t stored = 0;
  for (size_t i = 0; i < n; ++i) {
    const Block& b = *bs[i];
    if ((int)owners[i].size() < k) {
      if (!err)
        err = std::make_exception_ptr(TooFewPeers("erasure: " + std::to_string(owners[i].size()) +
                                                  " reachable owners, need " + std::to_string(k)));
      continue;
    }
    Placed& d = placed[i];
    d.a = b.address;
    d.pl.B = b.data.size();
    d.pl.salt = b.salt;
    d.pl.owner = b.owner;
    d.pl.holder.assign(total, Address());
    int reached = 0;
    for (size_t j = 0; j < owners[i].size(); ++j)
      if (ok[i * total + j]) {
        d.pl.holder[j] = owners[i][j]->id;
        ++reached;
      }
    d.set = true;
    if (reached < k) {
      if (!err)
        err = std::make_exception_ptr(TooFewPeers("erasure: stored " + std::to_string(reached) +
                                                  " shards, need " + std::to_string(k)));
    } else {
      ++stored;
    }
  }
  stored_ += stored;
  return err;
}

void ErasureConsensus::commit_placements(std::vector<Placed>& placed) {
  std::vector<NodeIndex::Change> ch;
  ch.reserve(placed.size());
  std::vector<Address> under;  // stored (>= k shards) but on fewer than k+m owners
  {
    std::unique_lock<std::shared_mutex> g(index_mu_);
    for (Placed& p : placed) {
      if (!p.set) continue;
      const int held = (int)std::count_if(p.pl.holder.begin(), p.pl.holder.end(),
                                          [](const Address& h) { return (bool)h; });
      if (held >= o_.k && held < o_.k + o_.m) under.push_back(p.a);
      NodeIndex::Change c;
      c.block = p.a;
      c.new_h = p.pl.holder;
      c.old_h = swap_placement_locked(p.a, std::move(p.pl));
      ch.push_back(std::move(c));
    }
  }
  nodes_.update_many(ch, &pool_);
  if (o_.auto_expand)
    for (auto& a : under) post(kUnderPlaced, a);
}

void ErasureConsensus::_store(std::unique_ptr<Block> block, StoreMode mode,
                              std::unique_ptr<ConflictResolver> resolver) {
  if (!block) throw Error("erasure: store of a null block");
  if (block->is_mutable || block->address.mutable_block())
    return backend_->store(std::move(block), mode, std::move(resolver));
  store_one(*block);
}

void ErasureConsensus::store_one(const Block& b) {
  if (!chb_valid(b.address, b.salt, b.owner, b.data)) throw ValidationFailed("CHB address mismatch");
  EncodeJob job{&b, {}};
  auto fut = job.parity.get_future();
  {
    std::lock_guard<std::mutex> g(bmu_);
    bq_.push_back(&job);
  }
  bcv_.notify_all();
  const Buffer parity = fut.get();
  place(b, parity.data());
}

void ErasureConsensus::store_many(const std::vector<Block>& blocks) {
  std::vector<const Block*> imm;
  for (auto& b : blocks) {
    if (b.is_mutable || b.address.mutable_block()) backend_->store(std::make_unique<Block>(b), STORE_INSERT, nullptr);
    else imm.push_back(&b);
  }
  // Chunks of up to stage_bytes of shards: the per-block host work (CHB
  // address check, copies into the batch, shard framing + stores) runs on
  // the pool over a whole chunk, and the encode is one GPU call per
  // shard-size bucket of it (thousands of 4 KiB blocks per pass: the pool's
  // fixed costs per pass stay small beside the work).
  for (size_t b0 = 0, n0 = 0; b0 < imm.size(); b0 += n0) {
    size_t bytes = 0;
    for (n0 = 0; b0 + n0 < imm.size() && (n0 == 0 || bytes < o_.stage_bytes); ++n0)
      bytes += (size_t)(o_.k + o_.m) * memo_ec_shard_size(imm[b0 + n0]->data.size(), o_.k);
    PhaseTimer tm("store_many");
    std::vector<char> valid(n0, 0);
    pool_.parallel_for(n0, [&](size_t i) {
      const Block* b = imm[b0 + i];
      valid[i] = chb_valid(b->address, b->salt, b->owner, b->data);
    });
    tm.lap("chb");
    std::map<int, std::vector<const Block*>> by_s;
    for (size_t i = 0; i < n0; ++i) {
      const Block* b = imm[b0 + i];
      if (!valid[i]) throw ValidationFailed("CHB address mismatch");
      by_s[size_bucket(memo_ec_shard_size(b->data.size(), o_.k))].push_back(b);
    }
    for (auto& g : by_s) {
      const size_t n = g.second.size();
      size_t S = 0;
      for (auto* b : g.second) S = std::max(S, memo_ec_shard_size(b->data.size(), o_.k));
      auto data = arena_.lease(n * o_.k * S), parity = arena_.lease(n * o_.m * S);
      tm.lap("alloc");
      pool_.parallel_for(n, [&](size_t i) {
        const auto& d = g.second[i]->data;
        copy_padded(d, o_.k, memo_ec_shard_size(d.size(), o_.k), data.data() + i * o_.k * S, S);
      });
      tm.lap("copy_in");
      codec_.encode(o_.k, o_.m, S, n, data.data(), parity.data(), data.pinned() && parity.pinned());
      tm.lap("encode");
      // shards straight from the batch buffers (a block's shard is the first
      // Sb bytes of its S-byte slot)
      // the shards go out on the pool; the batch's placements then enter
      // the index under one lock (also when some block fell short)
      std::vector<Placed> placed(n);
      std::exception_ptr err = place_batch(g.second, data.data(), parity.data(), S, placed);
      tm.lap("place");
      commit_placements(placed);
      tm.lap("index");
      if (err) std::rethrow_exception(err);
    }
  }
}

// Shards of block `a` until `want` distinct valid shards are in hand.
// Invalid shards count as erasures, and so do shards of another block or
// geometry: every accepted shard has the same header (but its index) as the
// placement record, or, for a block this client did not place, as the first
// shard accepted.  First from the owners the placement index records
// (Paxos::_node_blocks analogue): shard i from owner i, data shards first.
// Then, for blocks this client did not place or shards that moved, from
// every node in lookup order, in waves.  parallel = false works node by
// node (for callers already on the pool).
// With `block`, the payloads of data shards are validated on the silo's
// view and copied straight into their slots of *block (k x S, allocated on
// the first accepted shard); their entries in the result carry no bytes.
// Parity shards always come back whole (header + payload).
std::vector<std::pair<int, Buffer>> ErasureConsensus::gather_shards(const Address& a, int want,
                                                                    bool& any_down,
                                                                    ShardHeader* hdr,
                                                                    bool parallel,
                                                                    std::vector<Node*>* from,
                                                                    Buffer* block, bool index_locked) {
  const int k = o_.k, total = o_.k + o_.m;
  // the shard keys (one SHA-256 for the block), outside the parallel fetches
  std::array<Key, MEMO_EC_MAX_K + MEMO_EC_MAX_M> keys;
  {
    const ShardKeys sk(a);
    for (int i = 0; i < total; ++i) keys[i] = sk(i);
  }
  // shards in hand: got[i], their wire bytes in wires[i] (none for a data
  // shard copied into *block)
  std::array<char, MEMO_EC_MAX_K + MEMO_EC_MAX_M> got{};
  std::array<Buffer, MEMO_EC_MAX_K + MEMO_EC_MAX_M> wires;
  int ngot = 0;
  std::mutex gm;
  bool have_ref = false;
  ShardHeader ref;
  any_down = false;
  auto have = [&](int i) {
    std::lock_guard<std::mutex> g(gm);
    return got[i] != 0;
  };
  auto count = [&] {
    std::lock_guard<std::mutex> g(gm);
    return ngot;
  };
  // fetch shard i from nd; true if the node was reachable
  auto try_node = [&](const std::shared_ptr<Node>& nd, int i) -> bool {
    auto accept = [&](const uint8_t* w, size_t n) {
      const uint8_t* pay = nullptr;
      ShardHeader h;
      try {
        h = decode_shard_view(w, n, &pay);
      } catch (ValidationFailed&) {
        return;  // corrupted shard: an erasure
      }
      if (h.address != a || h.index != i || h.k != o_.k || h.m != o_.m) return;
      uint8_t* slot = nullptr;
      bool in_block = false;
      {
        std::lock_guard<std::mutex> g(gm);
        if (!have_ref) {
          ref = h;
          have_ref = true;
        } else if (!h.same_block(ref)) {
          return;  // another geometry, salt or owner: an erasure
        }
        if (got[i]) return;
        got[i] = 1;
        ++ngot;
        if (from) (*from)[i] = nd.get();
        if (block && i < k) {
          if (block->empty()) block->resize((size_t)k * ref.shard_size);
          slot = block->data() + (size_t)i * ref.shard_size;  // claimed: this thread's alone
          in_block = true;
        }
      }
      if (!in_block) wires[i].assign(w, w + n);
      else if (h.shard_size) std::memcpy(slot, pay, h.shard_size);
    };
    try {
      // in flight from this client (Paxos.cc:506-507), for the ordering below
      Counter& tr = transfers(nd.get());
      tr.add(1);
      struct Done {
        Counter& t;
        ~Done() { t.add(-1); }
      } done{tr};
      nd->try_read(keys[i], accept);
    } catch (Unavailable&) {
      std::lock_guard<std::mutex> g(gm);
      any_down = true;
      return false;
    }
    return true;
  };
  auto run = [&](size_t n, const std::function<void(size_t)>& fn) {
    if (parallel && n > 1) pool_.parallel_for(n, fn);
    else
      for (size_t t = 0; t < n && count() < want; ++t) fn(t);
  };

  std::vector<std::shared_ptr<Node>> holder(total);
  {
    // index_locked: the caller holds a reader lock across its whole parallel
    // gather (one lock for thousands of blocks instead of one each)
    std::shared_lock<std::shared_mutex> g(index_mu_, std::defer_lock);
    if (!index_locked) g.lock();
    auto it = index_.find(a);
    if (it != index_.end()) {
      ref = header_of(a, it->second, 0);
      have_ref = true;
      for (int i = 0; i < total && i < (int)it->second.holder.size(); ++i)
        if (it->second.holder[i]) holder[i] = overlay_.node(it->second.holder[i]);
    }
  }
  // the recorded holders of shards [i0, i1) worth asking (known-down ones
  // are skipped, without a fetch or an exception)
  auto candidates = [&](int i0, int i1) {
    std::vector<int> ids;
    for (int i = i0; i < i1; ++i) {
      if (!holder[i] || holder[i]->evicted || have(i)) continue;
      if (!holder[i]->up) {
        std::lock_guard<std::mutex> g(gm);
        any_down = true;
        continue;
      }
      ids.push_back(i);
    }
    return ids;
  };
  // pass 0: the data shards (no decode needed), all at once
  {
    const std::vector<int> ids = candidates(0, std::min(o_.k, total));
    run(ids.size(), [&](size_t t) { try_node(holder[ids[t]], ids[t]); });
  }
  // pass 1: only as many parity shards as the decode still needs (+ the
  // configured hedge on the first round), topped up from the remaining
  // holders while fetches fail.  The holders are shuffled, then taken in
  // order of in-flight transfers from this client, as the reference orders
  // a block's replicas (Paxos.cc:488-500; INFINIT_DISABLE_BALANCED_TRANSFERS
  // turns it off).
  if (count() < want) {
    std::vector<int> ids = candidates(o_.k, total);
    if (o_.balanced_transfers && ids.size() > 1) {
      thread_local std::mt19937_64 rng(std::random_device{}());
      std::shuffle(ids.begin(), ids.end(), rng);
      std::vector<std::pair<int, int>> load;
      for (int i : ids) load.push_back({(int)transfers(holder[i].get()).load(), i});
      std::stable_sort(load.begin(), load.end(),
                       [](const auto& x, const auto& y) { return x.first < y.first; });
      for (size_t t = 0; t < ids.size(); ++t) ids[t] = load[t].second;
    }
    size_t next = 0;
    int hedge = o_.fetch_hedge;
    while (next < ids.size()) {
      const int need = want - count();
      if (need <= 0) break;
      const size_t n = std::min(ids.size() - next, (size_t)(need + hedge));
      hedge = 0;
      run(n, [&](size_t t) { try_node(holder[ids[next + t]], ids[next + t]); });
      next += n;
    }
  }

  if (count() < want) {
    auto nodes = overlay_.lookup(a, (int)overlay_.size());
    auto from_node = [&](const std::shared_ptr<Node>& nd) {
      if (!nd->up) {
        std::lock_guard<std::mutex> g(gm);
        any_down = true;
        return;
      }
      for (int i = 0; i < total; ++i)
        if (!have(i) && !try_node(nd, i)) return;  // down: skip the node
    };
    size_t next = 0;
    while (count() < want && next < nodes.size()) {
      const size_t wave = std::min(nodes.size() - next, (size_t)std::max(total, 1));
      run(wave, [&](size_t w) { from_node(nodes[next + w]); });
      next += wave;
    }
  }
  if (hdr && have_ref) *hdr = ref;
  std::vector<std::pair<int, Buffer>> out;
  out.reserve(ngot);
  for (int i = 0; i < total; ++i)
    if (got[i]) out.emplace_back(i, std::move(wires[i]));
  return out;
}

ErasureConsensus::Gathered ErasureConsensus::collect(const Address& a, bool parallel, bool index_locked) {
  Gathered g;
  const int k = o_.k;
  try {
    bool any_down = false;
    g.shards = gather_shards(a, k, any_down, &g.h, parallel, nullptr, &g.block, index_locked);
    if (g.shards.empty()) {
      if (any_down) throw TooFewPeers("erasure: no shard reachable for " + a.hex());
      throw MissingBlock("missing block " + a.hex());
    }
    if ((int)g.shards.size() < k)
      throw TooFewPeers("erasure: " + std::to_string(g.shards.size()) +
                        " shards reachable, need " + std::to_string(k));
    std::sort(g.shards.begin(), g.shards.end(),
              [](const auto& x, const auto& y) { return x.first < y.first; });
    g.shards.resize(k);  // data shards first (sorted), then parity
    std::vector<bool> have(k, false);
    for (auto& s : g.shards)
      if (s.first < k) have[s.first] = true;
    for (int j = 0; j < k; ++j)
      if (!have[j]) g.lost.push_back((uint8_t)j);
  } catch (Error&) {
    g.err = std::current_exception();
  }
  return g;
}

const uint8_t* ErasureConsensus::Gathered::payload(size_t s) const {
  const auto& sh = shards[s];
  return sh.first < h.k ? block.data() + (size_t)sh.first * h.shard_size : sh.second.data() + ShardHeader::kSize;
}

std::unique_ptr<Block> ErasureConsensus::assemble(const Address& a, Gathered& g,
                                                  const uint8_t* rebuilt, size_t stride) {
  const int k = o_.k;
  const size_t S = g.h.shard_size;
  Buffer block = std::move(g.block);  // the data shards in hand are in place
  block.resize((size_t)k * S);
  for (size_t r = 0; r < g.lost.size(); ++r)
    std::memcpy(block.data() + (size_t)g.lost[r] * S, rebuilt + r * stride, S);
  block.resize(g.h.block_size);
  if (!chb_valid(a, g.h.salt, g.h.owner, block))
    throw AddressMismatch("erasure: reassembled block does not match its address");
  auto b = std::make_unique<Block>();
  b->address = a;
  b->data = std::move(block);
  b->salt = g.h.salt;
  b->owner = g.h.owner;
  ++fetched_;
  return b;
}

std::unique_ptr<Block> ErasureConsensus::_fetch(Address a, std::optional<int> local_version) {
  if (a.mutable_block()) return backend_->fetch(a, local_version);
  const int k = o_.k;
  Gathered g = collect(a, true);
  if (g.err) std::rethrow_exception(g.err);
  Buffer out;
  if (!g.lost.empty()) {
    // systematic shards missing: rebuild them from the k survivors (GPU)
    const size_t S = g.h.shard_size;
    std::vector<uint8_t> sidx(k);
    Buffer surv((size_t)k * S);
    for (int s = 0; s < k; ++s) {
      sidx[s] = (uint8_t)g.shards[s].first;
      std::memcpy(surv.data() + (size_t)s * S, g.payload(s), S);
    }
    out.resize(g.lost.size() * S);
    codec_.rebuild(k, o_.m, S, 1, sidx.data(), surv.data(), g.lost.data(), (int)g.lost.size(),
                   out.data());
    ++decoded_;
  }
  try {
    return assemble(a, g, out.data(), g.h.shard_size);
  } catch (AddressMismatch&) {
    if (o_.verify_subsets == 0) throw;
    return recover(a, true);
  }
}

namespace {
// Next combination c (ascending, |c| = d) of {0..n-1}; false after the last.
bool next_combination(std::vector<int>& c, int n) {
  const int d = (int)c.size();
  for (int i = d - 1; i >= 0; --i)
    if (c[i] < n - d + i) {
      ++c[i];
      for (int j = i + 1; j < d; ++j) c[j] = c[j - 1] + 1;
      return true;
    }
  return false;
}

// k-subsets of n shards in hand (positions, sorted by shard index: the
// first k are the lowest indices), in order of how many of the first k they
// replace by spares -- the first k themselves, then one wrong shard is
// found among the next k * (n - k) -- at most `limit` of them.  (The first
// k may differ from the failed attempt's: that one decoded from whichever
// parity holders answered first.)
std::vector<std::vector<int>> retry_subsets(int n, int k, int limit) {
  std::vector<std::vector<int>> out;
  const int spare = n - k;
  for (int d = 0; d <= std::min(spare, k); ++d) {
    std::vector<int> drop(d);
    for (int i = 0; i < d; ++i) drop[i] = i;
    do {
      std::vector<int> add(d);
      for (int i = 0; i < d; ++i) add[i] = i;
      do {
        if ((int)out.size() >= limit) return out;
        std::vector<int> sub;
        for (int p = 0, q = 0; p < k; ++p) {
          if (q < d && drop[q] == p) {
            ++q;
            continue;
          }
          sub.push_back(p);
        }
        for (int x : add) sub.push_back(k + x);
        out.push_back(std::move(sub));
      } while (next_combination(add, spare));
    } while (next_combination(drop, k));
  }
  return out;
}
}  // namespace

// The reassembly of `a` failed its CHB address although every shard passed
// its CRC: a holder returned a well-framed shard with the wrong bytes.  The
// reference moves on to the next replica on any error (Paxos.cc:502-517);
// with erasure coding the other shards can out-vote the wrong one.  Every
// reachable shard is fetched, k-subsets are decoded until one reassembles to
// the address (at most verify_subsets), and each shard in hand that
// disagrees with the verified block is rewritten on its holder.
std::unique_ptr<Block> ErasureConsensus::recover(const Address& a, bool parallel) {
  const int k = o_.k, m = o_.m, total = k + m;
  // k + 1 shards first (one spare out-votes one wrong shard, and a holder
  // that is down does not send the gather over the whole membership), all
  // of them when that finds no good subset
  if (k + 1 < total)
    if (auto b = recover_from(a, k + 1, parallel)) return b;
  if (auto b = recover_from(a, total, parallel)) return b;
  throw AddressMismatch("erasure: reassembled block does not match its address (no k-subset of the "
                        "reachable shards matches)");
}

std::unique_ptr<Block> ErasureConsensus::recover_from(const Address& a, int want, bool parallel) {
  const int k = o_.k, m = o_.m, total = k + m;
  const std::string what = "erasure: reassembled block does not match its address";
  bool any_down = false;
  ShardHeader h;
  std::vector<Node*> from(total, nullptr);
  auto have = gather_shards(a, want, any_down, &h, parallel, &from);
  std::sort(have.begin(), have.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
  const int n = (int)have.size();
  if (n <= k) {
    if (want < total) return nullptr;  // the wider gather may find more
    throw AddressMismatch(what + " (no spare shard to try)");
  }
  const size_t S = h.shard_size;
  std::vector<uint8_t> sidx(k), lost;
  Buffer surv((size_t)k * S), out((size_t)m * S), block;
  for (const auto& sub : retry_subsets(n, k, o_.verify_subsets)) {
    std::vector<bool> present(k, false);
    block.assign((size_t)k * S, 0);
    for (int t = 0; t < k; ++t) {
      const auto& sh = have[sub[t]];
      sidx[t] = (uint8_t)sh.first;
      const uint8_t* pay = sh.second.data() + ShardHeader::kSize;
      std::memcpy(surv.data() + (size_t)t * S, pay, S);
      if (sh.first < k) {
        present[sh.first] = true;
        std::memcpy(block.data() + (size_t)sh.first * S, pay, S);
      }
    }
    lost.clear();
    for (int j = 0; j < k; ++j)
      if (!present[j]) lost.push_back((uint8_t)j);
    if (!lost.empty()) {
      codec_.rebuild(k, m, S, 1, sidx.data(), surv.data(), lost.data(), (int)lost.size(), out.data());
      for (size_t r = 0; r < lost.size(); ++r)
        std::memcpy(block.data() + (size_t)lost[r] * S, out.data() + r * S, S);
    }
    Buffer padded_block = block;  // k x S, the verified shards
    block.resize(h.block_size);
    if (!chb_valid(a, h.salt, h.owner, block)) continue;
    // the block is verified: every shard in hand that differs from its
    // re-encoding is rewritten on the holder that served it
    Buffer parity((size_t)m * S);
    codec_.encode(k, m, S, 1, padded_block.data(), parity.data());
    const ShardKeys keys(a);
    for (const auto& sh : have) {
      const int i = sh.first;
      const uint8_t* want = i < k ? padded_block.data() + (size_t)i * S : parity.data() + (size_t)(i - k) * S;
      if (std::memcmp(sh.second.data() + ShardHeader::kSize, want, S) == 0 || !from[i]) continue;
      try {
        from[i]->store(keys(i), encode_shard(h, want, i));
        ++corrupt_rewritten_;
      } catch (Error&) {
        // unreachable now: the next fetch or repair meets it again
      }
    }
    ++subset_recoveries_;
    ++fetched_;
    auto b = std::make_unique<Block>();
    b->address = a;
    b->data = std::move(block);
    b->salt = h.salt;
    b->owner = h.owner;
    return b;
  }
  if (want < total) return nullptr;
  throw AddressMismatch(what + " (no k-subset of the " + std::to_string(n) +
                        " reachable shards matches)");
}

// Multi-address fetch: shards of all blocks gathered on the pool, then ONE
// codec call (memo_ec_rebuild_segments) for every block that misses data
// shards -- a segment per (shard-size bucket, erasure count) group, shards
// zero-padded to the group's largest, and per shared erasure pattern --
// then reassembly + CHB check on the pool; `res` is called in request
// order.  The reference hands the whole batch over at once too
// (Consensus::_fetch(vector<AddressVersion>), Consensus.cc:101-124).
void ErasureConsensus::_fetch(const std::vector<AddressVersion>& request, ReceiveBlock res) {
  const int k = o_.k, m = o_.m;
  const size_t n = request.size();
  std::vector<Address> addresses(n);
  for (size_t i = 0; i < n; ++i) addresses[i] = request[i].first;
  std::vector<std::unique_ptr<Block>> blocks(n);
  std::vector<std::exception_ptr> errs(n);
  std::vector<size_t> imm;
  for (size_t i = 0; i < n; ++i) {
    if (!addresses[i].mutable_block()) {
      imm.push_back(i);
      continue;
    }
    try {
      blocks[i] = backend_->fetch(addresses[i], request[i].second);
    } catch (Error&) {
      errs[i] = std::current_exception();
    }
  }
  PhaseTimer tm("fetch_many");
  std::vector<Gathered> g(n);
  {
    // one reader lock on the index for the whole parallel gather: a lock per
    // block is an atomic add on one shared line from every pool thread (the
    // gather tasks take no index lock of their own, and none of them waits
    // for a writer)
    std::shared_lock<std::shared_mutex> il(index_mu_);
    pool_.parallel_for(imm.size(), [&](size_t t) { g[imm[t]] = collect(addresses[imm[t]], false, true); });
  }
  tm.lap("gather");
  // degraded blocks by (S bucket, erasure pattern); patterns shared by at
  // least uniform_min blocks (a node down) take the uniform rebuild, the
  // rest group by (S bucket, e) for the per-block rebuild
  std::map<std::pair<int, std::vector<uint8_t>>, std::vector<size_t>> by_pat;
  std::vector<size_t> direct;
  for (size_t i : imm) {
    if (g[i].err) {
      errs[i] = g[i].err;
    } else if (g[i].lost.empty()) {
      direct.push_back(i);
    } else {
      std::vector<uint8_t> pat;
      for (auto& sh : g[i].shards) pat.push_back((uint8_t)sh.first);
      pat.insert(pat.end(), g[i].lost.begin(), g[i].lost.end());
      by_pat[{size_bucket(g[i].h.shard_size), std::move(pat)}].push_back(i);
    }
  }
  struct FGroup {
    int e;
    bool uniform;
    std::vector<uint8_t> pat;
    std::vector<size_t> ids;
  };
  std::vector<FGroup> groups;
  std::map<std::pair<int, size_t>, std::vector<size_t>> rest;
  for (auto& bp : by_pat) {
    const int e = (int)(bp.first.second.size() - (size_t)k);
    const size_t bytes = bp.second.size() * (size_t)k * ((size_t)64 << bp.first.first);
    if ((int)bp.second.size() >= o_.uniform_min && bytes >= o_.uniform_min_bytes)
      groups.push_back({e, true, bp.first.second, bp.second});
    else rest[{bp.first.first, (size_t)e}].insert(rest[{bp.first.first, (size_t)e}].end(),
                                                  bp.second.begin(), bp.second.end());
  }
  for (auto& r : rest) groups.push_back({(int)r.first.second, false, {}, r.second});
  auto finish = [&](size_t i, const uint8_t* rebuilt, size_t stride) {
    try {
      try {
        blocks[i] = assemble(addresses[i], g[i], rebuilt, stride);
      } catch (AddressMismatch&) {
        if (o_.verify_subsets == 0) throw;
        blocks[i] = recover(addresses[i], false);  // on this pool thread
      }
    } catch (Error&) {
      errs[i] = std::current_exception();
    }
  };
  pool_.parallel_for(direct.size(), [&](size_t t) { finish(direct[t], nullptr, 0); });
  tm.lap("assemble_direct");
  // every group's batches staged, then ONE codec call for all of them
  // (memo_ec_rebuild_segments: a segment per batch), then reassembly
  struct FBatch {
    const FGroup* grp;
    size_t b0, nb, S;
    std::vector<uint8_t> sidx, lidx;
    uint8_t* surv = nullptr;  // this batch's part of the call's two leases
    uint8_t* out = nullptr;
  };
  std::vector<FBatch> batches;
  for (auto& grp : groups)
    for (size_t b0 = 0; b0 < grp.ids.size(); b0 += o_.batch_max) {
      FBatch fb;
      fb.grp = &grp;
      fb.b0 = b0;
      fb.nb = std::min<size_t>(o_.batch_max, grp.ids.size() - b0);
      fb.S = 0;  // the batch's largest shard; smaller shards zero-padded
      for (size_t bi = 0; bi < fb.nb; ++bi) fb.S = std::max(fb.S, (size_t)g[grp.ids[b0 + bi]].h.shard_size);
      batches.push_back(std::move(fb));
    }
  // Chunks of batches with up to stage_bytes of survivors each: one
  // survivor and one output lease per chunk, carved per batch (a lease per
  // batch took a pinned allocation each beyond the arena's few kept buffers,
  // ~2 ms apiece: 240 ms for 16,384 4 KiB blocks), and ONE codec call per
  // chunk for all its batches (memo_ec_rebuild_segments: a segment per
  // batch).  A node-loss fetch of thousands of degraded blocks so stages at
  // most a chunk at a time instead of pinning GBs at once.
  std::vector<size_t> cuts{0};
  {
    size_t acc = 0;
    for (size_t x = 0; x < batches.size(); ++x) {
      const size_t sb = batches[x].nb * k * batches[x].S;
      if (acc > 0 && acc + sb > o_.stage_bytes) {
        cuts.push_back(x);
        acc = 0;
      }
      acc += sb;
    }
    if (cuts.back() != batches.size()) cuts.push_back(batches.size());
  }
  for (size_t ci = 0; ci + 1 < cuts.size(); ++ci) {
    const size_t x0 = cuts[ci], x1 = cuts[ci + 1];
    std::vector<size_t> o_surv(x1 - x0), o_out(x1 - x0);
    size_t surv_bytes = 0, out_bytes = 0;
    for (size_t x = x0; x < x1; ++x) {
      o_surv[x - x0] = surv_bytes;
      o_out[x - x0] = out_bytes;
      surv_bytes += (batches[x].nb * k * batches[x].S + 63) & ~(size_t)63;
      out_bytes += (batches[x].nb * batches[x].grp->e * batches[x].S + 63) & ~(size_t)63;
    }
    PinnedArena::Lease surv_all = arena_.lease(surv_bytes), out_all = arena_.lease(out_bytes);
    const bool pin = surv_all.pinned() && out_all.pinned();
    for (size_t x = x0; x < x1; ++x) {
      FBatch& fb = batches[x];
      const int e = fb.grp->e;
      fb.surv = surv_all.data() + o_surv[x - x0];
      fb.out = out_all.data() + o_out[x - x0];
      if (!fb.grp->uniform) {
        fb.sidx.resize(fb.nb * k);
        fb.lidx.resize(fb.nb * e);
      }
    }
    tm.lap("alloc");
    // (batch, block) pairs copied in on the pool
    std::vector<std::pair<size_t, size_t>> work;
    for (size_t x = x0; x < x1; ++x)
      for (size_t bi = 0; bi < batches[x].nb; ++bi) work.emplace_back(x, bi);
    pool_.parallel_for(work.size(), [&](size_t t) {
      FBatch& fb = batches[work[t].first];
      const size_t bi = work[t].second;
      Gathered& x = g[fb.grp->ids[fb.b0 + bi]];
      for (int s = 0; s < k; ++s) {
        uint8_t* slot = fb.surv + (bi * k + s) * fb.S;
        std::memcpy(slot, x.payload(s), x.h.shard_size);
        std::memset(slot + x.h.shard_size, 0, fb.S - x.h.shard_size);
        if (!fb.grp->uniform) fb.sidx[bi * k + s] = (uint8_t)x.shards[s].first;
      }
      if (!fb.grp->uniform) std::copy(x.lost.begin(), x.lost.end(), fb.lidx.begin() + bi * fb.grp->e);
    });
    tm.lap("copy_in");
    std::vector<memo_ec_rebuild_segment> segs;
    for (size_t x = x0; x < x1; ++x) {
      const FBatch& fb = batches[x];
      memo_ec_rebuild_segment sg{};
      sg.k = k;
      sg.m = m;
      sg.S = fb.S;
      sg.n = fb.nb;
      sg.e = fb.grp->e;
      sg.uniform = fb.grp->uniform ? 1 : 0;
      sg.surv = fb.surv;
      sg.out = fb.out;
      sg.surv_idx = fb.grp->uniform ? fb.grp->pat.data() : fb.sidx.data();
      sg.lost_idx = fb.grp->uniform ? fb.grp->pat.data() + k : fb.lidx.data();
      segs.push_back(sg);
    }
    codec_.rebuild_segments(segs, pin);
    tm.lap("rebuild");
    for (size_t x = x0; x < x1; ++x) decoded_ += batches[x].nb;
    pool_.parallel_for(work.size(), [&](size_t t) {
      FBatch& fb = batches[work[t].first];
      const size_t bi = work[t].second;
      finish(fb.grp->ids[fb.b0 + bi], fb.out + bi * fb.grp->e * fb.S, fb.S);
    });
    tm.lap("assemble");
  }
  for (size_t i = 0; i < n; ++i) res(addresses[i], std::move(blocks[i]), errs[i]);
}

void ErasureConsensus::_resign() { backend_->resign(); }

// Consensus::remove (Consensus.cc:135-164) -> Paxos::_remove ->
// Consensus::remove_many (Consensus.cc:178-240): every holder removes what
// it stores after validating the removal against it (Local::remove ->
// previous->validate_remove, Local.cc:260-278; for a CHB,
// CHB::_validate_remove, CHB.cc:203-259, here against the owner the shard
// header carries), in parallel; unreachable holders are skipped;
// MissingBlock when no holder removed anything.  A CHB's removal never
// conflicts (its validation has no conflict outcome), so the reference's
// re-sign-and-retry loop on Conflict has nothing to retry here.
void ErasureConsensus::_remove(Address a, RemoveSignature rs) {
  if (a.mutable_block()) return backend_->remove(a, std::move(rs));
  const int total = o_.k + o_.m;
  const ShardKeys keys(a);
  // (node, shard index; -1: every index) pairs to visit: the placement
  // index's holders, or, for a block this client has no placement of, the
  // nodes lookup(address, k+m) names, each asked for every shard
  struct Target {
    Node* node;
    int index;
  };
  std::vector<Target> targets;
  bool known = false;
  Address owner;
  {
    std::shared_lock<std::shared_mutex> g(index_mu_);
    auto it = index_.find(a);
    if (it != index_.end()) {
      known = true;
      owner = it->second.owner;
      for (int i = 0; i < (int)it->second.holder.size(); ++i)
        if (it->second.holder[i])
          if (auto nd = overlay_.node(it->second.holder[i])) targets.push_back({nd.get(), i});
    }
  }
  if (known) {
    // every holder would refuse an invalid removal: refuse it before
    // anything is touched (the shards and the placement stay)
    const std::string why = chb_validate_remove(a, owner, rs, owners_);
    if (!why.empty()) throw ValidationFailed("remove " + a.hex() + ": " + why);
    // forget the block first: a repair running concurrently will not
    // re-place it (evict_removed_blocks, tests/doughnut.cc:1693-1719)
    std::vector<Address> old;
    {
      std::unique_lock<std::shared_mutex> g(index_mu_);
      old = erase_placement_locked(a);
    }
    nodes_.update(a, old, {});
  } else {
    // No placement of the block here (another client stored it, or a
    // restart without rescan): every node is asked for every shard.  The
    // shards may sit past lookup(a, k+m) -- stored while top-ranked nodes
    // were down, or moved by a repair -- so the scan covers the whole
    // membership, as remove_many reaches every peer that holds the block.
    for (auto& nd : overlay_.lookup(a, (int)overlay_.size())) targets.push_back({nd.get(), -1});
  }
  std::atomic<int> removed{0};
  std::mutex emu;
  std::string refused;
  std::vector<std::pair<Address, OwedRemove>> deferred;  // holders down now
  // One removal request per node (Consensus::remove_many sends one per
  // peer, Consensus.cc:176-236), naming the shard keys it may hold; the
  // holder checks each shard against the owner its header records (a header
  // that does not parse is no shard of any block: removed).
  const auto check = [&](const Key&, const Buffer& head) {
    Address shard_owner = owner;
    try {
      shard_owner = decode_shard_header(head.data(), head.size()).owner;
    } catch (ValidationFailed&) {
    }
    return chb_validate_remove(a, shard_owner, rs, owners_);
  };
  pool_.parallel_for(targets.size(), [&](size_t t) {
    Node* nd = targets[t].node;
    const int i0 = targets[t].index < 0 ? 0 : targets[t].index;
    const int i1 = targets[t].index < 0 ? total : targets[t].index + 1;
    std::vector<Key> ks;
    for (int i = i0; i < i1; ++i) ks.push_back(keys(i));
    try {
      std::string why;
      removed += nd->remove_values(ks, ShardHeader::kSize, check, &why);
      if (!why.empty()) {
        std::lock_guard<std::mutex> g(emu);
        refused = why;
      }
    } catch (Unavailable&) {
      // the node is down: remove its shard(s) when it returns (or drop
      // the debt when it is evicted), so the block does not come back with
      // it.  For a block of unknown placement, every index it might hold.
      std::lock_guard<std::mutex> g(emu);
      deferred.push_back({nd->id, OwedRemove{a, targets[t].index, rs}});
    }
  });
  // owed removals: a known block's down holders; for a block of unknown
  // placement, the down nodes' possible shards once the removal took
  // effect somewhere (an address found nowhere owes nothing)
  if (!deferred.empty() && (known || removed.load() > 0)) {
    std::lock_guard<std::mutex> g(rm_mu_);
    for (auto& d : deferred) pending_rm_[d.first].push_back(d.second);
  }
  if (removed.load() == 0) {
    if (!refused.empty()) throw ValidationFailed("remove " + a.hex() + ": " + refused);
    if (!known || deferred.empty()) throw MissingBlock("remove: no shard of " + a.hex());
  }
}

size_t ErasureConsensus::pending_removes() const {
  std::lock_guard<std::mutex> g(rm_mu_);
  size_t n = 0;
  for (auto& kv : pending_rm_) n += kv.second.size();
  return n;
}

// Shards a removal could not reach on `node` (down at the time): erased now
// that it is back, or forgotten with its silo when it is evicted.  A shard
// is kept when the block lives again: stored again with this node holding
// it (this client's index), or with shards of it on other nodes (another
// client stored it after the removal); and when the removal's signature no
// longer validates against the owner its header records.
void ErasureConsensus::settle_removes(const Address& node, bool evicted) {
  std::vector<OwedRemove> owed;
  {
    std::lock_guard<std::mutex> g(rm_mu_);
    auto it = pending_rm_.find(node);
    if (it == pending_rm_.end()) return;
    owed.swap(it->second);
    pending_rm_.erase(it);
  }
  if (evicted) return;
  auto nd = overlay_.node(node);
  if (!nd) return;
  const int total = o_.k + o_.m;
  std::vector<OwedRemove> still;
  for (auto& r : owed) {
    // the block was stored again with this node holding that shard (a CHB
    // key is its content's): the shard is live, the debt is void
    bool restored = false;
    {
      std::shared_lock<std::shared_mutex> g(index_mu_);
      auto it = index_.find(r.block);
      if (it != index_.end())
        for (int i = 0; i < (int)it->second.holder.size(); ++i)
          restored = restored || ((r.index < 0 || r.index == i) && it->second.holder[i] == node);
    }
    if (restored) continue;
    try {
      if (held_elsewhere(r.block, node)) continue;  // stored again by another client
      const ShardKeys keys(r.block);
      std::vector<Key> ks;
      for (int i = r.index < 0 ? 0 : r.index; i < (r.index < 0 ? total : r.index + 1); ++i) ks.push_back(keys(i));
      // one request to the returned node; a shard is removed only while the
      // removal's signature validates against the owner its header records
      nd->remove_values(ks, ShardHeader::kSize, [&](const Key&, const Buffer& head) {
        Address shard_owner;
        try {
          shard_owner = decode_shard_header(head.data(), head.size()).owner;
        } catch (ValidationFailed&) {
          // no shard of any block under this key: removed
        }
        return chb_validate_remove(r.block, shard_owner, r.rs, owners_);
      });
    } catch (Unavailable&) {
      still.push_back(r);  // down again
    }
  }
  if (!still.empty()) {
    std::lock_guard<std::mutex> g(rm_mu_);
    auto& v = pending_rm_[node];
    v.insert(v.end(), still.begin(), still.end());
  }
}

bool ErasureConsensus::held_elsewhere(const Address& a, const Address& except) const {
  const int total = o_.k + o_.m;
  const ShardKeys keys(a);
  std::vector<Key> ks;
  for (int i = 0; i < total; ++i) ks.push_back(keys(i));
  // one request per node, naming every shard key of the block
  for (auto& nd : overlay_.lookup(a, (int)overlay_.size())) {
    if (nd->id == except) continue;
    try {
      if (nd->holds_any(ks)) return true;
    } catch (Unavailable&) {
    }
  }
  return false;
}

// ------------------------------------------------------------- repair
ErasureConsensus::RepairReport ErasureConsensus::repair_blocks(const std::vector<Address>& blocks,
                                                               bool include_down) {
  std::lock_guard<std::mutex> rl(repair_mu_);
  RepairReport rep;
  rep.blocks_checked = blocks.size();
  const int k = o_.k, m = o_.m, total = k + m;
  struct Todo {
    Address a;
    Placement pl;
    std::vector<int> lost;      // shards to rebuild
    std::vector<uint8_t> sidx;  // the k validated survivors' indices
    Buffer surv;                // their payloads, k x Sb, read in place from the silos
    bool skip = false;
  };
  // Chunks of blocks whose survivors are held in memory at once: up to
  // stage_bytes of shards (by the recorded block sizes), so that small blocks
  // still fill whole GPU batches per (size, e) group.
  std::vector<size_t> cuts{0};
  {
    std::shared_lock<std::shared_mutex> g(index_mu_);
    size_t acc = 0;
    for (size_t i = 0; i < blocks.size(); ++i) {
      auto it = index_.find(blocks[i]);
      acc += (size_t)k * memo_ec_shard_size(it == index_.end() ? 0 : it->second.B, k);
      if (acc >= o_.stage_bytes && i + 1 - cuts.back() >= (size_t)o_.batch_max) {
        cuts.push_back(i + 1);
        acc = 0;
      }
    }
    if (cuts.back() != blocks.size()) cuts.push_back(blocks.size());
  }
  for (size_t ci = 0; ci + 1 < cuts.size(); ++ci) {
    const size_t c0 = cuts[ci], cn = cuts[ci + 1] - c0;
    PhaseTimer tm("repair_chunk");
    std::vector<Todo> todo(cn);
    // Scan: a shard is lost when its holder is gone (null, evicted, down
    // with include_down), lacks it, or holds a copy that fails validation
    // or belongs to another block or geometry; the first k valid shards
    // found are the survivors.
    std::shared_lock<std::shared_mutex> scan_lock(index_mu_);  // for the whole scan (see _fetch)
    pool_.parallel_for(cn, [&](size_t t) {
      Todo& x = todo[t];
      x.a = blocks[c0 + t];
      {
        auto it = index_.find(x.a);
        if (it == index_.end()) {
          x.skip = true;  // removed meanwhile
          return;
        }
        x.pl = it->second;
      }
      const ShardHeader ref = header_of(x.a, x.pl, 0);
      const size_t Sb = ref.shard_size;
      const ShardKeys keys(x.a);
      x.surv.resize((size_t)k * Sb);
      for (int i = 0; i < total; ++i) {
        const Address& o = i < (int)x.pl.holder.size() ? x.pl.holder[i] : Address();
        auto nd = o ? overlay_.node(o) : nullptr;
        if (!nd || nd->evicted || (!nd->up && include_down)) {
          x.lost.push_back(i);
          continue;
        }
        if (!nd->up) continue;  // unreachable for now: neither lost nor usable
        const Key key = keys(i);
        if ((int)x.sidx.size() < k) {
          // validated on the silo's view, the payload copied into its
          // survivor slot (no copy of the whole shard)
          bool ok = false;
          auto take = [&](const uint8_t* w, size_t n) {
            try {
              const uint8_t* pay = nullptr;
              const ShardHeader h = decode_shard_view(w, n, &pay);
              if (h.index != i || !h.same_block(ref)) return;
              if (Sb) std::memcpy(x.surv.data() + x.sidx.size() * Sb, pay, Sb);
              ok = true;
            } catch (ValidationFailed&) {
            }
          };
          try {
            nd->try_read(key, take);
          } catch (Unavailable&) {
            continue;
          }
          if (ok) x.sidx.push_back((uint8_t)i);
          else x.lost.push_back(i);
        } else if (!nd->has(key)) {
          x.lost.push_back(i);
        }
      }
    });
    scan_lock.unlock();  // placement below takes the index exclusively
    tm.lap("scan");
    std::vector<Todo*> work;
    for (auto& x : todo) {
      if (x.skip || x.lost.empty()) continue;
      if ((int)x.sidx.size() < k) {
        ++rep.unrecoverable;
        continue;
      }
      work.push_back(&x);
    }
    struct Group {
      int e;
      bool uniform;
      std::vector<uint8_t> pat;  // survivors (k) || lost (e), uniform groups
      std::vector<Todo*> items;
    };
    std::map<std::pair<int, std::vector<uint8_t>>, std::vector<Todo*>> by_pat;
    for (auto* x : work) {
      std::vector<uint8_t> pat;
      pat.assign(x->sidx.begin(), x->sidx.end());
      for (int i : x->lost) pat.push_back((uint8_t)i);
      by_pat[{size_bucket(memo_ec_shard_size(x->pl.B, k)), std::move(pat)}].push_back(x);
    }
    std::vector<Group> gs;
    std::map<std::pair<int, size_t>, std::vector<Todo*>> rest;
    for (auto& bp : by_pat) {
      const int e = (int)(bp.first.second.size() - (size_t)k);
      const size_t bytes = bp.second.size() * (size_t)k * ((size_t)64 << bp.first.first);
      if ((int)bp.second.size() >= o_.uniform_min && bytes >= o_.uniform_min_bytes)
        gs.push_back({e, true, bp.first.second, bp.second});
      else
        for (auto* x : bp.second) rest[{bp.first.first, (size_t)e}].push_back(x);
    }
    for (auto& r : rest) gs.push_back({(int)r.first.second, false, {}, r.second});
    // Batches of blocks with the same (S bucket, e), or the same erasure
    // pattern (the repair of one lost node: shared tables, encode speed),
    // all rebuilt by ONE codec call per chunk (memo_ec_rebuild_segments, a
    // segment per batch), then placed batch by batch.
    struct RBatch {
      const Group* grp;
      size_t b0, n, S;
      std::vector<uint8_t> sidx, lidx;
      uint8_t* surv = nullptr;  // this batch's part of the chunk's two leases
      uint8_t* out = nullptr;
    };
    std::vector<RBatch> rbs;
    for (auto& grp : gs)
      for (size_t b0 = 0; b0 < grp.items.size(); b0 += o_.batch_max) {
        RBatch rb;
        rb.grp = &grp;
        rb.b0 = b0;
        rb.n = std::min<size_t>(o_.batch_max, grp.items.size() - b0);
        rb.S = 0;  // the batch's largest shard; smaller shards zero-padded
        for (size_t bi = 0; bi < rb.n; ++bi) rb.S = std::max(rb.S, memo_ec_shard_size(grp.items[b0 + bi]->pl.B, k));
        rb.sidx.resize(rb.n * k);
        rb.lidx.resize(rb.n * grp.e);
        rbs.push_back(std::move(rb));
      }
    // one survivor and one output lease for the chunk, carved per batch (as
    // in the multi-fetch: no pinned allocation per batch)
    size_t surv_bytes = 0, out_bytes = 0;
    std::vector<size_t> o_surv(rbs.size()), o_out(rbs.size());
    for (size_t x = 0; x < rbs.size(); ++x) {
      o_surv[x] = surv_bytes;
      o_out[x] = out_bytes;
      surv_bytes += (rbs[x].n * k * rbs[x].S + 63) & ~(size_t)63;
      out_bytes += (rbs[x].n * rbs[x].grp->e * rbs[x].S + 63) & ~(size_t)63;
    }
    PinnedArena::Lease surv_all, out_all;
    if (!rbs.empty()) {
      surv_all = arena_.lease(surv_bytes);
      out_all = arena_.lease(out_bytes);
    }
    tm.lap("alloc");
    const bool pin = rbs.empty() || (surv_all.pinned() && out_all.pinned());
    for (size_t x = 0; x < rbs.size(); ++x) {
      rbs[x].surv = surv_all.data() + o_surv[x];
      rbs[x].out = out_all.data() + o_out[x];
    }
    std::vector<std::pair<size_t, size_t>> units;  // (batch, block)
    for (size_t x = 0; x < rbs.size(); ++x)
      for (size_t bi = 0; bi < rbs[x].n; ++bi) units.emplace_back(x, bi);
    pool_.parallel_for(units.size(), [&](size_t t) {
      RBatch& rb = rbs[units[t].first];
      const size_t bi = units[t].second, S = rb.S;
      const int e = rb.grp->e;
      Todo& x = *rb.grp->items[rb.b0 + bi];
      const size_t Sb = memo_ec_shard_size(x.pl.B, k);
      for (int s = 0; s < k; ++s) {
        uint8_t* slot = rb.surv + (bi * k + s) * S;
        std::memcpy(slot, x.surv.data() + (size_t)s * Sb, Sb);
        std::memset(slot + Sb, 0, S - Sb);
        rb.sidx[bi * k + s] = x.sidx[s];
      }
      for (int r = 0; r < e; ++r) rb.lidx[bi * e + r] = (uint8_t)x.lost[r];
    });
    tm.lap("copy_in");
    pool_.parallel_for(units.size(), [&](size_t t) {
      Todo& x = *rbs[units[t].first].grp->items[rbs[units[t].first].b0 + units[t].second];
      Buffer().swap(x.surv);
    });
    tm.lap("free");
    if (!rbs.empty()) {
      std::vector<memo_ec_rebuild_segment> segs;
      for (auto& rb : rbs) {
        memo_ec_rebuild_segment sg{};
        sg.k = k;
        sg.m = m;
        sg.S = rb.S;
        sg.n = rb.n;
        sg.e = rb.grp->e;
        sg.uniform = rb.grp->uniform ? 1 : 0;
        sg.surv = rb.surv;
        sg.out = rb.out;
        sg.surv_idx = rb.grp->uniform ? rb.grp->pat.data() : rb.sidx.data();
        sg.lost_idx = rb.grp->uniform ? rb.grp->pat.data() + k : rb.lidx.data();
        segs.push_back(sg);
      }
      codec_.rebuild_segments(segs, pin);
      ++rep.codec_calls;
      tm.lap("rebuild");
    }
    // Place each rebuilt shard on a reachable node holding none of the
    // block's other shards (Overlay::allocate order); the stale copy on a
    // reachable old holder is dropped.  One pass over the chunk's blocks,
    // then one index update for all of them (per batch, the fixed costs of
    // the two steps outweighed the work at 4 KiB blocks).
    std::vector<int> placed(units.size(), 0);
    pool_.parallel_for(units.size(), [&](size_t t) {
      const RBatch& rb = rbs[units[t].first];
      const size_t bi = units[t].second, S = rb.S;
      const int e = rb.grp->e;
      Todo& x = *rb.grp->items[rb.b0 + bi];
      // the block's other holders (at most k + m: a flat list)
      std::vector<Address> taken;
      taken.reserve(total);
      for (int i = 0; i < total; ++i)
        if (x.pl.holder[i] && std::find(x.lost.begin(), x.lost.end(), i) == x.lost.end())
          taken.push_back(x.pl.holder[i]);
      auto cand = overlay_.allocate(x.a, (int)overlay_.size());
      const ShardKeys keys(x.a);
      const ShardHeader hdr = header_of(x.a, x.pl, 0);
      size_t ci = 0;
      for (int r = 0; r < e; ++r) {
        const int i = x.lost[r];
        const Address old = x.pl.holder[i];
        // framed once; each candidate's silo may keep a reference to it
        auto wire = std::make_shared<Buffer>(encode_shard(hdr, rb.out + (bi * e + r) * S, i));
        x.pl.holder[i] = Address();
        while (ci < cand.size()) {
          auto& nd = cand[ci++];
          if (std::find(taken.begin(), taken.end(), nd->id) != taken.end()) continue;
          try {
            nd->store_shared(keys(i), std::shared_ptr<const uint8_t>(wire, wire->data()), wire->size());
            x.pl.holder[i] = nd->id;
            taken.push_back(nd->id);
            ++placed[t];
            break;
          } catch (Error&) {  // unreachable or full: the next candidate
          }
        }
        if (old && old != x.pl.holder[i]) {
          auto on = overlay_.node(old);
          if (on && on->up && !on->evicted) {
            try {
              on->remove(keys(i));
            } catch (Error&) {
            }
          }
        }
      }
    });
    tm.lap("place");
    // the chunk's new placements enter the index under one lock
    // (the changes are built beforehand, on the pool: under the lock only
    // the lookups and swaps)
    std::vector<char> gone(units.size(), 0);
    std::vector<NodeIndex::Change> ch(units.size());
    pool_.parallel_for(units.size(), [&](size_t t) {
      const RBatch& rb = rbs[units[t].first];
      const Todo& x = *rb.grp->items[rb.b0 + units[t].second];
      ch[t].block = x.a;
      ch[t].new_h = x.pl.holder;
    });
    {
      std::unique_lock<std::shared_mutex> lk(index_mu_);
      for (size_t t = 0; t < units.size(); ++t) {
        const RBatch& rb = rbs[units[t].first];
        Todo& x = *rb.grp->items[rb.b0 + units[t].second];
        auto it = index_.find(x.a);
        if (it == index_.end()) {
          gone[t] = 1;
          continue;
        }
        ch[t].old_h = std::move(it->second.holder);
        it->second = std::move(x.pl);  // x.pl unused from here
      }
    }
    tm.lap("swap");
    for (size_t t = 0; t < units.size(); ++t)
      if (gone[t]) ch[t].new_h.clear();  // no index change for a removed block
    nodes_.update_many(ch, &pool_);
    tm.lap("index");
    for (size_t t = 0; t < units.size(); ++t) {
      const RBatch& rb = rbs[units[t].first];
      const int e = rb.grp->e;
      Todo& x = *rb.grp->items[rb.b0 + units[t].second];
      if (gone[t]) {  // removed while being repaired: drop the new shards
        for (int i : x.lost)
          if (x.pl.holder[i])
            if (auto nd = overlay_.node(x.pl.holder[i])) {
              try {
                nd->remove(shard_key(x.a, i));
              } catch (Error&) {
              }
            }
        continue;
      }
      ++rep.blocks_repaired;
      rep.shards_rebuilt += (size_t)placed[t];
      rep.shards_unplaced += (size_t)e - (size_t)placed[t];
      ++repaired_;
      if (rebalanced_ && placed[t]) rebalanced_(x.a);  // moved onto new owners
      if (placed[t] < e && under_placed_) {
        // no reachable node could take the rest (Paxos.cc:1120-1126)
        int held = 0;
        {
          std::shared_lock<std::shared_mutex> lk(index_mu_);
          auto it = index_.find(x.a);
          if (it != index_.end())
            for (auto& h : it->second.holder) held += h ? 1 : 0;
        }
        under_placed_(x.a, held);
      }
    }
  }
  return rep;
}

ErasureConsensus::RepairReport ErasureConsensus::repair(bool include_down) {
  std::vector<Address> all;
  {
    std::shared_lock<std::shared_mutex> g(index_mu_);
    all.reserve(index_.size());
    for (auto& kv : index_) all.push_back(kv.first);
  }
  return repair_blocks(all, include_down);
}

ErasureConsensus::RepairReport ErasureConsensus::evict(const Address& node) {
  if (auto nd = overlay_.node(node)) nd->evicted = true;  // lookup / allocate skip it
  {
    std::lock_guard<std::mutex> g(mmu_);
    evict_at_.erase(node);
  }
  settle_removes(node, true);
  const std::vector<Address> blocks = nodes_.blocks(node);
  ++evictions_;
  return repair_blocks(blocks, false);
}

ErasureConsensus::RepairReport ErasureConsensus::expand() {
  std::vector<Address> under;
  {
    std::shared_lock<std::shared_mutex> g(index_mu_);
    for (auto& kv : index_)
      for (auto& h : kv.second.holder)
        if (!h) {
          under.push_back(kv.first);
          break;
        }
  }
  return repair_blocks(under, false);
}

size_t ErasureConsensus::rescan() {
  const int total = o_.k + o_.m;
  struct Seen {
    ShardHeader h;
    Address node;
  };
  auto nodes = overlay_.nodes();
  std::vector<std::vector<Seen>> per(nodes.size());
  pool_.parallel_for(nodes.size(), [&](size_t ni) {
    auto& nd = nodes[ni];
    if (!nd->up || nd->evicted) return;
    for (const Key& key : nd->silo->list()) {
      Buffer w;  // the header only: payloads are checked when read
      if (!nd->silo->try_get_prefix(key, ShardHeader::kSize, w)) continue;
      try {
        ShardHeader h = decode_shard_header(w.data(), w.size());
        // this code's shards only, under their own key
        if (h.k != o_.k || h.m != o_.m || shard_key(h.address, h.index) != key) continue;
        per[ni].push_back({std::move(h), nd->id});
      } catch (ValidationFailed&) {
        // not a shard (a mutable block's replica) or a damaged one
      }
    }
  });
  std::unordered_map<Address, Placement, AddressHash> found;
  std::unordered_map<Address, ShardHeader, AddressHash> first;
  for (auto& v : per)
    for (auto& s : v) {
      auto f = first.find(s.h.address);
      if (f == first.end()) {
        first.emplace(s.h.address, s.h);
        Placement pl;
        pl.B = s.h.block_size;
        pl.salt = s.h.salt;
        pl.owner = s.h.owner;
        pl.holder.assign(total, Address());
        f = first.find(s.h.address);
        found.emplace(s.h.address, std::move(pl));
      } else if (!s.h.same_block(f->second)) {
        continue;  // disagrees with the block's first shard: not placed
      }
      Address& h = found[s.h.address].holder[s.h.index];
      if (!h) h = s.node;
    }
  std::vector<std::pair<Address, std::vector<Address>>> diff;  // (block, old holders)
  std::vector<std::vector<Address>> neu;
  {
    std::unique_lock<std::shared_mutex> g(index_mu_);
    for (auto& kv : found) {
      neu.push_back(kv.second.holder);
      diff.emplace_back(kv.first, swap_placement_locked(kv.first, std::move(kv.second)));
    }
  }
  for (size_t i = 0; i < diff.size(); ++i) nodes_.update(diff[i].first, diff[i].second, neu[i]);
  return found.size();
}

// ---------------------------------------------------------- membership
void ErasureConsensus::post(int kind, const Address& id) {
  {
    std::lock_guard<std::mutex> g(mmu_);
    mq_.emplace_back(kind, id);
  }
  mcv_.notify_all();
}

size_t ErasureConsensus::pending_evictions() const {
  std::lock_guard<std::mutex> g(mmu_);
  return evict_at_.size();
}

// Membership thread (Paxos::LocalPeer's on_disappearance / on_discovery
// handlers, Paxos.cc:730-745, 975-1009): a disappearance arms an eviction
// timer that a return cancels; an expired timer evicts the node (its blocks'
// shards rebuilt elsewhere); a discovery expands under-placed blocks.
void ErasureConsensus::membership_loop() {
  using clock = std::chrono::steady_clock;
  std::unique_lock<std::mutex> l(mmu_);
  while (!mstop_) {
    if (mq_.empty()) {
      if (evict_at_.empty() && under_.empty()) {
        mcv_.wait(l);
      } else {
        auto next = under_.empty() ? clock::time_point::max() : under_at_;
        for (auto& kv : evict_at_) next = std::min(next, kv.second);
        if (clock::now() < next) mcv_.wait_until(l, next);
      }
      if (mstop_) break;
    }
    bool expand_now = false;
    std::vector<Address> returned;  // nodes back up: removals owed to them
    while (!mq_.empty()) {
      const auto ev = mq_.front();
      mq_.pop_front();
      if (ev.first == kDisappeared) {
        if (o_.eviction_delay_ms >= 0)
          evict_at_[ev.second] = clock::now() + std::chrono::milliseconds(o_.eviction_delay_ms);
      } else if (ev.first == kAppeared) {
        // a returning node is a discovery too (Paxos::_discovered clears the
        // timeout and queues rebalancing, Paxos.cc:969-975): blocks stored
        // while it was away can take their missing shards now
        evict_at_.erase(ev.second);
        expand_now = expand_now || o_.auto_expand;
        returned.push_back(ev.second);
      } else if (ev.first == kUnderPlaced) {
        if (under_.empty()) under_at_ = clock::now();
        under_.insert(ev.second);
        under_backoff_ = std::chrono::milliseconds(10);
      } else {
        expand_now = expand_now || o_.auto_expand;
      }
    }
    // under-placed stores, retried with backoff (10 ms doubling to 10 s,
    // as Paxos's resign loop backs off, Paxos.cc:2098)
    std::vector<Address> retry;
    if (!under_.empty() && clock::now() >= under_at_) {
      retry.assign(under_.begin(), under_.end());
      under_.clear();
    }
    std::vector<Address> due;
    const auto now = clock::now();
    for (auto it = evict_at_.begin(); it != evict_at_.end();) {
      if (it->second <= now) {
        due.push_back(it->first);
        it = evict_at_.erase(it);
      } else {
        ++it;
      }
    }
    if (due.empty() && !expand_now && retry.empty() && returned.empty()) continue;
    l.unlock();
    for (auto& id : returned) settle_removes(id, false);
    std::vector<Address> again;
    if (!retry.empty()) {
      // Only blocks still short of k+m owners while some reachable node holds
      // none of their shards are worth a rebuild; the others wait for a
      // discovery (Paxos: _under_replicated when no new owner exists,
      // Paxos.cc:1120-1124), so a network smaller than k+m does not decode
      // every store's missing shards for nothing.
      // A block is placeable while some reachable node holds none of its
      // shards (holders that are down still count as holders: they keep
      // their shards); the others are reported under-placed.
      auto placeable = [&](const std::vector<Address>& v, std::vector<std::pair<Address, int>>* stuck) {
        std::vector<Address> reach;
        for (auto& n : overlay_.nodes())
          if (n->up && !n->evicted) reach.push_back(n->id);
        std::vector<Address> out;
        std::shared_lock<std::shared_mutex> g(index_mu_);
        for (auto& a : v) {
          auto it = index_.find(a);
          if (it == index_.end()) continue;  // removed
          const auto& hv = it->second.holder;
          const int held = (int)std::count_if(hv.begin(), hv.end(), [](const Address& h) { return (bool)h; });
          if (held == (int)hv.size()) continue;  // placed meanwhile
          const bool free = std::any_of(reach.begin(), reach.end(), [&](const Address& r) {
            return std::find(hv.begin(), hv.end(), r) == hv.end();
          });
          if (free) out.push_back(a);
          else if (stuck) stuck->emplace_back(a, held);
        }
        return out;
      };
      std::vector<std::pair<Address, int>> stuck;
      const std::vector<Address> todo = placeable(retry, &stuck);
      if (!todo.empty()) {
        try {
          repair_blocks(todo, false);
        } catch (std::exception& e) {
          std::fprintf(stderr, "erasure: rebalancing failed: %s\n", e.what());
        }
        again = placeable(todo, nullptr);  // e.g. the candidate refused: try again later
      }
      notify_under_placed(stuck);
    }
    for (auto& id : due) {
      auto nd = overlay_.node(id);
      if (!nd || nd->up) continue;  // came back
      try {
        evict(id);
      } catch (std::exception& e) {
        std::fprintf(stderr, "erasure: eviction of %s failed: %s\n", id.hex().c_str(), e.what());
      }
    }
    if (expand_now) {
      try {
        expand();
      } catch (std::exception& e) {
        std::fprintf(stderr, "erasure: rebalancing failed: %s\n", e.what());
      }
    }
    l.lock();
    if (!again.empty()) {
      const bool fresh = under_.empty();
      under_.insert(again.begin(), again.end());
      if (fresh) {
        under_at_ = clock::now() + under_backoff_;
        under_backoff_ = std::min(under_backoff_ * 2, std::chrono::milliseconds(10000));
      }
    }
  }
}

// "erasure" configuration: {"type": "erasure", "data-shards": k,
// "parity-shards": m, "backend-replication-factor": f, and optionally
// "device", "batch-max", "eviction-delay" (s), "stage-mb", "threads",
// "fetch-hedge", "verify-subsets"};
// kebab-case keys as "replication-factor" (Paxos.cc:2273-2276).
namespace {
struct RegisterErasure {
  RegisterErasure() {
    register_consensus("erasure", [](Overlay& ov, const ConfigMap& c) {
      ErasureOptions o;
      auto get = [&](const char* key, int dflt) {
        auto it = c.find(key);
        return it == c.end() ? dflt : std::stoi(it->second);
      };
      o.k = get("data-shards", 10);
      o.m = get("parity-shards", 4);
      o.device = get("device", 0);
      o.batch_max = get("batch-max", 256);
      o.eviction_delay_ms = (int64_t)get("eviction-delay", 600) * 1000;  // seconds
      const int stage_mb = get("stage-mb", (int)(kStageBytes >> 20));
      o.threads = get("threads", o.threads);
      o.fetch_hedge = get("fetch-hedge", o.fetch_hedge);
      o.verify_subsets = get("verify-subsets", o.verify_subsets);
      if (o.batch_max < 1 || stage_mb < 1 || o.threads < 1)
        throw Error("erasure: batch-max, stage-mb and threads must be positive");
      if (o.fetch_hedge < 0 || o.verify_subsets < 0)
        throw Error("erasure: fetch-hedge and verify-subsets must not be negative");
      o.stage_bytes = (size_t)stage_mb << 20;
      const int f = get("backend-replication-factor", 3);
      return std::unique_ptr<Consensus>(
          new ErasureConsensus(std::make_unique<ReplicationConsensus>(ov, f), ov, o));
    });
  }
} register_erasure_;
}  // namespace

}  // namespace memo_host
