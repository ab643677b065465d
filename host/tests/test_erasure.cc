// test_erasure.cc -- the reference's redundancy-path semantics tests, ported
// onto the erasure plugin (host/erasure_consensus.hh).  Each test names the
// reference test it follows.  Tests tagged GPU run the codec (libmemo_ec on
// an MI355X); the others need no GPU.
//   usage: test_erasure [--cpu-only] [filter]
#include <atomic>
#include <chrono>
#include <mutex>
#include <cstdio>
#include <cstring>
#include <filesystem>
#include <random>
#include <set>
#include <thread>

#include "../erasure_consensus.hh"

using namespace memo_host;

namespace {

struct TestCase {
  const char* name;
  bool gpu;
  void (*fn)();
};
std::vector<TestCase>& tests() {
  static std::vector<TestCase> t;
  return t;
}
struct Reg {
  Reg(const char* n, bool g, void (*f)()) { tests().push_back({n, g, f}); }
};
int g_fail = 0;

// Polls `pred` for up to `ms` milliseconds (background rebalancing).
template <class F>
bool wait_for(F pred, int ms = 20000) {
  for (int t = 0; t < ms; t += 5) {
    if (pred()) return true;
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
  return pred();
}

#define TEST(name, gpu)                      \
  static void test_##name();                 \
  static Reg reg_##name(#name, gpu, test_##name); \
  static void test_##name()
#define CHECK(x)                                                             \
  do {                                                                       \
    if (!(x)) {                                                              \
      std::fprintf(stderr, "  CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #x); \
      ++g_fail;                                                              \
    }                                                                        \
  } while (0)
#define CHECK_THROW(expr, Exc)                                               \
  do {                                                                       \
    bool thrown_ = false;                                                    \
    try {                                                                    \
      expr;                                                                  \
    } catch (Exc&) {                                                         \
      thrown_ = true;                                                        \
    } catch (std::exception & e_) {                                          \
      std::fprintf(stderr, "  %s:%d: wrong exception: %s\n", __FILE__, __LINE__, e_.what()); \
    }                                                                        \
    if (!thrown_) {                                                          \
      std::fprintf(stderr, "  CHECK_THROW failed %s:%d: %s\n", __FILE__, __LINE__, #expr); \
      ++g_fail;                                                              \
    }                                                                        \
  } while (0)

Buffer bytes(const char* s) { return Buffer(s, s + std::strlen(s)); }

// The reference's calls (Consensus.hh:38-49) for a test's block in hand:
// store a copy, no conflict resolver; fetch many addresses, no versions;
// remove with a signature or none.
void store(Consensus& c, const Block& b, StoreMode mode = STORE_INSERT) {
  c.store(std::make_unique<Block>(b), mode, nullptr);
}
void fetch_many(Consensus& c, const std::vector<Address>& as, const ReceiveBlock& res) {
  std::vector<Consensus::AddressVersion> req;
  for (auto& a : as) req.emplace_back(a, std::nullopt);
  c.fetch(req, res);
}
void remove(Consensus& c, const Address& a, const RemoveSignature& rs = {}) { c.remove(a, rs); }

Buffer random_bytes(size_t n, uint64_t seed) {
  std::mt19937_64 r(seed);
  Buffer b(n);
  for (auto& x : b) x = (uint8_t)r();
  return b;
}

// An in-process network like tests/DHT.hh: `nodes` nodes with memory silos
// on one overlay, and an erasure consensus client over it.
struct Net {
  Overlay overlay;
  std::vector<std::shared_ptr<Node>> nodes;
  std::unique_ptr<ErasureConsensus> ec;
  ErasureOptions o;
  // eviction_delay_ms < 0: no automatic eviction (tests that drop nodes
  // silently by Node::up are not disturbed)
  Net(int n, int k, int m, int batch_window_us = 200, int64_t eviction_delay_ms = -1) {
    for (int i = 0; i < n; ++i) add();
    o.k = k;
    o.m = m;
    o.batch_window_us = batch_window_us;
    o.eviction_delay_ms = eviction_delay_ms;
    restart();
  }
  std::shared_ptr<Node> add() {
    uint8_t id[32] = {0};
    id[0] = (uint8_t)(nodes.size() + 1);
    id[1] = 0x4d;
    // the node's peer is the erasure consensus's (ErasureConsensus::make_local
    // over a replication backend): shards checked by header, CRC and key
    nodes.push_back(overlay.add_node(Address(id, 0, false), make_shard_local(std::make_unique<MemorySilo>())));
    return nodes.back();
  }
  // A fresh consensus over the same silos (a node restart): its index comes
  // from the shard headers on disk.
  void restart() {
    ec.reset();
    ec = std::make_unique<ErasureConsensus>(std::make_unique<ReplicationConsensus>(overlay, 3),
                                            overlay, o);
  }
  // nodes holding at least one shard of `a`
  int holders(const Address& a, int total) {
    int h = 0;
    for (auto& n : nodes)
      for (int i = 0; i < total; ++i)
        if (!n->evicted && n->has(shard_key(a, i))) {
          ++h;
          break;
        }
    return h;
  }
  int shards(const Address& a, int total) {
    int s = 0;
    for (auto& n : nodes)
      for (int i = 0; i < total; ++i)
        if (!n->evicted && n->has(shard_key(a, i))) ++s;
    return s;
  }
};

}  // namespace

// ------------------------------------------------------------- CPU tests
// tests/storage.cc:15-45: the silo contract shards are stored under.
TEST(silo_memory_contract, false) {
  MemorySilo s;
  Key k1 = Address::random(flags::immutable_block), k2 = Address::random(flags::immutable_block);
  s.set(k1, bytes("the grey"));
  CHECK(s.get(k1) == bytes("the grey"));
  s.set(k1, bytes("the white"), false, true);
  CHECK(s.get(k1) == bytes("the white"));
  CHECK_THROW(s.set(k1, Buffer()), silo::Collision);
  CHECK(s.get(k1) == bytes("the white"));
  CHECK_THROW(s.get(k2), silo::MissingKey);
  CHECK_THROW(s.set(k2, Buffer(), false, true), silo::MissingKey);
  CHECK_THROW(s.erase(k2), silo::MissingKey);
  s.erase(k1);
  CHECK_THROW(s.get(k1), silo::MissingKey);
  CHECK(s.list().empty());
}

// Values that share one allocation (Silo::set_shared, the store's framed
// runs), views (Silo::read / read_prefix) and usage: each key holds exactly
// its own bytes, usage counts each value's length, and replacing or erasing
// one value leaves the others intact; a silo without sharing (filesystem)
// keeps a copy.
TEST(silo_shared_values_and_views, false) {
  auto run = std::shared_ptr<uint8_t>(new uint8_t[300], std::default_delete<uint8_t[]>());
  for (int i = 0; i < 300; ++i) run.get()[i] = (uint8_t)i;
  Key ks[3] = {Address::random(flags::immutable_block), Address::random(flags::immutable_block),
               Address::random(flags::immutable_block)};
  MemorySilo s;
  for (int i = 0; i < 3; ++i) s.set_shared(ks[i], std::shared_ptr<const uint8_t>(run, run.get() + 100 * i), 90);
  CHECK(s.usage() == 270);
  run.reset();  // the silo's values keep the allocation alive
  for (int i = 0; i < 3; ++i) {
    const Buffer v = s.get(ks[i]);
    CHECK(v.size() == 90 && v[0] == (uint8_t)(100 * i) && v[89] == (uint8_t)(100 * i + 89));
  }
  size_t seen = 0;
  uint8_t first = 0;
  auto view = [&](const uint8_t* p, size_t n) {
    seen = n;
    first = p[0];
  };
  CHECK(s.read(ks[1], view) && seen == 90 && first == 100);
  CHECK(s.read_prefix(ks[2], 4, view) && seen == 4 && first == 200);
  CHECK(s.read_prefix(ks[2], 1000, view) && seen == 90);
  CHECK(!s.read(Address::random(flags::immutable_block), view));
  s.set(ks[1], bytes("replaced"), false, true);
  CHECK(s.usage() == 188 && s.get(ks[1]) == bytes("replaced"));
  CHECK(s.get(ks[0])[5] == 5 && s.get(ks[2])[5] == 205);
  for (auto& k : ks) s.erase(k);
  CHECK(s.usage() == 0 && s.list().empty());
  // capacity counts shared values too
  MemorySilo small(100);
  auto r2 = std::shared_ptr<uint8_t>(new uint8_t[200](), std::default_delete<uint8_t[]>());
  small.set_shared(ks[0], r2, 80);
  CHECK_THROW(small.set_shared(ks[1], std::shared_ptr<const uint8_t>(r2, r2.get() + 100), 80),
              silo::InsufficientSpace);
}

std::string temp_dir(const char* tag) {
  char tmpl[256];
  std::snprintf(tmpl, sizeof tmpl, "/tmp/memo_ec_%s_XXXXXX", tag);
  const char* d = mkdtemp(tmpl);
  if (!d) throw Error("mkdtemp failed");
  return d;
}

// tests/storage.cc:15-45 on silo::Filesystem (Filesystem.cc:27-147): the
// same contract, and what was stored survives reopening the directory
// (usage recovered from the files).
TEST(silo_filesystem_contract, false) {
  const std::string root = temp_dir("silo");
  Key k1 = Address::random(flags::immutable_block), k2 = Address::random(flags::immutable_block);
  {
    FilesystemSilo s(root);
    s.set(k1, bytes("the grey"));
    CHECK(s.get(k1) == bytes("the grey"));
    s.set(k1, bytes("the white"), false, true);
    CHECK(s.get(k1) == bytes("the white"));
    CHECK_THROW(s.set(k1, Buffer()), silo::Collision);
    CHECK_THROW(s.get(k2), silo::MissingKey);
    CHECK_THROW(s.set(k2, Buffer(), false, true), silo::MissingKey);
    CHECK_THROW(s.erase(k2), silo::MissingKey);
    s.set(k2, Buffer(1000, 7));
    CHECK(s.usage() == 9 + 1000);
  }
  {
    FilesystemSilo s(root);  // reopened
    CHECK(s.usage() == 9 + 1000);
    auto keys = s.list();
    CHECK(keys.size() == 2);
    CHECK(s.get(k1) == bytes("the white"));
    s.erase(k1);
    CHECK_THROW(s.get(k1), silo::MissingKey);
    CHECK(s.usage() == 1000);
    // shared values are copied to their files; views and prefix views read them
    auto run = std::shared_ptr<uint8_t>(new uint8_t[64], std::default_delete<uint8_t[]>());
    for (int i = 0; i < 64; ++i) run.get()[i] = (uint8_t)(i + 1);
    s.set_shared(k1, std::shared_ptr<const uint8_t>(run, run.get() + 32), 32);
    run.reset();
    CHECK(s.get(k1).size() == 32 && s.get(k1)[0] == 33 && s.usage() == 1032);
    size_t seen = 0;
    uint8_t first = 0;
    auto view = [&](const uint8_t* p, size_t n) {
      seen = n;
      first = p[0];
    };
    CHECK(s.read(k2, view) && seen == 1000 && first == 7);
    CHECK(s.read_prefix(k1, 4, view) && seen == 4 && first == 33);
  }
  std::filesystem::remove_all(root);
}

// tests/storage.cc:47-84: capacity.
TEST(silo_capacity, false) {
  MemorySilo s(10);
  Key k = Address::random(flags::immutable_block);
  s.set(k, Buffer(8));
  CHECK(s.usage() == 8);
  CHECK_THROW(s.set(Address::random(flags::immutable_block), Buffer(8)), silo::InsufficientSpace);
  s.erase(k);
  CHECK(s.usage() == 0);
}

TEST(shard_format_round_trip_and_validation, false) {
  ShardHeader h;
  h.k = 10;
  h.m = 4;
  h.index = 12;
  h.block_size = 1000;
  h.shard_size = memo_ec_shard_size(1000, 10);
  h.address = Address::random(flags::immutable_block);
  h.salt = bytes("salt");
  h.owner = Address::random(flags::mutable_block);
  Buffer payload = random_bytes(h.shard_size, 7);
  Buffer w = encode_shard(h, payload.data());
  CHECK(w.size() == ShardHeader::kSize + h.shard_size);
  const uint8_t* p = nullptr;
  ShardHeader d = decode_shard(w, &p);
  CHECK(d.k == 10 && d.m == 4 && d.index == 12 && d.block_size == 1000);
  CHECK(d.address == h.address && d.salt == h.salt && d.owner == h.owner);
  CHECK(d.same_block(h));
  CHECK(std::memcmp(p, payload.data(), h.shard_size) == 0);
  ShardHeader hd = decode_shard_header(w.data(), ShardHeader::kSize);  // header bytes only
  CHECK(hd.same_block(h) && hd.index == 12 && hd.crc == d.crc);
  Buffer bad = w;
  bad[ShardHeader::kSize + 5] ^= 1;  // payload bit flip
  CHECK_THROW(decode_shard(bad, nullptr), ValidationFailed);
  bad = w;
  bad[16] ^= 1;  // shard size inconsistent with block size
  CHECK_THROW(decode_shard(bad, nullptr), ValidationFailed);
  for (size_t at : {size_t(8), size_t(60), size_t(100), size_t(30)}) {  // B, salt, owner, address
    bad = w;
    bad[at] ^= 0x10;  // the checksum covers the header
    CHECK_THROW(decode_shard(bad, nullptr), ValidationFailed);
  }
  bad = w;
  bad.resize(bad.size() - 1);
  CHECK_THROW(decode_shard(bad, nullptr), ValidationFailed);
  bad = w;
  bad[0] = 'X';
  CHECK_THROW(decode_shard(bad, nullptr), ValidationFailed);
  bad = w;
  bad[4] = 1;  // round-1 layout
  CHECK_THROW(decode_shard(bad, nullptr), ValidationFailed);
  // CRC32C known answer (RFC 3720 B.4: 32 bytes of zeros -> 0x8a9136aa), and
  // chaining: crc(a || b) = crc(b, crc(a))
  uint8_t z[32] = {0};
  CHECK(crc32c(z, 32) == 0x8a9136aau);
  CHECK(crc32c(z + 13, 19, crc32c(z, 13)) == 0x8a9136aau);
}

TEST(config_registry, false) {
  Overlay ov;
  auto c = from_json("{\"type\": \"erasure\", \"data-shards\": 10, \"parity-shards\": 4}");
  CHECK(c["type"] == "erasure" && c["data-shards"] == "10" && c["parity-shards"] == "4");
  CHECK(from_json(to_json(c)) == c);
  CHECK_THROW(make_consensus(ov, "{\"type\": \"nope\"}"), Error);
  CHECK_THROW(make_consensus(ov, "{\"data-shards\": 3}"), Error);
  CHECK_THROW(make_consensus(ov, "{\"type\": \"erasure\", \"stage-mb\": 0}"), Error);
  CHECK_THROW(make_consensus(ov, "{\"type\": \"erasure\", \"stage-mb\": -1}"), Error);
  CHECK_THROW(make_consensus(ov, "{\"type\": \"erasure\", \"fetch-hedge\": -1}"), Error);
  CHECK_THROW(make_consensus(ov, "{\"type\": \"erasure\", \"verify-subsets\": -2}"), Error);
  CHECK_THROW(make_consensus(ov, "{\"type\": \"erasure\", \"threads\": 0}"), Error);
  auto r = make_consensus(ov, "{\"type\": \"replication\", \"replication-factor\": 2}");
  CHECK(from_json(r->redundancy())["type"] == "replication");
}

// The peers the consensuses make (Consensus::make_local, Consensus.hh:100-
// 105): what LocalPeer::store validates (Paxos.cc:1568-1615), restated.
TEST(peers_validate_what_they_store, false) {
  // replication's peer: a CHB replica must hash to its key
  Overlay ov;
  ReplicationConsensus rc(ov, 2);
  auto a = ov.add_node(Address::random(0), rc.make_local(7000, IpAddress{"127.0.0.1"}, std::make_unique<MemorySilo>()));
  auto b = ov.add_node(Address::random(0), rc.make_local({}, {}, std::make_unique<MemorySilo>()));
  CHECK(a->local->port() == 7000 && a->local->listen_address()->text == "127.0.0.1");
  Block good = make_chb(bytes("payload"));
  store(rc, good);
  CHECK(rc.fetch(good.address)->data == good.data);
  Block forged = make_chb(bytes("payload"));
  forged.data = bytes("other bytes");  // the address no longer its content's
  CHECK_THROW(store(rc, forged), ValidationFailed);
  // a mutable block's version must grow: Conflict, resolved by the resolver
  Block m1 = make_mutable(Address::random(flags::mutable_block), bytes("v1"), 1);
  store(rc, m1);
  Block m1b = make_mutable(m1.address, bytes("v1 again"), 1);
  CHECK_THROW(store(rc, m1b, STORE_UPDATE), Conflict);
  struct Bump : ConflictResolver {
    int* calls;
    explicit Bump(int* c) : calls(c) {}
    std::unique_ptr<Block> operator()(Block& failed, Block& current) override {
      ++*calls;
      auto nb = std::make_unique<Block>(failed);
      nb->version = current.version + 1;
      return nb;
    }
    std::string description() const override { return "bump"; }
  };
  int calls = 0;  // the resolver is the store's (unique_ptr): count outside it
  rc.store(std::make_unique<Block>(m1b), STORE_UPDATE, std::make_unique<Bump>(&calls));
  CHECK(calls == 1);
  auto got = rc.fetch(m1.address);
  CHECK(got->data == bytes("v1 again") && got->version == 2);
  CHECK(rc.fetch(m1.address, 2) == nullptr);  // not newer than the caller's version
  CHECK(rc.fetch(m1.address, 1)->version == 2);
  // the erasure peer: shards by header, CRC and key; other values to the
  // replication peer's checks
  auto local = make_shard_local(std::make_unique<MemorySilo>());
  ShardHeader h;
  h.k = 10;
  h.m = 4;
  h.index = 3;
  h.block_size = 5000;
  h.shard_size = memo_ec_shard_size(5000, 10);
  h.address = good.address;
  const Buffer pay = random_bytes(h.shard_size, 5);
  Buffer w = encode_shard(h, pay.data());
  local->validate(shard_key(h.address, 3), w.data(), w.size());  // accepted
  CHECK_THROW(local->validate(shard_key(h.address, 4), w.data(), w.size()), ValidationFailed);
  Buffer bad = w;
  bad[ShardHeader::kSize + 17] ^= 1;
  CHECK_THROW(local->validate(shard_key(h.address, 3), bad.data(), bad.size()), ValidationFailed);
  // a shard may only replace a shard
  local->storage().set(shard_key(h.address, 3), bytes("not a shard"));
  CHECK_THROW(local->validate(shard_key(h.address, 3), w.data(), w.size()), ValidationFailed);
  Buffer rep(40, 0);  // an empty CHB replica under the wrong key
  CHECK_THROW(local->validate(good.address, rep.data(), rep.size()), ValidationFailed);
  // through a node: the refused value never reaches the silo
  Overlay ov2;
  auto n = ov2.add_node(Address::random(0), make_shard_local(std::make_unique<MemorySilo>()));
  CHECK_THROW(n->store(shard_key(h.address, 3), bad), ValidationFailed);
  CHECK(!n->has(shard_key(h.address, 3)));
  n->store(shard_key(h.address, 3), w);
  CHECK(n->has(shard_key(h.address, 3)));
}

// The stack and the factory (Consensus.hh:100-142): find<C> walks the
// stack, make_remote is the backend's, stat reports the placement.
TEST(stacked_consensus_surface, true) {
  Overlay ov;
  ErasureOptions o;
  o.k = 4;
  o.m = 2;
  o.device = 0;
  auto ec = std::unique_ptr<Consensus>(new ErasureConsensus(std::make_unique<ReplicationConsensus>(ov, 3), ov, o));
  CHECK(StackedConsensus::find<ErasureConsensus>(ec.get()) == ec.get());
  auto* rep = StackedConsensus::find<ReplicationConsensus>(ec.get());
  CHECK(rep != nullptr && rep->factor() == 3);
  CHECK(StackedConsensus::find<ReplicationConsensus>(rep) == rep);
  auto conn = std::make_shared<DockConnection>();
  conn->peer = Address::random(0);
  auto remote = ec->make_remote(conn);
  CHECK(remote && remote->id() == conn->peer);
  auto st = from_json(ec->stat(Address::random(flags::immutable_block))->json());
  CHECK(st["placed"] == "0" && st["k"] == "4" && st["m"] == "2");
  auto local = ec->make_local(9000, {}, std::make_unique<MemorySilo>());
  CHECK(dynamic_cast<ShardLocal*>(local.get()) != nullptr && local->port() == 9000);
}

TEST(placement_is_deterministic_and_distinct, false) {
  Overlay ov;
  for (int i = 0; i < 20; ++i) ov.add_node(Address::random(0), std::make_unique<MemorySilo>());
  auto a = Address::random(flags::immutable_block);
  auto o1 = ov.allocate(a, 14), o2 = ov.allocate(a, 14);
  CHECK(o1.size() == 14);
  std::set<Address> ids;
  for (size_t i = 0; i < o1.size(); ++i) {
    CHECK(o1[i]->id == o2[i]->id);
    ids.insert(o1[i]->id);
  }
  CHECK(ids.size() == 14);
  o1[3]->up = false;  // allocate skips unreachable nodes
  auto o3 = ov.allocate(a, 14);
  for (auto& n : o3) CHECK(n->up);
}

TEST(chb_address_is_content_hash, false) {
  Block b = make_chb(bytes("\\_o<"), bytes("salt"));
  CHECK(!b.address.mutable_block());
  CHECK(chb_valid(b.address, b.salt, b.owner, b.data));
  Buffer other = b.data;
  other[0] ^= 1;
  CHECK(!chb_valid(b.address, b.salt, b.owner, other));
}

// CHB::_hash_address (CHB.cc:264-289): SHA-256(salt || owner || data) when
// the owner is set and the version >= 0.4; the flag byte is combined from
// 0.5; validation ignores the flag byte (equal_unflagged).
TEST(chb_owner_and_version, false) {
  const Address owner = Address::random(flags::mutable_block);
  const Buffer data = bytes("owned block"), salt = bytes("pepper");
  Block b = make_chb(data, salt, owner);
  CHECK(b.owner == owner);
  Buffer so = salt;
  so.insert(so.end(), owner.value.begin(), owner.value.end());
  const auto h = sha256(so.data(), so.size(), data.data(), data.size());
  CHECK(std::memcmp(b.address.value.data(), h.data(), 31) == 0);
  CHECK(b.address.value[31] == flags::immutable_block);
  CHECK(chb_valid(b.address, salt, owner, data));
  CHECK(!chb_valid(b.address, salt, Address(), data));                       // owner dropped
  CHECK(!chb_valid(b.address, salt, Address::random(flags::mutable_block), data));  // other owner
  CHECK(make_chb(data, salt).address != b.address);
  // before 0.4 the owner is ignored (and not kept); before 0.5 the flag byte
  // is the hash's own
  Block old = make_chb(data, salt, owner, Version{0, 3, 0});
  CHECK(!old.owner);
  CHECK(old.address == make_chb(data, salt, Address(), Version{0, 3, 0}).address);
  const auto h0 = sha256(salt.data(), salt.size(), data.data(), data.size());
  CHECK(old.address.value[31] == h0[31]);
  CHECK(chb_valid(old.address, salt, owner, data, Version{0, 3, 0}));
}
// CHB::sign_remove / CHB::_validate_remove (CHB.cc:140-259): who may remove
// an owned CHB.
TEST(chb_remove_validation_rules, false) {
  const KeyPair owner_k = KeyPair::generate(), writer_k = KeyPair::generate(),
                other_k = KeyPair::generate();
  const Address owner = Address::random(flags::mutable_block);
  Block b = make_chb(bytes("owned"), bytes("s"), owner);
  Block free_b = make_chb(bytes("unowned"));
  OwnerDirectory dir;
  dir.set(owner, OwnerAcl{owner_k.public_key, {writer_k.public_key}, false, {}});
  // no owner: anyone, signed or not
  CHECK(chb_validate_remove(free_b.address, free_b.owner, {}, &dir).empty());
  // owned: the fields must be there and the signature must verify
  CHECK(chb_validate_remove(b.address, owner, {}, &dir) == "Missing field in signature");
  RemoveSignature rs = chb_sign_remove(b.address, owner_k);
  CHECK(chb_validate_remove(b.address, owner, rs, &dir).empty());
  RemoveSignature bad = rs;
  (*bad.signature)[3] ^= 1;
  CHECK(chb_validate_remove(b.address, owner, bad, &dir) == "Invalid signature");
  // a signature of another block's address does not transfer
  CHECK(chb_validate_remove(b.address, owner, chb_sign_remove(free_b.address, owner_k), &dir) ==
        "Invalid signature");
  // the key needs authority over the owner block: its owner or a writer
  CHECK(chb_validate_remove(b.address, owner, chb_sign_remove(b.address, writer_k), &dir).empty());
  CHECK(chb_validate_remove(b.address, owner, chb_sign_remove(b.address, other_k), &dir) ==
        "Key not found");
  dir.set(owner, OwnerAcl{owner_k.public_key, {}, true, {}});  // world-writable
  CHECK(chb_validate_remove(b.address, owner, chb_sign_remove(b.address, other_k), &dir).empty());
  // an owner block nobody knows: allowed once the signature verifies (the
  // reference warns and allows, CHB.cc:222-227)
  CHECK(chb_validate_remove(b.address, owner, chb_sign_remove(b.address, other_k), nullptr).empty());
  CHECK(chb_validate_remove(b.address, owner, {}, nullptr) == "Missing field in signature");
}

// CHB::_validate_remove's group branch (CHB.cc:243-258) and
// CHB::sign_remove's group signature (CHB.cc:170-186): a member removes an
// owned CHB with the key of a group that has write access on the owner.
TEST(chb_remove_group_key_rules, false) {
  const KeyPair owner_k = KeyPair::generate(), g1 = KeyPair::generate(), g2 = KeyPair::generate(),
                member_k = KeyPair::generate();
  const Buffer G = KeyPair::generate().public_key, H = KeyPair::generate().public_key;
  const Address owner = Address::random(flags::mutable_block);
  Block b = make_chb(bytes("group owned"), bytes("s"), owner);
  OwnerDirectory dir;
  dir.set_group(G, {g1.public_key, g2.public_key});  // versions 1 and 2
  dir.set_group(H, {g1.public_key});
  OwnerAcl acl{owner_k.public_key, {member_k.public_key}, false, {{G, true}, {H, false}}};
  dir.set(owner, acl);
  // the group's current key (version 2, index 1) and its first one (index 0)
  CHECK(chb_validate_remove(b.address, owner, chb_sign_remove_group(b.address, G, g2, 2), &dir).empty());
  CHECK(chb_validate_remove(b.address, owner, chb_sign_remove_group(b.address, G, g1, 1), &dir).empty());
  // the index must name the signing key's version
  CHECK(chb_validate_remove(b.address, owner, chb_sign_remove_group(b.address, G, g2, 1), &dir) ==
        "Key not found");
  CHECK(chb_validate_remove(b.address, owner, chb_sign_remove_group(b.address, G, g2, 3), &dir) ==
        "Key not found");
  CHECK(chb_validate_remove(b.address, owner, chb_sign_remove_group(b.address, G, g2, 0), &dir) ==
        "Key not found");
  RemoveSignature no_index = chb_sign_remove_group(b.address, G, g2, 2);
  no_index.group_index.reset();
  CHECK(chb_validate_remove(b.address, owner, no_index, &dir) == "Key not found");
  // a group entry without write access, a group not in the ACL, a group the
  // network does not know
  CHECK(chb_validate_remove(b.address, owner, chb_sign_remove_group(b.address, H, g1, 1), &dir) ==
        "Key not found");
  const Buffer U = KeyPair::generate().public_key;
  CHECK(chb_validate_remove(b.address, owner, chb_sign_remove_group(b.address, U, g1, 1), &dir) ==
        "Key not found");
  acl.groups.push_back({U, true});
  dir.set(owner, acl);
  CHECK(chb_validate_remove(b.address, owner, chb_sign_remove_group(b.address, U, g1, 1), &dir) ==
        "Key not found");
  // with a group in the signature the individual entries are not consulted
  // (CHB.cc:234-241 runs only without one): a writer signing "through" a
  // group it is no key of is refused, and the same key signing alone passes
  CHECK(chb_validate_remove(b.address, owner, chb_sign_remove_group(b.address, G, member_k, 2), &dir) ==
        "Key not found");
  CHECK(chb_validate_remove(b.address, owner, chb_sign_remove(b.address, member_k), &dir).empty());
  // the owner key passes with or without a group
  CHECK(chb_validate_remove(b.address, owner, chb_sign_remove_group(b.address, H, owner_k, 1), &dir)
            .empty());
  // the signature must still verify
  RemoveSignature bad = chb_sign_remove_group(b.address, G, g2, 2);
  (*bad.signature)[0] ^= 1;
  CHECK(chb_validate_remove(b.address, owner, bad, &dir) == "Invalid signature");
}

// The pinned arena keeps a few batch buffers for reuse, never one larger
// than kKeepMaxBytes (a node-loss fetch must not leave GBs pinned).
// Node::remove_values: one request (one Unavailable when down), keys absent
// skipped, each present key's prefix checked on the node, refusals kept.
TEST(node_remove_values_is_one_checked_request, false) {
  Overlay ov;
  auto n = ov.add_node(Address::random(0), std::make_unique<MemorySilo>());
  std::vector<Key> ks;
  for (int i = 0; i < 4; ++i) ks.push_back(Address::random(0));
  n->store(ks[0], bytes("allow-0 payload"));
  n->store(ks[1], bytes("refuse-1"));
  n->store(ks[3], bytes("allow-3"));
  std::vector<std::string> seen;
  auto check = [&](const Key&, const Buffer& head) {
    const std::string h(head.begin(), head.end());
    seen.push_back(h);
    return h.rfind("allow", 0) == 0 ? std::string() : std::string("no authority");
  };
  std::string refused;
  CHECK(n->remove_values(ks, 5, check, &refused) == 2);
  CHECK(n->remove_requests.load() == 1);
  CHECK(refused == "no authority");
  CHECK(seen.size() == 3);  // ks[2] was never there
  for (auto& h : seen) CHECK(h.size() == 5);  // the prefix only
  CHECK(!n->has(ks[0]) && n->has(ks[1]) && !n->has(ks[3]));
  CHECK(n->holds_any(ks) && !n->holds_any({ks[0], ks[2], ks[3]}));
  ov.set_up(n->id, false);
  CHECK_THROW(n->holds_any(ks), Unavailable);
  CHECK_THROW(n->remove_values(ks, 5, check), Unavailable);
  CHECK(n->remove_requests.load() == 1);  // refused before it was served
}

TEST(pinned_arena_drops_outsized_buffers, false) {
  PinnedArena a;
  {
    auto big = a.lease(PinnedArena::kKeepMaxBytes + 1);
    CHECK(big.data() != nullptr);
  }
  CHECK(a.kept_bytes() == 0);
  {
    auto small = a.lease(1000);
  }
  CHECK(a.kept_bytes() == (size_t)1 << 20);
  {
    auto again = a.lease(4000);  // reuses the kept buffer
  }
  CHECK(a.kept_bytes() == (size_t)1 << 20 && a.leases() == 3);
}

// -------------------------------------------------------------- GPU tests
// tests/doughnut.cc:320-335 (CHB): insert -> fetch equal -> remove.
TEST(CHB, true) {
  Net net(16, 10, 4);
  Block b = make_chb(bytes("\\_o<"));
  store(*net.ec, b);
  CHECK(net.holders(b.address, 14) == 14);
  auto st = from_json(net.ec->stat(b.address)->json());  // Consensus::stat
  CHECK(st["placed"] == "1" && st["reachable"] == "14" && st["block_size"] == "4");
  CHECK(net.ec->fetch(b.address)->data == b.data);
  auto f = net.ec->fetch(b.address);
  CHECK(f->data == b.data);
  remove(*net.ec, b.address);
  CHECK(net.shards(b.address, 14) == 0);
  CHECK_THROW(net.ec->fetch(b.address), MissingBlock);
}

// Removal of an owned CHB through the plugin (Local::remove ->
// CHB::_validate_remove at every holder, Local.cc:260-278, CHB.cc:203-259;
// Consensus::remove_many, Consensus.cc:178-240): unsigned or wrongly signed
// removals are refused with every shard left in place; the owner's signed
// removal takes every shard; an address nobody stored is MissingBlock.
TEST(remove_owned_chb_semantics, true) {
  Net net(16, 10, 4);
  OwnerDirectory dir;
  const KeyPair owner_k = KeyPair::generate(), other_k = KeyPair::generate();
  const Address owner = Address::random(flags::mutable_block);
  dir.set(owner, OwnerAcl{owner_k.public_key, {}, false, {}});
  net.ec->set_owner_directory(&dir);
  Block b = make_chb(random_bytes(70000, 77), bytes("salt"), owner);
  store(*net.ec, b);
  CHECK(net.shards(b.address, 14) == 14);
  CHECK_THROW(remove(*net.ec, b.address), ValidationFailed);
  CHECK_THROW(remove(*net.ec, b.address, chb_sign_remove(b.address, other_k)), ValidationFailed);
  RemoveSignature forged = chb_sign_remove(b.address, owner_k);
  forged.signature_key = other_k.public_key;
  CHECK_THROW(remove(*net.ec, b.address, forged), ValidationFailed);
  CHECK(net.shards(b.address, 14) == 14);
  CHECK(net.ec->fetch(b.address)->data == b.data);
  remove(*net.ec, b.address, chb_sign_remove(b.address, owner_k));
  CHECK(net.shards(b.address, 14) == 0);
  CHECK_THROW(net.ec->fetch(b.address), MissingBlock);
  CHECK_THROW(remove(*net.ec, b.address, chb_sign_remove(b.address, owner_k)), MissingBlock);
  CHECK_THROW(remove(*net.ec, Address::random(flags::immutable_block)), MissingBlock);
  // unowned blocks need no signature; a fresh client (no placement of the
  // block: a restart, index from the silos) removes them from the holders
  // lookup() names
  Block u = make_chb(random_bytes(5000, 78));
  store(*net.ec, u);
  net.o.rescan = false;
  net.restart();
  remove(*net.ec, u.address);
  CHECK(net.shards(u.address, 14) == 0);
}

// A removal while one holder is down: the reachable holders remove their
// shards at once; the down holder's shard is owed -- erased when the node
// returns, dropped when it is evicted -- and the eviction repairs nothing
// of the removed block (evict_removed_blocks, tests/doughnut.cc:1693-1719).
TEST(remove_with_holder_down, true) {
  Net net(16, 10, 4);
  Block a = make_chb(random_bytes(40000, 90)), c = make_chb(random_bytes(40000, 91));
  store(*net.ec, a);
  store(*net.ec, c);
  std::shared_ptr<Node> down, back;
  for (auto& n : net.nodes)
    for (int i = 0; i < 14; ++i)
      if (n->has(shard_key(a.address, i))) {
        if (!down) down = n;
        else if (!back && n != down) back = n;
      }
  CHECK(down && back);
  net.overlay.set_up(down->id, false);
  net.overlay.set_up(back->id, false);
  remove(*net.ec, a.address);
  CHECK(net.ec->pending_removes() == 2);
  // while holders are down a fetch cannot tell "removed" from "out of
  // reach" (as the single fetch with owners down: TooFewPeers)
  bool gone = false;
  try {
    net.ec->fetch(a.address);
  } catch (MissingBlock&) {
    gone = true;
  } catch (TooFewPeers&) {
    gone = true;
  }
  CHECK(gone);
  int left = 0;
  for (auto& n : net.nodes)
    for (int i = 0; i < 14; ++i) left += n->has(shard_key(a.address, i));
  CHECK(left == 2);  // one on each down node
  // one comes back: its shard goes
  net.overlay.set_up(back->id, true);
  CHECK(wait_for([&] { return net.ec->pending_removes() == 1; }));
  for (int i = 0; i < 14; ++i) CHECK(!back->has(shard_key(a.address, i)));
  // the other is evicted: its debt goes with its silo; only c is repaired
  const auto rep = net.ec->evict(down->id);
  CHECK(net.ec->pending_removes() == 0);
  CHECK(rep.blocks_checked <= 1);
  CHECK_THROW(net.ec->fetch(a.address), MissingBlock);
  CHECK(net.ec->fetch(c.address)->data == c.data);
  CHECK(net.shards(c.address, 14) == 14);
}

// Seeded random operations and membership changes: batched and single
// stores of mixed sizes, nodes going down and coming back (overlay events,
// so the membership thread runs its expansions and settles removals
// concurrently), evictions with their repair, removals.  After every step:
// with at most m nodes unreachable every live block reads back (multi-fetch
// and single fetch) bit-exact; a removed block does not; after an eviction
// every live block again has k + m shards on nodes that are not evicted.
// MEMO_EC_CHAOS_RUNS=N runs N seeds (default 1).
static void chaos_run(uint64_t run_seed) {
  const int k = 10, m = 4, total = k + m;
  Net net(22, k, m);  // at most 4 evictions leave 18 >= k + m nodes
  std::mt19937_64 rng(0x5EED0001 + run_seed);
  std::vector<std::pair<Address, Buffer>> live;
  std::vector<Address> removed;
  int evictions = 0;
  uint64_t seed = 7000 + run_seed * 1000;
  auto pick = [&](auto pred) -> std::shared_ptr<Node> {
    std::vector<std::shared_ptr<Node>> c;
    for (auto& n : net.nodes)
      if (pred(*n)) c.push_back(n);
    return c.empty() ? nullptr : c[rng() % c.size()];
  };
  auto down_count = [&] {
    int d = 0;
    for (auto& n : net.nodes) d += !n->up && !n->evicted;
    return d;
  };
  auto random_size = [&]() -> size_t {
    switch (rng() % 4) {
      case 0: return 4096;
      case 1: return 1 + rng() % 2000;
      case 2: return 1 + rng() % 200000;
      default: return 1 << 20;
    }
  };
  for (int step = 0; step < 60; ++step) {
    const int op = (int)(rng() % 7);
    if (op == 0 || op == 1) {  // a batch, or one block
      std::vector<Block> bs;
      const int nb = op == 0 ? 1 + (int)(rng() % 40) : 1;
      for (int i = 0; i < nb; ++i) bs.push_back(make_chb(random_bytes(random_size(), ++seed)));
      if (op == 0) net.ec->store_many(bs);
      else store(*net.ec, bs[0]);
      for (auto& b : bs) live.emplace_back(b.address, b.data);
    } else if (op == 2) {  // a node goes down
      if (down_count() < m)
        if (auto n = pick([](const Node& x) { return x.up && !x.evicted; })) net.overlay.set_up(n->id, false);
    } else if (op == 3) {  // a node comes back
      if (auto n = pick([](const Node& x) { return !x.up && !x.evicted; })) net.overlay.set_up(n->id, true);
    } else if (op == 4) {  // a down node is evicted: its shards rebuilt elsewhere
      if (evictions < 4)
        if (auto n = pick([](const Node& x) { return !x.up && !x.evicted; })) {
          const auto rep = net.ec->evict(n->id);
          ++evictions;
          CHECK(rep.unrecoverable == 0);
          for (auto& [a, d] : live) CHECK(net.shards(a, total) >= total);
        }
    } else if (op == 5 && !live.empty()) {  // a removal
      const size_t x = rng() % live.size();
      remove(*net.ec, live[x].first);
      removed.push_back(live[x].first);
      live.erase(live.begin() + (long)x);
    } else if (op == 6 && !live.empty()) {  // one block alone
      const auto& [a, d] = live[rng() % live.size()];
      CHECK(net.ec->fetch(a)->data == d);
    }
    // every live block, in one multi-fetch
    std::vector<Address> req;
    for (auto& [a, d] : live) req.push_back(a);
    size_t ok = 0;
    fetch_many(*net.ec, req, [&](const Address& a, std::unique_ptr<Block> b, std::exception_ptr) {
      for (auto& [x, d] : live)
        if (x == a && b && b->data == d) ++ok;
    });
    CHECK(ok == live.size());
    if (ok != live.size()) {
      std::fprintf(stderr, "  seed %llu step %d op %d: %zu of %zu live blocks read back\n",
                   (unsigned long long)run_seed, step, op, ok, live.size());
      return;
    }
    for (auto& a : removed) {
      bool gone = false;
      try {
        net.ec->fetch(a);
      } catch (MissingBlock&) {
        gone = true;
      } catch (TooFewPeers&) {
        gone = true;  // holders of its last shards down: "out of reach"
      }
      CHECK(gone);
    }
  }
  std::printf("  (seed %llu: %zu live, %zu removed, %d evictions)\n", (unsigned long long)run_seed,
              live.size(), removed.size(), evictions);
}

TEST(randomized_membership_and_operations, true) {
  const char* e = std::getenv("MEMO_EC_CHAOS_RUNS");
  const int runs = e ? std::max(1, std::atoi(e)) : 1;
  for (int r = 0; r < runs; ++r) {
    const int before = g_fail;
    chaos_run((uint64_t)r);
    if (g_fail != before) break;
  }
}

// store_many stages at most stage_bytes of shards per chunk: several encode
// calls for a request larger than that, mixed block sizes within a chunk,
// every shard on its owner and every block reads back; a block whose owners
// are too few does not stop the others.
TEST(store_many_stages_in_chunks, true) {
  Net net(16, 10, 4);
  net.o.stage_bytes = 1u << 20;  // ~7 blocks of 100 KiB (14 x 10 KiB shards each)
  net.restart();
  std::vector<Block> blocks;
  for (int i = 0; i < 40; ++i)
    blocks.push_back(make_chb(random_bytes(i % 5 == 0 ? 3000 : 100000 + 37 * i, 4000 + i)));
  const uint64_t calls0 = net.ec->codec().encode_calls();
  net.ec->store_many(blocks);
  CHECK(net.ec->codec().encode_calls() - calls0 >= 5);
  for (auto& b : blocks) {
    CHECK(net.holders(b.address, 14) == 14);
    CHECK(net.ec->fetch(b.address)->data == b.data);
  }
  // 6 of 16 nodes down: 10 reachable owners, every block still stored
  for (int i = 0; i < 6; ++i) net.nodes[i]->up = false;
  std::vector<Block> more;
  for (int i = 0; i < 12; ++i) more.push_back(make_chb(random_bytes(50000, 5000 + i)));
  net.ec->store_many(more);
  for (auto& b : more) CHECK(net.ec->fetch(b.address)->data == b.data);
  // 7 down: 9 reachable owners, below k -- TooFewPeers
  net.nodes[6]->up = false;
  std::vector<Block> last{make_chb(random_bytes(50000, 6000))};
  bool threw = false;
  try {
    net.ec->store_many(last);
  } catch (TooFewPeers&) {
    threw = true;
  }
  CHECK(threw);
}

// A large degraded multi-fetch (a node-loss event) stages its survivors in
// chunks of at most stage_bytes: one lease pair and one codec call per
// chunk, every block right, and no outsized pinned buffer kept afterwards.
TEST(multi_fetch_stages_in_chunks, true) {
  Net net(16, 10, 4);
  net.o.stage_bytes = 2u << 20;  // 2 MiB chunks: 20 x 256 KiB blocks' survivors ~ 5 MiB
  net.o.batch_max = 4;
  net.restart();
  std::vector<Block> blocks;
  for (int i = 0; i < 20; ++i) blocks.push_back(make_chb(random_bytes(256 << 10, 3000 + i)));
  net.ec->store_many(blocks);
  int down = 0;
  for (auto& n : net.nodes)
    if (down < 2 && !n->silo->list().empty()) {
      n->up = false;
      ++down;
    }
  std::vector<Address> req;
  for (auto& b : blocks) req.push_back(b.address);
  const uint64_t seg0 = net.ec->codec().segments_calls(), leases0 = net.ec->arena_leases();
  int ok = 0;
  fetch_many(*net.ec, req, [&](const Address& a, std::unique_ptr<Block> b, std::exception_ptr) {
    for (auto& x : blocks)
      if (b && x.address == a && b->data == x.data) ++ok;
  });
  CHECK(ok == 20);
  const uint64_t calls = net.ec->codec().segments_calls() - seg0;
  CHECK(calls >= 2);                                     // more than one chunk
  CHECK(net.ec->arena_leases() - leases0 == 2 * calls);  // a lease pair per chunk
}

// tests/doughnut.cc:361-373 (missing_block).
TEST(missing_block, true) {
  Net net(16, 10, 4);
  CHECK_THROW(net.ec->fetch(Address::random(flags::immutable_block)), MissingBlock);
  CHECK_THROW(net.ec->fetch(Address::random(flags::mutable_block)), MissingBlock);
}

// tests/doughnut.cc:840-846 (CHB_no_peer): no storage peer -> error.
TEST(CHB_no_peer, true) {
  Net net(4, 10, 4);  // fewer reachable owners than k
  CHECK_THROW(store(*net.ec, make_chb(bytes("no peer"))), TooFewPeers);
}

// Mutable blocks keep the backend (Paxos in memo) -- OKB, doughnut.cc:337-359.
TEST(mutable_blocks_use_backend, true) {
  Net net(16, 10, 4);
  Block b = make_mutable(Address::random(flags::mutable_block), bytes("foo"));
  store(*net.ec, b);
  CHECK(net.ec->fetch(b.address)->data == bytes("foo"));
  Block u = make_mutable(b.address, bytes("foobar"), 2);
  store(*net.ec, u, STORE_UPDATE);
  CHECK(net.ec->fetch(b.address)->data == bytes("foobar"));
}

// Consensus::resign (Consensus.cc:167-176): the plugin hands the leave to
// its mutable-block backend (Paxos::_resign rebalances mutable blocks only,
// Paxos.cc:2091-2131) and leaves its shards in place for the other nodes'
// eviction timers.
namespace {
struct CountingBackend : ReplicationConsensus {
  using ReplicationConsensus::ReplicationConsensus;
  int resigned = 0;
  void _resign() override { ++resigned; }
};
}  // namespace
TEST(resign_forwards_to_backend, true) {
  Overlay overlay;
  for (int i = 0; i < 16; ++i) {
    uint8_t id[32] = {0};
    id[0] = (uint8_t)(i + 1);
    id[1] = 0x52;
    overlay.add_node(Address(id, 0, false), std::make_unique<MemorySilo>());
  }
  auto backend = std::make_unique<CountingBackend>(overlay, 3);
  CountingBackend* bk = backend.get();
  ErasureOptions o;
  o.k = 10;
  o.m = 4;
  ErasureConsensus ec(std::move(backend), overlay, o);
  Block b = make_chb(random_bytes(100000, 77));
  store(ec, b);
  ec.resign();
  CHECK(bk->resigned == 1);
  int shards = 0;
  for (auto& n : overlay.nodes())
    for (int i = 0; i < 14; ++i) shards += n->has(shard_key(b.address, i)) ? 1 : 0;
  CHECK(shards == 14);
  CHECK(ec.fetch(b.address)->data == b.data);
}

// tests/consensus/paxos.cc:7-63 (availability_2/3), for k+m: reads survive
// up to m unreachable owners, a data-shard loss is rebuilt on the GPU, and
// more than m losses raise TooFewPeers.
TEST(availability, true) {
  for (size_t size : {size_t(1), size_t(1000), size_t(1) << 20, size_t(3000001)}) {
    Net net(14, 10, 4);
    Block b = make_chb(random_bytes(size, size));
    store(*net.ec, b);
    auto owners = net.overlay.allocate(b.address, 14);
    // lose 4 owners, three of them holding data shards
    for (int i : {0, 3, 9, 12}) owners[i]->up = false;
    auto f = net.ec->fetch(b.address);
    CHECK(f->data == b.data);
    owners[5]->up = false;  // 5 > m
    CHECK_THROW(net.ec->fetch(b.address), TooFewPeers);
  }
}

// Consensus::fetch(vector<AddressVersion>, ReceiveBlock) (Consensus.cc:101-124,
// used by Model::multifetch): every requested address gets exactly one
// callback, in request order, with the block or its exception; blocks that
// miss data shards are decoded in one GPU call per shard-size bucket instead
// of one call per block.
TEST(multi_fetch_batches_decodes, true) {
  Net net(24, 10, 4);
  std::vector<Block> blocks;
  for (int i = 0; i < 60; ++i)
    blocks.push_back(make_chb(random_bytes((i % 3 == 0 ? 4000 : i % 3 == 1 ? 60000 : 900000) + i, 100 + i)));
  net.ec->store_many(blocks);
  Block mut = make_mutable(Address::random(flags::mutable_block), bytes("meta"));
  store(*net.ec, mut);
  // two nodes down: many blocks lose data shards
  int down = 0;
  for (auto& n : net.nodes)
    if (down < 2 && !n->silo->list().empty()) {
      n->up = false;
      ++down;
    }
  std::vector<Address> req;
  for (auto& b : blocks) req.push_back(b.address);
  const Address missing = make_chb(bytes("never stored")).address;
  req.insert(req.begin() + 7, missing);
  req.push_back(mut.address);
  const uint64_t calls0 = net.ec->codec().rebuild_calls() + net.ec->codec().uniform_calls();
  const uint64_t seg0 = net.ec->codec().segments_calls();
  const uint64_t leases0 = net.ec->arena_leases();
  std::vector<Address> seen;
  int ok = 0, missing_seen = 0;
  fetch_many(*net.ec, req, [&](const Address& a, std::unique_ptr<Block> b, std::exception_ptr e) {
    seen.push_back(a);
    if (a == missing) {
      CHECK(!b && e);
      try {
        std::rethrow_exception(e);
      } catch (MissingBlock&) {  // as the single fetch: MissingBlock, or
        ++missing_seen;          // TooFewPeers while owners are down
      } catch (TooFewPeers&) {
        ++missing_seen;
      } catch (...) {
      }
      return;
    }
    CHECK(b && !e);
    if (!b) return;
    if (a == mut.address) {
      CHECK(b->data == bytes("meta"));
      ++ok;
      return;
    }
    for (auto& x : blocks)
      if (x.address == a) {
        CHECK(b->data == x.data);
        if (b->data == x.data) ++ok;
      }
  });
  CHECK(seen == req);
  CHECK(ok == 61);
  CHECK(missing_seen == 1);
  // the mixed batch (3 size buckets x e in {1, 2}) was ONE codec call
  // (memo_ec_rebuild_segments), no per-group rebuild calls
  const uint64_t batch_calls = net.ec->codec().segments_calls() - seg0;
  CHECK(net.ec->codec().rebuild_calls() + net.ec->codec().uniform_calls() == calls0);
  CHECK(batch_calls == 1);
  // one survivor and one output lease for all the batches of the call (a
  // lease per batch cost a pinned allocation each: 7x slower 4 KiB
  // degraded fetches, profiles/r03_bench_plugin_4k.json)
  CHECK(net.ec->arena_leases() - leases0 == 2);
  size_t need_decode = 0;
  for (auto& b : blocks) {
    const uint64_t c = net.ec->codec().rebuild_calls();
    CHECK(net.ec->fetch(b.address)->data == b.data);
    need_decode += net.ec->codec().rebuild_calls() - c;
  }
  std::fprintf(stderr, "  %zu of 60 blocks needed a decode; the batched fetch used %llu GPU calls\n",
               need_decode, (unsigned long long)batch_calls);
  CHECK(need_decode > 6);
}

// Corrupted shards are erasures: flip bytes in m shards, fetch still exact.
TEST(corrupted_shards_are_erasures, true) {
  Net net(14, 10, 4);
  Block b = make_chb(random_bytes(777777, 3));
  store(*net.ec, b);
  int flipped = 0;
  for (auto& n : net.nodes)
    for (int i : {1, 2, 11, 13}) {
      Key key = shard_key(b.address, i);
      if (!n->has(key)) continue;
      Buffer w = n->silo->get(key);
      w[ShardHeader::kSize + 100] ^= 0x5a;
      n->silo->set(key, w, false, true);
      ++flipped;
    }
  CHECK(flipped == 4);
  CHECK(net.ec->fetch(b.address)->data == b.data);
}

namespace {
// Shard i of `a` on whichever node holds it, re-framed with a valid header
// and CRC around `payload_xor`-damaged bytes: the holder serves a shard
// that passes every per-shard check but has the wrong bytes.
bool reframe_shard(Net& net, const Address& a, int i, uint8_t payload_xor) {
  const Key key = shard_key(a, i);
  for (auto& n : net.nodes) {
    if (!n->has(key)) continue;
    Buffer w = n->silo->get(key);
    const uint8_t* pay = nullptr;
    const ShardHeader h = decode_shard(w, &pay);
    Buffer bad(pay, pay + h.shard_size);
    for (size_t x = 0; x < bad.size(); x += 61) bad[x] ^= payload_xor;
    n->silo->set(key, encode_shard(h, bad.data(), i), false, true);
    return true;
  }
  return false;
}
uint64_t stat(ErasureConsensus& ec, const char* key) {
  return std::stoull(from_json(ec.stats())[key]);
}
int64_t total_fetches(const Net& net) {
  int64_t f = 0;
  for (auto& n : net.nodes) f += n->fetches.load();
  return f;
}
}  // namespace

// A shard with a valid CRC but wrong payload (a buggy holder re-framing, a
// stale shard under a matching header) makes the reassembly fail its CHB
// address.  The reference would move on to the next replica
// (Paxos.cc:502-517); here the other k-subsets of the reachable shards
// out-vote the wrong one, the fetch returns the exact bytes, and the bad
// shard is rewritten on its holder.  m + 1 wrong shards leave no good
// subset: ValidationFailed.
TEST(reframed_shard_recovered_by_subset_retry, true) {
  Net net(16, 10, 4);
  Block b = make_chb(random_bytes(300000, 61)), c = make_chb(random_bytes(90000, 62));
  store(*net.ec, b);
  store(*net.ec, c);
  // a data shard: the first attempt decodes nothing and fails the address
  CHECK(reframe_shard(net, b.address, 3, 0xa5));
  CHECK(net.ec->fetch(b.address)->data == b.data);
  CHECK(stat(*net.ec, "subset_recoveries") == 1);
  CHECK(stat(*net.ec, "corrupt_shards_rewritten") == 1);
  CHECK(net.ec->fetch(b.address)->data == b.data);  // repaired: no second recovery
  CHECK(stat(*net.ec, "subset_recoveries") == 1);
  // a parity shard used by a degraded decode, through the multi-fetch
  std::shared_ptr<Node> d0;
  for (auto& n : net.nodes)
    if (n->has(shard_key(c.address, 0))) d0 = n;
  CHECK(d0 != nullptr);
  for (int i = 10; i < 14; ++i) CHECK(reframe_shard(net, c.address, i, 0x3c));
  net.overlay.set_up(d0->id, false);
  // four wrong parity shards and one data shard out of reach: 13 shards in
  // hand, every k-subset holds a wrong one -- refused, not returned
  CHECK_THROW(net.ec->fetch(c.address), ValidationFailed);
  net.overlay.set_up(d0->id, true);
  // with the data holder back, the multi-fetch reassembles from the data
  // shards, needing no parity
  int got = 0;
  fetch_many(*net.ec, std::vector<Address>{c.address, b.address},
                [&](const Address& a, std::unique_ptr<Block> blk, std::exception_ptr e) {
                  if (!e && blk && blk->data == (a == c.address ? c.data : b.data)) ++got;
                });
  CHECK(got == 2);
  // one wrong parity shard in a degraded multi-fetch: recovered on the pool
  Block d = make_chb(random_bytes(120000, 63));
  store(*net.ec, d);
  std::shared_ptr<Node> dd;
  for (auto& n : net.nodes)
    if (n->has(shard_key(d.address, 5))) dd = n;
  // parities 11-13 wrong, 10 right: whichever parity the decode took, the
  // block comes back (a recovery when it was a wrong one)
  for (int i = 11; i < 14; ++i) CHECK(reframe_shard(net, d.address, i, 0x11));
  net.overlay.set_up(dd->id, false);
  for (int r = 0; r < 4; ++r) {
    got = 0;
    fetch_many(*net.ec, std::vector<Address>{d.address},
                  [&](const Address&, std::unique_ptr<Block> blk, std::exception_ptr e) {
                    if (!e && blk && blk->data == d.data) ++got;
                  });
    CHECK(got == 1);
    CHECK(net.ec->fetch(d.address)->data == d.data);
  }
  net.overlay.set_up(dd->id, true);
  // m + 1 = 5 wrong shards: no k-subset reassembles to the address
  Block e5 = make_chb(random_bytes(50000, 64));
  store(*net.ec, e5);
  for (int i : {0, 2, 4, 11, 13}) CHECK(reframe_shard(net, e5.address, i, 0x77));
  CHECK_THROW(net.ec->fetch(e5.address), ValidationFailed);
}

// A degraded fetch reads only what the decode needs: with one data holder
// down, k shard reads (9 data + 1 parity) instead of every parity shard,
// plus the configured hedge; the parity holders asked vary from fetch to
// fetch (shuffled, least-loaded first, Paxos.cc:488-500), and with the
// balancing off the first parity holder is always asked.
TEST(degraded_fetch_reads_k_shards, true) {
  for (int hedge : {0, 1}) {
    for (bool balanced : {true, false}) {
      Net net(16, 10, 4);
      net.o.fetch_hedge = hedge;
      net.o.balanced_transfers = balanced;
      net.restart();
      Block b = make_chb(random_bytes(200000, 70 + hedge));
      store(*net.ec, b);
      std::shared_ptr<Node> d2;
      std::map<int, std::shared_ptr<Node>> parity_holder;
      for (auto& n : net.nodes)
        for (int i = 0; i < 14; ++i)
          if (n->has(shard_key(b.address, i))) {
            if (i == 2) d2 = n;
            if (i >= 10) parity_holder[i] = n;
          }
      CHECK(d2 && parity_holder.size() == 4);
      // healthy: the k data shards only
      int64_t f0 = total_fetches(net);
      CHECK(net.ec->fetch(b.address)->data == b.data);
      CHECK(total_fetches(net) - f0 == 10);
      net.overlay.set_up(d2->id, false);
      std::set<int> asked;
      for (int r = 0; r < 24; ++r) {
        std::map<int, int64_t> before;
        for (auto& [i, n] : parity_holder) before[i] = n->fetches.load();
        f0 = total_fetches(net);
        CHECK(net.ec->fetch(b.address)->data == b.data);
        CHECK(total_fetches(net) - f0 == 10 + hedge);
        for (auto& [i, n] : parity_holder)
          if (n->fetches.load() > before[i]) asked.insert(i);
      }
      if (balanced) CHECK(asked.size() >= 3);
      else CHECK(asked.size() == (size_t)(1 + hedge) && asked.count(10) == 1);
      net.overlay.set_up(d2->id, true);
    }
  }
}

// A silo that refuses a shard (silo::InsufficientSpace) fails that shard
// only: the batch's other shards are stored and every stored shard is in
// the placement index (nothing orphaned in a silo), the blocks read back.
TEST(full_silo_fails_only_its_shards, true) {
  Net net(15, 10, 4);
  uint8_t id[32] = {0};
  id[0] = 0xf0;
  id[1] = 0x11;
  net.nodes.push_back(net.overlay.add_node(Address(id, 0, false), std::make_unique<MemorySilo>(3000)));
  net.o.auto_expand = false;
  net.restart();
  std::vector<Block> blocks;
  for (int i = 0; i < 64; ++i) blocks.push_back(make_chb(random_bytes(60000 + 13 * i, 400 + i)));
  net.ec->store_many(blocks);
  size_t indexed = 0, on_silos = 0;
  for (auto& n : net.nodes) indexed += net.ec->node_blocks(n->id);
  for (auto& b : blocks) {
    on_silos += net.holders(b.address, 14);
    CHECK(net.ec->fetch(b.address)->data == b.data);
  }
  CHECK(indexed == on_silos);
  CHECK(net.nodes.back()->silo->usage() == 0);  // every shard is > 3000 bytes
  CHECK(net.ec->under_placed() > 0);             // the blocks it was to hold
}

// A client with no placement of a block removes every shard of it, also
// shards on nodes ranked past k + m (stored while top-ranked nodes were
// down), by asking the whole membership.
TEST(remove_unknown_block_reaches_every_holder, true) {
  Net net(16, 10, 4);
  net.o.auto_expand = false;
  net.restart();
  Block b = make_chb(random_bytes(30000, 80));
  auto rank = net.overlay.rank(b.address);
  net.overlay.set_up(rank[0]->id, false);
  net.overlay.set_up(rank[1]->id, false);
  store(*net.ec, b);
  net.overlay.set_up(rank[0]->id, true);
  net.overlay.set_up(rank[1]->id, true);
  CHECK(net.shards(b.address, 14) == 14);
  CHECK(!rank[0]->has(shard_key(b.address, 0)));
  ErasureOptions o = net.o;
  o.rescan = false;
  ErasureConsensus other(std::make_unique<ReplicationConsensus>(net.overlay, 3), net.overlay, o);
  std::vector<int64_t> before;
  for (auto& n : net.nodes) before.push_back(n->remove_requests.load());
  remove(other, b.address);
  CHECK(net.shards(b.address, 14) == 0);
  // one removal request per node, naming every shard key (not k+m requests)
  for (size_t i = 0; i < net.nodes.size(); ++i) CHECK(net.nodes[i]->remove_requests.load() - before[i] == 1);
}

// A removal owed to a holder that was down is void when the block was
// stored again with that holder holding the shard before the node's return
// was processed: the live shard stays.
TEST(owed_removal_spares_restored_shard, true) {
  Net net(16, 10, 4);
  net.o.auto_expand = false;
  net.restart();
  Block b = make_chb(random_bytes(45000, 81));
  store(*net.ec, b);
  std::shared_ptr<Node> h;
  for (auto& n : net.nodes)
    if (n->has(shard_key(b.address, 4))) h = n;
  CHECK(h != nullptr);
  net.overlay.set_up(h->id, false);
  remove(*net.ec, b.address);
  CHECK(net.ec->pending_removes() == 1);
  h->up = true;  // back, its return not yet signalled
  store(*net.ec, b);
  CHECK(h->has(shard_key(b.address, 4)) && net.shards(b.address, 14) == 14);
  h->up = false;
  net.overlay.set_up(h->id, true);  // the return: owed removals settle
  CHECK(wait_for([&] { return net.ec->pending_removes() == 0; }));
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  CHECK(net.shards(b.address, 14) == 14);
  CHECK(net.ec->fetch(b.address)->data == b.data);
}

// CHB.cc:243-258 through the plugin: a group member's removal of a CHB whose
// owner grants the group write access takes every shard; a group without
// write access is refused with every shard left.
TEST(remove_owned_chb_by_group_member, true) {
  Net net(16, 10, 4);
  OwnerDirectory dir;
  const KeyPair owner_k = KeyPair::generate(), g1 = KeyPair::generate(), g2 = KeyPair::generate();
  const Buffer G = KeyPair::generate().public_key, R = KeyPair::generate().public_key;
  const Address owner = Address::random(flags::mutable_block);
  dir.set_group(G, {g1.public_key});
  dir.set_group(R, {g2.public_key});
  dir.set(owner, OwnerAcl{owner_k.public_key, {}, false, {{G, true}, {R, false}}});
  net.ec->set_owner_directory(&dir);
  Block b = make_chb(random_bytes(33000, 82), bytes("salt"), owner);
  store(*net.ec, b);
  CHECK_THROW(remove(*net.ec, b.address, chb_sign_remove_group(b.address, R, g2, 1)), ValidationFailed);
  CHECK_THROW(remove(*net.ec, b.address, chb_sign_remove_group(b.address, G, g1, 2)), ValidationFailed);
  CHECK(net.shards(b.address, 14) == 14);
  remove(*net.ec, b.address, chb_sign_remove_group(b.address, G, g1, 1));
  CHECK(net.shards(b.address, 14) == 0);
}

// tests/doughnut.cc:1651-1691 (evict_faulty), 1484-1512 (expand_new_block),
// 2158-2176 (CHB_unavailable): after owners are lost the shards are rebuilt
// on new owners, after which the block survives m further losses.
TEST(evict_and_repair, true) {
  Net net(24, 10, 4);
  std::vector<Block> blocks;
  for (int i = 0; i < 40; ++i) blocks.push_back(make_chb(random_bytes(50000 + 997 * i, i)));
  net.ec->store_many(blocks);
  // evict 4 nodes that hold shards
  int evicted = 0;
  for (auto& n : net.nodes)
    if (evicted < 4 && !n->silo->list().empty()) {
      n->evicted = true;
      ++evicted;
    }
  auto rep = net.ec->repair();
  CHECK(rep.unrecoverable == 0);
  CHECK(rep.blocks_repaired > 0);
  CHECK(rep.codec_calls >= 1 && rep.codec_calls < rep.blocks_repaired);  // batched
  for (auto& b : blocks) CHECK(net.shards(b.address, 14) == 14);
  // 4 more failures among the remaining nodes: still readable
  int down = 0;
  for (auto& n : net.nodes)
    if (!n->evicted && down < 4 && !n->silo->list().empty()) {
      n->up = false;
      ++down;
    }
  for (auto& b : blocks) CHECK(net.ec->fetch(b.address)->data == b.data);
}

// CHB_unavailable (doughnut.cc:2158-2176): an owner refusing the store (its
// store barrier raises Unavailable) leaves the block on k+m-1 owners; once
// the barrier opens, the background rebalancing of under-placed stores
// (rebalance_auto_expand, Paxos.cc:1428-1438) places the missing shard on
// it without any repair call.  Exactly k+m nodes: the refusing owner is the
// only node that can take the shard, so the retries before the barrier
// opens cannot place it elsewhere.
TEST(CHB_unavailable, true) {
  Net net(14, 10, 4);
  std::atomic<int> rebalanced{0}, under{0}, under_held{-1};
  net.ec->on_rebalanced([&](const Address&) { ++rebalanced; });
  net.ec->on_under_placed([&](const Address&, int held) {
    under_held = held;
    ++under;
  });
  Block b = make_chb(bytes("CHB_unavailable"));
  auto owners = net.overlay.allocate(b.address, 14);
  owners[2]->fail_stores = true;
  store(*net.ec, b);
  CHECK(net.shards(b.address, 14) == 13);
  CHECK(net.ec->under_placed() == 1);
  CHECK(net.ec->stats().find("\"under_placed\": 1") != std::string::npos);
  std::this_thread::sleep_for(std::chrono::milliseconds(50));  // retries meet the barrier
  CHECK(rebalanced.load() == 0 && net.shards(b.address, 14) == 13);
  // a retry that could not place the shard reported the block
  CHECK(wait_for([&] { return under.load() > 0; }));
  CHECK(under_held.load() == 13);
  owners[2]->fail_stores = false;
  CHECK(wait_for([&] { return rebalanced.load() > 0; }));
  CHECK(net.shards(b.address, 14) == 14);
  CHECK(net.holders(b.address, 14) == 14);
  CHECK(net.ec->under_placed() == 0);
  CHECK(net.ec->stats().find("\"under_placed\": 0") != std::string::npos);
  CHECK(net.ec->fetch(b.address)->data == b.data);
}

// evict_chain(expand) (tests/doughnut.cc:2008-2058): on exactly k+m nodes,
// evict an owner: no node can take its shard, so the block is reported
// under-placed (under_replicated(address, 2) there, (address, 13) here);
// a newcomer then gets the shard (rebalanced).  16 rotations.
TEST(evict_chain_expand, true) {
  Net net(14, 10, 4);
  std::mutex mu;
  std::vector<std::pair<Address, int>> under;
  std::atomic<int> rebalanced{0};
  net.ec->on_under_placed([&](const Address& a, int held) {
    std::lock_guard<std::mutex> g(mu);
    under.emplace_back(a, held);
  });
  net.ec->on_rebalanced([&](const Address&) { ++rebalanced; });
  Block b = make_chb(random_bytes(5000, 2008));
  store(*net.ec, b);
  CHECK(net.holders(b.address, 14) == 14);
  std::mt19937 rng(2008);
  for (int round = 0; round < 16; ++round) {
    std::vector<std::shared_ptr<Node>> live;
    for (auto& n : net.nodes)
      if (!n->evicted) live.push_back(n);
    auto victim = live[rng() % live.size()];
    victim->up = false;
    const size_t u0 = [&] {
      std::lock_guard<std::mutex> g(mu);
      return under.size();
    }();
    net.ec->evict(victim->id);
    {
      std::lock_guard<std::mutex> g(mu);
      CHECK(under.size() == u0 + 1);
      if (under.size() == u0 + 1) CHECK(under.back().first == b.address && under.back().second == 13);
    }
    CHECK(net.ec->under_placed() == 1);
    const int r0 = rebalanced.load();
    net.add();  // discovery: the block expands onto the newcomer
    CHECK(wait_for([&] { return rebalanced.load() > r0; }));
    CHECK(net.holders(b.address, 14) == 14);
    CHECK(net.ec->under_placed() == 0);
  }
  CHECK(net.ec->fetch(b.address)->data == b.data);
}

// A node that comes back is a discovery (Paxos::_discovered, Paxos.cc:969-
// 975): on exactly k+m nodes, a block stored while one node is away lands
// on k+m-1 owners (reported under-placed: no free node); when the node
// returns, its missing shard goes to it without any new node or repair call.
TEST(returning_node_takes_missing_shards, true) {
  Net net(14, 10, 4);
  std::atomic<int> under{0};
  net.ec->on_under_placed([&](const Address&, int) { ++under; });
  auto away = net.nodes[5];
  net.overlay.set_up(away->id, false);
  Block b = make_chb(random_bytes(40000, 969));
  store(*net.ec, b);
  CHECK(net.shards(b.address, 14) == 13);
  CHECK(wait_for([&] { return under.load() > 0; }));
  net.overlay.set_up(away->id, true);
  CHECK(wait_for([&] { return net.shards(b.address, 14) == 14; }));
  CHECK(net.holders(b.address, 14) == 14);
  CHECK(net.ec->under_placed() == 0);
}

// Background retries count free nodes, not node totals: with 3 of a block's
// 13 holders down and free nodes up, the block is still placeable (the down
// holders keep their shards and cannot take another).
TEST(retry_with_down_holders_and_free_nodes, true) {
  Net net(16, 10, 4);
  Block b = make_chb(random_bytes(30000, 1566));
  auto owners = net.overlay.allocate(b.address, 14);
  std::vector<std::shared_ptr<Node>> spare;
  for (auto& n : net.nodes)
    if (std::find(owners.begin(), owners.end(), n) == owners.end()) spare.push_back(n);
  CHECK(spare.size() == 2);
  owners[13]->fail_stores = true;
  for (auto& n : spare) n->fail_stores = true;
  store(*net.ec, b);
  CHECK(net.shards(b.address, 14) == 13);
  // three holders go away silently; the free nodes start accepting
  for (int i = 0; i < 3; ++i) owners[i]->up = false;
  for (auto& n : spare) n->fail_stores = false;
  owners[13]->fail_stores = false;
  CHECK(wait_for([&] { return net.ec->under_placed() == 0; }));
  int placed = 0;
  for (auto& n : net.nodes)
    if (n->up && n->has(shard_key(b.address, 13))) ++placed;
  CHECK(placed == 1);
}

// evict_faulty (doughnut.cc:1651-1691): a block stored on all k+m nodes; a
// newcomer joins; one owner disconnects and is evicted explicitly (the
// reference calls Local::evict() on the survivors) -> its shard is rebuilt on
// the newcomer, the only node without one, and the block then survives m
// further losses.
TEST(evict_faulty, true) {
  Net net(14, 10, 4);
  std::atomic<int> rebalanced{0};
  net.ec->on_rebalanced([&](const Address&) { ++rebalanced; });
  Block b = make_chb(random_bytes(200000, 1651));
  store(*net.ec, b);
  CHECK(net.holders(b.address, 14) == 14);
  auto d = net.add();  // fourth DHT: a discovery, nothing under-placed
  std::shared_ptr<Node> faulty;
  for (auto& n : net.nodes)
    if (n != d && n->has(shard_key(b.address, 5))) faulty = n;
  CHECK(faulty != nullptr);
  faulty->up = false;  // disconnect third DHT
  auto rep = net.ec->evict(faulty->id);
  CHECK(rep.blocks_repaired == 1 && rep.shards_rebuilt == 1 && rep.unrecoverable == 0);
  CHECK(rebalanced.load() == 1);
  CHECK(d->has(shard_key(b.address, 5)));
  int down = 0;  // disconnect first DHT (and m - 1 more owners)
  for (auto& n : net.nodes)
    if (n != d && n != faulty && down < 4) {
      n->up = false;
      ++down;
    }
  CHECK(net.ec->fetch(b.address)->data == b.data);
}

// expand_new_block (doughnut.cc:1484-1512): a block written while some of
// its owners refuse stores is rebalanced onto them once they accept, and then
// survives the loss of m other owners.
TEST(expand_new_block, true) {
  Net net(14, 10, 4);
  std::atomic<int> rebalanced{0};
  net.ec->on_rebalanced([&](const Address&) { ++rebalanced; });
  Block b = make_chb(random_bytes(300000, 1484));
  auto owners = net.overlay.allocate(b.address, 14);
  owners[6]->fail_stores = true;
  owners[11]->fail_stores = true;
  store(*net.ec, b);
  CHECK(net.shards(b.address, 14) == 12);
  owners[6]->fail_stores = false;
  owners[11]->fail_stores = false;
  CHECK(wait_for([&] { return net.shards(b.address, 14) == 14; }));
  CHECK(rebalanced.load() > 0);
  CHECK(net.holders(b.address, 14) == 14);
  for (int i : {0, 3, 8, 13}) owners[i]->up = false;  // m losses, none of them the late owners
  CHECK(net.ec->fetch(b.address)->data == b.data);
}

// Concurrent stores from many threads are batched into few GPU encodes.
TEST(concurrent_stores_batch_on_gpu, true) {
  Net net(16, 10, 4, 2000);
  std::vector<Block> blocks;
  for (int i = 0; i < 64; ++i) blocks.push_back(make_chb(random_bytes(65536, 100 + i)));
  std::vector<std::thread> ts;
  for (int t = 0; t < 16; ++t)
    ts.emplace_back([&, t] {
      for (int i = t; i < 64; i += 16) store(*net.ec, blocks[i]);
    });
  for (auto& t : ts) t.join();
  const auto calls = net.ec->codec().encode_calls();
  CHECK(calls < 64);
  for (auto& b : blocks) CHECK(net.ec->fetch(b.address)->data == b.data);
  std::printf("  (64 concurrent stores -> %llu GPU encode calls)\n", (unsigned long long)calls);
}

// Multi-GPU split: a batch cut into per-device block
// ranges, one host thread each, gives the single-device bytes.  The device
// list repeats GPU 0 so the split runs on a one-GPU box.
TEST(multi_device_split_matches_single, true) {
  const int k = 10, m = 4, n = 37;
  const size_t B = 30000, S = memo_ec_shard_size(B, k);
  Buffer data(n * k * S);
  for (size_t i = 0; i < data.size(); ++i) data[i] = (uint8_t)(i * 2654435761u >> 13);
  Buffer p1(n * m * S), p3(n * m * S);
  Codec one(0, 1), three(std::vector<int>{0, 0, 0}, 2);
  CHECK(three.devices() == 3);
  one.encode(k, m, S, n, data.data(), p1.data());
  three.encode(k, m, S, n, data.data(), p3.data());
  CHECK(p1 == p3);
  // rebuild shards 0 and 12 of every block from the other k
  std::vector<uint8_t> sidx(n * k), lidx(n * 2);
  Buffer surv(n * k * S), o1(n * 2 * S), o3(n * 2 * S);
  for (int b = 0; b < n; ++b) {
    int t = 0;
    for (int i = 0; i < k + m && t < k; ++i)
      if (i != 0 && i != 12) {
        sidx[b * k + t] = (uint8_t)i;
        const uint8_t* src = i < k ? &data[(b * k + i) * S] : &p1[(b * m + i - k) * S];
        std::memcpy(&surv[(b * k + t) * S], src, S);
        ++t;
      }
    lidx[b * 2] = 0;
    lidx[b * 2 + 1] = 12;
  }
  one.rebuild(k, m, S, n, sidx.data(), surv.data(), lidx.data(), 2, o1.data());
  three.rebuild(k, m, S, n, sidx.data(), surv.data(), lidx.data(), 2, o3.data());
  CHECK(o1 == o3);
  for (int b = 0; b < n; ++b) {
    CHECK(std::memcmp(&o1[(b * 2) * S], &data[(b * k) * S], S) == 0);
    CHECK(std::memcmp(&o1[(b * 2 + 1) * S], &p1[(b * m + 2) * S], S) == 0);
  }
  // the mixed-geometry call split the same way: every device takes its
  // share of each segment (per-block blocks 0..36 with e = 2; the same
  // blocks as a shared-pattern segment with e = 1, shard 12 only)
  Buffer s1(n * S), s3(n * S);
  const uint8_t pat_s[10] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10}, pat_l[1] = {12};
  for (Codec* c : {&one, &three}) {
    Buffer& so = c == &one ? s1 : s3;
    Buffer& po = c == &one ? o1 : o3;
    std::fill(po.begin(), po.end(), 0);
    memo_ec_rebuild_segment segs[2] = {
        {k, m, S, (size_t)n, sidx.data(), surv.data(), lidx.data(), 2, 0, po.data()},
        {k, m, S, (size_t)n, pat_s, surv.data(), pat_l, 1, 1, so.data()}};
    c->rebuild_segments(std::vector<memo_ec_rebuild_segment>(segs, segs + 2));
  }
  CHECK(o1 == o3 && s1 == s3);
  for (int b = 0; b < n; ++b) {
    CHECK(std::memcmp(&o1[(b * 2) * S], &data[(b * k) * S], S) == 0);
    CHECK(std::memcmp(&s1[b * S], &p1[(b * m + 2) * S], S) == 0);
  }
}


// An owned CHB (CHB.cc:264-289: the owner enters the address) stored as
// shards and read back with 4 owners down: the shards carry the owner, the
// reassembled block validates, and a shard set claiming another owner does
// not pass for it.
TEST(owned_chb_round_trip_degraded, true) {
  Net net(16, 10, 4);
  const Address owner = Address::random(flags::mutable_block);
  Block b = make_chb(random_bytes(300001, 41), bytes("salt!"), owner);
  store(*net.ec, b);
  auto owners = net.overlay.allocate(b.address, 14);
  for (int i : {0, 2, 5, 13}) owners[i]->up = false;
  auto f = net.ec->fetch(b.address);
  CHECK(f->data == b.data && f->owner == owner && f->salt == b.salt);
  CHECK(chb_valid(b.address, f->salt, f->owner, f->data));
  // every reachable shard re-framed with another owner (a valid CRC): the
  // fetch rejects them as another block's shards
  const Address other = Address::random(flags::mutable_block);
  for (auto& n : net.nodes)
    for (int i = 0; i < 14; ++i) {
      const Key key = shard_key(b.address, i);
      if (!n->up || !n->has(key)) continue;
      const uint8_t* p = nullptr;
      const Buffer w = n->silo->get(key);  // p points into it
      ShardHeader h = decode_shard(w, &p);
      h.owner = other;
      n->silo->set(key, encode_shard(h, p), false, true);
    }
  net.restart();  // no placement record: the first shard sets the reference
  CHECK_THROW(net.ec->fetch(b.address), ValidationFailed);
}

// a survivor's header is checked against the placement
// record before repair copies its payload.  A shard of another code planted
// under a survivor's key (valid CRC, larger shard size) is an erasure: it is
// rebuilt and replaced, not copied into the batch.
TEST(repair_rejects_foreign_shard, true) {
  Net net(20, 4, 2);
  Block b = make_chb(random_bytes(40000, 5));
  store(*net.ec, b);
  auto owners = net.overlay.allocate(b.address, 6);
  // shard 1 replaced by a k = 2 shard of a 3x larger block, same address
  ShardHeader h;
  h.k = 2;
  h.m = 1;
  h.index = 1;
  h.block_size = 120000;
  h.shard_size = memo_ec_shard_size(120000, 2);
  h.address = b.address;
  Buffer junk = random_bytes(h.shard_size, 9);
  owners[1]->silo->set(shard_key(b.address, 1), encode_shard(h, junk.data()), false, true);
  owners[4]->evicted = true;
  auto rep = net.ec->repair();
  CHECK(rep.unrecoverable == 0 && rep.blocks_repaired == 1);
  CHECK(rep.shards_rebuilt == 2);  // the evicted node's shard and the foreign one
  for (int i = 0; i < 6; ++i) {
    int valid = 0;
    for (auto& n : net.nodes) {
      Buffer w;
      if (n->evicted || !n->silo->try_get(shard_key(b.address, i), w)) continue;
      try {
        ShardHeader x = decode_shard(w, nullptr);
        valid += x.k == 4 && x.index == i;
      } catch (ValidationFailed&) {
      }
    }
    CHECK(valid == 1);
  }
  for (int i : {0, 2}) owners[i]->up = false;
  CHECK(net.ec->fetch(b.address)->data == b.data);
}

// tests/doughnut.cc:1514-1571 (expand_newcomer): a block stored while fewer
// than k+m owners were reachable is under-placed; when new nodes join, its
// missing shards are rebuilt onto them in the background.
TEST(expand_newcomer, true) {
  Net net(12, 10, 4);  // 12 nodes: shards 12 and 13 have no owner
  std::vector<Address> rebalanced;
  std::mutex mu;
  net.ec->on_rebalanced([&](const Address& a) {
    std::lock_guard<std::mutex> g(mu);
    rebalanced.push_back(a);
  });
  Block b = make_chb(random_bytes(100000, 77));
  store(*net.ec, b);
  CHECK(net.shards(b.address, 14) == 12);
  net.add();
  net.add();  // discovery -> rebalancing
  CHECK(wait_for([&] { std::lock_guard<std::mutex> g(mu); return !rebalanced.empty(); }));
  CHECK(net.shards(b.address, 14) == 14);
  CHECK(net.holders(b.address, 14) == 14);
  int down = 0;  // now m losses are survivable
  for (auto& n : net.nodes)
    if (down < 4 && net.ec->node_blocks(n->id)) {
      n->up = false;
      ++down;
    }
  CHECK(net.ec->fetch(b.address)->data == b.data);
}

// tests/doughnut.cc:1609-1634 (expand_from_disk): a fresh consensus over the
// same silos rebuilds its index from the shard headers; an under-placed
// block found there is expanded onto the nodes present, and evicting a node
// repairs exactly the blocks that node held (per-node index from disk).
TEST(expand_from_disk, true) {
  Net net(12, 10, 4);
  std::vector<Block> blocks;
  for (int i = 0; i < 24; ++i) blocks.push_back(make_chb(random_bytes(20000 + 777 * i, 300 + i)));
  net.ec->store_many(blocks);
  for (auto& b : blocks) CHECK(net.shards(b.address, 14) == 12);
  net.ec.reset();        // the node goes away ...
  net.add();
  net.add();             // ... the network grows meanwhile ...
  std::atomic<int> rebalanced{0};
  net.o.rescan = true;
  net.restart();         // ... and it restarts from its silos
  net.ec->on_rebalanced([&](const Address&) { ++rebalanced; });
  CHECK(wait_for([&] {
    for (auto& b : blocks)
      if (net.shards(b.address, 14) != 14) return false;
    return true;
  }));
  // per-node index rebuilt: evict one holder, exactly its blocks repaired
  std::shared_ptr<Node> victim;
  for (auto& n : net.nodes)
    if (!victim && net.ec->node_blocks(n->id) > 0) victim = n;
  const size_t held = net.ec->node_blocks(victim->id);
  CHECK(held > 0);
  net.restart();  // the index once more from disk only
  CHECK(net.ec->node_blocks(victim->id) == held);
  victim->up = false;
  auto rep = net.ec->evict(victim->id);
  CHECK(rep.blocks_checked == held && rep.blocks_repaired == held && rep.unrecoverable == 0);
  CHECK(net.ec->node_blocks(victim->id) == 0);
  for (auto& b : blocks) CHECK(net.ec->fetch(b.address)->data == b.data);
}

// tests/doughnut.cc:1693-1719 (evict_removed_blocks) with the eviction timer
// (Paxos.cc:985-1009): a node that disappears is evicted after the delay and
// its blocks repaired, a removed block is not brought back; a node that
// returns within the delay is not evicted.
TEST(evict_removed_blocks, true) {
  Net net(16, 10, 4, 200, /*eviction_delay_ms=*/150);
  std::vector<Block> bs;
  for (int i = 0; i < 3; ++i) bs.push_back(make_chb(random_bytes(50000, 900 + i)));
  for (auto& b : bs) store(*net.ec, b);
  remove(*net.ec, bs[1].address);
  CHECK(net.shards(bs[1].address, 14) == 0);
  std::shared_ptr<Node> a, c;
  for (auto& n : net.nodes) {
    if (!a && net.ec->node_blocks(n->id) == 2) a = n;
    else if (!c && net.ec->node_blocks(n->id) >= 1) c = n;
  }
  CHECK(a && c);
  // a blip shorter than the delay: no eviction
  net.overlay.set_up(c->id, false);
  CHECK(wait_for([&] { return net.ec->pending_evictions() == 1; }));
  std::this_thread::sleep_for(std::chrono::milliseconds(30));
  net.overlay.set_up(c->id, true);
  // a real disappearance: evicted after ~150 ms, blocks repaired
  net.overlay.set_up(a->id, false);
  CHECK(wait_for([&] { return a->evicted.load() && net.ec->node_blocks(a->id) == 0; }));
  CHECK(!c->evicted);
  CHECK(net.ec->pending_evictions() == 0);
  CHECK(net.shards(bs[0].address, 14) == 14 && net.shards(bs[2].address, 14) == 14);
  CHECK(net.shards(bs[1].address, 14) == 0);
  CHECK_THROW(net.ec->fetch(bs[1].address), MissingBlock);
  for (int i : {0, 2}) CHECK(net.ec->fetch(bs[i].address)->data == bs[i].data);
}

// The repair of one evicted node: every block that node held shard i of
// shares one erasure pattern, so those blocks form shared-pattern segments
// (product tables formed once), and the whole repair is one codec call
// (memo_ec_rebuild_segments), not one per block or group.
TEST(evict_one_node_uses_uniform_rebuild, true) {
  Net net(16, 10, 4);
  net.o.uniform_min_bytes = 0;  // small blocks here: take every shared pattern
  net.restart();
  std::vector<Block> blocks;
  for (int i = 0; i < 96; ++i) blocks.push_back(make_chb(random_bytes(30000 + 13 * i, 5000 + i)));
  net.ec->store_many(blocks);
  std::shared_ptr<Node> victim;
  for (auto& n : net.nodes)
    if (!victim || net.ec->node_blocks(n->id) > net.ec->node_blocks(victim->id)) victim = n;
  const size_t held = net.ec->node_blocks(victim->id);
  const uint64_t u0 = net.ec->codec().uniform_segments();
  const uint64_t leases0 = net.ec->arena_leases();
  victim->up = false;
  auto rep = net.ec->evict(victim->id);
  CHECK(rep.blocks_repaired == held && rep.unrecoverable == 0);
  CHECK(net.ec->arena_leases() - leases0 == 2);  // one lease pair per repair chunk
  const uint64_t uniform = net.ec->codec().uniform_segments() - u0;
  std::printf("  (%zu blocks repaired in %zu codec calls, %llu shared-pattern segments)\n", held,
              rep.codec_calls, (unsigned long long)uniform);
  CHECK(uniform >= 1);
  CHECK(rep.codec_calls == 1);
  for (auto& b : blocks) CHECK(net.ec->fetch(b.address)->data == b.data);
}

// A real restart: every node's shards in a filesystem silo; the whole
// in-process network (overlay, nodes, consensus) is torn down and rebuilt
// over the same directories.  The fresh consensus rebuilds its indices from
// the shard headers on disk, reads every block, and, after one node's disk
// is lost and the node evicted, repairs exactly that node's blocks.
TEST(restart_from_filesystem_silos, true) {
  const std::string root = temp_dir("net");
  const int N = 16;
  std::vector<Block> blocks;
  for (int i = 0; i < 40; ++i) blocks.push_back(make_chb(random_bytes(3000 + 4099 * i, 700 + i)));
  ErasureOptions o;
  o.k = 10;
  o.m = 4;
  o.eviction_delay_ms = -1;
  auto node_id = [](int i) {
    uint8_t id[32] = {0};
    id[0] = (uint8_t)(i + 1);
    id[1] = 0x46;
    return Address(id, 0, false);
  };
  {
    Overlay ov;
    for (int i = 0; i < N; ++i)
      ov.add_node(node_id(i), std::make_unique<FilesystemSilo>(root + "/n" + std::to_string(i)));
    ErasureConsensus ec(std::make_unique<ReplicationConsensus>(ov, 3), ov, o);
    ec.store_many(blocks);
  }
  Overlay ov;
  std::vector<std::shared_ptr<Node>> nodes;
  for (int i = 0; i < N; ++i)
    nodes.push_back(ov.add_node(node_id(i), std::make_unique<FilesystemSilo>(root + "/n" + std::to_string(i))));
  auto ec = std::make_unique<ErasureConsensus>(std::make_unique<ReplicationConsensus>(ov, 3), ov, o);
  CHECK(from_json(ec->stats())["blocks"] == "40");
  for (auto& b : blocks) CHECK(ec->fetch(b.address)->data == b.data);
  // node 3 loses its disk and is evicted
  const size_t held = ec->node_blocks(nodes[3]->id);
  CHECK(held > 0);
  nodes[3]->up = false;
  std::filesystem::remove_all(root + "/n3");
  auto rep = ec->evict(nodes[3]->id);
  CHECK(rep.blocks_repaired == held && rep.unrecoverable == 0);
  int down = 0;
  for (auto& n : nodes)
    if (n != nodes[3] && down < 4) {
      n->up = false;
      ++down;
    }
  for (auto& b : blocks) CHECK(ec->fetch(b.address)->data == b.data);
  ec.reset();
  std::filesystem::remove_all(root);
}

// Redundancy JSON (Consensus::redundancy, Paxos.cc:2218-2225 shape).
TEST(redundancy_json, true) {
  Net net(16, 10, 4);
  auto r = from_json(net.ec->redundancy());
  CHECK(r["type"] == "erasure" && r["k"] == "10" && r["m"] == "4" && r["desired_factor"] == "1.4");
  Overlay ov;
  for (int i = 0; i < 8; ++i) ov.add_node(Address::random(0), std::make_unique<MemorySilo>());
  auto c = make_consensus(ov, "{\"type\": \"erasure\", \"data-shards\": 4, \"parity-shards\": 2}");
  CHECK(from_json(c->redundancy())["k"] == "4");
  Block b = make_chb(random_bytes(4096, 9));
  store(*c, b);
  CHECK(c->fetch(b.address)->data == b.data);
}

int main(int argc, char** argv) {
  bool cpu_only = false;
  const char* filter = nullptr;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--cpu-only")) cpu_only = true;
    else filter = argv[i];
  }
  int run = 0, failed = 0;
  for (auto& t : tests()) {
    if (cpu_only && t.gpu) continue;
    if (filter && !std::strstr(t.name, filter)) continue;
    const int before = g_fail;
    std::printf("[ RUN  ] %s\n", t.name);
    std::fflush(stdout);
    try {
      t.fn();
    } catch (std::exception& e) {
      std::fprintf(stderr, "  uncaught: %s\n", e.what());
      ++g_fail;
    }
    ++run;
    const bool ok = g_fail == before;
    failed += !ok;
    std::printf("[ %s ] %s\n", ok ? " OK " : "FAIL", t.name);
  }
  std::printf("%d tests, %d failed\n", run, failed);
  return failed ? 1 : 0;
}
