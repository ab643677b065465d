// model.hh -- minimal, faithful restatement of the memo interfaces the
// erasure plugin sits behind (the reference needs boost/elle/drake and is not
// buildable here).  Each type cites the reference declaration
// whose contract it keeps; only what the redundancy path touches is kept.
#pragma once

#include <array>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <exception>
#include <functional>
#include <map>
#include <memory>
#include <optional>
#include <shared_mutex>
#include <unordered_map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace memo_host {

using Buffer = std::vector<uint8_t>;  // elle::Buffer (elle/src/elle/Buffer.hh:34)

// ---------------------------------------------------------------- errors
// elle::Error, model::MissingBlock (src/memo/model/MissingBlock.hh),
// athena::paxos::TooFewPeers / Unavailable (Paxos.cc:65-83),
// ValidationFailed (Paxos.cc:1572-1597), silo::MissingKey / Collision.
struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct MissingBlock : Error {
  using Error::Error;
};
struct TooFewPeers : Error {
  using Error::Error;
};
struct Unavailable : Error {
  using Error::Error;
};
struct ValidationFailed : Error {
  using Error::Error;
};
namespace silo {
struct MissingKey : Error {
  using Error::Error;
};
struct Collision : Error {
  using Error::Error;
};
struct InsufficientSpace : Error {
  using Error::Error;
};
}  // namespace silo

// --------------------------------------------------------------- address
// model::Address (src/memo/model/Address.hh:18-60): 32 bytes, the last byte
// carries the flags (0 mutable, 1 immutable) when `combine` is set.
namespace flags {
constexpr uint8_t mutable_block = 0;
constexpr uint8_t immutable_block = 1;
}  // namespace flags

struct Address {
  static constexpr int flag_byte = 31;
  std::array<uint8_t, 32> value{};
  Address() = default;
  Address(const uint8_t* v, uint8_t flags, bool combine) {
    std::memcpy(value.data(), v, 32);
    if (combine) value[flag_byte] = flags;
  }
  bool mutable_block() const { return value[flag_byte] == flags::mutable_block; }
  explicit operator bool() const {
    for (auto b : value)
      if (b) return true;
    return false;
  }
  bool operator==(const Address& o) const { return value == o.value; }
  bool operator!=(const Address& o) const { return value != o.value; }
  bool operator<(const Address& o) const { return value < o.value; }
  std::string hex() const;
  static Address random(uint8_t flags);
};

struct AddressHash {
  size_t operator()(const Address& a) const {
    size_t h;
    std::memcpy(&h, a.value.data(), sizeof h);
    return h;
  }
};

// SHA-256 (OpenSSL, as elle::cryptography::hash(..., Oneway::sha256)).
std::array<uint8_t, 32> sha256(const void* a, size_t na, const void* b = nullptr, size_t nb = 0);

// ----------------------------------------------------------------- blocks
// The model version a network runs (Doughnut::version(), elle::Version
// major.minor.patch).  CHB hashing depends on it (CHB.cc:270-289): the owner
// enters the hash from 0.4.0, the immutable flag is combined into the
// address from 0.5.0.
using Version = std::array<int, 3>;
constexpr Version kModelVersion{0, 9, 0};

// blocks::Block (src/memo/model/blocks/Block.hh:107-200): an address and the
// payload data() (Block.hh:142).  Immutable content-hash blocks are CHBs:
// address = SHA-256(salt || owner || data) (CHB::_hash_address,
// src/memo/model/doughnut/CHB.cc:264-289), the owner only when set and the
// version >= 0.4 (otherwise the block carries a null owner, CHB.cc:38-48).
struct Block {
  Address address;
  Buffer data;
  Buffer salt;
  Address owner;  // CHB owner (null: none); blocks::Block::owner()
  bool is_mutable = false;
  int version = 0;  // mutable blocks only
};

// CHB::_hash_address (CHB.cc:264-289).
Address chb_address(const Buffer& data, const Address& owner, const Buffer& salt,
                    const Version& version = kModelVersion);
Block make_chb(Buffer data, Buffer salt = {}, Address owner = {},
               const Version& version = kModelVersion);
Block make_mutable(Address address, Buffer data, int version = 1);
// CHB::_validate (CHB.cc:79-99): the address is the hash of the content,
// compared without the flag byte (equal_unflagged, Address.cc:135-141).
bool chb_valid(const Address& address, const Buffer& salt, const Address& owner,
               const Buffer& data, const Version& version = kModelVersion);

// ------------------------------------------------------------ remove keys
// The doughnut's signing keys (Doughnut::keys(), an elle::cryptography RSA
// pair in memo).  This restatement signs with Ed25519 (OpenSSL EVP): the
// same sign / verify contract over the same bytes, a smaller key.
struct KeyPair {
  Buffer public_key;   // 32 bytes, raw
  Buffer private_key;  // 32 bytes, raw
  static KeyPair generate();
  Buffer sign(const uint8_t* msg, size_t n) const;
};
bool verify_signature(const Buffer& public_key, const Buffer& signature, const uint8_t* msg,
                      size_t n);

// blocks::RemoveSignature (src/memo/model/blocks/Block.hh:21-35): the key
// that signed the removal and its signature of the block address; for a
// removal signed through a group, the group's key and the index of the
// group key version that signed (group_public_keys()[group_index] is
// signature_key, CHB.cc:243-258).
struct RemoveSignature {
  std::optional<Buffer> group_key;
  std::optional<int> group_index;
  std::optional<Buffer> signature_key;
  std::optional<Buffer> signature;
};

// What CHB::_validate_remove reads from a CHB's owner block, an ACB
// (CHB.cc:203-259): the owner key, the keys with write access (ACL
// entries), the group entries (acl_group_entries: a group key and whether
// the group may write) and the world-write permission.  model.fetch(owner)
// is restated as a directory the network's clients share.
struct GroupAclEntry {
  Buffer group_key;
  bool write = false;
};
struct OwnerAcl {
  Buffer owner_key;
  std::vector<Buffer> writers;
  bool world_write = false;
  std::vector<GroupAclEntry> groups;
};
// The directory also restates the group blocks a removal names
// (Group(dht, key).group_public_keys(), doughnut/Group.cc): per group key,
// the public key of every version, oldest first (version v at index v - 1).
class OwnerDirectory {
 public:
  void set(const Address& owner, OwnerAcl acl);
  std::optional<OwnerAcl> find(const Address& owner) const;
  void set_group(const Buffer& group_key, std::vector<Buffer> public_keys);
  std::optional<std::vector<Buffer>> group_public_keys(const Buffer& group_key) const;

 private:
  mutable std::mutex mu_;
  std::map<Address, OwnerAcl> acl_;
  std::map<Buffer, std::vector<Buffer>> groups_;
};

// CHB::sign_remove (CHB.cc:140-201): `keys` sign the block address.
RemoveSignature chb_sign_remove(const Address& chb, const KeyPair& keys);
// CHB::sign_remove's group branch (CHB.cc:170-186): the group's current
// key pair (version `version`, 1-based) signs, and the signature names the
// group and the key's index (version - 1).
RemoveSignature chb_sign_remove_group(const Address& chb, const Buffer& group_key,
                                      const KeyPair& current, int version);
// CHB::_validate_remove (CHB.cc:203-259) of a CHB at `chb` owned by `owner`:
// "" when the removal is allowed, else the failure reason.  No owner:
// allowed.  Owner set: the signature fields must be present ("Missing field
// in signature") and verify over the address ("Invalid signature"); an
// owner block the directory does not know is allowed (the reference warns
// and allows, CHB.cc:222-227); else the block is world-writable, or the key
// is the owner's, or -- without a group in the signature -- a writer's, or
// -- with one -- the group has a write entry and its key of index
// group_index is the signing key ("Key not found" otherwise; an unknown
// group or a missing / out-of-range index is refused).
std::string chb_validate_remove(const Address& chb, const Address& owner,
                                const RemoveSignature& rs, const OwnerDirectory* dir);

// ------------------------------------------------------------------- silo
// silo::Silo (src/memo/silo/Silo.hh:33-129): get/set/erase/list with the
// MissingKey / Collision contract; subclasses implement _get/_set/_erase/_list.
using Key = Address;

class Silo {
 public:
  explicit Silo(int64_t capacity = -1) : capacity_(capacity) {}
  virtual ~Silo() = default;
  Buffer get(const Key& k) const { return _get(k); }
  // get() without the MissingKey exception: false when absent.
  bool try_get(const Key& k, Buffer& out) const { return _try_get(k, out); }
  // The first n bytes of the value (all of it if shorter); false when
  // absent.  Index rescans read shard headers only.
  bool try_get_prefix(const Key& k, size_t n, Buffer& out) const { return _try_get_prefix(k, n, out); }
  bool contains(const Key& k) const { return _contains(k); }
  // insert: accept a new key; update: accept an existing key.
  int set(const Key& k, const Buffer& v, bool insert = true, bool update = false);
  // set() of a value the caller gives up (a silo may keep it without a copy)
  int set(const Key& k, Buffer&& v, bool insert = true, bool update = false);
  int erase(const Key& k);
  std::vector<Key> list() { return _list(); }
  virtual std::string type() const = 0;
  int64_t usage() const { return usage_; }
  int64_t capacity() const { return capacity_; }

 protected:
  virtual Buffer _get(const Key& k) const = 0;
  virtual bool _try_get(const Key& k, Buffer& out) const;  // default: _get + catch
  virtual bool _contains(const Key& k) const;                // default: _try_get
  virtual bool _try_get_prefix(const Key& k, size_t n, Buffer& out) const;  // default: _try_get
  virtual int _set(const Key& k, const Buffer& v, bool insert, bool update) = 0;
  virtual int _set_moved(const Key& k, Buffer&& v, bool insert, bool update) { return _set(k, v, insert, update); }
  virtual int _erase(const Key& k) = 0;
  virtual std::vector<Key> _list() = 0;
  int64_t capacity_;
  alignas(64) std::atomic<int64_t> usage_{0};  // written by every store thread
};

// silo::Memory (src/memo/silo/Memory.hh:10-61): the in-memory test silo.
class MemorySilo : public Silo {
 public:
  using Silo::Silo;
  std::string type() const override { return "memory"; }

 protected:
  Buffer _get(const Key& k) const override;
  bool _try_get(const Key& k, Buffer& out) const override;
  bool _contains(const Key& k) const override;
  int _set(const Key& k, const Buffer& v, bool insert, bool update) override;
  int _set_moved(const Key& k, Buffer&& v, bool insert, bool update) override;
  int _erase(const Key& k) override;
  std::vector<Key> _list() override;

 private:
  int put(const Key& k, std::shared_ptr<const Buffer> nv, bool insert, bool update);
  // Values are immutable once stored: readers take a reference under the
  // lock and copy outside it, writers copy before taking it.  Hashed, as
  // the reference's Memory silo (src/memo/silo/Memory.hh:15), in stripes
  // with a lock each (the reference's silo serves one reactor thread; this
  // one serves a pool).
  struct alignas(64) Stripe {
    mutable std::mutex mu;
    std::unordered_map<Key, std::shared_ptr<const Buffer>, AddressHash> blocks;
  };
  static constexpr size_t kStripes = 16;
  Stripe& stripe(const Key& k) const { return st_[(AddressHash()(k) >> 56) % kStripes]; }
  mutable std::array<Stripe, kStripes> st_;
};

// silo::Filesystem (src/memo/silo/Filesystem.cc:27-147): one file per key,
// named by the key's hex, in a subdirectory named by its first byte; usage
// recovered from the files present at construction.  Writes go to a temp
// file renamed into place, so a crash leaves the old value or the new one.
class FilesystemSilo : public Silo {
 public:
  explicit FilesystemSilo(std::string root, int64_t capacity = -1);
  std::string type() const override { return "filesystem"; }
  const std::string& root() const { return root_; }

 protected:
  Buffer _get(const Key& k) const override;
  bool _try_get(const Key& k, Buffer& out) const override;
  bool _contains(const Key& k) const override;
  bool _try_get_prefix(const Key& k, size_t n, Buffer& out) const override;
  int _set(const Key& k, const Buffer& v, bool insert, bool update) override;
  int _erase(const Key& k) override;
  std::vector<Key> _list() override;

 private:
  std::string path(const Key& k, bool make_dir) const;
  std::string root_;
  mutable std::mutex mu_;  // serialises writers of one key with its readers
};

// ------------------------------------------------------------ peers/overlay
// A storage node: doughnut::Local with its silo (Local.cc:180-257) as seen
// through Peer::store/fetch/remove (doughnut/Peer.hh:19-89).  `up` models
// reachability: a down node raises Unavailable like a failed RPC.
struct Node {
  Address id;
  std::unique_ptr<Silo> silo;
  std::atomic<bool> up{true};
  std::atomic<bool> evicted{false};
  // store barrier (tests/doughnut.cc:1048-1163 instrumented Local)
  std::atomic<bool> fail_stores{false};
  // counters written by every store / fetch thread: lines of their own, off
  // the flags above that every operation reads
  alignas(64) std::atomic<int64_t> stores{0};
  alignas(64) std::atomic<int64_t> fetches{0};

  void store(const Key& k, const Buffer& v);
  void store(const Key& k, Buffer&& v);
  Buffer fetch(const Key& k) const;
  // fetch() that reports a missing key by returning false (no exception);
  // throws Unavailable when the node is down.
  bool try_fetch(const Key& k, Buffer& out) const;
  // try_fetch() of the value's first n bytes (a shard header).
  bool try_fetch_prefix(const Key& k, size_t n, Buffer& out) const;
  void remove(const Key& k);
  bool has(const Key& k) const;
};

// overlay::Overlay (src/memo/overlay/Overlay.hh:34-188): allocate(address, n)
// chooses n owners for a new block, lookup(address, n) the nodes that may hold
// it.  This in-process overlay (like tests/DHT.hh's test overlay) ranks nodes
// by rendezvous hashing of (address, node id), so every client agrees.
class Overlay {
 public:
  // Membership signals (overlay::Overlay::on_discovery / on_disappearance,
  // src/memo/overlay/Overlay.hh:124-129; a node coming back is a discovery
  // there, `appeared` here).  Handlers run on the thread that changed the
  // membership and must not block.
  using NodeEvent = std::function<void(const Address& id)>;
  struct Handlers {
    NodeEvent discovered, disappeared, appeared;
  };
  int subscribe(Handlers h);
  void unsubscribe(int token);
  // Node::up with the signal (a test may still flip Node::up silently).
  void set_up(const Address& id, bool up);

  // Adds the node and signals its discovery.
  std::shared_ptr<Node> add_node(const Address& id, std::unique_ptr<Silo> silo);
  std::shared_ptr<Node> node(const Address& id) const;
  // Every node in rendezvous order for `address` (reachable or not).
  std::vector<std::shared_ptr<Node>> rank(const Address& address) const;
  // The first n reachable nodes for a new block (Overlay::allocate).
  std::vector<std::shared_ptr<Node>> allocate(const Address& address, int n) const;
  // The first n non-evicted nodes (Overlay::lookup); may include down nodes.
  std::vector<std::shared_ptr<Node>> lookup(const Address& address, int n) const;
  std::vector<std::shared_ptr<Node>> nodes() const;
  size_t size() const;

  Overlay();
  ~Overlay();
  Overlay(const Overlay&) = delete;
  Overlay& operator=(const Overlay&) = delete;

 private:
  // Nodes are only ever added (a node that leaves is marked down or
  // evicted), so the membership is an immutable snapshot replaced on each
  // add: lookups read it with one atomic load -- no lock, no shared
  // reference count touched by the many fetch/store threads -- and hand out
  // non-owning handles to nodes the overlay keeps alive for its lifetime.
  struct Snapshot {
    std::vector<Node*> nodes;
    std::unordered_map<Address, Node*, AddressHash> by_id;
  };
  const Snapshot* snap() const { return snap_.load(std::memory_order_acquire); }
  std::mutex mu_;                                  // writers (add_node)
  std::vector<std::shared_ptr<Node>> owned_;       // every node ever added
  std::vector<std::unique_ptr<Snapshot>> snaps_;   // every snapshot (kept: readers may hold one)
  std::atomic<const Snapshot*> snap_{nullptr};
  // Handlers run under hmu_: once unsubscribe() returns, none of that
  // subscriber's handlers is running or will run.
  std::mutex hmu_;
  std::map<int, Handlers> handlers_;
  int next_token_ = 0;
  template <class F>
  void notify(F pick, const Address& id) {
    std::lock_guard<std::mutex> g(hmu_);
    for (auto& kv : handlers_) {
      const NodeEvent& f = pick(kv.second);
      if (f) f(id);
    }
  }
};

// -------------------------------------------------------------- consensus
// consensus::Consensus (src/memo/model/doughnut/Consensus.hh:24-174): the
// redundancy plugin base.  store/fetch/remove dispatch to the virtuals.
enum StoreMode { STORE_INSERT, STORE_UPDATE };

// Model::ReceiveBlock (src/memo/model/Model.hh:199): called once per
// requested address with the block, or with null and the exception.
using ReceiveBlock =
    std::function<void(const Address&, std::unique_ptr<Block>, std::exception_ptr)>;

class Consensus {
 public:
  virtual ~Consensus() = default;
  void store(const Block& b, StoreMode mode = STORE_INSERT) { _store(b, mode); }
  std::unique_ptr<Block> fetch(const Address& a) { return _fetch(a); }
  // Consensus::fetch(vector<AddressVersion>, ReceiveBlock) (Consensus.cc:101-106).
  void fetch(const std::vector<Address>& addresses, const ReceiveBlock& res) {
    _fetch(addresses, res);
  }
  // Consensus::remove(Address, RemoveSignature) (Consensus.cc:135-164).
  void remove(const Address& a, const RemoveSignature& rs = {}) { _remove(a, rs); }
  // Consensus::resign (Consensus.cc:167-176): the local node is leaving.
  void resign() { _resign(); }
  // Consensus::redundancy / stats (Consensus.cc:350-357): JSON text.
  virtual std::string redundancy() const = 0;
  virtual std::string stats() const { return "{}"; }

 protected:
  virtual void _store(const Block& b, StoreMode mode) = 0;
  virtual std::unique_ptr<Block> _fetch(const Address& a) = 0;
  // Default: one fetch per address, errors passed to `res`
  // (Consensus::_fetch, Consensus.cc:108-124).
  virtual void _fetch(const std::vector<Address>& addresses, const ReceiveBlock& res);
  virtual void _remove(const Address& a, const RemoveSignature& rs) = 0;
  virtual void _resign() {}  // Consensus::_resign: nothing by default
};

// consensus::StackedConsensus (Consensus.hh:129-142).
class StackedConsensus : public Consensus {
 public:
  explicit StackedConsensus(std::unique_ptr<Consensus> backend) : backend_(std::move(backend)) {}
  Consensus& backend() { return *backend_; }

 protected:
  std::unique_ptr<Consensus> backend_;
};

// The replication path memo uses for every block today (Paxos with
// replication-factor N, immutable branch Paxos.cc:315-391 / 486-519),
// restated without the Paxos protocol: the full block on `factor` owners,
// read from the first replica that answers.  The erasure plugin keeps it for
// mutable (metadata) blocks.
class ReplicationConsensus : public Consensus {
 public:
  ReplicationConsensus(Overlay& overlay, int factor) : overlay_(overlay), factor_(factor) {}
  std::string redundancy() const override;

 protected:
  void _store(const Block& b, StoreMode mode) override;
  using Consensus::_fetch;
  std::unique_ptr<Block> _fetch(const Address& a) override;
  // Consensus::remove_many (Consensus.cc:178-240) over the `factor` replicas:
  // unreachable replicas are skipped, MissingBlock when none removed it.
  // (Mutable blocks' own remove validation is outside this path.)
  void _remove(const Address& a, const RemoveSignature& rs) override;

 private:
  Overlay& overlay_;
  int factor_;
};

// ----------------------------------------------------------- configuration
// consensus::Configuration (Consensus.hh:148-174): polymorphic, serialized
// with a "type" key; factories registered by name like
// Hierarchy<Configuration>::Register<Paxos::Configuration>("paxos")
// (Paxos.cc:2285-2286).  Flat JSON objects with kebab-case keys.
using ConfigMap = std::map<std::string, std::string>;
std::string to_json(const ConfigMap& m);
ConfigMap from_json(const std::string& text);

using ConsensusFactory = std::function<std::unique_ptr<Consensus>(Overlay&, const ConfigMap&)>;
void register_consensus(const std::string& type, ConsensusFactory f);
std::unique_ptr<Consensus> make_consensus(Overlay& overlay, const std::string& json_config);

}  // namespace memo_host
