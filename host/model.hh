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

// --------------------------------------------------------------- counters
// A counter that many threads add to: per-thread-slot atomics on lines of
// their own, summed by load().  One shared atomic line that every store or
// fetch thread writes moves between cores on each add, which on a many-core
// host costs more than the silo operation it counts.
class Counter {
 public:
  void add(int64_t d) { s_[slot()].v.fetch_add(d, std::memory_order_relaxed); }
  void operator++() { add(1); }
  void operator++(int) { add(1); }
  void operator+=(int64_t d) { add(d); }
  int64_t load() const {
    int64_t t = 0;
    for (auto& x : s_) t += x.v.load(std::memory_order_relaxed);
    return t;
  }
  operator int64_t() const { return load(); }

 private:
  static constexpr size_t kSlots = 16;
  static size_t slot();  // the calling thread's slot (assigned round robin)
  struct alignas(64) Slot {
    std::atomic<int64_t> v{0};
  };
  std::array<Slot, kSlots> s_;
};

// ------------------------------------------------------------------- silo
// silo::Silo (src/memo/silo/Silo.hh:33-129): get/set/erase/list with the
// MissingKey / Collision contract; subclasses implement _get/_set/_erase/_list.
using Key = Address;

// A non-owning callable (bytes, size) for Silo::read: no allocation per call.
class ReadSink {
 public:
  template <class F>
  ReadSink(F& f)  // NOLINT: implicit from any callable lvalue
      : obj_(&f), call_([](void* o, const uint8_t* p, size_t n) { (*static_cast<F*>(o))(p, n); }) {}
  void operator()(const uint8_t* p, size_t n) const { call_(obj_, p, n); }

 private:
  void* obj_;
  void (*call_)(void*, const uint8_t*, size_t);
};

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
  // The value handed to sink(bytes, size) -- a view valid during the call --
  // instead of copied out; false when absent.  The fetch paths validate a
  // shard and copy its payload into place in one pass.  The sink must not
  // call back into this silo (the memory silo runs it under a lock).
  bool read(const Key& k, const ReadSink& sink) const { return _read(k, sink); }
  // read() of the value's first n bytes (all of it if shorter): a peer's
  // check of the value a store replaces reads no more than it looks at.
  bool read_prefix(const Key& k, size_t n, const ReadSink& sink) const { return _read_prefix(k, n, sink); }
  // insert: accept a new key; update: accept an existing key.
  int set(const Key& k, const Buffer& v, bool insert = true, bool update = false);
  // set() of a value the caller gives up (a silo may keep it without a copy)
  int set(const Key& k, Buffer&& v, bool insert = true, bool update = false);
  // set() of the n bytes at `bytes`, which may share their allocation with
  // other keys' values (a batch of shards framed into one buffer); a silo
  // may keep the reference instead of a copy
  int set_shared(const Key& k, std::shared_ptr<const uint8_t> bytes, size_t n, bool insert = true,
                 bool update = false);
  int erase(const Key& k);
  std::vector<Key> list() { return _list(); }
  virtual std::string type() const = 0;
  int64_t usage() const { return usage_.load(); }
  int64_t capacity() const { return capacity_; }

 protected:
  virtual Buffer _get(const Key& k) const = 0;
  virtual bool _try_get(const Key& k, Buffer& out) const;  // default: _get + catch
  virtual bool _contains(const Key& k) const;                // default: _try_get
  virtual bool _try_get_prefix(const Key& k, size_t n, Buffer& out) const;  // default: _try_get
  virtual bool _read(const Key& k, const ReadSink& sink) const;              // default: _try_get
  virtual bool _read_prefix(const Key& k, size_t n, const ReadSink& sink) const;  // default: _try_get_prefix
  virtual int _set(const Key& k, const Buffer& v, bool insert, bool update) = 0;
  virtual int _set_moved(const Key& k, Buffer&& v, bool insert, bool update) { return _set(k, v, insert, update); }
  // default: a copy through _set_moved
  virtual int _set_shared(const Key& k, std::shared_ptr<const uint8_t> bytes, size_t n, bool insert,
                          bool update);
  virtual int _erase(const Key& k) = 0;
  virtual std::vector<Key> _list() = 0;
  void check_space(size_t n) const;
  int64_t capacity_;
  Counter usage_;  // written by every store thread
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
  bool _try_get_prefix(const Key& k, size_t n, Buffer& out) const override;
  bool _read(const Key& k, const ReadSink& sink) const override;
  bool _read_prefix(const Key& k, size_t n, const ReadSink& sink) const override;
  int _set(const Key& k, const Buffer& v, bool insert, bool update) override;
  int _set_moved(const Key& k, Buffer&& v, bool insert, bool update) override;
  int _set_shared(const Key& k, std::shared_ptr<const uint8_t> bytes, size_t n, bool insert,
                  bool update) override;
  int _erase(const Key& k) override;
  std::vector<Key> _list() override;

 private:
  // A stored value: n bytes at p, which may share an allocation with other
  // keys' values (set_shared; the allocation lives while any of them does).
  struct Value {
    std::shared_ptr<const uint8_t> p;
    size_t n = 0;
  };
  Value find(const Key& k) const;  // p null when absent
  int put(const Key& k, Value nv, bool insert, bool update);
  // Values are immutable once stored: readers take a reference under the
  // lock and copy (or read) outside it, writers copy before taking it.
  // Hashed, as the reference's Memory silo (src/memo/silo/Memory.hh:15), in
  // stripes with a lock each (the reference's silo serves one reactor
  // thread; this one serves a pool).
  struct alignas(64) Stripe {
    mutable std::mutex mu;
    std::unordered_map<Key, Value, AddressHash> blocks;
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
// boost::asio::ip::address stand-in: the textual address a Local listens on.
struct IpAddress {
  std::string text;
};

// doughnut::Local (src/memo/model/doughnut/Local.hh:22-120): the peer that
// serves a node's silo to the network.  What arrives is validated before the
// silo keeps it (Local::store, Local.cc:180-215; Paxos::LocalPeer::store
// re-hashes a CHB, Paxos.cc:1568-1615): validate() is that check, per
// consensus (Consensus::make_local).  This in-process model opens no port.
class Local {
 public:
  explicit Local(std::unique_ptr<Silo> storage, std::optional<int> port = {},
                 std::optional<IpAddress> listen_address = {});
  virtual ~Local() = default;
  Silo& storage() const { return *storage_; }
  int port() const { return port_; }
  const std::optional<IpAddress>& listen_address() const { return listen_; }
  // The check a value passes before the silo keeps it under key k (the base
  // peer accepts anything); throws ValidationFailed (or Conflict).
  virtual void validate(const Key& k, const uint8_t* v, size_t n) const;

 protected:
  // A peer over another peer's silo (a stacked consensus's Local adds its
  // checks in front of its backend's: both see one storage).
  explicit Local(const Local& inner) : storage_(inner.storage_), port_(inner.port_), listen_(inner.listen_) {}

 private:
  std::shared_ptr<Silo> storage_;
  int port_;
  std::optional<IpAddress> listen_;
};

// Dock::Connection stand-in (src/memo/model/doughnut/Dock.hh): this node's
// link to another node.
struct DockConnection {
  Address peer;
};

// doughnut::Remote (src/memo/model/doughnut/Remote.hh): a client's handle on
// another node over a connection (Consensus::make_remote).
class Remote {
 public:
  explicit Remote(std::shared_ptr<DockConnection> connection) : c_(std::move(connection)) {}
  virtual ~Remote() = default;
  const Address& id() const { return c_->peer; }
  const std::shared_ptr<DockConnection>& connection() const { return c_; }

 private:
  std::shared_ptr<DockConnection> c_;
};

// A storage node: doughnut::Local with its silo (Local.cc:180-257) as seen
// through Peer::store/fetch/remove (doughnut/Peer.hh:19-89).  `up` models
// reachability: a down node raises Unavailable like a failed RPC.  Stores
// go through the node's Local: validated, then kept.
struct Node {
  Address id;
  std::unique_ptr<Local> local;
  Silo* silo = nullptr;  // local->storage()
  std::atomic<bool> up{true};
  std::atomic<bool> evicted{false};
  // store barrier (tests/doughnut.cc:1048-1163 instrumented Local)
  std::atomic<bool> fail_stores{false};
  // counters written by every store / fetch thread (per-thread slots, off
  // the flags above that every operation reads)
  Counter stores;
  mutable Counter fetches;

  void store(const Key& k, const Buffer& v);
  void store(const Key& k, Buffer&& v);
  // store() of n bytes that share an allocation with other values
  // (Silo::set_shared)
  void store_shared(const Key& k, std::shared_ptr<const uint8_t> bytes, size_t n);
  Buffer fetch(const Key& k) const;
  // fetch() that reports a missing key by returning false (no exception);
  // throws Unavailable when the node is down.
  bool try_fetch(const Key& k, Buffer& out) const;
  // try_fetch() that hands the value to sink instead of copying it out
  // (Silo::read)
  bool try_read(const Key& k, const ReadSink& sink) const;
  // try_fetch() of the value's first n bytes (a shard header).
  bool try_fetch_prefix(const Key& k, size_t n, Buffer& out) const;
  void remove(const Key& k);
  bool has(const Key& k) const;
  // One removal request naming several keys (Peer::remove(address, rs),
  // doughnut/Peer.hh, answered by Local::remove, Local.cc:260-278, which
  // checks the signature against what it stores): on the node, each key
  // present has its first `prefix` bytes handed to `check`, and is erased
  // when check returns "" (otherwise the refusal is kept).  Returns the
  // number erased; throws Unavailable, once, when the node is down.
  using RemoveCheck = std::function<std::string(const Key& k, const Buffer& head)>;
  int remove_values(const std::vector<Key>& keys, size_t prefix, const RemoveCheck& check,
                    std::string* refused = nullptr);
  Counter remove_requests;  // remove() and remove_values() requests served
  // One request: does the node hold any of these keys?  Throws Unavailable
  // when the node is down.
  bool holds_any(const std::vector<Key>& keys) const;
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

  // Adds the node and signals its discovery: its peer made by a consensus
  // (Consensus::make_local), or a plain Local over `silo` (no validation).
  std::shared_ptr<Node> add_node(const Address& id, std::unique_ptr<Local> local);
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
// consensus::Consensus (src/memo/model/doughnut/Consensus.hh:24-127): the
// redundancy plugin base.  The public calls dispatch to the protected
// virtuals; the signatures are the reference's with std::optional for
// boost::optional, IpAddress / DockConnection for the asio and dock types,
// and JSON text for elle::json::Json.
enum StoreMode { STORE_INSERT, STORE_UPDATE };

// Model::ReceiveBlock (src/memo/model/Model.hh:199): called once per
// requested address with the block, or with null and the exception.
using ReceiveBlock =
    std::function<void(const Address&, std::unique_ptr<Block>, std::exception_ptr)>;

// model::ConflictResolver (src/memo/model/Model.hh:63-87): called when a
// mutable block's store conflicts with a newer stored version; returns the
// block to retry with, or null to give up.
class ConflictResolver {
 public:
  virtual ~ConflictResolver() = default;
  virtual std::unique_ptr<Block> operator()(Block& failed, Block& current) = 0;
  virtual std::string description() const = 0;
};

// doughnut::Conflict (src/memo/model/doughnut/Conflict.hh): a store refused
// because the stored version is as new or newer; carries that version.
struct Conflict : Error {
  Conflict(const std::string& what, std::unique_ptr<Block> current)
      : Error(what), current(std::move(current)) {}
  std::shared_ptr<Block> current;
};

class Consensus {
 public:
  using AddressVersion = std::pair<Address, std::optional<int>>;
  virtual ~Consensus() = default;

  // Blocks (Consensus.hh:38-61, Consensus.cc:34-141)
  void store(std::unique_ptr<Block> block, StoreMode mode, std::unique_ptr<ConflictResolver> resolver) {
    _store(std::move(block), mode, std::move(resolver));
  }
  void fetch(const std::vector<AddressVersion>& addresses, ReceiveBlock res) {
    _fetch(addresses, std::move(res));
  }
  std::unique_ptr<Block> fetch(Address address, std::optional<int> local_version = {}) {
    return _fetch(address, local_version);
  }
  void remove(Address address, RemoveSignature rs) { _remove(address, std::move(rs)); }
  void resign() { _resign(); }

  // Stat (Consensus.hh:85-95): what the consensus knows of one block;
  // Stat::serialize restated as JSON text.
  class Stat {
   public:
    virtual ~Stat() = default;
    virtual std::string json() const { return "{}"; }
  };
  virtual std::unique_ptr<Stat> stat(const Address& address);

  // Factory (Consensus.hh:100-108, Consensus.cc:330-353): the peer serving a
  // node's silo, and a client's handle on another node.
  virtual std::unique_ptr<Local> make_local(std::optional<int> port, std::optional<IpAddress> listen_address,
                                            std::unique_ptr<Silo> storage);
  virtual std::shared_ptr<Remote> make_remote(std::shared_ptr<DockConnection> connection);

  // Monitoring (Consensus.hh:113-119, Consensus.cc:359-378): JSON text.
  virtual std::string redundancy();
  virtual std::string stats();

 protected:
  virtual void _store(std::unique_ptr<Block> block, StoreMode mode,
                      std::unique_ptr<ConflictResolver> resolver) = 0;
  virtual std::unique_ptr<Block> _fetch(Address address, std::optional<int> local_version) = 0;
  // Default: one fetch per address, errors passed to `res`
  // (Consensus::_fetch, Consensus.cc:101-124).
  virtual void _fetch(const std::vector<AddressVersion>& addresses, ReceiveBlock res);
  virtual void _remove(Address address, RemoveSignature rs) = 0;
  virtual void _resign() {}  // Consensus::_resign: nothing by default
};

// consensus::StackedConsensus (Consensus.hh:129-142, Consensus.hxx,
// Consensus.cc:392-401): a consensus over a backend consensus.
class StackedConsensus : public Consensus {
 public:
  explicit StackedConsensus(std::unique_ptr<Consensus> backend) : backend_(std::move(backend)) {}
  std::shared_ptr<Remote> make_remote(std::shared_ptr<DockConnection> connection) override {
    return backend_->make_remote(std::move(connection));
  }
  // The first consensus of type C down the stack from `top` (itself
  // included), null if none.
  template <typename C>
  static C* find(Consensus* top) {
    if (auto res = dynamic_cast<C*>(top)) return res;
    if (auto res = dynamic_cast<StackedConsensus*>(top)) return find<C>(res->backend().get());
    return nullptr;
  }
  const std::unique_ptr<Consensus>& backend() const { return backend_; }

 protected:
  std::unique_ptr<Consensus> backend_;
};

// The replication path memo uses for every block today (Paxos with
// replication-factor N, immutable branch Paxos.cc:315-391 / 486-519),
// restated without the Paxos protocol: the full block on `factor` owners,
// read from the first replica that answers.  Its peers validate what they
// store as Paxos::LocalPeer::store does (Paxos.cc:1568-1615): a CHB replica
// is re-hashed against its address, and a value already stored under the
// key is read and checked first (an immutable block over a mutable one is
// refused; a mutable block's version must grow, else Conflict).  The
// erasure plugin keeps it for mutable (metadata) blocks.
class ReplicationConsensus : public Consensus {
 public:
  ReplicationConsensus(Overlay& overlay, int factor) : overlay_(overlay), factor_(factor) {}
  std::string redundancy() override;
  std::string stats() override;
  std::unique_ptr<Local> make_local(std::optional<int> port, std::optional<IpAddress> listen_address,
                                    std::unique_ptr<Silo> storage) override;
  int factor() const { return factor_; }

 protected:
  // Consensus::_store's loop (Consensus.cc:40-94): a Conflict goes to the
  // resolver, whose block is stored instead, until it gives up.
  void _store(std::unique_ptr<Block> block, StoreMode mode,
              std::unique_ptr<ConflictResolver> resolver) override;
  using Consensus::_fetch;
  // local_version: a mutable block no newer than it is not returned (null),
  // as Paxos::_fetch with a local version does.
  std::unique_ptr<Block> _fetch(Address address, std::optional<int> local_version) override;
  // Consensus::remove_many (Consensus.cc:178-240) over the `factor` replicas:
  // unreachable replicas are skipped, MissingBlock when none removed it.
  // (Mutable blocks' own remove validation is outside this path.)
  void _remove(Address address, RemoveSignature rs) override;

 private:
  Overlay& overlay_;
  int factor_;
};
// The peer ReplicationConsensus::make_local makes, over `storage` (for a
// network built before its consensus, as tests and benches do).
std::unique_ptr<Local> make_replica_local(std::unique_ptr<Silo> storage);
// The replica validation of ReplicationConsensus's peers (LocalPeer::store's
// block->validate, Paxos.cc:1571-1575): a replica value of key k must decode,
// and an immutable one must hash to k.  Throws ValidationFailed.
void validate_replica(const Key& k, const uint8_t* v, size_t n);

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
