// erasure_consensus.hh -- the "erasure" redundancy plugin over libmemo_ec.
//
// Drop-in for memo's immutable-block redundancy:
//   store  : replaces Paxos::_store -> Details::send_immutable_block
//            (src/memo/model/doughnut/consensus/Paxos.cc:1713-1732, 315-391):
//            the block is encoded (GPU, batched across concurrent stores) into
//            k data + m parity shards, shard i goes to owner i of
//            overlay.allocate(address, k+m);
//   fetch  : replaces Details::_fetch (Paxos.cc:486-519): any k valid shards;
//            the k data shards are concatenated as they are (systematic code),
//            otherwise the missing ones are rebuilt on the GPU; the CHB address
//            is re-checked on the reassembled block (CHB.cc:79-99).  The
//            multi-address fetch (Consensus::fetch(vector<AddressVersion>,
//            ReceiveBlock), Consensus.cc:101-124) decodes every block that
//            needs it in one GPU call per shard-size bucket;
//   repair : replaces _disappeared_evict / _rebalance (Paxos.cc:1012-1246):
//            every shard held by an evicted node is rebuilt in GPU-sized
//            batches and re-placed on a new owner.
// Mutable blocks stay on the backend (Paxos in memo, replication here).
#pragma once

#include <chrono>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <future>
#include <set>
#include <thread>
#include <unordered_set>

#include "../include/memo_ec.h"
#include "model.hh"

namespace memo_host {

// --------------------------------------------------------------- codec
// libmemo_ec contexts for host-memory calls.  A ctx serves one thread at a
// time (memo_ec.h); a small pool per GPU lets concurrent fetch threads
// decode.  With several GPUs a batch of n blocks is cut into contiguous
// block ranges, one per GPU, run by one host thread each:
// every GPU brings its own PCIe link and HBM.
class Codec {
 public:
  // device >= 0: that GPU; device < 0: every GPU memo_ec_device_count() sees.
  explicit Codec(int device = 0, int contexts = 4);
  // An explicit device list (a device may repeat: tests split over one GPU).
  Codec(const std::vector<int>& devices, int contexts_per_device);
  ~Codec();
  Codec(const Codec&) = delete;
  Codec& operator=(const Codec&) = delete;
  // pinned: both buffers come from memo_ec_host_alloc (MEMO_EC_HOST_PINNED:
  // the library DMAs straight from them, no bounce copies)
  void encode(int k, int m, size_t S, size_t n, const uint8_t* data, uint8_t* parity,
              bool pinned = false);
  void rebuild(int k, int m, size_t S, size_t n, const uint8_t* surv_idx, const uint8_t* surv,
               const uint8_t* lost_idx, int e, uint8_t* out, bool pinned = false);
  // One erasure pattern for all n blocks (memo_ec_rebuild_uniform):
  // surv_idx has k entries, lost_idx e.
  void rebuild_uniform(int k, int m, size_t S, size_t n, const uint8_t* surv_idx,
                       const uint8_t* surv, const uint8_t* lost_idx, int e, uint8_t* out,
                       bool pinned = false);
  // Groups with different shard sizes, erasure counts and per-block or
  // shared patterns in one library call per device
  // (memo_ec_rebuild_segments); every device takes its share of every group.
  void rebuild_segments(const std::vector<memo_ec_rebuild_segment>& segs, bool pinned = false);
  uint64_t encode_calls() const { return encode_calls_; }
  uint64_t rebuild_calls() const { return rebuild_calls_; }
  uint64_t uniform_calls() const { return uniform_calls_; }
  uint64_t segments_calls() const { return segments_calls_; }
  // segments with one shared erasure pattern passed to rebuild_segments
  uint64_t uniform_segments() const { return uniform_segments_; }
  size_t devices() const { return dev_.size(); }

 private:
  struct Dev {
    int id;
    std::vector<memo_ec_ctx*> free;
  };
  void init(const std::vector<int>& devices, int contexts);
  memo_ec_ctx* acquire(size_t d);
  void release(size_t d, memo_ec_ctx* c);
  // fn(device slot, first block, blocks) over the device partition of n
  void split(size_t n, const std::function<int(size_t, size_t, size_t)>& fn, const char* what);
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<memo_ec_ctx*> all_;
  std::vector<Dev> dev_;
  std::atomic<size_t> rr_{0};
  std::atomic<uint64_t> encode_calls_{0}, rebuild_calls_{0}, uniform_calls_{0}, segments_calls_{0},
      uniform_segments_{0};
};

// ------------------------------------------------------- pinned arena
// Reusable page-locked batch buffers (memo_ec_host_alloc).  The codec's
// host-memory calls then DMA straight from them (no staging copies in the
// library), and no batch pays for fresh pages or their release.  A buffer
// that cannot be pinned falls back to ordinary memory (pinned() false).
class PinnedArena {
 public:
  class Lease {
   public:
    Lease() = default;
    Lease(PinnedArena* a, uint8_t* p, size_t cap, bool pinned) : a_(a), p_(p), cap_(cap), pinned_(pinned) {}
    Lease(Lease&& o) noexcept { *this = std::move(o); }
    Lease& operator=(Lease&& o) noexcept;
    Lease(const Lease&) = delete;
    Lease& operator=(const Lease&) = delete;
    ~Lease();
    uint8_t* data() const { return p_; }
    bool pinned() const { return pinned_; }

   private:
    PinnedArena* a_ = nullptr;
    uint8_t* p_ = nullptr;
    size_t cap_ = 0;
    bool pinned_ = false;
  };
  // Buffers larger than this are released when their lease ends instead of
  // kept (the codec stages at most kStageBytes of survivors per call).
  static constexpr size_t kKeepMaxBytes = (size_t)1 << 30;
  explicit PinnedArena(size_t keep = 8) : keep_(keep) {}
  // free buffers kept and their bytes (tests)
  size_t kept_bytes() const;
  ~PinnedArena();
  PinnedArena(const PinnedArena&) = delete;
  PinnedArena& operator=(const PinnedArena&) = delete;
  Lease lease(size_t bytes);
  // leases handed out so far (tests: a multi-fetch or repair chunk takes
  // one survivor and one output lease, however many batches it has)
  uint64_t leases() const { return leases_.load(); }

 private:
  std::atomic<uint64_t> leases_{0};
  struct Buf {
    uint8_t* p;
    size_t cap;
    bool pinned;
  };
  void put(uint8_t* p, size_t cap, bool pinned);
  static void release(const Buf& b);
  mutable std::mutex mu_;
  std::vector<Buf> free_;
  size_t keep_;
};

// Shards of at most kFrameShardMax wire bytes are framed by the store in
// runs sharing one buffer of up to kFrameRunBytes (ErasureConsensus::place_batch).
constexpr size_t kFrameShardMax = (size_t)16 << 10;
constexpr size_t kFrameRunBytes = (size_t)256 << 10;

// Default shard bytes one store_many, fetch or repair chunk stages (pinned)
// and hands to one codec call at most (ErasureOptions::stage_bytes).
constexpr size_t kStageBytes = (size_t)512 << 20;

// ---------------------------------------------------------- shard format
// On-wire / on-silo shard: a 128-byte header + S payload bytes.  The header
// replaces the CHB re-hash of LocalPeer::store (Paxos.cc:1571-1575) as the
// per-shard validation (a shard is not a CHB), and carries what the block's
// own validation needs after reassembly (salt and owner, CHB.cc:264-289).
//   0 "MECS" | 4 version (2) | 5 k | 6 m | 7 index | 8 u64 B | 16 u64 S |
//   24 address[32] | 56 u32 salt_len | 60 salt[32] | 92 owner[32] |
//   124 u32 crc32c(bytes 0..123 || payload)
// The checksum covers the header too: a damaged size, salt or owner makes
// the shard an erasure, not a poisoned reassembly.
// A block reassembled from shards that each passed their CRC but together
// do not hash to the block's address (a holder served a well-framed shard
// with the wrong bytes).  Still a ValidationFailed to callers.
struct AddressMismatch : ValidationFailed {
  using ValidationFailed::ValidationFailed;
};

struct ShardHeader {
  static constexpr size_t kSize = 128;
  static constexpr uint8_t kVersion = 2;
  uint8_t version = kVersion;
  uint8_t k = 0, m = 0, index = 0;
  uint64_t block_size = 0, shard_size = 0;
  Address address;
  Buffer salt;
  Address owner;  // the CHB owner (null: none)
  uint32_t crc = 0;
  // Same block and code (every field but index and crc).
  bool same_block(const ShardHeader& o) const {
    return k == o.k && m == o.m && block_size == o.block_size && shard_size == o.shard_size &&
           address == o.address && salt == o.salt && owner == o.owner;
  }
};
Buffer encode_shard(const ShardHeader& h, const uint8_t* payload);
// encode_shard with `index` in place of h.index (one header per block shared
// by the threads framing its shards).
Buffer encode_shard(const ShardHeader& h, const uint8_t* payload, int index);
// encode_shard into kSize + h.shard_size bytes at w (a slot of a buffer that
// frames many shards).
void frame_shard(const ShardHeader& h, const uint8_t* payload, int index, uint8_t* w);
// Parses and validates (magic, version, geometry, S = memo_ec_shard_size(B,k),
// payload length, CRC32C over header and payload); throws ValidationFailed.
ShardHeader decode_shard(const Buffer& wire, const uint8_t** payload);
// decode_shard of the n bytes at w (a silo's view of a stored shard).
ShardHeader decode_shard_view(const uint8_t* w, size_t n, const uint8_t** payload);
// *payload would point into a temporary that dies with the call.
ShardHeader decode_shard(Buffer&& wire, const uint8_t** payload) = delete;
// The header alone (the first kSize bytes): magic, version and geometry are
// checked, the checksum cannot be (it covers the payload).  Index rescans
// use it; fetch and repair validate whole shards.
ShardHeader decode_shard_header(const uint8_t* wire, size_t n);
// Silo keys of the shards of block `address`: one SHA-256 of (address,
// tag) per block, shard i's key that hash with i folded into its first
// byte (keys of one block are distinct; the flag byte marks them immutable).
struct ShardKeys {
  std::array<uint8_t, 32> base;
  explicit ShardKeys(const Address& address);
  Key operator()(int index) const;
};
// Silo key of shard `index` of block `address` (ShardKeys(address)(index)).
Key shard_key(const Address& address, int index);
// The peer of a node in a network built before its consensus (tests,
// benches): a ShardLocal in front of make_replica_local(storage), what
// ErasureConsensus::make_local makes over a ReplicationConsensus backend.
std::unique_ptr<Local> make_shard_local(std::unique_ptr<Silo> storage);
uint32_t crc32c(const uint8_t* p, size_t n, uint32_t crc = 0);

// ------------------------------------------------------------ thread pool
// Parallel fan-out over peers (elle::reactor::for_each_parallel in memo).
class ThreadPool {
 public:
  explicit ThreadPool(int threads);
  ~ThreadPool();
  // Runs fn(0..n-1) on the pool and waits; rethrows the first exception.
  void parallel_for(size_t n, const std::function<void(size_t)>& fn);
  size_t size() const { return ts_.size(); }

 private:
  void worker();
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  std::vector<std::thread> ts_;
  bool stop_ = false;
};

// ------------------------------------------------------------ node index
// Node -> blocks it holds a shard of (Paxos::_node_blocks by_node,
// Paxos.hh:403-434), striped by node so that concurrent placements (the
// store pool) do not serialise on one lock.  Updated after the placement
// index: an eviction that races a placement may miss that block, which the
// full repair() scan still finds.
class NodeIndex {
 public:
  // old holders -> new holders of `block` (null addresses ignored)
  void update(const Address& block, const std::vector<Address>& old_h,
              const std::vector<Address>& new_h);
  struct Change {
    Address block;
    std::vector<Address> old_h, new_h;
  };
  // update() for many blocks, each stripe locked once; with a pool, the
  // stripes in parallel (a batch of 256 4 KiB blocks is ~3600 set inserts)
  void update_many(const std::vector<Change>& changes, ThreadPool* pool = nullptr);
  std::vector<Address> blocks(const Address& node) const;
  size_t count(const Address& node) const;

 private:
  static constexpr size_t kStripes = 32;
  struct alignas(64) Stripe {
    mutable std::mutex mu;
    std::unordered_map<Address, std::unordered_set<Address, AddressHash>, AddressHash> m;
  };
  Stripe& stripe(const Address& node) const;
  mutable std::array<Stripe, kStripes> st_;
};

// ---------------------------------------------------------------- options
struct ErasureOptions {
  int k = 10, m = 4;
  int device = -1;             // < 0: every GPU the library sees
  int batch_max = 256;         // blocks per batcher encode call / rebuild batch
  int batch_window_us = 200;   // how long the batcher waits for company
  int threads = 16;            // peer fan-out (memo's background pool is <= 16)
  // Blocks of one batch that share an erasure pattern (the repair of one
  // lost node) go to the uniform rebuild, at encode speed, once at least
  // uniform_min blocks and uniform_min_bytes of survivors share it (below
  // that a separate GPU call costs more than the per-block decode it saves);
  // the rest to the per-block rebuild.
  int uniform_min = 4;
  size_t uniform_min_bytes = 8u << 20;
  // Shard bytes a store_many (data + parity), fetch or repair (survivors)
  // stages (pinned) per chunk at most; larger requests run as several chunks.
  size_t stage_bytes = kStageBytes;
  // A node that disappears is evicted -- its shards rebuilt elsewhere --
  // after this long unless it comes back ("eviction-delay", Paxos.cc:985-1009,
  // default 10 min, Paxos.hxx:35).  < 0: never automatically.
  int64_t eviction_delay_ms = 10 * 60 * 1000;
  // Rebuild the placement index from the shard headers in the silos at
  // start (LocalPeer::initialize's rebalancing inspector, Paxos.cc:747-784).
  bool rescan = true;
  // Rebuild under-placed blocks' missing shards onto newly discovered nodes
  // (rebalance_auto_expand, Paxos.cc:1149-1244).
  bool auto_expand = true;
  // A degraded fetch asks for as many parity shards as the decode needs,
  // plus this many more on its first round ("fetch-hedge": a slow or
  // failing holder then costs no second round trip).
  int fetch_hedge = 0;
  // Parity holders are asked in order of in-flight transfers from this
  // client, shuffled first (Paxos.cc:488-500); false when the environment
  // sets INFINIT_DISABLE_BALANCED_TRANSFERS, as the reference reads it.
  bool balanced_transfers = true;
  // A reassembled block that fails its CHB address (a shard with a valid
  // CRC but wrong bytes) is retried from other k-subsets of every reachable
  // shard, at most this many ("verify-subsets"); the shards that disagree
  // with the verified block are rewritten.  0: fail at once.
  int verify_subsets = 64;
};

// The peer ErasureConsensus::make_local makes, in front of its backend's
// peer: a shard (the "MECS" framing) must pass its header checks and
// CRC32C and sit under its own key (shard_key(address, index)) -- the shard
// validation that replaces LocalPeer::store's CHB re-hash (Paxos.cc:1571-
// 1575) -- and may only replace a shard; any other value is the backend
// peer's to validate (the mutable blocks' replicas).
class ShardLocal : public Local {
 public:
  explicit ShardLocal(std::unique_ptr<Local> backend);
  void validate(const Key& k, const uint8_t* v, size_t n) const override;

 private:
  std::unique_ptr<Local> backend_;
};

class ErasureConsensus : public StackedConsensus {
 public:
  ErasureConsensus(std::unique_ptr<Consensus> backend, Overlay& overlay, ErasureOptions o);
  ~ErasureConsensus() override;

  // {"type":"erasure","k","m","desired_factor"}
  std::string redundancy() override;
  std::string stats() override;
  std::string stats_text() const;  // stats() for const callers
  // Where a block's shards are, as this client's placement index records
  // them (Consensus::stat, Consensus.hh:85-95; Paxos's PaxosStat lists the
  // quorum): {"placed", "k", "m", "block_size", "holders" (hex, "" for an
  // unplaced shard), "reachable"}.
  std::unique_ptr<Stat> stat(const Address& address) override;
  // A ShardLocal in front of the backend's peer (Consensus.hh:100-105).
  std::unique_ptr<Local> make_local(std::optional<int> port, std::optional<IpAddress> listen_address,
                                    std::unique_ptr<Silo> storage) override;

  struct RepairReport {
    size_t blocks_checked = 0, blocks_repaired = 0, shards_rebuilt = 0;
    size_t unrecoverable = 0, codec_calls = 0, shards_unplaced = 0;
  };
  // Rebuild every shard whose holder is evicted, lacks it or holds an
  // invalid copy, in batches of batch_max blocks per GPU call, and place it
  // on a new owner.  With include_down, shards on nodes that are merely
  // unreachable count as lost too.  A full scan of the index.
  RepairReport repair(bool include_down = false);
  // Evict a node now (Paxos::LocalPeer::_disappeared_evict, Paxos.cc:1012-
  // 1087): only the blocks the per-node index lists for it are repaired.
  RepairReport evict(const Address& node);
  // Place the missing shards of under-placed blocks (stored while fewer than
  // k+m owners were reachable) on reachable nodes that hold none of the
  // block's shards (the newcomer rebalancing of Paxos.cc:1149-1244).
  RepairReport expand();
  // Rebuild the placement and per-node indices from every reachable node's
  // silo (shard headers); returns the number of blocks found.
  size_t rescan();
  // Called after a block's shards were rebuilt or re-placed (the reference's
  // rebalanced() signal); runs on the repairing thread.
  void on_rebalanced(std::function<void(const Address&)> f);
  // Called with (block, holders) when a block is left on fewer than k+m
  // owners because no reachable node can take its missing shards (after a
  // repair, or when a background retry finds no free node): the reference's
  // under_replicated(address, quorum size) signal (Paxos.hh:366-370, fired
  // at Paxos.cc:1126).  Runs on the repairing / membership thread.
  void on_under_placed(std::function<void(const Address&, int)> f);
  // Blocks currently on fewer than k+m owners (the
  // underreplicated_immutable_blocks gauge, src/memo/overlay/Overlay.cc:35-40);
  // stats() reports it with a sample of up to 10 addresses.
  size_t under_placed() const;
  // Blocks the per-node index lists for `node` (Paxos.hh:403-434 by_node).
  size_t node_blocks(const Address& node) const;
  // Evictions scheduled and not yet run.
  size_t pending_evictions() const;
  // Store many immutable blocks with one encode call per batch (mutable ones
  // go to the backend one by one).
  void store_many(const std::vector<Block>& blocks);
  const Codec& codec() const { return codec_; }
  uint64_t arena_leases() const { return arena_.leases(); }
  size_t arena_kept_bytes() const { return arena_.kept_bytes(); }
  const ErasureOptions& options() const { return o_; }
  // The owner blocks removals of owned CHBs are checked against (the
  // model's fetch(owner) of CHB::_validate_remove); null: none known, so an
  // owned CHB's removal needs a valid signature by any key.
  void set_owner_directory(const OwnerDirectory* d) { owners_ = d; }
  // Shard removals owed to holders that were down at the removal.
  size_t pending_removes() const;

 protected:
  // Immutable blocks: encoded and placed (the resolver has nothing to
  // resolve: a CHB store never conflicts); mutable: the backend, resolver
  // and all.
  void _store(std::unique_ptr<Block> block, StoreMode mode,
              std::unique_ptr<ConflictResolver> resolver) override;
  // local_version: a mutable block's, passed to the backend (a CHB has no
  // version).
  std::unique_ptr<Block> _fetch(Address address, std::optional<int> local_version) override;
  void _fetch(const std::vector<AddressVersion>& addresses, ReceiveBlock res) override;
  // Consensus::remove (Consensus.cc:135-240) with CHB removal semantics
  // (CHB::_validate_remove, CHB.cc:203-259): see erasure_consensus.cc.
  void _remove(Address address, RemoveSignature rs) override;
  // Leaving the network: the mutable blocks' backend hands its blocks off
  // (Paxos::_resign, Paxos.cc:2091-2131, which rebalances mutable blocks
  // only); shards stay where they are, and the remaining nodes' eviction
  // timers repair them once this node is gone, as for Paxos's immutable
  // replicas.
  void _resign() override;

 private:
  struct Placement {
    uint64_t B = 0;
    Buffer salt;
    Address owner;                // CHB owner
    std::vector<Address> holder;  // node holding shard i (null: unplaced)
  };
  struct Placed {
    Address a;
    Placement pl;
    bool set = false;
  };
  void store_one(const Block& b);
  struct EncodeJob {
    const Block* block;
    std::promise<Buffer> parity;  // m x S
  };
  // A block's shards in hand for a fetch, and its missing data shards.
  struct Gathered {
    ShardHeader h;
    // the k used, sorted by index: data shards' payloads in `block`, parity
    // shards' wire bytes in the entry
    std::vector<std::pair<int, Buffer>> shards;
    Buffer block;               // k x S: the data shards in hand in their slots
    std::vector<uint8_t> lost;  // data-shard indices to rebuild
    std::exception_ptr err;
    const uint8_t* payload(size_t s) const;  // shards[s]'s S payload bytes
  };
  // index_locked: the caller holds a reader lock on index_mu_
  Gathered collect(const Address& a, bool parallel, bool index_locked = false);
  // The block from g's data shards and, for g.lost[r], the S bytes at
  // rebuilt + r * stride; checks the CHB address.
  std::unique_ptr<Block> assemble(const Address& a, Gathered& g, const uint8_t* rebuilt,
                                  size_t stride);
  Buffer padded(const Block& b, size_t S) const;
  ShardHeader header_of(const Address& a, const Placement& pl, int index) const;
  // The shards of b (its own payload, zero-padded, and m x S parity) to its
  // k + m owners, the placement recorded; TooFewPeers below k.
  struct Placed;
  void place(const Block& b, const uint8_t* parity);
  void commit_placements(std::vector<Placed>& placed);
  // place(..., defer) for a batch of blocks with their shards in S-byte
  // slots (block i's data shard j at data + (i*k + j)*S, parity shard r at
  // parity + (i*m + r)*S), the shards grouped by owner so that one pool task
  // stores an owner's run of shards.  Every block is tried; returns the
  // first failure (TooFewPeers) or null.
  std::exception_ptr place_batch(const std::vector<const Block*>& bs, const uint8_t* data,
                                 const uint8_t* parity, size_t S, std::vector<Placed>& placed);
  void batcher_loop();
  // from (k + m entries): the node each gathered shard came from
  // block: data shards' payloads straight into it (see the definition)
  std::vector<std::pair<int, Buffer>> gather_shards(const Address& a, int want, bool& any_down,
                                                    ShardHeader* hdr, bool parallel = true,
                                                    std::vector<Node*>* from = nullptr,
                                                    Buffer* block = nullptr, bool index_locked = false);
  // A block whose reassembly failed its address, from another k-subset of
  // its reachable shards; the disagreeing shards rewritten (AddressMismatch
  // when no subset within verify_subsets matches).
  std::unique_ptr<Block> recover(const Address& a, bool parallel);
  // recover() from the first `want` shards gathered: null when none of its
  // subsets matches and a wider gather is left to try
  std::unique_ptr<Block> recover_from(const Address& a, int want, bool parallel);
  // index_ updates under index_mu_ (held exclusively by the caller); they
  // return the block's previous holders for the node index, which the
  // caller updates after releasing the lock
  std::vector<Address> swap_placement_locked(const Address& a, Placement pl);
  std::vector<Address> erase_placement_locked(const Address& a);
  // The repair engine: rebuild and re-place the lost shards of `blocks`.
  RepairReport repair_blocks(const std::vector<Address>& blocks, bool include_down);
  void settle_removes(const Address& node, bool evicted);
  // membership: overlay events -> the membership thread
  void membership_loop();
  void post(int kind, const Address& id);

  Overlay& overlay_;
  ErasureOptions o_;
  Codec codec_;
  PinnedArena arena_;  // batch buffers of the codec calls
  ThreadPool pool_;
  mutable std::shared_mutex index_mu_;  // readers: fetch paths; writers: place, repair, remove
  std::unordered_map<Address, Placement, AddressHash> index_;  // Paxos::_quorums analogue
  NodeIndex nodes_;  // node -> blocks it holds a shard of
  std::mutex repair_mu_;  // one repair engine run at a time
  std::function<void(const Address&)> rebalanced_;
  std::function<void(const Address&, int)> under_placed_;  // guarded by repair_mu_
  void notify_under_placed(const std::vector<std::pair<Address, int>>& v);
  // batcher (host C++ batching of concurrent stores into one GPU call)
  std::mutex bmu_;
  std::condition_variable bcv_;
  std::deque<EncodeJob*> bq_;
  bool bstop_ = false;
  std::thread bthread_;
  // membership thread: discoveries, disappearances (eviction timers), returns
  mutable std::mutex mmu_;
  std::condition_variable mcv_;
  std::deque<std::pair<int, Address>> mq_;
  std::map<Address, std::chrono::steady_clock::time_point> evict_at_;
  // blocks stored on fewer than k+m owners, retried with backoff while a
  // reachable node holds none of their shards (Paxos's _rebalancable queue
  // after an under-replicated insert, Paxos.cc:1428-1438, 1089-1127)
  std::set<Address> under_;
  std::chrono::steady_clock::time_point under_at_{};
  std::chrono::milliseconds under_backoff_{10};
  bool mstop_ = false;
  int sub_token_ = -1;
  std::thread mthread_;
  // fetched_ and decoded_ are added to per block by every pool thread
  Counter stored_, fetched_, decoded_;
  std::atomic<uint64_t> repaired_{0}, evictions_{0};
  // reassemblies that failed their address and were recovered from another
  // k-subset; shards found wrong that way and rewritten
  std::atomic<uint64_t> subset_recoveries_{0}, corrupt_rewritten_{0};
  const OwnerDirectory* owners_ = nullptr;
  mutable std::mutex rm_mu_;
  // Shard removals owed to a node that was down: the block, the shard index
  // (-1: every index, for a block of unknown placement -- one record per
  // (node, block)) and the removal's signature, validated again against the
  // shard's header when the node returns
  struct OwedRemove {
    Address block;
    int index;
    RemoveSignature rs;
  };
  // Whether some node other than `except` holds a shard of `a` (a block
  // stored again after its removal).
  bool held_elsewhere(const Address& a, const Address& except) const;
  std::map<Address, std::vector<OwedRemove>> pending_rm_;  // node -> removals still owed
  // in-flight fetches from this client per node (the reference's
  // Paxos::_transfers), hashed into per-thread-slot counters: every shard
  // fetch adds and subtracts, only a degraded fetch's ordering reads them
  mutable std::array<Counter, 64> transfers_;
  Counter& transfers(const Node* nd) const {
    return transfers_[(reinterpret_cast<uintptr_t>(nd) >> 6) % transfers_.size()];
  }
};

}  // namespace memo_host
