// surface_check.cc -- compile-time check that ErasureConsensus overrides the
// restated consensus::Consensus surface signature for signature
// (src/memo/model/doughnut/Consensus.hh:24-142).  Built with -fsyntax-only
// by tests/test_host_plugin.py; nothing here runs.
//
// Taking &Probe::f of a member that ErasureConsensus declares gives a
// pointer of type R (ErasureConsensus::*)(A...); one it only inherits would
// have the base's class type, and one it declares with other parameters
// would not convert -- so each assertion pins both "declared here" and the
// exact reference signature.  The `override` keyword on each declaration
// pins the same signatures against the base's virtuals.
#include <type_traits>

#include "../erasure_consensus.hh"

using namespace memo_host;

namespace {

struct Probe : ErasureConsensus {
  using ErasureConsensus::ErasureConsensus;
  using EC = ErasureConsensus;
  using AV = Consensus::AddressVersion;

  // Blocks (Consensus.hh:63-80)
  static_assert(std::is_same_v<decltype(&Probe::_store),
                               void (EC::*)(std::unique_ptr<Block>, StoreMode, std::unique_ptr<ConflictResolver>)>,
                "_store(unique_ptr<Block>, StoreMode, unique_ptr<ConflictResolver>)");
  static constexpr std::unique_ptr<Block> (EC::*fetch_one)(Address, std::optional<int>) = &Probe::_fetch;
  static constexpr void (EC::*fetch_many)(const std::vector<AV>&, ReceiveBlock) = &Probe::_fetch;
  static_assert(std::is_same_v<decltype(&Probe::_remove), void (EC::*)(Address, RemoveSignature)>,
                "_remove(Address, RemoveSignature)");
  static_assert(std::is_same_v<decltype(&Probe::_resign), void (EC::*)()>, "_resign()");
};

// Stat (Consensus.hh:85-95)
static_assert(std::is_same_v<decltype(&ErasureConsensus::stat),
                             std::unique_ptr<Consensus::Stat> (ErasureConsensus::*)(const Address&)>,
              "stat(Address const&)");
// Factory (Consensus.hh:100-108): make_local here, make_remote from
// StackedConsensus (it asks the backend, Consensus.cc:392-401)
static_assert(std::is_same_v<decltype(&ErasureConsensus::make_local),
                             std::unique_ptr<Local> (ErasureConsensus::*)(
                                 std::optional<int>, std::optional<IpAddress>, std::unique_ptr<Silo>)>,
              "make_local(optional<int>, optional<ip::address>, unique_ptr<Silo>)");
static_assert(std::is_same_v<decltype(&ErasureConsensus::make_remote),
                             std::shared_ptr<Remote> (StackedConsensus::*)(std::shared_ptr<DockConnection>)>,
              "make_remote(shared_ptr<Dock::Connection>) from StackedConsensus");
// Monitoring (Consensus.hh:113-119)
static_assert(std::is_same_v<decltype(&ErasureConsensus::redundancy), std::string (ErasureConsensus::*)()>,
              "redundancy()");
static_assert(std::is_same_v<decltype(&ErasureConsensus::stats), std::string (ErasureConsensus::*)()>,
              "stats()");

// The public calls are the base's (Consensus.hh:39-61)
static_assert(std::is_same_v<decltype(static_cast<void (Consensus::*)(std::unique_ptr<Block>, StoreMode,
                                                                      std::unique_ptr<ConflictResolver>)>(
                                 &Consensus::store)),
                             void (Consensus::*)(std::unique_ptr<Block>, StoreMode, std::unique_ptr<ConflictResolver>)>);
static_assert(std::is_same_v<decltype(static_cast<std::unique_ptr<Block> (Consensus::*)(Address, std::optional<int>)>(
                                 &Consensus::fetch)),
                             std::unique_ptr<Block> (Consensus::*)(Address, std::optional<int>)>);
static_assert(std::is_same_v<decltype(static_cast<void (Consensus::*)(const std::vector<Consensus::AddressVersion>&,
                                                                      ReceiveBlock)>(&Consensus::fetch)),
                             void (Consensus::*)(const std::vector<Consensus::AddressVersion>&, ReceiveBlock)>);
static_assert(std::is_same_v<decltype(&Consensus::remove), void (Consensus::*)(Address, RemoveSignature)>);

// The stack (Consensus.hh:129-142): an erasure consensus is a stacked one,
// concrete, and StackedConsensus::find reaches it and its backend.
static_assert(std::is_base_of_v<StackedConsensus, ErasureConsensus>);
static_assert(!std::is_abstract_v<ErasureConsensus>);
static_assert(!std::is_abstract_v<ReplicationConsensus>);
static_assert(std::is_same_v<decltype(StackedConsensus::find<ReplicationConsensus>(nullptr)), ReplicationConsensus*>);
static_assert(std::is_same_v<decltype(std::declval<const StackedConsensus&>().backend()),
                             const std::unique_ptr<Consensus>&>);

}  // namespace
