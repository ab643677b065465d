// bench_plugin.cc -- plugin-level throughput of the erasure consensus
// (host/erasure_consensus.hh) against the replication path it replaces, on
// an in-process network of memory-silo nodes (tests/DHT.hh-style): store,
// healthy multi-fetch, degraded multi-fetch (m nodes down) and repair after
// eviction.  Everything a memo node does per block runs: CHB address check,
// shard framing + CRC32C, silo stores, GPU encode / decode through
// libmemo_ec; only the network is absent.
//
// The two sides run interleaved, `reps` times in one process (the order
// alternates: erasure first on even repetitions, replication first on odd
// ones), each repetition on fresh nodes, so that both see the same box state
// and a drift in the host's speed hits both.  Store, fetch and degraded
// fetch report steady-state rates (a cold pass first: the codec contexts
// allocate their scratch on first use) beside the cold ones.  Prints one JSON
// line with every repetition's rates as lists; bench.py (plugin_lines) turns
// them into median / min / max and per-repetition erasure / replication
// ratios.
//   usage: bench_plugin [blocks] [block_bytes] [reps]
//   env:   MEMO_EC_PLUGIN_THREADS  host pool size (scaling runs)
//          MEMO_EC_PLUGIN_HOSTONLY the host profiling build over
//                                  tests/null_codec.cc: degraded and repaired
//                                  reads timed, not checked
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../erasure_consensus.hh"

using namespace memo_host;

namespace {

double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

Buffer random_bytes(size_t n, uint64_t seed) {
  Buffer b(n);
  uint64_t x = seed * 0x9E3779B97F4A7C15ull + 1;
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
    std::memcpy(b.data() + i, &x, 8);
  }
  for (; i < n; ++i) b[i] = (uint8_t)(x >> (8 * (i & 7)));
  return b;
}

// n nodes, each one's peer made by `local` over a memory silo (the
// consensus's make_local: the validation its stores go through)
struct Net {
  Overlay overlay;
  std::vector<std::shared_ptr<Node>> nodes;
  template <class F>
  void populate(int n, F local) {
    for (int i = 0; i < n; ++i) {
      uint8_t id[32] = {0};
      id[0] = (uint8_t)(i + 1);
      id[1] = 0x42;
      nodes.push_back(overlay.add_node(Address(id, 0, false), local(std::make_unique<MemorySilo>())));
    }
  }
};

std::vector<Consensus::AddressVersion> request(const std::vector<Address>& addrs) {
  std::vector<Consensus::AddressVersion> r;
  for (auto& a : addrs) r.emplace_back(a, std::nullopt);
  return r;
}

double gib(size_t bytes, double s) { return bytes / s / (1u << 30); }

// "[a, b, c]" with two decimals
std::string list(const std::vector<double>& v) {
  std::string s = "[";
  char f[32];
  for (size_t i = 0; i < v.size(); ++i) {
    std::snprintf(f, sizeof f, "%s%.3f", i ? ", " : "", v[i]);
    s += f;
  }
  return s + "]";
}

struct ErasureRun {
  double store, store_cold, fetch, degraded, degraded_cold, repair;
  bool fetch_ok, degraded_ok, repaired_ok;
  uint64_t degraded_calls;
  size_t repaired, repair_calls, unrecoverable;
  std::string redundancy;
};

struct ReplicationRun {
  double store, fetch;
  bool fetch_ok;
};

const int k = 10, m = 4, factor = 3, N = 20;

ErasureRun run_erasure(const std::vector<Block>& first, const std::vector<Block>& second,
                       const std::vector<Address>& addrs, size_t B) {
  const size_t nb = addrs.size(), half = first.size(), total = nb * B;
  ErasureRun r{};
  Net en;
  ErasureOptions o;
  o.k = k;
  o.m = m;
  if (const char* t = std::getenv("MEMO_EC_PLUGIN_THREADS")) o.threads = std::atoi(t);
  ErasureConsensus ec(std::make_unique<ReplicationConsensus>(en.overlay, factor), en.overlay, o);
  // the nodes' peers are the consensus's: shards checked by CRC and key
  en.populate(N, [&](std::unique_ptr<Silo> s) { return ec.make_local({}, {}, std::move(s)); });
  r.redundancy = ec.redundancy();
  const auto req = request(addrs);
  // The first half of the blocks is stored cold (the codec contexts allocate
  // their pinned and device scratch on first use), the second half warm;
  // fetches run twice and report the second pass.
  double t = now();
  ec.store_many(first);
  r.store_cold = gib(half * B, now() - t);
  t = now();
  ec.store_many(second);
  r.store = gib((nb - half) * B, now() - t);

  size_t ok = 0;
  auto check = [&](const Address& a, std::unique_ptr<Block> b, std::exception_ptr e) {
    if (!e && b && b->address == a) ++ok;
  };
  ec.fetch(req, check);
  ok = 0;
  t = now();
  ec.fetch(req, check);
  r.fetch = gib(total, now() - t);
  r.fetch_ok = ok == nb;

  // host-side profiling over the null codec (make -C host hostprof): its
  // zeros fail every degraded read, so only the host work of the degraded
  // fetch and the repair is timed, not checked
  static const bool host_only = std::getenv("MEMO_EC_PLUGIN_HOSTONLY") != nullptr;
  // m nodes holding shards go down: every read needs the decode
  int down = 0;
  for (auto& n : en.nodes)
    if (down < m && !n->silo->list().empty()) {
      n->up = false;
      ++down;
    }
  ok = 0;
  t = now();
  ec.fetch(req, check);
  r.degraded_cold = gib(total, now() - t);
  r.degraded_ok = ok == nb;
  auto codec_calls = [&] {
    return ec.codec().rebuild_calls() + ec.codec().uniform_calls() + ec.codec().segments_calls();
  };
  const uint64_t dec0 = codec_calls();
  ok = 0;
  t = now();
  ec.fetch(req, check);
  r.degraded = gib(total, now() - t);
  r.degraded_ok = r.degraded_ok && ok == nb;
  r.degraded_calls = codec_calls() - dec0;

  // they are evicted: rebuild their shards onto other nodes
  for (auto& n : en.nodes)
    if (!n->up) n->evicted = true;
  t = now();
  const auto rep = ec.repair();
  r.repair = gib(rep.blocks_repaired * B, now() - t);
  r.repaired = rep.blocks_repaired;
  r.repair_calls = rep.codec_calls;
  r.unrecoverable = rep.unrecoverable;
  // every block reads back (CHB address re-checked on the reassembled
  // bytes) from the repaired placement, the evicted nodes gone
  ok = 0;
  ec.fetch(req, check);
  r.repaired_ok = ok == nb;
  if (host_only) r.degraded_ok = r.repaired_ok = true;
  return r;
}

// memo's path today: factor full copies, one block at a time.  validated:
// the nodes' peers are the consensus's (ReplicationConsensus::make_local:
// each replica re-hashed against its address and the key's previous value
// read first, as Paxos::LocalPeer::store does); otherwise plain peers that
// keep whatever arrives (the restatement of rounds 1-5).
ReplicationRun run_replication(const std::vector<Block>& first, const std::vector<Block>& second,
                               const std::vector<Address>& addrs, size_t B, bool validated) {
  const size_t nb = addrs.size();
  ReplicationRun r{};
  Net rn;
  ReplicationConsensus rc(rn.overlay, factor);
  if (validated) rn.populate(N, [&](std::unique_ptr<Silo> s) { return rc.make_local({}, {}, std::move(s)); });
  else rn.populate(N, [](std::unique_ptr<Silo> s) { return std::make_unique<Local>(std::move(s)); });
  // the blocks handed over (Consensus::store takes ownership), made outside
  // the timed region
  std::vector<std::unique_ptr<Block>> own;
  own.reserve(nb);
  for (auto* v : {&first, &second})
    for (auto& b : *v) own.push_back(std::make_unique<Block>(b));
  double t = now();
  for (auto& b : own) rc.store(std::move(b), STORE_INSERT, nullptr);
  r.store = gib(nb * B, now() - t);
  size_t ok = 0;
  auto check = [&](const Address& a, std::unique_ptr<Block> b, std::exception_ptr e) {
    if (!e && b && b->address == a) ++ok;
  };
  const auto req = request(addrs);
  t = now();
  rc.fetch(req, check);
  r.fetch = gib(nb * B, now() - t);
  r.fetch_ok = ok == nb;
  return r;
}

}  // namespace

int main(int argc, char** argv) {
  const size_t nb = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 512;
  const size_t B = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : (1u << 20);
  const int reps = argc > 3 ? std::max(1, std::atoi(argv[3])) : 5;
  const size_t total = nb * B;

  double t = now();
  std::vector<Block> blocks;
  blocks.reserve(nb);
  for (size_t i = 0; i < nb; ++i) blocks.push_back(make_chb(random_bytes(B, i + 1)));
  const double t_chb = now() - t;
  std::vector<Address> addrs;
  for (auto& b : blocks) addrs.push_back(b.address);
  const size_t half = nb / 2;
  std::vector<Block> first(std::make_move_iterator(blocks.begin()),
                           std::make_move_iterator(blocks.begin() + half));
  std::vector<Block> second(std::make_move_iterator(blocks.begin() + half),
                            std::make_move_iterator(blocks.end()));

  std::vector<ErasureRun> er;
  std::vector<ReplicationRun> rr, ru;  // replication, validating peers / plain peers
  std::string order;
  for (int rep = 0; rep < reps; ++rep) {
    if (rep % 2 == 0) {
      er.push_back(run_erasure(first, second, addrs, B));
      rr.push_back(run_replication(first, second, addrs, B, true));
      ru.push_back(run_replication(first, second, addrs, B, false));
      order += std::string(rep ? ", " : "") + "\"er\"";
    } else {
      ru.push_back(run_replication(first, second, addrs, B, false));
      rr.push_back(run_replication(first, second, addrs, B, true));
      er.push_back(run_erasure(first, second, addrs, B));
      order += std::string(rep ? ", " : "") + "\"re\"";
    }
  }
  auto col = [&](auto get, const auto& v) {
    std::vector<double> out;
    for (auto& x : v) out.push_back(get(x));
    return list(out);
  };
  bool fetch_ok = true, degraded_ok = true, repaired_ok = true, rfetch_ok = true;
  uint64_t degraded_calls = ~0ull;
  size_t repaired = ~(size_t)0, repair_calls = 0, unrecoverable = 0;
  for (auto& x : er) {
    fetch_ok = fetch_ok && x.fetch_ok;
    degraded_ok = degraded_ok && x.degraded_ok;
    repaired_ok = repaired_ok && x.repaired_ok;
    degraded_calls = std::min(degraded_calls, x.degraded_calls);
    repaired = std::min(repaired, x.repaired);
    repair_calls = std::max(repair_calls, x.repair_calls);
    unrecoverable = std::max(unrecoverable, x.unrecoverable);
  }
  for (auto* v : {&rr, &ru})
    for (auto& x : *v) rfetch_ok = rfetch_ok && x.fetch_ok;

  std::printf(
      "{\"workload\": \"%zu x %zu-byte CHBs, %d in-process memory-silo nodes\", \"reps\": %d, "
      "\"order\": [%s], \"chb_make_GiBs\": %.2f, "
      "\"erasure\": {\"code\": \"RS(%d,%d)\", \"redundancy\": %s, \"store_GiBs\": %s, "
      "\"store_cold_GiBs\": %s, \"fetch_GiBs\": %s, \"fetch_ok\": %s, \"degraded_fetch_GiBs\": %s, "
      "\"degraded_fetch_cold_GiBs\": %s, \"degraded_ok\": %s, \"degraded_codec_calls\": %llu, "
      "\"repair_GiBs\": %s, \"repaired_blocks\": %zu, \"repair_codec_calls\": %zu, "
      "\"unrecoverable\": %zu, \"fetch_after_repair_ok\": %s, \"stored_bytes_per_byte\": %.2f}, "
      "\"replication\": {\"factor\": %d, \"peers\": \"validating (LocalPeer::store)\", "
      "\"store_GiBs\": %s, \"fetch_GiBs\": %s, \"fetch_ok\": %s, \"stored_bytes_per_byte\": %d}, "
      "\"replication_unvalidated\": {\"factor\": %d, \"peers\": \"plain (rounds 1-5)\", "
      "\"store_GiBs\": %s, \"fetch_GiBs\": %s}}\n",
      nb, B, N, reps, order.c_str(), gib(total, t_chb), k, m, er[0].redundancy.c_str(),
      col([](const ErasureRun& x) { return x.store; }, er).c_str(),
      col([](const ErasureRun& x) { return x.store_cold; }, er).c_str(),
      col([](const ErasureRun& x) { return x.fetch; }, er).c_str(), fetch_ok ? "true" : "false",
      col([](const ErasureRun& x) { return x.degraded; }, er).c_str(),
      col([](const ErasureRun& x) { return x.degraded_cold; }, er).c_str(),
      degraded_ok ? "true" : "false", (unsigned long long)degraded_calls,
      col([](const ErasureRun& x) { return x.repair; }, er).c_str(), repaired, repair_calls,
      unrecoverable, repaired_ok ? "true" : "false",
      (double)(k + m) * memo_ec_shard_size(B, k) / B, factor,
      col([](const ReplicationRun& x) { return x.store; }, rr).c_str(),
      col([](const ReplicationRun& x) { return x.fetch; }, rr).c_str(), rfetch_ok ? "true" : "false",
      factor, factor, col([](const ReplicationRun& x) { return x.store; }, ru).c_str(),
      col([](const ReplicationRun& x) { return x.fetch; }, ru).c_str());
  return fetch_ok && degraded_ok && rfetch_ok && repaired_ok && unrecoverable == 0 ? 0 : 1;
}
