// bench_plugin.cc -- plugin-level throughput of the erasure consensus
// (host/erasure_consensus.hh) against the replication path it replaces, on
// an in-process network of memory-silo nodes (tests/DHT.hh-style): store,
// healthy multi-fetch, degraded multi-fetch (m nodes down) and repair after
// eviction.  Everything a memo node does per block runs: CHB address check,
// shard framing + CRC32C, silo stores, GPU encode / decode through
// libmemo_ec; only the network is absent.  Store, fetch and degraded fetch
// report steady-state rates (a cold pass first: the codec contexts allocate
// their scratch on first use) beside the cold ones.  Prints one JSON line.
//   usage: bench_plugin [blocks] [block_bytes]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

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

struct Net {
  Overlay overlay;
  std::vector<std::shared_ptr<Node>> nodes;
  explicit Net(int n) {
    for (int i = 0; i < n; ++i) {
      uint8_t id[32] = {0};
      id[0] = (uint8_t)(i + 1);
      id[1] = 0x42;
      nodes.push_back(overlay.add_node(Address(id, 0, false), std::make_unique<MemorySilo>()));
    }
  }
};

double gib(size_t bytes, double s) { return bytes / s / (1u << 30); }

}  // namespace

int main(int argc, char** argv) {
  const size_t nb = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 512;
  const size_t B = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : (1u << 20);
  const int k = 10, m = 4, factor = 3, N = 20;
  const size_t total = nb * B;

  double t = now();
  std::vector<Block> blocks;
  blocks.reserve(nb);
  for (size_t i = 0; i < nb; ++i) blocks.push_back(make_chb(random_bytes(B, i + 1)));
  const double t_chb = now() - t;
  std::vector<Address> addrs;
  for (auto& b : blocks) addrs.push_back(b.address);

  // ---- erasure: RS(10,4)
  Net en(N);
  ErasureOptions o;
  o.k = k;
  o.m = m;
  // MEMO_EC_PLUGIN_THREADS: host pool size (scaling runs)
  if (const char* t = std::getenv("MEMO_EC_PLUGIN_THREADS")) o.threads = std::atoi(t);
  ErasureConsensus ec(std::make_unique<ReplicationConsensus>(en.overlay, factor), en.overlay, o);
  // The first half of the blocks is stored cold (the codec contexts allocate
  // their pinned and device scratch on first use), the second half warm;
  // fetches run twice and report the second pass.
  const size_t half = nb / 2;
  std::vector<Block> first(std::make_move_iterator(blocks.begin()),
                           std::make_move_iterator(blocks.begin() + half));
  std::vector<Block> second(std::make_move_iterator(blocks.begin() + half),
                            std::make_move_iterator(blocks.end()));
  t = now();
  ec.store_many(first);
  const double t_store_cold = now() - t;
  t = now();
  ec.store_many(second);
  const double t_store = now() - t;

  size_t ok = 0;
  auto check = [&](const Address& a, std::unique_ptr<Block> b, std::exception_ptr e) {
    if (!e && b && b->address == a) ++ok;
  };
  ec.fetch(addrs, check);
  const double t0_fetch = now();
  ok = 0;
  ec.fetch(addrs, check);
  const double t_fetch = now() - t0_fetch;
  const bool fetch_ok = ok == nb;

  // m nodes holding shards go down: every read needs the decode
  int down = 0;
  for (auto& n : en.nodes)
    if (down < m && !n->silo->list().empty()) {
      n->up = false;
      ++down;
    }
  ok = 0;
  t = now();
  ec.fetch(addrs, check);
  const double t_degraded_cold = now() - t;
  bool degraded_ok = ok == nb;
  auto codec_calls = [&] {
    return ec.codec().rebuild_calls() + ec.codec().uniform_calls() + ec.codec().segments_calls();
  };
  const uint64_t dec0 = codec_calls();
  ok = 0;
  t = now();
  ec.fetch(addrs, check);
  const double t_degraded = now() - t;
  degraded_ok = degraded_ok && ok == nb;
  const uint64_t degraded_calls = codec_calls() - dec0;

  // they are evicted: rebuild their shards onto other nodes
  for (auto& n : en.nodes)
    if (!n->up) n->evicted = true;
  t = now();
  const auto rep = ec.repair();
  const double t_repair = now() - t;
  // every block reads back (CHB address re-checked on the reassembled
  // bytes) from the repaired placement, the evicted nodes gone
  ok = 0;
  ec.fetch(addrs, check);
  const bool repaired_ok = ok == nb;

  // ---- replication (memo's path today): factor full copies
  Net rn(N);
  ReplicationConsensus rc(rn.overlay, factor);
  t = now();
  for (auto* v : {&first, &second})
    for (auto& b : *v) rc.store(b);
  const double t_rstore = now() - t;
  ok = 0;
  t = now();
  rc.fetch(addrs, check);
  const double t_rfetch = now() - t;
  const bool rfetch_ok = ok == nb;

  std::printf(
      "{\"workload\": \"%zu x %zu-byte CHBs, %d in-process memory-silo nodes\", "
      "\"chb_make_GiBs\": %.2f, "
      "\"erasure\": {\"code\": \"RS(%d,%d)\", \"store_GiBs\": %.2f, \"store_cold_GiBs\": %.2f, "
      "\"fetch_GiBs\": %.2f, "
      "\"fetch_ok\": %s, \"degraded_fetch_GiBs\": %.2f, \"degraded_fetch_cold_GiBs\": %.2f, "
      "\"degraded_ok\": %s, "
      "\"degraded_codec_calls\": %llu, \"repair_GiBs\": %.2f, \"repaired_blocks\": %zu, "
      "\"repair_codec_calls\": %zu, \"unrecoverable\": %zu, \"fetch_after_repair_ok\": %s, "
      "\"stored_bytes_per_byte\": %.2f}, "
      "\"replication\": {\"factor\": %d, \"store_GiBs\": %.2f, \"fetch_GiBs\": %.2f, "
      "\"fetch_ok\": %s, \"stored_bytes_per_byte\": %d}}\n",
      nb, B, N, gib(total, t_chb), k, m, gib((nb - half) * B, t_store), gib(half * B, t_store_cold),
      gib(total, t_fetch), fetch_ok ? "true" : "false", gib(total, t_degraded),
      gib(total, t_degraded_cold), degraded_ok ? "true" : "false",
      (unsigned long long)degraded_calls, gib(rep.blocks_repaired * B, t_repair),
      rep.blocks_repaired, rep.codec_calls, rep.unrecoverable, repaired_ok ? "true" : "false",
      (double)(k + m) * memo_ec_shard_size(B, k) / B, factor, gib(total, t_rstore),
      gib(total, t_rfetch), rfetch_ok ? "true" : "false", factor);
  return fetch_ok && degraded_ok && rfetch_ok && repaired_ok && rep.unrecoverable == 0 ? 0 : 1;
}
