// CPU-only probe of the plugin's shard placement (ErasureConsensus::place
// without the codec): T threads frame and store k+m shards per block into
// in-process memory-silo nodes, as a 4 KiB RS(10,4) store batch does.
// Prints blocks/s per thread count and the time split between framing and
// silo stores, to see what limits the pool's scaling (DESIGN.md section 6,
// plugin level).  Build: see tools/place_probe.sh.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../host/erasure_consensus.hh"

using namespace memo_host;

int main(int argc, char** argv) {
  const size_t nb = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 65536;
  // 0 full, 1 frame only, 2 store only, 3 one silo (no nodes), 4 a bare
  // unordered_map of shared buffers
  const int mode = argc > 2 ? std::atoi(argv[2]) : 0;
  const int k = 10, m = 4, total = k + m;
  const size_t S = 448;
  std::vector<uint8_t> payload(S, 0x5a);
  for (int T : {1, 2, 4, 8, 16}) {
    Overlay ov;
    for (int i = 0; i < 20; ++i) {
      Address id;
      id.value[0] = (uint8_t)i;
      id.value[1] = 0x77;
      ov.add_node(id, std::make_unique<MemorySilo>());
    }
    std::atomic<size_t> next{0};
    MemorySilo one;
    std::mutex bm;
    std::unordered_map<Key, std::shared_ptr<const Buffer>, AddressHash> bare;
    auto work = [&] {
      for (;;) {
        const size_t b = next.fetch_add(1);
        if (b >= nb) break;
        Address a;
        for (int q = 0; q < 8; ++q) a.value[q] = (uint8_t)(b >> (8 * q));
        a.value[31] = 0x01;
        const ShardKeys keys(a);
        auto owners = ov.allocate(a, total);
        for (int i = 0; i < total; ++i) {
          ShardHeader h;
          h.k = k;
          h.m = m;
          h.index = (uint8_t)i;
          h.block_size = 4096;
          h.shard_size = S;
          h.address = a;
          if (mode == 3) {
            one.set(keys(i), Buffer(128 + S));
            continue;
          }
          if (mode == 4) {
            auto v = std::make_shared<const Buffer>(128 + S);
            std::lock_guard<std::mutex> g(bm);
            bare.emplace(keys(i), std::move(v));
            continue;
          }
          if (mode == 2) {
            Buffer w(128 + S);
            owners[i]->store(keys(i), std::move(w));
          } else {
            Buffer w = encode_shard(h, payload.data());
            if (mode == 0) owners[i]->store(keys(i), std::move(w));
          }
        }
      }
    };
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> ts;
    for (int t = 0; t < T; ++t) ts.emplace_back(work);
    for (auto& t : ts) t.join();
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("{\"mode\": %d, \"threads\": %d, \"blocks\": %zu, \"blocks_per_s\": %.0f, \"us_per_store_thread\": %.3f}\n",
                mode, T, nb, nb / s, s * T * 1e6 / (nb * total));
    std::fflush(stdout);
  }
  return 0;
}
