// hbm_probe.hip -- what HBM bandwidth does the RS shard access pattern allow
// on this MI355X?  Standalone diagnostic (not part of libmemo_ec.so).
//   copy     : out[i] = in[i], float4, grid-stride
//   read     : XOR-reduce in[], one store per thread
//   write    : out[i] = const
//   shards   : the codec's pattern without GF math -- per 16-byte column of
//              a block, load kin shards (stride S), store r outputs
// Build: hipcc --offload-arch=gfx950 -O3 -o hbm_probe tools/hbm_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                              \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <bool NT>
__global__ void __launch_bounds__(256) k_copy(const u32x4* in, u32x4* out, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    st<NT>(out + i, ld<NT>(in + i));
}

template <bool NT>
__global__ void __launch_bounds__(256) k_read(const u32x4* in, u32x4* out, size_t n) {
  u32x4 a = {0, 0, 0, 0};
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    a ^= ld<NT>(in + i);
  if (a.x == 0x12345678u) out[threadIdx.x] = a;  // keep live
}

template <bool NT>
__global__ void __launch_bounds__(256) k_write(u32x4* out, size_t n) {
  const u32x4 v = {1, 2, 3, 4};
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    st<NT>(out + i, v);
}

// One unit (16-byte column of one block) per thread per iteration.
template <int K, int R, bool NT>
__global__ void __launch_bounds__(256) k_shards(const uint8_t* in, uint8_t* out, size_t n,
                                                uint32_t C, size_t S, int per_thread) {
  const size_t total = n * (size_t)C;
  const size_t base = ((size_t)blockIdx.x * 256 * per_thread) + threadIdx.x;
  for (int q = 0; q < per_thread; ++q) {
    size_t u = base + (size_t)q * 256;
    if (u >= total) return;
    const size_t b = u / C, c = u - b * C;
    const uint8_t* p = in + b * K * S + c * 16;
    u32x4 d[K];
#pragma unroll
    for (int j = 0; j < K; ++j) d[j] = ld<NT>(reinterpret_cast<const u32x4*>(p + j * S));
    u32x4 a = d[0];
#pragma unroll
    for (int j = 1; j < K; ++j) a ^= d[j];
    uint8_t* o = out + b * R * S + c * 16;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      u32x4 v = a;
      v.x += i;
      st<NT>(reinterpret_cast<u32x4*>(o + i * S), v);
    }
  }
}

// Median launch time over `iters` back-to-back launches after 60 untimed
// back-to-back warmup launches: the clocks dip a few launches into a burst
// and settle after ~40 (profiles/r01_clock_ramp.jsonl), so neither a single
// warmup launch nor a sync between launches measures the steady state.
template <typename F>
static float time_ms(F f, int iters) {
  std::vector<hipEvent_t> ev(2 * iters);
  for (auto& evt : ev) CHK(hipEventCreate(&evt));
  for (int i = 0; i < 60; ++i) f();
  for (int i = 0; i < iters; ++i) {
    CHK(hipEventRecord(ev[2 * i]));
    f();
    CHK(hipEventRecord(ev[2 * i + 1]));
  }
  CHK(hipDeviceSynchronize());
  std::vector<float> ts;
  for (int i = 0; i < iters; ++i) {
    float ms;
    CHK(hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]));
    ts.push_back(ms);
  }
  for (auto& evt : ev) CHK(hipEventDestroy(evt));
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}


// Generalised shard pattern: WG threads T, each lane W consecutive uint4 of
// one shard column (W=1: 16 B, W=2: 32 B), ORDER 0 = tiles of one block are
// consecutive workgroups, 1 = consecutive workgroups walk different blocks.
template <int K, int R, int T, int W, int ORDER>
__global__ void __launch_bounds__(T) k_shards2(const uint8_t* in, uint8_t* out, size_t n,
                                               uint32_t C, size_t S) {
  const uint32_t cols_per_wg = T * W;
  const uint32_t tpb = (C + cols_per_wg - 1) / cols_per_wg;
  size_t b, t;
  if (ORDER == 0) { b = blockIdx.x / tpb; t = blockIdx.x % tpb; }
  else { b = blockIdx.x % n; t = blockIdx.x / n; }
  if (b >= n) return;
  const uint32_t c0 = t * cols_per_wg + threadIdx.x * W;
  if (c0 >= C) return;
  const uint8_t* p = in + b * K * S + (size_t)c0 * 16;
  u32x4 d[K][W];
#pragma unroll
  for (int j = 0; j < K; ++j)
#pragma unroll
    for (int w = 0; w < W; ++w)
      d[j][w] = (c0 + w < C) ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + j * S) + w)
                             : u32x4{0, 0, 0, 0};
  uint8_t* o = out + b * R * S + (size_t)c0 * 16;
#pragma unroll
  for (int w = 0; w < W; ++w) {
    u32x4 a = d[0][w];
#pragma unroll
    for (int j = 1; j < K; ++j) a ^= d[j][w];
    if (c0 + w < C)
#pragma unroll
      for (int i = 0; i < R; ++i) {
        u32x4 v = a;
        v.x += i;
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(o + i * S) + w);
      }
  }
}

template <int T, int W, int ORDER>
static void run2(const uint8_t* din, uint8_t* dout, size_t n, uint32_t C, size_t S, double alg) {
  const uint32_t tpb = (C + T * W - 1) / (T * W);
  const int grid = (int)(tpb * n);
  float t = time_ms([&] { k_shards2<10, 4, T, W, ORDER><<<grid, T>>>(din, dout, n, C, S); }, 10);
  printf("{\"probe\":\"shards2\",\"S\":%zu,\"T\":%d,\"W\":%d,\"order\":%d,\"ms\":%.4f,\"TBs\":%.3f}\n", S, T, W,
         ORDER, t, alg / t / 1e9);
}

int main() {
  const size_t bytes = 4ull << 30;  // 4 GiB each side
  uint8_t *in, *out;
  CHK(hipMalloc(&in, bytes + (64 << 20)));
  CHK(hipMalloc(&out, bytes + (64 << 20)));
  CHK(hipMemset(in, 1, bytes));
  CHK(hipMemset(out, 0, bytes));
  const size_t n4 = bytes / 16;
  const int iters = 20;
  for (int grid : {65536}) {
    float t;
    t = time_ms([&] { k_copy<false><<<grid, 256>>>((u32x4*)in, (u32x4*)out, n4); }, iters);
    printf("{\"probe\":\"copy\",\"nt\":0,\"grid\":%d,\"ms\":%.4f,\"TBs\":%.3f}\n", grid, t, 2.0 * bytes / t / 1e9);
    t = time_ms([&] { k_copy<true><<<grid, 256>>>((u32x4*)in, (u32x4*)out, n4); }, iters);
    printf("{\"probe\":\"copy\",\"nt\":1,\"grid\":%d,\"ms\":%.4f,\"TBs\":%.3f}\n", grid, t, 2.0 * bytes / t / 1e9);
    t = time_ms([&] { k_read<false><<<grid, 256>>>((u32x4*)in, (u32x4*)out, n4); }, iters);
    printf("{\"probe\":\"read\",\"nt\":0,\"grid\":%d,\"ms\":%.4f,\"TBs\":%.3f}\n", grid, t, 1.0 * bytes / t / 1e9);
    t = time_ms([&] { k_write<false><<<grid, 256>>>((u32x4*)out, n4); }, iters);
    printf("{\"probe\":\"write\",\"nt\":0,\"grid\":%d,\"ms\":%.4f,\"TBs\":%.3f}\n", grid, t, 1.0 * bytes / t / 1e9);
  }
  // shard pattern: 4096 x 1 MiB blocks RS(10,4): 4.3 GB in, 1.7 GB out
  const size_t n = 4096;
  for (size_t S : {(size_t)104896, (size_t)104960}) {
    uint8_t *din, *dout;
    CHK(hipMalloc(&din, n * 10 * S));
    CHK(hipMalloc(&dout, n * 4 * S));
    CHK(hipMemset(din, 3, n * 10 * S));
    const uint32_t C = S / 16;
    const double alg = (double)n * 14 * S;
    for (int pt : {1}) {
      const size_t total = n * C;
      const int grid = (int)((total + 256 * pt - 1) / (256 * pt));
      float t0 = time_ms([&] { k_shards<10, 4, false><<<grid, 256>>>(din, dout, n, C, S, pt); }, iters);
      float t1 = time_ms([&] { k_shards<10, 4, true><<<grid, 256>>>(din, dout, n, C, S, pt); }, iters);
      printf("{\"probe\":\"shards10x4\",\"S\":%zu,\"per_thread\":%d,\"ms_plain\":%.4f,\"TBs_plain\":%.3f,\"ms_nt\":%.4f,\"TBs_nt\":%.3f}\n",
             S, pt, t0, alg / t0 / 1e9, t1, alg / t1 / 1e9);
    }
    run2<64, 1, 0>(din, dout, n, C, S, alg);
    run2<128, 1, 0>(din, dout, n, C, S, alg);
    run2<256, 1, 0>(din, dout, n, C, S, alg);
    run2<512, 1, 0>(din, dout, n, C, S, alg);
    run2<1024, 1, 0>(din, dout, n, C, S, alg);
    run2<256, 1, 1>(din, dout, n, C, S, alg);
    run2<512, 1, 1>(din, dout, n, C, S, alg);
    run2<256, 2, 0>(din, dout, n, C, S, alg);
    run2<128, 2, 0>(din, dout, n, C, S, alg);
    run2<256, 2, 1>(din, dout, n, C, S, alg);
    CHK(hipFree(din));
    CHK(hipFree(dout));
  }
  return 0;
}
