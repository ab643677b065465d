// lds_dma_probe.hip -- does streaming the k input shards through LDS-DMA
// (global_load_lds_dwordx4) beat register loads for the MAC's access pattern?
// Standalone diagnostic (not part of libmemo_ec.so).  Four kernels over the
// C2 geometry (4096 blocks, k = 10, m = 4, S = 104896), one 256-column tile
// per workgroup, units numbered across blocks as gf_mac_kernel does:
//   reg_r  : 10 dwordx4 nt loads per lane into registers, XOR, no stores
//   dma_r  : the same bytes by global_load_lds_dwordx4 (nt), read back from LDS
//   reg_rw : reg_r + 4 dwordx4 nt stores per lane (the MAC's traffic, no GF math)
//   dma_rw : dma_r + the same stores
//   reg_rw_staged : reg_rw with the stores regrouped through LDS (one shard per wave)
//   write  : the 4 output shards only
//   reg_rw1 : reg_r + one output shard (a 1-erasure rebuild's traffic)
//   reg_rw_2tiles : reg_rw with two tiles per workgroup, all loads before all stores
// Interleaved rounds after a warm burst (clock ramp).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_bin/lds_dma_probe tools/lds_dma_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int K = 10, M = 4;

struct Geo {
  const uint8_t* in;
  uint8_t* out;
  uint64_t S, C, n;  // C = S / 16 columns per shard
};

__device__ __forceinline__ void unit_of(const Geo& g, uint64_t& in_off, uint64_t& out_off,
                                        bool& valid) {
  uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  valid = u < g.n * g.C;
  if (!valid) u = 0;
  const uint64_t b = u / g.C, c = u - b * g.C;
  in_off = b * K * g.S + c * 16;
  out_off = b * M * g.S + c * 16;
}

template <bool WRITE>
__global__ void __launch_bounds__(256) reg_kernel(Geo g) {
  uint64_t io, oo;
  bool valid;
  unit_of(g, io, oo, valid);
  u32x4 d[K];
#pragma unroll
  for (int j = 0; j < K; ++j)
    d[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(g.in + io + j * g.S));
  u32x4 a = d[0];
#pragma unroll
  for (int j = 1; j < K; ++j) a ^= d[j];
  if constexpr (WRITE) {
    if (valid)
#pragma unroll
      for (int i = 0; i < M; ++i)
        __builtin_nontemporal_store(a ^ d[i], reinterpret_cast<u32x4*>(g.out + oo + i * g.S));
  } else if (a.x == 0x9E3779B9u && a.y == 0x7F4A7C15u) {
    *reinterpret_cast<u32x4*>(g.out) = a;  // keep the loads live
  }
}

template <bool WRITE>
__global__ void __launch_bounds__(256) dma_kernel(Geo g) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[K * 4 * 1024];
  uint64_t io, oo;
  bool valid;
  unit_of(g, io, oo, valid);
  const int w = threadIdx.x / 64, l = threadIdx.x % 64;
#pragma unroll
  for (int j = 0; j < K; ++j)
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(g.in + io + j * g.S),
                                     (__attribute__((address_space(3))) void*)(lds + (j * 4 + w) * 1024),
                                     16, 0, 2 /* nt */);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  u32x4 d[K];
#pragma unroll
  for (int j = 0; j < K; ++j) d[j] = *reinterpret_cast<const u32x4*>(lds + (j * 4 + w) * 1024 + l * 16);
  u32x4 a = d[0];
#pragma unroll
  for (int j = 1; j < K; ++j) a ^= d[j];
  if constexpr (WRITE) {
    if (valid)
#pragma unroll
      for (int i = 0; i < M; ++i)
        __builtin_nontemporal_store(a ^ d[i], reinterpret_cast<u32x4*>(g.out + oo + i * g.S));
  } else if (a.x == 0x9E3779B9u && a.y == 0x7F4A7C15u) {
    *reinterpret_cast<u32x4*>(g.out) = a;
  }
}

// reg_rw with the stores regrouped through LDS: wave w writes output shard w's
// 4 KiB of the tile (4 contiguous 1 KiB instructions) instead of every wave
// writing 1 KiB of each of the 4 shards.
__global__ void __launch_bounds__(256) reg_rw_staged_kernel(Geo g) {
  __shared__ __attribute__((aligned(16))) u32x4 st[M][256];
  uint64_t io, oo;
  bool valid;
  unit_of(g, io, oo, valid);
  u32x4 d[K];
#pragma unroll
  for (int j = 0; j < K; ++j)
    d[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(g.in + io + j * g.S));
  u32x4 a = d[0];
#pragma unroll
  for (int j = 1; j < K; ++j) a ^= d[j];
#pragma unroll
  for (int i = 0; i < M; ++i) st[i][threadIdx.x] = a ^ d[i];
  __syncthreads();
  const int w = threadIdx.x / 64, l = threadIdx.x % 64;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint64_t u = (uint64_t)blockIdx.x * 256 + q * 64 + l;
    if (u < g.n * g.C) {
      const uint64_t b = u / g.C, c = u - b * g.C;
      __builtin_nontemporal_store(st[w][q * 64 + l],
                                  reinterpret_cast<u32x4*>(g.out + b * M * g.S + w * g.S + c * 16));
    }
  }
}

// reg_rw with one output shard (a 1-erasure rebuild's traffic)
__global__ void __launch_bounds__(256) reg_rw1_kernel(Geo g) {
  uint64_t io, oo;
  bool valid;
  unit_of(g, io, oo, valid);
  u32x4 d[K];
#pragma unroll
  for (int j = 0; j < K; ++j)
    d[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(g.in + io + j * g.S));
  u32x4 a = d[0];
#pragma unroll
  for (int j = 1; j < K; ++j) a ^= d[j];
  const uint64_t b = oo / (M * g.S);
  if (valid) __builtin_nontemporal_store(a, reinterpret_cast<u32x4*>(g.out + b * g.S + (oo - b * M * g.S)));
}

// reg_rw over two tiles per workgroup: both tiles' loads, then both tiles'
// stores (longer read and write runs per CU)
__global__ void __launch_bounds__(256) reg_rw_t2_kernel(Geo g) {
  u32x4 a[2], d0[2][M];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    uint64_t u = ((uint64_t)blockIdx.x * 2 + t) * 256 + threadIdx.x;
    if (u >= g.n * g.C) u = 0;
    const uint64_t b = u / g.C, c = u - b * g.C;
    const uint8_t* in = g.in + b * K * g.S + c * 16;
    u32x4 x = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(in + j * g.S));
      x ^= v;
      if (j < M) d0[t][j] = v;
    }
    a[t] = x;
  }
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const uint64_t u = ((uint64_t)blockIdx.x * 2 + t) * 256 + threadIdx.x;
    if (u >= g.n * g.C) continue;
    const uint64_t b = u / g.C, c = u - b * g.C;
#pragma unroll
    for (int i = 0; i < M; ++i)
      __builtin_nontemporal_store(a[t] ^ d0[t][i],
                                  reinterpret_cast<u32x4*>(g.out + b * M * g.S + i * g.S + c * 16));
  }
}

// write-only reference: the 4 output shards of every tile, nothing read
__global__ void __launch_bounds__(256) write_kernel(Geo g) {
  uint64_t io, oo;
  bool valid;
  unit_of(g, io, oo, valid);
  const u32x4 v = {(uint32_t)io, 1u, 2u, 3u};
  if (valid)
#pragma unroll
    for (int i = 0; i < M; ++i)
      __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(g.out + oo + i * g.S));
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 4096;
  const uint64_t S = 104896, C = S / 16;
  uint8_t *in, *out;
  CHK(hipMalloc(&in, n * K * S));
  CHK(hipMalloc(&out, n * M * S));
  CHK(hipMemset(in, 0x5A, n * K * S));
  CHK(hipMemset(out, 0, n * M * S));
  Geo g{in, out, S, C, n};
  const uint32_t grid = (uint32_t)((n * C + 255) / 256);
  const double rbytes = (double)n * K * S, wbytes = (double)n * M * S;
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  constexpr int NV = 8;
  const char* names[NV] = {"reg_r", "dma_r", "reg_rw", "dma_rw", "reg_rw_staged", "write", "reg_rw1",
                           "reg_rw_2tiles"};
  auto launch = [&](int v) {
    switch (v) {
      case 0: hipLaunchKernelGGL(reg_kernel<false>, dim3(grid), dim3(256), 0, 0, g); break;
      case 1: hipLaunchKernelGGL(dma_kernel<false>, dim3(grid), dim3(256), 0, 0, g); break;
      case 2: hipLaunchKernelGGL(reg_kernel<true>, dim3(grid), dim3(256), 0, 0, g); break;
      case 3: hipLaunchKernelGGL(dma_kernel<true>, dim3(grid), dim3(256), 0, 0, g); break;
      case 4: hipLaunchKernelGGL(reg_rw_staged_kernel, dim3(grid), dim3(256), 0, 0, g); break;
      case 5: hipLaunchKernelGGL(write_kernel, dim3(grid), dim3(256), 0, 0, g); break;
      case 6: hipLaunchKernelGGL(reg_rw1_kernel, dim3(grid), dim3(256), 0, 0, g); break;
      default: hipLaunchKernelGGL(reg_rw_t2_kernel, dim3((grid + 1) / 2), dim3(256), 0, 0, g); break;
    }
  };
  std::vector<std::vector<float>> ms(NV);
  for (int round = 0; round < 6; ++round)
    for (int v = 0; v < NV; ++v) {
      for (int i = 0; i < 40; ++i) launch(v);
      for (int i = 0; i < 10; ++i) {
        CHK(hipEventRecord(a, 0));
        launch(v);
        CHK(hipEventRecord(b, 0));
        CHK(hipEventSynchronize(b));
        float t;
        CHK(hipEventElapsedTime(&t, a, b));
        ms[v].push_back(t);
      }
    }
  CHK(hipGetLastError());
  for (int v = 0; v < NV; ++v) {
    std::sort(ms[v].begin(), ms[v].end());
    const double med = ms[v][ms[v].size() / 2];
    const double bytes = (v == 5 ? 0.0 : rbytes) + (v == 6 ? wbytes / M : v >= 2 ? wbytes : 0.0);
    printf("{\"probe\":\"%s\",\"blocks\":%llu,\"ms_med\":%.4f,\"TBs\":%.3f,\"frac\":%.4f}\n",
           names[v], (unsigned long long)n, med, bytes / (med * 1e-3) / 1e12,
           bytes / (med * 1e-3) / 8e12);
  }
  CHK(hipFree(in));
  CHK(hipFree(out));
  return 0;
}
