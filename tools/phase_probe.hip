// phase_probe.hip -- can a two-pass encode beat the one-pass kernel's
// interleaved read/write rate?  Standalone diagnostic (not part of
// libmemo_ec.so); the C2 shape, k = 10 input shards and m = 4 outputs per
// block, no GF math (the outputs are XORs of rotated inputs, the same for
// every variant, so the variants' outputs are compared byte for byte).
//
//   onepass     : per 16-byte column, load the 10 shards (nt), store the 4
//                 outputs (nt) -- the codec's traffic shape (75-76% of 8 TB/s)
//   twophase C  : blocks in chunks of C MB of outputs; per chunk, pass A
//                 loads the shards and stores the outputs into a scratch
//                 buffer reused by every chunk (meant to stay in the 256 MiB
//                 Infinity Cache), pass B copies scratch -> output (nt
//                 stores).  If the scratch stays on die, HBM sees a
//                 read-only phase and a write-only phase per chunk.
//   read / write: the loads alone, the stores alone (the phases' ceilings)
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_bin/phase_probe tools/phase_probe.hip
// Run:   tools/_bin/phase_probe [rounds]   (one JSON line per variant and round)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                  \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int K = 10, R = 4;

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
__device__ __forceinline__ u32x4 rotl(u32x4 v, int s) {
  return (v << s) | (v >> (32 - s));
}

// Units u = b*C + c (C = S/16 columns per shard), blocks [b0, b1).  Inputs
// at in + b*K*S + j*S, outputs at out + (b - ob)*R*S + i*S.
template <bool NT_OUT>
__global__ void __launch_bounds__(256) k_pass_a(const uint8_t* in, uint8_t* out, uint64_t S, uint64_t b0,
                                                uint64_t b1, uint64_t ob) {
  const uint64_t C = S / 16;
  const uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x + b0 * C;
  if (u >= b1 * C) return;
  const uint64_t b = u / C, c = u - b * C;
  const uint8_t* p = in + b * K * S + c * 16;
  u32x4 d[K];
#pragma unroll
  for (int j = 0; j < K; ++j) d[j] = ld<true>(reinterpret_cast<const u32x4*>(p + j * S));
  uint8_t* q = out + (b - ob) * R * S + c * 16;
#pragma unroll
  for (int i = 0; i < R; ++i) {
    u32x4 a = d[0];
#pragma unroll
    for (int j = 1; j < K; ++j) a ^= rotl(d[j], 1 + ((i + j) & 7));
    st<NT_OUT>(reinterpret_cast<u32x4*>(q + i * S), a);
  }
}

// scratch -> output for blocks [b0, b1): a flat copy of (b1-b0)*R*S bytes.
__global__ void __launch_bounds__(256) k_pass_b(const uint8_t* scratch, uint8_t* out, uint64_t nvec) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nvec) return;
  st<true>(reinterpret_cast<u32x4*>(out) + i, ld<false>(reinterpret_cast<const u32x4*>(scratch) + i));
}

__global__ void __launch_bounds__(256) k_read(const uint8_t* in, uint8_t* sink, uint64_t S, uint64_t n) {
  const uint64_t C = S / 16;
  const uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (u >= n * C) return;
  const uint64_t b = u / C, c = u - b * C;
  const uint8_t* p = in + b * K * S + c * 16;
  u32x4 a = {0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < K; ++j) a ^= ld<true>(reinterpret_cast<const u32x4*>(p + j * S));
  if (a.x == 0x9E3779B9u && a.y == 0x7F4A7C15u) *reinterpret_cast<u32x4*>(sink) = a;  // keep live
}

__global__ void __launch_bounds__(256) k_write(uint8_t* out, uint64_t S, uint64_t n) {
  const uint64_t C = S / 16;
  const uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (u >= n * C) return;
  const uint64_t b = u / C, c = u - b * C;
  uint8_t* q = out + b * R * S + c * 16;
  const u32x4 v = {(uint32_t)u, 2, 3, 4};
#pragma unroll
  for (int i = 0; i < R; ++i) st<true>(reinterpret_cast<u32x4*>(q + i * S), v);
}

__global__ void k_fill(uint8_t* p, uint64_t n, uint64_t seed) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n / 8; i += (uint64_t)gridDim.x * 256) {
    uint64_t z = (i + seed) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    reinterpret_cast<uint64_t*>(p)[i] = z ^ (z >> 31);
  }
}

__global__ void k_diff(const uint64_t* a, const uint64_t* b, uint64_t n, unsigned long long* bad) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    if (a[i] != b[i]) atomicAdd(bad, 1ull);
}

static unsigned grid_for(uint64_t units) { return (unsigned)((units + 255) / 256); }

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 3;
  const uint64_t n = 4096, S = 104896, C = S / 16;
  const uint64_t in_bytes = n * K * S, out_bytes = n * R * S;
  uint8_t *in, *out, *ref, *scratch, *sink;
  unsigned long long* bad;
  const uint64_t max_chunk = 128ull << 20;
  CHK(hipMalloc(&in, in_bytes));
  CHK(hipMalloc(&out, out_bytes));
  CHK(hipMalloc(&ref, out_bytes));
  CHK(hipMalloc(&scratch, max_chunk + R * S));
  CHK(hipMalloc(&sink, 64));
  CHK(hipMalloc(&bad, sizeof(*bad)));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, in, in_bytes, 1);
  CHK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));

  // the reference outputs
  hipLaunchKernelGGL(k_pass_a<true>, dim3(grid_for(n * C)), dim3(256), 0, 0, in, ref, S, 0, n, 0);
  CHK(hipDeviceSynchronize());

  struct Variant {
    const char* name;
    uint64_t chunk_mb;  // 0: one pass
    int kind;           // 0 onepass, 1 twophase (scratch plain stores), 2 twophase (scratch nt), 3 read, 4 write
  };
  std::vector<Variant> vs = {{"onepass", 0, 0},        {"read", 0, 3},          {"write", 0, 4},
                             {"twophase", 16, 1},      {"twophase", 32, 1},     {"twophase", 64, 1},
                             {"twophase", 128, 1},     {"twophase_nt", 32, 2},  {"twophase_nt", 64, 2}};
  auto run = [&](const Variant& v) {
    if (v.kind == 0) {
      hipLaunchKernelGGL(k_pass_a<true>, dim3(grid_for(n * C)), dim3(256), 0, 0, in, out, S, 0, n, 0);
    } else if (v.kind == 3) {
      hipLaunchKernelGGL(k_read, dim3(grid_for(n * C)), dim3(256), 0, 0, in, sink, S, n);
    } else if (v.kind == 4) {
      hipLaunchKernelGGL(k_write, dim3(grid_for(n * C)), dim3(256), 0, 0, out, S, n);
    } else {
      const uint64_t per = std::max<uint64_t>(1, (v.chunk_mb << 20) / (R * S));
      for (uint64_t b0 = 0; b0 < n; b0 += per) {
        const uint64_t b1 = std::min(n, b0 + per);
        if (v.kind == 1)
          hipLaunchKernelGGL(k_pass_a<false>, dim3(grid_for((b1 - b0) * C)), dim3(256), 0, 0, in, scratch, S, b0,
                             b1, b0);
        else
          hipLaunchKernelGGL(k_pass_a<true>, dim3(grid_for((b1 - b0) * C)), dim3(256), 0, 0, in, scratch, S, b0,
                             b1, b0);
        const uint64_t nvec = (b1 - b0) * R * S / 16;
        hipLaunchKernelGGL(k_pass_b, dim3(grid_for(nvec)), dim3(256), 0, 0, scratch, out + b0 * R * S, nvec);
      }
    }
  };
  const double alg = (double)(in_bytes + out_bytes);
  for (int r = 0; r < rounds; ++r) {
    for (auto& v : vs) {
      for (int w = 0; w < 20; ++w) run(v);  // settle clocks
      CHK(hipDeviceSynchronize());
      std::vector<float> ms;
      for (int t = 0; t < 20; ++t) {
        CHK(hipEventRecord(e0, 0));
        run(v);
        CHK(hipEventRecord(e1, 0));
        CHK(hipEventSynchronize(e1));
        float x;
        CHK(hipEventElapsedTime(&x, e0, e1));
        ms.push_back(x);
      }
      std::sort(ms.begin(), ms.end());
      const double med = ms[ms.size() / 2];
      double bytes = alg;
      if (v.kind == 3) bytes = (double)in_bytes;
      if (v.kind == 4) bytes = (double)out_bytes;
      long long nbad = -1;
      if (v.kind <= 2) {
        CHK(hipMemset(bad, 0, sizeof(*bad)));
        hipLaunchKernelGGL(k_diff, dim3(4096), dim3(256), 0, 0, (const uint64_t*)out, (const uint64_t*)ref,
                           out_bytes / 8, bad);
        unsigned long long h;
        CHK(hipMemcpy(&h, bad, sizeof(h), hipMemcpyDeviceToHost));
        nbad = (long long)h;
        CHK(hipMemset(out, 0, out_bytes));
      }
      printf("{\"variant\": \"%s\", \"chunk_mb\": %llu, \"round\": %d, \"ms\": %.4f, \"TBs\": %.3f, "
             "\"frac_of_8TBs\": %.4f, \"words_differing\": %lld}\n",
             v.name, (unsigned long long)v.chunk_mb, r, med, bytes / med / 1e9, bytes / med / 1e9 / 8.0, nbad);
      fflush(stdout);
    }
  }
  return 0;
}
