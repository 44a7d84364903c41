// hashbench.hip -- VALU cost of XXH64 formulations on gfx950 (diagnostic only).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I deequ_amd/csrc tools/hashbench.hip -o tools/hashbench.bin
// Each kernel hashes register-resident values (no memory traffic) with one formulation and folds the
// HLL register index/rank into a checksum; prints SIMD-cycles per hash and checks every formulation
// against the reference one.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "dq_hash.h"

using namespace dq;

// 64 x 64 -> low 64 multiply by a constant with three multiply instructions:
//   t = lo32(x_hi * c_lo); u = lo32(x_lo * c_hi + t); r = x_lo * c_lo + (u << 32)
__device__ __forceinline__ uint64_t mulc3(uint64_t x, uint64_t c) {
  const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
  const uint32_t cl = (uint32_t)c, ch = (uint32_t)(c >> 32);
  const uint32_t t = xh * cl;
  const uint32_t u = xl * ch + t;
  return (uint64_t)xl * cl + ((uint64_t)u << 32);
}

__device__ __forceinline__ uint64_t mad_u64_u32(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t r;
  asm volatile("v_mad_u64_u32 %0, s[100:101], %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(c) : "s100", "s101");
  return r;
}

__device__ __forceinline__ uint64_t mulc_asm(uint64_t x, uint64_t c) {
  const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
  const uint32_t cl = (uint32_t)c, ch = (uint32_t)(c >> 32);
  const uint32_t t = xh * cl;
  const uint64_t u = mad_u64_u32(xl, ch, (uint64_t)t);
  return mad_u64_u32(xl, cl, (uint64_t)(uint32_t)u << 32);
}

template <int F>
__device__ __forceinline__ uint64_t mul(uint64_t x, uint64_t c) {
  if constexpr (F == 0) return x * c;
  else if constexpr (F == 1) return mulc3(x, c);
  else return mulc_asm(x, c);
}

template <int F>
__device__ __forceinline__ uint64_t h_long(uint64_t v) {
  uint64_t h = kSeed + XP5 + 8;
  h ^= mul<F>(rotl64(mul<F>(v, XP2), 31), XP1);
  h = mul<F>(rotl64(h, 27), XP1) + XP4;
  h ^= h >> 33; h = mul<F>(h, XP2); h ^= h >> 29; h = mul<F>(h, XP3); h ^= h >> 32;
  return h;
}

template <int F>
__global__ __launch_bounds__(256) void k(uint64_t* out, uint64_t seed, int iters) {
  uint64_t v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = seed + (uint64_t)(blockIdx.x * 256 + threadIdx.x) * 8 + j;
  uint32_t acc = 0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint64_t h = h_long<F>(v[j]);
      const uint32_t idx = (uint32_t)(h >> 55);
      const uint32_t pw = (uint32_t)__clzll((long long)((h << 9) | 256ull)) + 1u;
      acc += idx ^ (pw << 9);
      v[j] += 0x10000001ull;
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int F>
float run(uint64_t* out, int grid, int iters) {
  hipLaunchKernelGGL(k<F>, dim3(grid), dim3(256), 0, 0, out, 7ull, iters);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(k<F>, dim3(grid), dim3(256), 0, 0, out, 7ull, iters);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  const int grid = 256 * 16, iters = 64;
  const size_t n = (size_t)grid * 256;
  uint64_t* out;
  (void)hipMalloc(&out, n * 8 * 3);
  int dev;
  hipDeviceProp_t p;
  (void)hipGetDevice(&dev);
  (void)hipGetDeviceProperties(&p, dev);
  float t[3] = {run<0>(out, grid, iters), run<1>(out + n, grid, iters), run<2>(out + 2 * n, grid, iters)};
  uint64_t* h = new uint64_t[n * 3];
  (void)hipMemcpy(h, out, n * 8 * 3, hipMemcpyDeviceToHost);
  bool ok1 = true, ok2 = true;
  for (size_t i = 0; i < n; ++i) {
    ok1 &= h[i] == h[n + i];
    ok2 &= h[i] == h[2 * n + i];
  }
  const double hashes = (double)n * iters * 8;
  const char* names[3] = {"compiler_mul", "mulc3", "mulc_asm"};
  for (int f = 0; f < 3; ++f) {
    const double simd_cyc = (double)p.clockRate * 1e3 * (t[f] / 1e3) * p.multiProcessorCount * 4;
    std::printf("{\"form\": \"%s\", \"ms\": %.3f, \"Ghash_per_s\": %.1f, \"simd_cycles_per_wave_hash\": %.1f, \"match\": %s}\n",
                names[f], t[f], hashes / t[f] / 1e6, simd_cyc / (hashes / 64), f == 0 ? "true" : ((f == 1 ? ok1 : ok2) ? "true" : "false"));
  }
  return 0;
}
