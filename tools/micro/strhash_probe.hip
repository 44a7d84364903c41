// strhash_probe.hip -- issue rate of the UTF8 HLL pass's hash with no memory traffic (diagnostic, not product).
//
// Every lane hashes a stream of synthetic strings (lengths 8..24 as C5's, bytes from a register xorshift) with
// the column pass's formulation (dq_hash.h: xxh64_stripes<2> + xxh64_tail_head with the b * P5 LDS table, the
// HLL key from the high word), the same exec-masked rounds, and max-updates HLL registers in LDS.  It reports
// SIMD cycles per wave-instruction (s_memtime of the slowest wave / VALU per SIMD, VALU counted from the code
// object by the caller) and strings per second, at W waves per SIMD, so the kernel's own rate (r3: ~4 cycles
// per VALU at 6 waves) can be compared with what the hash alone sustains.
//   hipcc --offload-arch=gfx950 -O3 -I deequ_amd/csrc tools/micro/strhash_probe.hip -o /tmp/strhash_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "dq_hash.h"

using namespace dq;

constexpr int kIters = 4096;

__device__ __forceinline__ int32_t ffbh_raw(uint32_t x) {
  int32_t r;
  asm("v_ffbh_u32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

template <int MODE>
__global__ __launch_bounds__(256) void probe(uint32_t* out, unsigned long long* t, const uint64_t* p5g) {
  __shared__ uint64_t p5[256];
  __shared__ int32_t regs[512];
  for (int i = threadIdx.x; i < 256; i += 256) p5[i] = p5g[i];
  for (int i = threadIdx.x; i < 512; i += 256) regs[i] = -1;
  __syncthreads();
  const auto bp = [](uint32_t b) { return p5[b]; };
  uint32_t x = 0x9E3779B9u * (blockIdx.x * 256 + threadIdx.x + 1);
  uint32_t acc = 0;
  const uint64_t c0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIters; ++it) {
    // 8 dwords of string bytes and a length 8..24 (17 values, as C5's) from one LCG step: ~11 VALU, measured
    // alone as MODE 9 and subtracted by the reader
    x = x * 1664525u + 1013904223u;
    uint32_t w[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) w[k] = x ^ (0x9E3779B9u * (uint32_t)(k + 1));
    const uint32_t len = 8u + __umulhi(x, 17u);
    if constexpr (MODE == 9) {
      acc += w[0] ^ w[7] ^ len;
      continue;
    }
    uint64_t d4p;
    const uint64_t h2 = xxh64_stripes<MODE == 1 ? 3 : 2>(w, len, d4p);
    const uint64_t b = xxh64_tail_head(h2, d4p, len, bp);
    const uint32_t bl = (uint32_t)b, bh = (uint32_t)(b >> 32);
    const uint32_t hi = __umulhi(bl, (uint32_t)XP3) + bl * (uint32_t)(XP3 >> 32) + bh * (uint32_t)XP3;
    const uint32_t addr = (hi >> 21) & 0x7FCu;
    const int32_t q = ffbh_raw(hi << 9);
    atomicMax(reinterpret_cast<int32_t*>(reinterpret_cast<char*>(regs) + addr), q);
  }
  const uint64_t c1 = __builtin_amdgcn_s_memtime();
  __syncthreads();
  acc += (uint32_t)regs[threadIdx.x] + (uint32_t)regs[threadIdx.x + 256];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
  if ((threadIdx.x & 63) == 0) t[blockIdx.x * 4 + (threadIdx.x >> 6)] = c1 - c0;
}

template <int MODE>
void run(const char* name, int wg_per_cu, const uint64_t* p5) {
  const int blocks = 256 * wg_per_cu;  // 4 waves per workgroup, one per SIMD: W = wg_per_cu waves per SIMD
  uint32_t* out;
  unsigned long long* t;
  hipMalloc(&out, 4 * 256 * blocks);
  hipMalloc(&t, 8 * 4 * blocks);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float ms = 0;
  for (int r = 0; r < 2; ++r) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(256), 0, 0, out, t, p5);
    hipEventRecord(e1);
    hipDeviceSynchronize();
  }
  hipEventElapsedTime(&ms, e0, e1);
  static unsigned long long h[4 * 256 * 16];
  hipMemcpy(h, t, 8 * 4 * blocks, hipMemcpyDeviceToHost);
  unsigned long long mc = 0;
  for (int i = 0; i < 4 * blocks; ++i) mc = h[i] > mc ? h[i] : mc;
  const double strings = (double)blocks * 256 * kIters;
  // per SIMD: wg_per_cu waves x kIters x 64 strings
  printf("%-12s W=%d  %.1f ms  %.3g strings/s  %.2f memtime cycles per (wave, string-row)\n", name, wg_per_cu, ms,
         strings / (ms * 1e-3), (double)mc / ((double)kIters * wg_per_cu));
  hipFree(out);
  hipFree(t);
}

int main() {
  uint64_t hp5[256];
  for (int b = 0; b < 256; ++b) hp5[b] = (uint64_t)b * XP5;
  uint64_t* p5;
  hipMalloc(&p5, sizeof hp5);
  hipMemcpy(p5, hp5, sizeof hp5, hipMemcpyHostToDevice);
  for (int W : {1, 2, 4, 6, 8}) {
    run<9>("gen_only", W, p5);
    run<0>("hash2+tail", W, p5);
    run<1>("hash3+tail", W, p5);
  }
  return 0;
}
