// issue_probe.hip -- VALU issue rate and dependent-chain latency on gfx950 (diagnostic, not product).
//
// For W waves per SIMD (256 CUs x 4 SIMDs x W waves, one 64-thread workgroup per wave) every wave runs C
// independent dependency chains of one instruction kind.  Reported: SIMD cycles per wave-instruction
// (s_memtime delta of the slowest wave / instructions per SIMD) and the shader clock measured against the
// constant 100 MHz s_memrealtime, so the numbers do not rest on an assumed clock.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/issue_probe.hip -o /tmp/issue_probe && /tmp/issue_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__device__ __forceinline__ uint64_t memtime() { return __builtin_amdgcn_s_memtime(); }
__device__ __forceinline__ uint64_t realtime() { return __builtin_amdgcn_s_memrealtime(); }

constexpr int kIters = 2048;

template <int C, int K>
__global__ __launch_bounds__(64) void probe(uint32_t* out, unsigned long long* t) {
  uint32_t u[C];
  uint64_t w[C];
#pragma unroll
  for (int i = 0; i < C; ++i) {
    u[i] = threadIdx.x * (i + 3) + 1;
    w[i] = (uint64_t)threadIdx.x * (i + 5) + 7;
  }
  const uint32_t k = 0x9E3779B1u, k2 = 0x85EBCA77u;
  __builtin_amdgcn_s_barrier();
  const uint64_t c0 = memtime(), r0 = realtime();
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int rep = 0; rep < 16 / C; ++rep) {
#pragma unroll
      for (int i = 0; i < C; ++i) {
        if constexpr (K == 0) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(u[i]) : "s"(k));
        if constexpr (K == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(u[i]) : "s"(k));
        if constexpr (K == 2) {
          uint64_t c;
          asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(w[i]), "=s"(c) : "v"((uint32_t)w[i]), "s"(k));
        }
        if constexpr (K == 3) asm volatile("v_alignbit_b32 %0, %0, %0, 5" : "+v"(u[i]));
        if constexpr (K == 4) asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(u[i]) : "s"(k));
        if constexpr (K == 5) asm volatile("v_add_f64 %0, %0, %0" : "+v"(w[i]));
        if constexpr (K == 6) {  // one XXH64 round-like step: 64-bit multiply (4) + rotate (2) = 6 instructions
          uint64_t p, c;
          uint32_t t1, t2, lo = (uint32_t)w[i], hi = (uint32_t)(w[i] >> 32);
          asm volatile(
              "v_mad_u64_u32 %[p], %[c], %[lo], %[k], 0\n\t"
              "v_mul_lo_u32 %[t1], %[lo], %[k2]\n\t"
              "v_mul_lo_u32 %[t2], %[hi], %[k]"
              : [p] "=&v"(p), [c] "=&s"(c), [t1] "=&v"(t1), [t2] "=&v"(t2)
              : [lo] "v"(lo), [hi] "v"(hi), [k] "s"(k), [k2] "s"(k2));
          asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(hi) : "v"(t1), "v"(t2), "v"((uint32_t)(p >> 32)));
          lo = (uint32_t)p;
          const uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, 5), nlo = __builtin_amdgcn_alignbit(lo, hi, 5);
          w[i] = ((uint64_t)nhi << 32) | nlo;
        }
      }
    }
  }
  const uint64_t c1 = memtime(), r1 = realtime();
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < C; ++i) s += u[i] + (uint32_t)w[i] + (uint32_t)(w[i] >> 32);
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    t[2 * blockIdx.x] = c1 - c0;
    t[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <int C, int K>
void run(const char* name, int insts_per_step, int waves_per_simd) {
  const int blocks = 256 * 4 * waves_per_simd;
  uint32_t* out;
  unsigned long long* t;
  hipMalloc(&out, 4 * 64 * blocks);
  hipMalloc(&t, 16 * blocks);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int r = 0; r < 2; ++r) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((probe<C, K>), dim3(blocks), dim3(64), 0, 0, out, t);
    hipEventRecord(e1);
    hipDeviceSynchronize();
  }
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  static unsigned long long h[2 * 256 * 4 * 16];
  hipMemcpy(h, t, 16 * blocks, hipMemcpyDeviceToHost);
  unsigned long long mc = 0, mr = 0;
  double clk = 0;
  for (int i = 0; i < blocks; ++i) {
    mc = h[2 * i] > mc ? h[2 * i] : mc;
    mr = h[2 * i + 1] > mr ? h[2 * i + 1] : mr;
    clk += (double)h[2 * i] / (double)h[2 * i + 1] * 100.0;  // MHz (realtime = 100 MHz)
  }
  clk /= blocks;
  const double insts = (double)kIters * 16 * insts_per_step;  // per wave
  // every SIMD runs waves_per_simd waves: cycles / (insts * waves) = SIMD cycles per wave-instruction
  const double wall_cyc = ms * 1e-3 * clk * 1e6;
  printf("%-10s C=%-2d W=%-2d  %.2f SIMD cyc/wave-inst (memtime), %.2f (wall x clock)  clock %.0f MHz  %.3f ms\n",
         name, C, waves_per_simd, (double)mc / (insts * waves_per_simd), wall_cyc / (insts * waves_per_simd),
         clk, ms);
  hipFree(out);
  hipFree(t);
}

int main() {
  for (int W : {1, 2, 4, 6, 8}) {
    run<16, 0>("xor", 1, W);
    run<1, 0>("xor", 1, W);
    run<16, 1>("mul_lo", 1, W);
    run<1, 1>("mul_lo", 1, W);
    run<16, 2>("mad_u64", 1, W);
    run<16, 3>("alignbit", 1, W);
    run<16, 4>("add3", 1, W);
    run<16, 5>("add_f64", 1, W);
    run<1, 6>("xxround", 6, W);
    run<2, 6>("xxround", 6, W);
    run<4, 6>("xxround", 6, W);
  }
  return 0;
}
