// rates.hip -- VALU issue rates of the integer ops XXH64 is built from, on gfx950 (diagnostic only).
// Build: hipcc --offload-arch=gfx950 -O3 tools/rates.hip -o tools/rates.bin
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x
template <int OP>
__global__ __launch_bounds__(256) void k(unsigned* out, unsigned seed) {
  unsigned a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  unsigned c = seed | 1;
  for (int it = 0; it < 256; ++it) {
    if (OP == 0) {  // v_mul_lo_u32
      REP8(asm volatile("v_mul_lo_u32 %0, %0, %8\n v_mul_lo_u32 %1, %1, %8\n v_mul_lo_u32 %2, %2, %8\n v_mul_lo_u32 %3, %3, %8\n"
                        "v_mul_lo_u32 %4, %4, %8\n v_mul_lo_u32 %5, %5, %8\n v_mul_lo_u32 %6, %6, %8\n v_mul_lo_u32 %7, %7, %8"
                        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(c));)
    } else if (OP == 1) {  // v_mul_hi_u32
      REP8(asm volatile("v_mul_hi_u32 %0, %0, %8\n v_mul_hi_u32 %1, %1, %8\n v_mul_hi_u32 %2, %2, %8\n v_mul_hi_u32 %3, %3, %8\n"
                        "v_mul_hi_u32 %4, %4, %8\n v_mul_hi_u32 %5, %5, %8\n v_mul_hi_u32 %6, %6, %8\n v_mul_hi_u32 %7, %7, %8"
                        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(c));)
    } else if (OP == 2) {  // v_mul_u32_u24
      REP8(asm volatile("v_mul_u32_u24 %0, %0, %8\n v_mul_u32_u24 %1, %1, %8\n v_mul_u32_u24 %2, %2, %8\n v_mul_u32_u24 %3, %3, %8\n"
                        "v_mul_u32_u24 %4, %4, %8\n v_mul_u32_u24 %5, %5, %8\n v_mul_u32_u24 %6, %6, %8\n v_mul_u32_u24 %7, %7, %8"
                        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(c));)
    } else if (OP == 3) {  // v_xor_b32
      REP8(asm volatile("v_xor_b32 %0, %8, %0\n v_xor_b32 %1, %8, %1\n v_xor_b32 %2, %8, %2\n v_xor_b32 %3, %8, %3\n"
                        "v_xor_b32 %4, %8, %4\n v_xor_b32 %5, %8, %5\n v_xor_b32 %6, %8, %6\n v_xor_b32 %7, %8, %7"
                        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(c));)
    } else if (OP == 4) {  // v_alignbit_b32
      REP8(asm volatile("v_alignbit_b32 %0, %0, %1, 7\n v_alignbit_b32 %1, %1, %2, 7\n v_alignbit_b32 %2, %2, %3, 7\n v_alignbit_b32 %3, %3, %4, 7\n"
                        "v_alignbit_b32 %4, %4, %5, 7\n v_alignbit_b32 %5, %5, %6, 7\n v_alignbit_b32 %6, %6, %7, 7\n v_alignbit_b32 %7, %7, %0, 7"
                        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(c));)
    } else if (OP == 5) {  // v_mad_u64_u32 (4 independent 64-bit accumulators)
      unsigned long long x0 = a0, x1 = a1, x2 = a2, x3 = a3;
      REP8(asm volatile("v_mad_u64_u32 %0, vcc, %4, %8, %0\n v_mad_u64_u32 %1, vcc, %5, %8, %1\n v_mad_u64_u32 %2, vcc, %6, %8, %2\n v_mad_u64_u32 %3, vcc, %7, %8, %3\n"
                        "v_mad_u64_u32 %0, vcc, %4, %8, %0\n v_mad_u64_u32 %1, vcc, %5, %8, %1\n v_mad_u64_u32 %2, vcc, %6, %8, %2\n v_mad_u64_u32 %3, vcc, %7, %8, %3"
                        : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(a4), "v"(a5), "v"(a6), "v"(a7), "s"(c) : "vcc");)
      a0 = (unsigned)x0 ^ (unsigned)(x1 >> 7) ^ (unsigned)x2 ^ (unsigned)x3;
    } else if (OP == 6) {  // v_fma_f64
      double d0 = a0, d1 = a1, d2 = a2, d3 = a3, e = 1.0000001;
      REP8(asm volatile("v_fma_f64 %0, %0, %4, %4\n v_fma_f64 %1, %1, %4, %4\n v_fma_f64 %2, %2, %4, %4\n v_fma_f64 %3, %3, %4, %4\n"
                        "v_fma_f64 %0, %0, %4, %4\n v_fma_f64 %1, %1, %4, %4\n v_fma_f64 %2, %2, %4, %4\n v_fma_f64 %3, %3, %4, %4"
                        : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3) : "v"(e));)
      a0 = (unsigned)(d0 + d1 + d2 + d3);
    } else if (OP == 7) {  // v_lshl_add_u64
      unsigned long long x0 = a0, x1 = a1, x2 = a2, x3 = a3, y = a4;
      REP8(asm volatile("v_lshl_add_u64 %0, %0, 1, %4\n v_lshl_add_u64 %1, %1, 1, %4\n v_lshl_add_u64 %2, %2, 1, %4\n v_lshl_add_u64 %3, %3, 1, %4\n"
                        "v_lshl_add_u64 %0, %0, 1, %4\n v_lshl_add_u64 %1, %1, 1, %4\n v_lshl_add_u64 %2, %2, 1, %4\n v_lshl_add_u64 %3, %3, 1, %4"
                        : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(y));)
      a0 = (unsigned)(x0 ^ x1 ^ x2 ^ x3);
    }
  }
  unsigned r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (r == 0x12345678u) out[0] = r;
}

template <int OP>
void run(const char* name, unsigned* out) {
  const int grid = 256 * 8 * 4;  // 8 waves/SIMD worth
  hipLaunchKernelGGL(k<OP>, dim3(grid), dim3(256), 0, 0, out, 3u);
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  (void)hipEventRecord(a);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(k<OP>, dim3(grid), dim3(256), 0, 0, out, 3u);
  (void)hipEventRecord(b); (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b); ms /= 5;
  const double wave_instr = (double)grid * 4 * 256 * 64;  // waves * iterations * instr per iteration
  int dev; hipDeviceProp_t p; (void)hipGetDevice(&dev); (void)hipGetDeviceProperties(&p, dev);
  const double cyc = (double)p.clockRate * 1e3 * (ms / 1e3) * p.multiProcessorCount * 4;  // SIMD-cycles
  std::printf("{\"op\": \"%s\", \"ms\": %.3f, \"simd_cycles_per_wave_instr\": %.2f, \"clock_mhz\": %d, \"cus\": %d}\n", name, ms,
              cyc / wave_instr, p.clockRate / 1000, p.multiProcessorCount);
}

int main() {
  unsigned* out; (void)hipMalloc(&out, 4);
  run<3>("v_xor_b32", out);
  run<4>("v_alignbit_b32", out);
  run<0>("v_mul_lo_u32", out);
  run<1>("v_mul_hi_u32", out);
  run<2>("v_mul_u32_u24", out);
  run<5>("v_mad_u64_u32", out);
  run<6>("v_fma_f64", out);
  run<7>("v_lshl_add_u64", out);
  return 0;
}
