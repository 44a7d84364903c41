// Micro-benchmark: SIMD issue cost of single VALU instructions on gfx950 (4 waves per SIMD, 16
// independent chains per wave).  Build: hipcc --offload-arch=gfx950 -O3 tools/micro/valu_rate_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define BODY(NAME, ASM)                                                                       \
  __global__ void NAME(uint32_t* out, int iters, long long* cyc) {                             \
    uint32_t u[16];                                                                            \
    uint64_t w[8];                                                                             \
    for (int i = 0; i < 16; ++i) u[i] = threadIdx.x * (i + 3) + 1;                            \
    for (int i = 0; i < 8; ++i) w[i] = (uint64_t)threadIdx.x * (i + 5) + 7;                   \
    uint32_t k = 0x9E3779B1u;                                                                  \
    long long c0 = clock64();                                                                  \
    for (int i = 0; i < iters; ++i) {                                                          \
      _Pragma("unroll") for (int j = 0; j < 16; ++j) { ASM; }                                  \
    }                                                                                          \
    long long c1 = clock64();                                                                  \
    uint32_t s = 0;                                                                            \
    for (int i = 0; i < 16; ++i) s += u[i];                                                    \
    for (int i = 0; i < 8; ++i) s += (uint32_t)w[i];                                           \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                            \
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)] = c1 - c0; \
  }

BODY(k_xor, asm volatile("v_xor_b32 %0, %0, %1" : "+v"(u[j]) : "s"(k)))
BODY(k_add3, asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(u[j]) : "s"(k)))
BODY(k_alignbit, asm volatile("v_alignbit_b32 %0, %0, %0, 5" : "+v"(u[j])))
BODY(k_mul_lo, asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(u[j]) : "s"(k)))
BODY(k_mul_hi, asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(u[j]) : "s"(k)))
BODY(k_mul_u24, asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(u[j]) : "s"(k)))
BODY(k_mad_u64, { uint64_t c; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(w[j & 7]), "=s"(c) : "v"(u[j]), "s"(k)); })
BODY(k_mad_u32_u24, asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(u[j]) : "s"(k)))
BODY(k_lshl_add_u64, asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(w[j & 7]) : "v"(w[(j + 1) & 7])))
BODY(k_mov_b64, asm volatile("v_mov_b64 %0, %1" : "=v"(w[j & 7]) : "v"(w[(j + 3) & 7])))
BODY(k_cndmask, asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[j]) : "v"(u[(j + 1) & 15])))
BODY(k_bfe, asm volatile("v_bfe_u32 %0, %0, 3, 8" : "+v"(u[j])))
BODY(k_perm, asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(u[j]) : "v"(u[(j + 1) & 15]), "s"(k)))

// fp64 ops (the Correlation pass's operand prep): 8 independent 64-bit chains per wave
BODY(k_add_f64, asm volatile("v_add_f64 %0, %0, %1" : "+v"(w[j & 7]) : "v"(w[(j + 1) & 7])))
BODY(k_mul_f64, asm volatile("v_mul_f64 %0, %0, %1" : "+v"(w[j & 7]) : "v"(w[(j + 1) & 7])))
BODY(k_fma_f64, asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(w[j & 7]) : "v"(w[(j + 1) & 7])))
BODY(k_cvt_f64_u32, asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(w[j & 7]) : "v"(u[j])))

typedef void (*KF)(uint32_t*, int, long long*);
void run(const char* name, KF f, int wps = 4, int threads = 256) {
  uint32_t* out; long long* cyc;
  const int blocks = 256 * 4 * wps * 64 / threads, nw = blocks * threads / 64, iters = 1024;
  hipMalloc(&out, 4 * blocks * threads);
  hipMalloc(&cyc, 8 * nw);
  for (int r = 0; r < 2; ++r) { hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, out, iters, cyc); hipDeviceSynchronize(); }
  static long long h[65536];
  hipMemcpy(h, cyc, 8 * nw, hipMemcpyDeviceToHost);
  long long mx = 0;
  for (int i = 0; i < nw; ++i) mx = h[i] > mx ? h[i] : mx;
  printf("%-16s %.2f SIMD cycles per wave-instruction (%d waves/SIMD, %d-thread blocks)\n", name,
         (double)mx / (iters * 16.0 * wps), wps, threads);
  hipFree(out); hipFree(cyc);
}
int main() {
  run("v_xor_b32", k_xor, 1, 256); run("v_xor_b32", k_xor, 2, 256); run("v_xor_b32", k_xor, 4, 1024);
  run("v_xor_b32", k_xor, 8, 256); run("v_mul_lo_u32", k_mul_lo, 1, 256); run("v_mul_lo_u32", k_mul_lo, 8, 256);
  run("v_xor_b32", k_xor); run("v_add3_u32", k_add3); run("v_alignbit_b32", k_alignbit); run("v_mul_lo_u32", k_mul_lo);
  run("v_mul_hi_u32", k_mul_hi); run("v_mul_u32_u24", k_mul_u24); run("v_mad_u64_u32", k_mad_u64);
  run("v_mad_u32_u24", k_mad_u32_u24); run("v_lshl_add_u64", k_lshl_add_u64); run("v_mov_b64", k_mov_b64);
  run("v_cndmask_b32", k_cndmask); run("v_bfe_u32", k_bfe); run("v_perm_b32", k_perm);
  run("v_add_f64", k_add_f64); run("v_mul_f64", k_mul_f64); run("v_fma_f64", k_fma_f64);
  run("v_cvt_f64_u32", k_cvt_f64_u32); run("v_mul_f64", k_mul_f64, 2, 256); run("v_mul_f64", k_mul_f64, 8, 256);
  return 0;
}
