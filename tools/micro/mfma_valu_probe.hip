// Micro-benchmark: does v_mfma_f64_16x16x4_f64 overlap with VALU work on gfx950?  Every CU runs 4 * wps
// waves (wps per SIMD); each wave loops `iters` steps of: M dependent f64 MFMAs + F independent v_fma_f64
// + B independent 32-bit VALU ops.  Reported: the slowest wave's clock64 cycles per step divided by the
// steps every SIMD executes (wps per step) = SIMD cycles per (wave-)step.  Waves with role = 1 (odd waves,
// when SPLIT) run only the VALU part, role 0 only the MFMA part.
// Build: hipcc --offload-arch=gfx950 -O3 tools/micro/mfma_valu_probe.hip -o tools/micro/mfma_valu_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int M, int F, int B, bool SPLIT>
__global__ void k(double* out, int iters, long long* cyc) {
  d4 acc = {0, 0, 0, 0};
  double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
  double f[16];
  unsigned u[16];
  for (int i = 0; i < 16; ++i) { f[i] = a * (i + 1); u[i] = threadIdx.x * (i + 3); }
  const int wave = threadIdx.x >> 6;
  const bool do_m = !SPLIT || (wave & 1) == 0, do_v = !SPLIT || (wave & 1) == 1;
  long long c0 = clock64();
  for (int i = 0; i < iters; ++i) {
    if (do_m) {
#pragma unroll
      for (int j = 0; j < M; ++j) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    }
    if (do_v) {
#pragma unroll
      for (int j = 0; j < F; ++j) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(f[j & 15]) : "v"(a), "v"(b));
#pragma unroll
      for (int j = 0; j < B; ++j) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(u[j & 15]) : "v"(wave));
    }
  }
  long long c1 = clock64();
  double s = acc[0] + acc[1] + acc[2] + acc[3];
  for (int i = 0; i < 16; ++i) s += f[i] + u[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + wave] = c1 - c0;
}

template <int M, int F, int B, bool SPLIT = false>
void run(int wps) {
  double* out; long long* cyc;
  const int blocks = 256, threads = 256 * wps, nw = blocks * threads / 64;
  hipMalloc(&out, sizeof(double) * threads * blocks);
  hipMalloc(&cyc, 8 * nw);
  const int iters = 2048;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL((k<M, F, B, SPLIT>), dim3(blocks), dim3(threads), 0, 0, out, iters, cyc);
    hipDeviceSynchronize();
  }
  long long h[4096]; hipMemcpy(h, cyc, 8 * nw, hipMemcpyDeviceToHost);
  long long mx = 0;
  for (int i = 0; i < nw; ++i) mx = h[i] > mx ? h[i] : mx;
  printf("waves/SIMD %d  mfma %d  fma_f64 %2d  b32 %2d %s: %.1f SIMD cycles per wave-step\n", wps, M, F, B,
         SPLIT ? "(split roles)" : "             ", (double)mx / iters / wps);
  hipFree(out); hipFree(cyc);
}

int main() {
  for (int w = 1; w <= 4; w *= 2) {
    run<1, 0, 0>(w);
    run<0, 16, 0>(w);
    run<0, 0, 32>(w);
    run<1, 8, 0>(w);
    run<1, 16, 0>(w);
    run<1, 0, 16>(w);
    run<1, 4, 16>(w);
  }
  run<1, 16, 0, true>(2);
  run<1, 16, 0, true>(4);
  run<1, 4, 16, true>(4);
  return 0;
}
