// Micro-benchmark: cost of VALU filler instructions placed between dependent v_mfma_f64_16x16x4_f64
// (one accumulator chain per wave), at 1..4 waves per SIMD.  Build:
//   hipcc --offload-arch=gfx950 -O3 tools/micro/mfma_valu_probe.hip -o tools/micro/mfma_valu_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NF64, int NB32>
__global__ void k(double* out, int iters, long long* cyc) {
  d4 acc = {0, 0, 0, 0};
  double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
  double f[8];
  unsigned u[8];
  for (int i = 0; i < 8; ++i) { f[i] = a * (i + 1); u[i] = threadIdx.x * (i + 3); }
  long long c0 = clock64();
  for (int i = 0; i < iters; ++i) {
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < NF64; ++j) asm volatile("v_add_f64 %0, %0, %1" : "+v"(f[j & 7]) : "v"(b));
#pragma unroll
    for (int j = 0; j < NB32; ++j) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(u[j & 7]) : "v"(i));
  }
  long long c1 = clock64();
  double s = acc[0] + acc[1] + acc[2] + acc[3];
  for (int i = 0; i < 8; ++i) s += f[i] + u[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = c1 - c0;
}

template <int NF64, int NB32>
void run(int wps) {  // waves per SIMD: one block of 4 * wps waves per CU, 256 blocks
  double* out; long long* cyc;
  const int blocks = 256, threads = 256 * wps;
  hipMalloc(&out, sizeof(double) * threads * blocks);
  hipMalloc(&cyc, 8);
  const int iters = 2048;
  hipLaunchKernelGGL((k<NF64, NB32>), dim3(blocks), dim3(threads), 0, 0, out, iters, cyc);
  hipDeviceSynchronize();
  hipLaunchKernelGGL((k<NF64, NB32>), dim3(blocks), dim3(threads), 0, 0, out, iters, cyc);
  hipDeviceSynchronize();
  long long h; hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
  printf("waves/SIMD %d  f64 adds %2d  b32 ops %2d : %.1f cycles per MFMA step per wave\n", wps, NF64, NB32,
         (double)h / iters);
  hipFree(out); hipFree(cyc);
}

int main() {
  for (int w = 1; w <= 4; w *= 2) {
    run<0, 0>(w);
    run<4, 0>(w);
    run<8, 0>(w);
    run<16, 0>(w);
    run<0, 8>(w);
    run<0, 16>(w);
    run<0, 32>(w);
    run<2, 14>(w);
  }
  return 0;
}
