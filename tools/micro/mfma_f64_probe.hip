// Micro-benchmark: cycles of v_mfma_f64_16x16x4_f64 on gfx950 (dependent chain vs independent accumulators,
// 1..4 waves per SIMD).  Build: hipcc --offload-arch=gfx950 -O3 tools/micro/mfma_f64_probe.hip -o /tmp/mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void chain(double* out, int iters, long long* cyc) {
  d4 acc[NACC];
  for (int k = 0; k < NACC; ++k) acc[k] = d4{0, 0, 0, 0};
  double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
  long long t0 = wall_clock64();
  long long c0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < NACC; ++k) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k], 0, 0, 0);
  }
  long long c1 = clock64();
  long long t1 = wall_clock64();
  double s = 0;
  for (int k = 0; k < NACC; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) { cyc[0] = c1 - c0; cyc[1] = t1 - t0; }
}

template <int NACC>
void run(int waves_per_block, int blocks) {
  double* out; long long* cyc;
  hipMalloc(&out, sizeof(double) * 64 * waves_per_block * blocks);
  hipMalloc(&cyc, 16);
  const int iters = 4096;
  hipLaunchKernelGGL(chain<NACC>, dim3(blocks), dim3(64 * waves_per_block), 0, 0, out, iters, cyc);
  hipDeviceSynchronize();
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(chain<NACC>, dim3(blocks), dim3(64 * waves_per_block), 0, 0, out, iters, cyc);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  long long h[2]; hipMemcpy(h, cyc, 16, hipMemcpyDeviceToHost);
  const double n_mfma = (double)iters * NACC;
  const double flops = n_mfma * 2048.0 * waves_per_block * blocks;
  printf("nacc=%d waves/block=%d blocks=%d: clock64 cycles per MFMA (wave 0) %.1f, wall %.3f ms, %.1f TFLOP/s\n", NACC,
         waves_per_block, blocks, h[0] / n_mfma, ms, flops / (ms * 1e-3) / 1e12);
  hipFree(out); hipFree(cyc);
}

int main() {
  run<1>(1, 1);
  run<4>(1, 1);
  run<1>(4, 1);    // 4 waves of one block: one per SIMD
  run<1>(8, 1);    // 2 per SIMD
  run<1>(16, 1);   // 4 per SIMD
  run<4>(4, 1);
  run<1>(4, 256 * 4);
  run<4>(4, 256 * 4);
  run<1>(16, 256 * 2);
  return 0;
}
