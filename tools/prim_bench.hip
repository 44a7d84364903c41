// prim_bench.hip -- A/B timing of the hand-written radix sort (deequ_amd/csrc/dq_prim.hip) against hipCUB's
// DeviceRadixSort on the same device-generated keys (diagnostic only; hipCUB is not in the product).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -c tools/prim_bench.hip -o /tmp/pb.o && hipcc --offload-arch=gfx950 /tmp/pb.o deequ_amd/build/dq_prim.o -o tools/prim_bench.bin
// Run:   tools/prim_bench.bin [n]
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../deequ_amd/csrc/dq_prim.h"

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

__global__ void gen(uint64_t* k, uint64_t* v, int64_t n, int bits, uint64_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    k[i] = bits >= 64 ? z : (z & ((1ull << bits) - 1));
    v[i] = (uint64_t)i;
  }
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? std::atoll(argv[1]) : 100000000;
  uint64_t *k, *v, *ko, *vo, *ko2, *vo2;
  CK(hipMalloc(&k, n * 8));
  CK(hipMalloc(&v, n * 8));
  CK(hipMalloc(&ko, n * 8));
  CK(hipMalloc(&vo, n * 8));
  CK(hipMalloc(&ko2, n * 8));
  CK(hipMalloc(&vo2, n * 8));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  struct Case { int bits; int vb; };
  const Case cases[] = {{64, 8}, {64, 0}, {27, 8}, {27, 0}, {20, 4}};
  for (const Case& c : cases) {
    hipLaunchKernelGGL(gen, dim3(4096), dim3(256), 0, 0, k, v, n, c.bits, 42ull);
    CK(hipDeviceSynchronize());
    size_t tb_cub = 0;
    if (c.vb == 8)
      CK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb_cub, k, ko2, v, vo2, (int)n, 0, c.bits));
    else if (c.vb == 4)
      CK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb_cub, k, ko2, (const uint32_t*)v, (uint32_t*)vo2, (int)n, 0, c.bits));
    else
      CK(hipcub::DeviceRadixSort::SortKeys(nullptr, tb_cub, k, ko2, (int)n, 0, c.bits));
    const size_t tb_own = dq::prim::sort_temp_bytes(n, c.vb);
    void *t_cub, *t_own;
    CK(hipMalloc(&t_cub, tb_cub));
    CK(hipMalloc(&t_own, tb_own));
    float ms_cub = 1e30f, ms_own = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipEventRecord(a, 0));
      if (c.vb == 8)
        CK(hipcub::DeviceRadixSort::SortPairs(t_cub, tb_cub, k, ko2, v, vo2, (int)n, 0, c.bits));
      else if (c.vb == 4)
        CK(hipcub::DeviceRadixSort::SortPairs(t_cub, tb_cub, k, ko2, (const uint32_t*)v, (uint32_t*)vo2, (int)n, 0, c.bits));
      else
        CK(hipcub::DeviceRadixSort::SortKeys(t_cub, tb_cub, k, ko2, (int)n, 0, c.bits));
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      ms_cub = std::min(ms_cub, ms);
      CK(hipEventRecord(a, 0));
      CK(dq::prim::sort_pairs(k, ko, c.vb ? v : nullptr, c.vb ? vo : nullptr, c.vb, n, 0, c.bits, false, t_own, tb_own, 0));
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      ms_own = std::min(ms_own, ms);
    }
    // results identical (both stable)
    std::vector<uint64_t> h1(n), h2(n);
    CK(hipMemcpy(h1.data(), ko, n * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), ko2, n * 8, hipMemcpyDeviceToHost));
    bool same = h1 == h2;
    if (c.vb) {
      CK(hipMemcpy(h1.data(), vo, n * c.vb, hipMemcpyDeviceToHost));
      CK(hipMemcpy(h2.data(), vo2, n * c.vb, hipMemcpyDeviceToHost));
      same = same && std::equal(h1.begin(), h1.begin() + n * c.vb / 8, h2.begin());
    }
    std::printf("n %lld bits %d vb %d: hipcub %.3f ms, dq_prim %.3f ms (%.2fx), identical %d\n", (long long)n, c.bits,
                c.vb, ms_cub, ms_own, ms_own / ms_cub, (int)same);
    std::fflush(stdout);
    CK(hipFree(t_cub));
    CK(hipFree(t_own));
  }
  return 0;
}
