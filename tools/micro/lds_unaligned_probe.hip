// lds_unaligned_probe.hip -- ds_read_b128 at byte-aligned addresses on gfx950 (diagnostic, not product).
//
// The UTF8 pass realigns each string's 32-byte window with 7 v_alignbyte per string; staged in LDS, a lane
// could read its string at its own byte offset instead (LLVM emits ds_read_b128 for an align-1 LDS access on
// gfx950: unaligned DS access mode).  This measures whether that read is exact and what it costs next to the
// 16-byte-aligned read: W waves per SIMD, every lane reading 2 x 16 bytes at (row offsets like C5's strings)
// + its byte shift, 4096 iterations, cycles per wave-instruction from s_memtime.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/lds_unaligned_probe.hip -o /tmp/lds_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kIters = 4096;

template <int MODE>  // 0: 16-byte aligned addresses, 1: byte addresses (string starts), 2: MODE 1 + alignbyte path
__global__ __launch_bounds__(256) void probe(uint32_t* out, unsigned long long* t, int* bad) {
  __shared__ __attribute__((aligned(16))) unsigned char buf[4 * 2304];
  unsigned char* mine = buf + (threadIdx.x >> 6) * 2304;
  for (int i = threadIdx.x & 63; i < 2304; i += 64) mine[i] = (unsigned char)(i * 7 + 3);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  uint32_t acc = 0, x = 0x9E3779B9u * (lane + 1);
  const uint64_t c0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIters; ++it) {
    x = x * 1664525u + 1013904223u;
    // string starts as C5's: 16 bytes apart on average, 8..24 long -> lane l near byte 16 l (+ up to 7)
    const uint32_t off = (uint32_t)lane * 16u + (x >> 29);
    u32x4 a, c;
    if constexpr (MODE == 0) {
      const unsigned char* p = mine + (off & ~15u);
      a = *reinterpret_cast<const u32x4*>(p);
      c = *reinterpret_cast<const u32x4*>(p + 16);
    } else {
      __builtin_memcpy(&a, mine + off, 16);
      __builtin_memcpy(&c, mine + off + 16, 16);
    }
    acc += a.x ^ a.y ^ a.z ^ a.w ^ c.x ^ c.y ^ c.z ^ c.w;
    if (MODE == 1 && it == 0) {  // exactness: the bytes read equal the bytes written
      uint32_t want[8];
      for (int k = 0; k < 32; ++k) reinterpret_cast<unsigned char*>(want)[k] = (unsigned char)((off + k) * 7 + 3);
      const uint32_t got[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
      for (int k = 0; k < 8; ++k)
        if (got[k] != want[k]) atomicAdd(bad, 1);
    }
  }
  const uint64_t c1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 256 + threadIdx.x] = acc;
  if (lane == 0) t[blockIdx.x * 4 + (threadIdx.x >> 6)] = c1 - c0;
}

template <int MODE>
void run(const char* name, int wg_per_cu) {
  const int blocks = 256 * wg_per_cu;
  uint32_t* out;
  unsigned long long* t;
  int* bad;
  hipMalloc(&out, 4 * 256 * blocks);
  hipMalloc(&t, 8 * 4 * blocks);
  hipMalloc(&bad, 4);
  hipMemset(bad, 0, 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float ms = 0;
  for (int r = 0; r < 2; ++r) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(256), 0, 0, out, t, bad);
    hipEventRecord(e1);
    hipDeviceSynchronize();
  }
  hipEventElapsedTime(&ms, e0, e1);
  static unsigned long long h[4 * 256 * 16];
  hipMemcpy(h, t, 8 * 4 * blocks, hipMemcpyDeviceToHost);
  int nbad = 0;
  hipMemcpy(&nbad, bad, 4, hipMemcpyDeviceToHost);
  unsigned long long mc = 0;
  for (int i = 0; i < 4 * blocks; ++i) mc = h[i] > mc ? h[i] : mc;
  // per CU: 4 * wg_per_cu waves x kIters x 2 reads
  printf("%-10s W=%d  %.3f ms  %.2f CU cycles per wave-read (memtime)  mismatches %d\n", name, wg_per_cu, ms,
         (double)mc / ((double)kIters * 2 * 4 * wg_per_cu), nbad);
  hipFree(out);
  hipFree(t);
  hipFree(bad);
}

int main() {
  for (int W : {2, 4, 6}) {
    run<0>("aligned", W);
    run<1>("unaligned", W);
  }
  return 0;
}
