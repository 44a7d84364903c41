// unaligned_test.hip -- do buffer_load_dword{,x2,x4} at byte-granular offsets return the bytes at that
// address on this GPU (SH_MEM_CONFIG unaligned mode)?  Diagnostic only; prints one JSON line.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void k(const uint8_t* data, int n, uint32_t* out) {
  const int off = threadIdx.x;  // 0..255 byte offsets
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(data), (short)0, n, 0x00020000);
  const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  const auto b = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
  const uint32_t c = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
  out[off * 7 + 0] = a.x; out[off * 7 + 1] = a.y; out[off * 7 + 2] = a.z; out[off * 7 + 3] = a.w;
  out[off * 7 + 4] = b[0]; out[off * 7 + 5] = b[1]; out[off * 7 + 6] = c;
}

int main() {
  const int n = 300;
  uint8_t h[n];
  for (int i = 0; i < n; ++i) h[i] = (uint8_t)(i * 37 + 11);
  uint8_t* d; uint32_t* o;
  (void)hipMalloc(&d, 512); (void)hipMalloc(&o, 256 * 7 * 4);
  (void)hipMemcpy(d, h, n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, d, n, o);
  uint32_t r[256 * 7];
  (void)hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost);
  int bad16 = 0, bad8 = 0, bad4 = 0, first_bad = -1;
  for (int off = 0; off < 256; ++off) {
    uint32_t e[4];
    for (int w = 0; w < 4; ++w) {
      uint32_t v = 0;
      for (int bb = 0; bb < 4; ++bb) { int i = off + 4 * w + bb; v |= (uint32_t)(i < n ? h[i] : 0) << (8 * bb); }
      e[w] = v;
    }
    if (off + 16 <= n && memcmp(e, &r[off * 7], 16)) { bad16++; if (first_bad < 0) first_bad = off; }
    if (off + 8 <= n && memcmp(e, &r[off * 7 + 4], 8)) bad8++;
    if (off + 4 <= n && e[0] != r[off * 7 + 6]) bad4++;
  }
  std::printf("{\"unaligned_b128_bad\": %d, \"b64_bad\": %d, \"b32_bad\": %d, \"first_bad_offset\": %d}\n", bad16, bad8, bad4, first_bad);
  return 0;
}
