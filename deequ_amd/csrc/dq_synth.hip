// dq_synth.hip -- seeded synthetic column generators for tests and bench.py (NOT the product path).
//
// Counter-based: every value is a pure function of (seed, row), so any chunk or shard can be
// regenerated independently and compared with the CPU oracle.  Distributions follow SURVEY §8d:
//   f64  : N(mean, sd)                                     (C2 / C5 fp64 columns)
//   corr : a*z0 + b*zc + offset, z ~ N(0,1)                 (C4 correlated columns)
//   i64  : uniform over [0, D)                             (C3 / C5 int64 columns)
//   utf8 : length uniform in [lmin, lmax], content a function of an id uniform over [0, D)
//   validity: each row null with probability null_frac
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t x) {  // splitmix64 finaliser
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__device__ __forceinline__ uint64_t rnd(uint64_t seed, uint64_t stream, int64_t i) {
  return mix64(mix64(seed * 0x100000001B3ull + stream) ^ (uint64_t)i);
}
__device__ __forceinline__ double u01(uint64_t r) { return ((r >> 11) + 0.5) * (1.0 / 9007199254740992.0); }
__device__ __forceinline__ double normal(uint64_t seed, uint64_t stream, int64_t i) {
  double u1 = u01(rnd(seed, stream, i)), u2 = u01(rnd(seed, stream ^ 0x5555, i));
  return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}

__global__ void k_f64(double* out, int64_t row0, int64_t n, uint64_t seed, double mean, double sd) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = mean + sd * normal(seed, 1, row0 + i);
}

__global__ void k_corr(double* out, int64_t row0, int64_t n, uint64_t seed, uint64_t col_seed, double a, double b,
                       double offset) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = a * normal(seed, 7, row0 + i) + b * normal(col_seed, 9, row0 + i) + offset;
}

__global__ void k_i64(int64_t* out, int64_t row0, int64_t n, uint64_t seed, uint64_t distinct, int64_t base) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t r = rnd(seed, 3, row0 + i);
    out[i] = base + (int64_t)(distinct ? r % distinct : r);
  }
}

// validity: one thread per 32-row word; row0 must be a multiple of 32
__global__ void k_validity(uint32_t* out, int64_t row0, int64_t n, uint64_t seed, double null_frac) {
  const int64_t words = (n + 31) / 32;
  const uint64_t thr = null_frac >= 1.0 ? ~0ull : (null_frac <= 0.0 ? 0ull : (uint64_t)(null_frac * 18446744073709551616.0));
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < words; w += (int64_t)gridDim.x * blockDim.x) {
    uint32_t bits = 0;
    for (int j = 0; j < 32; ++j) {
      int64_t i = w * 32 + j;
      if (i < n && rnd(seed, 11, row0 + i) >= thr) bits |= 1u << j;
    }
    out[w] = bits;
  }
}

__device__ __forceinline__ uint64_t str_id(uint64_t seed, int64_t row, uint64_t distinct) {
  uint64_t r = rnd(seed, 5, row);
  return distinct ? r % distinct : r;
}
__device__ __forceinline__ int32_t str_len(uint64_t seed, uint64_t id, int32_t lmin, int32_t lmax) {
  return lmin + (int32_t)(mix64(id ^ (seed << 1)) % (uint64_t)(lmax - lmin + 1));
}

__global__ void k_utf8_lengths(int64_t* lens, int64_t row0, int64_t n, uint64_t seed, uint64_t distinct, int32_t lmin,
                               int32_t lmax) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    lens[i] = str_len(seed, str_id(seed, row0 + i, distinct), lmin, lmax);
}

// bytes: printable ASCII, a function of the id only (equal ids -> equal strings)
__global__ void k_utf8_bytes(uint8_t* data, const int64_t* offs64, int64_t row0, int64_t n, uint64_t seed,
                             uint64_t distinct) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t id = str_id(seed, row0 + i, distinct);
    int64_t o0 = offs64[i], o1 = offs64[i + 1];
    uint64_t h = mix64(id * 0x2545F4914F6CDD1Dull + seed);
    for (int64_t p = o0; p < o1; ++p) {
      data[p] = (uint8_t)(33 + (h % 94));
      h = mix64(h + (uint64_t)p - (uint64_t)o0);
    }
  }
}

__global__ void k_i64_to_i32(int32_t* dst, const int64_t* src, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = (int32_t)src[i];
}

inline dim3 grid_for(int64_t n) {
  int64_t g = (n + 255) / 256;
  if (g > 65536) g = 65536;
  if (g < 1) g = 1;
  return dim3((unsigned)g);
}

}  // namespace

extern "C" {

int dqs_f64(void* out, int64_t row0, int64_t n, uint64_t seed, double mean, double sd, void* stream) {
  hipLaunchKernelGGL(k_f64, grid_for(n), dim3(256), 0, (hipStream_t)stream, (double*)out, row0, n, seed, mean, sd);
  return (int)hipGetLastError();
}
int dqs_corr(void* out, int64_t row0, int64_t n, uint64_t seed, uint64_t col_seed, double a, double b, double offset,
             void* stream) {
  hipLaunchKernelGGL(k_corr, grid_for(n), dim3(256), 0, (hipStream_t)stream, (double*)out, row0, n, seed, col_seed, a,
                     b, offset);
  return (int)hipGetLastError();
}
int dqs_i64(void* out, int64_t row0, int64_t n, uint64_t seed, uint64_t distinct, int64_t base, void* stream) {
  hipLaunchKernelGGL(k_i64, grid_for(n), dim3(256), 0, (hipStream_t)stream, (int64_t*)out, row0, n, seed, distinct, base);
  return (int)hipGetLastError();
}
int dqs_validity(void* out, int64_t row0, int64_t n, uint64_t seed, double null_frac, void* stream) {
  hipLaunchKernelGGL(k_validity, grid_for((n + 31) / 32), dim3(256), 0, (hipStream_t)stream, (uint32_t*)out, row0, n,
                     seed, null_frac);
  return (int)hipGetLastError();
}
int dqs_utf8_lengths(void* lens, int64_t row0, int64_t n, uint64_t seed, uint64_t distinct, int32_t lmin, int32_t lmax,
                     void* stream) {
  hipLaunchKernelGGL(k_utf8_lengths, grid_for(n), dim3(256), 0, (hipStream_t)stream, (int64_t*)lens, row0, n, seed,
                     distinct, lmin, lmax);
  return (int)hipGetLastError();
}
int dqs_utf8_bytes(void* data, const void* offs64, int64_t row0, int64_t n, uint64_t seed, uint64_t distinct,
                   void* stream) {
  hipLaunchKernelGGL(k_utf8_bytes, grid_for(n), dim3(256), 0, (hipStream_t)stream, (uint8_t*)data,
                     (const int64_t*)offs64, row0, n, seed, distinct);
  return (int)hipGetLastError();
}
int dqs_i64_to_i32(void* dst, const void* src, int64_t n, void* stream) {
  hipLaunchKernelGGL(k_i64_to_i32, grid_for(n), dim3(256), 0, (hipStream_t)stream, (int32_t*)dst, (const int64_t*)src, n);
  return (int)hipGetLastError();
}

}  // extern "C"
