// dq_lane.h -- small gfx950 device helpers shared by the scan kernels (lane-per-row layouts: lane l of a
// wave holds row base + l, so the selection of 64 rows is one 64-bit scalar mask).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace dq {

// Hardware v_min_f64 / v_max_f64 (IEEE mode: a NaN operand yields the other operand).  Inline asm
// keeps the compiler from canonicalising both inputs first (two extra v_max_f64 per call).
__device__ __forceinline__ double hw_min(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double hw_max(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// scalar (constant address space) loads: a bitmap word read with s_load into SGPRs
typedef const __attribute__((address_space(4))) uint32_t* const_u32s;

__device__ __forceinline__ uint64_t load_word64(const uint32_t* p, int64_t w) {
  return ((uint64_t)((const_u32s)p)[w + 1] << 32) | ((const_u32s)p)[w];
}

// this lane's bit of a wave-uniform 64-bit row mask (inverse ballot: no VALU work)
__device__ __forceinline__ bool lane_bit(uint64_t m) { return __builtin_amdgcn_inverse_ballot_w64(m); }

}  // namespace dq
