// dq_hash.h -- XXH64 as used by Spark's XxHash64Function (seed 42), host + device.
// Reference call site: analyzers/catalyst/StatefulHyperloglogPlus.scala:93.  Included by the
// kernels and by tests/hash_check.cpp (host build) so the device formulation is checked on the CPU.
#pragma once

#include <cstdint>

#if defined(__HIPCC__) || defined(__HIP__)
#define DQ_HD __host__ __device__ __forceinline__
#else
#define DQ_HD inline
#endif

namespace dq {

DQ_HD uint32_t alignbit32(uint32_t hi, uint32_t lo, uint32_t sh) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(hi, lo, sh);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (sh & 31));
#endif
}

constexpr uint64_t XP1 = 0x9E3779B185EBCA87ull;
constexpr uint64_t XP2 = 0xC2B2AE3D27D4EB4Full;
constexpr uint64_t XP3 = 0x165667B19E3779F9ull;
constexpr uint64_t XP4 = 0x85EBCA77C2B2AE63ull;
constexpr uint64_t XP5 = 0x27D4EB2F165667C5ull;
constexpr uint64_t kSeed = 42;

// 64-bit rotate by a constant 0 < r < 32.  On the device it is two v_alignbit_b32 on the halves:
// written as 64-bit shifts, LLVM folds `rotl(x * P, r)` into extra multiplies by P << r.
DQ_HD uint64_t rotl64(uint64_t x, int r) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  const uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, 32 - r);
  const uint32_t nlo = __builtin_amdgcn_alignbit(lo, hi, 32 - r);
  return ((uint64_t)nhi << 32) | nlo;
#else
  return (x << r) | (x >> (64 - r));
#endif
}
DQ_HD uint64_t fmix64(uint64_t h) {
  h ^= h >> 33; h *= XP2; h ^= h >> 29; h *= XP3; h ^= h >> 32; return h;
}
DQ_HD uint64_t xxh64_long(uint64_t v) {
  uint64_t h = kSeed + XP5 + 8;
  h ^= rotl64(v * XP2, 31) * XP1;
  h = rotl64(h, 27) * XP1 + XP4;
  return fmix64(h);
}
DQ_HD uint64_t xxh64_int(uint32_t v) {
  uint64_t h = kSeed + XP5 + 4;
  h ^= (uint64_t)v * XP1;
  h = rotl64(h, 23) * XP2 + XP3;
  return fmix64(h);
}

// XXH64.hashUnsafeBytes of a string of len <= 28 bytes held in w[0..6] (little-endian dwords of the
// string itself).  Branch-free: every lane runs 3 stripe rounds, one 4-byte round and 3 byte rounds
// and keeps the ones its length needs, so a wave of mixed lengths does not diverge.  The 4-byte
// round's dword w[2 nw] and the byte rounds' dword w[len >> 2] = w[2 nw + (len >> 2 & 1)] are
// picked up by the same predicates as the stripe rounds (no dynamic register indexing).
DQ_HD uint64_t xxh64_short(const uint32_t (&w)[7], uint32_t len) {
  uint64_t h = kSeed + XP5 + (uint64_t)len;
  const uint32_t nw = len >> 3;
  uint32_t d4 = w[0], d4n = w[1];  // w[2 nw], w[2 nw + 1] after the stripe rounds
#pragma unroll
  for (uint32_t k = 0; k < 3; ++k) {
    const uint64_t k1 = ((uint64_t)w[2 * k + 1] << 32) | w[2 * k];
    uint64_t hn = h ^ (rotl64(k1 * XP2, 31) * XP1);
    hn = rotl64(hn, 27) * XP1 + XP4;
    const bool take = k < nw;
    h = take ? hn : h;
    d4 = take ? w[2 * k + 2] : d4;
    d4n = take ? (k < 2 ? w[2 * k + 3] : 0u) : d4n;  // w[7] only for len 28, which has no byte rounds
  }
  // 4-byte round on dword 2 nw
  const bool has4 = (len & 4u) != 0;
  uint64_t h4 = h ^ ((uint64_t)d4 * XP1);
  h4 = rotl64(h4, 23) * XP2 + XP3;
  h = has4 ? h4 : h;
  // byte rounds on dword len >> 2
  const uint32_t db = has4 ? d4n : d4;
  const uint32_t nb = len & 3u;
#pragma unroll
  for (uint32_t j = 0; j < 3; ++j) {
    const uint64_t b = (db >> (8 * j)) & 0xFFu;
    uint64_t hb = h ^ (b * XP5);
    hb = rotl64(hb, 11) * XP1;
    h = j < nb ? hb : h;
  }
  return fmix64(h);
}


}  // namespace dq
