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
// x * c + a (mod 2^64) for constants c, a, written so the device code is one v_mad_u64_u32 (low
// product + addend), two v_mul_lo_u32 (cross products) and one add3.
DQ_HD uint64_t mul_add_c(uint64_t x, uint64_t c, uint64_t a) {
  const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
#if defined(__HIP_DEVICE_COMPILE__)
  // The three multiplies are pinned in asm: left to itself LLVM re-associates the cross products
  // into extra v_mad_u64_u32 + v_mov chains (up to 7 instructions).  The addend is a VGPR pair (a
  // loop-invariant constant; the VOP3 constant bus takes only the SGPR multiplier).
  uint64_t p, carry;
  uint32_t t1, t2;
  asm("v_mad_u64_u32 %[p], %[cy], %[xl], %[cl], %[a]\n\t"
      "v_mul_lo_u32 %[t1], %[xl], %[ch]\n\t"
      "v_mul_lo_u32 %[t2], %[xh], %[cl]"
      : [p] "=&v"(p), [cy] "=&s"(carry), [t1] "=&v"(t1), [t2] "=&v"(t2)
      : [xl] "v"(xl), [xh] "v"(xh), [cl] "s"((uint32_t)c), [ch] "s"((uint32_t)(c >> 32)), [a] "v"(a));
  (void)carry;
  const uint32_t hi = (uint32_t)(p >> 32) + t1 + t2;
#else
  const uint64_t p = (uint64_t)xl * (uint32_t)c + a;
  const uint32_t hi = (uint32_t)(p >> 32) + xl * (uint32_t)(c >> 32) + xh * (uint32_t)c;
#endif
  return ((uint64_t)hi << 32) | (uint32_t)p;
}

// x * c (mod 2^64) for a 32-bit x: one v_mad_u64_u32, one v_mul_lo_u32, one add.
DQ_HD uint64_t mul32_c(uint32_t x, uint64_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t p, carry;
  uint32_t t;
  asm("v_mad_u64_u32 %[p], %[cy], %[x], %[cl], 0\n\t"
      "v_mul_lo_u32 %[t], %[x], %[ch]"
      : [p] "=&v"(p), [cy] "=&s"(carry), [t] "=&v"(t)
      : [x] "v"(x), [cl] "s"((uint32_t)c), [ch] "s"((uint32_t)(c >> 32)));
  (void)carry;
  return ((uint64_t)((uint32_t)(p >> 32) + t) << 32) | (uint32_t)p;
#else
  return (uint64_t)x * c;
#endif
}

// fmix64 split in two: fmix_head(h) is the state before the last multiply; the final hash is
// fmix_tail(fmix_head(h)).  The HLL kernels only need the high word of fmix_tail, hi32(b * P3).
DQ_HD uint64_t fmix_head(uint64_t h) {
  h ^= h >> 33;
  h = mul_add_c(h, XP2, 0);
  return h ^ (h >> 29);
}
DQ_HD uint64_t fmix_tail(uint64_t b) {
  const uint64_t h = b * XP3;
  return h ^ (h >> 32);
}
DQ_HD uint64_t fmix64(uint64_t h) { return fmix_tail(fmix_head(h)); }

// XXH64.hashLong / hashInt (seed 42) up to fmix_head
DQ_HD uint64_t xxh64_long_head(uint64_t v) {
  const uint64_t k = rotl64(mul_add_c(v, XP2, 0), 31);
  const uint64_t h = mul_add_c(k, XP1, 0) ^ (kSeed + XP5 + 8);
  return fmix_head(mul_add_c(rotl64(h, 27), XP1, XP4));
}
DQ_HD uint64_t xxh64_int_head(uint32_t v) {
  const uint64_t h = mul32_c(v, XP1) ^ (kSeed + XP5 + 4);
  return fmix_head(mul_add_c(rotl64(h, 23), XP2, XP3));
}
DQ_HD uint64_t xxh64_long(uint64_t v) { return fmix_tail(xxh64_long_head(v)); }
DQ_HD uint64_t xxh64_int(uint32_t v) { return fmix_tail(xxh64_int_head(v)); }

// Predicated 64-bit move dst = cond ? src : dst.  On the device it is one exec-masked v_mov_b64
// (s_and_saveexec / s_mov exec around it) instead of two v_cndmask_b32.
#if defined(__HIP_DEVICE_COMPILE__) && defined(DQ_SEL64_CNDMASK)
__device__ __forceinline__ void sel64(uint64_t& dst, uint64_t src, bool cond) { dst = cond ? src : dst; }
#elif defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ void sel64(uint64_t& dst, uint64_t src, bool cond) {
  uint64_t save;
  asm("s_and_saveexec_b64 %[s], %[m]\n\t"
      "v_mov_b64 %[d], %[x]\n\t"
      "s_mov_b64 exec, %[s]"
      : [d] "+v"(dst), [s] "=&s"(save)
      : [x] "v"(src), [m] "s"(__builtin_amdgcn_ballot_w64(cond))
      : "scc");  // s_and_saveexec writes SCC
}
#else
inline void sel64(uint64_t& dst, uint64_t src, bool cond) { dst = cond ? src : dst; }
#endif

struct MulP5 {  // b * P5 for a byte b (host; the kernels read a 256-entry LDS table instead)
  DQ_HD uint64_t operator()(uint32_t b) const { return (uint64_t)b * XP5; }
};

// XXH64.hashUnsafeBytes of a string of len <= 28 bytes, up to fmix_head.  w[0..7]: the string's
// bytes as little-endian dwords (bytes past len may hold anything; w[7] is never read for a value
// that matters).  Branch-free: every lane runs 3 stripe rounds, one 4-byte round and 3 byte rounds
// and keeps the ones its length needs, so a wave of mixed lengths does not diverge.  The 4-byte
// round's dword w[2 nw] and the byte rounds' dword w[len >> 2] = w[2 nw + (len >> 2 & 1)] ride
// along the stripe rounds' predicates as one 64-bit pair (no dynamic register indexing).
// bp(b) = b * P5 for a byte b.
template <typename BP>
DQ_HD uint64_t xxh64_short_head(const uint32_t (&w)[8], uint32_t len, BP bp) {
  uint64_t h = kSeed + XP5 + (uint64_t)len;
  const uint32_t nw = len >> 3;
  uint64_t d4p = ((uint64_t)w[1] << 32) | w[0];  // {w[2 nw], w[2 nw + 1]} after the stripe rounds
#pragma unroll
  for (uint32_t k = 0; k < 3; ++k) {
    const uint64_t k1 = ((uint64_t)w[2 * k + 1] << 32) | w[2 * k];
    uint64_t hn = h ^ mul_add_c(rotl64(mul_add_c(k1, XP2, 0), 31), XP1, 0);
    hn = mul_add_c(rotl64(hn, 27), XP1, XP4);
    const bool take = k < nw;
    sel64(h, hn, take);
    sel64(d4p, ((uint64_t)w[2 * k + 3] << 32) | w[2 * k + 2], take);
  }
  const uint32_t d4 = (uint32_t)d4p, d4n = (uint32_t)(d4p >> 32);
  const bool has4 = (len & 4u) != 0;
  sel64(h, mul_add_c(rotl64(h ^ mul32_c(d4, XP1), 23), XP2, XP3), has4);
  const uint32_t db = has4 ? d4n : d4;
  const uint32_t nb = len & 3u;
#pragma unroll
  for (uint32_t j = 0; j < 3; ++j) sel64(h, mul_add_c(rotl64(h ^ bp((db >> (8 * j)) & 0xFFu), 11), XP1, 0), j < nb);
  return fmix_head(h);
}

}  // namespace dq
