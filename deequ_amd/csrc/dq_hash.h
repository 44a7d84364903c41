// dq_hash.h -- XXH64 as used by Spark's XxHash64Function (seed 42), host + device.
// Reference call site: analyzers/catalyst/StatefulHyperloglogPlus.scala:93.  Included by the
// kernels and by tests/hash_check.cpp (host build) so the device formulation is checked on the CPU.
#pragma once

#include <cstdint>

#if defined(__HIP__)
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
// product + addend), two v_mul_lo_u32 (cross products) and one add3.  VOL: the asm is volatile, for
// the string hash's conditional rounds -- LLVM would otherwise hoist a round out of its exec-masked
// branch, run it in every lane and select the result afterwards.
template <bool VOL = false>
DQ_HD uint64_t mul_add_c(uint64_t x, uint64_t c, uint64_t a) {
  const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
#if defined(__HIP_DEVICE_COMPILE__)
  // The three multiplies are pinned in asm: left to itself LLVM re-associates the cross products
  // into extra v_mad_u64_u32 + v_mov chains (up to 7 instructions).  The addend is a VGPR pair (a
  // loop-invariant constant; the VOP3 constant bus takes only the SGPR multiplier).
  uint64_t p, carry;
  uint32_t t1, t2;
#define DQ_MUL_BODY                                                                                  \
  ("v_mad_u64_u32 %[p], %[cy], %[xl], %[cl], %[a]\n\t"                                               \
   "v_mul_lo_u32 %[t1], %[xl], %[ch]\n\t"                                                             \
   "v_mul_lo_u32 %[t2], %[xh], %[cl]"                                                                \
   : [p] "=&v"(p), [cy] "=&s"(carry), [t1] "=&v"(t1), [t2] "=&v"(t2)                                 \
   : [xl] "v"(xl), [xh] "v"(xh), [cl] "s"((uint32_t)c), [ch] "s"((uint32_t)(c >> 32)), [a] "v"(a))
  if constexpr (VOL) asm volatile DQ_MUL_BODY;
  else asm DQ_MUL_BODY;
#undef DQ_MUL_BODY
  (void)carry;
  const uint32_t hi = (uint32_t)(p >> 32) + t1 + t2;
#else
  const uint64_t p = (uint64_t)xl * (uint32_t)c + a;
  const uint32_t hi = (uint32_t)(p >> 32) + xl * (uint32_t)(c >> 32) + xh * (uint32_t)c;
#endif
  return ((uint64_t)hi << 32) | (uint32_t)p;
}

// x * c (mod 2^64): mul_add_c with the addend an inline 0 (no zero register pair kept live)
template <bool VOL = false>
DQ_HD uint64_t mul_c(uint64_t x, uint64_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
  uint64_t p, carry;
  uint32_t t1, t2;
#define DQ_MUL_BODY                                                                                  \
  ("v_mad_u64_u32 %[p], %[cy], %[xl], %[cl], 0\n\t"                                                  \
   "v_mul_lo_u32 %[t1], %[xl], %[ch]\n\t"                                                             \
   "v_mul_lo_u32 %[t2], %[xh], %[cl]"                                                                \
   : [p] "=&v"(p), [cy] "=&s"(carry), [t1] "=&v"(t1), [t2] "=&v"(t2)                                 \
   : [xl] "v"(xl), [xh] "v"(xh), [cl] "s"((uint32_t)c), [ch] "s"((uint32_t)(c >> 32)))
  if constexpr (VOL) asm volatile DQ_MUL_BODY;
  else asm DQ_MUL_BODY;
#undef DQ_MUL_BODY
  (void)carry;
  const uint32_t hi = (uint32_t)(p >> 32) + t1 + t2;
  return ((uint64_t)hi << 32) | (uint32_t)p;
#else
  return x * c;
#endif
}

// x * c (mod 2^64) for a 32-bit x: one v_mad_u64_u32, one v_mul_lo_u32, one add.
template <bool VOL = false>
DQ_HD uint64_t mul32_c(uint32_t x, uint64_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t p, carry;
  uint32_t t;
#define DQ_MUL_BODY                                                                                  \
  ("v_mad_u64_u32 %[p], %[cy], %[x], %[cl], 0\n\t"                                                   \
   "v_mul_lo_u32 %[t], %[x], %[ch]"                                                                  \
   : [p] "=&v"(p), [cy] "=&s"(carry), [t] "=&v"(t)                                                   \
   : [x] "v"(x), [cl] "s"((uint32_t)c), [ch] "s"((uint32_t)(c >> 32)))
  if constexpr (VOL) asm volatile DQ_MUL_BODY;
  else asm DQ_MUL_BODY;
#undef DQ_MUL_BODY
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
  h = mul_c(h, XP2);
  return h ^ (h >> 29);
}
DQ_HD uint64_t fmix_tail(uint64_t b) {
  const uint64_t h = b * XP3;
  return h ^ (h >> 32);
}
DQ_HD uint64_t fmix64(uint64_t h) { return fmix_tail(fmix_head(h)); }

// XXH64.hashLong / hashInt (seed 42) up to fmix_head
DQ_HD uint64_t xxh64_long_head(uint64_t v) {
  const uint64_t k = rotl64(mul_c(v, XP2), 31);
  const uint64_t h = mul_c(k, XP1) ^ (kSeed + XP5 + 8);
  return fmix_head(mul_add_c(rotl64(h, 27), XP1, XP4));
}
DQ_HD uint64_t xxh64_int_head(uint32_t v) {
  const uint64_t h = mul32_c(v, XP1) ^ (kSeed + XP5 + 4);
  return fmix_head(mul_add_c(rotl64(h, 23), XP2, XP3));
}
DQ_HD uint64_t xxh64_long(uint64_t v) { return fmix_tail(xxh64_long_head(v)); }
DQ_HD uint64_t xxh64_int(uint32_t v) { return fmix_tail(xxh64_int_head(v)); }

struct MulP5 {  // b * P5 for a byte b (host; the kernels read a 256-entry LDS table instead)
  DQ_HD uint64_t operator()(uint32_t b) const { return (uint64_t)b * XP5; }
};

// XXH64.hashUnsafeBytes of a string of len <= 28 bytes, up to fmix_head, in the pieces the UTF8
// kernel runs.  w[0..7]: the string's bytes as little-endian dwords (bytes past len may hold anything;
// w[7] is never read for a value that matters).  Every round is conditional on the lane's length
// (on the device: an exec-masked branch, skipped by a wave none of whose lanes needs it), so a wave
// of mixed lengths does not diverge.  The 4-byte round's dword w[2 nw] and the byte rounds' dword
// w[len >> 2] = w[2 nw + (len >> 2 & 1)] ride along the stripe rounds as one 64-bit pair (no dynamic
// register indexing).  bp(b) = b * P5 for a byte b.

// One 8-byte round: h ^= rotl(k1 * P2, 31) * P1; h = rotl(h, 27) * P1 + P4.
template <bool VOL = false>
DQ_HD uint64_t xxh64_stripe_round(uint64_t h, uint64_t k1) {
  return mul_add_c<VOL>(rotl64(h ^ mul_c<VOL>(rotl64(mul_c<VOL>(k1, XP2), 31), XP1), 27), XP1, XP4);
}

// The first NR stripe rounds (min(NR, len >> 3) of them): returns h and d4p = {w[2 m], w[2 m + 1]},
// m = min(NR, len >> 3) -- the tail's dwords for len < 8 NR, else the next stripe word.
template <int NR>
DQ_HD uint64_t xxh64_stripes(const uint32_t (&w)[8], uint32_t len, uint64_t& d4p) {
  uint64_t h = kSeed + XP5 + (uint64_t)len;
  const uint32_t nw = len >> 3;
  d4p = ((uint64_t)w[1] << 32) | w[0];
#pragma unroll
  for (uint32_t k = 0; k < (uint32_t)NR; ++k) {
    if (k < nw) {
      h = xxh64_stripe_round<true>(h, ((uint64_t)w[2 * k + 1] << 32) | w[2 * k]);
      d4p = ((uint64_t)w[2 * k + 3] << 32) | w[2 * k + 2];
    }
  }
  return h;
}

// After the stripe rounds: the 4-byte round (len & 4) on the low dword of d4p and the (len & 3) byte
// rounds on the dword after it, up to fmix_head.  The byte rounds' b * P5 are fetched before any round.
template <typename BP>
DQ_HD uint64_t xxh64_tail_head(uint64_t h, uint64_t d4p, uint32_t len, BP bp) {
  const uint32_t d4 = (uint32_t)d4p;
#if defined(__HIP_DEVICE_COMPILE__) && !defined(DQ_JIT)
  // one compare for both uses (the select and the exec-masked round): written as a bool, LLVM emits an
  // eq compare for one and a ne compare for the other
  const bool has4 = __builtin_amdgcn_inverse_ballot_w64(__builtin_amdgcn_uicmp(len & 4u, 0u, 33 /* ICMP_NE */));
#else
  const bool has4 = (len & 4u) != 0;
#endif
  const uint32_t db = has4 ? (uint32_t)(d4p >> 32) : d4;
  const uint32_t nb = len & 3u;
  uint64_t kb[3];
#pragma unroll
  for (uint32_t j = 0; j < 3; ++j) kb[j] = bp((db >> (8 * j)) & 0xFFu);
  if (has4) h = mul_add_c<true>(rotl64(h ^ mul32_c<true>(d4, XP1), 23), XP2, XP3);
#pragma unroll
  for (uint32_t j = 0; j < 3; ++j)
    if (j < nb) h = mul_c<true>(rotl64(h ^ kb[j], 11), XP1);
  return fmix_head(h);
}

template <typename BP>
DQ_HD uint64_t xxh64_short_head(const uint32_t (&w)[8], uint32_t len, BP bp) {
  uint64_t d4p;
  const uint64_t h = xxh64_stripes<3>(w, len, d4p);
  return xxh64_tail_head(h, d4p, len, bp);
}

// The same hash split the way the UTF8 kernel runs it when a string of 24..28 bytes is deferred: two
// stripe rounds in the block loop, then -- packed with other deferred strings -- the third round on
// {w4, w5} (= d4p after two rounds) and the tail on {w6, w7}.
template <typename BP>
DQ_HD uint64_t xxh64_short_head_split(const uint32_t (&w)[8], uint32_t len, BP bp) {
  uint64_t d4p;
  uint64_t h = xxh64_stripes<2>(w, len, d4p);
  if ((len >> 3) < 3) return xxh64_tail_head(h, d4p, len, bp);
  h = xxh64_stripe_round<true>(h, d4p);
  return xxh64_tail_head(h, ((uint64_t)w[7] << 32) | w[6], len, bp);
}

// The rounds after a long string's 32-byte stripes, or all of a short string's: with h = the merged stripe
// state (or seed + P5) + len, the min(3, r >> 3) 8-byte rounds, the 4-byte and byte rounds of the r < 32
// bytes t[0..7] (bytes past r: anything), up to fmix_head.
template <typename BP>
DQ_HD uint64_t xxh64_rem_head(uint64_t h, const uint32_t (&t)[8], uint32_t r, BP bp) {
  const uint32_t nw = r >> 3;
  uint64_t d4p = ((uint64_t)t[1] << 32) | t[0];
  for (uint32_t k = 0; k < 3; ++k) {
    if (k < nw) {
      h = xxh64_stripe_round(h, ((uint64_t)t[2 * k + 1] << 32) | t[2 * k]);
      d4p = ((uint64_t)t[2 * k + 3] << 32) | t[2 * k + 2];
    }
  }
  return xxh64_tail_head(h, d4p, r, bp);
}

// One 32-byte stripe w[0..7] into the four accumulators (XXH64's long-input loop)
DQ_HD void xxh64_stripe32(uint64_t (&v)[4], const uint32_t* w) {
  for (int k = 0; k < 4; ++k)
    v[k] = mul_c(rotl64(v[k] + mul_c(((uint64_t)w[2 * k + 1] << 32) | w[2 * k], XP2), 31), XP1);
}
DQ_HD uint64_t xxh64_merge4(const uint64_t (&v)[4]) {
  uint64_t h = rotl64(v[0], 1) + rotl64(v[1], 7) + rotl64(v[2], 12) + rotl64(v[3], 18);
  for (int k = 0; k < 4; ++k) h = mul_add_c(h ^ mul_c(rotl64(mul_c(v[k], XP2), 31), XP1), XP1, XP4);
  return h;
}
constexpr uint64_t kXxhV0 = kSeed + XP1 + XP2, kXxhV1 = kSeed + XP2, kXxhV2 = kSeed, kXxhV3 = kSeed - XP1;

// XXH64.hashUnsafeBytes of a string of len <= 63 bytes up to fmix_head, from its bytes as little-endian dwords
// w[0..15] (bytes past len: anything): when len >= 32, one stripe and the merge; then the remainder.  The host
// check of the formulation the UTF8 kernel's rare path runs (dq_kernels.hip xxh64_window_head, which loops the
// stripes for any length).
template <typename BP>
DQ_HD uint64_t xxh64_upto63_head(const uint32_t (&w)[16], uint32_t len, BP bp) {
  uint64_t h = kSeed + XP5;
  uint32_t t[8];
  for (int k = 0; k < 8; ++k) t[k] = w[k];
  uint32_t r = len;
  if (len >= 32) {
    uint64_t v[4] = {kXxhV0, kXxhV1, kXxhV2, kXxhV3};
    xxh64_stripe32(v, w);
    h = xxh64_merge4(v);
    for (int k = 0; k < 8; ++k) t[k] = w[8 + k];
    r = len - 32;
  }
  return xxh64_rem_head(h + (uint64_t)len, t, r, bp);
}

}  // namespace dq
