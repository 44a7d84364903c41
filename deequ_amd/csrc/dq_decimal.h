// dq_decimal.h -- DecimalType (Arrow decimal128: 16-byte two's-complement unscaled values, precision <= 38) as
// Spark 2.2 reads it, host + device:
//   * Decimal.toDouble = java.math.BigDecimal.doubleValue: the correctly rounded (to nearest, ties to even)
//     double of unscaled / 10^scale -- what Cast(child, DoubleType) gives every numeric analyzer
//     (Minimum.scala:40, Maximum.scala:40, Sum.scala:40 after the exact decimal sum, StdDevPop / Corr inputs);
//   * the XxHash64 input (InterpretedHashFunction.hash, Decimal case): hashLong(unscaled) for precision <= 18,
//     else hashUnsafeBytes of BigInteger.toByteArray (minimal big-endian two's complement);
//   * the DataType class of its string (Decimal.toString = BigDecimal.toString: plain notation -- FRACTIONAL,
//     or INTEGRAL at scale 0 -- unless the adjusted exponent is below -6, then "1.5E-7": a STRING).
// The conversion: the value as a double-double (its 32-bit limbs added by TwoSums) times 10^-s as a double-double
// (tables from tools/gen_dec_tables.py) -- within 2^-101 of the quotient -- rounded once; a result whose
// residual lies within 2^-95 of a rounding midpoint (rare: exact ties exist, e.g. 9007199254740992.5) is settled
// by an exact integer comparison of a * 2^k with the midpoint times 10^s (320-bit limbs).
// Checked on the host against Python's exact Fraction -> float (tests/test_decimal_host.py) and on the GPU
// against the oracle (tests/test_decimal_gpu.py).
#pragma once

#include <cstdint>

#include "dq_hash.h"

#if defined(__HIP__)
#define DQ_HD_COLD static __host__ __device__ __attribute__((noinline))
#else
#define DQ_HD_COLD static inline
#endif

namespace dq {

using u128 = unsigned __int128;
using i128 = __int128;

constexpr int kDecMaxPrecision = 38;

// the conversion's constants (dq_dec_tables.inc: host arrays, or the kernels' __constant__ copies)
struct DecTab {
  const uint64_t* p10lo;
  const uint64_t* p10hi;
  const double* rh;
  const double* rl;
};

DQ_HD u128 dec_u128(uint64_t lo, uint64_t hi) { return ((u128)hi << 64) | lo; }
DQ_HD u128 dec_p10(const DecTab& t, int s) { return dec_u128(t.p10lo[s], t.p10hi[s]); }
// |unscaled| of a two's-complement value (unsigned negation: no overflow for any bit pattern)
DQ_HD u128 dec_mag(uint64_t lo, uint64_t hi) {
  const u128 u = dec_u128(lo, hi);
  return (int64_t)hi < 0 ? (u128)0 - u : u;
}

DQ_HD uint64_t dec_bits(double d) { return __builtin_bit_cast(uint64_t, d); }
DQ_HD double dec_from_bits(uint64_t b) { return __builtin_bit_cast(double, b); }

// ---- exact midpoint test: sign of a / 10^s - M 2^E (320-bit unsigned limbs) ----
struct U320 {
  uint64_t w[5];
};
DQ_HD void u320_shl(U320& x, int n) {  // 0 <= n < 320, bits shifted past 320 are dropped (never set here)
  const int q = n >> 6, r = n & 63;
  for (int i = 4; i >= 0; --i) {
    const uint64_t v = i - q >= 0 ? x.w[i - q] : 0;
    const uint64_t u = (r != 0 && i - q - 1 >= 0) ? x.w[i - q - 1] : 0;
    x.w[i] = r != 0 ? (v << r) | (u >> (64 - r)) : v;
  }
}
DQ_HD int u320_cmp(const U320& a, const U320& b) {
  for (int i = 4; i >= 0; --i)
    if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
  return 0;
}
// -1 / 0 / 1 as a / 10^s <, =, > M 2^E  (a < 2^128, 10^s < 2^127, M < 2^55, -190 < E < 80)
DQ_HD int dec_cmp_mid(u128 a, u128 p10, uint64_t M, int E) {
  U320 L{{(uint64_t)a, (uint64_t)(a >> 64), 0, 0, 0}};
  U320 R{};
  const u128 q0 = (u128)(uint64_t)p10 * M, q1 = (u128)(uint64_t)(p10 >> 64) * M;
  const u128 mid = (q0 >> 64) + (u128)(uint64_t)q1;
  R.w[0] = (uint64_t)q0;
  R.w[1] = (uint64_t)mid;
  R.w[2] = (uint64_t)(q1 >> 64) + (uint64_t)(mid >> 64);
  if (E < 0) u320_shl(L, -E);
  else u320_shl(R, E);
  return u320_cmp(L, R);
}

// the double nearest a / 10^s given y, the double-double estimate's rounding, and which of its two midpoints is
// in doubt (up: between y and its successor, else between y and its predecessor).  y > 0, normal.
DQ_HD_COLD double dec_settle(u128 a, u128 p10, double y, bool up) {  // (rare: out of line)
  const uint64_t yb = dec_bits(y);
  const int ey = (int)((yb >> 52) & 0x7FF) - 1075;
  const uint64_t Y = (yb & ((1ull << 52) - 1)) | (1ull << 52);
  uint64_t M;
  int E;
  if (up) {
    M = 2 * Y + 1;
    E = ey - 1;
  } else if (Y > (1ull << 52)) {
    M = 2 * Y - 1;
    E = ey - 1;
  } else {  // y a power of two: the predecessor is half an ulp below
    M = (1ull << 54) - 1;
    E = ey - 2;
  }
  const int c = dec_cmp_mid(a, p10, M, E);
  const bool even = (Y & 1) == 0;
  if (up) return c > 0 || (c == 0 && !even) ? dec_from_bits(yb + 1) : y;
  return c < 0 || (c == 0 && !even) ? dec_from_bits(yb - 1) : y;
}

// Knuth's TwoSum: s + e == a + b exactly
DQ_HD void dec_two_sum(double a, double b, double& s, double& e) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
  s = a + b;
  const double bb = s - a;
  e = (a - (s - bb)) + (b - bb);
}

// Decimal.toDouble of unscaled (lo, hi) at scale s (0 <= s <= 38).  narrow: the value fits a signed long (precision
// <= 18: hi is lo's sign extension).  The signed value's 32-bit limbs (two's complement: the top limb signed) are
// exact doubles; TwoSums add them into h + l (within 2^-104), which times 10^-s (rh + rl) is rounded once.
DQ_HD double dec_to_double(uint64_t lo, uint64_t hi, int s, const DecTab& t, bool narrow = false) {
#if defined(__clang__)
#pragma clang fp contract(off)  // the error-free products and sums below must not be fused (device default: fast)
#endif
  double h, l;
  if (narrow) {
    dec_two_sum((double)(int32_t)(uint32_t)(lo >> 32) * 0x1p32, (double)(uint32_t)lo, h, l);
  } else {
    double e1, e2;
    dec_two_sum((double)(int32_t)(uint32_t)(hi >> 32) * 0x1p96, (double)(uint32_t)hi * 0x1p64, h, l);
    dec_two_sum(h, (double)(uint32_t)(lo >> 32) * 0x1p32, h, e1);
    dec_two_sum(h, (double)(uint32_t)lo, h, e2);
    l = l + e1 + e2;
  }
  if (h == 0.0) return 0.0;  // (the value 0: every limb term vanished)
  const bool neg = h < 0.0;
  if (neg) {
    h = -h;
    l = -l;
  }
  const double rh = t.rh[s], rl = t.rl[s];
  const double p = h * rh;
  const double e = __builtin_fma(h, rh, -p);
  const double tt = __builtin_fma(h, rl, __builtin_fma(l, rh, e));
  double y = p + tt;
  const double r = (p - y) + tt;  // ~ a / 10^s - y, within 2^-101 y
  // a rounding midpoint near y + r: half an ulp of y from its exponent (a quarter below a power of two)
  const double hu = dec_from_bits(((dec_bits(y) >> 52) - 53) << 52);
  const double tol = y * 0x1p-95, ar = __builtin_fabs(r);
  if (__builtin_fabs(ar - hu) <= tol || __builtin_fabs(ar - 0.5 * hu) <= tol)
    y = dec_settle(dec_mag(lo, hi), dec_p10(t, s), y, r > 0.0);
  return neg ? -y : y;
}

// BigInteger.toByteArray of the unscaled value as XXH64 input: its length (1..16) and the bytes as little-endian
// dwords w[0..3] (w[4..7] = 0)
DQ_HD uint32_t dec_be_bytes(uint64_t lo, uint64_t hi, uint32_t (&w)[8]) {
  const bool neg = (int64_t)hi < 0;
  const uint64_t th = neg ? ~hi : hi, tl = neg ? ~lo : lo;  // bitLength of v = bit length of (v < 0 ? ~v : v)
  const int bl = th ? 128 - __builtin_clzll(th) : (tl ? 64 - __builtin_clzll(tl) : 0);
  const uint32_t len = (uint32_t)(bl / 8 + 1);
  // byte i of the sequence = byte len - 1 - i of v: the byte-reversed 16 bytes shifted down by 16 - len bytes
  const u128 rev = ((u128)__builtin_bswap64(lo) << 64) | __builtin_bswap64(hi);
  const u128 seq = len == 16 ? rev : rev >> (8 * (16 - len));
  w[0] = (uint32_t)seq;
  w[1] = (uint32_t)(seq >> 32);
  w[2] = (uint32_t)(seq >> 64);
  w[3] = (uint32_t)(seq >> 96);
  w[4] = w[5] = w[6] = w[7] = 0;
  return len;
}

// XXH64 (seed 42) of a decimal value as Spark 2.2 hashes it, up to fmix_head
DQ_HD uint64_t dec_hash_head(uint64_t lo, uint64_t hi, int precision) {
  if (precision <= 18) return xxh64_long_head(lo);
  uint32_t w[8];
  const uint32_t len = dec_be_bytes(lo, hi, w);
  return xxh64_short_head(w, len, MulP5());
}
DQ_HD uint64_t dec_hash(uint64_t lo, uint64_t hi, int precision) { return fmix_tail(dec_hash_head(lo, hi, precision)); }

// DataType class of the value's string (StatefulDataType.scala:36-38): 1 FRACTIONAL, 2 INTEGRAL, 4 STRING.
// BigDecimal.toString is plain iff the adjusted exponent digits(a) - 1 - s >= -6, i.e. s <= 6 or a >= 10^(s-6).
DQ_HD int dec_dt_class(uint64_t lo, uint64_t hi, int s, const DecTab& t) {
  if (s == 0) return 2;
  if (s <= 6) return 1;
  return dec_mag(lo, hi) >= dec_p10(t, s - 6) ? 1 : 4;
}

}  // namespace dq
