// dq_kernels.hip -- gfx950 (MI355X, CDNA4) kernels of the fused Deequ metric scan.
//
// The reference computes these aggregates with one Spark job (AnalysisRunner.scala:303): a
// per-partition partial aggregate followed by a final merge.  Here one scan of a row chunk is:
//   1. dq_pred_scan   (only if predicates exist): three-valued predicate program per row ->
//                     Compliance / conditional-count counters, and `where` TRUE bitmaps.
//   2. dq_column_scan<V>: single-column tasks (Completeness, Sum, Mean, StandardDeviation,
//                     Minimum, Maximum, ApproxCountDistinct), one launch per variant V (column kind x
//                     accumulators).
//   3. dq_pair_stage_scan (dq_pair.hip, only if Correlations exist): co-moments of the pair groups
//                     (<= 8 columns staged HBM -> LDS once) fused with the moments of their columns.
//   4. dq_finalize:   fixed-order merge of the per-workgroup partials, then in-order merge into
//                     the plan's accumulators (chunk order) -> results are deterministic.
// Streaming loads are 16 B per lane (global_load_dwordx4) for 8-/4-byte columns; there are no
// global atomics; HLL registers are privatised per workgroup in LDS (ds_max_u32).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "dq_device.h"
#include "dq_hash.h"
#include "dq_decimal.h"
#include "dq_lane.h"

namespace dq {

// DecimalType conversion constants (tools/gen_dec_tables.py) in constant memory
#define DQ_DEC_TABLE static __constant__ const
#include "dq_dec_tables.inc"
#undef DQ_DEC_TABLE
__device__ __forceinline__ DecTab dec_dev_tab() { return DecTab{kDecP10Lo, kDecP10Hi, kDecRcpHi, kDecRcpLo}; }

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------------
// XXH64 (Spark XxHash64Function, seed 42) -- StatefulHyperloglogPlus.scala:93
// ------------------------------------------------------------------------------------------
// Byte reads from a 4-byte aligned buffer at an arbitrary byte position, via aligned dwords.
__device__ __forceinline__ uint32_t ld32(const uint8_t* base, int64_t a) {
  return *reinterpret_cast<const uint32_t*>(base + a);
}
__device__ __forceinline__ uint32_t read4(const uint8_t* base, int64_t pos) {
  int64_t a = pos & ~int64_t(3);
  uint32_t sh = (uint32_t)(pos & 3) * 8u;
  uint32_t w0 = ld32(base, a);
  if (sh == 0) return w0;
  uint32_t w1 = ld32(base, a + 4);
  return alignbit32(w1, w0, sh);
}
__device__ __forceinline__ uint64_t read8(const uint8_t* base, int64_t pos) {
  int64_t a = pos & ~int64_t(3);
  uint32_t sh = (uint32_t)(pos & 3) * 8u;
  uint32_t w0 = ld32(base, a), w1 = ld32(base, a + 4);
  if (sh == 0) return ((uint64_t)w1 << 32) | w0;
  uint32_t w2 = ld32(base, a + 8);
  uint32_t lo = alignbit32(w1, w0, sh);
  uint32_t hi = alignbit32(w2, w1, sh);
  return ((uint64_t)hi << 32) | lo;
}

// XXH64.hashUnsafeBytes over data[pos, pos + n)
__device__ uint64_t xxh64_bytes(const uint8_t* data, int64_t pos, int64_t n) {
  int64_t off = pos, end = pos + n;
  uint64_t h;
  if (n >= 32) {
    uint64_t v1 = kSeed + XP1 + XP2, v2 = kSeed + XP2, v3 = kSeed, v4 = kSeed - XP1;
    for (; off <= end - 32; off += 32) {
      v1 = rotl64(v1 + read8(data, off) * XP2, 31) * XP1;
      v2 = rotl64(v2 + read8(data, off + 8) * XP2, 31) * XP1;
      v3 = rotl64(v3 + read8(data, off + 16) * XP2, 31) * XP1;
      v4 = rotl64(v4 + read8(data, off + 24) * XP2, 31) * XP1;
    }
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h ^= rotl64(v1 * XP2, 31) * XP1; h = h * XP1 + XP4;
    h ^= rotl64(v2 * XP2, 31) * XP1; h = h * XP1 + XP4;
    h ^= rotl64(v3 * XP2, 31) * XP1; h = h * XP1 + XP4;
    h ^= rotl64(v4 * XP2, 31) * XP1; h = h * XP1 + XP4;
  } else {
    h = kSeed + XP5;
  }
  h += (uint64_t)n;
  for (; off <= end - 8; off += 8) {
    h ^= rotl64(read8(data, off) * XP2, 31) * XP1;
    h = rotl64(h, 27) * XP1 + XP4;
  }
  if (off + 4 <= end) {
    h ^= (uint64_t)read4(data, off) * XP1;
    h = rotl64(h, 23) * XP2 + XP3;
    off += 4;
  }
  for (; off < end; ++off) {
    h ^= (uint64_t)(read4(data, off) & 0xFFu) * XP5;
    h = rotl64(h, 11) * XP1;
  }
  return fmix64(h);
}

// HLL++ registers (StatefulHyperloglogPlus.scala:96-113) live in LDS as int32 q = pw - 1, with -1 for
// an empty register: pw = nlz((x << 9) | 256) + 1, so q = nlz(...) is the leading-zero count itself and
// an update is one ds_max_i32; the workgroup merge writes q + 1 (0 for empty) to the accumulator.
__device__ __forceinline__ int32_t hll_q_exact(uint64_t x) {
  return (int32_t)__clzll((long long)((x << 9) | 256ull));
}

__device__ __forceinline__ void hll_update(int32_t* regs, uint64_t x) {
  atomicMax(&regs[(uint32_t)(x >> 55)], hll_q_exact(x));
}

// Branch-free predicated update: an unselected row does ds_max(reg, -1), a no-op.
__device__ __forceinline__ void hll_update_if(int32_t* regs, uint64_t x, bool b) {
  atomicMax(&regs[(uint32_t)(x >> 55)], b ? hll_q_exact(x) : -1);
}

// v_ffbh_u32 as the hardware defines it: leading-zero count, 0xFFFFFFFF (= -1) for a zero input.
__device__ __forceinline__ int32_t ffbh_raw(uint32_t x) {
  int32_t r;
  asm("v_ffbh_u32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

// HLL key of an XXH64 state b = fmix_head(h) (dq_hash.h), i.e. before fmix64's last multiply:
// the final hash's high word is hi32(b * P3) (the closing `h ^= h >> 32` only changes the low word),
// which carries the register index (bits 63..55) and, unless its bits 54..32 are all zero
// (probability 2^-23), the rank.  `addr` is the LDS byte offset of register idx; `q` = pw - 1, or -1
// when the rank needs the low word (the caller then recomputes that value exactly).
struct HllKey {
  uint32_t addr;
  int32_t q;
};
__device__ __forceinline__ HllKey hll_key_from_fmix(uint64_t b) {
  const uint32_t bl = (uint32_t)b, bh = (uint32_t)(b >> 32);
  const uint32_t hi = __umulhi(bl, (uint32_t)XP3) + bl * (uint32_t)(XP3 >> 32) + bh * (uint32_t)XP3;
  return {(hi >> 21) & 0x7FCu, ffbh_raw(hi << 9)};
}
// XXH64.hashLong / hashInt (seed 42) -> HLL key (StatefulHyperloglogPlus.scala:93 via XxHash64Function)
__device__ __forceinline__ HllKey hll_key_long(uint64_t v) { return hll_key_from_fmix(xxh64_long_head(v)); }
__device__ __forceinline__ HllKey hll_key_int(uint32_t v) { return hll_key_from_fmix(xxh64_int_head(v)); }


// ------------------------------------------------------------------------------------------
// Chan-mergeable column statistics
// ------------------------------------------------------------------------------------------
struct ColStats {
  double n, mean, m2, sum;
  int64_t isum, count, nan_count;
  double fmin, fmax;
  int64_t pinf, ninf;  // selected +-inf values of an F64 column (outside n / mean / m2 / sum)
  int64_t isum_hi;     // D128: (isum, isum_hi) = the exact 128-bit sum (wrapping)
};

__device__ __forceinline__ void stats_init(ColStats& s) {
  s.n = 0.0; s.mean = 0.0; s.m2 = 0.0; s.sum = 0.0;
  s.isum = 0; s.count = 0; s.nan_count = 0;
  s.fmin = __longlong_as_double(0x7FF0000000000000ll);   // +inf
  s.fmax = __longlong_as_double((long long)0xFFF0000000000000ull);  // -inf
  s.pinf = 0; s.ninf = 0;
  s.isum_hi = 0;
}

// a <- a (+) b ; exact Chan/Welford combination (same algebra as StandardDeviationState.sum)
__device__ __forceinline__ void stats_merge(ColStats& a, const ColStats& b) {
  double n = a.n + b.n;
  if (b.n != 0.0) {
    if (a.n == 0.0) {
      a.mean = b.mean; a.m2 = b.m2;
    } else {
      double delta = b.mean - a.mean;
      double r = b.n / n;
      a.mean = a.mean + delta * r;
      a.m2 = a.m2 + b.m2 + delta * delta * a.n * r;
    }
  }
  a.n = n;
  a.sum += b.sum;
  {  // 128-bit add (the high word only matters for decimal columns)
    const uint64_t lo = (uint64_t)a.isum + (uint64_t)b.isum;
    a.isum_hi = (int64_t)((uint64_t)a.isum_hi + (uint64_t)b.isum_hi + (lo < (uint64_t)a.isum ? 1u : 0u));
    a.isum = (int64_t)lo;
  }
  a.count += b.count;
  a.nan_count += b.nan_count;
  a.fmin = hw_min(a.fmin, b.fmin);
  a.fmax = hw_max(a.fmax, b.fmax);
  a.pinf += b.pinf;
  a.ninf += b.ninf;
}

__device__ __forceinline__ ColStats stats_shfl_xor(const ColStats& s, int m) {
  ColStats o;
  o.n = __shfl_xor(s.n, m); o.mean = __shfl_xor(s.mean, m); o.m2 = __shfl_xor(s.m2, m);
  o.sum = __shfl_xor(s.sum, m);
  o.isum = __shfl_xor(s.isum, m); o.count = __shfl_xor(s.count, m); o.nan_count = __shfl_xor(s.nan_count, m);
  o.fmin = __shfl_xor(s.fmin, m); o.fmax = __shfl_xor(s.fmax, m);
  o.pinf = __shfl_xor(s.pinf, m); o.ninf = __shfl_xor(s.ninf, m);
  o.isum_hi = __shfl_xor(s.isum_hi, m);
  return o;
}

__device__ __forceinline__ void stats_store(ColPartial* p, const ColStats& s) {
  p->n = s.n; p->mean = s.mean; p->m2 = s.m2; p->sum = s.sum; p->isum = s.isum; p->count = s.count;
  p->nan_count = s.nan_count; p->fmin = s.fmin; p->fmax = s.fmax; p->pinf_count = s.pinf; p->ninf_count = s.ninf;
  p->isum_hi = s.isum_hi;
}
__device__ __forceinline__ ColStats stats_load(const ColPartial* p) {
  ColStats s;
  s.n = p->n; s.mean = p->mean; s.m2 = p->m2; s.sum = p->sum; s.isum = p->isum; s.count = p->count;
  s.nan_count = p->nan_count; s.fmin = p->fmin; s.fmax = p->fmax; s.pinf = p->pinf_count; s.ninf = p->ninf_count;
  s.isum_hi = p->isum_hi;
  return s;
}

// Reduce the 256 threads' statistics -> one ColPartial (fixed order: lanes by butterfly, waves 0..3).
__device__ void block_reduce_store(ColStats s, ColPartial* out, ColStats* lds) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    ColStats o = stats_shfl_xor(s, m);
    stats_merge(s, o);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) lds[wave] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    ColStats a = lds[0];
#pragma unroll
    for (int w = 1; w < kWaves; ++w) stats_merge(a, lds[w]);
    stats_store(out, a);
  }
}

// Branch-free optional bitmap word: a missing bitmap reads word 0 of an all-ones buffer (the
// pointer / index selects are wave-uniform scalar ops, so the loop body has no branches).
__device__ const uint32_t kAllOnes[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
__device__ __forceinline__ uint32_t word_or_ones(const uint32_t* p, int64_t i) {
  const uint32_t* q = p ? p : kAllOnes;
  return q[p ? i : 0];
}

// Validity / `where` words of one workgroup row range [row0, row1) (row0 a multiple of 32) through a
// raw buffer resource.  A missing bitmap is a zero-size resource (loads return 0) OR-ed with an
// all-ones wave-uniform fill: no pointer selects, no flat loads, and a word past the range reads 0.
struct RangeBits {
  __amdgpu_buffer_rsrc_t r;
  uint32_t fill;
  __device__ __forceinline__ RangeBits(const uint32_t* p, int64_t row0, int64_t row1) {
    const int32_t nbytes = p ? (int32_t)(((row1 - row0 + 31) >> 5) * 4) : 0;
    r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(p ? p + (row0 >> 5) : nullptr), (short)0, nbytes,
                                          0x00020000);
    fill = p ? 0u : 0xFFFFFFFFu;
  }
  // word i of the range (rows row0 + 32 i .. + 31)
  __device__ __forceinline__ uint32_t word(int32_t i) const {
    return __builtin_amdgcn_raw_buffer_load_b32(r, i * 4, 0, 0) | fill;
  }
};

// ------------------------------------------------------------------------------------------
// Row masks as scalar lane masks.  Lane l of a wave handles rows r + l (r a multiple of 64), so the
// selection of 64 rows is one 64-bit word of the validity (& where) bitmap: it is loaded with scalar
// loads into SGPRs and used directly as the lane mask of v_cndmask (inverse ballot) -- no VALU work
// per row for validity, and counts come from s_bcnt1.
// ------------------------------------------------------------------------------------------

// selected-row masks of the 8 lane groups [base + 64 j, + 64) of a wave's block (base a multiple of
// 64; rem = row1 - base, <= 0 for a wave past the range's end; `full`: the whole block lies below row1).
// All branches are wave-uniform, and every comparison is a 32-bit one on rem: the scalar unit has no 64-bit
// ordered compare, so 64-bit row comparisons became VALU compares of SGPR pairs.
__device__ __forceinline__ void block_masks(const uint32_t* validity, const uint32_t* mask, int64_t base, int32_t rem,
                                            bool full, uint64_t (&m)[8]) {
  const int64_t w0 = base >> 5;
  if (full) {
    if (validity) {
#pragma unroll
      for (int j = 0; j < 8; ++j) m[j] = load_word64(validity, w0 + 2 * j);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) m[j] = ~0ull;
    }
    if (mask) {
#pragma unroll
      for (int j = 0; j < 8; ++j) m[j] &= load_word64(mask, w0 + 2 * j);
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int32_t left = rem - 64 * j;  // rows of group j below row1
    const int64_t w = w0 + 2 * j;
    uint64_t x = 0;
    if (left > 0) {
      const bool two = left > 32;  // the second dword holds rows below row1
      x = ~0ull;
      if (validity) x = ((uint64_t)(two ? ((const_u32s)validity)[w + 1] : 0u) << 32) | ((const_u32s)validity)[w];
      if (mask) x &= ((uint64_t)(two ? ((const_u32s)mask)[w + 1] : 0u) << 32) | ((const_u32s)mask)[w];
      if (left < 64) x &= (1ull << left) - 1ull;
    }
    m[j] = x;
  }
}


// Moments of a numeric column (lane l of a wave owns rows base + 64 j + l) as shifted sums over the whole
// workgroup range: sd = sum(x - shift), sdd = sum((x - shift)^2) per lane under the selection mask --
// exec-masked updates, so an unselected row costs no VALU work -- with ONE shift for the range (wave-uniform,
// in SGPRs): the mean of the range's first 64-row group holding finite selected values.  The selected-row
// count is a popcount of the masks (scalar), so no lane keeps a count, and nothing is merged inside the loop;
// at the range's end the wave's sums give (n, mean = shift + S1 / n, m2 = S2 - S1^2 / n), which merge across
// waves / ranges / chunks with StandardDeviationState.sum's algebra (Chan, StandardDeviation.scala:37-44).
// Accuracy: the range's first group is part of the range, so n (shift - mean)^2 <= (rows / 64) m2 for any
// data and the cancellation in m2 costs at most ~1e-13 relative at 2^16-row ranges (the Correlation pass
// uses the same shifts: tests/test_pair_lane.py drift test; full-scale C2 / C5 in tests/fullscale_parity.py).
struct LaneMoments {
  double sd, sdd;
  int64_t is;  // wrapping int64 sum (integral kinds; Spark Sum on LongType)
};

// this lane's value of row r of a range (buffer resource over the range's values; rows past it read 0)
template <int KIND>
__device__ __forceinline__ double range_value(__amdgpu_buffer_rsrc_t vr, int64_t rel) {
  if constexpr (KIND == CK_I32) return (double)(int32_t)__builtin_amdgcn_raw_buffer_load_b32(vr, (int)(rel * 4), 0, 0);
  if constexpr (KIND == CK_F32)
    return (double)__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(vr, (int)(rel * 4), 0, 0));
  if constexpr (KIND == CK_I16) return (double)(int16_t)__builtin_amdgcn_raw_buffer_load_b16(vr, (int)(rel * 2), 0, 0);
  if constexpr (KIND == CK_I8) return (double)(int8_t)__builtin_amdgcn_raw_buffer_load_b8(vr, (int)rel, 0, 0);
  const auto w2 = __builtin_amdgcn_raw_buffer_load_b64(vr, (int)(rel * 8), 0, 0);
  if constexpr (KIND == CK_F64) return __builtin_bit_cast(double, ((uint64_t)w2[1] << 32) | w2[0]);
  return __builtin_fma((double)(int32_t)w2[1], 4294967296.0, (double)w2[0]);
}
__device__ __forceinline__ double wave_uniform(double v) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b), hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}
__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = (int64_t)((uint64_t)v + (uint64_t)__shfl_xor(v, m));
  return v;
}

// the range's shift: mean of its first 64-row group with finite selected values (0 if none); groups with no
// selected row are skipped on their bitmap words alone
template <int KIND>
__device__ double range_shift_of(__amdgpu_buffer_rsrc_t vr, const uint32_t* validity, const uint32_t* mask, int64_t row0,
                                 int64_t row1, int lane) {
  for (int64_t r = row0; r < row1; r += 64) {
    uint64_t sel = ~0ull;
    {
      const int64_t w = r >> 5;
      const bool two = r + 32 < row1;
      if (validity) sel = ((uint64_t)(two ? ((const_u32s)validity)[w + 1] : 0u) << 32) | ((const_u32s)validity)[w];
      if (mask) sel &= ((uint64_t)(two ? ((const_u32s)mask)[w + 1] : 0u) << 32) | ((const_u32s)mask)[w];
      if (r + 64 > row1) sel &= (1ull << (row1 - r)) - 1ull;
    }
    if (sel == 0) continue;
    const double x = range_value<KIND>(vr, r - row0 + lane);
    const uint64_t fm = __builtin_amdgcn_ballot_w64(__builtin_isfinite(x)) & sel;
    if (fm != 0) return wave_uniform(wave_sum_f64(lane_bit(fm) ? x : 0.0) / (double)__builtin_popcountll(fm));
  }
  return 0.0;
}

// Exec-masked moment / min / max update of one value (inline asm so the accumulators are plain
// read-write operands: a C++ `if` on a lane mask makes the compiler copy every accumulator into
// its phi register before the branch).  exec &= ma for the moments, exec &= mb for min / max
// (MINMAX_SEP: mb excludes NaN rows), then restored; the outer exec is respected (s_and_saveexec).
// The shift is an SGPR pair (wave-uniform).
template <bool INTEGRAL, bool MINMAX_SEP>
__device__ __forceinline__ void masked_moments(LaneMoments& a, double& lo, double& hi, double x, uint64_t b,
                                               double shift, uint64_t ma, uint64_t mb) {
  double d;
  uint64_t save;
  if constexpr (INTEGRAL) {
    asm volatile(
        "s_and_saveexec_b64 %[save], %[ma]\n\t"
        "v_add_f64 %[d], %[x], -%[sh]\n\t"
        "v_lshl_add_u64 %[is], %[b], 0, %[is]\n\t"
        "v_min_f64 %[lo], %[lo], %[x]\n\t"
        "v_max_f64 %[hi], %[hi], %[x]\n\t"
        "v_add_f64 %[sd], %[sd], %[d]\n\t"
        "v_fma_f64 %[sdd], %[d], %[d], %[sdd]\n\t"
        "s_mov_b64 exec, %[save]"
        : [sd] "+v"(a.sd), [sdd] "+v"(a.sdd), [is] "+v"(a.is), [lo] "+v"(lo), [hi] "+v"(hi), [d] "=&v"(d),
          [save] "=&s"(save)
        : [x] "v"(x), [sh] "s"(shift), [b] "v"(b), [ma] "s"(ma)
        : "scc");
  } else if constexpr (!MINMAX_SEP) {
    asm volatile(
        "s_and_saveexec_b64 %[save], %[ma]\n\t"
        "v_add_f64 %[d], %[x], -%[sh]\n\t"
        "v_min_f64 %[lo], %[lo], %[x]\n\t"
        "v_max_f64 %[hi], %[hi], %[x]\n\t"
        "v_add_f64 %[sd], %[sd], %[d]\n\t"
        "v_fma_f64 %[sdd], %[d], %[d], %[sdd]\n\t"
        "s_mov_b64 exec, %[save]"
        : [sd] "+v"(a.sd), [sdd] "+v"(a.sdd), [lo] "+v"(lo), [hi] "+v"(hi), [d] "=&v"(d), [save] "=&s"(save)
        : [x] "v"(x), [sh] "s"(shift), [ma] "s"(ma)
        : "scc");
  } else {
    asm volatile(
        "s_and_saveexec_b64 %[save], %[ma]\n\t"
        "v_add_f64 %[d], %[x], -%[sh]\n\t"
        "v_add_f64 %[sd], %[sd], %[d]\n\t"
        "v_fma_f64 %[sdd], %[d], %[d], %[sdd]\n\t"
        "s_and_b64 exec, %[save], %[mb]\n\t"
        "v_min_f64 %[lo], %[lo], %[x]\n\t"
        "v_max_f64 %[hi], %[hi], %[x]\n\t"
        "s_mov_b64 exec, %[save]"
        : [sd] "+v"(a.sd), [sdd] "+v"(a.sdd), [lo] "+v"(lo), [hi] "+v"(hi), [d] "=&v"(d), [save] "=&s"(save)
        : [x] "v"(x), [sh] "s"(shift), [ma] "s"(ma), [mb] "s"(mb)
        : "scc");
  }
}

// One 512-row block of a wave: x[j] the lane's value of row group j as a double, bits[j] its raw 64-bit
// pattern (i32 / i16 / i8: sign-extended; f32: its 32 bits), m[j] the selection masks (every selected value finite: a block with a
// selected NaN / +-inf takes the caller's rolled path).
template <int KIND, bool STATS, bool HLL>
__device__ __forceinline__ void numeric_block(const double (&x)[8], const uint64_t (&bits)[8], const uint64_t (&m)[8],
                                              double shift, ColStats& s, LaneMoments& a, int32_t* regs, int32_t& qmin) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (STATS) masked_moments<!ck_float(KIND), false>(a, s.fmin, s.fmax, x[j], bits[j], shift, m[j], m[j]);
    if (HLL) {
      const HllKey key = ck_bytes(KIND) <= 4 ? hll_key_int((uint32_t)bits[j]) : hll_key_long(bits[j]);
      qmin = min(qmin, key.q);
      if (lane_bit(m[j])) atomicMax(reinterpret_cast<int32_t*>(reinterpret_cast<char*>(regs) + key.addr), key.q);
    }
  }
  if (HLL) {
    // rare (2^-23 per value): a rank that needs the hash's low word -- redo the block's selected
    // values exactly (register max is idempotent)
    if (__builtin_amdgcn_ballot_w64(qmin < 0) != 0) {
#pragma unroll 1
      for (int j = 0; j < 8; ++j) {
        if (lane_bit(m[j])) hll_update(regs, ck_bytes(KIND) <= 4 ? xxh64_int((uint32_t)bits[j]) : xxh64_long(bits[j]));
      }
      qmin = 0;
    }
  }
}

// The checked form of one 512-row block of a floating-point column (a selected NaN / +-inf in it, or the whole
// range re-run by numeric_range): one row group at a time, values re-read and the selection rebuilt per group -- a
// rolled loop whose state is one group's, so it adds no registers to the common path.  NaN rows hash as the
// canonical NaN (doubleToLongBits / floatToIntBits) and stay out of min / max (Spark orders NaN above every value)
// but enter the moments (which become NaN, as Spark's); +-inf rows stay out of the shifted moments and are
// counted: dq_finish adds them back into the sum (Spark's sequential sum is then +-inf, or NaN with both signs) and
// the moments become NaN.  KIND: CK_F64 (hashLong of the bits) or CK_F32 (the value widened to double exactly,
// hashInt of the bits: Spark 2.2's XxHash64 of a FloatType value).
template <int KIND, bool STATS, bool HLL>
__device__ __forceinline__ void float_block_checked(__amdgpu_buffer_rsrc_t vr, const uint32_t* validity,
                                                    const uint32_t* mask, int64_t base, int32_t rem, int32_t vo,
                                                    double shift, ColStats& s, LaneMoments& a, int32_t* regs,
                                                    int64_t& cnt_w, int64_t& nan_v, int64_t& pinf_v, int64_t& ninf_v) {
  constexpr bool kF32 = KIND == CK_F32;
  const int lane = threadIdx.x & 63;
#pragma unroll 1
  for (int j = 0; j < 8; ++j) {
    const int32_t left = rem - 64 * j;
    if (left <= 0) break;
    const int64_t r = base + 64 * j;
    uint64_t mj = ~0ull;
    {
      const int64_t w = r >> 5;
      const bool two = left > 32;
      if (validity) mj = ((uint64_t)(two ? ((const_u32s)validity)[w + 1] : 0u) << 32) | ((const_u32s)validity)[w];
      if (mask) mj &= ((uint64_t)(two ? ((const_u32s)mask)[w + 1] : 0u) << 32) | ((const_u32s)mask)[w];
      if (left < 64) mj &= (1ull << left) - 1ull;
    }
    uint64_t b;
    double xv;
    if constexpr (kF32) {
      b = __builtin_amdgcn_raw_buffer_load_b32(vr, vo + j * 256, 0, 2 /* nt */);
      xv = (double)__builtin_bit_cast(float, (uint32_t)b);
    } else {
      const auto w2 = __builtin_amdgcn_raw_buffer_load_b64(vr, vo + j * 512, 0, 2 /* nt */);
      b = ((uint64_t)w2[1] << 32) | w2[0];
      xv = __builtin_bit_cast(double, b);
    }
    const uint64_t nf = __builtin_amdgcn_ballot_w64(!__builtin_isfinite(xv)) & mj;
    const uint64_t nanm = __builtin_amdgcn_ballot_w64(xv != xv) & mj;
    const uint64_t inf = nf & ~nanm, pinf = __builtin_amdgcn_ballot_w64(xv > 0.0) & inf;
    if (lane == 0) {
      nan_v += __builtin_popcountll(nanm);
      pinf_v += __builtin_popcountll(pinf);
      ninf_v += __builtin_popcountll(inf & ~pinf);
    }
    if (STATS) {
      const uint64_t mm = mj & ~inf;
      cnt_w += __builtin_popcountll(mm);
      masked_moments<false, true>(a, s.fmin, s.fmax, xv, b, shift, mm, mj & ~nanm);
    } else {
      cnt_w += __builtin_popcountll(mj);
    }
    if (HLL) {
      if (lane_bit(nanm)) b = kF32 ? 0x7FC00000ull : 0x7FF8000000000000ull;
      const HllKey key = kF32 ? hll_key_int((uint32_t)b) : hll_key_long(b);
      if (lane_bit(mj)) {
        if (key.q >= 0) atomicMax(reinterpret_cast<int32_t*>(reinterpret_cast<char*>(regs) + key.addr), key.q);
        else hll_update(regs, kF32 ? xxh64_int((uint32_t)b) : xxh64_long(b));
      }
    }
  }
}

// Numeric column (f64 / f32 / i64 / i32 / i16 / i8): each wave takes 512-row blocks, lane l holding rows
// base + 64 j + l (j < 8): coalesced 512-byte (8-byte types) loads per instruction, selection masks
// in SGPRs.  Per row: stats as shifted sums (STATS), XXH64 + exec-masked LDS register max (HLL).
//
// Non-finite fp64 values.  With moments (STATS) the common pass does not classify values at all: a selected
// NaN / +-inf makes the wave's shifted sums non-finite (as does a finite value whose square overflows), which
// the workgroup checks at the range's end; if any wave saw one, the workgroup resets its HLL registers and
// re-runs the range in the checked form (float_block_checked: canonical NaN hash, +-inf out of the moments,
// counts) -- one VALU per value less on the common path.  Without moments (HLL only) each value is
// classified (one v_cmp_class) and a block holding a selected non-finite value takes the checked form.
template <int K> struct KindT { using T = double; };
template <> struct KindT<CK_I64> { using T = int64_t; };
template <> struct KindT<CK_I32> { using T = int32_t; };
template <> struct KindT<CK_F32> { using T = float; };
template <> struct KindT<CK_I16> { using T = int16_t; };
template <> struct KindT<CK_I8> { using T = int8_t; };

template <int KIND, bool STATS, bool HLL>
__device__ void numeric_range(const void* values, const uint32_t* validity, const uint32_t* mask,
                              int64_t row0, int64_t row1, ColStats& s, int32_t* regs) {
  using T = typename KindT<KIND>::T;
  constexpr bool kLazy = ck_float(KIND) && STATS;  // non-finite values found from the sums at the range's end
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const T* v = reinterpret_cast<const T*>(values);
  // values of [row0, row1) through a bounds-checked buffer resource: the row offset in voffset (lane + block
  // row; the row group's 64 j folds into the instruction's immediate offset) -- the descriptor's range check
  // covers voffset + immediate, so rows past row1 read 0 (they are masked out) and nothing past the column is
  // touched.  dq_scan bounds a chunk to < 2^31 rows, so a range is < 2^31 bytes.
  const __amdgpu_buffer_rsrc_t vr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<T*>(v + row0), (short)0, (int)((row1 - row0) * (int64_t)sizeof(T)), 0x00020000);
  // counts of selected NaN / +inf / -inf values, kept by lane 0 in VGPRs (as wave-uniform SGPR
  // counters they pushed the loop's SGPR pressure into spills)
  int64_t nan_v = 0, pinf_v = 0, ninf_v = 0;
  int64_t cnt_w = 0;  // wave-uniform count of the rows in the moments (STATS) / selected rows (HLL only)
  LaneMoments a{0.0, 0.0, 0};
  const double shift = STATS ? range_shift_of<KIND>(vr, validity, mask, row0, row1, lane) : 0.0;
  int32_t qmin = 0;
  const int32_t nr = (int32_t)(row1 - row0);  // range-relative rows: 32-bit (scalar) loop control and compares
  for (int32_t rb = 0; rb < nr; rb += kRowsPerIter) {
    const int64_t base = row0 + rb + wave * 512;
    const int32_t rem = nr - rb - wave * 512;  // rows of the range from this wave's block on
    const bool full = rb + kRowsPerIter <= nr;
    uint64_t bits[8], m[8];
    double x[8];
    const int32_t vo = (rb + wave * 512 + lane) * (int32_t)sizeof(T);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (sizeof(T) == 8) {
        const auto w2 = __builtin_amdgcn_raw_buffer_load_b64(vr, vo + j * 512, 0, 2 /* nt */);
        bits[j] = ((uint64_t)w2[1] << 32) | w2[0];
        if (KIND == CK_F64) x[j] = __builtin_bit_cast(double, bits[j]);
        else x[j] = __builtin_fma((double)(int32_t)w2[1], 4294967296.0, (double)w2[0]);  // exact int64 -> double
      } else if constexpr (KIND == CK_F32) {  // FloatType: Spark's Cast(child, DoubleType) is exact
        const uint32_t w = __builtin_amdgcn_raw_buffer_load_b32(vr, vo + j * 256, 0, 2 /* nt */);
        bits[j] = w;
        x[j] = (double)__builtin_bit_cast(float, w);
      } else {  // IntegerType / ShortType / ByteType: sign-extending loads (buffer_load_sshort / sbyte)
        int32_t w;
        if constexpr (sizeof(T) == 4) w = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(vr, vo + j * 256, 0, 2 /* nt */);
        else if constexpr (sizeof(T) == 2) w = (int16_t)__builtin_amdgcn_raw_buffer_load_b16(vr, vo + j * 128, 0, 2 /* nt */);
        else w = (int8_t)__builtin_amdgcn_raw_buffer_load_b8(vr, vo + j * 64, 0, 2 /* nt */);
        bits[j] = (uint64_t)(int64_t)w;
        x[j] = (double)w;
      }
    }
    block_masks(validity, mask, base, rem, full, m);
    // HLL-only fp64: one v_cmp_class per value (NaN or +-inf); only their OR stays live on the common path
    // (keeping the 8 masks for the rare path spilled SGPRs into v_writelane / v_readlane on every block)
    uint64_t nf_any = 0;
    if constexpr (ck_float(KIND) && !kLazy) {
#pragma unroll
      for (int j = 0; j < 8; ++j) nf_any |= __builtin_amdgcn_ballot_w64(!__builtin_isfinite(x[j])) & m[j];
    }
    if (ck_float(KIND) && !kLazy && nf_any != 0) {
      float_block_checked<KIND, STATS, HLL>(vr, validity, mask, base, rem, vo, shift, s, a, regs, cnt_w, nan_v, pinf_v,
                                            ninf_v);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) cnt_w += __builtin_popcountll(m[j]);
      numeric_block<KIND, STATS, HLL>(x, bits, m, shift, s, a, regs, qmin);
    }
  }
  if constexpr (kLazy) {
    // a selected non-finite value (or an overflowing square) in any wave: the workgroup re-runs the range in
    // the checked form from fresh registers (the common pass hashed a NaN by its raw bits)
    __shared__ int32_t redo;
    if (threadIdx.x == 0) redo = 0;
    __syncthreads();
    const bool bad = !__builtin_isfinite(a.sd) || !__builtin_isfinite(a.sdd);
    if (__builtin_amdgcn_ballot_w64(bad) != 0 && lane == 0) redo = 1;
    __syncthreads();
    if (redo) {
      if (HLL) {
        for (int i = threadIdx.x; i < 512; i += kBlock) regs[i] = -1;
      }
      stats_init(s);
      a = LaneMoments{0.0, 0.0, 0};
      cnt_w = 0;
      __syncthreads();
      for (int32_t rb = 0; rb < nr; rb += kRowsPerIter) {
        const int32_t vo = (rb + wave * 512 + lane) * (int32_t)sizeof(T);
        float_block_checked<KIND, STATS, HLL>(vr, validity, mask, row0 + rb + wave * 512, nr - rb - wave * 512, vo,
                                              shift, s, a, regs, cnt_w, nan_v, pinf_v, ninf_v);
      }
    }
  }
  if (STATS) {
    // the wave's moments from its lanes' shifted sums (fixed butterfly order: deterministic); lane 0 holds
    // them, the other lanes only min / max (n = 0: neutral in stats_merge)
    const double S1 = wave_sum_f64(a.sd), S2 = wave_sum_f64(a.sdd);
    const int64_t is = ck_float(KIND) ? 0 : wave_sum_i64(a.is);
    if (lane == 0 && cnt_w > 0) {
      const double n = (double)cnt_w, q = S1 / n;
      s.n = n;
      s.mean = shift + q;
      const double m2 = __builtin_fma(-S1, q, S2);
      s.m2 = m2 < 0.0 ? 0.0 : m2;  // rounding can leave a constant column's m2 at -ulp; a NaN stays NaN
      if (ck_float(KIND)) s.sum = __builtin_fma(n, shift, S1);
      else s.isum = is;
    }
  }
  if (lane == 0) s.count += cnt_w;
  if (ck_float(KIND) && lane == 0) {
    s.nan_count += nan_v;
    s.pinf += pinf_v;
    s.ninf += ninf_v;
    if (STATS) s.count += pinf_v + ninf_v;  // the moments counted only the finite / NaN rows
  }
}

// ------------------------------------------------------------------------------------------
// DataType classification of a string value (catalyst/StatefulDataType.scala:36-38, 62-67): the
// first of FRACTIONAL ^(-|\+)? ?\d*\.\d*$, INTEGRAL ^(-|\+)? ?\d*$, BOOLEAN ^(true|false)$ that
// matches the whole value, else STRING.  The patterns only accept ASCII and Java's \d is [0-9], so
// matching the UTF-8 bytes is the same as matching the decoded Java string (any byte >= 0x80, an
// invalid sequence, a NUL or a trailing newline makes the value a STRING).
// ------------------------------------------------------------------------------------------
enum DtClass : uint32_t { DT_FRACTIONAL = 1, DT_INTEGRAL = 2, DT_BOOLEAN = 3, DT_STRING = 4 };

__device__ __forceinline__ uint32_t dt_class_of(bool numeric, uint32_t dots, bool boolean) {
  return numeric && dots <= 1 ? (dots ? DT_FRACTIONAL : DT_INTEGRAL) : (boolean ? DT_BOOLEAN : DT_STRING);
}

// bit 7 of every byte i of a dword with lo <= i < hi
__device__ __forceinline__ uint32_t dt_keep(int lo, int hi) {
  const uint32_t below_hi = hi >= 4 ? 0x80808080u : (hi <= 0 ? 0u : 0x80808080u & ((1u << (8 * hi)) - 1u));
  const uint32_t from_lo = lo <= 0 ? 0x80808080u : (lo >= 4 ? 0u : 0x80808080u & ~((1u << (8 * lo)) - 1u));
  return below_hi & from_lo;
}

// A string of len <= 28 bytes given as little-endian dwords w[0..6] (bytes past len: anything).
// SWAR per dword: bit 7 of ((t & 0x7F..) + 0x76..) | t, t = w ^ '0'.., is set for the bytes that are
// not digits; the same with '.' and + 0x7F.. for the bytes that are not dots.  The dword loop stops as
// soon as no lane of the wave can still be numeric (text columns: after one dword).
__device__ __forceinline__ uint32_t dt_class_short(const uint32_t (&w)[8], uint32_t len, bool active) {
  const uint32_t b0 = w[0] & 0xFFu;
  const uint32_t sgn = (len > 0 && (b0 == 0x2Bu || b0 == 0x2Du)) ? 1u : 0u;  // '+' / '-'
  const uint32_t start = sgn + ((sgn < len && ((w[0] >> (8 * sgn)) & 0xFFu) == 0x20u) ? 1u : 0u);  // ' '
  uint32_t bad = 0, dots = 0;
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    if (k > 0 && __builtin_amdgcn_ballot_w64(active && bad == 0 && dots <= 1 && (uint32_t)(4 * k) < len) == 0) break;
    const uint32_t keep = dt_keep((int)start - 4 * k, (int)len - 4 * k);
    const uint32_t t = w[k] ^ 0x30303030u, z = w[k] ^ 0x2E2E2E2Eu;
    const uint32_t nd = ((t & 0x7F7F7F7Fu) + 0x76767676u) | t;
    const uint32_t nz = ((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z;
    bad |= nd & nz & keep;
    dots += __builtin_popcount(~nz & keep);
  }
  const bool boolean = (len == 4 && w[0] == 0x65757274u) ||                            // "true"
                       (len == 5 && w[0] == 0x736C6166u && (w[1] & 0xFFu) == 0x65u);   // "false"
  return dt_class_of(bad == 0, dots, boolean);
}

// Any length, byte by byte (the rare path: strings longer than 28 bytes or at the end of the data).
__device__ uint32_t dt_class_bytes(const uint8_t* p, int64_t len) {
  int64_t i = 0;
  if (len > 0 && (p[0] == '+' || p[0] == '-')) i = 1;
  if (i < len && p[i] == ' ') ++i;
  bool numeric = true;
  uint32_t dots = 0;
  for (; i < len && numeric; ++i) {
    const uint8_t c = p[i];
    if (c == '.') ++dots;
    else if (c < '0' || c > '9') numeric = false;
  }
  const bool boolean = (len == 4 && p[0] == 't' && p[1] == 'r' && p[2] == 'u' && p[3] == 'e') ||
                       (len == 5 && p[0] == 'f' && p[1] == 'a' && p[2] == 'l' && p[3] == 's' && p[4] == 'e');
  return dt_class_of(numeric, dots, boolean);
}

// Per-lane DataType counters of the selected values (STRING = count - the others, NULL = rows - count).
struct DtCounts {
  uint32_t frac = 0, integ = 0, boolean = 0;
  __device__ __forceinline__ void add(uint32_t cls, bool sel) {
    frac += sel && cls == DT_FRACTIONAL;
    integ += sel && cls == DT_INTEGRAL;
    boolean += sel && cls == DT_BOOLEAN;
  }
  // into the UTF8 task's otherwise unused additive ColStats fields (merged by stats_merge / finalize)
  __device__ __forceinline__ void flush(ColStats& s) const {
    s.isum += frac;
    s.nan_count += integ;
    s.sum += (double)boolean;
  }
};

// UTF8 column: lane l of a wave takes rows base + 64 j + l (j < 8) of its 512-row block, so the
// selection masks are scalar bitmap words (as in numeric_range).  Offsets come through a
// bounds-checked buffer resource over offsets[row0 .. row1]; every lane fetches its string with two
// dword-aligned 16-byte buffer loads (byte-granular loads are exact on gfx950 but run at ~60% of the
// aligned rate) from a window over the chunk's string bytes, realigns them with v_alignbit and hashes
// the string branch-free as one of <= 28 bytes (xxh64_short_head; byte rounds read b * P5 from the
// LDS table p5).  A string that is longer, or whose 32-byte window would cross the end of the chunk's
// bytes, is flagged in an SGPR mask and rehashed by the general XXH64 loop after the block (rare;
// ds_max is idempotent, so the block's selected rows are simply redone there).
//
// Strings of 24..28 bytes (three stripe rounds; 1 in 17 of C5's 8..24-byte strings) are deferred: the
// block loop runs two stripe rounds for every lane, and a selected lane that needs the third pushes
// its state (h, the third stripe word, the tail dword, len) into a per-wave LDS queue (SoA, kDefCap
// slots); every 64 queued strings are finished together (third round, tail, HLL update), so the third
// round costs one packed pass per 64 strings instead of a masked round in every lane of every row.
#ifndef DQ_STR_AHEAD
#define DQ_STR_AHEAD 2
#endif
constexpr int kStrAhead = DQ_STR_AHEAD;  // string windows in flight ahead of the one being hashed (1..7)
constexpr uint32_t kDefCap = 128;  // < 64 left after a drain + <= 64 pushed per row group
constexpr int kDefFields = 6;      // h lo, h hi, w4, w5, w6, len
// Round 6: the short-string hash by stripe-count class.  The block loop loads and realigns
// every string's window in row order as before, then pushes each selected string's window into one of two
// per-wave LDS stacks -- class A: < 16 bytes (at most one 8-byte round), class B: 16..28 bytes (two, the third
// deferred as before) -- and hashes a class 64 strings at a time once it holds 64: NULL rows never reach a
// hash, and class A never runs the second round that a wave of mixed lengths otherwise runs for all 64 lanes.
// Class A entries: the 16 window bytes with len in byte 15 (unused below 16 bytes); class B: bytes 0..27 + len.
#ifndef DQ_STR_CLS
#define DQ_STR_CLS 0
#endif
// Capacities: a class is hashed once it holds >= 64 (so < 64 are left); a push that would overflow it first
// hashes what it holds (partial: only when one row group brings > kClsCap - 64 of a class, i.e. > 32).  96
// entries per class and 96 deferred strings keep the string pass at 5 workgroups (waves per SIMD) per CU:
// 5 x (4.4 KB + 4 x 6.75 KB) of the 160 KB LDS.
constexpr uint32_t kClsCap = 96;
constexpr uint32_t kClsWords = kClsCap * (4 + 8);     // per wave: A quads, then B's two quad arrays
constexpr uint32_t kDefCapCls = 96;                   // the deferred queue of the class instantiation

// 32 bytes from byte `pos` of a window resource as little-endian dwords: three 16-byte loads from pos & ~3,
// realigned with v_alignbyte
__device__ __forceinline__ void load_bytes32(__amdgpu_buffer_rsrc_t rsrc, uint32_t pos, uint32_t (&w)[8]) {
  const int32_t a0 = (int32_t)(pos & ~3u);
  const u32x4 q0 = __builtin_amdgcn_raw_buffer_load_b128(rsrc, a0, 0, 0);
  const u32x4 q1 = __builtin_amdgcn_raw_buffer_load_b128(rsrc, a0 + 16, 0, 0);
  const u32x4 q2 = __builtin_amdgcn_raw_buffer_load_b128(rsrc, a0 + 32, 0, 0);
  const uint32_t d[9] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x};
#pragma unroll
  for (int k = 0; k < 8; ++k) w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], pos);
}

// XXH64.hashUnsafeBytes (up to fmix_head) of the n bytes at byte `rel` of a window resource, for the LONG string
// pass's rare path: 32-byte stripes from 16-byte loads (a lane leaves the loop after its last stripe), the merge,
// then the remainder's rounds (dq_hash.h xxh64_rem_head; xxh64_upto63_head is the same formulation on the host).
// Every load lies below ((rel + (n & ~31)) & ~3) + 48, which the caller keeps inside the resource.
template <typename BP>
__device__ uint64_t xxh64_window_head(__amdgpu_buffer_rsrc_t rsrc, uint32_t rel, uint32_t n, BP bp) {
  uint64_t h = kSeed + XP5;
  uint32_t pos = rel;
  if (n >= 32) {
    uint64_t v[4] = {kXxhV0, kXxhV1, kXxhV2, kXxhV3};
    const uint32_t end = rel + (n & ~31u);
    do {
      uint32_t w[8];
      load_bytes32(rsrc, pos, w);
      xxh64_stripe32(v, w);
      pos += 32;
    } while (pos < end);
    h = xxh64_merge4(v);
  }
  uint32_t t[8];
  load_bytes32(rsrc, pos, t);
  return xxh64_rem_head(h + (uint64_t)n, t, n & 31u, bp);
}

template <typename OffT, bool HLL, bool DT, bool LONG>
__device__ void utf8_range(const uint8_t* data, const OffT* offsets, const uint32_t* validity,
                           const uint32_t* mask, int64_t row0, int64_t row1, int64_t n_rows, ColStats& s,
                           int32_t* regs, const uint64_t* p5, uint32_t* dq, uint32_t* rare, uint32_t* cls) {
  constexpr bool CLS = DQ_STR_CLS && HLL && !DT && !LONG;
  constexpr uint32_t DCAP = CLS ? kDefCapCls : kDefCap;  // the deferred queue's capacity (its SoA stride)
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (row0 >= row1) return;
  constexpr int W = (int)sizeof(OffT);
  // byte window [lo, end of the chunk's strings) with 32-bit offsets from lo: int32 offsets address
  // the chunk's bytes directly (lo = 0, a UTF8 chunk holds < 2 GiB); int64 offsets from this range's
  // first string (dword-aligned)
  const int64_t lo = W == 4 ? 0 : ((int64_t)offsets[row0] & ~int64_t(3));
  const int64_t span = (int64_t)offsets[n_rows] - lo;
  const bool fast_ok = span < (int64_t)0x7FFFFF00;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(data + lo), (short)0, fast_ok ? (int)span : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<OffT*>(offsets + row0), (short)0, (int)((row1 - row0 + 1) * W), 0x00020000);
  const int32_t win = fast_ok ? (int32_t)span - 32 : -1;  // fast iff off <= win: both loads in range
  int64_t cnt_w = 0;  // wave-uniform count of selected rows
  int32_t qmin = 0;
  DtCounts dtc;
  const auto bp = [p5](uint32_t b) { return p5[b]; };
  const int32_t win3 = win < 0 ? -1 : (win | 3);  // (rel & ~3) <= win  <=>  rel <= win | 3
  if constexpr (LONG) {
    // Columns of mostly long strings: every selected row hashed once from 16-byte loads (xxh64_window_head:
    // the 32-byte stripe loop for the long ones, the remainder rounds for all), no fast path to redo.  Row
    // j + 1's offsets are loaded while row j is hashed; the rows the fast path would have skipped are still
    // counted (dq_scan keeps this instantiation while they stay over 1 / 4096).
    auto offs = [&](int32_t vo, int j, OffT& a, OffT& b) {
      if constexpr (W == 4) {
        a = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(orsrc, vo + j * 256, 0, 0);
        b = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(orsrc, vo + j * 256 + 4, 0, 0);
      } else {
        const auto a0 = __builtin_amdgcn_raw_buffer_load_b64(orsrc, vo + j * 512, 0, 0);
        const auto a1 = __builtin_amdgcn_raw_buffer_load_b64(orsrc, vo + j * 512 + 8, 0, 0);
        a = (int64_t)(((uint64_t)a0[1] << 32) | a0[0]);
        b = (int64_t)(((uint64_t)a1[1] << 32) | a1[0]);
      }
    };
    const int32_t nr = (int32_t)(row1 - row0);
    for (int32_t rb = 0; rb < nr; rb += kRowsPerIter) {
      const int64_t base = row0 + rb + wave * 512;
      const int32_t rem = nr - rb - wave * 512;
      const bool full = rb + kRowsPerIter <= nr;
      const int32_t vo = (rb + wave * 512 + lane) * W;  // the lane's row of the block, from row0, in bytes
      uint64_t m[8];
      block_masks(validity, mask, base, rem, full, m);
      OffT na, nb;
      offs(vo, 0, na, nb);
#pragma unroll 1
      for (int j = 0; j < 8; ++j) {
        const OffT ca = na, cb = nb;
        if (j < 7) offs(vo, j + 1, na, nb);
        cnt_w += __builtin_popcountll(m[j]);
        const int64_t rel = (int64_t)ca - lo, n = (int64_t)cb - (int64_t)ca;
        const bool sel = lane_bit(m[j]);
        const uint64_t longm = __builtin_amdgcn_ballot_w64(sel && !(n <= 28 && rel <= (int64_t)win3));
        if (lane == 0 && longm != 0) atomicAdd(rare, (uint32_t)__builtin_popcountll(longm));
        if (sel) {
          if constexpr (HLL) {
            if (win >= 0 && (((rel + (n & ~int64_t(31))) & ~int64_t(3)) + 48 <= (int64_t)win + 32)) {
              const uint64_t b = xxh64_window_head(rsrc, (uint32_t)rel, (uint32_t)n, bp);
              const HllKey key = hll_key_from_fmix(b);
              if (key.q >= 0) atomicMax(reinterpret_cast<int32_t*>(reinterpret_cast<char*>(regs) + key.addr), key.q);
              else hll_update(regs, fmix_tail(b));
            } else {
              hll_update(regs, xxh64_bytes(data, lo + rel, n));
            }
          }
          if constexpr (DT) {
            if (n <= 28 && win >= 0 && (rel & ~int64_t(3)) + 48 <= (int64_t)win + 32) {  // SWAR on the window
              uint32_t w8[8];
              load_bytes32(rsrc, (uint32_t)rel, w8);
              dtc.add(dt_class_short(w8, (uint32_t)n, true), true);
            } else {
              dtc.add(dt_class_bytes(data + lo + rel, n), true);
            }
          }
        }
      }
    }
    if (lane == 0) s.count += cnt_w;
    if constexpr (DT) dtc.flush(s);
    return;
  }
  // Software pipeline over the lane's rows j = 0..7 of each block, continuing into the next block:
  // row j + 4's offsets are loaded into the ring slot row j frees (kOffRing = 4 rows of offsets in
  // registers, loaded 4 rows before use), and the 32-byte windows of rows j + 1 .. j + kStrAhead are in
  // flight while row j is hashed.  Each row's exec-masked ds_max ends a basic block, so the order written
  // here is the issue order; the prefetches are unconditional (past row1 the descriptors read 0: a
  // conditional one makes the wait counts of both paths merge).
  constexpr int kOffRing = 4;
  OffT ra[kOffRing], rb[kOffRing];  // offsets o0, o1 of rows j .. j + 3 (slot = row & 3)
  // the row offset of a load in voffset (the block's lane row in a VGPR, set once per block; the row group's
  // 64 j W bytes in the instruction's immediate offset): the descriptor's range check covers voffset +
  // immediate, so the next block's prefetch past the range's last row reads 0 -- nothing past the offsets
  auto lane_off = [&](int64_t blk) -> int32_t { return (int32_t)((blk + (int64_t)wave * 512 - row0 + lane) * W); };
  // (round 4 A/B, profiles/r4_ab.txt r4g: the round-3 form with the row offset in soffset measured 1.916-1.919 vs
  // 1.902-1.907 ms per 125 M rows x 4)
  auto load_offsets = [&](int32_t vo, int j) {
    const int q = j & (kOffRing - 1);
    if constexpr (W == 4) {
      ra[q] = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(orsrc, vo + j * 256, 0, 0);
      rb[q] = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(orsrc, vo + j * 256 + 4, 0, 0);
    } else {
      const auto a0 = __builtin_amdgcn_raw_buffer_load_b64(orsrc, vo + j * 512, 0, 0);
      const auto a1 = __builtin_amdgcn_raw_buffer_load_b64(orsrc, vo + j * 512 + 8, 0, 0);
      ra[q] = (int64_t)(((uint64_t)a0[1] << 32) | a0[0]);
      rb[q] = (int64_t)(((uint64_t)a1[1] << 32) | a1[0]);
    }
  };
  int32_t vo_cur = lane_off(row0);
#pragma unroll
  for (int j = 0; j < kOffRing; ++j) load_offsets(vo_cur, j);
  // o0 rel. to the window (low 2 bits = the string's byte alignment) and len of the row in slot j & 3
  auto rel_of = [&](int j) -> uint32_t {
    const int q = j & (kOffRing - 1);
    return W == 4 ? (uint32_t)ra[q] : (uint32_t)((int64_t)ra[q] - lo);
  };
  auto len_of = [&](int j) -> uint32_t {
    const int q = j & (kOffRing - 1);
    const int64_t l = (int64_t)rb[q] - (int64_t)ra[q];
    return W == 4 ? (uint32_t)l : (l > 28 ? 29u : (uint32_t)l);
  };
  // the 32-byte windows of the next kStrAhead strings in flight (rows 0 .. kStrAhead - 1 of the first block)
  u32x4 win_a[kStrAhead], win_c[kStrAhead];
#pragma unroll
  for (int q = 0; q < kStrAhead; ++q) {
    win_a[q] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int32_t)(rel_of(q) & ~3u), 0, 0);
    win_c[q] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int32_t)(rel_of(q) & ~3u) + 16, 0, 0);
  }
  uint32_t qtail = 0;  // wave-uniform: deferred strings in dq[.][0, qtail)
  // finish deferred strings [0, n): third stripe round, tail, HLL register max (exact rank when the
  // high word does not carry it)
  auto drain = [&](uint32_t n) __attribute__((always_inline)) {
    if ((uint32_t)lane < n) {
      const uint64_t h = ((uint64_t)dq[1 * DCAP + lane] << 32) | dq[0 * DCAP + lane];
      const uint64_t k1 = ((uint64_t)dq[3 * DCAP + lane] << 32) | dq[2 * DCAP + lane];
      const uint64_t b = xxh64_tail_head(xxh64_stripe_round(h, k1), (uint64_t)dq[4 * DCAP + lane],
                                         dq[5 * DCAP + lane], bp);
      const HllKey key = hll_key_from_fmix(b);
      if (key.q >= 0) atomicMax(reinterpret_cast<int32_t*>(reinterpret_cast<char*>(regs) + key.addr), key.q);
      else hll_update(regs, fmix_tail(b));
    }
  };
  // the first 64, then the rest moves down (< 64 entries; one wave's LDS ops run in order)
  auto drain_full = [&]() __attribute__((always_inline)) {
    drain(64u);
    const uint32_t rest = qtail - 64u;
    if ((uint32_t)lane < rest) {
      uint32_t v[kDefFields];
#pragma unroll
      for (int f = 0; f < kDefFields; ++f) v[f] = dq[f * DCAP + 64 + lane];
#pragma unroll
      for (int f = 0; f < kDefFields; ++f) dq[f * DCAP + lane] = v[f];
    }
    qtail = rest;
  };
  // class stacks (CLS): the wave's entries [0, qa) of class A and [0, qb) of class B
  uint32_t qa = 0, qb = 0;
  // hash n <= 64 entries [top, top + n) of class A (isb false: at most one 8-byte round) or B (two rounds; a string of
  // 24..28 bytes goes on to the deferred queue for its third) -- one body for both classes (class A's lanes skip the
  // second round, so its waves skip it): the row loop has one drain site per row group, like its inline hash had
  auto cls_drain = [&](uint32_t top, uint32_t n, bool isb) __attribute__((always_inline)) {
    const bool act = (uint32_t)lane < n;
    uint32_t w[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    uint32_t L = 0;
    if (act) {
      if (isb) {
        const u32x4 q0 = reinterpret_cast<const u32x4*>(cls + 4 * kClsCap)[top + lane];
        const u32x4 q1 = reinterpret_cast<const u32x4*>(cls + 8 * kClsCap)[top + lane];
        w[0] = q0.x; w[1] = q0.y; w[2] = q0.z; w[3] = q0.w; w[4] = q1.x; w[5] = q1.y; w[6] = q1.z;
        L = q1.w;
      } else {
        const u32x4 q = reinterpret_cast<const u32x4*>(cls)[top + lane];
        w[0] = q.x; w[1] = q.y; w[2] = q.z; w[3] = q.w;
        L = q.w >> 24;
      }
    }
    uint64_t d4p;
    const uint64_t h2 = xxh64_stripes<2>(w, L, d4p);
    const uint64_t dm = __builtin_amdgcn_ballot_w64(act && L >= 24u);
    if (qtail + (uint32_t)__builtin_popcountll(dm) > DCAP) {  // (rare) make room: finish what the queue holds
      drain(qtail);
      qtail = 0;
    }
    if (dm != 0) {
      const uint32_t pos = qtail + __builtin_amdgcn_mbcnt_hi((uint32_t)(dm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)dm, 0u));
      if (lane_bit(dm)) {
        dq[0 * DCAP + pos] = (uint32_t)h2;
        dq[1 * DCAP + pos] = (uint32_t)(h2 >> 32);
        dq[2 * DCAP + pos] = (uint32_t)d4p;
        dq[3 * DCAP + pos] = (uint32_t)(d4p >> 32);
        dq[4 * DCAP + pos] = w[6];
        dq[5 * DCAP + pos] = L;
      }
      qtail += (uint32_t)__builtin_popcountll(dm);
    }
    if (act && L < 24u) {
      const uint64_t b = xxh64_tail_head(h2, d4p, L, bp);
      const HllKey key = hll_key_from_fmix(b);
      if (key.q >= 0) atomicMax(reinterpret_cast<int32_t*>(reinterpret_cast<char*>(regs) + key.addr), key.q);
      else hll_update(regs, fmix_tail(b));
    }
  };
  // drain what class A / B must give up before a push of na / nb entries: 64 once a class holds >= 64 (< 64 are
  // left), or everything when the push would overflow kClsCap (only a class with < 64 and > kClsCap - na); one
  // drain site (a rolled loop over the two classes)
  auto cls_make_room = [&](uint32_t na, uint32_t nb) __attribute__((always_inline)) {
    const uint32_t da = qa >= 64u ? 64u : (qa + na > kClsCap ? qa : 0u);
    const uint32_t db = qb >= 64u ? 64u : (qb + nb > kClsCap ? qb : 0u);
#pragma unroll 1
    for (int c = 0; c < 2; ++c) {
      const uint32_t n = c ? db : da;
      if (n == 0) continue;
      const uint32_t top = (c ? qb : qa) - n;
      cls_drain(top, n, c != 0);
      if (c) qb = top;
      else qa = top;
    }
    if (qtail >= 64u) drain_full();
  };
  // every 32-byte window of the range lies inside the chunk's bytes iff its last row's does (offsets only
  // grow): then no row needs the per-row window compare (all but the chunk's last range; one scalar load --
  // per block, its latency showed in the block loop)
  const bool wins_in = win >= 0 && (int32_t)((int64_t)offsets[row1 - 1] - lo) <= win3;
  const int32_t nr = (int32_t)(row1 - row0);  // range-relative rows: 32-bit (scalar) loop control and compares
  for (int32_t rb = 0; rb < nr; rb += kRowsPerIter) {
    const int64_t blk = row0 + rb;
    const int64_t base = blk + wave * 512;
    const int32_t rem = nr - rb - wave * 512;  // rows of the range from this wave's block on
    const bool full = rb + kRowsPerIter <= nr;
    const int32_t vo_next = lane_off(blk + kRowsPerIter);
    uint64_t m[8];  // selected rows that take the fast path (SGPR budget: the rare path reloads the masks)
    block_masks(validity, mask, base, rem, full, m);

    uint64_t slow = 0;  // OR of the selected rows that need the general hash
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      {  // selected rows that take the fast path (row j's offsets are in its ring slot)
        cnt_w += __builtin_popcountll(m[j]);
        // the compares' own masks (llvm.amdgcn.icmp; signedness from the predicate) ANDed in SGPRs: a
        // ballot of the combined bool materialises it in a VGPR and compares again (2 VALU per row)
        uint64_t fastm = __builtin_amdgcn_uicmp(len_of(j), 28u, 37 /* ICMP_ULE */);
        // (the round-3 compare on every row, no branch: 1.911-1.915 vs 1.902-1.907 ms, r4g)
        if (!wins_in) {  // a uniform branch (the chunk's last range): the compare, in asm so it is not hoisted
          uint64_t wm;
          asm volatile("v_cmp_le_i32_e64 %0, %1, %2" : "=s"(wm) : "v"(rel_of(j)), "s"(win3));
          fastm &= wm;
        }
        slow |= m[j] & ~fastm;
        m[j] &= fastm;
      }
      // the window of row j + kStrAhead (of the next block once j + kStrAhead >= 8): its offsets are in
      // ring slot (j + kStrAhead) & 3, so the windows stay in flight across block boundaries
      u32x4 an, cn;
      {
        const int32_t offn = (int32_t)(rel_of((j + kStrAhead) & 7) & ~3u);
        an = __builtin_amdgcn_raw_buffer_load_b128(rsrc, offn, 0, 0);
        cn = __builtin_amdgcn_raw_buffer_load_b128(rsrc, offn + 16, 0, 0);
      }
      const u32x4 a = win_a[0], c = win_c[0];
      const uint32_t d[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
      // (byte-granular unaligned window loads instead of this realignment -- 8 fewer VALU per string --
      // measured 2.70-2.73 vs 1.90-1.92 ms per 125 M rows x 4: the unaligned 16-byte loads are address-bound)
      // v_alignbyte reads the byte shift from the low 2 bits of rel = o0 & 3 (v_alignbit would need rel << 3)
      const uint32_t sh = rel_of(j);
      uint32_t wv[8];
#pragma unroll
      for (int k = 0; k < 7; ++k) wv[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
      wv[7] = d[7];  // only ever feeds the unused half of the tail pair for len >= 24
      if constexpr (DT) dtc.add(dt_class_short(wv, len_of(j), lane_bit(m[j])), lane_bit(m[j]));
      if constexpr (CLS) {
        // push the row group's selected fast-path strings by class: rank among the pushing lanes, class A from
        // qa up, class B from qb up (rank_B = rank - rank_A: one mbcnt pair less)
        const uint32_t L = len_of(j);
        const uint64_t mb = m[j] & __builtin_amdgcn_ballot_w64(L >= 16u);
        const uint64_t ma = m[j] & ~mb;
        cls_make_room((uint32_t)__builtin_popcountll(ma), (uint32_t)__builtin_popcountll(mb));
        const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(m[j] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m[j], 0u));
        const uint32_t ra = __builtin_amdgcn_mbcnt_hi((uint32_t)(ma >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ma, 0u));
        if (lane_bit(ma)) {
          u32x4 q;
          q.x = wv[0]; q.y = wv[1]; q.z = wv[2]; q.w = (wv[3] & 0x00FFFFFFu) | (L << 24);
          reinterpret_cast<u32x4*>(cls)[qa + ra] = q;
        } else if (lane_bit(mb)) {
          const uint32_t pb = qb + rk - ra;
          u32x4 q0, q1;
          q0.x = wv[0]; q0.y = wv[1]; q0.z = wv[2]; q0.w = wv[3];
          q1.x = wv[4]; q1.y = wv[5]; q1.z = wv[6]; q1.w = L;
          reinterpret_cast<u32x4*>(cls + 4 * kClsCap)[pb] = q0;
          reinterpret_cast<u32x4*>(cls + 8 * kClsCap)[pb] = q1;
        }
        qa += (uint32_t)__builtin_popcountll(ma);
        qb += (uint32_t)__builtin_popcountll(mb);
      } else if constexpr (HLL) {
        uint64_t d4p;
        const uint64_t h2 = xxh64_stripes<2>(wv, len_of(j), d4p);
        const uint64_t dm = m[j] & __builtin_amdgcn_ballot_w64(len_of(j) >= 24u);  // needs the third round
        if (dm != 0) {
          // position = qtail + the lane's rank among the pushing lanes (qtail joins the scalar LDS base: no
          // v_mov of it into the mbcnt)
          const uint32_t pos = qtail + __builtin_amdgcn_mbcnt_hi((uint32_t)(dm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)dm, 0u));
          if (lane_bit(dm)) {
            dq[0 * DCAP + pos] = (uint32_t)h2;
            dq[1 * DCAP + pos] = (uint32_t)(h2 >> 32);
            dq[2 * DCAP + pos] = (uint32_t)d4p;
            dq[3 * DCAP + pos] = (uint32_t)(d4p >> 32);
            dq[4 * DCAP + pos] = wv[6];
            dq[5 * DCAP + pos] = len_of(j);
          }
          qtail += (uint32_t)__builtin_popcountll(dm);
        }
        const HllKey key = hll_key_from_fmix(xxh64_tail_head(h2, d4p, len_of(j), bp));
        qmin = min(qmin, key.q);
        if (lane_bit(m[j] & ~dm)) atomicMax(reinterpret_cast<int32_t*>(reinterpret_cast<char*>(regs) + key.addr), key.q);
        if (qtail >= 64u) drain_full();
      }
      // row j + 4 into the slot row j frees (of the next block for j >= 4)
      if (j + kOffRing < 8) load_offsets(vo_cur, j + kOffRing);
      else load_offsets(vo_next, j + kOffRing - 8);
#pragma unroll
      for (int q = 0; q + 1 < kStrAhead; ++q) {
        win_a[q] = win_a[q + 1];
        win_c[q] = win_c[q + 1];
      }
      win_a[kStrAhead - 1] = an;
      win_c[kStrAhead - 1] = cn;
    }
    vo_cur = vo_next;
    // rare: long / window-crossing strings, or a rank that needs the hash's low word (2^-23).  The
    // HLL update is idempotent, so the block's selected rows are simply redone; DataType counts only
    // the rows the fast path skipped.  (Columns with many such rows run the LONG instantiation above.)
    if ((slow | __builtin_amdgcn_ballot_w64(qmin < 0)) != 0) {
      // the rows the fast path skipped, counted per row as the LONG instantiation counts them (`slow` is an OR
      // over the block's row groups, i.e. lanes, not rows), in the wave's LDS slot (no register across the
      // block loop)
      block_masks(validity, mask, base, rem, full, m);
      uint32_t skipped = 0;
#pragma unroll 1
      for (int j = 0; j < 8; ++j) {
        bool was_fast = true;
        if (lane_bit(m[j])) {
          const int64_t row = base + j * 64 + lane;
          const int64_t o0 = (int64_t)offsets[row], o1 = (int64_t)offsets[row + 1];
          was_fast = o1 - o0 <= 28 && o0 - lo <= (int64_t)win3;
          if constexpr (HLL) hll_update(regs, xxh64_bytes(data, o0, o1 - o0));
          if constexpr (DT) {
            if (!was_fast) dtc.add(dt_class_bytes(data + o0, o1 - o0), true);
          }
        }
        skipped += (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(!was_fast));
      }
      if (lane == 0 && skipped) atomicAdd(rare, skipped);
      qmin = 0;
    }
  }
  if constexpr (CLS) {  // the classes' last entries (each <= kClsCap: one or two drains)
#pragma unroll 1
    while (qa | qb) cls_make_room(kClsCap, kClsCap);
  }
  if constexpr (HLL) {
    if (qtail != 0) drain(qtail);
  }
  if (lane == 0) s.count += cnt_w;
  if constexpr (DT) dtc.flush(s);
}

// DataType of a double / float column: Spark casts the value to a string with Double.toString /
// Float.toString, which is plain decimal (matches FRACTIONAL) iff the value is finite and zero or
// 1e-3 <= |x| < 1e7 (the exact value: the float nearest 1e-3 lies above the double 1e-3, so the test
// in double is the float's), and otherwise "NaN", "Infinity" or computerized scientific notation
// ("1.0E7": a STRING).  Counts the selected rows (s.count) and the fractional ones (s.isum).
template <typename T>
__device__ void float_dtype_range(const T* values, const uint32_t* validity, const uint32_t* mask, int64_t row0,
                                  int64_t row1, ColStats& s) {
  // lane-per-row 512-row blocks as numeric_range: coalesced loads through a bounds-checked descriptor, the
  // selection as scalar lane masks, counts from popcounts (wave-uniform)
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const __amdgpu_buffer_rsrc_t vr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<T*>(values + row0), (short)0, (int)((row1 - row0) * (int64_t)sizeof(T)), 0x00020000);
  int64_t cnt = 0, frac = 0;
  const int32_t nr = (int32_t)(row1 - row0);
  for (int32_t rb = 0; rb < nr; rb += kRowsPerIter) {
    const int64_t base = row0 + rb + wave * 512;
    const int32_t rem = nr - rb - wave * 512;
    uint64_t m[8];
    block_masks(validity, mask, base, rem, rb + kRowsPerIter <= nr, m);
    const int32_t vo = (rb + wave * 512 + lane) * (int32_t)sizeof(T);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      double x;
      if constexpr (sizeof(T) == 8) {
        const auto w2 = __builtin_amdgcn_raw_buffer_load_b64(vr, vo + j * 512, 0, 2 /* nt */);
        x = __builtin_bit_cast(double, ((uint64_t)w2[1] << 32) | w2[0]);
      } else {
        x = (double)__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(vr, vo + j * 256, 0, 2 /* nt */));
      }
      const double a = __builtin_fabs(x);
      cnt += __builtin_popcountll(m[j]);
      frac += __builtin_popcountll(__builtin_amdgcn_ballot_w64(x == 0.0 || (a >= 1e-3 && a < 1e7)) & m[j]);
    }
  }
  if (lane == 0) {
    s.count += cnt;
    s.isum += frac;
  }
}

// BooleanType column: the selected rows (s.count) and the selected TRUE values (s.isum) from popcounts of the
// value / validity (& where) words; the workgroup's `any TRUE` / `any FALSE` (ApproxCountDistinct: Spark 2.2
// hashes a boolean as hashInt(1 / 0), so the registers follow from those two facts) go to flags[0] / flags[1].
__device__ void bool_range(const uint32_t* values, const uint32_t* validity, const uint32_t* mask, int64_t row0,
                           int64_t row1, ColStats& s, int32_t* flags) {
  const int64_t w0 = row0 >> 5, w1 = (row1 + 31) >> 5;  // row0 is a multiple of 2048
  int64_t c = 0, t = 0;
  for (int64_t w = w0 + threadIdx.x; w < w1; w += kBlock) {
    uint32_t sel = word_or_ones(validity, w);
    if (mask) sel &= mask[w];
    const int64_t r = w << 5;
    if (r + 32 > row1) sel &= (1u << (row1 - r)) - 1u;
    const uint32_t v = values[w];
    c += __popc(sel);
    t += __popc(sel & v);
  }
  s.count += c;
  s.isum += t;
  if (t) flags[0] = 1;
  if (c > t) flags[1] = 1;
}

// DecimalType column (ColTask::arg = precision | scale << 8; 16-byte two's-complement unscaled values):
// lane-per-row 512-row blocks with the selection as scalar lane masks, as numeric_range.  STATS: every selected value
// cast to double as Spark's Decimal.toDouble (correctly rounded, dq_decimal.h) into the shifted moments and min / max
// (the cast is monotone: min of the casts = the cast of Spark's decimal min), the exact 128-bit sum into (isum,
// isum_hi) and the fp64 sum of the casts into `sum` (dq_finish's overflow guard); HLL: Spark 2.2's decimal hash
// (hashLong of the unscaled long, or of BigInteger.toByteArray's bytes above precision 18); DT: the count of values
// whose BigDecimal.toString is plain decimal (isum) -- dq_finish makes them FRACTIONAL (scale > 0; the rest STRING)
// or all INTEGRAL (scale 0).  Rows past row1 are not read (exec-masked loads); values are 16-byte aligned.
template <bool STATS, bool HLL, bool DT>
__device__ void decimal_range(const void* values, const uint32_t* validity, const uint32_t* mask, int64_t row0,
                              int64_t row1, ColStats& s, int32_t* regs, int32_t arg) {
  const int prec = arg & 0xFF, sc = (arg >> 8) & 0xFF;
  const DecTab tab = dec_dev_tab();
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t* v = reinterpret_cast<const uint64_t*>(values);
  auto load = [&](int64_t r, uint64_t& lo, uint64_t& hi) {
    lo = hi = 0;
    if (r < row1) {
      lo = __builtin_nontemporal_load(v + 2 * r);
      hi = __builtin_nontemporal_load(v + 2 * r + 1);
    }
  };
  // the range's shift: mean of the casts of its first 64-row group with a selected value
  double shift = 0.0;
  if (STATS) {
    for (int64_t r = row0; r < row1; r += 64) {
      uint64_t sel = ~0ull;
      const int64_t w = r >> 5;
      const bool two = r + 32 < row1;
      if (validity) sel = ((uint64_t)(two ? ((const_u32s)validity)[w + 1] : 0u) << 32) | ((const_u32s)validity)[w];
      if (mask) sel &= ((uint64_t)(two ? ((const_u32s)mask)[w + 1] : 0u) << 32) | ((const_u32s)mask)[w];
      if (r + 64 > row1) sel &= (1ull << (row1 - r)) - 1ull;
      if (sel == 0) continue;
      uint64_t lo, hi;
      load(r + lane, lo, hi);
      const double x = lane_bit(sel) ? dec_to_double(lo, hi, sc, tab, prec <= 18) : 0.0;
      shift = wave_uniform(wave_sum_f64(x) / (double)__builtin_popcountll(sel));
      break;
    }
  }
  LaneMoments a{0.0, 0.0, 0};
  uint64_t slo = 0, shi = 0;  // the lane's exact sum (128-bit, wrapping)
  double guard = 0.0;
  int64_t cnt_w = 0, frac = 0;
  const int32_t nr = (int32_t)(row1 - row0);
  for (int32_t rb = 0; rb < nr; rb += kRowsPerIter) {
    const int64_t base = row0 + rb + wave * 512;
    const int32_t rem = nr - rb - wave * 512;
    uint64_t m[8];
    block_masks(validity, mask, base, rem, rb + kRowsPerIter <= nr, m);
    uint64_t lo[8], hi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) load(base + 64 * j + lane, lo[j], hi[j]);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      cnt_w += __builtin_popcountll(m[j]);
      const bool sel = lane_bit(m[j]);
      if constexpr (STATS) {
        const double x = dec_to_double(lo[j], hi[j], sc, tab, prec <= 18);
        masked_moments<false, false>(a, s.fmin, s.fmax, x, 0, shift, m[j], m[j]);
        if (sel) {
          const uint64_t l2 = slo + lo[j];
          shi += hi[j] + (l2 < slo ? 1u : 0u);
          slo = l2;
          guard += x;
        }
      }
      if constexpr (HLL) {
        const uint64_t b = dec_hash_head(lo[j], hi[j], prec);
        const HllKey key = hll_key_from_fmix(b);
        if (sel) {
          if (key.q >= 0) atomicMax(reinterpret_cast<int32_t*>(reinterpret_cast<char*>(regs) + key.addr), key.q);
          else hll_update(regs, fmix_tail(b));
        }
      }
      if constexpr (DT) frac += __builtin_popcountll(__builtin_amdgcn_ballot_w64(dec_dt_class(lo[j], hi[j], sc, tab) == 1) & m[j]);
    }
  }
  if constexpr (STATS) {
    const double S1 = wave_sum_f64(a.sd), S2 = wave_sum_f64(a.sdd), G = wave_sum_f64(guard);
#pragma unroll
    for (int k = 32; k >= 1; k >>= 1) {
      const uint64_t olo = __shfl_xor(slo, k), ohi = __shfl_xor(shi, k);
      const uint64_t l2 = slo + olo;
      shi = shi + ohi + (l2 < slo ? 1u : 0u);
      slo = l2;
    }
    if (lane == 0 && cnt_w > 0) {
      const double n = (double)cnt_w, q = S1 / n;
      s.n = n;
      s.mean = shift + q;
      const double m2 = __builtin_fma(-S1, q, S2);
      s.m2 = m2 < 0.0 ? 0.0 : m2;
      s.sum = G;
      s.isum = (int64_t)slo;
      s.isum_hi = (int64_t)shi;
    }
  }
  if (lane == 0) {
    s.count += cnt_w;
    if (DT) s.isum += frac;
  }
}

// Only the count of selected rows (Completeness): popcount of validity (& where) words.
__device__ void validity_range(const uint32_t* validity, const uint32_t* mask, int64_t row0, int64_t row1, ColStats& s) {
  // row0 is a multiple of 2048 -> word aligned; each thread handles whole 32-row words
  const int64_t w0 = row0 >> 5, w1 = (row1 + 31) >> 5;
  int64_t c = 0;
  for (int64_t w = w0 + threadIdx.x; w < w1; w += kBlock) {
    uint32_t bits = word_or_ones(validity, w);
    if (mask) bits &= mask[w];
    const int64_t r = w << 5;
    if (r + 32 > row1) bits &= (1u << (row1 - r)) - 1u;
    c += __popc(bits);
  }
  s.count += c;
}

template <int KIND, bool STATS, bool HLL>
__device__ void run_numeric(const ColTask& t, const ScanCols& cols, const ScanBitmaps& bm, int64_t row0, int64_t row1,
                            ColStats& s, int32_t* regs) {
  const uint32_t* mask = t.where >= 0 ? reinterpret_cast<const uint32_t*>(bm.where_bits[t.where]) : nullptr;
  numeric_range<KIND, STATS, HLL>(cols.values[t.col], cols.validity[t.col], mask, row0, row1, s, regs);
}

// ------------------------------------------------------------------------------------------
// Kernel 2: single-column tasks.  One kernel instantiation per variant (kind x accumulators), so
// each launch carries only its own inner loop (small I-cache footprint); the tasks of one variant
// share a launch, interleaved task-fastest: workgroup b -> task b % ntasks, row range b / ntasks.
// ------------------------------------------------------------------------------------------
template <int V, bool LONG>
__device__ __forceinline__ void run_variant(const ColTask& t, const ScanCols& cols, const uint32_t* mask, int64_t row0,
                                            int64_t row1, int64_t n_rows, ColStats& s, int32_t* regs,
                                            const uint64_t* p5, uint32_t* dq, uint32_t* rare, uint32_t* cls) {
  const void* v = cols.values[t.col];
  const uint32_t* val = cols.validity[t.col];
  if constexpr (V == CV_VALIDITY) validity_range(val, mask, row0, row1, s);
  else if constexpr (V == CV_F64_S) numeric_range<CK_F64, true, false>(v, val, mask, row0, row1, s, regs);
  else if constexpr (V == CV_F64_SH) numeric_range<CK_F64, true, true>(v, val, mask, row0, row1, s, regs);
  else if constexpr (V == CV_F64_H) numeric_range<CK_F64, false, true>(v, val, mask, row0, row1, s, regs);
  else if constexpr (V == CV_I64_S) numeric_range<CK_I64, true, false>(v, val, mask, row0, row1, s, regs);
  else if constexpr (V == CV_I64_SH) numeric_range<CK_I64, true, true>(v, val, mask, row0, row1, s, regs);
  else if constexpr (V == CV_I64_H) numeric_range<CK_I64, false, true>(v, val, mask, row0, row1, s, regs);
  else if constexpr (V == CV_I32_S) numeric_range<CK_I32, true, false>(v, val, mask, row0, row1, s, regs);
  else if constexpr (V == CV_I32_SH) numeric_range<CK_I32, true, true>(v, val, mask, row0, row1, s, regs);
  else if constexpr (V == CV_I32_H) numeric_range<CK_I32, false, true>(v, val, mask, row0, row1, s, regs);
  else if constexpr (V == CV_F32_S) numeric_range<CK_F32, true, false>(v, val, mask, row0, row1, s, regs);
  else if constexpr (V == CV_F32_SH) numeric_range<CK_F32, true, true>(v, val, mask, row0, row1, s, regs);
  else if constexpr (V == CV_F32_H) numeric_range<CK_F32, false, true>(v, val, mask, row0, row1, s, regs);
  else if constexpr (V == CV_I16_S) numeric_range<CK_I16, true, false>(v, val, mask, row0, row1, s, regs);
  else if constexpr (V == CV_I16_SH) numeric_range<CK_I16, true, true>(v, val, mask, row0, row1, s, regs);
  else if constexpr (V == CV_I16_H) numeric_range<CK_I16, false, true>(v, val, mask, row0, row1, s, regs);
  else if constexpr (V == CV_I8_S) numeric_range<CK_I8, true, false>(v, val, mask, row0, row1, s, regs);
  else if constexpr (V == CV_I8_SH) numeric_range<CK_I8, true, true>(v, val, mask, row0, row1, s, regs);
  else if constexpr (V == CV_I8_H) numeric_range<CK_I8, false, true>(v, val, mask, row0, row1, s, regs);
  else if constexpr (V == CV_F64_D) float_dtype_range(reinterpret_cast<const double*>(v), val, mask, row0, row1, s);
  else if constexpr (V == CV_F32_D) float_dtype_range(reinterpret_cast<const float*>(v), val, mask, row0, row1, s);
  else if constexpr (V == CV_BOOL) bool_range(reinterpret_cast<const uint32_t*>(v), val, mask, row0, row1, s, regs);
  else if constexpr (V == CV_D128_S) decimal_range<true, false, false>(v, val, mask, row0, row1, s, regs, t.arg);
  else if constexpr (V == CV_D128_SH) decimal_range<true, true, false>(v, val, mask, row0, row1, s, regs, t.arg);
  else if constexpr (V == CV_D128_H) decimal_range<false, true, false>(v, val, mask, row0, row1, s, regs, t.arg);
  else if constexpr (V == CV_D128_D) decimal_range<false, false, true>(v, val, mask, row0, row1, s, regs, t.arg);
  else if constexpr (V == CV_UTF8_H || V == CV_UTF8_D || V == CV_UTF8_HD)
    utf8_range<int32_t, V != CV_UTF8_D, V != CV_UTF8_H, LONG>(
        reinterpret_cast<const uint8_t*>(v), reinterpret_cast<const int32_t*>(cols.offsets[t.col]), val, mask, row0,
        row1, n_rows, s, regs, p5, dq, rare, cls);
  else
    utf8_range<int64_t, V != CV_LUTF8_D, V != CV_LUTF8_H, LONG>(
        reinterpret_cast<const uint8_t*>(v), reinterpret_cast<const int64_t*>(cols.offsets[t.col]), val, mask, row0,
        row1, n_rows, s, regs, p5, dq, rare, cls);
}

// Minimum waves per SIMD the register allocator must leave room for (0 = no constraint); a
// diagnostic build switch for the issue-bound string hash variants.
#ifndef DQ_STR_WAVES
#define DQ_STR_WAVES 6  // 80 VGPRs with the 4-row offset ring (81 unconstrained: 5 waves); A/B within 1 %
#endif
// fp64 / int64 stats+HLL: 6 waves per SIMD (80 VGPRs; the 2 spilled registers are reloaded only in the
// prologue / epilogue): f64 1.538 -> 1.522 ms per 125 M rows x 8 columns against the unconstrained 82
#ifndef DQ_NUM_WAVES
#define DQ_NUM_WAVES 6
#endif
template <int V, bool LONG>
constexpr int kMinWaves = V == CV_UTF8_H && !LONG && DQ_STR_CLS ? 5  // (the class stacks' LDS: 5 workgroups per CU)
                          : V == CV_UTF8_H && DQ_STR_WAVES > 0 ? DQ_STR_WAVES
                          : (V == CV_F64_SH || V == CV_I64_SH) && DQ_NUM_WAVES > 0 ? DQ_NUM_WAVES
                          : V == CV_LUTF8_H && LONG ? 5  // (the register window would otherwise cost a wave)
                                                    : 1;

// LONG: the string variants' rare path for columns of long strings (utf8_range)
template <int V, bool LONG = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kMinWaves<V, LONG>))) void dq_column_scan(const ColTask* __restrict__ tasks, int32_t ntasks,
                                                         int32_t part_base, ScanCols cols, ScanBitmaps bm,
                                                         int64_t n_rows, int64_t rows_per_range,
                                                         ColPartial* __restrict__ partials,
                                                         uint32_t* __restrict__ hll_acc) {
  constexpr bool kHll = !(V == CV_VALIDITY || V == CV_F64_S || V == CV_I64_S || V == CV_I32_S || V == CV_F64_D ||
                         V == CV_UTF8_D || V == CV_LUTF8_D || V == CV_F32_S || V == CV_I16_S || V == CV_I8_S ||
                         V == CV_F32_D || V == CV_BOOL || V == CV_D128_S || V == CV_D128_D);
  constexpr bool kBool = V == CV_BOOL;  // (its two HLL hashes are constants: flags instead of registers)
  constexpr bool kStr = V == CV_UTF8_H || V == CV_LUTF8_H || V == CV_UTF8_HD || V == CV_LUTF8_HD;
  __shared__ int32_t regs[kHll ? 512 : 2];  // q = pw - 1, -1 = empty (see hll_q_exact); CV_BOOL: any TRUE / FALSE
  __shared__ uint64_t p5[kStr ? 256 : 1];   // b * P5 for the byte rounds of the string hash
  constexpr uint32_t kDCap = DQ_STR_CLS && (V == CV_UTF8_H || V == CV_LUTF8_H) && !LONG ? kDefCapCls : kDefCap;
  __shared__ uint32_t dfq[kStr ? kWaves * kDefFields * kDCap : 1];  // deferred 24..28-byte strings
  __shared__ uint32_t rare[kStr ? kWaves : 1];  // per wave: the rows the string fast path skipped
  constexpr bool kCls = DQ_STR_CLS && (V == CV_UTF8_H || V == CV_LUTF8_H) && !LONG;
  __shared__ __attribute__((aligned(16))) uint32_t clsbuf[kCls ? kWaves * kClsWords : 4];  // class stacks
  __shared__ ColStats red[kWaves];
  const int32_t ti = blockIdx.x % ntasks;
  const int32_t range = blockIdx.x / ntasks;
  const ColTask t = tasks[ti];
  const int64_t row0 = (int64_t)range * rows_per_range;
  int64_t row1 = row0 + rows_per_range;
  if (row1 > n_rows) row1 = n_rows;
  if constexpr (kBool) {
    if (threadIdx.x < 2) regs[threadIdx.x] = 0;
    __syncthreads();
  }
  if constexpr (kHll) {
    for (int i = threadIdx.x; i < 512; i += kBlock) regs[i] = -1;
    if constexpr (kStr) {
      p5[threadIdx.x] = (uint64_t)threadIdx.x * XP5;
      if (threadIdx.x < kWaves) rare[threadIdx.x] = 0;
    }
    __syncthreads();
  }
  ColStats s;
  stats_init(s);
  const uint32_t* mask = t.where >= 0 ? reinterpret_cast<const uint32_t*>(bm.where_bits[t.where]) : nullptr;
  const int32_t wv = kStr ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0;
  run_variant<V, LONG>(t, cols, mask, row0, row1, n_rows, s, regs, p5, dfq + wv * kDefFields * kDCap, rare + wv,
                       clsbuf + (kCls ? wv * kClsWords : 0));
  block_reduce_store(s, partials + (size_t)(part_base + ti) * kMaxWG + range, red);
  if constexpr (kStr) {
    // the task's rare-path rows for dq_scan's choice of variant (finalize publishes them to the host)
    if (threadIdx.x == 0 && bm.rare_rows) {
      uint32_t r = 0;
      for (int w = 0; w < kWaves; ++w) r += rare[w];
      if (r) atomicAdd(reinterpret_cast<unsigned long long*>(bm.rare_rows + part_base + ti), (unsigned long long)r);
    }
  }
  if constexpr (kBool) {
    // (block_reduce_store's barrier ordered every thread's flag store before this read)
    if (threadIdx.x == 0 && t.hll_slot >= 0) {
      uint32_t* dst = hll_acc + ((size_t)t.hll_slot * kHllCopies + (blockIdx.x % kHllCopies)) * 512;
      for (int b = 0; b < 2; ++b) {
        if (!regs[b]) continue;
        const uint64_t x = xxh64_int(b == 0 ? 1u : 0u);  // hashInt(true -> 1, false -> 0)
        atomicMax(dst + (uint32_t)(x >> 55), (uint32_t)(hll_q_exact(x) + 1));
      }
    }
  }
  if constexpr (kHll) {
    // registers only grow: merge into the plan accumulator with device-scope atomicMax, skipping
    // registers the (possibly stale) accumulator already covers -- max is order-free, so the
    // result is deterministic.
    __syncthreads();
    // one of kHllCopies accumulator copies per workgroup: a one-column launch otherwise funnels every
    // workgroup's 512 atomics into the same 2 KB (dq_finish takes the max over the copies)
    uint32_t* dst = hll_acc + ((size_t)t.hll_slot * kHllCopies + (blockIdx.x % kHllCopies)) * 512;
    for (int i = threadIdx.x; i < 512; i += kBlock) {
      const uint32_t v = (uint32_t)(regs[i] + 1);
      if (v > __builtin_nontemporal_load(dst + i)) atomicMax(dst + i, v);
    }
  }
}

// ------------------------------------------------------------------------------------------
// Correlation co-moment state (Corr update/merge algebra, Correlation.scala:37-52).
// ------------------------------------------------------------------------------------------
struct CorrStats { double n, xa, ya, ck, xm, ym; };

__device__ __forceinline__ void corr_merge(CorrStats& a, const CorrStats& b) {
  double n = a.n + b.n;
  if (b.n != 0.0) {
    if (a.n == 0.0) { a.xa = b.xa; a.ya = b.ya; a.ck = b.ck; a.xm = b.xm; a.ym = b.ym; }
    else {
      double dx = b.xa - a.xa, dy = b.ya - a.ya;
      double r = b.n / n;
      double dxr = dx * r, dyr = dy * r;
      a.ck = a.ck + b.ck + dx * dyr * a.n;
      a.xm = a.xm + b.xm + dx * dxr * a.n;
      a.ym = a.ym + b.ym + dy * dyr * a.n;
      a.xa = a.xa + dxr;
      a.ya = a.ya + dyr;
    }
  }
  a.n = n;
}

// ------------------------------------------------------------------------------------------
// Kernel 1: predicate program (three-valued logic) -- Compliance / conditional counts and `where`
// bitmaps (Compliance.scala:37-53, Analyzer.scala:404-408).  A wave takes 512-row blocks (lane l:
// rows base + 64 j + l, j < 8).  Each atom of the postfix program is evaluated for the whole block:
// its 8 (or 16) value loads are in flight together, the comparison is ballot-ed into TRUE / NULL
// row masks (validity and COALESCE fallbacks applied on the scalar masks).  The logic then runs on
// 32-row mask words: lanes 0..15 each own one word of the block, with the operand stack, the stored
// roots and per-lane counter partials in the wave's LDS scratch.  Counters reach the accumulator by
// 64-bit integer atomics (order-free, so the result is deterministic).
// ------------------------------------------------------------------------------------------
// Spark comparison of doubles (nanSafeCompare / genEqual): NaN == NaN, NaN > everything.
__device__ __forceinline__ int cmp_dbl(double a, double b) {
  bool an = a != a, bn = b != b;
  if (an || bn) return (an && bn) ? 0 : (an ? 1 : -1);
  return (a > b) - (a < b);
}
__device__ __forceinline__ bool apply_cmp(int op, int c) {
  switch (op) {
    case C_LT: return c < 0;
    case C_LE: return c <= 0;
    case C_GT: return c > 0;
    case C_GE: return c >= 0;
    case C_EQ: return c == 0;
    case C_NE: return c != 0;
    case C_TRUE: return true;
    default: return false;
  }
}

// One wave's LDS scratch (dynamic, sized by the plan: pred_scratch_words per wave), 32-bit mask
// words of the current 512-row block, each array [entry][16 word lanes]: operand stack (TRUE,
// NULL), stored roots (TRUE, NULL), per-lane counter partials (TRUE, NOT NULL).
struct PredScratch {
  uint32_t *st, *sn, *rt, *rn, *ct, *cn;
  __device__ PredScratch(uint32_t* w, int depth, int roots, int counters) {
    st = w; sn = st + 16 * depth; rt = sn + 16 * depth; rn = rt + 16 * roots; ct = rn + 16 * roots; cn = ct + 16 * counters;
  }
};

// raw values of one column for the block (all 8 row-group loads issued before any is used) as 64-bit words:
// integers sign-extended (i32 / i16 / i8 / date32; a boolean 0 / 1), fp64 bits, f32 as the bits of the exactly
// widened double -- through a bounds-checked buffer descriptor over the workgroup's rows [row0, row1): rows past
// row1 read 0
__device__ __forceinline__ void pred_load(const void* p, int kind, int64_t row0, int64_t row1, int64_t base, int lane,
                                          uint64_t (&v)[8]) {
  if (kind == CK_BOOL) {  // value bits: row r is bit r & 31 of word r >> 5 (row0 is a multiple of 256)
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(reinterpret_cast<const char*>(p) + (row0 >> 3)), (short)0, (int)(((row1 - row0 + 31) >> 5) * 4),
        0x00020000);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t w = __builtin_amdgcn_raw_buffer_load_b32(r, (int)(((base - row0) >> 5) + 2 * j + (lane >> 5)) * 4, 0, 0);
      v[j] = (w >> (lane & 31)) & 1u;
    }
    return;
  }
  const int sz = ck_bytes(kind);
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<char*>(reinterpret_cast<const char*>(p) + row0 * sz), (short)0, (int)((row1 - row0) * sz), 0x00020000);
  if (kind == CK_I32) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      v[j] = (uint64_t)(int64_t)(int32_t)__builtin_amdgcn_raw_buffer_load_b32(r, lane * 4, (int)((base - row0 + 64 * j) * 4), 2);
  } else if (kind == CK_F32) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      v[j] = __builtin_bit_cast(uint64_t, (double)__builtin_bit_cast(
                                              float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)((base - row0 + 64 * j + lane) * 4), 0, 2)));
  } else if (kind == CK_I16) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      v[j] = (uint64_t)(int64_t)(int16_t)__builtin_amdgcn_raw_buffer_load_b16(r, (int)((base - row0 + 64 * j + lane) * 2), 0, 2);
  } else if (kind == CK_I8) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      v[j] = (uint64_t)(int64_t)(int8_t)__builtin_amdgcn_raw_buffer_load_b8(r, (int)(base - row0 + 64 * j + lane), 0, 2);
  } else if (kind >= CK_D128_LO) {
    // a decimal's 64-bit half (16-byte rows): the low word (CK_D128_LOU: sign bit flipped, so that a signed
    // compare orders it unsigned) or the high word
    const int off = kind == CK_D128_HI ? 8 : 0;
    const uint64_t flip = kind == CK_D128_LOU ? (1ull << 63) : 0ull;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const auto w2 = __builtin_amdgcn_raw_buffer_load_b64(r, lane * 16 + off, (int)((base - row0 + 64 * j) * 16), 2);
      v[j] = (((uint64_t)w2[1] << 32) | w2[0]) ^ flip;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const auto w2 = __builtin_amdgcn_raw_buffer_load_b64(r, lane * 8, (int)((base - row0 + 64 * j) * 8), 2);
      v[j] = ((uint64_t)w2[1] << 32) | w2[0];
    }
  }
}
__device__ __forceinline__ double pred_as_double(uint64_t v, int kind) {
  return ck_float(kind) ? __builtin_bit_cast(double, v) : (double)(int64_t)v;
}

// validity word of the lane's 32 rows (lanes 0..15: rows base + 32 L .. + 31) through a bounds-checked
// descriptor over the bitmap of [0, n_rows) (past it: 0); all ones without a bitmap
__device__ __forceinline__ uint32_t pred_valid_word(const uint32_t* v, int64_t base, int64_t n_rows, int lane) {
  if (!v) return ~0u;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(v), (short)0,
                                                                    (int)(((n_rows + 31) >> 5) * 4), 0x00020000);
  return __builtin_amdgcn_raw_buffer_load_b32(r, (lane & 15) * 4, (int)((base >> 5) * 4), 0);
}

// Loads of one atom for a block: raw values of column a / b (ATOM_CMP) and the lane's validity words.
struct AtomBuf {
  uint64_t a[8], b[8];
  uint32_t va, vb;
  // what the buffer holds (wave-uniform): block base, columns of a / b (-1: none), values loaded (CMP)
  int64_t t_base = -1;
  int32_t t_col_a = -1, t_col_b = -1;
  int32_t t_kind_a = 0, t_kind_b = 0;  // the loaded views (a decimal column is read as different halves)
  bool t_vals = false;
};

// One ATOM_CMP for a block from its operands' raw values (a, b: rows base + 64 j + lane) and validity words:
// the lane's 32-bit TRUE / NULL words (lanes 0..15).
__device__ __forceinline__ void pred_atom_cmp(const PredInstr& ins, const uint64_t (&La)[8], uint32_t Lva,
                                              const uint64_t (&Lb)[8], uint32_t Lvb, int lane, uint32_t& wt,
                                              uint32_t& wn) {
  // result = (lt & Klt) | (eq & Keq) | (gt & Kgt) | NaN terms (Spark: NaN = NaN, NaN > all)
  const int cmp = ins.cmp;
  const uint64_t Klt = (cmp == C_LT || cmp == C_LE || cmp == C_NE || cmp == C_TRUE) ? ~0ull : 0ull;
  const uint64_t Keq = (cmp == C_LE || cmp == C_GE || cmp == C_EQ || cmp == C_TRUE) ? ~0ull : 0ull;
  const uint64_t Kgt = (cmp == C_GT || cmp == C_GE || cmp == C_NE || cmp == C_TRUE) ? ~0ull : 0ull;
  const uint64_t Kbn = (cmp == C_LT || cmp == C_LE || cmp == C_NE || cmp == C_TRUE) ? ~0ull : 0ull;  // only b NaN
  const uint64_t Kan = (cmp == C_GT || cmp == C_GE || cmp == C_NE || cmp == C_TRUE) ? ~0ull : 0ull;  // only a NaN
  const uint64_t Kab = (cmp == C_LE || cmp == C_GE || cmp == C_EQ || cmp == C_TRUE) ? ~0ull : 0ull;  // both NaN
  const bool two = ins.col_b >= 0;
  const bool is_int = ins.ctype == CT_INT;
  uint32_t wc = 0;
  // row group j's 64-bit mask -> word lanes 2 j, 2 j + 1 (lanes 0..15 own the block's 16 words)
  // v_writelane: the scalar halves go straight into lanes 2 j, 2 j + 1.  The mask usually comes straight
  // from a v_cmp (VCC): a VALU-written SGPR read by v_writelane needs wait states the compiler cannot
  // insert for inline asm, hence the s_nop.
  auto put = [&](int j, uint64_t cm) {
    const uint32_t lo = (uint32_t)cm, hi = (uint32_t)(cm >> 32);
    asm volatile("s_nop 4\n\tv_writelane_b32 %0, %1, %2" : "+v"(wc) : "s"(lo), "i"(2 * j));
    asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(wc) : "s"(hi), "i"(2 * j + 1));
  };
  if (is_int) {
    // integers have no NaN: one compare per row group, the operator chosen once (uniform switch)
    auto run = [&](auto op) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t x = (int64_t)La[j], y = two ? (int64_t)Lb[j] : ins.lit_i;
        put(j, __builtin_amdgcn_ballot_w64(op(x, y)));
      }
    };
    switch (cmp) {
      case C_LT: run([](int64_t x, int64_t y) { return x < y; }); break;
      case C_LE: run([](int64_t x, int64_t y) { return x <= y; }); break;
      case C_GT: run([](int64_t x, int64_t y) { return x > y; }); break;
      case C_GE: run([](int64_t x, int64_t y) { return x >= y; }); break;
      case C_EQ: run([](int64_t x, int64_t y) { return x == y; }); break;
      case C_NE: run([](int64_t x, int64_t y) { return x != y; }); break;
      case C_TRUE: wc = ~0u; break;
      default: wc = 0u; break;
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (is_int) break;
    uint64_t lt, eq, gt, an = 0, bn = 0;
    {
      const double x = pred_as_double(La[j], ins.kind_a), y = two ? pred_as_double(Lb[j], ins.kind_b) : ins.lit_d;
      lt = __builtin_amdgcn_ballot_w64(x < y);
      eq = __builtin_amdgcn_ballot_w64(x == y);
      gt = __builtin_amdgcn_ballot_w64(x > y);
      an = __builtin_amdgcn_ballot_w64(x != x);
      bn = __builtin_amdgcn_ballot_w64(y != y);
    }
    const uint64_t cm = (lt & Klt) | (eq & Keq) | (gt & Kgt) | (~an & bn & Kbn) | (an & ~bn & Kan) | (an & bn & Kab);
    put(j, cm);  // row group j -> the word lanes (lanes 0..15: word L = rows 32 L .. + 31 of the block)
  }
  // NULL operand b -> NULL; NULL a -> the COALESCE fallback result (NULL without one)
  const uint32_t va = Lva, vb = two ? Lvb : ~0u;
  const uint32_t nr_true = ins.null_res == NR_TRUE ? ~0u : 0u, nr_null = ins.null_res == NR_NULL ? ~0u : 0u;
  wt = (va & vb & wc) | (~va & vb & nr_true);
  wn = ~vb | (~va & nr_null);
}

__device__ __forceinline__ void pred_atom_cmp(const PredInstr& ins, const AtomBuf& L, int lane, uint32_t& wt,
                                              uint32_t& wn) {
  pred_atom_cmp(ins, L.a, L.va, L.b, L.vb, lane, wt, wn);
}

// One ATOM_REGEX for a block (PatternMatch.scala:48-49 / RLIKE): lane l walks the search DFA (staged in
// LDS) over the UTF-8 bytes of rows base + 64 j + l, four bytes per aligned dword load; the walk stops
// in the dead (0) or sticky-accept (1) state.  Rows past row1 and NULL rows are masked by the caller's
// validity / in-range words.  The aligned dword holding a value byte never leaves the value's page.
__device__ __forceinline__ void pred_atom_regex(const PredInstr& ins, const uint16_t* __restrict__ dfa,
                                                const uint8_t* __restrict__ bytes, const void* __restrict__ offs,
                                                int64_t row1, int64_t base, int lane, uint32_t va, uint32_t& wt,
                                                uint32_t& wn) {
  const int ns = dfa[0], nc = dfa[1], start = dfa[2];
  const uint16_t* cls = dfa + 4;
  const uint16_t* acc = cls + 256;
  const uint16_t* tr = acc + ns;
  const bool large = ins.kind_a == CK_LUTF8;
  uint32_t wc = 0;
  for (int j = 0; j < 8; ++j) {
    const int64_t r = base + 64 * j + lane;
    bool m = false;
    if (r < row1) {
      int64_t o0, o1;
      if (large) {
        o0 = reinterpret_cast<const int64_t*>(offs)[r];
        o1 = reinterpret_cast<const int64_t*>(offs)[r + 1];
      } else {
        o0 = reinterpret_cast<const int32_t*>(offs)[r];
        o1 = reinterpret_cast<const int32_t*>(offs)[r + 1];
      }
      int st = start;
      int64_t i = o0;
      while (i < o1 && st >= 2) {
        const uint32_t w = *reinterpret_cast<const uint32_t*>(bytes + (i & ~(int64_t)3));
        const int64_t end = (i | 3) + 1 < o1 ? (i | 3) + 1 : o1;
        do {
          st = tr[st * nc + cls[(w >> (8 * (i & 3))) & 0xFFu]];
          ++i;
        } while (i < end && st >= 2);
      }
      m = acc[st] != 0;
    }
    const uint64_t cm = __builtin_amdgcn_ballot_w64(m);
    if ((lane >> 1) == j) wc = (lane & 1) ? (uint32_t)(cm >> 32) : (uint32_t)cm;
  }
  wt = va & wc;
  wn = ins.null_res == NR_NULL ? ~va : 0u;
}

// ATOM_REGEX over int32 offsets: the lane's 8 row offsets are loaded together, and each row's first
// 32 bytes come in as two 16-byte buffer loads (bounds-checked over the chunk's bytes) issued while the
// previous row is walked; the first 28 bytes are realigned in registers and walked branch-free
// (select on `p < len && live`), in 4-byte groups skipped as soon as no lane of the wave needs them.
// The rare value longer than 28 bytes continues with dword loads, as does a value whose 32-byte window
// would reach past the last whole dword of the chunk's bytes (a buffer load zeroes such dwords).
__device__ __forceinline__ void pred_atom_regex_utf8(const PredInstr& ins, const uint16_t* __restrict__ dfa,
                                                     const uint8_t* __restrict__ bytes,
                                                     const int32_t* __restrict__ offs, int64_t n_rows, int64_t row1,
                                                     int64_t base, int lane, uint32_t va, uint32_t& wt, uint32_t& wn) {
  const int ns = dfa[0], nc = dfa[1];
  const uint32_t start = dfa[2];
  const uint16_t* cls = dfa + 4;
  const uint16_t* acc = cls + 256;
  const uint16_t* tr = acc + ns;
  const int32_t total = offs[n_rows];
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(bytes), (short)0, total, 0x00020000);
  const int32_t win = (total & ~3) - 32;  // window of a value at o0 is whole iff (o0 & ~3) <= win
  int32_t o0[8], ln[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int64_t r = base + 64 * j + lane;
    o0[j] = r < row1 ? offs[r] : 0;
    ln[j] = r < row1 ? offs[r + 1] - o0[j] : 0;
  }
  u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rsrc, o0[0] & ~3, 0, 0);
  u32x4 c = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (o0[0] & ~3) + 16, 0, 0);
  uint32_t wc = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    u32x4 an = a, cn = c;
    if (j < 7) {
      an = __builtin_amdgcn_raw_buffer_load_b128(rsrc, o0[j + 1] & ~3, 0, 0);
      cn = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (o0[j + 1] & ~3) + 16, 0, 0);
    }
    const uint32_t d[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
    const uint32_t sh = (uint32_t)o0[j] << 3;
    uint32_t wv[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) wv[k] = alignbit32(d[k + 1], d[k], sh);
    const int32_t L = ln[j];
    const int32_t Lw = (o0[j] & ~3) <= win ? L : 0;  // bytes walked from the window
    uint32_t st = start;
#pragma unroll
    for (int g = 0; g < 7; ++g) {
      if (!__builtin_amdgcn_ballot_w64(Lw > 4 * g && st >= 2u)) break;  // wave-uniform
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint32_t nx = tr[st * nc + cls[(wv[g] >> (8 * b)) & 0xFFu]];
        st = (4 * g + b < Lw && st >= 2u) ? nx : st;
      }
    }
    const int32_t done = Lw < 28 ? Lw : 28;
    if (L > done && st >= 2u) {  // long value / window past the end: the rest with dword loads
      int64_t i = (int64_t)o0[j] + done;
      const int64_t e = (int64_t)o0[j] + L;
      while (i < e && st >= 2u) {
        const uint32_t w = *reinterpret_cast<const uint32_t*>(bytes + (i & ~(int64_t)3));
        const int64_t end = (i | 3) + 1 < e ? (i | 3) + 1 : e;
        do {
          st = tr[st * nc + cls[(w >> (8 * (i & 3))) & 0xFFu]];
          ++i;
        } while (i < end && st >= 2u);
      }
    }
    const uint64_t cm = __builtin_amdgcn_ballot_w64(acc[st] != 0);
    if ((lane >> 1) == j) wc = (lane & 1) ? (uint32_t)(cm >> 32) : (uint32_t)cm;
    a = an;
    c = cn;
  }
  wt = va & wc;
  wn = ins.null_res == NR_NULL ? ~va : 0u;
}

// One instruction of the program, read from the workgroup's LDS copy and made wave-uniform (SGPRs).  The
// interpreter used to read each field with scalar loads from global memory inside the block loop: every
// LDS stack access then also waited for those out-of-order SMEM returns (lgkmcnt(0)), serialising the
// block on scalar-load latency (rocprof: ~126 SMEM and ~30k wave cycles per 512-row block).
__device__ __forceinline__ PredInstr uniform_instr(const PredInstr* p) {
  static_assert(sizeof(PredInstr) % 4 == 0, "PredInstr words");
  PredInstr r;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(p);
  uint32_t* o = reinterpret_cast<uint32_t*>(&r);
#pragma unroll
  for (int k = 0; k < (int)(sizeof(PredInstr) / 4); ++k) o[k] = __builtin_amdgcn_readfirstlane(w[k]);
  return r;
}

// The fields an ATOM_CMP evaluation reads (cmp, ctype, null_res, col_b, kinds, literals), wave-uniform: 10
// readfirstlanes instead of the whole instruction's 14 (the block loop decodes every instruction per block).
__device__ __forceinline__ PredInstr uniform_cmp_fields(const PredInstr* p) {
  PredInstr r{};
  const uint32_t* w = reinterpret_cast<const uint32_t*>(p);
  uint32_t* o = reinterpret_cast<uint32_t*>(&r);
  constexpr int kF[10] = {1, 2, 3, 5, 6, 7, 8, 9, 10, 11};
  static_assert(offsetof(PredInstr, lit_d) == 40 && offsetof(PredInstr, col_b) == 20, "PredInstr layout");
#pragma unroll
  for (int k = 0; k < 10; ++k) o[kF[k]] = __builtin_amdgcn_readfirstlane(w[kF[k]]);
  return r;
}

// Compact per-instruction words staged in LDS by the interpreter, one readfirstlane each:
//   op word:   op | null_res << 8 | slot << 16            (every instruction; logic ops need nothing else)
//   load word: op | (col_a + 1) << 4 | (col_b + 1) << 12 | kind_a << 20 | kind_b << 24   (atoms)
__device__ __forceinline__ uint32_t pred_op_word(const PredInstr& ins) {
  return (uint32_t)ins.op | (uint32_t)ins.null_res << 8 | (uint32_t)ins.slot << 16;
}
__device__ __forceinline__ uint32_t pred_load_word(const PredInstr& ins) {
  return (uint32_t)ins.op | (uint32_t)(ins.col_a + 1) << 4 | (uint32_t)(ins.col_b + 1) << 12 | (uint32_t)ins.kind_a << 20 |
         (uint32_t)ins.kind_b << 24;
}

// Three-valued logic ops of the program on the wave's 16 word lanes (operand stack in LDS):
// CONST / AND / OR / NOT / STORE (w: the op word); atoms push their own results.
__device__ __forceinline__ void pred_logic_op(uint32_t w, const PredScratch& S, int& sp, int lane) {
  const int op = (int)(w & 0xFFu), null_res = (int)((w >> 8) & 0xFFu), slot = (int)(w >> 16);
  const bool wl = lane < 16;
  if (op == PO_CONST) {
    if (wl) { S.st[(sp) * 16 + lane] = null_res == NR_TRUE ? ~0u : 0u; S.sn[(sp) * 16 + lane] = null_res == NR_NULL ? ~0u : 0u; }
    ++sp;
  } else if (op == PO_AND || op == PO_OR) {
    if (wl) {
      const uint32_t at = S.st[(sp - 2) * 16 + lane], an = S.sn[(sp - 2) * 16 + lane];
      const uint32_t bt = S.st[(sp - 1) * 16 + lane], bn = S.sn[(sp - 1) * 16 + lane];
      const uint32_t af = ~at & ~an, bf = ~bt & ~bn;
      const uint32_t rt = op == PO_AND ? (at & bt) : (at | bt);
      const uint32_t rf = op == PO_AND ? (af | bf) : (af & bf);
      S.st[(sp - 2) * 16 + lane] = rt;
      S.sn[(sp - 2) * 16 + lane] = ~rt & ~rf;
    }
    --sp;
  } else if (op == PO_NOT) {
    if (wl) {
      const uint32_t at = S.st[(sp - 1) * 16 + lane], an = S.sn[(sp - 1) * 16 + lane];
      S.st[(sp - 1) * 16 + lane] = ~at & ~an;
    }
  } else if (op == PO_STORE) {
    if (wl) { S.rt[(slot) * 16 + lane] = S.st[(sp - 1) * 16 + lane]; S.rn[(slot) * 16 + lane] = S.sn[(sp - 1) * 16 + lane]; }
    --sp;
  }
}

// End of a block: counters (TRUE / NOT NULL of each (predicate, where) pair over the in-range rows) and
// the `where` bitmaps, on the word lanes (wr = first row of the lane's word).
__device__ __forceinline__ void pred_block_out(const PredScratch& S, const PredCounter* s_ctr, int n_counters,
                                               const int32_t* s_bmroot, int n_bitmaps, const ScanBitmaps& bm,
                                               int64_t wr, uint32_t inr, int64_t n_rows, int lane) {
  if (lane >= 16) return;
  for (int c = 0; c < n_counters; ++c) {
    const PredCounter pc = s_ctr[c];
    const uint32_t tw = (pc.where < 0 ? ~0u : S.rt[(pc.where) * 16 + lane]) & inr;
    S.ct[(c) * 16 + lane] += __popc(S.rt[(pc.pred) * 16 + lane] & tw);
    S.cn[(c) * 16 + lane] += __popc(~S.rn[(pc.pred) * 16 + lane] & tw);
  }
  if (wr < n_rows) {
    for (int b = 0; b < n_bitmaps; ++b)
      reinterpret_cast<uint32_t*>(bm.where_bits[b])[wr >> 5] = S.rt[s_bmroot[b] * 16 + lane] & inr;
  }
}

// Workgroup partials -> accumulator copy (integer atomics: order-free); waits for every wave's counters.
__device__ __forceinline__ void pred_counters_out(const uint32_t* pred_lds, int wave_words, const PredProgram& prog,
                                                  PredPartial* acc) {
  __syncthreads();
  if (threadIdx.x < prog.n_counters) {
    const int c = threadIdx.x;
    int64_t t = 0, nn = 0;
    for (int w = 0; w < kWaves; ++w)
      for (int l = 0; l < 16; ++l) {
        const PredScratch W(const_cast<uint32_t*>(pred_lds) + w * wave_words, prog.stack_depth, prog.n_roots,
                            prog.n_counters);
        t += W.ct[c * 16 + l];
        nn += W.cn[c * 16 + l];
      }
    // one of kPredAccCopies accumulator copies per workgroup (the host adds them): every workgroup's atomics
    // on the same addresses serialize at the end of the launch
    PredPartial* a = acc + (blockIdx.x % kPredAccCopies);
    atomicAdd(reinterpret_cast<unsigned long long*>(&a->t[c]), (unsigned long long)t);
    atomicAdd(reinterpret_cast<unsigned long long*>(&a->nn[c]), (unsigned long long)nn);
  }
}

// RX: the program holds regex atoms.  Instantiated separately so that the DFA walk's registers (142
// VGPRs with it, 119 without: 3 vs 4 waves per SIMD) do not cost the plain numeric programs occupancy.
template <bool RX>
__global__ __launch_bounds__(kBlock) void dq_pred_scan(const PredProgram* __restrict__ prog_g, ScanCols cols,
                                                       ScanBitmaps bm, int64_t n_rows, int64_t rows_per_range,
                                                       PredPartial* __restrict__ acc) {
  extern __shared__ uint32_t pred_lds[];
  __shared__ PredInstr s_instr[kMaxInstr];
  __shared__ uint32_t s_op[kMaxInstr];    // op words (pred_op_word)
  __shared__ uint32_t s_ldw[kMaxInstr];   // atom k's load word (pred_load_word)
  __shared__ PredCounter s_ctr[kMaxCounters];
  __shared__ int32_t s_bmroot[kMaxWhere];
  const PredProgram& prog = *prog_g;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wave_words = 32 * (prog.stack_depth + prog.n_roots + prog.n_counters);
  PredScratch S(pred_lds + wave * wave_words, prog.stack_depth, prog.n_roots, prog.n_counters);
  const bool wl = lane < 16;  // word lanes
  const int n_instr = prog.n_instr, n_counters = prog.n_counters, n_bitmaps = prog.n_bitmaps, n_loads = prog.n_loads;
  // the program -> LDS once per workgroup
  for (int k = threadIdx.x; k < n_instr * (int)(sizeof(PredInstr) / 4); k += kBlock)
    reinterpret_cast<uint32_t*>(s_instr)[k] = reinterpret_cast<const uint32_t*>(prog.instr)[k];
  for (int k = threadIdx.x; k < n_instr; k += kBlock) s_op[k] = pred_op_word(prog.instr[k]);
  for (int k = threadIdx.x; k < n_loads; k += kBlock) s_ldw[k] = pred_load_word(prog.instr[prog.load_instr[k]]);
  for (int k = threadIdx.x; k < n_counters; k += kBlock) s_ctr[k] = prog.counters[k];
  for (int k = threadIdx.x; k < n_bitmaps; k += kBlock) s_bmroot[k] = prog.bitmap_root[k];
  __syncthreads();
  if (wl) {
    for (int c = 0; c < n_counters; ++c) { S.ct[(c) * 16 + lane] = 0; S.cn[(c) * 16 + lane] = 0; }
  }
  // compiled regex DFAs -> LDS after the waves' scratch
  uint16_t* dfa_lds = reinterpret_cast<uint16_t*>(pred_lds + kWaves * wave_words);
  if (RX && prog.regex_words > 0) {
    for (int k = threadIdx.x; k < prog.regex_words; k += kBlock) dfa_lds[k] = prog.regex[k];
    __syncthreads();
  }
  const int64_t row0 = (int64_t)blockIdx.x * rows_per_range;
  int64_t row1 = row0 + rows_per_range;
  if (row1 > n_rows) row1 = n_rows;
  // Two-deep pipeline over the atoms, across blocks: atom g (a wave-uniform running count) uses
  // buffer g & 1, and the loads of atom g + 1 go into the other buffer before atom g is evaluated.
  AtomBuf B0, B1;
  // Loads of atom k of the block at `base` into L; C is the buffer of the atom evaluated meanwhile (the
  // previous atom): a column it already holds for the same block is copied, not re-read -- C3 reads i1 in
  // three consecutive atoms and i3 in two, and those re-reads missed L2 (FETCH_SIZE 1.41x algorithmic).
  auto issue = [&](int k, int64_t base, AtomBuf& L, const AtomBuf& C) {
    const uint32_t lw = __builtin_amdgcn_readfirstlane(s_ldw[k]);
    const int op = (int)(lw & 15u), col_a = (int)((lw >> 4) & 0xFFu) - 1, col_b = (int)((lw >> 12) & 0xFFu) - 1;
    const int kind_a = (int)((lw >> 20) & 15u), kind_b = (int)((lw >> 24) & 15u);
    const bool same_blk = C.t_base == base;
    auto fetch = [&](int col, int kind, bool vals, uint64_t (&dst)[8], uint32_t& vdst) __attribute__((always_inline)) {
      if (same_blk && col == C.t_col_a && (!vals || (C.t_vals && kind == C.t_kind_a))) {
        if (vals) {
#pragma unroll
          for (int j = 0; j < 8; ++j) dst[j] = C.a[j];
        }
        vdst = C.va;
      } else if (same_blk && col == C.t_col_b && C.t_vals && (!vals || kind == C.t_kind_b)) {
        if (vals) {
#pragma unroll
          for (int j = 0; j < 8; ++j) dst[j] = C.b[j];
        }
        vdst = C.vb;
      } else {
        if (vals) pred_load(cols.values[col], kind, row0, row1, base, lane, dst);
        vdst = pred_valid_word(cols.validity[col], base, n_rows, lane);
      }
    };
    const bool cmp = op == PO_ATOM_CMP;
    if (cmp && col_b >= 0) fetch(col_b, kind_b, true, L.b, L.vb);
    fetch(col_a, kind_a, cmp, L.a, L.va);
    L.t_base = base;
    L.t_col_a = col_a;
    L.t_col_b = cmp ? col_b : -1;
    L.t_kind_a = kind_a;
    L.t_kind_b = kind_b;
    L.t_vals = cmp;
  };
  if (n_loads > 0) issue(0, row0 + (int64_t)wave * 512, B0, B1);
  uint32_t g = 0;

  for (int64_t blk = row0; blk < row1; blk += kRowsPerIter) {
    const int64_t base = blk + (int64_t)wave * 512;
    if (base >= row1) break;  // wave-uniform
    // in-range rows of this lane's word
    const int64_t wr = base + 32 * (lane & 15);
    const uint32_t inr = wr >= row1 ? 0u : (wr + 32 <= row1 ? ~0u : ((1u << (row1 - wr)) - 1u));
    int sp = 0, k = 0;
    for (int i = 0; i < n_instr; ++i) {
      const uint32_t ow = __builtin_amdgcn_readfirstlane(s_op[i]);
      const int op = (int)(ow & 0xFFu);
      if (op == PO_ATOM_CMP || op == PO_ATOM_ISNULL || op == PO_ATOM_NOTNULL || op == PO_ATOM_REGEX) {
        // next atom: the following one of this block, else the first of the next block
        const int kn = k + 1 < n_loads ? k + 1 : 0;
        const int64_t bn = k + 1 < n_loads ? base : base + kRowsPerIter;
        uint32_t wt, wn;
        const AtomBuf& cur = (g & 1u) ? B1 : B0;
        if ((g & 1u) == 0) issue(kn, bn, B1, B0);
        else issue(kn, bn, B0, B1);
        if (op == PO_ATOM_CMP) {
          const PredInstr ins = uniform_cmp_fields(&s_instr[i]);
          if ((g & 1u) == 0) pred_atom_cmp(ins, B0, lane, wt, wn);
          else pred_atom_cmp(ins, B1, lane, wt, wn);
        } else if (RX && op == PO_ATOM_REGEX) {
          const PredInstr ins = uniform_instr(&s_instr[i]);
          const uint32_t va = (g & 1u) ? B1.va : B0.va;
          if (ins.kind_a == CK_UTF8)
            pred_atom_regex_utf8(ins, dfa_lds + ins.lit_i, reinterpret_cast<const uint8_t*>(cols.values[ins.col_a]),
                                 reinterpret_cast<const int32_t*>(cols.offsets[ins.col_a]), n_rows, row1, base, lane,
                                 va, wt, wn);
          else
            pred_atom_regex(ins, dfa_lds + ins.lit_i, reinterpret_cast<const uint8_t*>(cols.values[ins.col_a]),
                            cols.offsets[ins.col_a], row1, base, lane, va, wt, wn);
        } else {
          const uint32_t va = (g & 1u) ? B1.va : B0.va;
          wt = op == PO_ATOM_ISNULL ? ~va : va;
          wn = 0u;
        }
        (void)cur;
        ++g;
        ++k;
        if (wl) { S.st[(sp) * 16 + lane] = wt; S.sn[(sp) * 16 + lane] = wn; }
        ++sp;
      } else {
        pred_logic_op(ow, S, sp, lane);
      }
    }
    pred_block_out(S, s_ctr, n_counters, s_bmroot, n_bitmaps, bm, wr, inr, n_rows, lane);
  }
  pred_counters_out(pred_lds, wave_words, prog, acc);
}

// ------------------------------------------------------------------------------------------
// Kernel 4: fixed-order merge of per-workgroup partials into the plan accumulators.
// blockIdx.x: [0, ncol) column tasks, [ncol, ncol + npair) pairs, then one block for counters.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void dq_finalize(int32_t ncol, int32_t nranges_col,
                                                      const ColPartial* __restrict__ col_part,
                                                      ColPartial* __restrict__ col_acc, int32_t npair, int32_t nranges_pair,
                                                      const CorrPartial* __restrict__ pair_part,
                                                      CorrPartial* __restrict__ pair_acc, int32_t has_pred,
                                                      int32_t nranges_pred, const PredPartial* __restrict__ pred_part,
                                                      PredPartial* __restrict__ pred_acc, FinRanges fr,
                                                      int64_t* __restrict__ rare_dev, int64_t* rare_host) {
  __shared__ ColStats cs[kBlock];
  __shared__ CorrStats ps[kBlock];
  const int b = blockIdx.x, tid = threadIdx.x;
  if (b < ncol) {
    int32_t nr = nranges_col;  // the variant launch's own range count, if it had one
    for (int i = 0; i < fr.n; ++i)
      if (b >= fr.first[i] && b < fr.end[i]) nr = fr.nr[i];
    ColStats s;
    stats_init(s);
    for (int r = tid; r < nr; r += kBlock) stats_merge(s, stats_load(col_part + (size_t)b * kMaxWG + r));
    cs[tid] = s;
    __syncthreads();
    for (int stride = kBlock / 2; stride >= 1; stride >>= 1) {
      if (tid < stride) { ColStats a = cs[tid]; stats_merge(a, cs[tid + stride]); cs[tid] = a; }
      __syncthreads();
    }
    if (tid == 0) {
      ColStats acc = stats_load(col_acc + b);
      stats_merge(acc, cs[0]);
      stats_store(col_acc + b, acc);
      // the task's rare-path rows since the reset, to the host (mapped pinned memory; dq_scan reads it
      // without waiting, to choose the string pass's variant for the next chunks)
      // (only a changed count crosses PCIe: rare_dev[ncol + b] is the value last published)
      if (rare_host && rare_dev[b] != rare_dev[ncol + b]) {
        rare_dev[ncol + b] = rare_dev[b];
        __hip_atomic_store(rare_host + b, rare_dev[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  } else if (b < ncol + npair) {
    const int p = b - ncol;
    CorrStats s = {0, 0, 0, 0, 0, 0};
    for (int r = tid; r < nranges_pair; r += kBlock) {
      const CorrPartial& q = pair_part[(size_t)p * kMaxWG + r];
      CorrStats o = {q.n, q.xa, q.ya, q.ck, q.xm, q.ym};
      corr_merge(s, o);
    }
    ps[tid] = s;
    __syncthreads();
    for (int stride = kBlock / 2; stride >= 1; stride >>= 1) {
      if (tid < stride) { CorrStats a = ps[tid]; corr_merge(a, ps[tid + stride]); ps[tid] = a; }
      __syncthreads();
    }
    if (tid == 0) {
      CorrPartial& q = pair_acc[p];
      CorrStats acc = {q.n, q.xa, q.ya, q.ck, q.xm, q.ym};
      corr_merge(acc, ps[0]);
      q.n = acc.n; q.xa = acc.xa; q.ya = acc.ya; q.ck = acc.ck; q.xm = acc.xm; q.ym = acc.ym;
    }
  } else if (has_pred) {
    // 256 threads = kMaxCounters counters x 8 range groups; integer sums are order-free
    static_assert(kBlock % kMaxCounters == 0, "counter layout");
    constexpr int G = kBlock / kMaxCounters;
    __shared__ int64_t st[G][kMaxCounters], sn[G][kMaxCounters];
    const int c = tid % kMaxCounters, g = tid / kMaxCounters;
    int64_t t = 0, nn = 0;
    for (int r = g; r < nranges_pred; r += G) { t += pred_part[r].t[c]; nn += pred_part[r].nn[c]; }
    st[g][c] = t;
    sn[g][c] = nn;
    __syncthreads();
    if (tid < kMaxCounters) {
      int64_t a = pred_acc->t[tid], b = pred_acc->nn[tid];
      for (int k = 0; k < G; ++k) { a += st[k][tid]; b += sn[k][tid]; }
      pred_acc->t[tid] = a;
      pred_acc->nn[tid] = b;
    }
  }
}

__global__ void dq_init_acc(ColPartial* col_acc, int32_t ncol, CorrPartial* pair_acc, int32_t npair, int64_t* rare_dev) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < ncol) {
    ColStats s;
    stats_init(s);
    stats_store(col_acc + i, s);
    if (rare_dev) rare_dev[i] = 0;
  }
  if (i < npair) {
    CorrPartial& q = pair_acc[i];
    q.n = q.xa = q.ya = q.ck = q.xm = q.ym = q.pad0 = q.pad1 = 0.0;
  }
}

// ------------------------------------------------------------------------------------------
// host-side launchers (called from dq_plan.cpp)
// ------------------------------------------------------------------------------------------
hipError_t launch_pred_scan(const PredProgram* prog, const ScanCols& cols, const ScanBitmaps& bm, int64_t n_rows,
                            int64_t rows_per_range, int32_t nranges, PredPartial* acc, int32_t lds_bytes, hipStream_t st,
                            bool has_regex) {
  if (has_regex)
    hipLaunchKernelGGL(dq_pred_scan<true>, dim3(nranges), dim3(kBlock), (size_t)lds_bytes, st, prog, cols, bm, n_rows,
                       rows_per_range, acc);
  else
    hipLaunchKernelGGL(dq_pred_scan<false>, dim3(nranges), dim3(kBlock), (size_t)lds_bytes, st, prog, cols, bm, n_rows,
                       rows_per_range, acc);
  return hipGetLastError();
}

template <int V>
static void launch_v(const ColTask* tasks, int32_t ntasks, int32_t part_base, const ScanCols& cols,
                     const ScanBitmaps& bm, int64_t n_rows, int64_t rows_per_range, int32_t nranges,
                     ColPartial* partials, uint32_t* hll_acc, bool long_str, hipStream_t st) {
  constexpr bool kStrHll = V == CV_UTF8_H || V == CV_LUTF8_H || V == CV_UTF8_HD || V == CV_LUTF8_HD;
  if constexpr (kStrHll) {
    if (long_str) {
      hipLaunchKernelGGL((dq_column_scan<V, true>), dim3((uint32_t)ntasks * (uint32_t)nranges), dim3(kBlock), 0, st,
                         tasks, ntasks, part_base, cols, bm, n_rows, rows_per_range, partials, hll_acc);
      return;
    }
  }
  hipLaunchKernelGGL(dq_column_scan<V>, dim3((uint32_t)ntasks * (uint32_t)nranges), dim3(kBlock), 0, st, tasks, ntasks,
                     part_base, cols, bm, n_rows, rows_per_range, partials, hll_acc);
}

// tasks [first, first + ntasks) of the plan's task table all have variant `variant`
hipError_t launch_column_scan(int32_t variant, const ColTask* tasks, int32_t ntasks, int32_t part_base,
                              const ScanCols& cols, const ScanBitmaps& bm, int64_t n_rows, int64_t rows_per_range,
                              int32_t nranges, ColPartial* partials, uint32_t* hll_acc, bool long_str, hipStream_t st) {
#define DQ_V(V)                                                                                            \
  case V:                                                                                                  \
    launch_v<V>(tasks, ntasks, part_base, cols, bm, n_rows, rows_per_range, nranges, partials, hll_acc, long_str, \
                st);                                                                                       \
    break;
  switch (variant) {
    DQ_V(CV_VALIDITY) DQ_V(CV_F64_S) DQ_V(CV_F64_SH) DQ_V(CV_F64_H) DQ_V(CV_I64_S) DQ_V(CV_I64_SH) DQ_V(CV_I64_H)
    DQ_V(CV_I32_S) DQ_V(CV_I32_SH) DQ_V(CV_I32_H) DQ_V(CV_UTF8_H) DQ_V(CV_LUTF8_H)
    DQ_V(CV_UTF8_D) DQ_V(CV_UTF8_HD) DQ_V(CV_LUTF8_D) DQ_V(CV_LUTF8_HD) DQ_V(CV_F64_D)
    DQ_V(CV_F32_S) DQ_V(CV_F32_SH) DQ_V(CV_F32_H) DQ_V(CV_I16_S) DQ_V(CV_I16_SH) DQ_V(CV_I16_H)
    DQ_V(CV_I8_S) DQ_V(CV_I8_SH) DQ_V(CV_I8_H) DQ_V(CV_F32_D) DQ_V(CV_BOOL)
    DQ_V(CV_D128_S) DQ_V(CV_D128_SH) DQ_V(CV_D128_H) DQ_V(CV_D128_D)
    default: return hipErrorInvalidValue;
  }
#undef DQ_V
  return hipGetLastError();
}


hipError_t launch_finalize(int32_t ncol, int32_t nranges_col, const ColPartial* col_part, ColPartial* col_acc,
                           int32_t npair, int32_t nranges_pair, const CorrPartial* pair_part, CorrPartial* pair_acc,
                           int32_t has_pred, int32_t nranges_pred, const PredPartial* pred_part, PredPartial* pred_acc,
                           const FinRanges& fr, int64_t* rare_dev, int64_t* rare_host, hipStream_t st) {
  const uint32_t nb = (uint32_t)(ncol + npair + (has_pred ? 1 : 0));
  if (nb == 0) return hipSuccess;
  hipLaunchKernelGGL(dq_finalize, dim3(nb), dim3(kBlock), 0, st, ncol, nranges_col, col_part, col_acc, npair,
                     nranges_pair, pair_part, pair_acc, has_pred, nranges_pred, pred_part, pred_acc, fr, rare_dev,
                     rare_host);
  return hipGetLastError();
}

hipError_t launch_init_acc(ColPartial* col_acc, int32_t ncol, CorrPartial* pair_acc, int32_t npair, int64_t* rare_dev,
                           hipStream_t st) {
  const int n = ncol > npair ? ncol : npair;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(dq_init_acc, dim3((n + 255) / 256), dim3(256), 0, st, col_acc, ncol, pair_acc, npair, rare_dev);
  return hipGetLastError();
}

}  // namespace dq
