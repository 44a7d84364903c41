// dq_pair.hip -- gfx950 kernels of the Correlation pass fused with the column moments of the same columns.
//
// Reference: Correlation (analyzers/Correlation.scala:26-105, catalyst/StatefulCorrelation.scala:24-49:
// Spark's Corr co-moments, merged with Chan's formula Correlation.scala:37-52) and the moments of Mean /
// StandardDeviation / Sum / Minimum / Maximum (StandardDeviation.scala:37-44 merge) -- all aggregates of
// the one data.agg(...) pass (AnalysisRunner.scala:303).  Config C4 asks for 28 correlations over 8 fp64
// columns fused with their Mean and StdDev: every column is read from HBM once for all of that.
//
// Layout.  A workgroup task (PairWG, planned on the host) is one pair group (<= 8 columns, one `where`)
// and two wave tasks; a workgroup is two waves and one row range.  Wave w's position p holds the group's
// local column (p + w) % 8 and runs the fixed 14-slot pattern kPairSlotA / kPairSlotB over its positions --
// the two rotations of the pattern are the 28 pairs of 8 columns, each once -- plus the moments of its even
// positions.  Lane l takes row l of each 64-row group.  All-fp64, 16-byte aligned groups (RING) are staged
// HBM -> LDS by global_load_lds DMA into a ring of kRing slots of two 64-row groups: each wave brings four
// columns (one 1 KB instruction per column, all 64 lanes, nt policy) and its selection words, 3 slots ahead,
// one s_barrier per slot; the selection masks come out of LDS by v_readlane.  Other groups load the values
// into VGPRs two groups ahead and the masks by scalar loads.  Per pair and 64 rows the fold is five fp64
// VALU under exec = sel(a) & sel(b) (the rows selected in both columns, nothing zeroed):
//   Sa += za   Sb += zb   Sab += za zb   Saa += za^2   Sbb += zb^2        (z = x - shift)
// and nothing for the counts: a pair's count (rows selected in both columns) and a column's count are
// popcounts of bitmap words, taken at the end of the range by a lane-per-word pass over the bitmaps (1/64 of
// the value bytes).
//
// Non-finite values.  The fold above assumes every selected value is finite.  A selected NaN / +-inf (or
// a finite value whose square overflows) turns some active sum non-finite; the wave then flags its range
// (redo[]) instead of writing partials, and dq_pair_redo re-runs exactly those (wave, range) units with
// the checked fold: selections cut to finite rows, Spark's poisoning of the pairs holding a NaN / inf in
// a row selected in both columns, NaN / +-inf counts and min / max over the inf rows for the moments.
//
// Shifts.  Per (range, position): the mean of the column's first 64-row group holding finite selected
// values.  That makes the closing formulas m2 = Saa - Sa^2 / n and ck = Sab - Sa Sb / n safe:
// |shift - mean|^2 <= (rows / 64) var for any data, so the cancellation costs at most ~1e-13 relative at
// 2^16-row ranges (tests/test_pair_lane.py::test_pair_pass_drift_and_offset_columns against a
// double-double reference; the full-scale C4 check in tests/fullscale_parity.py).  Each pair and each
// moments column belongs to exactly one wave: at the end of the range the wave reduces its lanes (fixed
// butterfly order) and writes its CorrPartial / ColPartial records; dq_finalize merges the ranges in order.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "dq_decimal.h"
#include "dq_device.h"
#include "dq_lane.h"

namespace dq {

namespace {

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}
__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = (int64_t)((uint64_t)v + (uint64_t)__shfl_xor(v, m));
  return v;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += (uint32_t)__shfl_xor((int)v, m);
  return v;
}
__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = hw_min(v, __shfl_xor(v, m));
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = hw_max(v, __shfl_xor(v, m));
  return v;
}
__device__ __forceinline__ double uniform(double v) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b), hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// the 64-bit bitmap word at byte offset `off` (uniform: one scalar load; the bitmap holds it whole)
__device__ __forceinline__ uint64_t sword_at(const uint32_t* bm, uint32_t off) {
  const const_u32s w = (const_u32s)((const __attribute__((address_space(4))) char*)bm + off);
  return ((uint64_t)w[1] << 32) | w[0];
}
// bits of rows [base, base + 64) of a bitmap, clipped to rows below row1 (base < row1, base % 64 == 0; a
// dword holding no row below row1 is not read).  Uniform base: scalar loads; per-lane base: vector loads.
__device__ __forceinline__ uint64_t bits64_tail(const uint32_t* bm, int64_t base, int64_t row1) {
  const int64_t w = base >> 5;
  const bool two = base + 32 < row1;
  uint64_t x = ((uint64_t)(two ? ((const_u32s)bm)[w + 1] : 0u) << 32) | ((const_u32s)bm)[w];
  if (base + 64 > row1) x &= (1ull << (row1 - base)) - 1ull;
  return x;
}
__device__ __forceinline__ uint64_t vbits64_tail(const uint32_t* bm, int64_t base, int64_t row1) {
  const int64_t w = base >> 5;
  const bool two = base + 32 < row1;
  uint64_t x = ((uint64_t)(two ? bm[w + 1] : 0u) << 32) | bm[w];
  if (base + 64 > row1) x &= (1ull << (row1 - base)) - 1ull;
  return x;
}

// DecimalType conversion constants (tools/gen_dec_tables.py)
#define DQ_DEC_TABLE static __constant__ const
#include "dq_dec_tables.inc"
#undef DQ_DEC_TABLE

// raw 64-bit value of element `idx` of a column (fp64 bits; f32: the bits of the exactly widened double, Spark's
// Cast(child, DoubleType); a decimal (kind CK_D128 | scale << 8 | narrow << 16): the bits of Decimal.toDouble, the
// correctly rounded cast Corr's input gets; integers sign-extended) and its double
__device__ __forceinline__ int64_t load_raw(const char* col, int kind, int64_t idx) {
  switch (kind & 0xFF) {
    case CK_I32: return reinterpret_cast<const int32_t*>(col)[idx];
    case CK_I16: return reinterpret_cast<const int16_t*>(col)[idx];
    case CK_I8: return reinterpret_cast<const int8_t*>(col)[idx];
    case CK_F32: return __builtin_bit_cast(int64_t, (double)reinterpret_cast<const float*>(col)[idx]);
    case CK_D128: {
      const uint64_t* v = reinterpret_cast<const uint64_t*>(col) + 2 * idx;
      const DecTab tab{kDecP10Lo, kDecP10Hi, kDecRcpHi, kDecRcpLo};
      return __builtin_bit_cast(int64_t, dec_to_double(v[0], v[1], (kind >> 8) & 0xFF, tab, (kind >> 16) & 1));
    }
    default: return reinterpret_cast<const int64_t*>(col)[idx];
  }
}
// the kind's raw value is the bits of its double (fp64, f32 widened, a decimal's cast), not an integer
__device__ __forceinline__ bool raw_is_double(int kind) { return ck_float(kind) || (kind & 0xFF) == CK_D128; }
__device__ __forceinline__ double raw_to_double(int64_t raw, int kind) {
  if (raw_is_double(kind)) return __builtin_bit_cast(double, raw);
  return __builtin_fma((double)(int32_t)(raw >> 32), 4294967296.0, (double)(uint32_t)raw);  // exact int64 -> double
}
__device__ __forceinline__ int elem_bytes(int kind) { return ck_bytes(kind & 0xFF); }

// the shift of a column in a range (pointers at the range's first row, nr rows): the mean of its first 64-row group holding finite selected values
__device__ double range_shift(const char* col, int kind, const uint32_t* vb, const uint32_t* where, int64_t nr,
                              int lane) {
  for (int64_t gr = 0; gr < nr; gr += 64) {
    const int64_t r = gr + lane < nr ? gr + lane : nr - 1;
    const double x = raw_to_double(load_raw(col, kind, r), kind);
    const uint64_t fm = __builtin_amdgcn_ballot_w64(__builtin_isfinite(x)) & bits64_tail(vb, gr, nr) &
                        bits64_tail(where, gr, nr);
    if (fm != 0) return wave_sum(lane_bit(fm) ? x : 0.0) / (double)__builtin_popcountll(fm);
  }
  return 0.0;
}

// LDS ring of the fp64 path, per workgroup: kRing slots of two 64-row groups -- the 8 columns (1 KB each) and
// the 36 selection words (4 per stream: where + 8 columns); 4 slots = 33 KB, 4 workgroups per CU (deeper rings
// at 2-3 workgroups per CU measured slower: profiles/r3_pred_ab.txt, r3s)
constexpr int kRing = 4;
constexpr int kSlotBytes = 8 * 1024 + 256;
constexpr int kSlotMaskWord = 8 * 256;  // dword index of the selection words in a slot
// the fp64 ring without Min / Max reads each slot into registers one slot ahead (round 4); 0 = the round-3
// loop (kept for A/B builds: -DDQ_PAIR_PIPE=0)
#ifndef DQ_PAIR_PIPE
#define DQ_PAIR_PIPE 1
#endif
constexpr bool kPairPipe = DQ_PAIR_PIPE;
// (round 4, r4s: raising the wave's issue priority (s_setprio 2) from the slot hand-off until its DMA and LDS
// reads of the next slot are issued measured 1.535-1.540 vs 1.527-1.534 ms per 125 M rows; for the fold of a
// slot's first group instead 1.553-1.567 -- removed)


// per-lane sums of one wave task over its range
struct PairAcc {
  double s[kPairSlots][5];  // Sa, Sb, Sab, Saa, Sbb over rows selected in both positions (z = x - shift)
  double sd[kPairMoments], sdd[kPairMoments], lo[kPairMoments], hi[kPairMoments];
  int64_t is[kPairMoments];                 // wrapping int64 sums (integer columns)
  uint32_t poison;                          // checked fold: slots with a non-finite value in a row of both
  uint32_t nan[kPairMoments], pinf[kPairMoments], ninf[kPairMoments];  // checked fold (wave-uniform)
};

// Fold one 64-row group: raw values of the 8 positions, their selections m (validity & where, rows past
// the range cut).  CHECKED: selections cut to finite rows, non-finite rows accounted as Spark does.
template <bool CHECKED, bool F64, bool MINMAX>
__device__ __forceinline__ void fold(PairAcc& A, const int64_t (&raw)[kPairPos], const uint64_t (&m)[kPairPos],
                                     const double (&shift)[kPairPos], const int (&kind)[kPairPos]) {
  double x[kPairPos], z[kPairPos];
  uint64_t sel[kPairPos];
#pragma unroll
  for (int p = 0; p < kPairPos; ++p) {
    x[p] = F64 ? __builtin_bit_cast(double, raw[p]) : raw_to_double(raw[p], kind[p]);
    sel[p] = m[p];
  }
  if constexpr (CHECKED) {
    uint64_t nf[kPairPos], bad = 0;
#pragma unroll
    for (int p = 0; p < kPairPos; ++p) {
      nf[p] = m[p] & ~__builtin_amdgcn_ballot_w64(__builtin_isfinite(x[p]));
      sel[p] = m[p] & ~nf[p];
      bad |= nf[p];
    }
    if (bad != 0) {
#pragma unroll
      for (int q = 0; q < kPairSlots; ++q) {
        const int a = kPairSlotA[q], b = kPairSlotB[q];
        if (((nf[a] | nf[b]) & m[a] & m[b]) != 0) A.poison |= 1u << q;
      }
#pragma unroll
      for (int k = 0; k < kPairMoments; ++k) {
        const int p = 2 * k;
        const uint64_t nanm = __builtin_amdgcn_ballot_w64(x[p] != x[p]) & m[p];
        const uint64_t inf = nf[p] & ~nanm, pinf = __builtin_amdgcn_ballot_w64(x[p] > 0.0) & inf;
        A.nan[k] += (uint32_t)__builtin_popcountll(nanm);
        A.pinf[k] += (uint32_t)__builtin_popcountll(pinf);
        A.ninf[k] += (uint32_t)__builtin_popcountll(inf & ~pinf);
        if (MINMAX && lane_bit(inf)) {  // +-inf rows take part in min / max (NaN rows do not)
          A.lo[k] = hw_min(A.lo[k], x[p]);
          A.hi[k] = hw_max(A.hi[k], x[p]);
        }
      }
    }
  }
#pragma unroll
  for (int p = 0; p < kPairPos; ++p) z[p] = lane_bit(sel[p]) ? x[p] - shift[p] : 0.0;
  // exec-masked updates grouped by position c: the sums of the rows selected in c
#pragma unroll
  for (int c = 0; c < kPairPos; ++c) {
    if (lane_bit(sel[c])) {
#pragma unroll
      for (int q = 0; q < kPairSlots; ++q) {
        if (kPairSlotA[q] == c) {
          const double zb = z[kPairSlotB[q]];
          A.s[q][1] += zb;
          A.s[q][4] = __builtin_fma(zb, zb, A.s[q][4]);
          A.s[q][2] = __builtin_fma(z[c], zb, A.s[q][2]);
        }
        if (kPairSlotB[q] == c) {
          const double za = z[kPairSlotA[q]];
          A.s[q][0] += za;
          A.s[q][3] = __builtin_fma(za, za, A.s[q][3]);
        }
      }
      if (c % 2 == 0) {
        const int k = c / 2;
        A.sd[k] += z[c];
        A.sdd[k] = __builtin_fma(z[c], z[c], A.sdd[k]);
        if constexpr (MINMAX) {
          A.lo[k] = hw_min(A.lo[k], x[c]);
          A.hi[k] = hw_max(A.hi[k], x[c]);
        }
        if constexpr (!F64) A.is[k] = (int64_t)((uint64_t)A.is[k] + (uint64_t)(!raw_is_double(kind[c]) ? raw[c] : 0));
      }
    }
  }
}

// The unchecked fold of one 64-row group (every selected value assumed finite; a non-finite one shows in
// the sums and sends the range to the checked fold): z = x - shift in every lane, then each pair's five
// sums under exec = m(a) & m(b) -- the rows selected in both positions, so nothing is zeroed -- and each
// moments position's under exec = m(c).  One asm statement per update group, exec restored to all lanes
// at its end (the compiler never sees a partial exec).
__device__ __forceinline__ void pair_update2(double (&a)[5], double (&b)[5], double za, double zb, double zc, double zd,
                                             uint64_t ma, uint64_t mb, uint64_t mc, uint64_t md) {
  asm volatile(
      "s_and_b64 exec, %[ma], %[mb]\n\t"
      "v_add_f64 %[a0], %[a0], %[za]\n\t"
      "v_add_f64 %[a1], %[a1], %[zb]\n\t"
      "v_fma_f64 %[a2], %[za], %[zb], %[a2]\n\t"
      "v_fma_f64 %[a3], %[za], %[za], %[a3]\n\t"
      "v_fma_f64 %[a4], %[zb], %[zb], %[a4]\n\t"
      "s_and_b64 exec, %[mc], %[md]\n\t"
      "v_add_f64 %[b0], %[b0], %[zc]\n\t"
      "v_add_f64 %[b1], %[b1], %[zd]\n\t"
      "v_fma_f64 %[b2], %[zc], %[zd], %[b2]\n\t"
      "v_fma_f64 %[b3], %[zc], %[zc], %[b3]\n\t"
      "v_fma_f64 %[b4], %[zd], %[zd], %[b4]\n\t"
      "s_mov_b64 exec, -1"
      : [a0] "+v"(a[0]), [a1] "+v"(a[1]), [a2] "+v"(a[2]), [a3] "+v"(a[3]), [a4] "+v"(a[4]), [b0] "+v"(b[0]),
        [b1] "+v"(b[1]), [b2] "+v"(b[2]), [b3] "+v"(b[3]), [b4] "+v"(b[4])
      : [za] "v"(za), [zb] "v"(zb), [zc] "v"(zc), [zd] "v"(zd), [ma] "s"(ma), [mb] "s"(mb), [mc] "s"(mc), [md] "s"(md)
      : "scc");
}
// the four moments positions 0, 2, 4, 6 in one statement
template <bool MINMAX>
__device__ __forceinline__ void moment_update4(PairAcc& A, const double (&z)[kPairPos], const double (&x)[kPairPos],
                                               const uint64_t (&m)[kPairPos]) {
  if constexpr (MINMAX) {
    asm volatile(
        "s_mov_b64 exec, %[m0]\n\t"
        "v_add_f64 %[s0], %[s0], %[z0]\n\t"
        "v_fma_f64 %[t0], %[z0], %[z0], %[t0]\n\t"
        "v_min_f64 %[l0], %[l0], %[x0]\n\t"
        "v_max_f64 %[h0], %[h0], %[x0]\n\t"
        "s_mov_b64 exec, %[m1]\n\t"
        "v_add_f64 %[s1], %[s1], %[z1]\n\t"
        "v_fma_f64 %[t1], %[z1], %[z1], %[t1]\n\t"
        "v_min_f64 %[l1], %[l1], %[x1]\n\t"
        "v_max_f64 %[h1], %[h1], %[x1]\n\t"
        "s_mov_b64 exec, %[m2]\n\t"
        "v_add_f64 %[s2], %[s2], %[z2]\n\t"
        "v_fma_f64 %[t2], %[z2], %[z2], %[t2]\n\t"
        "v_min_f64 %[l2], %[l2], %[x2]\n\t"
        "v_max_f64 %[h2], %[h2], %[x2]\n\t"
        "s_mov_b64 exec, %[m3]\n\t"
        "v_add_f64 %[s3], %[s3], %[z3]\n\t"
        "v_fma_f64 %[t3], %[z3], %[z3], %[t3]\n\t"
        "v_min_f64 %[l3], %[l3], %[x3]\n\t"
        "v_max_f64 %[h3], %[h3], %[x3]\n\t"
        "s_mov_b64 exec, -1"
        : [s0] "+v"(A.sd[0]), [t0] "+v"(A.sdd[0]), [l0] "+v"(A.lo[0]), [h0] "+v"(A.hi[0]), [s1] "+v"(A.sd[1]),
          [t1] "+v"(A.sdd[1]), [l1] "+v"(A.lo[1]), [h1] "+v"(A.hi[1]), [s2] "+v"(A.sd[2]), [t2] "+v"(A.sdd[2]),
          [l2] "+v"(A.lo[2]), [h2] "+v"(A.hi[2]), [s3] "+v"(A.sd[3]), [t3] "+v"(A.sdd[3]), [l3] "+v"(A.lo[3]),
          [h3] "+v"(A.hi[3])
        : [z0] "v"(z[0]), [z1] "v"(z[2]), [z2] "v"(z[4]), [z3] "v"(z[6]), [x0] "v"(x[0]), [x1] "v"(x[2]),
          [x2] "v"(x[4]), [x3] "v"(x[6]), [m0] "s"(m[0]), [m1] "s"(m[2]), [m2] "s"(m[4]), [m3] "s"(m[6]));
  } else {
    asm volatile(
        "s_mov_b64 exec, %[m0]\n\t"
        "v_add_f64 %[s0], %[s0], %[z0]\n\t"
        "v_fma_f64 %[t0], %[z0], %[z0], %[t0]\n\t"
        "s_mov_b64 exec, %[m1]\n\t"
        "v_add_f64 %[s1], %[s1], %[z1]\n\t"
        "v_fma_f64 %[t1], %[z1], %[z1], %[t1]\n\t"
        "s_mov_b64 exec, %[m2]\n\t"
        "v_add_f64 %[s2], %[s2], %[z2]\n\t"
        "v_fma_f64 %[t2], %[z2], %[z2], %[t2]\n\t"
        "s_mov_b64 exec, %[m3]\n\t"
        "v_add_f64 %[s3], %[s3], %[z3]\n\t"
        "v_fma_f64 %[t3], %[z3], %[z3], %[t3]\n\t"
        "s_mov_b64 exec, -1"
        : [s0] "+v"(A.sd[0]), [t0] "+v"(A.sdd[0]), [s1] "+v"(A.sd[1]), [t1] "+v"(A.sdd[1]), [s2] "+v"(A.sd[2]),
          [t2] "+v"(A.sdd[2]), [s3] "+v"(A.sd[3]), [t3] "+v"(A.sdd[3])
        : [z0] "v"(z[0]), [z1] "v"(z[2]), [z2] "v"(z[4]), [z3] "v"(z[6]), [m0] "s"(m[0]), [m1] "s"(m[2]),
          [m2] "s"(m[4]), [m3] "s"(m[6]));
  }
}
template <int Q, int N>
struct SlotLoop {
  template <typename F>
  __device__ __forceinline__ static void run(F&& f) {
    f(std::integral_constant<int, Q>{});
    SlotLoop<Q + 1, N>::run(f);
  }
};
template <int N>
struct SlotLoop<N, N> {
  template <typename F>
  __device__ __forceinline__ static void run(F&&) {}
};
template <bool F64, bool MINMAX>
__device__ __forceinline__ void fold_fast(PairAcc& A, const int64_t (&raw)[kPairPos], const uint64_t (&m)[kPairPos],
                                          const double (&shift)[kPairPos], const int (&kind)[kPairPos]) {
  double x[kPairPos], z[kPairPos];
#pragma unroll
  for (int p = 0; p < kPairPos; ++p) {
    x[p] = F64 ? __builtin_bit_cast(double, raw[p]) : raw_to_double(raw[p], kind[p]);
    z[p] = x[p] - shift[p];
  }
  static_assert(kPairSlots % 2 == 0, "slots go in twos");
  SlotLoop<0, kPairSlots / 2>::run([&](auto qc) {
    constexpr int q = 2 * decltype(qc)::value;
    constexpr int a = kPairSlotA[q], b = kPairSlotB[q], c = kPairSlotA[q + 1], d = kPairSlotB[q + 1];
    pair_update2(A.s[q], A.s[q + 1], z[a], z[b], z[c], z[d], m[a], m[b], m[c], m[d]);
  });
  moment_update4<MINMAX>(A, z, x, m);
  if constexpr (!F64) {
#pragma unroll
    for (int k = 0; k < kPairMoments; ++k)
      if (!raw_is_double(kind[2 * k]) && lane_bit(m[2 * k])) A.is[k] = (int64_t)((uint64_t)A.is[k] + (uint64_t)raw[2 * k]);
  }
}

// One wave task over one row range: fold every 64-row group, then (CHECKED or all sums finite) the counts
// and the CorrPartial / ColPartial records.  Returns false (nothing written) when an unchecked fold met a
// non-finite sum.
template <bool CHECKED, bool F64, bool MINMAX, bool RING>
__device__ __forceinline__ bool pair_range(const PairWaveTask& T, const ScanCols& cols, const uint32_t* where,
                                           const uint32_t* ones, int64_t row0, int64_t row1, int32_t range,
                                           CorrPartial* __restrict__ pair_part, ColPartial* __restrict__ col_part,
                                           int64_t* ring, bool active) {
  const int lane = threadIdx.x & 63;
  // everything from here on in range-local rows [0, nr): base pointers moved to row0 (a multiple of 64)
  const int64_t nr = row1 - row0;
  const char* vp[kPairPos];      // values
  const uint32_t* vw[kPairPos];  // validity bitmaps (all-ones stand-in)
  int kind[kPairPos];
  double shift[kPairPos];        // wave-uniform (SGPRs)
  const uint32_t* ww = where + (row0 >> 5);
#pragma unroll
  for (int p = 0; p < kPairPos; ++p) {
    const int c = T.cols[p];
    kind[p] = F64 ? CK_F64 : T.kinds[p];
    vw[p] = (cols.validity[c] ? cols.validity[c] : ones) + (row0 >> 5);
    vp[p] = reinterpret_cast<const char*>(cols.values[c]) + row0 * elem_bytes(kind[p]);
    shift[p] = uniform(range_shift(vp[p], kind[p], vw[p], ww, nr, lane));
  }
  PairAcc A;
#pragma unroll
  for (int q = 0; q < kPairSlots; ++q)
#pragma unroll
    for (int k = 0; k < 5; ++k) A.s[q][k] = 0.0;
#pragma unroll
  for (int k = 0; k < kPairMoments; ++k) {
    A.sd[k] = A.sdd[k] = 0.0;
    A.lo[k] = __builtin_bit_cast(double, 0x7FF0000000000000ull);
    A.hi[k] = __builtin_bit_cast(double, 0xFFF0000000000000ull);
    A.is[k] = 0;
    A.nan[k] = A.pinf[k] = A.ninf[k] = 0;
  }
  A.poison = 0;

  const int64_t nfull = nr >> 6;
  if constexpr (RING) {
    // ---- full groups through the workgroup's LDS ring (kRing slots of two 64-row groups each): the two
    // waves stage each slot together, wave 0 the slot's columns 0-3 and the where / column 0-3 selection
    // words, wave 1 columns 4-7 and their selection words -- five DMA loads each (global_load_lds; every
    // lane brings 16 bytes = 2 rows of a column, the 1 KB of a column's two groups in one instruction; one
    // lane per selection dword, 4 per stream), kRing - 1 slots ahead of the fold, no VGPRs held.  One
    // s_barrier per slot: past it the partner's loads of slot s have landed (each wave waits for its own
    // first) and the partner has folded slot s - 1, whose ring slot is then restaged.
    static_assert(F64 && !CHECKED, "the ring path stages fp64 values");
    constexpr int D = kRing - 1;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)ring);
    const bool has_where = T.where >= 0;
    // selection dwords of a slot: stream s (0 = where, 1 + c = column c) at 4 s .. 4 s + 3 (two words per
    // group); wave 0 stages streams 0-4 (lanes 0-19), wave 1 streams 5-8 (lanes 0-15); wave w's position p
    // is column p + w (mod 8).
    const uint32_t* mp;
    if (wave == 0) {
      mp = ww;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (lane >> 2 == c + 1) mp = vw[c];
    } else {
      mp = vw[3];
#pragma unroll
      for (int c = 1; c < 4; ++c)
        if (lane >> 2 == c) mp = vw[3 + c];
    }
    mp += lane & 3;
    const uint64_t mexec = wave == 0 ? 0xFFFFFull : 0xFFFFull;
    const uint32_t moff = (uint32_t)kSlotMaskWord * 4u + (wave == 0 ? 0u : 80u);
    // the four columns this wave stages: wave 0 positions 0-3, wave 1 positions 3-6 (= columns 4-7)
    const char* dp[4];
    const int p0 = wave == 0 ? 0 : 3;
#pragma unroll
    for (int k = 0; k < 4; ++k) dp[k] = reinterpret_cast<const char*>(cols.values[T.cols[p0 + k]]) + row0 * 8;
    const uint32_t dcol = wave == 0 ? 0u : 4096u;  // LDS byte offset of the first staged column
    const int64_t npair = nfull >> 1;             // ring slots (two full groups each)
    auto dma = [&](int64_t s, uint32_t slot) __attribute__((always_inline)) {
      const uint32_t sc = (uint32_t)(s < npair ? s : npair - 1);
      const uint32_t voff = sc * 1024u + (uint32_t)lane * 16u;
      const uint32_t d = lds0 + slot * (uint32_t)kSlotBytes + dcol;
      const uint32_t dm = lds0 + slot * (uint32_t)kSlotBytes + moff;
      const uint32_t* ma = mp + 4 * sc;
      uint32_t keep;
      uint64_t sv;
      asm volatile(
          "s_mov_b32 %[keep], m0\n\t"
          "s_mov_b64 %[sv], exec\n\t"
          "s_mov_b32 m0, %[d]\n\t"
          "s_nop 0\n\t"
          "global_load_lds_dwordx4 %[vo], %[b0] nt\n\t"
          "s_add_u32 m0, %[d], 0x400\n\t"
          "s_nop 0\n\t"
          "global_load_lds_dwordx4 %[vo], %[b1] nt\n\t"
          "s_add_u32 m0, %[d], 0x800\n\t"
          "s_nop 0\n\t"
          "global_load_lds_dwordx4 %[vo], %[b2] nt\n\t"
          "s_add_u32 m0, %[d], 0xc00\n\t"
          "s_nop 0\n\t"
          "global_load_lds_dwordx4 %[vo], %[b3] nt\n\t"
          "s_mov_b64 exec, %[me]\n\t"
          "s_mov_b32 m0, %[dm]\n\t"
          "s_nop 0\n\t"
          "global_load_lds_dword %[ma], off\n\t"
          "s_mov_b64 exec, %[sv]\n\t"
          "s_mov_b32 m0, %[keep]"
          : [keep] "=&s"(keep), [sv] "=&s"(sv)
          : [vo] "v"(voff), [d] "s"(d), [dm] "s"(dm), [me] "s"(mexec), [b0] "s"(dp[0]), [b1] "s"(dp[1]),
            [b2] "s"(dp[2]), [b3] "s"(dp[3]), [ma] "v"(ma)
          : "memory", "scc");
    };
    if constexpr (kPairPipe && !MINMAX) {
      // ---- pipelined ring (round 4): a slot's values and selection words are read into registers one slot
      // ahead, so the LDS latency hides behind the second half of the previous slot's fold, and the barrier
      // sits between the two halves.  Iteration s: fold group 0 of slot s; wait until this wave's slot s
      // registers and its own DMA of slot s + 1 have landed; s_barrier (past it the partner holds slot s in
      // registers and its DMA of slot s + 1 has landed); DMA slot s + kRing into slot s's ring position; read
      // slot s + 1; fold group 1 of slot s.  (The barrier is not what limits the pass: a diagnostic build
      // without it -- results wrong -- ran 1.554-1.556 vs 1.535-1.536 ms per 125 M rows, r4j.)  Branch-free addressing: position p reads ring column
      // (p + wave) % 8, i.e. positions 0-6 at xa + 128 p and position 7 at xb.
      const int64_t* xa = ring + lane + wave * 128;
      const int64_t* xb = ring + lane + (wave == 0 ? 7 * 128 : 0);
      // selection dwords of both groups in one read: lanes 0-15 the stream of position lane / 2, lanes 16
      // and 17 the where stream (dword 2 further on = the slot's second group)
      const uint32_t* mq = reinterpret_cast<const uint32_t*>(ring) + kSlotMaskWord +
                           (lane < 16 ? 4 + 4 * (((lane >> 1) + wave) & 7) + (lane & 1) : (lane & 1));
      struct SlotRegs {
        int64_t v[2][kPairPos];
        uint32_t m[2];
      };
      auto rd = [&](SlotRegs& R, uint32_t slot) __attribute__((always_inline)) {
        const int64_t* a = xa + slot * (uint32_t)(kSlotBytes / 8);
        const int64_t* b = xb + slot * (uint32_t)(kSlotBytes / 8);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
          for (int p = 0; p < kPairPos - 1; ++p) R.v[h][p] = a[p * 128 + 64 * h];
          R.v[h][kPairPos - 1] = b[64 * h];
        }
        const uint32_t* q = mq + slot * (uint32_t)(kSlotBytes / 4);
        R.m[0] = q[0];
        R.m[1] = q[2];
      };
      auto fold_group = [&](const int64_t (&v)[kPairPos], uint32_t mv) __attribute__((always_inline)) {
        auto word = [](uint32_t x, int i) {
          return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(x, i + 1) << 32) |
                 (uint32_t)__builtin_amdgcn_readlane(x, i);
        };
        uint64_t m[kPairPos];
#pragma unroll
        for (int p = 0; p < kPairPos; ++p) m[p] = word(mv, 2 * p);
        if (has_where) {
          const uint64_t wm = word(mv, 16);
#pragma unroll
          for (int p = 0; p < kPairPos; ++p) m[p] &= wm;
        }
        if (active) fold_fast<true, false>(A, v, m, shift, kind);
      };
      // this wave's own DMA of slot t landed, with `after` slots issued after it (uniform; 5 loads per slot)
      static_assert(kRing == 4, "the waits below count up to three slots after the awaited one");
      auto wait_slot = [](int32_t after) __attribute__((always_inline)) {
        if (after >= 3) asm volatile("s_waitcnt vmcnt(15) lgkmcnt(0)" ::: "memory");
        else if (after == 2) asm volatile("s_waitcnt vmcnt(10) lgkmcnt(0)" ::: "memory");
        else if (after == 1) asm volatile("s_waitcnt vmcnt(5) lgkmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      };
      // one ring slot: R holds slot s (its reads issued), N receives slot s + 1.  Slots past the range's
      // last are never staged (no wasted loads; the waits count what was issued).  32-bit slot numbers: the
      // scalar unit has no 64-bit ordered compare.
      const int32_t ns = (int32_t)npair;
      auto iter = [&](SlotRegs& R, SlotRegs& N, int32_t s, uint32_t slot) __attribute__((always_inline)) {
        fold_group(R.v[0], R.m[0]);
        if (s + 1 < ns) {
          // issued after slot s + 1: slots s + 2 .. min(s + kRing - 1, ns - 1)
          const int32_t last = s + kRing - 1 < ns - 1 ? s + kRing - 1 : ns - 1;
          wait_slot(last - (s + 1));
          __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");
          if (s + kRing < ns) dma(s + kRing, slot);
          rd(N, (slot + 1) & (kRing - 1));
        }
        fold_group(R.v[1], R.m[1]);
      };
      if (ns > 0) {
#pragma unroll
        for (int d = 0; d < kRing; ++d)
          if (d < ns) dma(d, (uint32_t)d);
        wait_slot((ns < kRing ? ns : kRing) - 1);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        SlotRegs R0, R1;
        rd(R0, 0u);
        uint32_t slot = 0;
        int32_t s = 0;
        for (; s + 2 <= ns; s += 2) {
          iter(R0, R1, s, slot);
          iter(R1, R0, s + 1, slot + 1);
          slot = (slot + 2) & (kRing - 1);
        }
        if (s < ns) iter(R0, R1, s, slot);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may outlive the workgroup (its LDS is reused)
      }
    } else {
    // this wave's positions: ring column (p + wave) % 8; selection words of half h: lanes 0, 1 of the first
    // read = where, lanes 2 p, 2 p + 1 of the second = position p
    const int64_t* xs0 = ring + lane;
    const uint32_t* ms0 = reinterpret_cast<const uint32_t*>(ring) + kSlotMaskWord;
    const int mlw = lane & 1, mlc = lane < 16 ? 4 + 4 * (((lane >> 1) + wave) & 7) + (lane & 1) : 0;
    auto half = [&](const int64_t* xs, const uint32_t* ms) __attribute__((always_inline)) {
      int64_t b[kPairPos];
      if (wave == 0) {
#pragma unroll
        for (int p = 0; p < kPairPos; ++p) b[p] = xs[p * 128];
      } else {
#pragma unroll
        for (int p = 0; p < kPairPos; ++p) b[p] = xs[((p + 1) % kPairPos) * 128];
      }
      const uint32_t mc = ms[mlc];
      auto word = [](uint32_t v, int i) {
        return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(v, i + 1) << 32) | (uint32_t)__builtin_amdgcn_readlane(v, i);
      };
      uint64_t m[kPairPos];
#pragma unroll
      for (int p = 0; p < kPairPos; ++p) m[p] = word(mc, 2 * p);
      if (has_where) {
        const uint64_t wm = word(ms[mlw], 0);
#pragma unroll
        for (int p = 0; p < kPairPos; ++p) m[p] &= wm;
      }
      if (active) fold_fast<true, MINMAX>(A, b, m, shift, kind);
    };
    auto one = [&](int64_t s, uint32_t slot) __attribute__((always_inline)) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(5 * (D - 1)) : "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      dma(s + D, slot == 0 ? (uint32_t)(kRing - 1) : slot - 1);
      const int64_t* xs = xs0 + slot * (kSlotBytes / 8);
      const uint32_t* ms = ms0 + slot * (kSlotBytes / 4);
      half(xs, ms);
      half(xs + 64, ms + 2);
    };
    if (npair > 0) {
#pragma unroll
      for (int d = 0; d < D; ++d) dma(d, (uint32_t)d);
      uint32_t slot = 0;
      for (int64_t s = 0; s < npair; ++s) {
        one(s, slot);
        slot = slot + 1 == kRing ? 0 : slot + 1;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may outlive the workgroup (its LDS is reused)
    }
    }
    if (!active) return true;
    // the column pointers again for the tail and the counts (reloaded, not held in SGPRs through the loop)
    const PairWaveTask* tp = &T;  // laundered: the column indices are loaded again (never &cols: that copies
    asm volatile("" : "+s"(tp));  // the kernel-argument struct to scratch)
#pragma unroll
    for (int p = 0; p < kPairPos; ++p) {
      const int c = tp->cols[p];
      vw[p] = (cols.validity[c] ? cols.validity[c] : ones) + (row0 >> 5);
      vp[p] = reinterpret_cast<const char*>(cols.values[c]) + row0 * 8;
    }
    // an odd last full group (only at the end of the scan): values and masks loaded directly
    for (int64_t g = 2 * npair; g < nfull; ++g) {
      int64_t b[kPairPos];
      uint64_t m[kPairPos];
      const uint32_t off = (uint32_t)g * 8u;
      const uint64_t wm = sword_at(ww, off);
#pragma unroll
      for (int p = 0; p < kPairPos; ++p) {
        b[p] = *reinterpret_cast<const int64_t*>(vp[p] + ((uint32_t)g * 64u + (uint32_t)lane) * 8u);
        const uint64_t mv = sword_at(vw[p], off) & wm;  // uniform, but the reloaded pointers look divergent
        m[p] = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(mv >> 32)) << 32) |
               (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)mv);
      }
      fold_fast<true, MINMAX>(A, b, m, shift, kind);
    }
  } else {
  // ---- full groups: values two groups ahead of the fold (three rotating buffers; two with Min / Max or
  // conversions, for VGPRs), masks by scalar loads; 32-bit offsets from the scalar base pointers
  auto load = [&](int64_t (&b)[kPairPos], int64_t g) __attribute__((always_inline)) {
    const uint32_t li = (uint32_t)(g < nfull ? g : nfull - 1) * 64u + (uint32_t)lane;
#pragma unroll
    for (int p = 0; p < kPairPos; ++p)
      b[p] = F64 ? *reinterpret_cast<const int64_t*>(vp[p] + li * 8u) : load_raw(vp[p], kind[p], li);
  };
  auto step = [&](const int64_t (&b)[kPairPos], int64_t g) __attribute__((always_inline)) {
    const uint32_t off = (uint32_t)g * 8u;
    const uint64_t wm = sword_at(ww, off);
    uint64_t m[kPairPos];
#pragma unroll
    for (int p = 0; p < kPairPos; ++p) m[p] = sword_at(vw[p], off) & wm;
    if constexpr (CHECKED) fold<true, F64, MINMAX>(A, b, m, shift, kind);
    else fold_fast<F64, MINMAX>(A, b, m, shift, kind);
  };
  if (nfull > 0) {
    int64_t b0[kPairPos], b1[kPairPos];
    load(b0, 0);
    load(b1, 1);
    int64_t g = 0;
    if constexpr (F64 && !MINMAX) {
      int64_t b2[kPairPos];
      for (; g + 3 <= nfull; g += 3) {
        load(b2, g + 2);
        step(b0, g);
        load(b0, g + 3);
        step(b1, g + 1);
        load(b1, g + 4);
        step(b2, g + 2);
      }
    } else {
      for (; g + 2 <= nfull; g += 2) {
        step(b0, g);
        load(b0, g + 2);
        step(b1, g + 1);
        load(b1, g + 3);
      }
    }
    if (g < nfull) step(b0, g);
    if (g + 1 < nfull) step(b1, g + 1);
  }
  }
  // ---- the range's last rows (< 64; only at the end of the scan)
  const int64_t tb = nfull * 64;
  if (tb < nr) {
    const int64_t r = tb + lane < nr ? tb + lane : nr - 1;
    int64_t b[kPairPos];
    uint64_t m[kPairPos];
    const uint64_t wm = bits64_tail(ww, tb, nr);
#pragma unroll
    for (int p = 0; p < kPairPos; ++p) {
      b[p] = load_raw(vp[p], kind[p], r);
      m[p] = bits64_tail(vw[p], tb, nr) & wm;
    }
    fold<CHECKED, F64, MINMAX>(A, b, m, shift, kind);
  }

  if constexpr (!CHECKED) {  // a non-finite active sum: leave the range to the checked fold
    bool ok = true;
#pragma unroll
    for (int q = 0; q < kPairSlots; ++q)
      if ((T.pair_mask >> q) & 1u)
#pragma unroll
        for (int k = 0; k < 5; ++k) ok = ok && __builtin_isfinite(A.s[q][k]);
#pragma unroll
    for (int k = 0; k < kPairMoments; ++k)
      if ((T.mom_mask >> k) & 1u) ok = ok && __builtin_isfinite(A.sd[k]) && __builtin_isfinite(A.sdd[k]);
    if (__builtin_amdgcn_ballot_w64(!ok) != 0) return false;
  }

  // ---- counts: rows selected in both positions of a slot / in a moments position (lane per bitmap word)
  uint32_t pc[kPairSlots], mc[kPairMoments];
#pragma unroll
  for (int q = 0; q < kPairSlots; ++q) pc[q] = 0;
#pragma unroll
  for (int k = 0; k < kPairMoments; ++k) mc[k] = 0;
  for (int64_t base = 64 * lane; base < nr; base += 64 * 64) {
    const uint64_t wm = vbits64_tail(ww, base, nr);
    uint64_t w[kPairPos];
#pragma unroll
    for (int p = 0; p < kPairPos; ++p) w[p] = vbits64_tail(vw[p], base, nr) & wm;
#pragma unroll
    for (int q = 0; q < kPairSlots; ++q) pc[q] += (uint32_t)__builtin_popcountll(w[kPairSlotA[q]] & w[kPairSlotB[q]]);
#pragma unroll
    for (int k = 0; k < kPairMoments; ++k) mc[k] += (uint32_t)__builtin_popcountll(w[2 * k]);
  }

  // ---- close: wave sums (fixed butterfly order), then the (n, means, co-moments) of this range
#pragma unroll
  for (int q = 0; q < kPairSlots; ++q) {
    if (!((T.pair_mask >> q) & 1u)) continue;
    double S[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) S[k] = wave_sum(A.s[q][k]);
    const uint32_t cnt = wave_sum_u32(pc[q]);
    if (lane == 0) {
      CorrPartial* o = pair_part + (size_t)T.pair_out[q] * kMaxWG + range;
      const double n = (double)cnt;
      CorrPartial r{0, 0, 0, 0, 0, 0, 0, 0};
      if (cnt > 0 && ((A.poison >> q) & 1u)) {
        const double nan = __builtin_bit_cast(double, 0x7FF8000000000000ull);
        r = CorrPartial{n, nan, nan, nan, nan, nan, 0, 0};
      } else if (cnt > 0) {
        const double qx = S[0] / n, qy = S[1] / n;
        const double xa = shift[kPairSlotA[q]] + qx, ya = shift[kPairSlotB[q]] + qy;
        const double xm = S[3] - S[0] * qx, ym = S[4] - S[1] * qy;
        const bool sw = (T.swap_mask >> q) & 1u;  // Correlation(first, second) with first at position B
        r.n = n;
        r.xa = sw ? ya : xa;
        r.ya = sw ? xa : ya;
        r.ck = S[2] - S[0] * qy;
        r.xm = sw ? ym : xm;
        r.ym = sw ? xm : ym;
      }
      *o = r;
    }
  }
#pragma unroll
  for (int k = 0; k < kPairMoments; ++k) {
    if (!((T.mom_mask >> k) & 1u)) continue;
    const double S1 = wave_sum(A.sd[k]), S2 = wave_sum(A.sdd[k]);
    const double fmin = wave_min(A.lo[k]), fmax = wave_max(A.hi[k]);
    const int64_t isum = wave_sum_i64(A.is[k]);
    const int64_t count = wave_sum_u32(mc[k]);
    const int64_t nan = A.nan[k], pinf = A.pinf[k], ninf = A.ninf[k];
    if (lane == 0) {
      const int64_t nm = count - pinf - ninf;
      const double sh = shift[2 * k];
      ColPartial r;
      r.n = (double)nm;
      r.mean = 0.0;
      r.m2 = 0.0;
      r.sum = 0.0;
      if (nm > 0) {
        const double q1 = S1 / (double)nm;
        r.mean = sh + q1;
        r.m2 = S2 - S1 * q1;
        r.sum = __builtin_fma((double)nm, sh, S1);
        if (nan > 0) {  // NaN rows were kept out of the sums: Spark's moments and sum are NaN
          r.mean = r.m2 = r.sum = __builtin_bit_cast(double, 0x7FF8000000000000ull);
        }
      }
      r.isum = isum;
      r.count = count;
      r.nan_count = nan;
      r.fmin = fmin;
      r.fmax = fmax;
      r.pinf_count = pinf;
      r.ninf_count = ninf;
      r.isum_hi = 0;
      col_part[(size_t)T.mom_out[k] * kMaxWG + range] = r;
    }
  }
  return true;
}

}  // namespace

// F64: every position fp64 (no conversions, no integral sums).  MINMAX: a moments task feeds Min / Max.
// RING: fp64 values staged through the per-wave LDS ring (16-byte aligned columns).  Two waves per SIMD
// (<= 256 VGPRs): the other wave's VALU hides this one's scalar work and waits.
template <bool F64, bool MINMAX, bool RING>
__global__ __launch_bounds__(64 * kPairWaves) __attribute__((amdgpu_waves_per_eu(2))) void dq_pair_scan(
    const PairWG* __restrict__ wgs, int32_t nwg, ScanCols cols, ScanBitmaps bm, const uint32_t* ones, int64_t n_rows,
    int64_t rows_per_range, CorrPartial* __restrict__ pair_part, ColPartial* __restrict__ col_part,
    int32_t* __restrict__ redo) {
  const int gi = blockIdx.x % nwg, range = blockIdx.x / nwg;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const PairWaveTask& T = wgs[gi].wave[wave];
  const bool active = (T.pair_mask | T.mom_mask) != 0;
  // the ring path's waves stage the group together: an idle wave still stages its half
  if (RING ? !active && (wgs[gi].wave[wave ^ 1].pair_mask | wgs[gi].wave[wave ^ 1].mom_mask) == 0 : !active) return;
  const int64_t row0 = (int64_t)range * rows_per_range;
  const int64_t row1 = row0 + rows_per_range < n_rows ? row0 + rows_per_range : n_rows;
  const uint32_t* where = T.where >= 0 ? reinterpret_cast<const uint32_t*>(bm.where_bits[T.where]) : ones;
  int64_t* ring = nullptr;
  if constexpr (RING) {
    __shared__ __attribute__((aligned(16))) int64_t ring_lds[kRing * kSlotBytes / 8];
    ring = ring_lds;
  }
  const bool done = pair_range<false, F64, MINMAX, RING>(T, cols, where, ones, row0, row1, range, pair_part,
                                                          col_part, ring, active);
  if ((threadIdx.x & 63) == 0) redo[((size_t)gi * kPairWaves + wave) * kMaxWG + range] = done ? 0 : 1;
}

// the (wave task, range) units dq_pair_scan flagged, re-run with the checked fold
__global__ __launch_bounds__(64 * kPairWaves) void dq_pair_redo(const PairWG* __restrict__ wgs, int32_t nwg,
                                                                ScanCols cols, ScanBitmaps bm, const uint32_t* ones,
                                                                int64_t n_rows, int64_t rows_per_range,
                                                                CorrPartial* __restrict__ pair_part,
                                                                ColPartial* __restrict__ col_part,
                                                                const int32_t* __restrict__ redo) {
  const int gi = blockIdx.x % nwg, range = blockIdx.x / nwg;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const PairWaveTask& T = wgs[gi].wave[wave];
  if ((T.pair_mask | T.mom_mask) == 0) return;
  if (redo[((size_t)gi * kPairWaves + wave) * kMaxWG + range] == 0) return;
  const int64_t row0 = (int64_t)range * rows_per_range;
  const int64_t row1 = row0 + rows_per_range < n_rows ? row0 + rows_per_range : n_rows;
  const uint32_t* where = T.where >= 0 ? reinterpret_cast<const uint32_t*>(bm.where_bits[T.where]) : ones;
  (void)pair_range<true, false, true, false>(T, cols, where, ones, row0, row1, range, pair_part, col_part, nullptr,
                                             true);
}

// workgroups of the pair pass one CU holds at once (the occupancy API for the launch the flags select)
hipError_t pair_scan_residency(bool all_f64, bool ring, bool minmax, int32_t* per_cu) {
  int nb = 0;
  hipError_t e;
  const int threads = 64 * kPairWaves;
  if (all_f64 && ring) {
    e = minmax ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, dq_pair_scan<true, true, true>, threads, 0)
               : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, dq_pair_scan<true, false, true>, threads, 0);
  } else if (all_f64) {
    e = minmax ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, dq_pair_scan<true, true, false>, threads, 0)
               : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, dq_pair_scan<true, false, false>, threads, 0);
  } else {
    e = minmax ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, dq_pair_scan<false, true, false>, threads, 0)
               : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, dq_pair_scan<false, false, false>, threads, 0);
  }
  *per_cu = nb;
  return e;
}

hipError_t launch_pair_scan(const PairWG* wgs, int32_t nwg, const ScanCols& cols, const ScanBitmaps& bm,
                            const uint32_t* ones, int64_t n_rows, int64_t rows_per_range, int32_t nranges,
                            CorrPartial* pair_part, ColPartial* col_part, int32_t* redo, bool all_f64, bool ring,
                            bool minmax, hipStream_t st) {
  const uint32_t blocks = (uint32_t)nwg * (uint32_t)nranges;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64 * kPairWaves), 0, st, wgs, nwg, cols, bm, ones, n_rows,
                       rows_per_range, pair_part, col_part, redo);
  };
  if (all_f64 && ring) {
    if (minmax) go(dq_pair_scan<true, true, true>);
    else go(dq_pair_scan<true, false, true>);
  } else if (all_f64) {
    if (minmax) go(dq_pair_scan<true, true, false>);
    else go(dq_pair_scan<true, false, false>);
  } else {
    if (minmax) go(dq_pair_scan<false, true, false>);
    else go(dq_pair_scan<false, false, false>);
  }
  hipLaunchKernelGGL(dq_pair_redo, dim3(blocks), dim3(64 * kPairWaves), 0, st, wgs, nwg, cols, bm, ones, n_rows,
                     rows_per_range, pair_part, col_part, (const int32_t*)redo);
  return hipGetLastError();
}

}  // namespace dq
