// dq_pair.hip -- gfx950 kernels of the Correlation pass fused with the column moments of the same columns.
//
// Reference: Correlation (analyzers/Correlation.scala:26-105, catalyst/StatefulCorrelation.scala:24-49:
// Spark's Corr co-moments, merged with Chan's formula Correlation.scala:37-52) and the moments of Mean /
// StandardDeviation / Sum / Minimum / Maximum (StandardDeviation.scala:37-44 merge) -- all aggregates of
// the one data.agg(...) pass (AnalysisRunner.scala:303).  Config C4 asks for 28 correlations over 8 fp64
// columns fused with their Mean and StdDev: every column is read from HBM once for all of that.
//
// Layout.  A workgroup task (PairWG, planned on the host) is one pair group (<= 8 columns, one `where`)
// and two wave tasks; a workgroup is two waves and one row range, and the waves never synchronise.  Wave
// w's position p holds the group's local column (p + w) % 8 and runs the fixed 14-slot pattern
// kPairSlotA / kPairSlotB over its positions -- the two rotations of the pattern are the 28 pairs of 8
// columns, each once -- plus the moments of its even positions.  Lane l takes row l of each 64-row group:
// the 8 values come straight from HBM into VGPRs (two groups in flight ahead of the fold; the other wave
// of the workgroup reads the same lines, an L1 / L2 hit), a position's selection (validity & where) is a
// 64-bit SGPR mask read by a scalar load, and with z = x - shift zeroed outside the selection the pair
// sums are exec-masked VALU updates grouped by position:
//   exec = sel(a):  Sb += zb   Sbb += zb^2   Sab += za zb        exec = sel(b):  Sa += za   Saa += za^2
// i.e. five fp64 VALU per pair and 64 rows, nothing for the counts: a pair's count (rows selected in both
// columns) and a column's count are popcounts of bitmap words, taken at the end of the range by a
// lane-per-word pass over the bitmaps (1/64 of the value bytes).
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

// raw 64-bit value of element `idx` of a column (fp64 bits, or the integer sign-extended) and its double
__device__ __forceinline__ int64_t load_raw(const char* col, int kind, int64_t idx) {
  if (kind == CK_I32) return reinterpret_cast<const int32_t*>(col)[idx];
  return reinterpret_cast<const int64_t*>(col)[idx];
}
__device__ __forceinline__ double raw_to_double(int64_t raw, int kind) {
  if (kind == CK_F64) return __builtin_bit_cast(double, raw);
  return __builtin_fma((double)(int32_t)(raw >> 32), 4294967296.0, (double)(uint32_t)raw);  // exact int64 -> double
}
__device__ __forceinline__ int elem_bytes(int kind) { return kind == CK_I32 ? 4 : 8; }

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
        if constexpr (!F64) A.is[k] = (int64_t)((uint64_t)A.is[k] + (uint64_t)(kind[c] != CK_F64 ? raw[c] : 0));
      }
    }
  }
}

// One wave task over one row range: fold every 64-row group, then (CHECKED or all sums finite) the counts
// and the CorrPartial / ColPartial records.  Returns false (nothing written) when an unchecked fold met a
// non-finite sum.
template <bool CHECKED, bool F64, bool MINMAX>
__device__ __forceinline__ bool pair_range(const PairWaveTask& T, const ScanCols& cols, const uint32_t* where,
                                           const uint32_t* ones, int64_t row0, int64_t row1, int32_t range,
                                           CorrPartial* __restrict__ pair_part, ColPartial* __restrict__ col_part) {
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

  // ---- full groups: values two groups ahead of the fold (three rotating buffers; two with Min / Max or
  // conversions, for VGPRs), masks by scalar loads; 32-bit offsets from the scalar base pointers
  const int64_t nfull = nr >> 6;
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
    fold<CHECKED, F64, MINMAX>(A, b, m, shift, kind);
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
      r.pad = 0;
      col_part[(size_t)T.mom_out[k] * kMaxWG + range] = r;
    }
  }
  return true;
}

}  // namespace

// F64: every position fp64 (no conversions, no integral sums).  MINMAX: a moments task feeds Min / Max.
// Two waves per SIMD (<= 256 VGPRs): the other wave's VALU hides this one's scalar work and load waits.
template <bool F64, bool MINMAX>
__global__ __launch_bounds__(64 * kPairWaves) __attribute__((amdgpu_waves_per_eu(2))) void dq_pair_scan(
    const PairWG* __restrict__ wgs, int32_t nwg, ScanCols cols, ScanBitmaps bm, const uint32_t* ones, int64_t n_rows,
    int64_t rows_per_range, CorrPartial* __restrict__ pair_part, ColPartial* __restrict__ col_part,
    int32_t* __restrict__ redo) {
  const int gi = blockIdx.x % nwg, range = blockIdx.x / nwg;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const PairWaveTask& T = wgs[gi].wave[wave];
  if ((T.pair_mask | T.mom_mask) == 0) return;
  const int64_t row0 = (int64_t)range * rows_per_range;
  const int64_t row1 = row0 + rows_per_range < n_rows ? row0 + rows_per_range : n_rows;
  const uint32_t* where = T.where >= 0 ? reinterpret_cast<const uint32_t*>(bm.where_bits[T.where]) : ones;
  const bool done = pair_range<false, F64, MINMAX>(T, cols, where, ones, row0, row1, range, pair_part, col_part);
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
  (void)pair_range<true, false, true>(T, cols, where, ones, row0, row1, range, pair_part, col_part);
}

hipError_t launch_pair_scan(const PairWG* wgs, int32_t nwg, const ScanCols& cols, const ScanBitmaps& bm,
                            const uint32_t* ones, int64_t n_rows, int64_t rows_per_range, int32_t nranges,
                            CorrPartial* pair_part, ColPartial* col_part, int32_t* redo, bool all_f64, bool minmax,
                            hipStream_t st) {
  const uint32_t blocks = (uint32_t)nwg * (uint32_t)nranges;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64 * kPairWaves), 0, st, wgs, nwg, cols, bm, ones, n_rows,
                       rows_per_range, pair_part, col_part, redo);
  };
  if (all_f64) {
    if (minmax) go(dq_pair_scan<true, true>);
    else go(dq_pair_scan<true, false>);
  } else {
    if (minmax) go(dq_pair_scan<false, true>);
    else go(dq_pair_scan<false, false>);
  }
  hipLaunchKernelGGL(dq_pair_redo, dim3(blocks), dim3(64 * kPairWaves), 0, st, wgs, nwg, cols, bm, ones, n_rows,
                     rows_per_range, pair_part, col_part, (const int32_t*)redo);
  return hipGetLastError();
}

}  // namespace dq
