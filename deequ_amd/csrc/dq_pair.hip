// dq_pair.hip -- gfx950 kernel of the Correlation pass fused with the column moments of the same columns.
//
// Reference: Correlation (analyzers/Correlation.scala:26-105, catalyst/StatefulCorrelation.scala:24-49:
// Spark's Corr co-moments, merged with Chan's formula Correlation.scala:37-52) and the moments of Mean /
// StandardDeviation / Sum / Minimum / Maximum (StandardDeviation.scala:37-44 merge) -- all aggregates of
// the one data.agg(...) pass (AnalysisRunner.scala:303).  Config C4 asks for 28 correlations over 8 fp64
// columns fused with their Mean and StdDev: every column is read from HBM ONCE for all of that.
//
// Layout: lane-per-row.  A wave task (PairWaveTask, planned on the host) owns up to 5 columns of a pair
// group ("positions"), the pairs among them it is responsible for (active slots of the fixed 10-slot
// pattern of all position pairs, so register indices are compile-time) and the moment tasks of positions
// 0 and 1.  Lane l of the wave holds row base + l of every position: values come in as coalesced 512-byte
// loads, the validity (& where) bits of 64 rows are one 64-bit SGPR mask per column, a pair's selection is
// one s_and of two masks, and its update is exec-masked -- 5 fp64 VALU per pair and row, nothing for an
// unselected row.  Sums are kept around a per-(wave, range) shift per column (the mean of its first
// finite selected values), so the closing formulas m2 = S2 - S1^2 / n and ck = Sxy - Sx Sy / n lose
// nothing measurable (full-scale check: tests/fullscale_parity.py).  Counts are SGPR popcounts.  Waves
// are independent (no LDS, no barriers): wave 4 b + w of the grid takes task (4 b + w) % ntasks of row
// range (4 b + w) / ntasks; the host pads ntasks to a multiple of 4, so the 4 waves of a workgroup share
// one row range and the columns several tasks read come from L1 / L2, not HBM, a second time.
// Every (task, range) writes CorrPartial / ColPartial records that dq_finalize merges in range order.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

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

// bits of rows [base, base + 64) of a bitmap, clipped to rows below row1 (base < row1, base % 64 == 0; a
// dword holding no row below row1 is not read)
__device__ __forceinline__ uint64_t bits64_tail(const uint32_t* bm, int64_t base, int64_t row1) {
  const int64_t w = base >> 5;
  const bool two = base + 32 < row1;
  uint64_t x = ((uint64_t)(two ? ((const_u32s)bm)[w + 1] : 0u) << 32) | ((const_u32s)bm)[w];
  if (base + 64 > row1) x &= (1ull << (row1 - base)) - 1ull;
  return x;
}

// value of row `idx` of a column (values pointer at row 0 of the chunk), as double; raw = the int64 value
struct PosLoad {
  double x;
  int64_t raw;
};
template <bool F64>
__device__ __forceinline__ PosLoad load_row(const char* col, int kind, int64_t idx) {
  PosLoad p;
  if (F64 || kind == CK_F64) {
    p.raw = reinterpret_cast<const int64_t*>(col)[idx];
    p.x = __builtin_bit_cast(double, p.raw);
  } else if (kind == CK_I64) {
    p.raw = reinterpret_cast<const int64_t*>(col)[idx];
    p.x = __builtin_fma((double)(int32_t)(p.raw >> 32), 4294967296.0, (double)(uint32_t)p.raw);  // exact int64 -> double
  } else {
    p.raw = reinterpret_cast<const int32_t*>(col)[idx];
    p.x = (double)p.raw;
  }
  return p;
}

// One pair slot's update for a 64-row group, skipped as a whole when the slot is not one of the task's
// pairs: the slot test, the SGPR pair count (popcount of the two selection masks) and the five FMAs of the
// multiplicative form sit in ONE asm block with a scalar branch around them (LLVM otherwise rebuilds each
// uniform slot test as lane-mask VALU / SALU sequences and spills SGPRs to hold them).
template <int Q>
__device__ __forceinline__ void slot_update(double (&a)[5], uint32_t& cnt, uint32_t pm, double za, double zb, double fa,
                                            double fb, double qa, double qb, uint64_t ma, uint64_t mb) {
  const uint64_t both = ma & mb;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)both), hi = __builtin_amdgcn_readfirstlane((uint32_t)(both >> 32));
  uint32_t t0, t1;
  asm volatile(
      "s_bitcmp0_b32 %[pm], %[q]\n\t"
      "s_cbranch_scc1 .Lslot_skip%=\n\t"
      "s_bcnt1_i32_b32 %[t0], %[lo]\n\t"
      "s_bcnt1_i32_b32 %[t1], %[hi]\n\t"
      "s_add_u32 %[cnt], %[cnt], %[t0]\n\t"
      "s_add_u32 %[cnt], %[cnt], %[t1]\n\t"
      "v_fma_f64 %[sx], %[za], %[fb], %[sx]\n\t"
      "v_fma_f64 %[sy], %[zb], %[fa], %[sy]\n\t"
      "v_fma_f64 %[sxy], %[za], %[zb], %[sxy]\n\t"
      "v_fma_f64 %[sxx], %[qa], %[fb], %[sxx]\n\t"
      "v_fma_f64 %[syy], %[qb], %[fa], %[syy]\n\t"
      ".Lslot_skip%=:"
      : [sx] "+v"(a[0]), [sy] "+v"(a[1]), [sxy] "+v"(a[2]), [sxx] "+v"(a[3]), [syy] "+v"(a[4]), [cnt] "+s"(cnt),
        [t0] "=&s"(t0), [t1] "=&s"(t1)
      : [pm] "s"(pm), [q] "i"(Q), [za] "v"(za), [zb] "v"(zb), [fa] "v"(fa), [fb] "v"(fb), [qa] "v"(qa), [qb] "v"(qb),
        [lo] "s"(lo), [hi] "s"(hi)
      : "scc");
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

constexpr int kLaneGroups = 1;  // row groups of 64 rows loaded together per iteration (VGPR budget)

}  // namespace

// F64: every position of every task is an fp64 column (no conversions, no integral sums)
template <bool F64>
__global__ __launch_bounds__(kBlock) void dq_pair_lane_scan(const PairWaveTask* __restrict__ tasks, int32_t ntasks,
                                                            ScanCols cols, ScanBitmaps bm, const uint32_t* ones,
                                                            int64_t n_rows, int64_t rows_per_range, int32_t nranges,
                                                            CorrPartial* __restrict__ pair_part,
                                                            ColPartial* __restrict__ col_part) {
  const int lane = threadIdx.x & 63;
  const int wid = (int)blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ti = wid % ntasks, range = wid / ntasks;
  const PairWaveTask& t = tasks[ti];
  const int nc = t.ncols;
  if (range >= nranges || nc == 0) return;  // wave-uniform: padding waves / tasks
  const int64_t row0 = (int64_t)range * rows_per_range;
  const int64_t row1 = row0 + rows_per_range < n_rows ? row0 + rows_per_range : n_rows;
  // a missing validity / where bitmap reads the all-ones bitmap (no per-row pointer tests)
  const uint32_t* where = t.where >= 0 ? reinterpret_cast<const uint32_t*>(bm.where_bits[t.where]) : ones;
  const uint32_t* where_v = where;
  asm volatile("" : "+v"(where_v));
  const uint32_t pmask = t.pair_mask, mmask = t.mom_mask;

  // positions >= ncols repeat a real column (host padding): no per-position conditionals in the loop
  const char* colp[kLaneCols];
  const uint32_t* valid[kLaneCols];
  int kind[kLaneCols];
  double shift[kLaneCols];
#pragma unroll
  for (int c = 0; c < kLaneCols; ++c) {
    kind[c] = F64 ? CK_F64 : t.kinds[c];
    const int col = t.cols[c];
    colp[c] = reinterpret_cast<const char*>(cols.values[col]);
    valid[c] = cols.validity[col] ? cols.validity[col] : ones;
    // the stream pointers live in VGPRs (uniform values; the SGPR file holds the masks and counters)
    asm volatile("" : "+v"(colp[c]), "+v"(valid[c]));
    // shift: mean of the first 64-row group holding finite selected values (0 if none in the range)
    double s = 0.0;
    if (c < nc) {
      for (int64_t g = row0; g < row1; g += 64) {
        const int64_t r = g + lane < row1 ? g + lane : row1 - 1;
        const double x = load_row<F64>(colp[c], kind[c], r).x;
        const uint64_t fm = __builtin_amdgcn_ballot_w64(__builtin_isfinite(x)) & bits64_tail(valid[c], g, row1) &
                            bits64_tail(where, g, row1);
        if (fm != 0) {
          s = wave_sum(lane_bit(fm) ? x : 0.0) / (double)__builtin_popcountll(fm);
          break;
        }
      }
    }
    shift[c] = s;
  }

  double acc[kLaneSlots][5];
  uint32_t pcnt[kLaneSlots];  // pair counts: SGPR popcounts of the two selection masks
  uint32_t poison = 0;         // slots with a selected NaN / +-inf in a row of both columns
#pragma unroll
  for (int q = 0; q < kLaneSlots; ++q) {
    pcnt[q] = 0;
#pragma unroll
    for (int k = 0; k < 5; ++k) acc[q][k] = 0.0;
  }
  double sd[kLaneMoments], sdd[kLaneMoments], lo[kLaneMoments], hi[kLaneMoments];
  int64_t is[kLaneMoments], nanv[kLaneMoments], pinfv[kLaneMoments], ninfv[kLaneMoments];
  uint32_t mcnt[kLaneMoments];
#pragma unroll
  for (int p = 0; p < kLaneMoments; ++p) {
    sd[p] = sdd[p] = 0.0;
    lo[p] = __builtin_bit_cast(double, 0x7FF0000000000000ull);
    hi[p] = __builtin_bit_cast(double, 0xFFF0000000000000ull);
    is[p] = nanv[p] = pinfv[p] = ninfv[p] = 0;
    mcnt[p] = 0;
  }

  // one block of kLaneGroups 64-row groups; TAIL: the block reaches past row1 (clamped loads, clipped masks)
  // One block's loads.  Full blocks also bring the validity / where words through the VECTOR memory path
  // (an address the compiler cannot prove uniform): scalar loads of a streamed bitmap miss to HBM every
  // 16 groups and each miss parks the wave, while vector loads ride the software pipeline with the values.
  struct BlockData {
    PosLoad v[kLaneGroups][kLaneCols];
    uint32_t mw[kLaneGroups][kLaneCols + 1][2];  // validity words of the positions, then the where word
  };
  int zero_v;
  asm volatile("v_mov_b32 %0, 0" : "=v"(zero_v));
  auto load_block = [&](int64_t blk, BlockData& b, auto tail_tag) {
    constexpr bool TAIL = decltype(tail_tag)::value;
#pragma unroll
    for (int j = 0; j < kLaneGroups; ++j) {
#pragma unroll
      for (int c = 0; c < kLaneCols; ++c) {
        int64_t r = blk + 64 * j + lane;
        if (TAIL) r = r < row1 ? r : row1 - 1;
        b.v[j][c] = load_row<F64>(colp[c], kind[c], r);
      }
      if (!TAIL) {
        const int64_t w = ((blk + 64 * j) >> 5) + zero_v;
#pragma unroll
        for (int c = 0; c <= kLaneCols; ++c) {
          const uint32_t* bmp = c < kLaneCols ? valid[c] : where_v;
          b.mw[j][c][0] = bmp[w];
          b.mw[j][c][1] = bmp[w + 1];
        }
      }
    }
  };
  auto word = [](const uint32_t (&w)[2]) {
    return ((uint64_t)__builtin_amdgcn_readfirstlane(w[1]) << 32) | (uint32_t)__builtin_amdgcn_readfirstlane(w[0]);
  };
  auto block = [&](int64_t blk, const BlockData& b, auto tail_tag) {
    constexpr bool TAIL = decltype(tail_tag)::value;
    const auto& v = b.v;
#pragma unroll
    for (int j = 0; j < kLaneGroups; ++j) {
      const int64_t base = blk + 64 * j;
      if (TAIL && base >= row1) break;
      // re-materialise the task masks as opaque SGPR values each group: LLVM otherwise hoists the slot tests
      // as i1 lane masks and rebuilds every branch condition with v_cndmask + v_cmp (2 VALU per slot)
      uint32_t pm = pmask;
      asm volatile("" : "+s"(pm));
      const uint64_t wm = TAIL ? bits64_tail(where, base, row1) : word(b.mw[j][kLaneCols]);
      uint64_t m[kLaneCols];
      double d[kLaneCols];
#pragma unroll
      for (int c = 0; c < kLaneCols; ++c) {
        m[c] = (TAIL ? bits64_tail(valid[c], base, row1) : word(b.mw[j][c])) & wm;
        d[c] = v[j][c].x - shift[c];
      }
      // Multiplicative form, no EXEC switching: z = d on a selected finite row and 0 otherwise, f = 1 on a
      // selected row and 0 otherwise, q = z^2; a pair's sums over the rows selected in BOTH columns are then
      // plain FMAs -- Sx = sum z_a f_b, Sy = sum z_b f_a, Sxy = sum z_a z_b, Sxx = sum q_a f_b,
      // Syy = sum q_b f_a -- exact, every term being a product with 0 or 1 of finite values.  A selected
      // NaN / +-inf (rare) is kept out of the sums: a pair holding one in a row selected in both columns
      // is poisoned (its co-moments become NaN, as Spark's Corr update turns them), and the moments of a
      // column follow the column pass: NaN rows make avg / m2 / sum NaN, +-inf rows are counted and
      // excluded (dq_finish).
      uint64_t nf[kLaneCols], zm[kLaneCols], bad = 0;
#pragma unroll
      for (int c = 0; c < kLaneCols; ++c) {
        nf[c] = __builtin_amdgcn_ballot_w64(!__builtin_isfinite(d[c])) & m[c];
        bad |= nf[c];
        zm[c] = m[c];
      }
      uint64_t mb[kLaneMoments];
#pragma unroll
      for (int p = 0; p < kLaneMoments; ++p) {
        mb[p] = m[p];
        mcnt[p] += (uint32_t)__builtin_popcountll(m[p]);  // moments of positions 0, 1 run unconditionally
      }
      if (bad != 0) {  // rare
#pragma unroll
        for (int c = 0; c < kLaneCols; ++c) zm[c] = m[c] & ~nf[c];
#pragma unroll
        for (int q = 0; q < kLaneSlots; ++q) {
          const int a = kLaneSlotA[q], b2 = kLaneSlotB[q];
          if (((nf[a] | nf[b2]) & m[a] & m[b2]) != 0) poison |= 1u << q;
        }
#pragma unroll
        for (int p = 0; p < kLaneMoments; ++p) {
          if (nf[p] == 0) continue;
          const double x = v[j][p].x;
          const uint64_t nan = __builtin_amdgcn_ballot_w64(x != x) & m[p];
          const uint64_t inf = nf[p] & ~nan, pinf = __builtin_amdgcn_ballot_w64(x > 0.0) & inf;
          if (lane == 0) {
            nanv[p] += __builtin_popcountll(nan);
            pinfv[p] += __builtin_popcountll(pinf);
            ninfv[p] += __builtin_popcountll(inf & ~pinf);
          }
          mb[p] = m[p] & ~nan;
        }
      }
      double z[kLaneCols], f[kLaneCols], q2[kLaneCols];
#pragma unroll
      for (int c = 0; c < kLaneCols; ++c) {
        z[c] = lane_bit(zm[c]) ? d[c] : 0.0;
        f[c] = lane_bit(m[c]) ? 1.0 : 0.0;
        q2[c] = z[c] * z[c];
      }
#pragma unroll
      for (int p = 0; p < kLaneMoments; ++p) {
        const double x = v[j][p].x;
        sd[p] += z[p];
        sdd[p] += q2[p];
        lo[p] = hw_min(lo[p], lane_bit(mb[p]) ? x : __builtin_bit_cast(double, 0x7FF0000000000000ull));
        hi[p] = hw_max(hi[p], lane_bit(mb[p]) ? x : __builtin_bit_cast(double, 0xFFF0000000000000ull));
        if (!F64 && kind[p] != CK_F64) is[p] = (int64_t)((uint64_t)is[p] + (uint64_t)(lane_bit(m[p]) ? v[j][p].raw : 0));
      }
      SlotLoop<0, kLaneSlots>::run([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        constexpr int a = kLaneSlotA[q], b2 = kLaneSlotB[q];
        slot_update<q>(acc[q], pcnt[q], pm, z[a], z[b2], f[a], f[b2], q2[a], q2[b2], m[a], m[b2]);
      });
    }
  };
  // full blocks, software-pipelined: the next block's values are in flight while this one is folded
  constexpr int64_t kB = 64 * kLaneGroups;
  int64_t blk = row0;
  if (blk + kB <= row1) {
    BlockData nxt;
    load_block(blk, nxt, std::false_type{});
    for (; blk + kB <= row1; blk += kB) {
      const BlockData cur = nxt;
      if (blk + 2 * kB <= row1) load_block(blk + kB, nxt, std::false_type{});
      block(blk, cur, std::false_type{});
    }
  }
  if (blk < row1) {
    BlockData cur;
    load_block(blk, cur, std::true_type{});
    block(blk, cur, std::true_type{});
  }

  // ---- close: wave sums (fixed butterfly order), then the (n, means, co-moments) of this range
#pragma unroll
  for (int q = 0; q < kLaneSlots; ++q) {
    if (!((pmask >> q) & 1u)) continue;
    double S[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) S[k] = wave_sum(acc[q][k]);
    const int32_t cnt = (int32_t)pcnt[q];
    if (lane == 0) {
      CorrPartial* o = pair_part + (size_t)t.pair_out[q] * kMaxWG + range;
      const double n = (double)cnt;
      CorrPartial r{0, 0, 0, 0, 0, 0, 0, 0};
      if (cnt > 0 && ((poison >> q) & 1u)) {
        const double nan = __builtin_bit_cast(double, 0x7FF8000000000000ull);
        r = CorrPartial{n, nan, nan, nan, nan, nan, 0, 0};
      } else if (cnt > 0) {
        const double qx = S[0] / n, qy = S[1] / n;
        const double xa = shift[kLaneSlotA[q]] + qx, ya = shift[kLaneSlotB[q]] + qy;
        const double xm = S[3] - S[0] * qx, ym = S[4] - S[1] * qy;
        const bool sw = (t.swap_mask >> q) & 1u;  // Correlation(first, second) with first at position B
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
  for (int p = 0; p < kLaneMoments; ++p) {
    if (!((mmask >> p) & 1u)) continue;
    const double S1 = wave_sum(sd[p]), S2 = wave_sum(sdd[p]);
    const double fmin = wave_min(lo[p]), fmax = wave_max(hi[p]);
    const int64_t isum = wave_sum_i64(is[p]);
    const int64_t nan = __builtin_amdgcn_readfirstlane((int)nanv[p]) , pinf = __builtin_amdgcn_readfirstlane((int)pinfv[p]),
                  ninf = __builtin_amdgcn_readfirstlane((int)ninfv[p]);
    if (lane == 0) {
      const int64_t count = mcnt[p];
      const int64_t nm = count - pinf - ninf;
      ColPartial r;
      r.n = (double)nm;
      r.mean = 0.0;
      r.m2 = 0.0;
      r.sum = 0.0;
      if (nm > 0) {
        const double q1 = S1 / (double)nm;
        r.mean = shift[p] + q1;
        r.m2 = S2 - S1 * q1;
        r.sum = __builtin_fma((double)nm, shift[p], S1);
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
      col_part[(size_t)t.mom_out[p] * kMaxWG + range] = r;
    }
  }
}

hipError_t launch_pair_lane_scan(const PairWaveTask* tasks, int32_t ntasks, const ScanCols& cols,
                                 const ScanBitmaps& bm, const uint32_t* ones, int64_t n_rows, int64_t rows_per_range, int32_t nranges,
                                 CorrPartial* pair_part, ColPartial* col_part, bool all_f64, hipStream_t st) {
  const int64_t waves = (int64_t)ntasks * nranges;
  const uint32_t blocks = (uint32_t)((waves + kWaves - 1) / kWaves);
  if (all_f64)
    hipLaunchKernelGGL(dq_pair_lane_scan<true>, dim3(blocks), dim3(kBlock), 0, st, tasks, ntasks, cols, bm, ones, n_rows,
                       rows_per_range, nranges, pair_part, col_part);
  else
    hipLaunchKernelGGL(dq_pair_lane_scan<false>, dim3(blocks), dim3(kBlock), 0, st, tasks, ntasks, cols, bm, ones, n_rows,
                       rows_per_range, nranges, pair_part, col_part);
  return hipGetLastError();
}



// ================================================================================================
// Gram-matrix form on the matrix cores (v_mfma_f64_16x16x4_f64).
//
// For the <= 8 columns of a pair group and a row k, let z_c = d_c (= x_c - shift_c) if the row is selected
// in column c (valid, `where`, finite) and 0 otherwise, f_c = 1 if selected (incl. non-finite) else 0,
// q_c = z_c^2.  With A = [z_0..z_7 | q_0..q_7] and B = [f_0..f_7 | z_0..z_7] (16 features per row),
// C = sum_k A_k^T B_k is a 16 x 16 tile holding, for EVERY pair (a, b):
//   Sx = C[a][b] = sum z_a f_b   Sy = C[b][a]   Sxy = C[a][8 + b]   Sxx = C[8 + a][b]   Syy = C[8 + b][a]
// -- the co-moment sums over the rows selected in both columns (products with 0 / 1 are exact) -- and,
// on its diagonal, each column's own moments: S = C[c][c], Q = C[8 + c][c].  One MFMA folds 4 rows of all
// 28 pairs and 8 columns.  Lane l supplies feature (l & 15) of row (l >> 4) of each 4-row step: it loads
// its own element straight from HBM (column l & 7), so no LDS staging; pair counts are SGPR popcounts of
// the selection masks.  The 4 waves of a workgroup fold interleaved 64-row groups of its row range with
// the same shifts, then add their tiles in wave order (LDS) into one partial per range.
//
// Cost model (measured, tools/micro/mfma_*_probe.hip): one v_mfma_f64_16x16x4_f64 issues every 64 cycles per
// SIMD (74 TF/s chip-wide) and does NOT co-execute with any VALU instruction (f64 FMA or 32-bit): the f64
// matrix op runs on the SIMD's vector datapath.  A 64-row group therefore costs 16 x 64 MFMA cycles plus
// its ~14 VALU per step, with no overlap -- about 1.7k cycles per SIMD; it still beats the lane-per-row
// VALU kernel above (per-task column duplication, SALU slot control) and the LDS tile + column pass pair.
// ================================================================================================
typedef double dq_d4 __attribute__((ext_vector_type(4)));
#ifndef DQ_PAIR_SLOTS
#define DQ_PAIR_SLOTS 2
#endif
// waves per SIMD the LDS-DMA kernel's registers must allow: 2 slots (35 KB per workgroup) let 4
// workgroups share a CU, and 4 waves (128 VGPRs, 8 spilled) measured 1.80 -> 1.76 ms per 125 M rows
// against 3 slots at 3 waves (52 KB, 136 VGPRs)
#ifndef DQ_PAIR_WAVES
#define DQ_PAIR_WAVES 4
#endif
constexpr int kStageSlots = DQ_PAIR_SLOTS;  // LDS-DMA group slots per wave (kStageSlots - 1 groups in flight beside the fold)

// F64: every column of every group is fp64; MINMAX: a fused moments task feeds Minimum / Maximum
// GLDS (with F64): full groups staged through LDS by DMA (every column 16-byte aligned: the host checks)
template <bool F64, bool MINMAX, bool GLDS = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(GLDS ? DQ_PAIR_WAVES : 1))) void dq_pair_mfma_scan(const PairGroup* __restrict__ groups, int32_t ngroups,
                                                            ScanCols cols, ScanBitmaps bm, const uint32_t* ones,
                                                            int64_t n_rows, int64_t rows_per_range, int32_t nranges,
                                                            CorrPartial* __restrict__ pair_part,
                                                            ColPartial* __restrict__ col_part) {
  __shared__ double shift_s[kTileCols];
  // the workgroup merge's arrays share LDS with the DMA stage slots (GLDS: used only after every wave has
  // left its group loop -- a barrier separates them)
  struct MergeLds {
    double tile[kWaves][16][17];  // the waves' C tiles (+1: bank spread)
    uint32_t cnt_s[kWaves][kTileCols][kTileCols];
    int64_t nan_s[kWaves][kTileCols], pinf_s[kWaves][kTileCols], ninf_s[kWaves][kTileCols];
    int64_t isum_s[kWaves][kTileCols];
    double lo_s[kWaves][kTileCols], hi_s[kWaves][kTileCols];
    uint64_t poison_s[kWaves];
  };
  struct StageLds {
    double x[kWaves][kStageSlots][kTileCols * 64];  // [column][row] of a 64-row group
    uint32_t w[kWaves][kStageSlots][64];             // selection words (lanes 0..17 of the DMA)
  };
  constexpr size_t kSmem = GLDS && sizeof(StageLds) > sizeof(MergeLds) ? sizeof(StageLds) : sizeof(MergeLds);
  __shared__ __attribute__((aligned(16))) char smem[kSmem];
  MergeLds& ml = *reinterpret_cast<MergeLds*>(smem);
  StageLds& sl = *reinterpret_cast<StageLds*>(smem);
  auto& tile = ml.tile;
  auto& cnt_s = ml.cnt_s;
  auto& nan_s = ml.nan_s;
  auto& pinf_s = ml.pinf_s;
  auto& ninf_s = ml.ninf_s;
  auto& isum_s = ml.isum_s;
  auto& lo_s = ml.lo_s;
  auto& hi_s = ml.hi_s;
  auto& poison_s = ml.poison_s;
  auto& stage_x = sl.x;
  auto& stage_w = sl.w;
  const int gi = blockIdx.x % ngroups, range = blockIdx.x / ngroups;
  const PairGroup& g = groups[gi];
  const int nc = g.ncols;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t row0 = (int64_t)range * rows_per_range;
  const int64_t row1 = row0 + rows_per_range < n_rows ? row0 + rows_per_range : n_rows;
  const uint32_t* where = g.where >= 0 ? reinterpret_cast<const uint32_t*>(bm.where_bits[g.where]) : ones;

  // ---- shifts (workgroup-uniform): wave 0 computes the mean of each column's first finite selected group
  if (wave == 0) {
    for (int c = 0; c < nc; ++c) {
      const int col = g.cols[c];
      const uint32_t* vb = cols.validity[col] ? cols.validity[col] : ones;
      double s = 0.0;
      for (int64_t gr = row0; gr < row1; gr += 64) {
        const int64_t r = gr + lane < row1 ? gr + lane : row1 - 1;
        const int k = F64 ? CK_F64 : g.kinds[c];
        const double x = load_row<F64>(reinterpret_cast<const char*>(cols.values[col]), k, r).x;
        const uint64_t fm = __builtin_amdgcn_ballot_w64(__builtin_isfinite(x)) & bits64_tail(vb, gr, row1) &
                            bits64_tail(where, gr, row1);
        if (fm != 0) {
          s = wave_sum(lane_bit(fm) ? x : 0.0) / (double)__builtin_popcountll(fm);
          break;
        }
      }
      if (lane == 0) shift_s[c] = s;
    }
  }
  __syncthreads();

  // ---- this lane's feature: column c = lane & 7 (lanes of columns >= ncols stay zero), A/B half hi,
  // row slot rs.  Step j (0..15) of the 64-row group at `base` folds row base + 8 (j >> 1) + 2 rs + (j & 1):
  // a lane's two rows of steps 2 t, 2 t + 1 are adjacent, so one 16-byte load brings both (fp64).
  const int feat = lane & 15, c = feat & 7, rs = lane >> 4;
  const bool hi = (feat >> 3) != 0;
  const bool live = c < nc;
  const int colc = live ? g.cols[c] : g.cols[0];
  const int kind = F64 ? CK_F64 : g.kinds[live ? c : 0];
  const char* colp = reinterpret_cast<const char*>(cols.values[colc]);
  const double sh = live ? shift_s[c] : 0.0;
  // 16-byte loads need 16-byte aligned columns (a table sliced at an odd row is not): wave-uniform choice
  const bool vec16 = F64 && __builtin_amdgcn_ballot_w64((reinterpret_cast<uintptr_t>(colp) & 15u) != 0) == 0;
  // selection words come through the vector path: lane l reads the validity word of column a = l & 7 (its
  // own feature column) and of column b = (l >> 3) & 7, so lane l also owns the count and the poison flag
  // of the ordered column pair (a, b) -- no SGPR arrays, no scalar loads of streamed bitmaps
  const int pb = (lane >> 3) & 7;
  const bool live_b = pb < nc;
  const uint32_t* va;
  const uint32_t* vb;
  {
    const int ca = g.cols[live ? c : 0], cb = g.cols[live_b ? pb : 0];
    va = cols.validity[ca] ? cols.validity[ca] : ones;
    vb = cols.validity[cb] ? cols.validity[cb] : ones;
  }
  // the `where` words come through the vector path too (a VGPR copy of the uniform pointer; global
  // address space, so the loads stay out of the scalar / LDS counters and the prefetch is not waited for)
  typedef const __attribute__((address_space(1))) uint32_t* gu32;
  gu32 where_v = (gu32)where;
  asm volatile("" : "+v"(where_v));

  // two tiles, even / odd steps: consecutive MFMAs do not wait for each other's accumulator
  dq_d4 acc = {0.0, 0.0, 0.0, 0.0}, accb = {0.0, 0.0, 0.0, 0.0};
  // w = hi ? d : 1 as one FMA: d * hd + omh (exact for finite d)
  const double hd = hi ? 1.0 : 0.0, omh = hi ? 0.0 : 1.0;
  uint32_t cnt = 0;           // rows selected in both a and b (lane (a, b)); a == b: the column count
  bool poison = false;        // pair (a, b) met a selected NaN / +-inf of column a in a row selected in b
  int64_t nanv = 0, pinfv = 0, ninfv = 0, isum = 0;  // column c's rows of slot rs (lanes with hi == 0)
  double lo = __builtin_bit_cast(double, 0x7FF0000000000000ull), hiv = __builtin_bit_cast(double, 0xFFF0000000000000ull);
  const double qnan = __builtin_bit_cast(double, 0x7FF8000000000000ull);

  typedef double d2 __attribute__((ext_vector_type(2)));
  struct Grp {
    double x[16];
    int64_t raw[F64 ? 1 : 16];
    uint32_t wa[2], wb[2], wm[2];
  };
  // one 64-row group's values and selection words; TAIL: rows at or past row1 are clamped (masked later)
  // VEC: the 16-byte loads of a full group of aligned fp64 columns; TAIL: rows at or past row1 are clamped
  auto load = [&](int64_t base, Grp& gr, auto vec_tag, auto tail_tag) __attribute__((always_inline)) {
    constexpr bool VEC = decltype(vec_tag)::value, TAIL = decltype(tail_tag)::value;
    const int64_t w = base >> 5;
    const bool two = !TAIL || base + 32 < row1;  // the second dword holds a row below row1
    gr.wa[0] = va[w];
    gr.wb[0] = vb[w];
    gr.wm[0] = where_v[w];
    gr.wa[1] = two ? va[w + 1] : 0u;
    gr.wb[1] = two ? vb[w + 1] : 0u;
    gr.wm[1] = two ? where_v[w + 1] : 0u;
    if (VEC && !TAIL) {
      const d2* p = reinterpret_cast<const d2*>(colp) + ((base >> 1) + rs);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const d2 v = p[4 * t];
        gr.x[2 * t] = v.x;
        gr.x[2 * t + 1] = v.y;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        int64_t r = base + 8 * (j >> 1) + 2 * rs + (j & 1);
        if (TAIL) r = r < row1 ? r : row1 - 1;
        const PosLoad pl = load_row<F64>(colp, kind, r);
        gr.x[j] = pl.x;
        if (!F64) gr.raw[j] = pl.raw;
      }
    }
  };
  // Fold one group.  Fast path: z = x - shift on a selected row (no finiteness tests).  A selected NaN / +-inf
  // reaches at least the tile's diagonal term z_a f_a of its column, so a tile that is finite after the
  // group proves there was none; otherwise (rare) the group is folded again from the saved tile with the
  // non-finite values kept out, counted, and their pairs poisoned.  Min / max / integral sums are taken
  // once, in the fast path (min / max see the same values either way; NaN is skipped by v_min / v_max).
  // wa_raw / wb_raw / wm_raw: the 64-row selection words (column a, column b, `where`); xpair(t): this
  // lane's values of steps 2 t and 2 t + 1; rawv(j): the integral value of step j (!F64)
  auto fold = [&](int64_t base, uint64_t wa_raw, uint64_t wb_raw, uint64_t wm_raw, auto xpair, auto rawv,
                  auto tail_tag) __attribute__((always_inline)) {
    constexpr bool TAIL = decltype(tail_tag)::value;
    uint64_t wm = wm_raw;
    if (TAIL && base + 64 > row1) wm &= (1ull << (row1 - base)) - 1ull;
    const uint64_t wa = live ? wa_raw & wm : 0ull;
    const uint64_t wb = live_b ? wb_raw & wm : 0ull;
    cnt += (uint32_t)__builtin_popcountll(wa & wb);
    const uint64_t wr = wa >> (2 * rs);  // step j's bit: 8 (j >> 1) + (j & 1)
    const uint32_t wlo = (uint32_t)wr, whi = (uint32_t)(wr >> 32);
    const dq_d4 acc0 = acc, accb0 = accb;
    // Operands are prepared kPrepBatch steps at a time and their MFMAs issued after them as one batch: a
    // step's VALU chain (bfe -> cvt -> mul -> mul) interleaved 1:1 with the MFMAs leaves every f64 result's
    // latency exposed (the other wave's MFMA cannot cover it: no co-issue), batched the chains overlap.
#ifndef DQ_PAIR_BATCH
#define DQ_PAIR_BATCH 4
#endif
    constexpr int kPrepBatch = DQ_PAIR_BATCH;
#pragma unroll
    for (int j0 = 0; j0 < 16; j0 += kPrepBatch) {
      double av[kPrepBatch], bv[kPrepBatch], xb[kPrepBatch];
#pragma unroll
      for (int t = 0; t < kPrepBatch / 2; ++t) {
        const d2 v = xpair(j0 / 2 + t);
        xb[2 * t] = v.x;
        xb[2 * t + 1] = v.y;
      }
#pragma unroll
      for (int jj = 0; jj < kPrepBatch; ++jj) {
        const int j = j0 + jj;
        const int bit = 8 * (j >> 1) + (j & 1);
        // multiplicative operands, 7 VALU per step: f = selection as 0.0 / 1.0, z = d f, w = (hi ? d : 1),
        // A = z w (lo: z, hi: z^2), B = w f (lo: f, hi: z) -- exact (products with 0 / 1).  A non-finite d
        // (selected, or garbage in an unselected slot: inf * 0) makes the tile non-finite -> refold below.
        const uint32_t sb = ((bit < 32 ? wlo : whi) >> (bit & 31)) & 1u;
        // (f built from the bit with integer ops instead of v_cvt_f64_u32: 2.09 vs 2.04 ms per 125 M rows)
        const double f = (double)sb;
        const double x = xb[jj];
        const double d = x - sh;
        const double z = d * f;
        const double w = __builtin_fma(d, hd, omh);
        av[jj] = z * w;
        bv[jj] = w * f;
        const bool sel = sb != 0u;
        if (!F64 && kind != CK_F64) isum = (int64_t)((uint64_t)isum + (uint64_t)(sel ? rawv(j) : 0));
        if (MINMAX) {
          const double xm = sel ? x : qnan;  // v_min / v_max (IEEE mode) skip a NaN operand: unselected, NaN rows
          lo = hw_min(lo, xm);
          hiv = hw_max(hiv, xm);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int jj = 0; jj < kPrepBatch; ++jj) {
        if (jj & 1) accb = __builtin_amdgcn_mfma_f64_16x16x4f64(av[jj], bv[jj], accb, 0, 0, 0);
        else acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[jj], bv[jj], acc, 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    const bool tile_fin = __builtin_isfinite(acc[0]) && __builtin_isfinite(acc[1]) && __builtin_isfinite(acc[2]) &&
                          __builtin_isfinite(acc[3]) && __builtin_isfinite(accb[0]) && __builtin_isfinite(accb[1]) &&
                          __builtin_isfinite(accb[2]) && __builtin_isfinite(accb[3]);
    if (__builtin_amdgcn_ballot_w64(!tile_fin) != 0) {  // rare (unrolled: no indexed register arrays)
      acc = acc0;
      accb = accb0;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int bit = 8 * (j >> 1) + (j & 1);
        const bool sel = ((bit < 32 ? wlo : whi) >> (bit & 31)) & 1u;
        const d2 xp = xpair(j >> 1);
        const double x = (j & 1) ? xp.y : xp.x;
        const bool fin = __builtin_isfinite(x);
        const double z = sel && fin ? x - sh : 0.0;
        const double av = hi ? z * z : z;
        const double bv = hi ? z : (sel ? 1.0 : 0.0);
        if (j & 1) accb = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, accb, 0, 0, 0);
        else acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
        const bool nf = sel && !fin;
        const uint64_t m = __builtin_amdgcn_ballot_w64(nf && !hi);  // lane a + 16 rs: column a, row slot rs
        if (m == 0) continue;
        const bool own = nf && !hi, isn = x != x;  // branch-free: keeps the counters in registers
        nanv += own && isn;
        pinfv += own && !isn && x > 0.0;
        ninfv += own && !isn && x < 0.0;
        const uint64_t t = m >> (lane & 7);  // column a's non-finite rows of slots 0..3
        const uint32_t ma = (uint32_t)((t & 1ull) | ((t >> 15) & 2ull) | ((t >> 30) & 4ull) | ((t >> 45) & 8ull));
        const uint64_t bs = wb >> bit;  // column b's selection of the same rows (slot k: bit 2 k)
        const uint32_t mb = (uint32_t)((bs & 1ull) | ((bs >> 1) & 2ull) | ((bs >> 2) & 4ull) | ((bs >> 3) & 8ull));
        if (ma & mb) poison = true;
      }
    }
  };

  auto fold_regs = [&](int64_t base, const Grp& gr, auto tail_tag) __attribute__((always_inline)) {
    fold(base, ((uint64_t)gr.wa[1] << 32) | gr.wa[0], ((uint64_t)gr.wb[1] << 32) | gr.wb[0],
         ((uint64_t)gr.wm[1] << 32) | gr.wm[0], [&](int t) { return d2{gr.x[2 * t], gr.x[2 * t + 1]}; },
         [&](int j) { return gr.raw[F64 ? 0 : j]; }, tail_tag);
  };

  // full groups, software-pipelined over two buffers: the next group's loads fly while this one folds.  The
  // prefetch is unconditional (the last one re-reads the current group) so every path into a fold has the
  // same loads in flight and the wait before it stays a partial vmcnt, not a drain.
  const int64_t full_end = row0 + ((row1 - row0) >> 6 << 6);
  constexpr int64_t kStride = 64 * kWaves;
  int64_t base = row0 + 64 * (int64_t)wave;
  auto run_full = [&](auto vec_tag) __attribute__((always_inline)) {
    Grp b0, b1;
    if (base >= full_end) return;
    load(base, b0, vec_tag, std::false_type{});
    // sched_barrier: the scheduler would otherwise sink the prefetch behind most of the fold's MFMAs,
    // leaving only the last steps to cover its latency
    while (true) {
      load(base + kStride < full_end ? base + kStride : base, b1, vec_tag, std::false_type{});
      __builtin_amdgcn_sched_barrier(0);
      fold_regs(base, b0, std::false_type{});
      base += kStride;
      if (base >= full_end) break;
      load(base + kStride < full_end ? base + kStride : base, b0, vec_tag, std::false_type{});
      __builtin_amdgcn_sched_barrier(0);
      fold_regs(base, b1, std::false_type{});
      base += kStride;
      if (base >= full_end) break;
    }
  };
  // LDS-DMA staged full groups (aligned fp64 columns): a group's 8 columns x 64 rows go HBM -> LDS with
  // 4 global_load_lds_dwordx4 (lane l: column 2 k + (l >> 5), rows 2 (l & 31), +1 -> LDS [column][row],
  // lane-linear) and its selection words with one global_load_lds_dword (lanes 0..15: 2 words of each
  // column's validity, 16..17: `where`).  No VGPRs hold a group in flight, so the wave keeps kStageSlots - 1
  // groups in flight beside the fold at the occupancy of the fold alone.  Only this wave reads its slots.
  // The DMAs are asm (hipcc does not count them): the waits are explicit vmcnt, with no other vector
  // memory instruction in the loop.
  auto run_glds = [&]() __attribute__((always_inline)) {
    if (base >= full_end) return;
    const char* srcx[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int cc = 2 * k + (lane >> 5);
      srcx[k] = reinterpret_cast<const char*>(cols.values[g.cols[cc < nc ? cc : 0]]) + (size_t)(2 * (lane & 31)) * 8;
    }
    const uint32_t* srcw;
    {
      const int cc = lane < 16 ? lane >> 1 : 0;
      const uint32_t* vv = cols.validity[g.cols[cc < nc ? cc : 0]];
      srcw = lane < 16 ? (vv ? vv : ones) + (lane & 1) : (lane < 18 ? where + (lane - 16) : ones);
    }
    auto stage = [&](int64_t gb, int slot) __attribute__((always_inline)) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const char* src = srcx[k] + gb * 8;
        const uint32_t dst = (uint32_t)(uintptr_t)&stage_x[wave][slot][k * 128];
        uint32_t keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
      }
      const uint32_t* srcb = srcw + (gb >> 5);
      const uint32_t dstb = (uint32_t)(uintptr_t)&stage_w[wave][slot][0];
      uint32_t keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(srcb), "s"(dstb) : "memory");
    };
    constexpr int D = kStageSlots - 1;  // groups in flight beside the fold
    auto wait_dma = [](int groups_after) __attribute__((always_inline)) {  // 5 DMAs per group
      if (groups_after >= 2) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
      else if (groups_after == 1) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    static_assert(D >= 1 && D <= 2, "wait_dma covers up to 2 groups in flight");
    int slot = 0;
#pragma unroll
    for (int d = 0; d < D; ++d)
      if (d == 0 || base + d * kStride < full_end) stage(base + d * kStride, d);
    while (true) {
      const int64_t ahead = base + D * kStride;
      if (ahead < full_end) stage(ahead, slot + D < kStageSlots ? slot + D : slot + D - kStageSlots);
      const int64_t left = (full_end - base - 1) / kStride;  // this wave's groups after the current one
      wait_dma(left < D ? (int)left : D);
      const uint64_t* wl = reinterpret_cast<const uint64_t*>(&stage_w[wave][slot][0]);
      const d2* xs = reinterpret_cast<const d2*>(&stage_x[wave][slot][c * 64 + 2 * rs]);
      fold(base, wl[c], wl[pb], wl[8], [&](int t) { return xs[4 * t]; }, [&](int) { return (int64_t)0; },
           std::false_type{});
      base += kStride;
      slot = slot + 1 < kStageSlots ? slot + 1 : 0;
      if (base >= full_end) break;
    }
  };
  if constexpr (GLDS && F64) run_glds();
  else if (vec16) run_full(std::true_type{});
  else run_full(std::false_type{});
  if (base < row1) {
    Grp bt;
    load(base, bt, std::false_type{}, std::true_type{});
    fold_regs(base, bt, std::true_type{});
  }

  // ---- workgroup merge (fixed order: waves 0..3) and the per-range partials
  if constexpr (GLDS) __syncthreads();  // every wave is done with the stage slots the merge arrays overlay
#pragma unroll
  for (int r = 0; r < 4; ++r) tile[wave][(lane >> 4) + 4 * r][lane & 15] = acc[r] + accb[r];
  cnt_s[wave][lane >> 3][lane & 7] = cnt;  // [b][a]
  {
    const uint64_t pz = __builtin_amdgcn_ballot_w64(poison);
    if (lane == 0) poison_s[wave] = pz;
  }
  // per-column lane values: lanes with hi == 0 of column c (4 row offsets) -> reduce within the wave
  {
    int64_t nv = nanv, pv = pinfv, mv = ninfv, iv = isum;
    double l2 = lo, h2 = hiv;
    // lanes c, c + 16, c + 32, c + 48 hold column c's hi == 0 partials
    for (int off = 16; off <= 32; off <<= 1) {
      nv += __shfl_xor(nv, off);
      pv += __shfl_xor(pv, off);
      mv += __shfl_xor(mv, off);
      iv = (int64_t)((uint64_t)iv + (uint64_t)__shfl_xor(iv, off));
      l2 = hw_min(l2, __shfl_xor(l2, off));
      h2 = hw_max(h2, __shfl_xor(h2, off));
    }
    if (lane < kTileCols) {
      nan_s[wave][lane] = nv;
      pinf_s[wave][lane] = pv;
      ninf_s[wave][lane] = mv;
      isum_s[wave][lane] = iv;
      lo_s[wave][lane] = l2;
      hi_s[wave][lane] = h2;
    }
  }
  __syncthreads();
  const int t = threadIdx.x;
  if (t < g.npairs) {
    const int a = g.pi[t], b = g.pj[t];
    double Sx = 0, Sy = 0, Sxy = 0, Sxx = 0, Syy = 0;
    int64_t n = 0;
    uint64_t pz = 0;
    for (int wv = 0; wv < kWaves; ++wv) {
      Sx += tile[wv][a][b];
      Sy += tile[wv][b][a];
      Sxy += tile[wv][a][8 + b];
      Sxx += tile[wv][8 + a][b];
      Syy += tile[wv][8 + b][a];
      n += cnt_s[wv][b][a];
      pz |= poison_s[wv];
    }
    CorrPartial r{0, 0, 0, 0, 0, 0, 0, 0};
    if (n > 0) {
      const double nd = (double)n;
      if (((pz >> (a + 8 * b)) | (pz >> (b + 8 * a))) & 1ull) {
        const double nan = __builtin_bit_cast(double, 0x7FF8000000000000ull);
        r = CorrPartial{nd, nan, nan, nan, nan, nan, 0, 0};
      } else {
        const double qx = Sx / nd, qy = Sy / nd;
        r.n = nd;
        r.xa = shift_s[a] + qx;
        r.ya = shift_s[b] + qy;
        r.ck = Sxy - Sx * qy;
        r.xm = Sxx - Sx * qx;
        r.ym = Syy - Sy * qy;
      }
    }
    pair_part[(size_t)(g.first_pair + t) * kMaxWG + range] = r;
  } else if (t >= 64 && t < 64 + nc && g.mom_task[t - 64] >= 0) {
    const int cc = t - 64;
    double S = 0, Q = 0, fmin = __builtin_bit_cast(double, 0x7FF0000000000000ull),
           fmax = __builtin_bit_cast(double, 0xFFF0000000000000ull);
    int64_t count = 0, nan = 0, pinf = 0, ninf = 0, is = 0;
    for (int wv = 0; wv < kWaves; ++wv) {
      S += tile[wv][cc][cc];
      Q += tile[wv][8 + cc][cc];
      count += cnt_s[wv][cc][cc];
      nan += nan_s[wv][cc];
      pinf += pinf_s[wv][cc];
      ninf += ninf_s[wv][cc];
      is = (int64_t)((uint64_t)is + (uint64_t)isum_s[wv][cc]);
      fmin = hw_min(fmin, lo_s[wv][cc]);
      fmax = hw_max(fmax, hi_s[wv][cc]);
    }
    ColPartial r;
    const int64_t nm = count - pinf - ninf;
    r.n = (double)nm;
    r.mean = r.m2 = r.sum = 0.0;
    if (nm > 0) {
      const double q1 = S / (double)nm;
      r.mean = shift_s[cc] + q1;
      r.m2 = Q - S * q1;
      r.sum = __builtin_fma((double)nm, shift_s[cc], S);
      if (nan > 0) r.mean = r.m2 = r.sum = __builtin_bit_cast(double, 0x7FF8000000000000ull);
    }
    r.isum = is;
    r.count = count;
    r.nan_count = nan;
    r.fmin = fmin;
    r.fmax = fmax;
    r.pinf_count = pinf;
    r.ninf_count = ninf;
    r.pad = 0;
    col_part[(size_t)g.mom_task[cc] * kMaxWG + range] = r;
  }
}

hipError_t launch_pair_mfma_scan(const PairGroup* groups, int32_t ngroups, const ScanCols& cols,
                                 const ScanBitmaps& bm, const uint32_t* ones, int64_t n_rows, int64_t rows_per_range,
                                 int32_t nranges, CorrPartial* pair_part, ColPartial* col_part, bool all_f64,
                                 bool minmax, bool glds, hipStream_t st) {
  const uint32_t blocks = (uint32_t)ngroups * (uint32_t)nranges;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(kBlock), 0, st, groups, ngroups, cols, bm, ones, n_rows, rows_per_range,
                       nranges, pair_part, col_part);
  };
  if (all_f64 && glds) {
    if (minmax) go(dq_pair_mfma_scan<true, true, true>);
    else go(dq_pair_mfma_scan<true, false, true>);
  } else if (all_f64) {
    if (minmax) go(dq_pair_mfma_scan<true, true>);
    else go(dq_pair_mfma_scan<true, false>);
  } else {
    if (minmax) go(dq_pair_mfma_scan<false, true>);
    else go(dq_pair_mfma_scan<false, false>);
  }
  return hipGetLastError();
}

}  // namespace dq
