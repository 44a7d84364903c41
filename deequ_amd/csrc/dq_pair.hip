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
// the same for a whole 64-row group below row1: one s_load_dwordx2
__device__ __forceinline__ uint64_t bits64(const uint32_t* bm, int64_t base) {
  return load_word64(bm, base >> 5);
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

}  // namespace dq
