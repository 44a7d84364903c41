// dq_prim.hip -- device-wide primitives of the grouping and quantile paths (dq_prim.h), hand-written for gfx950.
//
// Radix sort: stable LSD over 8-bit digits, three launches per digit (reduce, then scan, then scatter):
//   sort_hist      a fixed grid of <= 1024 workgroups (one resident round: 4 per CU), each over a contiguous segment
//                  of 2048-key tiles, counts its segment's digits in LDS (one 256-bin copy per wave, ds_add);
//   sort_scan_rows one workgroup per digit scans that digit's row of per-workgroup counts (its offsets);
//   sort_scatter   each workgroup walks its tiles in order (the next tile's keys loaded while this one is written):
//                  wave w of a tile holds its keys [512 w, 512 w + 512), 64 consecutive per load; a wave ranks its 8
//                  rows of 64 keys in turn -- the lanes holding equal digits are found by one ballot per digit bit
//                  (the peer mask), a lane's rank is the wave's running count of its digit (LDS) plus mbcnt of its
//                  peers, and the lowest peer advances that count; thread d turns the 4 waves' counts of digit d into
//                  offsets, the workgroup scans the 256 digit totals, and every key lands at its stable tile position
//                  in an LDS stage, from which consecutive threads write consecutive addresses of each digit's run
//                  (values follow through the same stage).
// The peer-mask ranking keeps the order stable without relying on the order in which LDS atomics of one wave
// instruction are applied.  Scans: reduce -> scan of the partials -> rescan with the carry, over <= 1024 contiguous
// segments.  Runs: head flags (key != previous key) scanned the same way.
#include "dq_prim.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace dq {
namespace prim {
namespace {

constexpr int kT = 256;                   // threads per workgroup (4 waves)
constexpr int kScanIpt = 4;               // items per thread and tile (scans, runs)
constexpr int kScanTile = kT * kScanIpt;  // 1024
constexpr int kMaxWg = 1024;              // workgroups of a scan / sort pass (= kT * kScanIpt partials)
#ifndef DQ_SORT_ITEMS
#define DQ_SORT_ITEMS 16
#endif
#ifndef DQ_SORT_THREADS
#define DQ_SORT_THREADS 512
#endif
#ifndef DQ_SORT_MAXWG
#define DQ_SORT_MAXWG 1024
#endif
constexpr int kST = DQ_SORT_THREADS;        // threads of a sort_scatter workgroup
constexpr int kSW = kST / 64;               // its waves
constexpr int kSortItems = DQ_SORT_ITEMS;  // keys per thread and tile
constexpr int kSortTile = kST * kSortItems;
constexpr int kSortMaxWg = DQ_SORT_MAXWG;   // <= kMaxWg (sort_scan_rows scans a row of <= 1024)
constexpr int kRadix = 256;

typedef uint32_t __attribute__((may_alias)) u32a;

struct Geom {
  int nwg;      // workgroups
  int64_t tpw;  // tiles per workgroup
};
Geom geom(int64_t n, int tile, int max_wg = kMaxWg) {
  const int64_t tiles = std::max<int64_t>(1, (n + tile - 1) / tile);
  const int64_t tpw = (tiles + max_wg - 1) / max_wg;
  return {(int)((tiles + tpw - 1) / tpw), tpw};
}
size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }
int grid_for(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(8192, (n + kT - 1) / kT)); }

// inclusive scan over the 64 lanes of a wave (wrapping unsigned arithmetic)
template <typename T>
__device__ __forceinline__ T wave_incl(T v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const T u = __shfl_up(v, d, 64);
    if (lane >= d) v += u;
  }
  return v;
}
// exclusive scan over a workgroup of NW waves; total = the sum over all threads.  lds: NW entries.  Every thread
// of the workgroup must call it (two barriers).
template <typename T, int NW>
__device__ __forceinline__ T wg_excl(T v, T& total, T* lds) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const T inc = wave_incl(v);
  if (lane == 63) lds[w] = inc;
  __syncthreads();
  T before = 0, all = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const T x = lds[i];
    before += i < w ? x : T(0);
    all += x;
  }
  __syncthreads();
  total = all;
  return before + inc - v;
}

// ---------------------------------------------------------------------------------------------------------------
// scans
template <typename T>
__global__ __launch_bounds__(kT) void scan_reduce(const T* in, int64_t n, int64_t tpw, T* __restrict__ part) {
  __shared__ T lds[4];
  const int64_t lo = (int64_t)blockIdx.x * tpw * kScanTile, hi = std::min<int64_t>(n, lo + tpw * kScanTile);
  T s = 0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += kT) s += in[i];
  T tot;
  (void)wg_excl<T, 4>(s, tot, lds);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// exclusive scan of the <= 1024 partials in place (one workgroup, 4 per thread)
template <typename T>
__global__ __launch_bounds__(kT) void scan_parts(T* part, int nwg) {
  __shared__ T lds[4];
  const int i0 = threadIdx.x * 4;
  T v[4], s = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v[q] = i0 + q < nwg ? part[i0 + q] : T(0);
    s += v[q];
  }
  T tot;
  T run = wg_excl<T, 4>(s, tot, lds);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (i0 + q < nwg) part[i0 + q] = run;
    run += v[q];
  }
}

// the segment's prefix sums with the carry of the segments before (in and out may alias: a thread reads its items
// before the workgroup's barrier and writes them after it)
template <typename T, bool INCL>
__global__ __launch_bounds__(kT) void scan_final(const T* in, T* out, int64_t n, int64_t tpw, const T* __restrict__ part) {
  __shared__ T lds[4];
  T carry = part[blockIdx.x];
  const int64_t lo = (int64_t)blockIdx.x * tpw * kScanTile, hi = std::min<int64_t>(n, lo + tpw * kScanTile);
  for (int64_t base = lo; base < hi; base += kScanTile) {
    const int64_t i0 = base + threadIdx.x * kScanIpt;
    T v[kScanIpt], s = 0;
#pragma unroll
    for (int q = 0; q < kScanIpt; ++q) {
      v[q] = i0 + q < hi ? in[i0 + q] : T(0);
      s += v[q];
    }
    T tot;
    T run = carry + wg_excl<T, 4>(s, tot, lds);
#pragma unroll
    for (int q = 0; q < kScanIpt; ++q) {
      if (INCL) run += v[q];
      if (i0 + q < hi) out[i0 + q] = run;
      if (!INCL) run += v[q];
    }
    carry += tot;
  }
}

template <typename T, bool INCL>
hipError_t scan_impl(const T* in, T* out, int64_t n, void* temp, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const Geom g = geom(n, kScanTile);
  T* part = static_cast<T*>(temp);
  hipLaunchKernelGGL(scan_reduce<T>, dim3(g.nwg), dim3(kT), 0, stream, in, n, g.tpw, part);
  hipLaunchKernelGGL(scan_parts<T>, dim3(1), dim3(kT), 0, stream, part, g.nwg);
  hipLaunchKernelGGL((scan_final<T, INCL>), dim3(g.nwg), dim3(kT), 0, stream, in, out, n, g.tpw, part);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------------------------
// runs of equal keys
__device__ __forceinline__ bool is_head(const uint64_t* keys, int64_t i) { return i == 0 || keys[i] != keys[i - 1]; }

__global__ __launch_bounds__(kT) void runs_count(const uint64_t* __restrict__ keys, int64_t n, int64_t tpw,
                                                  uint64_t* __restrict__ part) {
  __shared__ uint64_t lds[4];
  const int64_t lo = (int64_t)blockIdx.x * tpw * kScanTile, hi = std::min<int64_t>(n, lo + tpw * kScanTile);
  uint64_t c = 0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += kT) c += is_head(keys, i) ? 1u : 0u;
  uint64_t tot;
  (void)wg_excl<uint64_t, 4>(c, tot, lds);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kT) void runs_write(const uint64_t* __restrict__ keys, int64_t n, int64_t tpw,
                                                  const uint64_t* __restrict__ part, int nwg, uint64_t* __restrict__ unique,
                                                  int64_t* __restrict__ starts, int64_t* __restrict__ num_runs,
                                                  int32_t* __restrict__ run_of) {
  __shared__ uint64_t lds[4];
  uint64_t carry = part[blockIdx.x];
  const int64_t lo = (int64_t)blockIdx.x * tpw * kScanTile, hi = std::min<int64_t>(n, lo + tpw * kScanTile);
  for (int64_t base = lo; base < hi; base += kScanTile) {
    const int64_t i0 = base + threadIdx.x * kScanIpt;
    bool f[kScanIpt];
    uint64_t s = 0;
#pragma unroll
    for (int q = 0; q < kScanIpt; ++q) {
      f[q] = i0 + q < hi && is_head(keys, i0 + q);
      s += f[q] ? 1u : 0u;
    }
    uint64_t tot;
    uint64_t r = carry + wg_excl<uint64_t, 4>(s, tot, lds);
#pragma unroll
    for (int q = 0; q < kScanIpt; ++q) {
      if (f[q]) {
        if (unique) unique[r] = keys[i0 + q];
        starts[r] = i0 + q;
        ++r;
      }
      if (run_of && i0 + q < hi) run_of[i0 + q] = (int32_t)(r - 1);  // the run holding position i0 + q
    }
    carry += tot;
  }
  if (blockIdx.x == nwg - 1 && threadIdx.x == 0) *num_runs = (int64_t)carry;  // the last segment's end: all runs
}

__global__ void runs_lengths(const int64_t* __restrict__ starts, const int64_t* __restrict__ num_runs, int64_t n,
                             int64_t* __restrict__ lengths) {
  const int64_t R = *num_runs;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < R; r += (int64_t)gridDim.x * blockDim.x)
    lengths[r] = (r + 1 < R ? starts[r + 1] : n) - starts[r];
}

// sums[r] = P[end of run r] - P[start of run r], P = the exclusive prefix sums of vals (P[n] = P[n - 1] + vals[n - 1])
__global__ void runs_sum_from_prefix(const uint64_t* __restrict__ P, const int64_t* __restrict__ vals, int64_t n,
                                     const int64_t* __restrict__ starts, const int64_t* __restrict__ num_runs,
                                     int64_t* __restrict__ sums) {
  const int64_t R = *num_runs;
  const uint64_t total = P[n - 1] + (uint64_t)vals[n - 1];
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < R; r += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t end = r + 1 < R ? P[starts[r + 1]] : total;
    sums[r] = (int64_t)(end - P[starts[r]]);
  }
}

__global__ void runs_gather(const uint64_t* __restrict__ vals, const int64_t* __restrict__ starts,
                            const int64_t* __restrict__ num_runs, uint64_t* __restrict__ out) {
  const int64_t R = *num_runs;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < R; r += (int64_t)gridDim.x * blockDim.x)
    out[r] = vals[starts[r]];
}

// ---------------------------------------------------------------------------------------------------------------
// radix sort
__device__ __forceinline__ uint32_t digit_of(uint64_t k, int shift, uint32_t mask, bool desc) {
  const uint32_t d = (uint32_t)(k >> shift) & mask;
  return desc ? mask - d : d;
}

__global__ __launch_bounds__(kT) void sort_hist(const uint64_t* __restrict__ keys, int64_t n, int shift, int nbits,
                                                 int desc, int64_t tpw, uint32_t* __restrict__ hist, int nwg) {
  __shared__ uint32_t h[4][kRadix];
  const int tid = threadIdx.x, w = tid >> 6;
  const uint32_t mask = (1u << nbits) - 1u;
#pragma unroll
  for (int q = 0; q < 4; ++q) h[q][tid] = 0u;
  __syncthreads();
  const int64_t lo = (int64_t)blockIdx.x * tpw * kSortTile, hi = std::min<int64_t>(n, lo + tpw * kSortTile);
  for (int64_t base = lo; base < hi; base += kSortTile) {
    constexpr int kPer = kSortTile / kT;
    uint64_t k[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int64_t i = base + j * kT + tid;
      k[j] = i < hi ? keys[i] : 0ull;
    }
#pragma unroll
    for (int j = 0; j < kPer; ++j)
      if (base + j * kT + tid < hi) atomicAdd(&h[w][digit_of(k[j], shift, mask, desc != 0)], 1u);
  }
  __syncthreads();
  hist[(int64_t)tid * nwg + blockIdx.x] = h[0][tid] + h[1][tid] + h[2][tid] + h[3][tid];
}

// One-sweep sorts: every pass's digit totals from one read of the keys (LDS counts per pass, then one global atomic
// per workgroup, pass and digit)
__global__ __launch_bounds__(kT) void sort_count_all(const uint64_t* __restrict__ keys, int64_t n, int begin_bit,
                                                      int end_bit, int desc, uint32_t* __restrict__ gcount) {
  __shared__ uint32_t h[8][kRadix];
  const int tid = threadIdx.x;
  const int passes = (end_bit - begin_bit + 7) / 8;
#pragma unroll
  for (int p = 0; p < 8; ++p) h[p][tid] = 0u;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * kT * 4;
  for (int64_t i0 = (int64_t)blockIdx.x * kT * 4 + tid; i0 < n; i0 += stride) {
    uint64_t k[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) k[q] = i0 + q * kT < n ? keys[i0 + q * kT] : 0ull;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (i0 + q * kT >= n) continue;
      for (int p = 0; p < passes; ++p) {
        const int shift = begin_bit + 8 * p, nb = std::min(8, end_bit - shift);
        atomicAdd(&h[p][digit_of(k[q], shift, (1u << nb) - 1u, desc != 0)], 1u);
      }
    }
  }
  __syncthreads();
  for (int p = 0; p < passes; ++p) {
    const uint32_t c = h[p][tid];
    if (c) atomicAdd(&gcount[p * kRadix + tid], c);
  }
}

// digit-major (digit, workgroup) counts: workgroup d scans digit d's row in place (exclusive; the workgroup's offset
// among the digit's keys) and writes the digit's total (sort_scatter adds the totals of the digits below)
__global__ __launch_bounds__(kT) void sort_scan_rows(uint32_t* __restrict__ hist, int nwg, uint32_t* __restrict__ totals) {
  __shared__ uint32_t lds[4];
  uint32_t* row = hist + (int64_t)blockIdx.x * nwg;
  const int i0 = threadIdx.x * 4;  // nwg <= kMaxWg = 4 x 256
  uint32_t v[4], s = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v[q] = i0 + q < nwg ? row[i0 + q] : 0u;
    s += v[q];
  }
  uint32_t tot;
  uint32_t run = wg_excl<uint32_t, 4>(s, tot, lds);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (i0 + q < nwg) row[i0 + q] = run;
    run += v[q];
  }
  if (threadIdx.x == 0) totals[blockIdx.x] = tot;
}

// One pass of the sort over the workgroup's tiles.  Within a tile, wave w holds the contiguous 512 keys
// [512 w, 512 w + 512) (item j of lane l = key 512 w + 64 j + l: each load instruction reads 64 consecutive keys), so
// the input order is (wave, j, lane).  A wave ranks its items j = 0..7 in turn against its own 256 digit counters
// (wcnt[w][d]: read by every lane of a peer group, then advanced by the group's lowest lane -- one wave's LDS
// operations complete in order); thread d then turns the four waves' counts of digit d into offsets, and the
// workgroup scans the digit totals.  The next tile's keys (and values) are loaded into registers while this tile is
// ranked and written.
constexpr uint32_t kFlagAgg = 1u << 30, kFlagPre = 2u << 30, kCntMask = (1u << 30) - 1u;
constexpr int kSpinMax = 1 << 20;  // look-back polls of one status word before giving up (err): never a hang

template <int VB, bool ONE>
__global__ __launch_bounds__(kST) __attribute__((amdgpu_waves_per_eu(ONE ? 4 : 2))) void sort_scatter(
    const uint64_t* __restrict__ kin, uint64_t* __restrict__ kout, const void* __restrict__ vin, void* __restrict__ vout,
    int64_t n, int shift, int nbits, int desc, int64_t tpw, const uint32_t* __restrict__ hist,
    const uint32_t* __restrict__ totals, int nwg, uint32_t* __restrict__ status, uint32_t* __restrict__ ticket,
    int32_t* __restrict__ err) {
  using V = std::conditional_t<VB == 8, uint64_t, uint32_t>;
  __shared__ uint16_t wcnt[kSW][kRadix];  // per wave and digit: running count, then the wave's offset in the digit
  __shared__ uint32_t run[kRadix];        // next global position of each digit for this workgroup
  __shared__ uint32_t tstart[kRadix];     // a digit's first position in the tile's sorted order
  __shared__ uint32_t wsum[kSW];
  __shared__ uint64_t stage[kSortTile];   // the tile's keys in sorted order, then its values
  __shared__ uint32_t s_tile;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (ONE && tid == 0) s_tile = atomicAdd(ticket, 1u);  // tiles in the order workgroups start: look-back never waits
                                                        // on a workgroup that has not started
  const uint32_t mask = (1u << nbits) - 1u;
  const bool dsc = desc != 0;
  const V* vi = static_cast<const V*>(vin);
  V* vo = static_cast<V*>(vout);
  V* vstage = reinterpret_cast<V*>(stage);
  {
    // run[d] = (keys of the digits below d) + (keys of digit d in the workgroups before this one)
    uint32_t tot;
    const uint32_t before = wg_excl<uint32_t, kSW>(tid < kRadix ? totals[tid] : 0u, tot, wsum);
    if (tid < kRadix) run[tid] = before + (ONE ? 0u : hist[(int64_t)tid * nwg + blockIdx.x]);
  }
  // ONE: this workgroup's single tile (s_tile is visible past wg_excl's barriers)
  const int64_t tile = ONE ? (int64_t)s_tile : 0;
  const int64_t lo = ONE ? tile * kSortTile : (int64_t)blockIdx.x * tpw * kSortTile;
  const int64_t hi = std::min<int64_t>(n, lo + (ONE ? 1 : tpw) * kSortTile);
  const int sub = w * (kSortTile / kSW) + lane;  // the thread's item 0 within a tile
  for (int64_t base = lo; base < hi; base += kSortTile) {
    const int nvalid = (int)std::min<int64_t>(kSortTile, hi - base);
    uint64_t k[kSortItems];
#pragma unroll
    for (int j = 0; j < kSortItems; ++j) k[j] = sub + 64 * j < nvalid ? kin[base + sub + 64 * j] : 0ull;
    reinterpret_cast<u32a*>(&wcnt[0][0])[tid] = 0u;  // kSW x 256 x 2 bytes = 2 dwords per thread
    reinterpret_cast<u32a*>(&wcnt[0][0])[tid + kST] = 0u;
    __syncthreads();  // counters zeroed
    uint32_t dr[kSortItems];  // digit | rank within the wave's keys of that digit << 8
#pragma unroll
    for (int j = 0; j < kSortItems; ++j) {
      const bool ok = sub + 64 * j < nvalid;
      const uint32_t d = digit_of(k[j], shift, mask, dsc);
      uint64_t peers = __builtin_amdgcn_ballot_w64(ok);
      for (int b = 0; b < nbits; ++b) {
        const bool bit = (d >> b) & 1u;
        const uint64_t bb = __builtin_amdgcn_ballot_w64(bit);
        peers &= bit ? bb : ~bb;
      }
      const uint32_t below =
          __builtin_amdgcn_mbcnt_hi((uint32_t)(peers >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)peers, 0u));
      uint32_t c = 0;
      if (ok) c = wcnt[w][d];
      dr[j] = d | (c + below) << 8;
      if (ok && below == 0) wcnt[w][d] = (uint16_t)(c + __builtin_popcountll(peers));
    }
    V v[kSortItems];  // in flight while the tile's keys are placed and written
    if constexpr (VB != 0) {
#pragma unroll
      for (int j = 0; j < kSortItems; ++j) v[j] = sub + 64 * j < nvalid ? vi[base + sub + 64 * j] : V(0);
    }
    __syncthreads();
    uint32_t acc = 0;  // thread tid < 256: digit tid's count in the tile
    if (tid < kRadix) {
#pragma unroll
      for (int q = 0; q < kSW; ++q) {
        const uint32_t c = wcnt[q][tid];
        wcnt[q][tid] = (uint16_t)acc;
        acc += c;
      }
      // publish the tile's count of digit tid (tile 0: already its inclusive prefix)
      if (ONE)
        __hip_atomic_store(status + tile * kRadix + tid, (tile == 0 ? kFlagPre : kFlagAgg) | acc, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    uint32_t total;
    const uint32_t ts = wg_excl<uint32_t, kSW>(acc, total, wsum);
    if (tid < kRadix) tstart[tid] = ts;
    if (ONE && tid < kRadix && tile > 0) {
      // decoupled look-back: the keys of digit tid in the tiles before, from their aggregates back to the first
      // published inclusive prefix
      uint32_t excl = 0;
      int64_t j = tile - 1;
      int spins = 0;
      while (true) {
        const uint32_t st = __hip_atomic_load(status + j * kRadix + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((st & ~kCntMask) == 0u) {
          if (++spins > kSpinMax) {
            *err = 1;
            break;
          }
          continue;
        }
        excl += st & kCntMask;
        if ((st & ~kCntMask) == kFlagPre || j == 0) break;
        --j;
      }
      __hip_atomic_store(status + tile * kRadix + tid, kFlagPre | (excl + acc), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      run[tid] += excl;
    }
    __syncthreads();
    auto lpos = [&](int j) __attribute__((always_inline)) {
      const uint32_t d = dr[j] & 0xFFu;
      return tstart[d] + wcnt[w][d] + (dr[j] >> 8);
    };
#pragma unroll
    for (int j = 0; j < kSortItems; ++j)
      if (sub + 64 * j < nvalid) stage[lpos(j)] = k[j];
    __syncthreads();
    uint32_t gpos[kSortItems];
#pragma unroll
    for (int j = 0; j < kSortItems; ++j) {
      const int i = j * kST + tid;
      gpos[j] = 0;
      if (i < nvalid) {
        const uint64_t key = stage[i];
        const uint32_t dd = digit_of(key, shift, mask, dsc);
        gpos[j] = run[dd] + (uint32_t)i - tstart[dd];
        kout[gpos[j]] = key;
      }
    }
    if constexpr (VB != 0) {
      __syncthreads();  // every key read out of the stage
#pragma unroll
      for (int j = 0; j < kSortItems; ++j)
        if (sub + 64 * j < nvalid) vstage[lpos(j)] = v[j];
      __syncthreads();
#pragma unroll
      for (int j = 0; j < kSortItems; ++j) {
        const int i = j * kST + tid;
        if (i < nvalid) vo[gpos[j]] = vstage[i];
      }
    }
    __syncthreads();  // stage, wcnt and run read by every thread before the next tile rewrites them
    if (tid < kRadix) run[tid] += acc;
  }
}

}  // namespace

size_t scan_temp_bytes(int64_t) { return align256((size_t)kMaxWg * 8); }

hipError_t exclusive_sum_i64(const int64_t* in, int64_t* out, int64_t n, void* temp, hipStream_t stream) {
  return scan_impl<uint64_t, false>(reinterpret_cast<const uint64_t*>(in), reinterpret_cast<uint64_t*>(out), n, temp,
                                    stream);
}
hipError_t inclusive_sum_u32(const uint32_t* in, uint32_t* out, int64_t n, void* temp, hipStream_t stream) {
  return scan_impl<uint32_t, true>(in, out, n, temp, stream);
}

size_t runs_temp_bytes(int64_t n) { return align256((size_t)kMaxWg * 8) + align256((size_t)std::max<int64_t>(1, n) * 8); }

hipError_t runs(const uint64_t* keys, int64_t n, uint64_t* unique, int64_t* starts, int64_t* lengths,
                int64_t* num_runs, void* temp, hipStream_t stream, int32_t* run_of) {
  if (n <= 0) return hipMemsetAsync(num_runs, 0, sizeof(int64_t), stream);
  char* t = static_cast<char*>(temp);
  uint64_t* part = reinterpret_cast<uint64_t*>(t);
  int64_t* st = starts ? starts : reinterpret_cast<int64_t*>(t + align256((size_t)kMaxWg * 8));
  const Geom g = geom(n, kScanTile);
  hipLaunchKernelGGL(runs_count, dim3(g.nwg), dim3(kT), 0, stream, keys, n, g.tpw, part);
  hipLaunchKernelGGL(scan_parts<uint64_t>, dim3(1), dim3(kT), 0, stream, part, g.nwg);
  hipLaunchKernelGGL(runs_write, dim3(g.nwg), dim3(kT), 0, stream, keys, n, g.tpw, part, g.nwg, unique, st, num_runs,
                     run_of);
  if (lengths) hipLaunchKernelGGL(runs_lengths, dim3(grid_for(n)), dim3(kT), 0, stream, st, num_runs, n, lengths);
  return hipGetLastError();
}

size_t run_sums_temp_bytes(int64_t n) { return align256((size_t)std::max<int64_t>(1, n) * 8) + scan_temp_bytes(n); }

hipError_t run_sums_i64(const int64_t* vals, int64_t n, const int64_t* starts, const int64_t* num_runs, int64_t* sums,
                        void* temp, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  char* t = static_cast<char*>(temp);
  uint64_t* P = reinterpret_cast<uint64_t*>(t);
  if (hipError_t e = scan_impl<uint64_t, false>(reinterpret_cast<const uint64_t*>(vals), P, n,
                                                t + align256((size_t)n * 8), stream))
    return e;
  hipLaunchKernelGGL(runs_sum_from_prefix, dim3(grid_for(n)), dim3(kT), 0, stream, P, vals, n, starts, num_runs, sums);
  return hipGetLastError();
}

hipError_t run_firsts_u64(const uint64_t* vals, int64_t n, const int64_t* starts, const int64_t* num_runs,
                          uint64_t* firsts, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(runs_gather, dim3(grid_for(n)), dim3(kT), 0, stream, vals, starts, num_runs, firsts);
  return hipGetLastError();
}

// one-sweep passes (every pass's digit totals counted up front, each tile's offsets by look-back) below 2^30 keys: the
// status words hold 30-bit counts; the segmented reduce-then-scan passes above
bool one_sweep(int64_t n) {
  static const bool segmented = std::getenv("DQ_SORT_SEGMENTED") != nullptr;  // test knob: the other pass form
  return n < (int64_t(1) << 30) && !segmented;
}
int64_t sort_tiles(int64_t n) { return std::max<int64_t>(1, (n + kSortTile - 1) / kSortTile); }

size_t sort_temp_bytes(int64_t n, int val_bytes) {
  const Geom g = geom(n, kSortTile, kSortMaxWg);
  const size_t m = (size_t)std::max<int64_t>(1, n);
  const size_t bufs = align256(m * 8) + align256(m * (size_t)val_bytes);
  if (one_sweep(n))  // gcount[8][256] + tickets[8] + err, then the status words of one pass
    return bufs + align256(8 * kRadix * 4 + 8 * 4 + 4) + align256((size_t)sort_tiles(n) * kRadix * 4);
  return bufs + align256((size_t)kRadix * g.nwg * 4) + align256(kRadix * 4);
}

hipError_t sort_pairs(const uint64_t* keys_in, uint64_t* keys_out, const void* vals_in, void* vals_out, int val_bytes,
                      int64_t n, int begin_bit, int end_bit, bool descending, void* temp, size_t temp_bytes,
                      hipStream_t stream) {
  if (val_bytes != 0 && val_bytes != 4 && val_bytes != 8) return hipErrorInvalidValue;
  if (n <= 0) return hipSuccess;
  if (n >= (int64_t(1) << 31) || temp_bytes < sort_temp_bytes(n, val_bytes)) return hipErrorInvalidValue;
  begin_bit = std::max(0, begin_bit);
  end_bit = std::min(64, end_bit);
  if (begin_bit >= end_bit) {  // nothing to order by: the input order is the stable order
    if (hipError_t e = hipMemcpyAsync(keys_out, keys_in, (size_t)n * 8, hipMemcpyDeviceToDevice, stream)) return e;
    if (val_bytes) return hipMemcpyAsync(vals_out, vals_in, (size_t)n * val_bytes, hipMemcpyDeviceToDevice, stream);
    return hipSuccess;
  }
  const Geom g = geom(n, kSortTile, kSortMaxWg);
  char* t = static_cast<char*>(temp);
  const size_t m = (size_t)n;
  uint64_t* alt_k = reinterpret_cast<uint64_t*>(t);
  void* alt_v = t + align256(m * 8);
  char* rest = t + align256(m * 8) + align256(m * (size_t)val_bytes);
  const bool one = one_sweep(n);
  uint32_t *hist = nullptr, *totals = nullptr, *gcount = nullptr, *tickets = nullptr, *status = nullptr;
  int32_t* err = nullptr;
  const int64_t ntiles = sort_tiles(n);
  if (one) {
    gcount = reinterpret_cast<uint32_t*>(rest);
    tickets = gcount + 8 * kRadix;
    err = reinterpret_cast<int32_t*>(tickets + 8);
    status = reinterpret_cast<uint32_t*>(rest + align256(8 * kRadix * 4 + 8 * 4 + 4));
    if (hipError_t e = hipMemsetAsync(gcount, 0, 8 * kRadix * 4 + 8 * 4 + 4, stream)) return e;
    hipLaunchKernelGGL(sort_count_all, dim3((int)std::min<int64_t>(1024, (n + 4 * kT - 1) / (4 * kT))), dim3(kT), 0,
                       stream, keys_in, n, begin_bit, end_bit, (int)descending, gcount);
  } else {
    hist = reinterpret_cast<uint32_t*>(rest);
    totals = reinterpret_cast<uint32_t*>(rest + align256((size_t)kRadix * g.nwg * 4));
  }
  const int passes = (end_bit - begin_bit + 7) / 8;
  const uint64_t* src_k = keys_in;
  const void* src_v = vals_in;
  for (int p = 0; p < passes; ++p) {
    const int shift = begin_bit + 8 * p, nbits = std::min(8, end_bit - shift);
    const bool to_out = (passes - 1 - p) % 2 == 0;  // the last pass writes the output
    uint64_t* dst_k = to_out ? keys_out : alt_k;
    void* dst_v = to_out ? vals_out : alt_v;
    const int desc = (int)descending;
    if (one) {
      if (hipError_t e = hipMemsetAsync(status, 0, (size_t)ntiles * kRadix * 4, stream)) return e;
      const uint32_t* tot = gcount + p * kRadix;
      uint32_t* tk = tickets + p;
      const dim3 grid((unsigned)ntiles);
      if (val_bytes == 0)
        hipLaunchKernelGGL((sort_scatter<0, true>), grid, dim3(kST), 0, stream, src_k, dst_k, nullptr, nullptr, n, shift,
                           nbits, desc, (int64_t)1, nullptr, tot, 1, status, tk, err);
      else if (val_bytes == 4)
        hipLaunchKernelGGL((sort_scatter<4, true>), grid, dim3(kST), 0, stream, src_k, dst_k, src_v, dst_v, n, shift,
                           nbits, desc, (int64_t)1, nullptr, tot, 1, status, tk, err);
      else
        hipLaunchKernelGGL((sort_scatter<8, true>), grid, dim3(kST), 0, stream, src_k, dst_k, src_v, dst_v, n, shift,
                           nbits, desc, (int64_t)1, nullptr, tot, 1, status, tk, err);
    } else {
      hipLaunchKernelGGL(sort_hist, dim3(g.nwg), dim3(kT), 0, stream, src_k, n, shift, nbits, desc, g.tpw, hist, g.nwg);
      hipLaunchKernelGGL(sort_scan_rows, dim3(kRadix), dim3(kT), 0, stream, hist, g.nwg, totals);
      if (val_bytes == 0)
        hipLaunchKernelGGL((sort_scatter<0, false>), dim3(g.nwg), dim3(kST), 0, stream, src_k, dst_k, nullptr, nullptr,
                           n, shift, nbits, desc, g.tpw, hist, totals, g.nwg, nullptr, nullptr, nullptr);
      else if (val_bytes == 4)
        hipLaunchKernelGGL((sort_scatter<4, false>), dim3(g.nwg), dim3(kST), 0, stream, src_k, dst_k, src_v, dst_v, n,
                           shift, nbits, desc, g.tpw, hist, totals, g.nwg, nullptr, nullptr, nullptr);
      else
        hipLaunchKernelGGL((sort_scatter<8, false>), dim3(g.nwg), dim3(kST), 0, stream, src_k, dst_k, src_v, dst_v, n,
                           shift, nbits, desc, g.tpw, hist, totals, g.nwg, nullptr, nullptr, nullptr);
    }
    if (hipError_t e = hipGetLastError()) return e;
    src_k = dst_k;
    src_v = dst_v;
  }
  if (one) {  // a look-back that gave up (never expected) fails the sort instead of leaving a wrong order
    int32_t h_err = 0;
    if (hipError_t e = hipMemcpyAsync(&h_err, err, 4, hipMemcpyDeviceToHost, stream)) return e;
    if (hipError_t e = hipStreamSynchronize(stream)) return e;
    if (h_err) return hipErrorLaunchTimeOut;
  }
  return hipSuccess;
}

}  // namespace prim
}  // namespace dq
