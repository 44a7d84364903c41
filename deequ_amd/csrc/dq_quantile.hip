// dq_quantile.hip -- ApproxQuantile / ApproxQuantiles (first half) on the GPU.
//
// Reference: ApproxQuantile.scala:49-103 / ApproxQuantiles.scala:30-105 aggregate the column with
// Spark 2.2's ApproximatePercentile (a Greenwald-Khanna QuantileSummaries with the given relative
// error) and read the metric with PercentileDigest.getPercentiles -> QuantileSummaries.query:
// q <= relativeError -> the smallest value, q >= 1 - relativeError -> the largest, otherwise a value
// whose rank is within ceil(relativeError * n) of ceil(q * n).  GK's answer depends on the order the
// rows arrive in (partitioning, buffer flushes, compression), so no GPU restatement can reproduce it
// bit for bit.  This path answers the exact order statistic of rank ceil(q * n) (or rank 1 / n at the
// two ends, as query does) -- a value GK's guarantee admits for every relativeError, which is what the
// reference's own tests check (AnalyzerTests.scala:533-565: a band around the true quantile).
//
// Algorithm: MSD radix select over the order-preserving 64-bit key of each non-null value (f64:
// IEEE bits with the sign flipped / negatives inverted, NaN canonical and largest as
// java.lang.Double.compare orders it, -0.0 < 0.0; i64 / i32: two's complement with the sign bit
// flipped).  Six passes over the column (digits of 11,11,11,11,11,9 bits); each pass histograms, per
// requested quantile, the next digit of the keys that share that quantile's selected prefix
// (LDS histogram, flushed to HBM with one 64-bit atomic per non-empty bin), and the host picks the bin
// holding the target rank.  Each pass streams the values once (8 or 4 B per row + 1/8 B validity): HBM
// bound, no sort, no scratch the size of the column.  Chunks and row shards add their histograms, so
// the same select runs over any number of chunks (and across ranks with one all-reduce per pass).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <type_traits>
#include <vector>

#include "dq_internal.h"
#include "dq_prim.h"

namespace dq {
namespace {

constexpr int kQBlock = 256;
constexpr int kQBins = 2048;  // 11-bit digits
constexpr int kQUnroll = 4;   // 16-byte vectors in flight per thread
constexpr int kQPasses = 6;
constexpr int kQStage = 256;  // APPEND: candidate keys staged in LDS per quantile and workgroup
constexpr int kQAndOrCopies = 16;  // pass 0's AND / OR of the keys: copies the workgroups spread over
constexpr int kQShift[kQPasses] = {53, 42, 31, 20, 9, 0};
constexpr int kQWidth[kQPasses] = {11, 11, 11, 11, 11, 9};

struct QSelect {
  uint64_t prefix[DQ_MAX_QUANTILES];
  uint64_t pmask[DQ_MAX_QUANTILES];
  unsigned long long* cand[DQ_MAX_QUANTILES];  // APPEND: keys matching prefix[q] go to cand[q][...]
  unsigned long long* cand_cnt;                // APPEND: nq append cursors
};

__device__ __forceinline__ uint64_t order_key_f64(uint64_t b) {
  if ((b & 0x7FFFFFFFFFFFFFFFull) > 0x7FF0000000000000ull) b = 0x7FF8000000000000ull;  // NaN canonical
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

template <int TYPE>
__device__ __forceinline__ uint64_t order_key(uint64_t raw) {
  if constexpr (TYPE == DQ_TYPE_F64) return order_key_f64(raw);
  else if constexpr (TYPE == DQ_TYPE_I64) return raw ^ 0x8000000000000000ull;
  else return (uint64_t)(int64_t)(int32_t)(uint32_t)raw ^ 0x8000000000000000ull;
}

// One key into the digit histograms of every quantile whose prefix it matches; with APPEND the
// matching keys are also appended to that quantile's candidate list (one global atomic per wave).
template <bool APPEND>
__device__ __forceinline__ void q_count(uint64_t key, bool ok, int32_t shift, uint32_t dmask, int32_t nq,
                                        const QSelect& sel, uint32_t* lds_hist) {
  const uint32_t d = (uint32_t)(key >> shift) & dmask;
  for (int q = 0; q < nq; ++q) {
    const bool m = ok && (key & sel.pmask[q]) == sel.prefix[q];
    if (m) atomicAdd(&lds_hist[q * kQBins + d], 1u);
    if constexpr (APPEND) {
      const uint64_t b = __builtin_amdgcn_ballot_w64(m);
      if (b) {
        const int lane = threadIdx.x & 63, first = __builtin_ctzll(b);
        unsigned long long base = 0;
        if (lane == first) base = atomicAdd(&sel.cand_cnt[q], (unsigned long long)__builtin_popcountll(b));
        base = __shfl(base, first);
        if (m) sel.cand[q][base + __builtin_popcountll(b & ((1ull << lane) - 1ull))] = key;
      }
    }
  }
}

// Pass over a column chunk: each thread reads 16-byte vectors (V rows; V = 1 when the values are not
// 16-byte aligned), kQUnroll of them in flight, grid-stride; one validity word per vector.
template <int TYPE, int V, bool APPEND>
__global__ __launch_bounds__(kQBlock) void dq_quantile_hist(const void* __restrict__ values,
                                                            const uint32_t* __restrict__ validity, int64_t n,
                                                            int32_t shift, uint32_t dmask, int32_t nq, QSelect sel,
                                                            unsigned long long* __restrict__ hist,
                                                            unsigned long long* __restrict__ andor) {
  using T = typename std::conditional<TYPE == DQ_TYPE_I32, uint32_t, uint64_t>::type;
  // LDS: nq x kQBins digit counts; APPEND: + nq x kQStage staged keys + nq reserved / nq staged counts
  extern __shared__ uint32_t lds_hist[];
  unsigned long long* stage = reinterpret_cast<unsigned long long*>(lds_hist + nq * kQBins);
  uint32_t* st_res = reinterpret_cast<uint32_t*>(stage + (APPEND ? nq * kQStage : 0));
  uint32_t* st_ok = st_res + nq;
  for (int i = threadIdx.x; i < nq * kQBins; i += kQBlock) lds_hist[i] = 0;
  if (APPEND && threadIdx.x < 2 * nq) st_res[threadIdx.x] = 0;
  __syncthreads();
  const T* v = reinterpret_cast<const T*>(values);
  uint64_t k_and = ~0ull, k_or = 0;  // andor != nullptr (pass 0): AND / OR of the non-null keys
  const int64_t nvec = (n + V - 1) / V;
  const int64_t stride = (int64_t)gridDim.x * kQBlock;
  for (int64_t v0 = (int64_t)blockIdx.x * kQBlock + threadIdx.x; v0 - threadIdx.x < nvec; v0 += stride * kQUnroll) {
    // (round 4, r4z2: loading the next iteration's vectors before this one's histogram work, as the digest passes
    // do, measured no change here -- 0.213 / 0.310 vs 0.208 / 0.308 ms per 1e8 rows: kQUnroll vectors per thread
    // are in flight already)
    T raw[kQUnroll][V];
    uint32_t vw[kQUnroll];
#pragma unroll
    for (int u = 0; u < kQUnroll; ++u) {
      const int64_t vi = v0 + u * stride;
      const int64_t r = vi * V;
      vw[u] = 0;
      if (r + V <= n) {
        if constexpr (V > 1) {
          typedef T vec_t __attribute__((ext_vector_type(V)));
          const vec_t x = __builtin_nontemporal_load(reinterpret_cast<const vec_t*>(v + r));
#pragma unroll
          for (int e = 0; e < V; ++e) raw[u][e] = x[e];
        } else {
          raw[u][0] = __builtin_nontemporal_load(v + r);
        }
        vw[u] = validity ? (validity[r >> 5] >> (r & 31)) : 0xFFFFFFFFu;
      } else {
#pragma unroll
        for (int e = 0; e < V; ++e) {
          raw[u][e] = r + e < n ? v[r + e] : 0;
          if (r + e < n) vw[u] |= (validity ? (validity[(r + e) >> 5] >> ((r + e) & 31)) & 1u : 1u) << e;
        }
      }
    }
    // order keys and digits once per row (the quantile loops below are not unrolled)
    uint64_t key[kQUnroll * V];
    uint32_t dig[kQUnroll * V];
#pragma unroll
    for (int u = 0; u < kQUnroll; ++u)
#pragma unroll
      for (int e = 0; e < V; ++e) {
        key[u * V + e] = order_key<TYPE>(raw[u][e]);
        dig[u * V + e] = (uint32_t)(key[u * V + e] >> shift) & dmask;
      }
    if constexpr (!APPEND) {
      if (andor) {
#pragma unroll
        for (int u = 0; u < kQUnroll; ++u)
#pragma unroll
          for (int e = 0; e < V; ++e)
            if ((vw[u] >> e) & 1u) {
              k_and &= key[u * V + e];
              k_or |= key[u * V + e];
            }
      }
      for (int q = 0; q < nq; ++q) {
        const uint64_t pm = sel.pmask[q], pf = sel.prefix[q];
        uint32_t* hq = lds_hist + q * kQBins;
#pragma unroll
        for (int u = 0; u < kQUnroll; ++u)
#pragma unroll
          for (int e = 0; e < V; ++e)
            if (((vw[u] >> e) & 1u) && (key[u * V + e] & pm) == pf) atomicAdd(&hq[dig[u * V + e]], 1u);
      }
    } else {
      // histogram as above (the common path: no lane of the wave matches), then, only in waves with a
      // match, per quantile one append reservation per wave for all kQUnroll x V rows of its lanes (a
      // wave-wide exclusive scan of the lanes' match counts)
      bool any = false;
      for (int q = 0; q < nq; ++q) {
        const uint64_t pm = sel.pmask[q], pf = sel.prefix[q];
        uint32_t* hq = lds_hist + q * kQBins;
#pragma unroll
        for (int u = 0; u < kQUnroll; ++u)
#pragma unroll
          for (int e = 0; e < V; ++e)
            if (((vw[u] >> e) & 1u) && (key[u * V + e] & pm) == pf) {
              atomicAdd(&hq[dig[u * V + e]], 1u);
              any = true;
            }
      }
      if (__builtin_amdgcn_ballot_w64(any) != 0) {
        const int lane = threadIdx.x & 63;
        for (int q = 0; q < nq; ++q) {
          const uint64_t pm = sel.pmask[q], pf = sel.prefix[q];
          uint32_t mbits = 0;
#pragma unroll
          for (int u = 0; u < kQUnroll; ++u)
#pragma unroll
            for (int e = 0; e < V; ++e)
              mbits |= (uint32_t)(((vw[u] >> e) & 1u) && (key[u * V + e] & pm) == pf) << (u * V + e);
          if (__builtin_amdgcn_ballot_w64(mbits != 0) == 0) continue;
          const uint32_t cnt = __builtin_popcount(mbits);
          uint32_t incl = cnt;
#pragma unroll
          for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(incl, d);
            if (lane >= d) incl += y;
          }
          const uint32_t total = __shfl(incl, 63);
          // reserve in the workgroup's LDS stage (flushed with one global atomic per workgroup); a wave
          // whose keys do not fit goes to the global list directly.  Reservations are ordered, so the
          // staged keys are exactly [0, st_ok[q]): every wave before the first misfit fitted.
          uint32_t spos = 0;
          if (lane == 0) spos = atomicAdd(&st_res[q], total);
          spos = __shfl(spos, 0);
          unsigned long long* cq;
          unsigned long long pos;
          if (spos + total <= (uint32_t)kQStage) {
            if (lane == 0) atomicAdd(&st_ok[q], total);
            cq = stage + q * kQStage;
            pos = spos + (incl - cnt);
          } else {
            unsigned long long base = 0;
            if (lane == 0) base = atomicAdd(&sel.cand_cnt[q], (unsigned long long)total);
            base = __shfl(base, 0);
            cq = sel.cand[q];
            pos = base + (incl - cnt);
          }
#pragma unroll
          for (int u = 0; u < kQUnroll; ++u)
#pragma unroll
            for (int e = 0; e < V; ++e)
              if ((mbits >> (u * V + e)) & 1u) cq[pos++] = key[u * V + e];
        }
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nq * kQBins; i += kQBlock)
    if (lds_hist[i]) atomicAdd(&hist[i], (unsigned long long)lds_hist[i]);
  if (!APPEND && andor) {
    // the keys agree on every bit where AND == OR: the host skips the later passes whose digit lies there.  Lanes,
    // then waves (LDS), then one atomic pair per workgroup into one of kQAndOrCopies copies (blockIdx % copies; the
    // host combines them): every wave's atomics on one pair of addresses had serialized (+0.3 ms per launch)
    __shared__ unsigned long long w_and[kQBlock / 64], w_or[kQBlock / 64];
    for (int d = 32; d >= 1; d >>= 1) {
      k_and &= __shfl_xor(k_and, d);
      k_or |= __shfl_xor(k_or, d);
    }
    if ((threadIdx.x & 63) == 0) {
      w_and[threadIdx.x >> 6] = k_and;
      w_or[threadIdx.x >> 6] = k_or;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int w = 1; w < kQBlock / 64; ++w) {
        k_and &= w_and[w];
        k_or |= w_or[w];
      }
      unsigned long long* const c = andor + 2 * (blockIdx.x % kQAndOrCopies);
      if (k_and != ~0ull) atomicAnd(&c[0], (unsigned long long)k_and);
      if (k_or != 0) atomicOr(&c[1], (unsigned long long)k_or);
    }
  }
  if constexpr (APPEND) {
    __shared__ unsigned long long flush_base[DQ_MAX_QUANTILES];
    if (threadIdx.x < nq && st_ok[threadIdx.x] > 0)
      flush_base[threadIdx.x] = atomicAdd(&sel.cand_cnt[threadIdx.x], (unsigned long long)st_ok[threadIdx.x]);
    __syncthreads();
    for (int q = 0; q < nq; ++q) {
      const uint32_t k = st_ok[q];
      for (uint32_t i = threadIdx.x; i < k; i += kQBlock) sel.cand[q][flush_base[q] + i] = stage[q * kQStage + i];
    }
  }
}

// Later passes over one quantile's candidate keys (already order keys, all non-null).
__global__ __launch_bounds__(kQBlock) void dq_quantile_cand_hist(const unsigned long long* __restrict__ keys,
                                                                 int64_t n, int32_t shift, uint32_t dmask,
                                                                 uint64_t prefix, uint64_t pmask,
                                                                 unsigned long long* __restrict__ hist) {
  __shared__ uint32_t lds_hist[kQBins];
  for (int i = threadIdx.x; i < kQBins; i += kQBlock) lds_hist[i] = 0;
  __syncthreads();
  for (int64_t r = (int64_t)blockIdx.x * kQBlock + threadIdx.x; r < n; r += (int64_t)gridDim.x * kQBlock) {
    const uint64_t key = keys[r];
    if ((key & pmask) == prefix) atomicAdd(&lds_hist[(uint32_t)(key >> shift) & dmask], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kQBins; i += kQBlock)
    if (lds_hist[i]) atomicAdd(&hist[i], (unsigned long long)lds_hist[i]);
}

template <int TYPE, int V>
void launch_hist(bool append, int grid, size_t lds, hipStream_t st, const void* values, const uint32_t* val,
                 int64_t rows, int shift, uint32_t dmask, int nq, const QSelect& sel, unsigned long long* hist,
                 unsigned long long* andor) {
  if (append)
    hipLaunchKernelGGL((dq_quantile_hist<TYPE, V, true>), dim3(grid), dim3(kQBlock), lds, st, values, val, rows, shift,
                       dmask, nq, sel, hist, nullptr);
  else
    hipLaunchKernelGGL((dq_quantile_hist<TYPE, V, false>), dim3(grid), dim3(kQBlock), lds, st, values, val, rows,
                       shift, dmask, nq, sel, hist, andor);
}

#define QHIP(x)                                                                             \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) return set_error(DQ_E_HIP, "%s: %s", #x, hipGetErrorString(e_)); \
  } while (0)

struct DevHist {
  unsigned long long* p = nullptr;
  DevHist() = default;
  DevHist(const DevHist&) = delete;
  ~DevHist() {
    if (p) (void)hipFree(p);
  }
};

// stream-ordered scratch from a pool of this library's own per device (hipMallocFromPoolAsync): the digest's
// temporaries cost no hipMalloc / hipFree round trips across calls, while blocks beyond kPoolKeep bytes go
// back to the device at the next synchronisation -- and torch's (the device default) pool is left alone
constexpr uint64_t kPoolKeep = 256ull << 20;
hipError_t scratch_pool(int device, hipMemPool_t* out) {
  static std::mutex mu;
  static std::map<int, hipMemPool_t> pools;
  std::lock_guard<std::mutex> lock(mu);
  auto it = pools.find(device);
  if (it != pools.end()) {
    *out = it->second;
    return hipSuccess;
  }
  hipMemPoolProps props{};
  props.allocType = hipMemAllocationTypePinned;
  props.location.type = hipMemLocationTypeDevice;
  props.location.id = device;
  hipMemPool_t pool = nullptr;
  hipError_t e = hipMemPoolCreate(&pool, &props);
  if (e != hipSuccess) return e;
  uint64_t keep = kPoolKeep;
  e = hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
  if (e != hipSuccess) {
    (void)hipMemPoolDestroy(pool);
    return e;
  }
  pools[device] = pool;
  *out = pool;
  return hipSuccess;
}

struct StreamTmp {
  void* p = nullptr;
  hipStream_t s = nullptr;
  StreamTmp() = default;
  StreamTmp(const StreamTmp&) = delete;
  ~StreamTmp() {
    if (p) (void)hipFreeAsync(p, s);
  }
  hipError_t alloc(size_t bytes, hipMemPool_t pool, hipStream_t st) {
    if (p) (void)hipFreeAsync(p, s);
    p = nullptr;
    s = st;
    return hipMallocFromPoolAsync(&p, std::max<size_t>(bytes, 16), pool, st);
  }
};

double key_to_double(int32_t type, uint64_t key) {
  if (type == DQ_TYPE_F64) {
    const uint64_t b = (key >> 63) ? (key & 0x7FFFFFFFFFFFFFFFull) : ~key;
    double d;
    std::memcpy(&d, &b, 8);
    return d;
  }
  return (double)(int64_t)(key ^ 0x8000000000000000ull);
}

// ---- the digest's multi-rank select (dq_quantile_digest): every sample rank of the digest in two passes over
// the column.  Splitters from an evenly spaced sample of the keys cut the key range into kDBuckets buckets of
// about equal population; pass 1 counts each bucket's keys, the host finds the bucket of every sample rank,
// pass 2 compacts the keys of those buckets only (about m / kDBuckets of the column for m samples) and one
// radix sort of that small set gives every sample rank's exact key.  A skewed column (one value in most
// rows) only makes a target bucket larger: the sort then covers it, still exactly.
constexpr int kDBuckets = 2048;              // buckets (kDBuckets - 1 splitters, a branchless 11-step search)
constexpr int kDSample = 16384;              // keys sampled for the splitters
constexpr int kDCountCopies = 8;             // bucket-count copies (blockIdx % 8; the host adds them): a skewed
                                             // column's hot bucket gets every workgroup's atomic at the launch's end
constexpr int kDStage = 2048;                // candidate keys staged per workgroup (flushed past kDStage - 1024)
constexpr int kDCells = 2048;                // cells of the splitters' lookup table (DigestCells)
constexpr int kDAndOrCopies = 16;            // the candidates' AND / OR: copies the workgroups spread over
constexpr int64_t kDCandBudget = int64_t(1) << 26;  // candidates per compaction batch (~1.6 GB of scratch)

// the key of row i * n / m of a chunk (i < m; ~0 for a NULL row), and whether the row is non-null
template <int TYPE>
__global__ __launch_bounds__(kQBlock) void dq_digest_sample(const void* __restrict__ values,
                                                            const uint32_t* __restrict__ validity, int64_t n, int64_t m,
                                                            unsigned long long* __restrict__ keys,
                                                            unsigned char* __restrict__ ok) {
  const int64_t i = (int64_t)blockIdx.x * kQBlock + threadIdx.x;
  if (i >= m) return;
  const int64_t r = i * (n / m) + (i * (n % m)) / m;  // floor(i n / m) without 128-bit products (m <= 16384)
  uint64_t raw;
  if constexpr (TYPE == DQ_TYPE_I32) raw = (uint32_t)reinterpret_cast<const int32_t*>(values)[r];
  else raw = reinterpret_cast<const uint64_t*>(values)[r];
  const bool valid = validity ? ((validity[r >> 5] >> (r & 31)) & 1u) != 0 : true;
  keys[i] = valid ? order_key<TYPE>(raw) : ~0ull;  // a NULL sorts last (the host keeps the first #valid keys)
  ok[i] = (unsigned char)valid;
}

constexpr int kDRows = 4;                    // rows per thread and iteration (independent searches in flight)

// The splitters' lookup table: the value range [vlo, vlo + (kDCells - 1) / scale] of the finite splitters cut into
// kDCells cells linear in the value (cell 0 also takes every smaller value and -inf, the last cell every larger
// value, +inf and NaN), and first[c] = #{splitters whose cell is < c} (first[kDCells] = kDBuckets - 1).  The cell
// is non-decreasing in the key order, so a key of cell c has first[c] + #{j in [first[c], first[c + 1]) :
// spl[j] <= key} splitters <= it.  Linear in the value, not in the key bits: a double's key bits are close to
// logarithmic in its magnitude, which put hundreds of splitters in the cells of a normal column's bulk.  The
// host evaluates the same cell function (same IEEE operations) on the splitters.
struct DigestCells {
  double vlo, scale;
};

__host__ __device__ __forceinline__ uint32_t digest_cell(double v, DigestCells C) {
  if (!(v - v == 0.0)) return v < 0.0 ? 0u : (uint32_t)(kDCells - 1);  // -inf; +inf or NaN
  const double t = (v - C.vlo) * C.scale;
  return t >= (double)(kDCells - 1) ? (uint32_t)(kDCells - 1) : (t > 0.0 ? (uint32_t)t : 0u);
}

template <int TYPE>
__host__ __device__ __forceinline__ double digest_value(uint64_t raw) {
  if constexpr (TYPE == DQ_TYPE_F64) {
    double d;
    __builtin_memcpy(&d, &raw, 8);
    return d;
  } else if constexpr (TYPE == DQ_TYPE_I64) {
    return (double)(int64_t)raw;
  } else {
    return (double)(int32_t)(uint32_t)raw;
  }
}

// buckets of kDRows keys: the number of splitters <= key (spl: kDBuckets - 1 sorted keys in LDS), narrowed to the
// key's cell and finished by binary lifting inside it -- as many steps as the most crowded cell among the
// thread's keys needs (about 1-2 for a smooth column, 11 when the splitters crowd one cell, e.g. a column of a few
// distinct values); the searches of the thread's keys interleaved step by step.  (The plain 11-step search over
// all splitters: LDS bank conflicts were ~ 3e8 cycles per launch at 1e8 rows, `r4w`.)
__device__ __forceinline__ void digest_buckets(const unsigned long long* spl, const uint16_t* first,
                                               const uint64_t (&key)[kDRows], const uint32_t (&cell)[kDRows],
                                               uint32_t (&pos)[kDRows]) {
  uint32_t end[kDRows], wmax = 0;
#pragma unroll
  for (int u = 0; u < kDRows; ++u) {
    pos[u] = first[cell[u]];
    end[u] = first[cell[u] + 1];
    wmax = max(wmax, end[u] - pos[u]);
  }
  for (uint32_t step = wmax ? (1u << (31 - __builtin_clz(wmax))) : 0u; step != 0; step >>= 1) {
#pragma unroll
    for (int u = 0; u < kDRows; ++u) {
      const uint32_t j = pos[u] + step - 1;
      const unsigned long long v = spl[j < (uint32_t)(kDBuckets - 2) ? j : (uint32_t)(kDBuckets - 2)];
      if (j < end[u] && v <= key[u]) pos[u] += step;
    }
  }
}

// Pass over a chunk: COUNT -- per-bucket key counts into counts[kDCountCopies][kDBuckets]; else the keys of the flagged
// buckets appended to cand[*cursor ...] (order free: sorted next), staged in the workgroup's LDS and flushed
// with one global atomic per kDStage - kQBlock keys (one cursor for the whole launch: a per-wave global atomic
// on it ran 17 ms per 1e8 rows, r4l)
template <int TYPE, bool COUNT>
__global__ __launch_bounds__(kQBlock) void dq_digest_pass(const void* __restrict__ values,
                                                          const uint32_t* __restrict__ validity, int64_t n,
                                                          const unsigned long long* __restrict__ splitters,
                                                          const uint16_t* __restrict__ first_g, DigestCells C,
                                                          unsigned long long* __restrict__ counts,
                                                          const unsigned char* __restrict__ target,
                                                          unsigned long long* __restrict__ cand,
                                                          unsigned long long* __restrict__ cursor,
                                                          unsigned long long cand_cap) {
  __shared__ unsigned long long spl[kDBuckets - 1];
  __shared__ uint16_t first[kDCells + 1];
  __shared__ uint32_t hist[COUNT ? kDBuckets : 1];
  __shared__ uint32_t eqh[COUNT ? kDBuckets : 1];  // keys equal to their bucket's lower splitter
  __shared__ unsigned char tgt[COUNT ? 1 : kDBuckets];
  __shared__ unsigned long long stage[COUNT ? 1 : kDStage];
  __shared__ uint32_t st_n;
  __shared__ unsigned long long st_base;
  if (threadIdx.x == 0) st_n = 0;
  for (int i = threadIdx.x; i < kDBuckets - 1; i += kQBlock) spl[i] = splitters[i];
  for (int i = threadIdx.x; i <= kDCells; i += kQBlock) first[i] = first_g[i];
  if constexpr (COUNT) {
    for (int i = threadIdx.x; i < kDBuckets; i += kQBlock) hist[i] = eqh[i] = 0;
  } else {
    for (int i = threadIdx.x; i < kDBuckets; i += kQBlock) tgt[i] = target[i];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  uint64_t c_and = ~0ull, c_or = 0;  // !COUNT: AND / OR of the thread's candidate keys
  constexpr int kIter = kQBlock * kDRows;  // rows per workgroup and iteration
  // the next iteration's values and validity words are loaded before this iteration's searches (in flight
  // behind them): per 1e8 rows the count pass 0.49 -> 0.23 ms, the compaction pass 0.63 -> 0.35 ms (r4y)
  const int64_t stride = (int64_t)gridDim.x * kIter;
  uint64_t raw_n[kDRows];
  uint32_t vw_n[kDRows];
  auto fetch = [&](int64_t r0) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < kDRows; ++u) {
      const int64_t r = r0 + u * kQBlock + threadIdx.x;
      raw_n[u] = 0;
      vw_n[u] = 0;
      if (r < n) {
        vw_n[u] = validity ? validity[r >> 5] : 0xFFFFFFFFu;
        if constexpr (TYPE == DQ_TYPE_I32) raw_n[u] = (uint32_t)__builtin_nontemporal_load(reinterpret_cast<const int32_t*>(values) + r);
        else raw_n[u] = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(values) + r);
      }
    }
  };
  fetch((int64_t)blockIdx.x * kIter);
  for (int64_t r0 = (int64_t)blockIdx.x * kIter; r0 < n; r0 += stride) {
    bool ok[kDRows];
    uint64_t key[kDRows];
    uint32_t cell[kDRows];
#pragma unroll
    for (int u = 0; u < kDRows; ++u) {
      const int64_t r = r0 + u * kQBlock + threadIdx.x;
      ok[u] = r < n && ((vw_n[u] >> (r & 31)) & 1u);
      key[u] = order_key<TYPE>(raw_n[u]);
      cell[u] = digest_cell(digest_value<TYPE>(raw_n[u]), C);
    }
    if (r0 + stride < n) fetch(r0 + stride);
    uint32_t bk[kDRows];
    digest_buckets(spl, first, key, cell, bk);
    if constexpr (COUNT) {
#pragma unroll
      for (int u = 0; u < kDRows; ++u)
        if (ok[u]) {
          atomicAdd(&hist[bk[u]], 1u);
          if (bk[u] > 0 && key[u] == spl[bk[u] - 1]) atomicAdd(&eqh[bk[u]], 1u);
        }
    } else {
      // (every thread of the workgroup runs the same iterations: the flush below is workgroup-uniform)
#pragma unroll
      for (int u = 0; u < kDRows; ++u) {
        // a key equal to its bucket's lower splitter is known without compaction (a hot value's rows)
        const bool take = ok[u] && tgt[bk[u]] && !(bk[u] > 0 && key[u] == spl[bk[u] - 1]);
        if (take) {
          c_and &= key[u];
          c_or |= key[u];
        }
        const uint64_t bal = __builtin_amdgcn_ballot_w64(take);
        if (bal != 0) {
          const int first = __builtin_ctzll(bal);
          uint32_t pos = 0;
          if (lane == first) pos = atomicAdd(&st_n, (uint32_t)__builtin_popcountll(bal));
          pos = __shfl(pos, first);  // <= kDStage - kIter before this iteration: fits
          if (take) stage[pos + __builtin_popcountll(bal & ((1ull << lane) - 1ull))] = key[u];
        }
      }
      __syncthreads();
      const uint32_t staged = st_n;
      if (staged > (uint32_t)(kDStage - kIter)) {
        if (threadIdx.x == 0) st_base = atomicAdd(cursor, (unsigned long long)staged);
        __syncthreads();
        const unsigned long long b = st_base;
        for (uint32_t i = threadIdx.x; i < staged; i += kQBlock)
          if (b + i < cand_cap) cand[b + i] = stage[i];  // (the host checks the cursor against the count pass)
        __syncthreads();
        if (threadIdx.x == 0) st_n = 0;
        __syncthreads();
      }
    }
  }
  __syncthreads();
  if constexpr (COUNT) {
    for (int i = threadIdx.x; i < kDBuckets; i += kQBlock) {
      if (hist[i]) atomicAdd(&counts[(blockIdx.x % kDCountCopies) * kDBuckets + i], (unsigned long long)hist[i]);
      if (eqh[i])
        atomicAdd(&counts[(kDCountCopies + blockIdx.x % kDCountCopies) * kDBuckets + i], (unsigned long long)eqh[i]);
    }
  } else {
    const uint32_t staged = st_n;
    if (staged > 0) {
      if (threadIdx.x == 0) st_base = atomicAdd(cursor, (unsigned long long)staged);
      __syncthreads();
      const unsigned long long b = st_base;
      for (uint32_t i = threadIdx.x; i < staged; i += kQBlock)
        if (b + i < cand_cap) cand[b + i] = stage[i];
    }
    // the candidates' AND / OR (lanes, waves, then one pair per workgroup into copy blockIdx % kDAndOrCopies of
    // cursor[1 ..]): the sort skips the high bits every candidate shares
    __shared__ unsigned long long w_and[kQBlock / 64], w_or[kQBlock / 64];
    for (int d = 32; d >= 1; d >>= 1) {
      c_and &= __shfl_xor(c_and, d);
      c_or |= __shfl_xor(c_or, d);
    }
    if (lane == 0) {
      w_and[threadIdx.x >> 6] = c_and;
      w_or[threadIdx.x >> 6] = c_or;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int w = 1; w < kQBlock / 64; ++w) {
        c_and &= w_and[w];
        c_or |= w_or[w];
      }
      unsigned long long* const c = cursor + 1 + 2 * (blockIdx.x % kDAndOrCopies);
      if (c_and != ~0ull) atomicAnd(&c[0], (unsigned long long)c_and);
      if (c_or != 0) atomicOr(&c[1], (unsigned long long)c_or);
    }
  }
}

// The cells of the sorted splitters (DigestCells): the finite splitters' value range over kDCells cells, and
// first[c] = #{splitters whose cell is < c}, by the device's own cell function.
DigestCells digest_cells(int32_t type, const std::vector<unsigned long long>& spl, std::vector<uint16_t>& first) {
  double lo = 0.0, hi = 0.0;
  bool any = false;
  for (unsigned long long k : spl) {
    const double v = key_to_double(type, k);
    if (v - v != 0.0) continue;  // +-inf, NaN
    lo = any ? std::min(lo, v) : v;
    hi = any ? std::max(hi, v) : v;
    any = true;
  }
  const double w = hi - lo;
  DigestCells C{lo, (w > 0.0 && w - w == 0.0) ? (double)(kDCells - 1) / w : 0.0};
  if (C.scale - C.scale != 0.0) C.scale = 0.0;
  first.assign((size_t)kDCells + 1, 0);
  // count per cell, then the exclusive prefix
  std::vector<uint32_t> per((size_t)kDCells, 0);
  for (unsigned long long k : spl) ++per[digest_cell(key_to_double(type, k), C)];
  uint32_t run = 0;
  for (int c = 0; c < kDCells; ++c) {
    first[(size_t)c] = (uint16_t)run;
    run += per[(size_t)c];
  }
  first[(size_t)kDCells] = (uint16_t)run;
  return C;
}

// a compaction pass's cursor and its candidates' (AND, OR) copies reset on the stream (no host round trip)
__global__ void dq_digest_cursor_init(unsigned long long* __restrict__ cursor) {
  const int i = threadIdx.x;
  if (i == 0) cursor[0] = 0ull;
  if (i < kDAndOrCopies) {
    cursor[1 + 2 * i] = ~0ull;
    cursor[2 + 2 * i] = 0ull;
  }
}

// out[i] = sorted[idx[i]]
__global__ void dq_digest_gather(const unsigned long long* __restrict__ sorted, const long long* __restrict__ idx,
                                 int64_t m, unsigned long long* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) out[i] = idx[i] >= 0 ? sorted[idx[i]] : 0ull;  // -1: a sample known without compaction
}

// FloatType / ShortType / ByteType columns (ApproxQuantile's isNumeric precondition takes them): widened on the
// device into a scratch column per chunk -- float -> double and short / byte -> int are exact, and the order
// statistic of the widened values is the widened order statistic -- then the F64 / I32 select and digest run
// unchanged.  One extra streaming pass (read 1-4 B, write 4-8 B per row) ahead of passes that read the column
// several times.
// DecimalType columns the same way: each value cast to double as Spark's Decimal.toDouble (correctly rounded,
// dq_decimal.h -- StatefulApproxQuantile's input is Cast(child, DoubleType)), so the F64 passes see what Spark's
// digest sees.
#define DQ_DEC_TABLE static __constant__ const
#include "dq_dec_tables.inc"
#undef DQ_DEC_TABLE
__global__ void widen_column(const void* __restrict__ src, int32_t type, void* __restrict__ dst, int64_t n) {
  const DecTab tab{kDecP10Lo, kDecP10Hi, kDecRcpHi, kDecRcpLo};
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    if (DQ_TYPE_BASE(type) == DQ_TYPE_DECIMAL128) {
      const uint64_t* v = reinterpret_cast<const uint64_t*>(src) + 2 * r;
      reinterpret_cast<double*>(dst)[r] =
          dec_to_double(__builtin_nontemporal_load(v), __builtin_nontemporal_load(v + 1), DQ_DECIMAL_SCALE(type), tab,
                        DQ_DECIMAL_PRECISION(type) <= 18);
    } else if (type == DQ_TYPE_F32) reinterpret_cast<double*>(dst)[r] = (double)__builtin_nontemporal_load(reinterpret_cast<const float*>(src) + r);
    else if (type == DQ_TYPE_I16) reinterpret_cast<int32_t*>(dst)[r] = __builtin_nontemporal_load(reinterpret_cast<const int16_t*>(src) + r);
    else reinterpret_cast<int32_t*>(dst)[r] = __builtin_nontemporal_load(reinterpret_cast<const int8_t*>(src) + r);
  }
}

struct Widened {
  int32_t type = 0;
  std::vector<dq_column_view> views;
  std::vector<void*> bufs;
  hipStream_t stream = nullptr;
  ~Widened() {
    if (!bufs.empty()) (void)hipStreamSynchronize(stream);
    for (void* b : bufs) (void)hipFree(b);
  }
};

bool is_narrow(int32_t type) {
  return type == DQ_TYPE_F32 || type == DQ_TYPE_I16 || type == DQ_TYPE_I8 || (type_valid(type) && is_decimal(type));
}

dq_status widen(int32_t type, const dq_column_view* cols, const int64_t* chunk_rows, int32_t n_chunks, int32_t device,
                hipStream_t stream, Widened& w) {
  QHIP(hipSetDevice(device));
  const bool to_f64 = type == DQ_TYPE_F32 || is_decimal(type);
  w.type = to_f64 ? DQ_TYPE_F64 : DQ_TYPE_I32;
  w.stream = stream;
  const int64_t bytes = to_f64 ? 8 : 4;
  w.views.assign(cols, cols + n_chunks);
  for (int c = 0; c < n_chunks; ++c) {
    const int64_t n = chunk_rows[c];
    if (n == 0) continue;
    void* d = nullptr;
    QHIP(hipMalloc(&d, (size_t)(n * bytes + 16)));
    w.bufs.push_back(d);
    const int grid = (int)std::min<int64_t>(4096, (n + 255) / 256);
    hipLaunchKernelGGL(widen_column, dim3(grid), dim3(256), 0, stream, cols[c].values, type, d, n);
    QHIP(hipGetLastError());
    w.views[c].values = d;
  }
  return DQ_OK;
}

}  // namespace
}  // namespace dq

using namespace dq;

extern "C" {

dq_status dq_approx_quantiles(int32_t type, const dq_column_view* cols, const int64_t* chunk_rows, int32_t n_chunks,
                              const double* quantiles, int32_t n_q, double relative_error, int32_t device,
                              void* hip_stream, double* out, int64_t* count) {
  if (!cols || !chunk_rows || !quantiles || !out || !count || n_chunks < 0)
    return set_error(DQ_E_INVALID, "dq_approx_quantiles: NULL argument");
  if (n_q < 1 || n_q > DQ_MAX_QUANTILES)
    return set_error(DQ_E_INVALID, "dq_approx_quantiles: %d quantiles (1..%d per call)", n_q, DQ_MAX_QUANTILES);
  if (is_narrow(type)) {
    for (int c = 0; c < n_chunks; ++c)
      if (chunk_rows[c] > 0 && !cols[c].values) return set_error(DQ_E_INVALID, "dq_approx_quantiles: chunk %d has no values", c);
    Widened w;
    if (dq_status s = widen(type, cols, chunk_rows, n_chunks, device, reinterpret_cast<hipStream_t>(hip_stream), w)) return s;
    return dq_approx_quantiles(w.type, w.views.data(), chunk_rows, n_chunks, quantiles, n_q, relative_error, device,
                               hip_stream, out, count);
  }
  if (type != DQ_TYPE_F64 && type != DQ_TYPE_I64 && type != DQ_TYPE_I32)
    return set_error(DQ_E_TYPE, "dq_approx_quantiles: column type %d is not numeric", type);
  // ApproxQuantile.scala:46-56 PARAM_CHECKS (MetricCalculationException messages)
  for (int q = 0; q < n_q; ++q)
    if (!(quantiles[q] >= 0.0 && quantiles[q] <= 1.0))
      return set_error(DQ_E_INVALID,
                       "Quantile parameter must be in the closed interval [0, 1]. Currently, the value is: %g!",
                       quantiles[q]);
  if (!(relative_error >= 0.0 && relative_error <= 1.0))
    return set_error(DQ_E_INVALID,
                     "Relative error parameter must be in the closed interval [0, 1]. Currently, the value is: %g!",
                     relative_error);
  for (int c = 0; c < n_chunks; ++c) {
    if (chunk_rows[c] < 0 || chunk_rows[c] > ((int64_t)1 << 40))
      return set_error(DQ_E_INVALID, "dq_approx_quantiles: chunk %d has %lld rows", c, (long long)chunk_rows[c]);
    if (chunk_rows[c] > 0 && !cols[c].values)
      return set_error(DQ_E_INVALID, "dq_approx_quantiles: chunk %d has no values", c);
    if (cols[c].reserved != 0) return set_error(DQ_E_INVALID, "dq_approx_quantiles: reserved field must be 0");
  }
  QHIP(hipSetDevice(device));
  hipStream_t stream = reinterpret_cast<hipStream_t>(hip_stream);
  const size_t hist_bytes = (size_t)n_q * kQBins * sizeof(unsigned long long);
  DevHist dh;
  QHIP(hipMalloc(&dh.p, hist_bytes));
  std::vector<unsigned long long> h((size_t)n_q * kQBins);
  QSelect sel{};
  std::vector<int64_t> rank(n_q, 0);  // 1-based rank still to find inside the selected prefix
  int64_t n = 0;
  // candidate lists: once every quantile's remaining candidates (the rows matching its selected
  // prefix) fit in n / 16 keys in total, the next column pass appends them, and the passes after it
  // read only those keys instead of the column
  DevHist cand, cand_cnt;
  bool compacted = false;
  std::vector<int64_t> remaining(n_q, 0), cand_off(n_q, 0), cand_len(n_q, 0);
  std::vector<int> hrow(n_q);  // histogram row of quantile q in this pass
  // pass 0 also leaves the AND / OR of the non-null keys: a later pass whose digit bits are equal in every key
  // (a small-range integer column's high digits) is skipped -- its digit is known and no rank moves
  DevHist andor_buf;
  QHIP(hipMalloc(&andor_buf.p, 16 * kQAndOrCopies));
  unsigned long long* const d_andor = andor_buf.p;
  unsigned long long andor0[2 * kQAndOrCopies];
  for (int i = 0; i < kQAndOrCopies; ++i) {
    andor0[2 * i] = ~0ull;
    andor0[2 * i + 1] = 0ull;
  }
  QHIP(hipMemcpyAsync(d_andor, andor0, sizeof(andor0), hipMemcpyHostToDevice, stream));
  uint64_t same_bits = 0;  // bits equal in every non-null key (known after pass 0)
  uint64_t or_bits = 0;
  for (int pass = 0; pass < kQPasses; ++pass) {
    if (pass > 0) {
      const uint64_t dm = ((1ull << kQWidth[pass]) - 1ull) << kQShift[pass];
      if ((same_bits & dm) == dm) {
        for (int q = 0; q < n_q; ++q) {
          sel.prefix[q] |= or_bits & dm;
          sel.pmask[q] |= dm;
        }
        continue;
      }
    }
    QHIP(hipMemsetAsync(dh.p, 0, hist_bytes, stream));
    for (int q = 0; q < n_q; ++q) hrow[q] = q;
    const uint32_t dmask32 = (1u << kQWidth[pass]) - 1u;
    if (compacted) {
      for (int q = 0; q < n_q; ++q) {
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(1024, (cand_len[q] + kQBlock * 8 - 1) / (kQBlock * 8)));
        hipLaunchKernelGGL(dq_quantile_cand_hist, dim3(grid), dim3(kQBlock), 0, stream, cand.p + cand_off[q],
                           (int64_t)cand_len[q], kQShift[pass], dmask32, sel.prefix[q], sel.pmask[q],
                           dh.p + (size_t)q * kQBins);
        QHIP(hipGetLastError());
      }
    } else {
      // quantiles that share a selected prefix (all of them in pass 0) share one histogram row and one
      // candidate list: the column pass does each distinct (prefix, digit) count once
      QSelect usel{};
      int nu = 0;
      std::vector<int64_t> uremaining;
      for (int q = 0; q < n_q; ++q) {
        int u = 0;
        while (u < nu && !(usel.prefix[u] == sel.prefix[q] && usel.pmask[u] == sel.pmask[q])) ++u;
        if (u == nu) {
          usel.prefix[nu] = sel.prefix[q];
          usel.pmask[nu] = sel.pmask[q];
          uremaining.push_back(remaining[q]);
          ++nu;
        }
        hrow[q] = u;
      }
      bool append = false;
      if (pass > 0 && pass < kQPasses - 1) {
        int64_t total = 0;
        for (int u = 0; u < nu; ++u) total += uremaining[u];
        if (total <= std::max<int64_t>(n / 16, 1 << 16)) {
          QHIP(hipMalloc(&cand.p, (size_t)std::max<int64_t>(total, 1) * 8));
          QHIP(hipMalloc(&cand_cnt.p, DQ_MAX_QUANTILES * 8));
          QHIP(hipMemsetAsync(cand_cnt.p, 0, DQ_MAX_QUANTILES * 8, stream));
          std::vector<int64_t> uoff(nu, 0);
          int64_t off = 0;
          for (int u = 0; u < nu; ++u) {
            uoff[u] = off;
            usel.cand[u] = cand.p + off;
            off += uremaining[u];
          }
          for (int q = 0; q < n_q; ++q) {
            cand_off[q] = uoff[hrow[q]];
            cand_len[q] = uremaining[hrow[q]];
          }
          usel.cand_cnt = cand_cnt.p;
          append = true;
        }
      }
      for (int c = 0; c < n_chunks; ++c) {
        const int64_t rows = chunk_rows[c];
        if (rows == 0) continue;
        const auto* val = reinterpret_cast<const uint32_t*>(cols[c].validity);
        const size_t lds = (size_t)nu * kQBins * sizeof(uint32_t) +
                           (append ? (size_t)nu * kQStage * 8 + (size_t)2 * nu * sizeof(uint32_t) : 0);
        const bool aligned = (reinterpret_cast<uintptr_t>(cols[c].values) & 15u) == 0;
        const int64_t rows_per_vec = aligned ? (type == DQ_TYPE_I32 ? 4 : 2) : 1;
        const int64_t per_block = (int64_t)kQBlock * kQUnroll * rows_per_vec;
        const int grid = (int)std::min<int64_t>(4096, (rows + per_block - 1) / per_block);
        const void* vals = cols[c].values;
        const int sh = kQShift[pass];
        unsigned long long* const ao_p = pass == 0 ? d_andor : nullptr;
        if (type == DQ_TYPE_F64) {
          if (aligned) launch_hist<DQ_TYPE_F64, 2>(append, grid, lds, stream, vals, val, rows, sh, dmask32, nu, usel, dh.p, ao_p);
          else launch_hist<DQ_TYPE_F64, 1>(append, grid, lds, stream, vals, val, rows, sh, dmask32, nu, usel, dh.p, ao_p);
        } else if (type == DQ_TYPE_I64) {
          if (aligned) launch_hist<DQ_TYPE_I64, 2>(append, grid, lds, stream, vals, val, rows, sh, dmask32, nu, usel, dh.p, ao_p);
          else launch_hist<DQ_TYPE_I64, 1>(append, grid, lds, stream, vals, val, rows, sh, dmask32, nu, usel, dh.p, ao_p);
        } else {
          if (aligned) launch_hist<DQ_TYPE_I32, 4>(append, grid, lds, stream, vals, val, rows, sh, dmask32, nu, usel, dh.p, ao_p);
          else launch_hist<DQ_TYPE_I32, 1>(append, grid, lds, stream, vals, val, rows, sh, dmask32, nu, usel, dh.p, ao_p);
        }
        QHIP(hipGetLastError());
      }
      if (append) {
        std::vector<unsigned long long> got(DQ_MAX_QUANTILES);
        QHIP(hipMemcpyAsync(got.data(), cand_cnt.p, DQ_MAX_QUANTILES * 8, hipMemcpyDeviceToHost, stream));
        QHIP(hipStreamSynchronize(stream));
        for (int u = 0; u < nu; ++u)
          if ((int64_t)got[u] != uremaining[u])
            return set_error(DQ_E_HIP, "dq_approx_quantiles: %llu candidates for prefix %d, expected %lld (data changed?)",
                             got[u], u, (long long)uremaining[u]);
        compacted = true;
      }
    }
    QHIP(hipMemcpyAsync(h.data(), dh.p, hist_bytes, hipMemcpyDeviceToHost, stream));
    QHIP(hipStreamSynchronize(stream));
    if (pass == 0) {
      unsigned long long ao[2 * kQAndOrCopies];
      QHIP(hipMemcpyAsync(ao, d_andor, sizeof(ao), hipMemcpyDeviceToHost, stream));
      QHIP(hipStreamSynchronize(stream));
      uint64_t k_and = ~0ull;
      or_bits = 0;
      for (int i = 0; i < kQAndOrCopies; ++i) {
        k_and &= ao[2 * i];
        or_bits |= ao[2 * i + 1];
      }
      same_bits = ~(k_and ^ or_bits);
      for (int b = 0; b < kQBins; ++b) n += (int64_t)h[b];  // every non-null row matches the empty prefix (row 0)
      *count = n;
      if (n == 0) return DQ_OK;  // all values NULL: no digest (fromAggregationResult -> None)
      for (int q = 0; q < n_q; ++q) {
        // QuantileSummaries.query (Spark 2.2): the two ends answer min / max, otherwise rank ceil(q n)
        const double qq = quantiles[q];
        int64_t r;
        if (qq <= relative_error) r = 1;
        else if (qq >= 1.0 - relative_error) r = n;
        else r = (int64_t)std::ceil(qq * (double)n);
        rank[q] = std::min<int64_t>(n, std::max<int64_t>(1, r));
      }
    }
    const uint64_t dmask = (1ull << kQWidth[pass]) - 1ull;
    for (int q = 0; q < n_q; ++q) {
      const unsigned long long* hq = h.data() + (size_t)hrow[q] * kQBins;
      int64_t cum = 0;
      int b = 0;
      for (; b < (int)dmask; ++b) {
        if (cum + (int64_t)hq[b] >= rank[q]) break;
        cum += (int64_t)hq[b];
      }
      if (cum + (int64_t)hq[b] < rank[q])
        return set_error(DQ_E_HIP, "dq_approx_quantiles: histogram of pass %d lost rows (data changed?)", pass);
      rank[q] -= cum;
      remaining[q] = (int64_t)hq[b];
      sel.prefix[q] |= (uint64_t)b << kQShift[pass];
      sel.pmask[q] |= dmask << kQShift[pass];
    }
  }
  for (int q = 0; q < n_q; ++q) out[q] = key_to_double(type, sel.prefix[q]);
  return DQ_OK;
}

dq_status dq_quantile_digest(int32_t type, const dq_column_view* cols, const int64_t* chunk_rows, int32_t n_chunks,
                             double relative_error, int32_t device, void* hip_stream, double* values, int64_t* ranks,
                             int64_t cap, int64_t* n_samples, int64_t* count) {
  if (!cols || !chunk_rows || !n_samples || !count || n_chunks < 0 || cap < 0 || (cap > 0 && (!values || !ranks)))
    return set_error(DQ_E_INVALID, "dq_quantile_digest: NULL argument");
  if (is_narrow(type)) {
    for (int c = 0; c < n_chunks; ++c)
      if (chunk_rows[c] > 0 && !cols[c].values) return set_error(DQ_E_INVALID, "dq_quantile_digest: chunk %d has no values", c);
    Widened w;
    if (dq_status s = widen(type, cols, chunk_rows, n_chunks, device, reinterpret_cast<hipStream_t>(hip_stream), w)) return s;
    return dq_quantile_digest(w.type, w.views.data(), chunk_rows, n_chunks, relative_error, device, hip_stream, values,
                              ranks, cap, n_samples, count);
  }
  if (type != DQ_TYPE_F64 && type != DQ_TYPE_I64 && type != DQ_TYPE_I32)
    return set_error(DQ_E_TYPE, "dq_quantile_digest: column type %d is not numeric", type);
  if (!(relative_error >= 0.0 && relative_error <= 1.0))
    return set_error(DQ_E_INVALID,
                     "Relative error parameter must be in the closed interval [0, 1]. Currently, the value is: %g!",
                     relative_error);
  int64_t total = 0;
  for (int c = 0; c < n_chunks; ++c) {
    if (chunk_rows[c] < 0 || chunk_rows[c] > ((int64_t)1 << 40))
      return set_error(DQ_E_INVALID, "dq_quantile_digest: chunk %d has %lld rows", c, (long long)chunk_rows[c]);
    if (chunk_rows[c] > 0 && !cols[c].values)
      return set_error(DQ_E_INVALID, "dq_quantile_digest: chunk %d has no values", c);
    if (cols[c].reserved != 0) return set_error(DQ_E_INVALID, "dq_quantile_digest: reserved field must be 0");
    total += chunk_rows[c];
  }
  *n_samples = 0;
  *count = 0;
  QHIP(hipSetDevice(device));
  hipStream_t stream = reinterpret_cast<hipStream_t>(hip_stream);
  if (total == 0) return DQ_OK;
  auto for_chunks = [&](auto&& launch) -> dq_status {
    for (int c = 0; c < n_chunks; ++c) {
      const int64_t rows = chunk_rows[c];
      if (rows == 0) continue;
      const int grid = (int)std::min<int64_t>(4096, (rows + kQBlock * kDRows - 1) / (kQBlock * kDRows));
      auto go = [&](auto kern) { launch(kern, grid, c, rows); };
      if (type == DQ_TYPE_F64) go(std::integral_constant<int, DQ_TYPE_F64>{});
      else if (type == DQ_TYPE_I64) go(std::integral_constant<int, DQ_TYPE_I64>{});
      else go(std::integral_constant<int, DQ_TYPE_I32>{});
      QHIP(hipGetLastError());
    }
    return DQ_OK;
  };
  // 1. splitters from an evenly spaced sample of every chunk's rows (nulls dropped on the host)
  std::vector<int64_t> s_off((size_t)n_chunks + 1, 0);
  for (int c = 0; c < n_chunks; ++c) {
    const int64_t want = chunk_rows[c] == 0 ? 0 : std::max<int64_t>(1, (int64_t)((double)kDSample * chunk_rows[c] / total));
    s_off[(size_t)c + 1] = s_off[(size_t)c] + std::min<int64_t>(want, chunk_rows[c]);
  }
  const int64_t ns_all = s_off[(size_t)n_chunks];
  // one scratch block: sample keys | splitters | counts (per bucket, then keys equal to the bucket's lower
  // splitter) | cursor | sample flags | bucket flags | sorted sample keys | the sample sort's temp
  hipMemPool_t pool = nullptr;
  QHIP(scratch_pool(device, &pool));
  StreamTmp small;
  const size_t o_spl = (size_t)ns_all * 8, o_cnt = o_spl + (size_t)(kDBuckets - 1) * 8,
               o_cur = o_cnt + (size_t)2 * kDCountCopies * kDBuckets * 8,
               o_first = o_cur + 8 + (size_t)kDAndOrCopies * 16,
               o_ok = o_first + ((size_t)(kDCells + 1) * 2 + 7) / 8 * 8, o_tgt = o_ok + (size_t)ns_all,
               o_ssorted = (o_tgt + kDBuckets + 255) & ~(size_t)255, o_stmp = o_ssorted + ((size_t)ns_all * 8 + 255) / 256 * 256;
  const size_t stb = prim::sort_temp_bytes(ns_all, 0);
  QHIP(small.alloc(o_stmp + stb, pool, stream));
  char* const sb = static_cast<char*>(small.p);
  uint16_t* const d_first = reinterpret_cast<uint16_t*>(sb + o_first);
  struct {
    unsigned long long* p;
  } d_sample{reinterpret_cast<unsigned long long*>(sb)}, d_spl{reinterpret_cast<unsigned long long*>(sb + o_spl)},
      d_counts{reinterpret_cast<unsigned long long*>(sb + o_cnt)},
      d_cursor{reinterpret_cast<unsigned long long*>(sb + o_cur)};
  struct {
    unsigned char* p;
  } d_ok{reinterpret_cast<unsigned char*>(sb + o_ok)}, d_target{reinterpret_cast<unsigned char*>(sb + o_tgt)};
  if (dq_status st = for_chunks([&](auto tk, int grid, int c, int64_t rows) {
        (void)grid;
        const int64_t mc = s_off[(size_t)c + 1] - s_off[(size_t)c];
        hipLaunchKernelGGL((dq_digest_sample<decltype(tk)::value>), dim3((unsigned)((mc + kQBlock - 1) / kQBlock)),
                           dim3(kQBlock), 0, stream, cols[c].values, reinterpret_cast<const uint32_t*>(cols[c].validity),
                           rows, mc, d_sample.p + s_off[(size_t)c], d_ok.p + s_off[(size_t)c]);
      }))
    return st;
  // the sample sorted on the device (NULLs last; a host std::sort of 16384 keys took ~0.6-1 ms per digest, r6dg)
  unsigned long long* const d_ssorted = reinterpret_cast<unsigned long long*>(sb + o_ssorted);
  QHIP(prim::sort_pairs(reinterpret_cast<const uint64_t*>(d_sample.p), reinterpret_cast<uint64_t*>(d_ssorted), nullptr,
                        nullptr, 0, ns_all, 0, 64, false, sb + o_stmp, stb, stream));
  std::vector<unsigned long long> samp((size_t)ns_all);
  std::vector<unsigned char> sok((size_t)ns_all);
  QHIP(hipMemcpyAsync(samp.data(), d_ssorted, (size_t)ns_all * 8, hipMemcpyDeviceToHost, stream));
  QHIP(hipMemcpyAsync(sok.data(), d_ok.p, (size_t)ns_all, hipMemcpyDeviceToHost, stream));
  QHIP(hipStreamSynchronize(stream));
  size_t nv = 0;
  for (unsigned char f : sok) nv += f;
  samp.resize(nv);  // the valid keys in order: every NULL's ~0 is at or past position nv
  std::vector<unsigned long long> spl(kDBuckets - 1, ~0ull);  // no sample: one bucket holds every key
  for (int k = 1; k < kDBuckets && nv > 0; ++k) spl[(size_t)k - 1] = samp[(size_t)k * nv / kDBuckets];
  QHIP(hipMemcpyAsync(d_spl.p, spl.data(), (size_t)(kDBuckets - 1) * 8, hipMemcpyHostToDevice, stream));
  std::vector<uint16_t> first;
  const DigestCells C = digest_cells(type, spl, first);
  QHIP(hipMemcpyAsync(d_first, first.data(), first.size() * 2, hipMemcpyHostToDevice, stream));
  QHIP(hipMemsetAsync(d_counts.p, 0, (size_t)2 * kDCountCopies * kDBuckets * 8, stream));
  // 2. per-bucket counts (and of each bucket's keys equal to its lower splitter)
  if (dq_status st = for_chunks([&](auto tk, int grid, int c, int64_t rows) {
        hipLaunchKernelGGL((dq_digest_pass<decltype(tk)::value, true>), dim3(grid), dim3(kQBlock), 0, stream,
                           cols[c].values, reinterpret_cast<const uint32_t*>(cols[c].validity), rows, d_spl.p, d_first,
                           C, d_counts.p, nullptr, nullptr, nullptr, 0ull);
      }))
    return st;
  std::vector<unsigned long long> cnt_copies((size_t)2 * kDCountCopies * kDBuckets), cnt((size_t)kDBuckets, 0),
      eq((size_t)kDBuckets, 0);
  QHIP(hipMemcpyAsync(cnt_copies.data(), d_counts.p, cnt_copies.size() * 8, hipMemcpyDeviceToHost, stream));
  QHIP(hipStreamSynchronize(stream));
  for (size_t i = 0; i < (size_t)kDCountCopies * kDBuckets; ++i) {
    cnt[i % kDBuckets] += cnt_copies[i];
    eq[i % kDBuckets] += cnt_copies[(size_t)kDCountCopies * kDBuckets + i];
  }
  int64_t n = 0;
  for (unsigned long long x : cnt) n += (int64_t)x;
  *count = n;
  if (n == 0) return DQ_OK;  // all values NULL: no digest
  // the digest's sample ranks (deequ_amd/quantiles.py digest_ranks): 1, 1 + s, ..., n, s = max(1, floor(2 e n))
  const int64_t s = std::max<int64_t>(1, (int64_t)std::floor(2.0 * relative_error * (double)n));
  const int64_t m = (n - 1) / s + 1 + ((n - 1) % s != 0 ? 1 : 0);
  *n_samples = m;
  if (m > cap) return set_error(DQ_E_INVALID, "dq_quantile_digest: %lld samples, room for %lld", (long long)m, (long long)cap);
  // 3. the bucket of every sample rank.  Bucket b holds the keys in [spl[b - 1], spl[b]); its first eq[b] ranks are
  // spl[b - 1] itself (known: no compaction), the others are candidates -- its keys above spl[b - 1]
  std::vector<int64_t> before((size_t)kDBuckets + 1, 0);
  for (int b = 0; b < kDBuckets; ++b) before[(size_t)b + 1] = before[(size_t)b] + (int64_t)cnt[(size_t)b];
  std::vector<unsigned char> need((size_t)kDBuckets, 0);
  std::vector<int64_t> rank((size_t)m);
  std::vector<int> rb((size_t)m);
  std::vector<unsigned long long> key_of((size_t)m, 0);
  std::vector<unsigned char> known((size_t)m, 0);
  for (int64_t i = 0, b = 0; i < m; ++i) {
    rank[(size_t)i] = i == m - 1 ? n : 1 + i * s;
    while (before[(size_t)b + 1] < rank[(size_t)i]) ++b;  // ranks ascend: bucket b holds ranks (before[b], before[b + 1]]
    rb[(size_t)i] = (int)b;
    if (rank[(size_t)i] - 1 - before[(size_t)b] < (int64_t)eq[(size_t)b]) {
      known[(size_t)i] = 1;
      key_of[(size_t)i] = spl[(size_t)b - 1];  // (eq[0] == 0: b > 0 here)
    } else {
      need[(size_t)b] = 1;
    }
  }
  // the flagged buckets in key order, in batches of at most `budget` candidates (one compaction pass + one sort
  // each): scratch stays bounded whatever the relative error (every bucket flagged when m > kDBuckets) or the skew
  int64_t budget = kDCandBudget;
  if (const char* e = std::getenv("DQ_DIGEST_CAND_BUDGET"))  // test knob: exercise the batching at small sizes
    budget = std::max<int64_t>(1, std::atoll(e));
  std::vector<std::pair<int, int>> batches;  // [first bucket, end bucket)
  int64_t batch_max = 0;
  {
    int b0 = -1;
    int64_t acc = 0;
    for (int b = 0; b < kDBuckets; ++b) {
      if (!need[(size_t)b]) continue;
      const int64_t cb = (int64_t)(cnt[(size_t)b] - eq[(size_t)b]);
      if (cb > budget || cb > (int64_t)0x7FFFFFFF)
        return set_error(DQ_E_UNSUPPORTED, "dq_quantile_digest: %lld candidate values in one bucket (budget %lld)",
                         (long long)cb, (long long)budget);
      if (b0 >= 0 && acc + cb > budget) {
        batches.push_back({b0, b});
        batch_max = std::max(batch_max, acc);
        b0 = -1;
        acc = 0;
      }
      if (b0 < 0) b0 = b;
      acc += cb;
    }
    if (b0 >= 0) {
      batches.push_back({b0, kDBuckets});
      batch_max = std::max(batch_max, acc);
    }
  }
  // second scratch block: candidates | sorted candidates | sample indices | gathered keys | radix-sort temp
  const size_t tb = prim::sort_temp_bytes(std::max<int64_t>(1, batch_max), 0);
  StreamTmp big;
  const size_t o_sorted = (size_t)batch_max * 8, o_idx = o_sorted + (size_t)batch_max * 8,
               o_got = o_idx + (size_t)m * 8, o_tmp = (o_got + (size_t)m * 8 + 255) & ~(size_t)255;
  QHIP(big.alloc(o_tmp + tb, pool, stream));
  char* const bb = static_cast<char*>(big.p);
  unsigned long long* const cand = reinterpret_cast<unsigned long long*>(bb);
  unsigned long long* const sorted = reinterpret_cast<unsigned long long*>(bb + o_sorted);
  long long* const d_idx = reinterpret_cast<long long*>(bb + o_idx);
  unsigned long long* const d_got = reinterpret_cast<unsigned long long*>(bb + o_got);
  std::vector<unsigned char> tgt((size_t)kDBuckets);
  std::vector<long long> idx;
  std::vector<unsigned long long> got((size_t)m);
  size_t si = 0;  // next sample (ranks ascend with the buckets)
  for (const auto& bt : batches) {
    std::fill(tgt.begin(), tgt.end(), 0);
    std::vector<int64_t> cand_before((size_t)kDBuckets + 1, 0);  // candidates of this batch's buckets before b
    int64_t nc = 0;
    for (int b = bt.first; b < bt.second; ++b) {
      cand_before[(size_t)b] = nc;
      if (need[(size_t)b]) {
        tgt[(size_t)b] = 1;
        nc += (int64_t)(cnt[(size_t)b] - eq[(size_t)b]);
      }
    }
    QHIP(hipMemcpyAsync(d_target.p, tgt.data(), (size_t)kDBuckets, hipMemcpyHostToDevice, stream));
    hipLaunchKernelGGL(dq_digest_cursor_init, dim3(1), dim3(64), 0, stream, d_cursor.p);
    QHIP(hipGetLastError());
    if (dq_status st = for_chunks([&](auto tk, int grid, int c, int64_t rows) {
          hipLaunchKernelGGL((dq_digest_pass<decltype(tk)::value, false>), dim3(grid), dim3(kQBlock), 0, stream,
                             cols[c].values, reinterpret_cast<const uint32_t*>(cols[c].validity), rows, d_spl.p,
                             d_first, C, nullptr, d_target.p, cand, d_cursor.p, (unsigned long long)nc);
        }))
      return st;
    // the candidates agree above their highest differing bit: sorting the bits below gives the full order
    unsigned long long cur[1 + 2 * kDAndOrCopies];
    QHIP(hipMemcpyAsync(cur, d_cursor.p, sizeof(cur), hipMemcpyDeviceToHost, stream));
    QHIP(hipStreamSynchronize(stream));
    if ((int64_t)cur[0] != nc)
      return set_error(DQ_E_HIP, "dq_quantile_digest: %llu candidates, the count pass expected %lld (data changed?)",
                       cur[0], (long long)nc);
    uint64_t c_and = ~0ull, c_or = 0;
    for (int i = 0; i < kDAndOrCopies; ++i) {
      c_and &= cur[1 + 2 * i];
      c_or |= cur[2 + 2 * i];
    }
    const int end_bit = (c_and ^ c_or) ? 64 - __builtin_clzll(c_and ^ c_or) : 1;
    if (nc > 0)
      QHIP(prim::sort_pairs(reinterpret_cast<const uint64_t*>(cand), reinterpret_cast<uint64_t*>(sorted), nullptr, nullptr,
                            0, nc, 0, end_bit, false, bb + o_tmp, tb, stream));
    // 4. sample i = the sorted candidate at (its rank within its bucket, past the bucket's eq keys) + (the batch's
    // candidates of the buckets before)
    idx.clear();
    const size_t s0 = si;
    for (; si < (size_t)m && rb[si] < bt.second; ++si) {
      const int b = rb[si];
      idx.push_back(known[si] ? -1
                              : (long long)(rank[si] - 1 - before[(size_t)b] - (int64_t)eq[(size_t)b] + cand_before[(size_t)b]));
    }
    const int64_t mb = (int64_t)idx.size();
    if (mb > 0) {
      QHIP(hipMemcpyAsync(d_idx, idx.data(), (size_t)mb * 8, hipMemcpyHostToDevice, stream));
      hipLaunchKernelGGL(dq_digest_gather, dim3((unsigned)((mb + 255) / 256)), dim3(256), 0, stream, sorted, d_idx, mb,
                         d_got);
      QHIP(hipGetLastError());
      QHIP(hipMemcpyAsync(got.data() + s0, d_got, (size_t)mb * 8, hipMemcpyDeviceToHost, stream));
      QHIP(hipStreamSynchronize(stream));
    }
  }
  for (int64_t i = 0; i < m; ++i) {
    values[i] = key_to_double(type, known[(size_t)i] || si <= (size_t)i ? key_of[(size_t)i] : got[(size_t)i]);
    ranks[i] = rank[(size_t)i];
  }
  return DQ_OK;
}

}  // extern "C"
