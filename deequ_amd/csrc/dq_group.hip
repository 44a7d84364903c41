// dq_group.hip -- frequencies of the grouping analyzers on the GPU (sort-based group-by count).
//
// Reference: FrequencyBasedAnalyzer.computeFrequencies (analyzers/GroupingAnalyzers.scala:44-82):
//   SELECT cols, COUNT(*) FROM data WHERE col_1 IS NOT NULL AND ... GROUP BY cols
// plus numRows = data.count(), and the metrics of Uniqueness / Distinctness / CountDistinct /
// Entropy / UniqueValueRatio, which only need the multiset of group counts (Uniqueness.scala:27-29,
// Distinctness.scala:29-31, CountDistinct.scala:25-31, Entropy.scala:29-41, UniqueValueRatio.scala:25-36).
// FrequenciesAndNumRows.sum (GroupingAnalyzers.scala:118-138) = outer join adding counts.
//
// Layout: every row whose grouping columns are all non-null yields one 64-bit key.  A single 8-byte /
// 4-byte numeric column is its own exact key (f64: NaN canonicalised as Spark's UnsafeRow.setDouble
// does; -0.0 and 0.0 stay distinct groups in Spark 2.2).  Otherwise (strings, several columns) the key
// is a 64-bit hash of the tuple, the rows ride along the sort, and every pair of neighbours with equal
// keys is compared exactly: a collision between distinct tuples is reported (DQ_E_UNSUPPORTED), never
// merged silently.  Keys are radix-sorted and run-length encoded into (key, count) groups by dq_prim.hip's
// hand-written kernels; the summary is a fixed-order two-level reduction, so results are deterministic.  A hashed table also
// keeps a second, independently seeded 64-bit hash per group (its representative row's tuple), so that
// dq_freq_merge -- which no longer has the rows -- detects two distinct tuples whose first hashes collide
// (equal first hash, different second hash: DQ_E_UNSUPPORTED) instead of adding their counts.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "dq_device.h"
#include "dq_hash.h"
#include "dq_internal.h"
#include "dq_prim.h"

namespace dq {
namespace {

constexpr int kMaxGroupCols = 8;
constexpr int kMaxGroupChunks = 4096;
constexpr int kRowBits = 40;  // row id = chunk << 40 | row

struct GroupCols {
  const void* values[kMaxGroupCols];
  const uint32_t* validity[kMaxGroupCols];
  const void* offsets[kMaxGroupCols];
  int32_t type[kMaxGroupCols];
  int32_t n_cols;
  uint64_t key_mask;  // applied to the primary tuple hash: ~0, or fewer bits from DQ_TEST_GROUP_HASH_MASK (tests)
};

constexpr uint64_t kSeed2 = 0x9E3779B97F4A7C15ull;  // seed of the second (verification) tuple hash

__device__ __forceinline__ bool row_valid(const GroupCols& g, int64_t r) {
  for (int c = 0; c < g.n_cols; ++c)
    if (g.validity[c] && !((g.validity[c][r >> 5] >> (r & 31)) & 1u)) return false;
  return true;
}

__device__ __forceinline__ uint64_t canon_f64(uint64_t bits) {
  const uint64_t mag = bits & 0x7FFFFFFFFFFFFFFFull;
  return mag > 0x7FF0000000000000ull ? 0x7FF8000000000000ull : bits;  // any NaN -> Double.NaN
}

// the grouping key of a fixed-width value: its exact bits (UnsafeRow's binary equality: NaN canonical, -0.0 and
// 0.0 distinct), integers sign-extended, a boolean 0 / 1
__device__ __forceinline__ uint64_t value_bits(const GroupCols& g, int c, int64_t r) {
  switch (g.type[c]) {
    case DQ_TYPE_F64: return canon_f64(reinterpret_cast<const uint64_t*>(g.values[c])[r]);
    case DQ_TYPE_I64: case DQ_TYPE_TIMESTAMP: return reinterpret_cast<const uint64_t*>(g.values[c])[r];
    case DQ_TYPE_F32: {
      const uint32_t b = reinterpret_cast<const uint32_t*>(g.values[c])[r];
      return (b & 0x7FFFFFFFu) > 0x7F800000u ? 0x7FC00000ull : (uint64_t)b;  // any NaN -> Float.NaN
    }
    case DQ_TYPE_I16: return (uint64_t)(int64_t)reinterpret_cast<const int16_t*>(g.values[c])[r];
    case DQ_TYPE_I8: return (uint64_t)(int64_t)reinterpret_cast<const int8_t*>(g.values[c])[r];
    case DQ_TYPE_BOOL: return (reinterpret_cast<const uint32_t*>(g.values[c])[r >> 5] >> (r & 31)) & 1u;
    default: return (uint64_t)(int64_t)reinterpret_cast<const int32_t*>(g.values[c])[r];  // IntegerType, DateType
  }
}

// a DecimalType column: grouped (like strings) by a hash of its 16-byte unscaled value, checked word by word
__device__ __forceinline__ bool is_dec(int32_t t) { return DQ_TYPE_BASE(t) == DQ_TYPE_DECIMAL128; }
__device__ __forceinline__ const uint64_t* dec_at(const GroupCols& g, int c, int64_t r) {
  return reinterpret_cast<const uint64_t*>(g.values[c]) + 2 * r;
}

__device__ __forceinline__ void str_of(const GroupCols& g, int c, int64_t r, const uint8_t*& p, int64_t& len) {
  int64_t o0, o1;
  if (g.type[c] == DQ_TYPE_LARGE_UTF8) {
    o0 = reinterpret_cast<const int64_t*>(g.offsets[c])[r];
    o1 = reinterpret_cast<const int64_t*>(g.offsets[c])[r + 1];
  } else {
    o0 = reinterpret_cast<const int32_t*>(g.offsets[c])[r];
    o1 = reinterpret_cast<const int32_t*>(g.offsets[c])[r + 1];
  }
  p = reinterpret_cast<const uint8_t*>(g.values[c]) + o0;
  len = o1 - o0;
}

__device__ __forceinline__ uint64_t mix8(uint64_t h, uint64_t k) {
  return mul_add_c(rotl64(h ^ mul_add_c(k, XP2, 0), 27), XP1, XP4);
}

// 64-bit hash of the row's tuple (columns in order; strings by bytes and length)
__device__ uint64_t tuple_hash(const GroupCols& g, int64_t r, uint64_t seed = kSeed) {
  uint64_t h = seed + XP5;
  for (int c = 0; c < g.n_cols; ++c) {
    if (g.type[c] == DQ_TYPE_UTF8 || g.type[c] == DQ_TYPE_LARGE_UTF8) {
      const uint8_t* p;
      int64_t len;
      str_of(g, c, r, p, len);
      // little-endian words by (unaligned) 8- / 4-byte loads -- the same k as assembling the bytes one by one
      typedef uint64_t u64u __attribute__((aligned(1)));
      typedef uint32_t u32u __attribute__((aligned(1)));
      int64_t i = 0;
      for (; i + 8 <= len; i += 8) h = mix8(h, *reinterpret_cast<const u64u*>(p + i));
      uint64_t k = 0;
      int b = 0;
      if (i + 4 <= len) {
        k = *reinterpret_cast<const u32u*>(p + i);
        b = 4;
      }
      for (; i + b < len; ++b) k |= (uint64_t)p[i + b] << (8 * b);
      h = mix8(h, k ^ ((uint64_t)len << 56) ^ 0xA5);
    } else if (is_dec(g.type[c])) {
      const uint64_t* v = dec_at(g, c, r);
      h = mix8(mix8(h, v[0]), v[1]);
    } else {
      h = mix8(h, value_bits(g, c, r));
    }
  }
  return fmix64(h);
}
__device__ uint64_t tuple_key(const GroupCols& g, int64_t r) { return tuple_hash(g, r) & g.key_mask; }

__device__ __forceinline__ bool tuple_equal_rows(const GroupCols& ga, const GroupCols& gb, int64_t a, int64_t b) {
  for (int c = 0; c < ga.n_cols; ++c) {
    if (ga.type[c] == DQ_TYPE_UTF8 || ga.type[c] == DQ_TYPE_LARGE_UTF8) {
      const uint8_t *pa, *pb;
      int64_t la, lb;
      str_of(ga, c, a, pa, la);
      str_of(gb, c, b, pb, lb);
      if (la != lb) return false;
      // 8 bytes, then 4, then single bytes per step (gfx950 global loads take any byte address; none reads past
      // either string): 8x fewer scattered loads than a byte loop (verify_runs over 1e8 C5 strings 17.4 ms, r4g3)
      typedef uint64_t u64u __attribute__((aligned(1)));
      typedef uint32_t u32u __attribute__((aligned(1)));
      int64_t i = 0;
      for (; i + 8 <= la; i += 8)
        if (*reinterpret_cast<const u64u*>(pa + i) != *reinterpret_cast<const u64u*>(pb + i)) return false;
      if (i + 4 <= la) {
        if (*reinterpret_cast<const u32u*>(pa + i) != *reinterpret_cast<const u32u*>(pb + i)) return false;
        i += 4;
      }
      for (; i < la; ++i)
        if (pa[i] != pb[i]) return false;
    } else if (is_dec(ga.type[c])) {
      const uint64_t *va = dec_at(ga, c, a), *vb = dec_at(gb, c, b);
      if (va[0] != vb[0] || va[1] != vb[1]) return false;
    } else if (value_bits(ga, c, a) != value_bits(gb, c, b)) {
      return false;
    }
  }
  return true;
}
__device__ bool tuple_equal(const GroupCols* chunks, uint64_t ra, uint64_t rb) {
  return tuple_equal_rows(chunks[ra >> kRowBits], chunks[rb >> kRowBits], (int64_t)(ra & ((1ull << kRowBits) - 1)),
                          (int64_t)(rb & ((1ull << kRowBits) - 1)));
}

// The non-null rows' keys (and, hashed, their row ids) of a chunk appended to out_keys / out_rows at the launch-wide
// cursor, in no particular order (the radix sort comes next; any row of a group may represent it: its tuple equals
// the others').  A workgroup takes kCompactRows rows per tile, ballots its rows' validity, and reserves the tile's
// slots with one global atomic.  (Replaced group_keys + hipCUB's order-preserving DeviceSelect::Flagged, one per
// output array: 3.0 ms per 1e8 rows and select, r4g2.)
constexpr int kCompactPer = 8;                        // rows per thread and tile
constexpr int kCompactRows = 256 * kCompactPer;
// cursor[0]: the append cursor; cursor[1] / cursor[2]: AND / OR of every appended key (their XOR has the bits in
// which the keys differ: the radix sort skips the common high bits)
// HASHED: keys are tuple hashes (any columns); else one numeric column whose value bits are the keys -- its next
// tile's values and validity words are loaded before this tile's work (in flight behind it)
template <bool HASHED>
__global__ __launch_bounds__(256) void group_compact(GroupCols g, int64_t n, int64_t chunk,
                                                     uint64_t* __restrict__ out_keys, uint64_t* __restrict__ out_rows,
                                                     unsigned long long* __restrict__ cursor) {
  __shared__ uint32_t wave_n[4];
  __shared__ unsigned long long tile_base;
  __shared__ unsigned long long wave_and[4], wave_or[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool hashed = HASHED;
  uint64_t k_and = ~0ull, k_or = 0;
  const int64_t tstride = (int64_t)gridDim.x * kCompactRows;
  uint64_t nval[HASHED ? 1 : kCompactPer];
  uint32_t nvw[HASHED ? 1 : kCompactPer];
  auto fetch = [&](int64_t t0) __attribute__((always_inline)) {
    if constexpr (!HASHED) {
#pragma unroll
      for (int u = 0; u < kCompactPer; ++u) {
        const int64_t r = t0 + u * 256 + threadIdx.x;
        nval[u] = 0;
        nvw[u] = 0;
        if (r < n) {
          nval[u] = value_bits(g, 0, r);
          nvw[u] = g.validity[0] ? g.validity[0][r >> 5] : 0xFFFFFFFFu;
        }
      }
    }
  };
  fetch((int64_t)blockIdx.x * kCompactRows);
  for (int64_t t0 = (int64_t)blockIdx.x * kCompactRows; t0 < n; t0 += tstride) {
    uint64_t key[kCompactPer];
    uint64_t bal[kCompactPer];
    uint32_t cnt = 0;
    uint64_t cval[HASHED ? 1 : kCompactPer];
    uint32_t cvw[HASHED ? 1 : kCompactPer];
    if constexpr (!HASHED) {
#pragma unroll
      for (int u = 0; u < kCompactPer; ++u) {
        cval[u] = nval[u];
        cvw[u] = nvw[u];
      }
      if (t0 + tstride < n) fetch(t0 + tstride);
    }
#pragma unroll
    for (int u = 0; u < kCompactPer; ++u) {
      const int64_t r = t0 + u * 256 + threadIdx.x;
      bool v;
      if constexpr (HASHED) {
        v = r < n && row_valid(g, r);
        key[u] = v ? tuple_key(g, r) : 0;
      } else {
        v = r < n && ((cvw[u] >> (r & 31)) & 1u);
        key[u] = v ? cval[u] : 0;
      }
      if (v) {
        k_and &= key[u];
        k_or |= key[u];
      }
      bal[u] = __builtin_amdgcn_ballot_w64(v);
      cnt += (uint32_t)__builtin_popcountll(bal[u]);
    }
    if (lane == 0) wave_n[wave] = cnt;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      before += w < wave ? wave_n[w] : 0u;
      total += wave_n[w];
    }
    if (threadIdx.x == 0 && total) tile_base = atomicAdd(cursor, (unsigned long long)total);
    __syncthreads();
    unsigned long long pos = tile_base + before;
#pragma unroll
    for (int u = 0; u < kCompactPer; ++u) {
      if ((bal[u] >> lane) & 1ull) {
        const unsigned long long at =
            pos + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal[u] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal[u], 0u));
        out_keys[at] = key[u];
        if (hashed) out_rows[at] = ((uint64_t)chunk << kRowBits) | (uint64_t)(t0 + u * 256 + threadIdx.x);
      }
      pos += (unsigned long long)__builtin_popcountll(bal[u]);
    }
    __syncthreads();  // wave_n / tile_base are rewritten by the next tile
  }
  // the workgroup's AND / OR: lanes, then waves, then one atomic pair
  for (int d = 32; d >= 1; d >>= 1) {
    k_and &= __shfl_xor(k_and, d);
    k_or |= __shfl_xor(k_or, d);
  }
  if (lane == 0) {
    wave_and[wave] = k_and;
    wave_or[wave] = k_or;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t a = wave_and[0] & wave_and[1] & wave_and[2] & wave_and[3];
    const uint64_t o = wave_or[0] | wave_or[1] | wave_or[2] | wave_or[3];
    if (a != ~0ull) atomicAnd(&cursor[1], (unsigned long long)a);
    if (o != 0) atomicOr(&cursor[2], (unsigned long long)o);
  }
}

// neighbours with equal hash keys must hold equal tuples.  A wave takes 64 consecutive sorted positions; a position
// that continues a run is compared with the run's first position within the wave (found from the ballot of run
// heads), or -- the wave's first position -- with the one before it: by transitivity every run is checked exactly,
// and the compared-against tuple is shared by the wave's lanes of a run, so its scattered loads hit the cache (a
// column of few distinct values used to load two random strings per pair).  ONE: a single chunk, whose column
// descriptor comes in the kernel arguments (scalar loads) instead of from a per-row lookup in global memory
template <bool ONE>
__global__ void verify_runs(const uint64_t* __restrict__ keys, const uint64_t* __restrict__ rows, int64_t n,
                            const GroupCols* __restrict__ chunks, GroupCols g0, int32_t* __restrict__ collision) {
  const uint64_t rmask = (1ull << kRowBits) - 1ull;
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;  // a multiple of 64: waves stay 64-aligned
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x - lane; i0 < n; i0 += stride) {
    const int64_t i = i0 + lane;
    const bool in = i < n;
    const uint64_t k = in ? keys[i] : 0ull;
    const bool head = !in || i == 0 || keys[i - 1] != k;
    const uint64_t heads = __builtin_amdgcn_ballot_w64(head);
    if (head) continue;
    const uint64_t upto = heads & (lane == 63 ? ~0ull : ((1ull << (lane + 1)) - 1ull));
    const int first = upto ? 63 - __builtin_clzll(upto) : 0;  // the run's first lane in this wave (< lane), or 0
    const int64_t partner = lane == 0 ? i - 1 : i0 + first;
    const uint64_t ra = rows[partner], rb = rows[i];
    const bool eq = ONE ? tuple_equal_rows(g0, g0, (int64_t)(ra & rmask), (int64_t)(rb & rmask)) : tuple_equal(chunks, ra, rb);
    if (!eq) atomicOr(collision, 1);
  }
}

// The compaction-order form of the exact check, for tables of few groups (most rows share their group with many
// others: the sorted-order check then loads one scattered string per row).  It walks the keys and row ids as the
// compaction kernel appended them (each workgroup tile's rows in row order, so a row's own tuple is read nearly
// sequentially), finds the row's group by binary search of its key in the table's sorted group keys (LDS-sampled),
// and compares
// the row with the group's representative row, whose tuple the group's rows share (cache hits).
constexpr int kVSample = 2048;  // group keys sampled into LDS: the search's first steps
template <bool ONE>
__global__ __launch_bounds__(256) void verify_compacted(const uint64_t* __restrict__ keys, const uint64_t* __restrict__ rows,
                                                        int64_t nv, const uint64_t* __restrict__ gkeys, int64_t G,
                                                        const uint64_t* __restrict__ rep, const GroupCols* __restrict__ chunks,
                                                        GroupCols g0, int32_t* __restrict__ collision) {
  __shared__ uint64_t smp[kVSample];  // every stride-th group key (all of them for G <= 2048)
  const uint64_t rmask = (1ull << kRowBits) - 1ull;
  const int64_t stride = (G + kVSample - 1) / kVSample;
  const int ns = (int)((G + stride - 1) / stride);
  for (int s = threadIdx.x; s < ns; s += blockDim.x) smp[s] = gkeys[(int64_t)s * stride];
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = keys[i], self = rows[i];
    int lo = 0, hi = ns - 1;  // the last sample <= k (k is one of the group keys, so smp[0] <= k)
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (smp[mid] <= k) lo = mid;
      else hi = mid - 1;
    }
    int64_t a = (int64_t)lo * stride, b = (a + stride < G ? a + stride : G) - 1;  // then within its stride
    while (a < b) {
      const int64_t mid = (a + b) >> 1;
      if (gkeys[mid] < k) a = mid + 1;
      else b = mid;
    }
    const uint64_t rp = rep[a];
    if (rp == self) continue;
    const bool eq = ONE ? tuple_equal_rows(g0, g0, (int64_t)(rp & rmask), (int64_t)(self & rmask))
                        : tuple_equal(chunks, rp, self);
    if (!eq) atomicOr(collision, 1);
  }
}

constexpr int kSumBlocks = 1024;
constexpr int64_t kRowOrderVerify = 8;  // compaction-order check when the table has <= 1 group per 8 grouped rows
constexpr int64_t kCompactedMaxGroups = 1 << 16;  // ... and its group keys (the binary search) stay cache-resident
struct SumPart { int64_t unique; double ent; };

// fixed-order partials: block b sums groups b, b + kSumBlocks, ... in a fixed tree
__global__ __launch_bounds__(256) void summary_part(const int64_t* __restrict__ counts, int64_t n, double num_rows,
                                                    SumPart* __restrict__ part) {
  __shared__ int64_t su[256];
  __shared__ double se[256];
  int64_t u = 0;
  double e = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double c = (double)counts[i];
    u += counts[i] == 1 ? 1 : 0;
    // Entropy.scala:31-37: -(count / numRows) * ln(count / numRows), 0 for a zero count
    if (c != 0.0) e += -(c / num_rows) * log(c / num_rows);
  }
  su[threadIdx.x] = u;
  se[threadIdx.x] = e;
  __syncthreads();
  for (int s = 128; s >= 1; s >>= 1) {
    if ((int)threadIdx.x < s) { su[threadIdx.x] += su[threadIdx.x + s]; se[threadIdx.x] += se[threadIdx.x + s]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = SumPart{su[0], se[0]};
}

__global__ void summary_final(const SumPart* __restrict__ part, int32_t nparts, SumPart* __restrict__ out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    SumPart t{0, 0.0};
    for (int i = 0; i < nparts; ++i) { t.unique += part[i].unique; t.ent += part[i].ent; }
    *out = t;
  }
}

// key of one column of a row (exact value for numeric columns, 64-bit hash of the bytes for strings)
__device__ uint64_t col_key(const GroupCols& g, int c, int64_t r) {
  if (g.type[c] != DQ_TYPE_UTF8 && g.type[c] != DQ_TYPE_LARGE_UTF8 && !is_dec(g.type[c])) return value_bits(g, c, r);
  GroupCols one = g;
  one.n_cols = 1;
  one.values[0] = g.values[c];
  one.offsets[0] = g.offsets[c];
  one.type[0] = g.type[c];
  return tuple_key(one, r);
}

__device__ bool col_equal(const GroupCols* chunks, int c, uint64_t ra, uint64_t rb) {
  const GroupCols& ga = chunks[ra >> kRowBits];
  const GroupCols& gb = chunks[rb >> kRowBits];
  const int64_t a = (int64_t)(ra & ((1ull << kRowBits) - 1)), b = (int64_t)(rb & ((1ull << kRowBits) - 1));
  if (is_dec(ga.type[c])) {
    const uint64_t *va = dec_at(ga, c, a), *vb = dec_at(gb, c, b);
    return va[0] == vb[0] && va[1] == vb[1];
  }
  if (ga.type[c] != DQ_TYPE_UTF8 && ga.type[c] != DQ_TYPE_LARGE_UTF8) return value_bits(ga, c, a) == value_bits(gb, c, b);
  const uint8_t *pa, *pb;
  int64_t la, lb;
  str_of(ga, c, a, pa, la);
  str_of(gb, c, b, pb, lb);
  if (la != lb) return false;
  for (int64_t i = 0; i < la; ++i)
    if (pa[i] != pb[i]) return false;
  return true;
}

// MutualInformation: per joint group g its representative row and the keys of both columns
__global__ void mi_group_keys(const uint64_t* __restrict__ sorted_rows, const int64_t* __restrict__ starts, int64_t G,
                              const GroupCols* __restrict__ chunks, uint64_t* __restrict__ rep, uint64_t* __restrict__ xk,
                              uint64_t* __restrict__ yk, uint64_t* __restrict__ idx) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < G; g += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t r = sorted_rows[starts[g]];
    const GroupCols& gc = chunks[r >> kRowBits];
    const int64_t lr = (int64_t)(r & ((1ull << kRowBits) - 1));
    rep[g] = r;
    xk[g] = col_key(gc, 0, lr);
    yk[g] = col_key(gc, 1, lr);
    idx[g] = (uint64_t)g;
  }
}

// marginal of column c over the joint groups sorted by that column's key: segment heads, an exact
// check of equal-hash neighbours (strings), then segment sums of the joint counts (integer atomics)
__global__ void mi_heads(const uint64_t* __restrict__ sk, const uint64_t* __restrict__ sidx, const uint64_t* __restrict__ rep,
                         int64_t G, const GroupCols* __restrict__ chunks, int c, uint32_t* __restrict__ head,
                         int32_t* __restrict__ collision) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < G; i += (int64_t)gridDim.x * blockDim.x) {
    const bool h = i == 0 || sk[i] != sk[i - 1];
    head[i] = h ? 1u : 0u;
    if (!h && !col_equal(chunks, c, rep[sidx[i]], rep[sidx[i - 1]])) atomicOr(collision, 1);
  }
}
__global__ void mi_segsum(const uint64_t* __restrict__ sidx, const uint32_t* __restrict__ seg, const int64_t* __restrict__ gc,
                          int64_t G, unsigned long long* __restrict__ segsum) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < G; i += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(&segsum[seg[i] - 1], (unsigned long long)gc[sidx[i]]);
}
__global__ void mi_scatter(const uint64_t* __restrict__ sidx, const uint32_t* __restrict__ seg,
                           const unsigned long long* __restrict__ segsum, int64_t G, int64_t* __restrict__ pm) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < G; i += (int64_t)gridDim.x * blockDim.x)
    pm[sidx[i]] = (int64_t)segsum[seg[i] - 1];
}
// fixed-order partial sums of (pxy / N) * ln((pxy / N) / ((px / N) * (py / N)))  (MutualInformation.scala:53-56)
__global__ __launch_bounds__(256) void mi_part(const int64_t* __restrict__ gc, const int64_t* __restrict__ px,
                                               const int64_t* __restrict__ py, int64_t G, double total,
                                               double* __restrict__ part) {
  __shared__ double se[256];
  double e = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < G; i += (int64_t)gridDim.x * 256) {
    const double pxy = (double)gc[i], a = (double)px[i], b = (double)py[i];
    e += (pxy / total) * log((pxy / total) / ((a / total) * (b / total)));
  }
  se[threadIdx.x] = e;
  __syncthreads();
  for (int s = 128; s >= 1; s >>= 1) {
    if ((int)threadIdx.x < s) se[threadIdx.x] += se[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = se[0];
}
__global__ void mi_final(const double* __restrict__ part, int32_t nparts, double* __restrict__ out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i < nparts; ++i) t += part[i];
    *out = t;
  }
}

#define GHIP(x)                                                                                  \
  do {                                                                                           \
    hipError_t e_ = (x);                                                                         \
    if (e_ != hipSuccess) return set_error(DQ_E_HIP, "%s: %s", #x, hipGetErrorString(e_));      \
  } while (0)

// Scratch buffers come from a per-device arena of named slots that only grows: a GROUP BY over a
// 62.5 M-row chunk needs ~2 GB of temporaries, and hipMalloc / hipFree of that much per call costs more
// than the sort itself.  Calls are serialised by g_arena_mu (the arena is shared by all plans).
std::mutex g_arena_mu;
struct Slot { void* p = nullptr; size_t cap = 0; };
std::map<std::pair<int, int>, Slot> g_arena;  // (device, slot) -> buffer

struct DevBuf {
  int dev = 0, slot = 0;
  void* p = nullptr;
  DevBuf(int device, int s) : dev(device), slot(s) {}
  dq_status alloc(size_t bytes) {
    bytes = std::max<size_t>(bytes, 256);
    Slot& sl = g_arena[{dev, slot}];
    if (sl.cap < bytes) {
      if (sl.p) (void)hipFree(sl.p);
      sl.p = nullptr;
      sl.cap = 0;
      const size_t want = bytes + bytes / 8;  // headroom for the next, slightly larger call
      if (hipMalloc(&sl.p, want) != hipSuccess) return set_error(DQ_E_OOM, "hipMalloc(%zu) failed", want);
      sl.cap = want;
    }
    p = sl.p;
    return DQ_OK;
  }
  template <typename T> T* as() const { return reinterpret_cast<T*>(p); }
};

int grid_for(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(8192, (n + 255) / 256)); }

}  // namespace
}  // namespace dq

using namespace dq;

struct dq_freq_table {
  int32_t device = 0;
  hipStream_t stream = nullptr;
  int32_t hashed = 0;
  std::vector<int32_t> types;
  int64_t n_groups = 0;
  int64_t n_values = 0;  // rows with all grouping columns non-null
  uint64_t* d_keys = nullptr;
  int64_t* d_counts = nullptr;
  uint64_t* d_rep = nullptr;  // hashed tables built from data: one row id (chunk << 40 | row) per group
  uint64_t* d_keys2 = nullptr;  // hashed tables: second tuple hash per group (merge collision check)
  ~dq_freq_table() {
    if (d_keys) (void)hipFree(d_keys);
    if (d_keys2) (void)hipFree(d_keys2);
    if (d_counts) (void)hipFree(d_counts);
    if (d_rep) (void)hipFree(d_rep);
  }
};

namespace dq {
namespace {
__global__ void gather_rep(const uint64_t* __restrict__ sorted_rows, const int64_t* __restrict__ starts, int64_t G,
                           uint64_t* __restrict__ rep) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < G; g += (int64_t)gridDim.x * blockDim.x)
    rep[g] = sorted_rows[starts[g]];
}
// The dictionary form of a low-cardinality table (dict_table): the keys of an evenly spaced sample of the compacted
// keys (with their row ids), then every compacted key counted against the sample's distinct keys.
__global__ void dict_sample(const uint64_t* __restrict__ keys, const uint64_t* __restrict__ rows, int64_t n, int m,
                            uint64_t* __restrict__ skeys, uint64_t* __restrict__ srows) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const int64_t r = (int64_t)i * (n / m) + ((int64_t)i * (n % m)) / m;  // floor(i n / m), m <= kDictSample
  skeys[i] = keys[r];
  if (rows) srows[i] = rows[r];
}

constexpr int kDictMax = 2048;      // distinct sample keys the dictionary form takes (LDS: 16 KB keys + 8 KB counts)
constexpr int kDictSample = 16384;  // keys sampled: by default the form needs >= 16 samples per distinct key, so a
                                    // group of >= 1 / 1024 of the keys is missed with probability < e^-16
// the distinct keys of the sorted sample (one workgroup of 1024 threads, 16 consecutive keys each): unique[0 .. *nd)
__global__ __launch_bounds__(1024) void dict_unique(const uint64_t* __restrict__ sorted, int m,
                                                    uint64_t* __restrict__ unique, int64_t* __restrict__ nd) {
  __shared__ int part[1024];
  constexpr int kPer = kDictSample / 1024;
  const int t = threadIdx.x, i0 = t * kPer;
  int heads = 0;
  for (int j = 0; j < kPer; ++j) {
    const int i = i0 + j;
    heads += (i < m && (i == 0 || sorted[i] != sorted[i - 1])) ? 1 : 0;
  }
  part[t] = heads;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {  // inclusive scan of the per-thread head counts
    const int v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int at = part[t] - heads;
  for (int j = 0; j < kPer; ++j) {
    const int i = i0 + j;
    if (i < m && (i == 0 || sorted[i] != sorted[i - 1])) unique[at++] = sorted[i];
  }
  if (t == 1023) nd[0] = part[1023];
}
// rep[g] = the smallest sampled row id of group g (every sampled key is one of dict's nd keys; rep preset to ~0)
__global__ void dict_rep(const uint64_t* __restrict__ skeys, const uint64_t* __restrict__ srows, int m,
                         const uint64_t* __restrict__ dict, int nd, unsigned long long* __restrict__ rep) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint64_t k = skeys[i];
  int lo = 0, hi = nd - 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (dict[mid] < k) lo = mid + 1;
    else hi = mid;
  }
  atomicMin(&rep[lo], (unsigned long long)srows[i]);
}
constexpr int kDictPer = 4;         // keys per thread and iteration (independent searches in flight)
// counts[g] += #{compacted keys == dict[g]} (dict: nd sorted distinct keys, pw = the power of two >= nd); a key
// outside the dictionary raises *miss (the caller then sorts instead)
__global__ __launch_bounds__(256) void dict_count(const uint64_t* __restrict__ keys, int64_t n,
                                                  const uint64_t* __restrict__ dict, int nd, int pw,
                                                  unsigned long long* __restrict__ counts, int32_t* __restrict__ miss) {
  __shared__ uint64_t d[kDictMax];
  __shared__ uint32_t c[kDictMax];
  for (int i = threadIdx.x; i < nd; i += 256) {
    d[i] = dict[i];
    c[i] = 0;
  }
  __syncthreads();
  bool missed = false;
  const int64_t stride = (int64_t)gridDim.x * 256 * kDictPer;
  for (int64_t base = (int64_t)blockIdx.x * 256 * kDictPer; base < n; base += stride) {
    uint64_t k[kDictPer];
    int pos[kDictPer];
#pragma unroll
    for (int u = 0; u < kDictPer; ++u) {
      const int64_t i = base + u * 256 + threadIdx.x;
      k[u] = i < n ? __builtin_nontemporal_load(keys + i) : d[0];
      pos[u] = 0;
    }
    for (int step = pw >> 1; step > 0; step >>= 1) {  // the last dictionary key <= k
#pragma unroll
      for (int u = 0; u < kDictPer; ++u) {
        const int j = pos[u] + step;
        if (j < nd && d[j] <= k[u]) pos[u] = j;
      }
    }
#pragma unroll
    for (int u = 0; u < kDictPer; ++u) {
      if (base + u * 256 + threadIdx.x >= n) continue;
      if (d[pos[u]] == k[u]) atomicAdd(&c[pos[u]], 1u);
      else missed = true;
    }
  }
  if (missed) miss[0] = 1;
  __syncthreads();
  for (int i = threadIdx.x; i < nd; i += 256)
    if (c[i]) atomicAdd(&counts[i], (unsigned long long)c[i]);
}

// second hash of every group's representative row (hashed tables built from data)
__global__ void group_keys2(const uint64_t* __restrict__ rep, int64_t G, const GroupCols* __restrict__ chunks,
                            uint64_t* __restrict__ keys2) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < G; g += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t r = rep[g];
    keys2[g] = tuple_hash(chunks[r >> kRowBits], (int64_t)(r & ((1ull << kRowBits) - 1)), kSeed2);
  }
}
__global__ void iota_u64(uint64_t* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (uint64_t)i;
}
// merge of hashed tables: (second hash, count) in first-hash order; equal first hashes with different
// second hashes are distinct tuples
__global__ void merge_gather_check(const uint64_t* __restrict__ k1s, const uint64_t* __restrict__ pos,
                                   const uint64_t* __restrict__ k2, const int64_t* __restrict__ c, int64_t n,
                                   uint64_t* __restrict__ k2s, int64_t* __restrict__ cs, int32_t* __restrict__ collision) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t p = pos[i];
    k2s[i] = k2[p];
    cs[i] = c[p];
    if (i > 0 && k1s[i] == k1s[i - 1] && k2[p] != k2[pos[i - 1]]) atomicOr(collision, 1);
  }
}
__global__ void iota_u32(uint32_t* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (uint32_t)i;
}
__global__ void gather_top(const uint32_t* __restrict__ idx, int32_t n, const uint64_t* __restrict__ keys,
                           const int64_t* __restrict__ counts, const uint64_t* __restrict__ rep,
                           uint64_t* __restrict__ ok, int64_t* __restrict__ oc, uint64_t* __restrict__ orp) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const uint32_t g = idx[i];
    ok[i] = keys[g];
    oc[i] = counts[g];
    orp[i] = rep ? rep[g] : ~0ull;
  }
}
}  // namespace
}  // namespace dq

static dq_status rle_into(dq_freq_table* t, const uint64_t* sorted, int64_t n, const uint64_t* sorted_rows = nullptr) {
  DevBuf nruns(t->device, 20), tmp(t->device, 21), starts(t->device, 22);
  if (dq_status s = nruns.alloc(sizeof(int64_t))) return s;
  GHIP(hipMalloc(&t->d_keys, std::max<int64_t>(1, n) * sizeof(uint64_t)));
  GHIP(hipMalloc(&t->d_counts, std::max<int64_t>(1, n) * sizeof(int64_t)));
  if (n == 0) { t->n_groups = 0; return DQ_OK; }
  if (dq_status s = tmp.alloc(prim::runs_temp_bytes(n))) return s;
  if (dq_status s = starts.alloc((size_t)n * 8)) return s;
  GHIP(prim::runs(sorted, n, t->d_keys, starts.as<int64_t>(), t->d_counts, nruns.as<int64_t>(), tmp.p, t->stream));
  GHIP(hipMemcpyAsync(&t->n_groups, nruns.p, sizeof(int64_t), hipMemcpyDeviceToHost, t->stream));
  GHIP(hipStreamSynchronize(t->stream));
  if (sorted_rows && t->n_groups > 0) {  // representative row of every group (Histogram renders its value)
    GHIP(hipMalloc(&t->d_rep, t->n_groups * 8));
    hipLaunchKernelGGL(gather_rep, dim3(grid_for(t->n_groups)), dim3(256), 0, t->stream, sorted_rows,
                       starts.as<int64_t>(), t->n_groups, t->d_rep);
    GHIP(hipGetLastError());
    GHIP(hipStreamSynchronize(t->stream));
  }
  return DQ_OK;
}

// the exact check of equal-hash neighbours in sorted order (verify_runs); nsel's first word is the collision flag
static dq_status verify_sorted(dq_freq_table* t, const uint64_t* sorted_keys, const uint64_t* sorted_rows, int64_t nv,
                               const std::vector<GroupCols>& gcs, DevBuf& d_chunks, DevBuf& nsel) {
  GHIP(hipMemsetAsync(nsel.p, 0, 8, t->stream));
  if (gcs.size() == 1)
    hipLaunchKernelGGL(verify_runs<true>, dim3(grid_for(nv)), dim3(256), 0, t->stream, sorted_keys, sorted_rows, nv,
                       d_chunks.as<GroupCols>(), gcs[0], nsel.as<int32_t>());
  else
    hipLaunchKernelGGL(verify_runs<false>, dim3(grid_for(nv)), dim3(256), 0, t->stream, sorted_keys, sorted_rows, nv,
                       d_chunks.as<GroupCols>(), gcs[0], nsel.as<int32_t>());
  GHIP(hipGetLastError());
  int32_t coll = 0;
  GHIP(hipMemcpyAsync(&coll, nsel.p, 4, hipMemcpyDeviceToHost, t->stream));
  GHIP(hipStreamSynchronize(t->stream));
  if (coll) return set_error(DQ_E_UNSUPPORTED, "dq_freq_build: 64-bit tuple-hash collision between distinct values");
  return DQ_OK;
}

// The dictionary form of a table (no sort): when an evenly spaced sample of the compacted keys holds at most
// 1 / 16 as many distinct keys (at most kDictMax), every key is counted against the sample's distinct keys in one
// pass; the groups are then those keys in ascending order -- what the sort and its runs yield -- with the smallest
// sampled row id of each as its representative.  A key outside the sample (a group the sample missed) sets
// *done = false and the caller sorts.  DQ_GROUP_DICT=0 turns it off, =1 lifts the size thresholds (tests).
static dq_status dict_table(dq_freq_table* t, const uint64_t* keys, const uint64_t* rows, int64_t nv, int end_bit,
                            bool* done) {
  *done = false;
  const char* knob = std::getenv("DQ_GROUP_DICT");
  const bool forced = knob && knob[0] == '1';
  if (knob && knob[0] == '0') return DQ_OK;
  // only where the sort would run 5+ digit passes (tuple hashes, wide numeric keys) over 1 M+ keys: a table the
  // form declines pays ~0.15 ms (the sample's sort and read-back), measured against 4.0 ms for 1e8 27-bit keys
  if (!forced && (nv < (int64_t)1 << 20 || end_bit <= 32)) return DQ_OK;
  const int D = t->device;
  const int m = (int)std::min<int64_t>(kDictSample, nv);
  DevBuf sk(D, 50), sr(D, 51), sks(D, 52), nr(D, 54), tmp(D, 55);
  if (dq_status s = sk.alloc((size_t)m * 8)) return s;
  if (dq_status s = sks.alloc((size_t)m * 8)) return s;
  if (dq_status s = nr.alloc(16)) return s;
  if (rows)
    if (dq_status s = sr.alloc((size_t)m * 8)) return s;
  const size_t tb = prim::sort_temp_bytes(m, 0);
  if (dq_status s = tmp.alloc(tb)) return s;
  hipLaunchKernelGGL(dict_sample, dim3((m + 255) / 256), dim3(256), 0, t->stream, keys, rows, nv, m, sk.as<uint64_t>(),
                     rows ? sr.as<uint64_t>() : nullptr);
  GHIP(hipGetLastError());
  // keys only: a table the form does not take costs this sort of 16 K keys, one small kernel and one read-back
  GHIP(prim::sort_pairs(sk.as<uint64_t>(), sks.as<uint64_t>(), nullptr, nullptr, 0, m, 0, end_bit, false, tmp.p, tb,
                        t->stream));
  DevBuf dict(D, 53);
  if (dq_status s = dict.alloc((size_t)m * 8)) return s;
  hipLaunchKernelGGL(dict_unique, dim3(1), dim3(1024), 0, t->stream, sks.as<uint64_t>(), m, dict.as<uint64_t>(),
                     nr.as<int64_t>());
  GHIP(hipGetLastError());
  int64_t nd = 0;
  GHIP(hipMemcpyAsync(&nd, nr.p, 8, hipMemcpyDeviceToHost, t->stream));
  GHIP(hipStreamSynchronize(t->stream));
  if (nd < 1 || nd > kDictMax || (!forced && nd * 16 > m)) return DQ_OK;
  int pw = 1;
  while (pw < nd) pw <<= 1;
  GHIP(hipMalloc(&t->d_keys, (size_t)nd * 8));
  GHIP(hipMalloc(&t->d_counts, (size_t)nd * 8));
  GHIP(hipMemcpyAsync(t->d_keys, dict.p, (size_t)nd * 8, hipMemcpyDeviceToDevice, t->stream));
  GHIP(hipMemsetAsync(t->d_counts, 0, (size_t)nd * 8, t->stream));
  GHIP(hipMemsetAsync(nr.as<char>() + 8, 0, 4, t->stream));
  if (rows) {
    GHIP(hipMalloc(&t->d_rep, (size_t)nd * 8));
    GHIP(hipMemsetAsync(t->d_rep, 0xFF, (size_t)nd * 8, t->stream));
    hipLaunchKernelGGL(dict_rep, dim3((m + 255) / 256), dim3(256), 0, t->stream, sk.as<uint64_t>(), sr.as<uint64_t>(), m,
                       t->d_keys, (int)nd, reinterpret_cast<unsigned long long*>(t->d_rep));
    GHIP(hipGetLastError());
  }
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(2048, (nv + 256 * kDictPer - 1) / (256 * kDictPer)));
  hipLaunchKernelGGL(dict_count, dim3(grid), dim3(256), 0, t->stream, keys, nv, t->d_keys, (int)nd, pw,
                     reinterpret_cast<unsigned long long*>(t->d_counts), reinterpret_cast<int32_t*>(nr.as<char>() + 8));
  GHIP(hipGetLastError());
  int32_t miss = 0;
  GHIP(hipMemcpyAsync(&miss, nr.as<char>() + 8, 4, hipMemcpyDeviceToHost, t->stream));
  GHIP(hipStreamSynchronize(t->stream));
  if (miss) {  // a group outside the sample: back to the sort (the caller allocates the table's arrays afresh)
    (void)hipFree(t->d_keys);
    (void)hipFree(t->d_counts);
    if (t->d_rep) (void)hipFree(t->d_rep);
    t->d_keys = nullptr;
    t->d_counts = nullptr;
    t->d_rep = nullptr;
    return DQ_OK;
  }
  t->n_groups = nd;
  *done = true;
  return DQ_OK;
}

extern "C" {

struct MiRequest { double total; double* value; int32_t* defined; };
static dq_status mi_from_joint(dq_freq_table* t, const uint64_t* sorted_keys, const uint64_t* sorted_rows, int64_t nv,
                               const GroupCols* d_chunks, const MiRequest& mi);

static dq_status freq_build_impl(const int32_t* types, int32_t n_cols, const dq_column_view* cols,
                                 const int64_t* chunk_rows, int32_t n_chunks, int32_t device, void* hip_stream,
                                 dq_freq_table** out, const MiRequest* mi) {
  if (!out) return set_error(DQ_E_INVALID, "dq_freq_build: out is NULL");
  *out = nullptr;
  if (n_cols < 1 || n_cols > kMaxGroupCols || !types)
    return set_error(DQ_E_INVALID, "dq_freq_build: 1..%d grouping columns", kMaxGroupCols);
  if (n_chunks < 0 || n_chunks > kMaxGroupChunks || (n_chunks > 0 && (!cols || !chunk_rows)))
    return set_error(DQ_E_INVALID, "dq_freq_build: bad chunks (at most %d)", kMaxGroupChunks);
  for (int c = 0; c < n_cols; ++c) {
    if (!type_valid(types[c]))
      return set_error(DQ_E_TYPE, "dq_freq_build: column %d has unknown type %d", c, types[c]);
  }
  int64_t total = 0;
  for (int k = 0; k < n_chunks; ++k) {
    if (chunk_rows[k] < 0 || chunk_rows[k] >= (1ll << kRowBits)) return set_error(DQ_E_INVALID, "chunk rows");
    total += chunk_rows[k];
  }
  if (total >= (1ll << 31)) return set_error(DQ_E_UNSUPPORTED, "dq_freq_build: at most 2^31 - 1 rows per table");
  GHIP(hipSetDevice(device));
  auto* t = new dq_freq_table();
  std::unique_ptr<dq_freq_table> guard(t);
  t->device = device;
  t->stream = reinterpret_cast<hipStream_t>(hip_stream);
  t->types.assign(types, types + n_cols);
  // one fixed-width column: grouped by its exact value bits (strings and tuples: by hash, checked exactly)
  const bool numeric1 = n_cols == 1 && types[0] != DQ_TYPE_UTF8 && types[0] != DQ_TYPE_LARGE_UTF8 && !is_decimal(types[0]);
  t->hashed = numeric1 && !mi ? 0 : 1;

  // test hook: keep only some bits of the primary tuple hash, to force collisions between distinct tuples
  uint64_t key_mask = ~0ull;
  if (const char* e = std::getenv("DQ_TEST_GROUP_HASH_MASK")) key_mask = std::strtoull(e, nullptr, 16);
  std::vector<GroupCols> gcs(std::max(1, n_chunks));
  for (int k = 0; k < n_chunks; ++k) {
    GroupCols& g = gcs[k];
    std::memset(&g, 0, sizeof(g));
    g.n_cols = n_cols;
    g.key_mask = key_mask;
    for (int c = 0; c < n_cols; ++c) {
      const dq_column_view& v = cols[(size_t)k * n_cols + c];
      g.values[c] = v.values;
      g.validity[c] = reinterpret_cast<const uint32_t*>(v.validity);
      g.offsets[c] = v.offsets;
      g.type[c] = types[c];
    }
  }
  std::lock_guard<std::mutex> lock(g_arena_mu);
  const int D = device;
  DevBuf sel_keys(D, 2), sel_rows(D, 4), nsel(D, 5), tmp(D, 6), sorted_keys(D, 7), sorted_rows(D, 8), d_chunks(D, 9);
  if (dq_status s = nsel.alloc(24)) return s;
  if (dq_status s = sel_keys.alloc(std::max<int64_t>(1, total) * 8)) return s;
  if (t->hashed) {
    if (dq_status s = sel_rows.alloc(std::max<int64_t>(1, total) * 8)) return s;
  }
  int64_t nv = 0;
  const unsigned long long cur0[3] = {0ull, ~0ull, 0ull};  // count, AND, OR of the appended keys
  GHIP(hipMemcpyAsync(nsel.p, cur0, sizeof(cur0), hipMemcpyHostToDevice, t->stream));
  for (int k = 0; k < n_chunks; ++k) {
    const int64_t n = chunk_rows[k];
    if (n == 0) continue;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(2048, (n + kCompactRows - 1) / kCompactRows));
    if (t->hashed)
      hipLaunchKernelGGL(group_compact<true>, dim3(grid), dim3(256), 0, t->stream, gcs[k], n, (int64_t)k,
                         sel_keys.as<uint64_t>(), sel_rows.as<uint64_t>(), nsel.as<unsigned long long>());
    else
      hipLaunchKernelGGL(group_compact<false>, dim3(grid), dim3(256), 0, t->stream, gcs[k], n, (int64_t)k,
                         sel_keys.as<uint64_t>(), nullptr, nsel.as<unsigned long long>());
    GHIP(hipGetLastError());
  }
  unsigned long long cur[3];
  GHIP(hipMemcpyAsync(cur, nsel.p, sizeof(cur), hipMemcpyDeviceToHost, t->stream));
  GHIP(hipStreamSynchronize(t->stream));
  nv = (int64_t)cur[0];
  // the keys agree above their highest differing bit: sorting bits [0, end_bit) gives the same order as all 64
  // (small-range integer columns: 2 digit passes instead of 6)
  const uint64_t differ = nv > 0 ? (uint64_t)(cur[1] ^ cur[2]) : 0ull;
  const int end_bit = differ ? 64 - __builtin_clzll(differ) : 1;
  t->n_values = nv;
  if (t->hashed) {
    if (dq_status s = d_chunks.alloc(gcs.size() * sizeof(GroupCols))) return s;
    GHIP(hipMemcpyAsync(d_chunks.p, gcs.data(), gcs.size() * sizeof(GroupCols), hipMemcpyHostToDevice, t->stream));
  }
  static const char* force = std::getenv("DQ_GROUP_VERIFY");  // A/B knob: "sorted" / "compacted"
  bool dict = false;  // low cardinality: the dictionary form (no sort; the check in compaction order)
  if (!mi && nv > 0 && !(force && force[0] == 's'))
    if (dq_status s = dict_table(t, sel_keys.as<uint64_t>(), t->hashed ? sel_rows.as<uint64_t>() : nullptr, nv,
                                 end_bit, &dict))
      return s;
  if (dq_status s = sorted_keys.alloc(std::max<int64_t>(1, nv) * 8)) return s;
  if (nv > 0 && !dict) {
    if (t->hashed) {
      if (dq_status s = sorted_rows.alloc(nv * 8)) return s;
      const size_t tb = prim::sort_temp_bytes(nv, 8);
      if (dq_status s = tmp.alloc(tb)) return s;
      GHIP(prim::sort_pairs(sel_keys.as<uint64_t>(), sorted_keys.as<uint64_t>(), sel_rows.as<uint64_t>(),
                            sorted_rows.as<uint64_t>(), 8, nv, 0, end_bit, false, tmp.p, tb, t->stream));
      // exact check of equal-hash neighbours in sorted order here for MutualInformation; the frequency table's runs
      // choose between the two forms below
      if (mi)
        if (dq_status s = verify_sorted(t, sorted_keys.as<uint64_t>(), sorted_rows.as<uint64_t>(), nv, gcs, d_chunks, nsel))
          return s;
    } else {
      const size_t tb = prim::sort_temp_bytes(nv, 0);
      if (dq_status s = tmp.alloc(tb)) return s;
      GHIP(prim::sort_pairs(sel_keys.as<uint64_t>(), sorted_keys.as<uint64_t>(), nullptr, nullptr, 0, nv, 0, end_bit,
                            false, tmp.p, tb, t->stream));
    }
  }
  if (mi) return mi_from_joint(t, sorted_keys.as<uint64_t>(), sorted_rows.as<uint64_t>(), nv, d_chunks.as<GroupCols>(), *mi);
  if (!dict)
    if (dq_status s = rle_into(t, sorted_keys.as<uint64_t>(), nv, t->hashed ? sorted_rows.as<uint64_t>() : nullptr))
      return s;
  if (t->hashed && nv > 0) {
    // few groups (rows repeat their group's tuple many times): each row checked against its group's representative
    // in compaction order; otherwise equal-hash neighbours in sorted order (which the dictionary form has not made)
    const bool compacted = dict || (force ? force[0] == 'c'
                                          : t->n_groups <= kCompactedMaxGroups && t->n_groups * kRowOrderVerify <= nv);
    if (compacted) {
      GHIP(hipMemsetAsync(nsel.p, 0, 8, t->stream));
      if (gcs.size() == 1)
        hipLaunchKernelGGL(verify_compacted<true>, dim3(grid_for(nv)), dim3(256), 0, t->stream, sel_keys.as<uint64_t>(),
                           sel_rows.as<uint64_t>(), nv, t->d_keys, t->n_groups, t->d_rep, d_chunks.as<GroupCols>(),
                           gcs[0], nsel.as<int32_t>());
      else
        hipLaunchKernelGGL(verify_compacted<false>, dim3(grid_for(nv)), dim3(256), 0, t->stream,
                           sel_keys.as<uint64_t>(), sel_rows.as<uint64_t>(), nv, t->d_keys, t->n_groups, t->d_rep,
                           d_chunks.as<GroupCols>(), gcs[0], nsel.as<int32_t>());
      GHIP(hipGetLastError());
      int32_t coll = 0;
      GHIP(hipMemcpyAsync(&coll, nsel.p, 4, hipMemcpyDeviceToHost, t->stream));
      GHIP(hipStreamSynchronize(t->stream));
      if (coll) return set_error(DQ_E_UNSUPPORTED, "dq_freq_build: 64-bit tuple-hash collision between distinct values");
    } else if (dq_status s = verify_sorted(t, sorted_keys.as<uint64_t>(), sorted_rows.as<uint64_t>(), nv, gcs, d_chunks,
                                          nsel)) {
      return s;
    }
  }
  if (t->hashed) {
    GHIP(hipMalloc(&t->d_keys2, std::max<int64_t>(1, t->n_groups) * 8));
    if (t->n_groups > 0) {
      hipLaunchKernelGGL(group_keys2, dim3(grid_for(t->n_groups)), dim3(256), 0, t->stream, t->d_rep, t->n_groups,
                         d_chunks.as<GroupCols>(), t->d_keys2);
      GHIP(hipGetLastError());
      GHIP(hipStreamSynchronize(t->stream));
    }
  }
  *out = guard.release();
  return DQ_OK;
}

static dq_status mi_from_joint(dq_freq_table* t, const uint64_t* sorted_keys, const uint64_t* sorted_rows, int64_t nv,
                               const GroupCols* d_chunks, const MiRequest& mi) {
  *mi.defined = 0;
  *mi.value = 0.0;
  if (nv == 0) return DQ_OK;  // sum over an empty join is NULL -> metricFromEmpty
  const int D = t->device;
  const hipStream_t S = t->stream;
  DevBuf gk(D, 30), gc(D, 31), nruns(D, 32), starts(D, 33), rep(D, 34), xk(D, 35), yk(D, 36), idx(D, 37), sk(D, 38),
      sidx(D, 39), head(D, 40), seg(D, 41), segsum(D, 42), px(D, 43), py(D, 44), tmp(D, 45), part(D, 46), res(D, 47),
      coll(D, 48);
  for (DevBuf* b : {&gk, &gc, &starts, &rep, &xk, &yk, &idx, &sk, &sidx, &segsum, &px, &py})
    if (dq_status s = b->alloc(nv * 8)) return s;
  for (DevBuf* b : {&head, &seg})
    if (dq_status s = b->alloc(nv * 4)) return s;
  for (DevBuf* b : {&nruns, &res, &coll})
    if (dq_status s = b->alloc(8)) return s;
  if (dq_status s = part.alloc(kSumBlocks * sizeof(double))) return s;
  const size_t tb = std::max({prim::runs_temp_bytes(nv), prim::sort_temp_bytes(nv, 8), prim::scan_temp_bytes(nv)});
  if (dq_status s = tmp.alloc(tb)) return s;
  // joint groups: keys, counts and first positions of the runs of the sorted joint keys
  GHIP(prim::runs(sorted_keys, nv, gk.as<uint64_t>(), starts.as<int64_t>(), gc.as<int64_t>(), nruns.as<int64_t>(), tmp.p, S));
  int64_t G = 0;
  GHIP(hipMemcpyAsync(&G, nruns.p, 8, hipMemcpyDeviceToHost, S));
  GHIP(hipStreamSynchronize(S));
  hipLaunchKernelGGL(mi_group_keys, dim3(grid_for(G)), dim3(256), 0, S, sorted_rows, starts.as<int64_t>(), G, d_chunks,
                     rep.as<uint64_t>(), xk.as<uint64_t>(), yk.as<uint64_t>(), idx.as<uint64_t>());
  GHIP(hipGetLastError());
  GHIP(hipMemsetAsync(coll.p, 0, 8, S));
  for (int c = 0; c < 2; ++c) {
    GHIP(prim::sort_pairs((c == 0 ? xk : yk).as<uint64_t>(), sk.as<uint64_t>(), idx.as<uint64_t>(),
                          sidx.as<uint64_t>(), 8, G, 0, 64, false, tmp.p, tb, S));
    hipLaunchKernelGGL(mi_heads, dim3(grid_for(G)), dim3(256), 0, S, sk.as<uint64_t>(), sidx.as<uint64_t>(),
                       rep.as<uint64_t>(), G, d_chunks, c, head.as<uint32_t>(), coll.as<int32_t>());
    GHIP(hipGetLastError());
    GHIP(prim::inclusive_sum_u32(head.as<uint32_t>(), seg.as<uint32_t>(), G, tmp.p, S));
    GHIP(hipMemsetAsync(segsum.p, 0, G * 8, S));
    hipLaunchKernelGGL(mi_segsum, dim3(grid_for(G)), dim3(256), 0, S, sidx.as<uint64_t>(), seg.as<uint32_t>(),
                       gc.as<int64_t>(), G, segsum.as<unsigned long long>());
    GHIP(hipGetLastError());
    hipLaunchKernelGGL(mi_scatter, dim3(grid_for(G)), dim3(256), 0, S, sidx.as<uint64_t>(), seg.as<uint32_t>(),
                       segsum.as<unsigned long long>(), G, (c == 0 ? px : py).as<int64_t>());
    GHIP(hipGetLastError());
  }
  const int nb = (int)std::min<int64_t>(kSumBlocks, (G + 255) / 256);
  hipLaunchKernelGGL(mi_part, dim3(nb), dim3(256), 0, S, gc.as<int64_t>(), px.as<int64_t>(), py.as<int64_t>(), G,
                     mi.total, part.as<double>());
  GHIP(hipGetLastError());
  hipLaunchKernelGGL(mi_final, dim3(1), dim3(64), 0, S, part.as<double>(), nb, res.as<double>());
  GHIP(hipGetLastError());
  int32_t collided = 0;
  GHIP(hipMemcpyAsync(&collided, coll.p, 4, hipMemcpyDeviceToHost, S));
  GHIP(hipMemcpyAsync(mi.value, res.p, 8, hipMemcpyDeviceToHost, S));
  GHIP(hipStreamSynchronize(S));
  if (collided) return set_error(DQ_E_UNSUPPORTED, "dq_mutual_information: 64-bit key collision between distinct values");
  *mi.defined = 1;
  return DQ_OK;
}

dq_status dq_freq_build(const int32_t* types, int32_t n_cols, const dq_column_view* cols, const int64_t* chunk_rows,
                        int32_t n_chunks, int32_t device, void* hip_stream, dq_freq_table** out) {
  return freq_build_impl(types, n_cols, cols, chunk_rows, n_chunks, device, hip_stream, out, nullptr);
}

dq_status dq_mutual_information(const int32_t* types, const dq_column_view* cols, const int64_t* chunk_rows,
                                int32_t n_chunks, int64_t num_rows, int32_t device, void* hip_stream, double* value,
                                int32_t* defined) {
  if (!value || !defined) return set_error(DQ_E_INVALID, "dq_mutual_information: NULL output");
  MiRequest mi{(double)num_rows, value, defined};
  dq_freq_table* unused = nullptr;
  dq_status s = freq_build_impl(types, 2, cols, chunk_rows, n_chunks, device, hip_stream, &unused, &mi);
  if (unused) dq_freq_destroy(unused);
  return s;
}

dq_status dq_freq_merge(const dq_freq_table* a, const dq_freq_table* b, dq_freq_table** out) {
  if (!a || !b || !out) return set_error(DQ_E_INVALID, "dq_freq_merge: NULL argument");
  *out = nullptr;
  if (a->types != b->types || a->hashed != b->hashed)
    return set_error(DQ_E_STATE, "dq_freq_merge: frequency tables over different column types");
  const int64_t n = a->n_groups + b->n_groups;
  if (n >= (int64_t(1) << 31))  // dq_prim's sort positions are 32-bit
    return set_error(DQ_E_UNSUPPORTED, "dq_freq_merge: %lld groups in the two tables (at most 2^31 - 1)", (long long)n);
  if (a->hashed && ((a->n_groups > 0 && !a->d_keys2) || (b->n_groups > 0 && !b->d_keys2)))
    return set_error(DQ_E_STATE, "dq_freq_merge: hashed table without its verification hashes");
  GHIP(hipSetDevice(a->device));
  auto* t = new dq_freq_table();
  std::unique_ptr<dq_freq_table> guard(t);
  t->device = a->device;
  t->stream = a->stream;
  t->types = a->types;
  t->hashed = a->hashed;
  t->n_values = a->n_values + b->n_values;
  std::lock_guard<std::mutex> lock(g_arena_mu);
  const int D = a->device;
  DevBuf k_in(D, 10), c_in(D, 11), k_s(D, 12), c_s(D, 13), nruns(D, 14), tmp(D, 15), k2_in(D, 16), pos(D, 17),
      pos_s(D, 18), k2_s(D, 19), coll(D, 23), kdrop(D, 24);
  for (DevBuf* d : {&k_in, &c_in, &k_s, &c_s})
    if (dq_status s = d->alloc(std::max<int64_t>(1, n) * 8)) return s;
  if (dq_status s = nruns.alloc(8)) return s;
  GHIP(hipMemcpyAsync(k_in.p, a->d_keys, a->n_groups * 8, hipMemcpyDeviceToDevice, t->stream));
  GHIP(hipMemcpyAsync(k_in.as<uint64_t>() + a->n_groups, b->d_keys, b->n_groups * 8, hipMemcpyDeviceToDevice, t->stream));
  GHIP(hipMemcpyAsync(c_in.p, a->d_counts, a->n_groups * 8, hipMemcpyDeviceToDevice, t->stream));
  GHIP(hipMemcpyAsync(c_in.as<int64_t>() + a->n_groups, b->d_counts, b->n_groups * 8, hipMemcpyDeviceToDevice, t->stream));
  GHIP(hipMalloc(&t->d_keys, std::max<int64_t>(1, n) * 8));
  GHIP(hipMalloc(&t->d_counts, std::max<int64_t>(1, n) * 8));
  if (t->hashed) GHIP(hipMalloc(&t->d_keys2, std::max<int64_t>(1, n) * 8));
  if (n > 0 && !t->hashed) {
    // both tables' keys are sorted: every key lies between the smaller first and the larger last key, and so
    // shares their common high bits -- the sort covers only the bits below (same order as all 64)
    uint64_t ends[4] = {~0ull, 0ull, ~0ull, 0ull};
    if (a->n_groups > 0) {
      GHIP(hipMemcpyAsync(&ends[0], a->d_keys, 8, hipMemcpyDeviceToHost, t->stream));
      GHIP(hipMemcpyAsync(&ends[1], a->d_keys + (a->n_groups - 1), 8, hipMemcpyDeviceToHost, t->stream));
    }
    if (b->n_groups > 0) {
      GHIP(hipMemcpyAsync(&ends[2], b->d_keys, 8, hipMemcpyDeviceToHost, t->stream));
      GHIP(hipMemcpyAsync(&ends[3], b->d_keys + (b->n_groups - 1), 8, hipMemcpyDeviceToHost, t->stream));
    }
    GHIP(hipStreamSynchronize(t->stream));
    const uint64_t lo = std::min(ends[0], ends[2]), hi = std::max(ends[1], ends[3]);
    const int end_bit = (lo ^ hi) ? 64 - __builtin_clzll(lo ^ hi) : 1;
    const size_t tb = std::max({prim::sort_temp_bytes(n, 8), prim::runs_temp_bytes(n), prim::run_sums_temp_bytes(n)});
    if (dq_status s = tmp.alloc(tb)) return s;
    if (dq_status s = pos.alloc(n * 8)) return s;  // the runs' starts
    GHIP(prim::sort_pairs(k_in.as<uint64_t>(), k_s.as<uint64_t>(), c_in.as<int64_t>(), c_s.as<int64_t>(), 8, n, 0,
                          end_bit, false, tmp.p, tb, t->stream));
    // equal keys of the two tables are now neighbours: one group each, counts added
    GHIP(prim::runs(k_s.as<uint64_t>(), n, t->d_keys, pos.as<int64_t>(), nullptr, nruns.as<int64_t>(), tmp.p, t->stream));
    GHIP(prim::run_sums_i64(c_s.as<int64_t>(), n, pos.as<int64_t>(), nruns.as<int64_t>(), t->d_counts, tmp.p, t->stream));
    GHIP(hipMemcpyAsync(&t->n_groups, nruns.p, 8, hipMemcpyDeviceToHost, t->stream));
  } else if (n > 0) {
    // hashed keys: sort by the first hash carrying positions, gather (second hash, count), refuse equal first
    // hashes with different second hashes, then reduce counts and keep each group's second hash
    for (DevBuf* d : {&k2_in, &pos, &pos_s, &k2_s, &kdrop})
      if (dq_status s = d->alloc(n * 8)) return s;
    if (dq_status s = coll.alloc(8)) return s;
    GHIP(hipMemcpyAsync(k2_in.p, a->d_keys2, a->n_groups * 8, hipMemcpyDeviceToDevice, t->stream));
    GHIP(hipMemcpyAsync(k2_in.as<uint64_t>() + a->n_groups, b->d_keys2, b->n_groups * 8, hipMemcpyDeviceToDevice,
                        t->stream));
    hipLaunchKernelGGL(iota_u64, dim3(grid_for(n)), dim3(256), 0, t->stream, pos.as<uint64_t>(), n);
    GHIP(hipGetLastError());
    const size_t tb = std::max({prim::sort_temp_bytes(n, 8), prim::runs_temp_bytes(n), prim::run_sums_temp_bytes(n)});
    if (dq_status s = tmp.alloc(tb)) return s;
    GHIP(prim::sort_pairs(k_in.as<uint64_t>(), k_s.as<uint64_t>(), pos.as<uint64_t>(), pos_s.as<uint64_t>(), 8, n, 0, 64,
                          false, tmp.p, tb, t->stream));
    GHIP(hipMemsetAsync(coll.p, 0, 8, t->stream));
    hipLaunchKernelGGL(merge_gather_check, dim3(grid_for(n)), dim3(256), 0, t->stream, k_s.as<uint64_t>(),
                       pos_s.as<uint64_t>(), k2_in.as<uint64_t>(), c_in.as<int64_t>(), n, k2_s.as<uint64_t>(),
                       c_s.as<int64_t>(), coll.as<int32_t>());
    GHIP(hipGetLastError());
    // runs of equal first hashes (kdrop: their starts): counts added, the first second hash kept
    GHIP(prim::runs(k_s.as<uint64_t>(), n, t->d_keys, kdrop.as<int64_t>(), nullptr, nruns.as<int64_t>(), tmp.p, t->stream));
    GHIP(prim::run_sums_i64(c_s.as<int64_t>(), n, kdrop.as<int64_t>(), nruns.as<int64_t>(), t->d_counts, tmp.p, t->stream));
    GHIP(prim::run_firsts_u64(k2_s.as<uint64_t>(), n, kdrop.as<int64_t>(), nruns.as<int64_t>(), t->d_keys2, t->stream));
    int32_t collided = 0;
    GHIP(hipMemcpyAsync(&collided, coll.p, 4, hipMemcpyDeviceToHost, t->stream));
    GHIP(hipMemcpyAsync(&t->n_groups, nruns.p, 8, hipMemcpyDeviceToHost, t->stream));
    GHIP(hipStreamSynchronize(t->stream));
    if (collided)
      return set_error(DQ_E_UNSUPPORTED, "dq_freq_merge: 64-bit tuple-hash collision between distinct values of the two tables");
  }
  GHIP(hipStreamSynchronize(t->stream));
  *out = guard.release();
  return DQ_OK;
}

dq_status dq_freq_summarize(const dq_freq_table* t, int64_t num_rows, dq_freq_summary* out) {
  if (!t || !out) return set_error(DQ_E_INVALID, "dq_freq_summarize: NULL argument");
  GHIP(hipSetDevice(t->device));
  std::memset(out, 0, sizeof(*out));
  out->num_groups = t->n_groups;
  out->num_values = t->n_values;
  if (t->n_groups == 0) return DQ_OK;
  std::lock_guard<std::mutex> lock(g_arena_mu);
  DevBuf part(t->device, 16), res(t->device, 17);
  if (dq_status s = part.alloc(kSumBlocks * sizeof(SumPart))) return s;
  if (dq_status s = res.alloc(sizeof(SumPart))) return s;
  const int nb = (int)std::min<int64_t>(kSumBlocks, (t->n_groups + 255) / 256);
  hipLaunchKernelGGL(summary_part, dim3(nb), dim3(256), 0, t->stream, t->d_counts, t->n_groups, (double)num_rows,
                     part.as<SumPart>());
  GHIP(hipGetLastError());
  hipLaunchKernelGGL(summary_final, dim3(1), dim3(64), 0, t->stream, part.as<SumPart>(), nb, res.as<SumPart>());
  GHIP(hipGetLastError());
  SumPart h{};
  GHIP(hipMemcpyAsync(&h, res.p, sizeof(h), hipMemcpyDeviceToHost, t->stream));
  GHIP(hipStreamSynchronize(t->stream));
  out->num_unique = h.unique;
  out->entropy = h.ent;
  return DQ_OK;
}

int64_t dq_freq_num_groups(const dq_freq_table* t) { return t ? t->n_groups : -1; }

dq_status dq_freq_export(const dq_freq_table* t, uint64_t* keys, int64_t* counts, int64_t cap) {
  if (!t || cap < t->n_groups || (t->n_groups > 0 && (!keys || !counts)))
    return set_error(DQ_E_INVALID, "dq_freq_export: bad arguments");
  GHIP(hipSetDevice(t->device));
  if (t->n_groups > 0) {
    GHIP(hipMemcpyAsync(keys, t->d_keys, t->n_groups * 8, hipMemcpyDeviceToHost, t->stream));
    GHIP(hipMemcpyAsync(counts, t->d_counts, t->n_groups * 8, hipMemcpyDeviceToHost, t->stream));
  }
  GHIP(hipStreamSynchronize(t->stream));
  return DQ_OK;
}

void dq_freq_destroy(dq_freq_table* t) { delete t; }

dq_status dq_freq_top(const dq_freq_table* t, int32_t n, uint64_t* keys, int64_t* counts, uint64_t* rep_rows,
                      int32_t* n_out) {
  if (!t || n < 0 || !n_out || (n > 0 && (!keys || !counts || !rep_rows)))
    return set_error(DQ_E_INVALID, "dq_freq_top: bad arguments");
  const int32_t m = (int32_t)std::min<int64_t>(n, t->n_groups);
  *n_out = m;
  if (m == 0) return DQ_OK;
  GHIP(hipSetDevice(t->device));
  std::lock_guard<std::mutex> lock(g_arena_mu);
  const int D = t->device;
  const int64_t G = t->n_groups;
  DevBuf idx(D, 50), sidx(D, 51), sc(D, 52), tmp(D, 53), ok(D, 54), oc(D, 55), orp(D, 56);
  if (dq_status s = idx.alloc(G * 4)) return s;
  if (dq_status s = sidx.alloc(G * 4)) return s;
  if (dq_status s = sc.alloc(G * 8)) return s;
  for (DevBuf* b : {&ok, &oc, &orp})
    if (dq_status s = b->alloc((size_t)m * 8)) return s;
  hipLaunchKernelGGL(iota_u32, dim3(grid_for(G)), dim3(256), 0, t->stream, idx.as<uint32_t>(), G);
  GHIP(hipGetLastError());
  // counts descending, ties in key order (stable radix sort over groups already in key order); every count is in
  // [1, n_values], so the bits above n_values' highest set bit are zero in all of them
  const int end_bit = t->n_values > 0 ? 64 - __builtin_clzll((unsigned long long)t->n_values) : 1;
  const size_t tb = prim::sort_temp_bytes(G, 4);
  if (dq_status s = tmp.alloc(tb)) return s;
  GHIP(prim::sort_pairs(reinterpret_cast<const uint64_t*>(t->d_counts), sc.as<uint64_t>(), idx.as<uint32_t>(),
                        sidx.as<uint32_t>(), 4, G, 0, end_bit, true, tmp.p, tb, t->stream));
  hipLaunchKernelGGL(gather_top, dim3((m + 255) / 256), dim3(256), 0, t->stream, sidx.as<uint32_t>(), m, t->d_keys,
                     t->d_counts, t->d_rep, ok.as<uint64_t>(), oc.as<int64_t>(), orp.as<uint64_t>());
  GHIP(hipGetLastError());
  GHIP(hipMemcpyAsync(keys, ok.p, (size_t)m * 8, hipMemcpyDeviceToHost, t->stream));
  GHIP(hipMemcpyAsync(counts, oc.p, (size_t)m * 8, hipMemcpyDeviceToHost, t->stream));
  GHIP(hipMemcpyAsync(rep_rows, orp.p, (size_t)m * 8, hipMemcpyDeviceToHost, t->stream));
  GHIP(hipStreamSynchronize(t->stream));
  return DQ_OK;
}

}  // extern "C"
