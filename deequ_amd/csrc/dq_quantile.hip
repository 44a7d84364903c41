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
#include <cstring>
#include <vector>

#include "dq_internal.h"

namespace dq {
namespace {

constexpr int kQBlock = 256;
constexpr int kQBins = 2048;  // 11-bit digits
constexpr int kQRowsPerThread = 8;
constexpr int kQPasses = 6;
constexpr int kQShift[kQPasses] = {53, 42, 31, 20, 9, 0};
constexpr int kQWidth[kQPasses] = {11, 11, 11, 11, 11, 9};

struct QSelect {
  uint64_t prefix[DQ_MAX_QUANTILES];
  uint64_t pmask[DQ_MAX_QUANTILES];
};

__device__ __forceinline__ uint64_t order_key_f64(uint64_t b) {
  if ((b & 0x7FFFFFFFFFFFFFFFull) > 0x7FF0000000000000ull) b = 0x7FF8000000000000ull;  // NaN canonical
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

template <int TYPE>
__global__ __launch_bounds__(kQBlock) void dq_quantile_hist(const void* __restrict__ values,
                                                            const uint32_t* __restrict__ validity, int64_t n,
                                                            int32_t shift, uint32_t dmask, int32_t nq, QSelect sel,
                                                            unsigned long long* __restrict__ hist) {
  extern __shared__ uint32_t lds_hist[];  // nq x kQBins
  for (int i = threadIdx.x; i < nq * kQBins; i += kQBlock) lds_hist[i] = 0;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * kQBlock;
  for (int64_t r0 = (int64_t)blockIdx.x * kQBlock + threadIdx.x; r0 < n; r0 += stride * kQRowsPerThread) {
    uint64_t key[kQRowsPerThread];
    bool ok[kQRowsPerThread];
#pragma unroll
    for (int j = 0; j < kQRowsPerThread; ++j) {
      const int64_t r = r0 + j * stride;
      ok[j] = r < n;
      uint64_t k = 0;
      if (ok[j]) {
        if constexpr (TYPE == DQ_TYPE_F64)
          k = order_key_f64(__builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(values) + r));
        else if constexpr (TYPE == DQ_TYPE_I64)
          k = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(values) + r) ^ 0x8000000000000000ull;
        else
          k = (uint64_t)(int64_t)__builtin_nontemporal_load(reinterpret_cast<const int32_t*>(values) + r) ^
              0x8000000000000000ull;
        if (validity) ok[j] = (validity[r >> 5] >> (r & 31)) & 1u;
      }
      key[j] = k;
    }
#pragma unroll
    for (int j = 0; j < kQRowsPerThread; ++j) {
      const uint32_t d = (uint32_t)(key[j] >> shift) & dmask;
      for (int q = 0; q < nq; ++q)
        if (ok[j] && (key[j] & sel.pmask[q]) == sel.prefix[q]) atomicAdd(&lds_hist[q * kQBins + d], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nq * kQBins; i += kQBlock)
    if (lds_hist[i]) atomicAdd(&hist[i], (unsigned long long)lds_hist[i]);
}

#define QHIP(x)                                                                             \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) return set_error(DQ_E_HIP, "%s: %s", #x, hipGetErrorString(e_)); \
  } while (0)

struct DevHist {
  unsigned long long* p = nullptr;
  ~DevHist() {
    if (p) (void)hipFree(p);
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
  for (int pass = 0; pass < kQPasses; ++pass) {
    QHIP(hipMemsetAsync(dh.p, 0, hist_bytes, stream));
    for (int c = 0; c < n_chunks; ++c) {
      const int64_t rows = chunk_rows[c];
      if (rows == 0) continue;
      const int64_t per_block = (int64_t)kQBlock * kQRowsPerThread;
      const int grid = (int)std::min<int64_t>(8192, (rows + per_block - 1) / per_block);
      const auto* val = reinterpret_cast<const uint32_t*>(cols[c].validity);
      const uint32_t dmask = (1u << kQWidth[pass]) - 1u;
      const size_t lds = (size_t)n_q * kQBins * sizeof(uint32_t);
      if (type == DQ_TYPE_F64)
        hipLaunchKernelGGL(dq_quantile_hist<DQ_TYPE_F64>, dim3(grid), dim3(kQBlock), lds, stream, cols[c].values, val,
                           rows, kQShift[pass], dmask, n_q, sel, dh.p);
      else if (type == DQ_TYPE_I64)
        hipLaunchKernelGGL(dq_quantile_hist<DQ_TYPE_I64>, dim3(grid), dim3(kQBlock), lds, stream, cols[c].values, val,
                           rows, kQShift[pass], dmask, n_q, sel, dh.p);
      else
        hipLaunchKernelGGL(dq_quantile_hist<DQ_TYPE_I32>, dim3(grid), dim3(kQBlock), lds, stream, cols[c].values, val,
                           rows, kQShift[pass], dmask, n_q, sel, dh.p);
      QHIP(hipGetLastError());
    }
    QHIP(hipMemcpyAsync(h.data(), dh.p, hist_bytes, hipMemcpyDeviceToHost, stream));
    QHIP(hipStreamSynchronize(stream));
    if (pass == 0) {
      for (int b = 0; b < kQBins; ++b) n += (int64_t)h[b];  // every non-null row matches the empty prefix
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
      const unsigned long long* hq = h.data() + (size_t)q * kQBins;
      int64_t cum = 0;
      int b = 0;
      for (; b < (int)dmask; ++b) {
        if (cum + (int64_t)hq[b] >= rank[q]) break;
        cum += (int64_t)hq[b];
      }
      if (cum + (int64_t)hq[b] < rank[q])
        return set_error(DQ_E_HIP, "dq_approx_quantiles: histogram of pass %d lost rows (data changed?)", pass);
      rank[q] -= cum;
      sel.prefix[q] |= (uint64_t)b << kQShift[pass];
      sel.pmask[q] |= dmask << kQShift[pass];
    }
  }
  for (int q = 0; q < n_q; ++q) out[q] = key_to_double(type, sel.prefix[q]);
  return DQ_OK;
}

}  // extern "C"
