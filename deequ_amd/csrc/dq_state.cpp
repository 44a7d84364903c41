// dq_state.cpp -- host-side state algebra of the C ABI (pure C++, no device code).
//
// Reference (paths relative to src/main/scala/com/amazon/deequ/):
//   State.sum of every hot-path state          analyzers/{Size,Sum,Mean,StandardDeviation,Minimum,
//                                              Maximum,Correlation,ApproxCountDistinct}.scala,
//                                              analyzers/Analyzer.scala:220-234
//   Analyzers.merge (Option semantics)         analyzers/Analyzer.scala:343-362
//   fromAggregationResult null rules           analyzers/Analyzer.scala:244-252, 365-379 and per analyzer
//   HLL++ merge / count / estimateBias         analyzers/catalyst/StatefulHyperloglogPlus.scala:188-297
//   HdfsStateProvider byte images, identifier  analyzers/StateProvider.scala:81-83, 176-294
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>

#include "dq_internal.h"

#include "hll_p9_tables.inc"
#define DQ_DEC_TABLE static const
#include "dq_dec_tables.inc"
#undef DQ_DEC_TABLE

namespace dq {

// ---------------------------------------------------------------------------------------------
// Java numeric semantics
// ---------------------------------------------------------------------------------------------

static inline bool is_nan(double x) { return x != x; }

// java.lang.Math.min / max(double, double): NaN propagates, -0.0 < +0.0.
double java_min(double a, double b) {
  if (is_nan(a)) return a;
  if (is_nan(b)) return b;
  if (a == 0.0 && b == 0.0) return std::signbit(a) ? a : b;
  return a <= b ? a : b;
}
double java_max(double a, double b) {
  if (is_nan(a)) return a;
  if (is_nan(b)) return b;
  if (a == 0.0 && b == 0.0) return std::signbit(a) ? b : a;
  return a >= b ? a : b;
}

// Spark ordering for double min/max aggregates: NaN is larger than every other value.
static inline bool nan_safe_lt(double a, double b) {
  bool an = is_nan(a), bn = is_nan(b);
  if (an || bn) return !an && bn;
  return a < b;
}

// java.lang.Math.round(double) -> long (JDK 8 bit algorithm = floor(a + 1/2) exactly).
int64_t java_math_round(double a) {
  if (is_nan(a)) return 0;
  int64_t bits;
  std::memcpy(&bits, &a, 8);
  int64_t biased_exp = (bits & 0x7FF0000000000000LL) >> 52;
  int64_t shift = (52 - 1 + 1023) - biased_exp;
  if ((shift & -64) == 0) {
    int64_t r = (bits & 0x000FFFFFFFFFFFFFLL) | 0x0010000000000000LL;
    if (bits < 0) r = -r;
    return ((r >> shift) + 1) >> 1;
  }
  if (a >= 9.223372036854775807e18) return std::numeric_limits<int64_t>::max();
  if (a <= -9.223372036854775808e18) return std::numeric_limits<int64_t>::min();
  return (int64_t)a;
}

// ---------------------------------------------------------------------------------------------
// HLL++ words (52 x u64, 10 six-bit registers per word)
// ---------------------------------------------------------------------------------------------

void hll_registers_to_words(const uint8_t* regs512, int64_t* words52) {
  uint64_t w[kHllWords] = {0};
  for (int i = 0; i < kHllM; ++i) {
    int wo = i / kHllRegsPerWord;
    int shift = kHllRegisterBits * (i - wo * kHllRegsPerWord);
    w[wo] |= (uint64_t)(regs512[i] & 63u) << shift;
  }
  for (int i = 0; i < kHllWords; ++i) words52[i] = (int64_t)w[i];
}

// DeequHyperLogLogPlusPlusUtils.merge (:188-208)
static void hll_merge_words(const int64_t* a, const int64_t* b, int64_t* out) {
  int idx = 0;
  for (int wo = 0; wo < kHllWords; ++wo) {
    uint64_t w1 = (uint64_t)a[wo], w2 = (uint64_t)b[wo], word = 0, mask = 63;
    for (int i = 0; idx < kHllM && i < kHllRegsPerWord; ++i, ++idx) {
      uint64_t x = w1 & mask, y = w2 & mask;
      word |= x > y ? x : y;
      mask <<= kHllRegisterBits;
    }
    out[wo] = (int64_t)word;
  }
}

// estimateBias (:259-297), Arrays.binarySearch semantics.
static double hll_estimate_bias(double e) {
  const double* est = kHllRawEstimateP9;
  const int n = kHllP9Points;
  int lo = 0, hi = n - 1, nearest = -1;
  while (lo <= hi) {
    int mid = (int)((unsigned)(lo + hi) >> 1);
    double v = est[mid];
    if (v < e) lo = mid + 1;
    else if (v > e) hi = mid - 1;
    else { nearest = mid; break; }
  }
  if (nearest < 0) nearest = lo;
  auto distance = [&](int i) { double d = e - est[i]; return d * d; };
  int low = nearest - kHllK + 1;
  if (low < 0) low = 0;
  int high = low + kHllK < n ? low + kHllK : n;
  while (high < n && distance(high) < distance(low)) { ++low; ++high; }
  double s = 0.0;
  for (int i = low; i < high; ++i) s += kHllBiasP9[i];
  return s / (double)(high - low);
}

// count (:210-257), including the JVM `1 << Midx` Int shift (count masked to 5 bits).
double hll_count(const int64_t* words52) {
  double z_inverse = 0.0, V = 0.0;
  int idx = 0;
  for (int wo = 0; wo < kHllWords; ++wo) {
    uint64_t word = (uint64_t)words52[wo];
    int shift = 0;
    for (int i = 0; idx < kHllM && i < kHllRegsPerWord; ++i, ++idx) {
      uint64_t m = (word >> shift) & 63u;
      int32_t denom = (int32_t)(1u << (unsigned)(m & 31));
      z_inverse += 1.0 / (double)denom;
      if (m == 0) V += 1.0;
      shift += kHllRegisterBits;
    }
  }
  const double M = (double)kHllM;
  const double alpha_m2 = (0.7213 / (1.0 + 1.079 / M)) * M * M;
  auto e_bias_corrected = [&]() {
    double e = alpha_m2 / z_inverse;
    if (kHllP < 19 && e < 5.0 * M) return e - hll_estimate_bias(e);
    return e;
  };
  double estimate;
  if (V > 0) {
    double H = M * std::log(M / V);
    estimate = H <= 400.0 /* THRESHOLDS(P - 4) */ ? H : e_bias_corrected();
  } else {
    estimate = e_bias_corrected();
  }
  return (double)java_math_round(estimate);
}

// ---------------------------------------------------------------------------------------------
// State algebra
// ---------------------------------------------------------------------------------------------

static inline int64_t wrap_add(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }

const DecTab& dec_host_tab() {
  static const DecTab t{kDecP10Lo, kDecP10Hi, kDecRcpHi, kDecRcpLo};
  return t;
}

bool dec_sum_value(int64_t lo, int64_t hi, double guard, int s, int digits, double& out) {
  const DecTab& t = dec_host_tab();
  if (s < 0 || s > kDecMaxPrecision || digits < 1 || digits > kDecMaxPrecision) return false;
  // the wrapped 128-bit image is the sum while |sum| < 2^127 (~1.7e38 unscaled): the fp64 guard rules out the rest
  if (!(std::fabs(guard) * std::pow(10.0, s) < 1.6e38)) return false;
  if (dec_mag((uint64_t)lo, (uint64_t)hi) >= dec_p10(t, digits)) return false;
  out = dec_to_double((uint64_t)lo, (uint64_t)hi, s, t);
  return true;
}

// a Sum / Mean state of a DECIMAL128 column holding Spark's NULL (an overflowing decimal sum)
static bool dec_overflow(const dq_state& s) {
  if (s.integral != 2) return false;
  double v;
  if (s.op == DQ_OP_SUM) return !dec_sum_value(s.u.sum.partial, s.u.sum.partial_hi, s.u.sum.guard, s.u.sum.dec_scale,
                                               s.u.sum.dec_digits, v);
  if (s.op == DQ_OP_MEAN)
    return !dec_sum_value(s.u.mean.partial, s.u.mean.partial_hi, s.u.mean.guard, s.u.mean.dec_scale,
                          s.u.mean.dec_digits, v);
  return false;
}

// 128-bit wrapping add of decimal partials
static void dec_add(int64_t alo, int64_t ahi, int64_t blo, int64_t bhi, int64_t& lo, int64_t& hi) {
  const uint64_t l = (uint64_t)alo + (uint64_t)blo;
  hi = (int64_t)((uint64_t)ahi + (uint64_t)bhi + (l < (uint64_t)alo ? 1u : 0u));
  lo = (int64_t)l;
}

int32_t state_is_defined(const dq_state& s) {
  if (!s.has_value[0] || !s.has_value[1]) return 0;
  if (dec_overflow(s)) return 0;  // sum(decimal) overflowed: Spark's NULL
  if (s.op == DQ_OP_STDDEV) return s.u.stddev.n > 0.0;   // StandardDeviation.scala:40-51
  if (s.op == DQ_OP_CORRELATION) return s.u.corr.n > 0.0; // Correlation.scala:66-82
  return 1;
}

// Chan/Welford merge exactly as StandardDeviationState.sum / CentralMomentAgg.mergeExpressions.
static void stddev_sum(const dq_state& a, const dq_state& b, dq_state& o) {
  double n = a.u.stddev.n, on = b.u.stddev.n;
  double newN = n + on;
  double delta = b.u.stddev.avg - a.u.stddev.avg;
  double deltaN = newN == 0.0 ? 0.0 : delta / newN;
  o.u.stddev.avg = a.u.stddev.avg + deltaN * on;
  o.u.stddev.m2 = a.u.stddev.m2 + b.u.stddev.m2 + delta * deltaN * n * on;
  o.u.stddev.n = newN;
}

// CorrelationState.sum (Correlation.scala:37-52) == Corr.mergeExpressions.
static void corr_sum(const dq_state& a, const dq_state& b, dq_state& o) {
  double n1 = a.u.corr.n, n2 = b.u.corr.n, newN = n1 + n2;
  double dx = b.u.corr.x_avg - a.u.corr.x_avg;
  double dxN = newN == 0.0 ? 0.0 : dx / newN;
  double dy = b.u.corr.y_avg - a.u.corr.y_avg;
  double dyN = newN == 0.0 ? 0.0 : dy / newN;
  double xa = a.u.corr.x_avg + dxN * n2, ya = a.u.corr.y_avg + dyN * n2;
  double ck = a.u.corr.ck + b.u.corr.ck + dx * dyN * n1 * n2;
  double xm = a.u.corr.x_mk + b.u.corr.x_mk + dx * dxN * n1 * n2;
  double ym = a.u.corr.y_mk + b.u.corr.y_mk + dy * dyN * n1 * n2;
  o.u.corr.n = newN; o.u.corr.x_avg = xa; o.u.corr.y_avg = ya;
  o.u.corr.ck = ck; o.u.corr.x_mk = xm; o.u.corr.y_mk = ym;
}

// DataTypeHistogram.sum (DataType.scala:48-51) == StatefulDataType.merge (StatefulDataType.scala:71-77).
static void dtype_sum(const dq_state& a, const dq_state& b, dq_state& o) {
  o.u.dtype.num_null = wrap_add(a.u.dtype.num_null, b.u.dtype.num_null);
  o.u.dtype.num_fractional = wrap_add(a.u.dtype.num_fractional, b.u.dtype.num_fractional);
  o.u.dtype.num_integral = wrap_add(a.u.dtype.num_integral, b.u.dtype.num_integral);
  o.u.dtype.num_boolean = wrap_add(a.u.dtype.num_boolean, b.u.dtype.num_boolean);
  o.u.dtype.num_string = wrap_add(a.u.dtype.num_string, b.u.dtype.num_string);
}

// Sum of two DEFINED states (State.sum).
static void state_sum_defined(const dq_state& a, const dq_state& b, dq_state& o) {
  o = a;
  switch (a.op) {
    case DQ_OP_SIZE: o.u.size.num_matches = wrap_add(a.u.size.num_matches, b.u.size.num_matches); break;
    case DQ_OP_COMPLETENESS:
    case DQ_OP_COMPLIANCE:
    case DQ_OP_PATTERN_MATCH:
      o.u.ratio.num_matches = wrap_add(a.u.ratio.num_matches, b.u.ratio.num_matches);
      o.u.ratio.count = wrap_add(a.u.ratio.count, b.u.ratio.count);
      break;
    // State.sum of persisted states: SumState / MeanState hold doubles (Sum.scala:27-29, Mean.scala:27-31)
    case DQ_OP_SUM: o.u.sum.sum = a.u.sum.sum + b.u.sum.sum; o.integral = 0; o.u.sum.partial = 0; break;
    case DQ_OP_MEAN:
      o.u.mean.sum = a.u.mean.sum + b.u.mean.sum;
      o.integral = 0;
      o.u.mean.partial = 0;
      o.u.mean.count = wrap_add(a.u.mean.count, b.u.mean.count);
      break;
    case DQ_OP_STDDEV: stddev_sum(a, b, o); break;
    case DQ_OP_MIN: o.u.minmax.value = java_min(a.u.minmax.value, b.u.minmax.value); break;
    case DQ_OP_MAX: o.u.minmax.value = java_max(a.u.minmax.value, b.u.minmax.value); break;
    case DQ_OP_CORRELATION: corr_sum(a, b, o); break;
    case DQ_OP_APPROX_COUNT_DISTINCT: hll_merge_words(a.u.hll.words, b.u.hll.words, o.u.hll.words); break;
    case DQ_OP_DATATYPE: dtype_sum(a, b, o); break;
  }
}

dq_status state_merge(const dq_state& a, const dq_state& b, dq_state& o) {
  if (a.op != b.op) return set_error(DQ_E_STATE, "dq_state_merge: op mismatch (%d vs %d)", a.op, b.op);
  bool da = state_is_defined(a), db = state_is_defined(b);
  if (da && db) state_sum_defined(a, b, o);
  else if (da) o = a;
  else o = b;  // (None, Some) -> b; (None, None) -> None (b carries has_value = 0)
  return DQ_OK;
}

// Spark partial-aggregate merge, slot by slot, with SQL null skipping.
dq_status state_combine(const dq_state& a, const dq_state& b, dq_state& o) {
  if (a.op != b.op) return set_error(DQ_E_STATE, "dq_state_combine: op mismatch (%d vs %d)", a.op, b.op);
  o = a;
  for (int i = 0; i < 2; ++i) o.has_value[i] = a.has_value[i] | b.has_value[i];
  auto pick = [&](int slot, auto fa, auto fb, auto both) {
    if (a.has_value[slot] && b.has_value[slot]) both();
    else if (b.has_value[slot]) fb();
    else fa();
  };
  switch (a.op) {
    case DQ_OP_SIZE:
      pick(0, [] {}, [&] { o.u.size = b.u.size; },
           [&] { o.u.size.num_matches = wrap_add(a.u.size.num_matches, b.u.size.num_matches); });
      break;
    case DQ_OP_COMPLETENESS:
    case DQ_OP_COMPLIANCE:
    case DQ_OP_PATTERN_MATCH:
      pick(0, [] {}, [&] { o.u.ratio.num_matches = b.u.ratio.num_matches; },
           [&] { o.u.ratio.num_matches = wrap_add(a.u.ratio.num_matches, b.u.ratio.num_matches); });
      pick(1, [] {}, [&] { o.u.ratio.count = b.u.ratio.count; },
           [&] { o.u.ratio.count = wrap_add(a.u.ratio.count, b.u.ratio.count); });
      break;
    // integral columns: Spark's partial buffers hold the LongType sum, the final merge adds them (wrapping)
    // and the CAST to double comes last -- adding the cast doubles would differ once a shard's sum wraps.
    // A partial that is already a double (a deserialized or Analyzers.merge-d state: SumState / MeanState
    // hold doubles, Sum.scala:27-29, Mean.scala:27-31) combines by double addition.
    case DQ_OP_SUM:
      pick(0, [] {}, [&] { o.u.sum = b.u.sum; o.integral = b.integral; }, [&] {
        if (a.integral == 2 && b.integral == 2 && a.u.sum.dec_scale == b.u.sum.dec_scale &&
            a.u.sum.dec_digits == b.u.sum.dec_digits) {  // decimal partials: exact sum, cast at the end
          dec_add(a.u.sum.partial, a.u.sum.partial_hi, b.u.sum.partial, b.u.sum.partial_hi, o.u.sum.partial,
                  o.u.sum.partial_hi);
          o.u.sum.guard = a.u.sum.guard + b.u.sum.guard;
          if (!dec_sum_value(o.u.sum.partial, o.u.sum.partial_hi, o.u.sum.guard, o.u.sum.dec_scale,
                             o.u.sum.dec_digits, o.u.sum.sum))
            o.u.sum.sum = std::numeric_limits<double>::quiet_NaN();
        } else if (a.integral == 1 && b.integral == 1) {
          o.u.sum.partial = wrap_add(a.u.sum.partial, b.u.sum.partial);
          o.u.sum.sum = (double)o.u.sum.partial;
        } else {
          o.u.sum.sum = a.u.sum.sum + b.u.sum.sum;
          o.u.sum.partial = 0;
          o.integral = 0;
        }
      });
      break;
    case DQ_OP_MEAN:
      pick(0, [] {}, [&] {
             const int64_t cnt = o.u.mean.count;  // (slot 1, picked below)
             o.u.mean = b.u.mean;
             o.u.mean.count = cnt;
             o.integral = b.integral;
           },
           [&] {
             if (a.integral == 2 && b.integral == 2 && a.u.mean.dec_scale == b.u.mean.dec_scale &&
                 a.u.mean.dec_digits == b.u.mean.dec_digits) {
               dec_add(a.u.mean.partial, a.u.mean.partial_hi, b.u.mean.partial, b.u.mean.partial_hi, o.u.mean.partial,
                       o.u.mean.partial_hi);
               o.u.mean.guard = a.u.mean.guard + b.u.mean.guard;
               if (!dec_sum_value(o.u.mean.partial, o.u.mean.partial_hi, o.u.mean.guard, o.u.mean.dec_scale,
                                  o.u.mean.dec_digits, o.u.mean.sum))
                 o.u.mean.sum = std::numeric_limits<double>::quiet_NaN();
             } else if (a.integral == 1 && b.integral == 1) {
               o.u.mean.partial = wrap_add(a.u.mean.partial, b.u.mean.partial);
               o.u.mean.sum = (double)o.u.mean.partial;
             } else {
               o.u.mean.sum = a.u.mean.sum + b.u.mean.sum;
               o.u.mean.partial = 0;
               o.integral = 0;
             }
           });
      pick(1, [] {}, [&] { o.u.mean.count = b.u.mean.count; },
           [&] { o.u.mean.count = wrap_add(a.u.mean.count, b.u.mean.count); });
      break;
    case DQ_OP_STDDEV:
      stddev_sum(a, b, o);
      break;
    case DQ_OP_MIN:
      pick(0, [] {}, [&] { o.u.minmax = b.u.minmax; }, [&] {
        o.u.minmax.value = nan_safe_lt(b.u.minmax.value, a.u.minmax.value) ? b.u.minmax.value : a.u.minmax.value;
      });
      break;
    case DQ_OP_MAX:
      pick(0, [] {}, [&] { o.u.minmax = b.u.minmax; }, [&] {
        o.u.minmax.value = nan_safe_lt(a.u.minmax.value, b.u.minmax.value) ? b.u.minmax.value : a.u.minmax.value;
      });
      break;
    case DQ_OP_CORRELATION:
      corr_sum(a, b, o);
      break;
    case DQ_OP_APPROX_COUNT_DISTINCT:
      hll_merge_words(a.u.hll.words, b.u.hll.words, o.u.hll.words);
      break;
    case DQ_OP_DATATYPE:  // the UDAF buffer is never NULL: partial buffers add field by field
      dtype_sum(a, b, o);
      break;
    default:
      return set_error(DQ_E_STATE, "dq_state_combine: bad op %d", a.op);
  }
  return DQ_OK;
}

static inline double jdiv(double a, double b) { return a / b; }  // IEEE, as the JVM

dq_status state_metric(const dq_state& s, double& out) {
  if (!state_is_defined(s)) return set_error(DQ_E_STATE, "dq_state_metric: state is empty (None)");
  switch (s.op) {
    case DQ_OP_SIZE: out = (double)s.u.size.num_matches; break;
    case DQ_OP_COMPLETENESS:
    case DQ_OP_COMPLIANCE:
    case DQ_OP_PATTERN_MATCH:
      out = s.u.ratio.count == 0 ? std::numeric_limits<double>::quiet_NaN()
                                 : jdiv((double)s.u.ratio.num_matches, (double)s.u.ratio.count);
      break;
    case DQ_OP_SUM: out = s.u.sum.sum; break;
    case DQ_OP_MEAN:
      out = s.u.mean.count == 0 ? std::numeric_limits<double>::quiet_NaN()
                                : jdiv(s.u.mean.sum, (double)s.u.mean.count);
      break;
    case DQ_OP_STDDEV: out = std::sqrt(s.u.stddev.m2 / s.u.stddev.n); break;
    case DQ_OP_MIN:
    case DQ_OP_MAX: out = s.u.minmax.value; break;
    case DQ_OP_CORRELATION: out = s.u.corr.ck / std::sqrt(s.u.corr.x_mk * s.u.corr.y_mk); break;
    case DQ_OP_APPROX_COUNT_DISTINCT: out = hll_count(s.u.hll.words); break;
    case DQ_OP_DATATYPE:
      return set_error(DQ_E_STATE, "dq_state_metric: DataType yields a HistogramMetric, not a double");
    default: return set_error(DQ_E_STATE, "dq_state_metric: bad op %d", s.op);
  }
  return DQ_OK;
}

// ---------------------------------------------------------------------------------------------
// HdfsStateProvider byte images (Java DataOutputStream, big-endian)
// ---------------------------------------------------------------------------------------------

static inline void put_be64(uint8_t* p, uint64_t v) {
  for (int i = 7; i >= 0; --i) { p[i] = (uint8_t)(v & 0xFF); v >>= 8; }
}
static inline uint64_t get_be64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
  return v;
}
static inline uint64_t dbits(double d) { uint64_t u; std::memcpy(&u, &d, 8); return u; }
static inline double bitsd(uint64_t u) { double d; std::memcpy(&d, &u, 8); return d; }

int64_t state_to_bytes(const dq_state& s, uint8_t* buf, int64_t cap) {
  uint8_t tmp[8 * 6 + 4 + 416];
  int64_t n = 0;
  auto w64 = [&](uint64_t v) { put_be64(tmp + n, v); n += 8; };
  switch (s.op) {
    case DQ_OP_SIZE: w64((uint64_t)s.u.size.num_matches); break;                  // persistLongState
    case DQ_OP_COMPLETENESS:
    case DQ_OP_COMPLIANCE:
    case DQ_OP_PATTERN_MATCH: w64((uint64_t)s.u.ratio.num_matches); w64((uint64_t)s.u.ratio.count); break;
    case DQ_OP_SUM: w64(dbits(s.u.sum.sum)); break;                               // persistDoubleState
    case DQ_OP_MEAN: w64(dbits(s.u.mean.sum)); w64((uint64_t)s.u.mean.count); break;
    case DQ_OP_MIN:
    case DQ_OP_MAX: w64(dbits(s.u.minmax.value)); break;
    case DQ_OP_STDDEV: w64(dbits(s.u.stddev.n)); w64(dbits(s.u.stddev.avg)); w64(dbits(s.u.stddev.m2)); break;
    case DQ_OP_CORRELATION:
      w64(dbits(s.u.corr.n)); w64(dbits(s.u.corr.x_avg)); w64(dbits(s.u.corr.y_avg));
      w64(dbits(s.u.corr.ck)); w64(dbits(s.u.corr.x_mk)); w64(dbits(s.u.corr.y_mk));
      break;
    case DQ_OP_APPROX_COUNT_DISTINCT:  // persistBytes: int length + wordsToBytes (big-endian longs)
      tmp[0] = 0; tmp[1] = 0; tmp[2] = (416 >> 8) & 0xFF; tmp[3] = 416 & 0xFF;
      n = 4;
      for (int i = 0; i < kHllWords; ++i) w64((uint64_t)s.u.hll.words[i]);
      break;
    case DQ_OP_DATATYPE:  // persistBytes(DataTypeHistogram.toBytes(...)): int length 40 + 5 big-endian longs
      tmp[0] = 0; tmp[1] = 0; tmp[2] = 0; tmp[3] = 40;
      n = 4;
      w64((uint64_t)s.u.dtype.num_null); w64((uint64_t)s.u.dtype.num_fractional);
      w64((uint64_t)s.u.dtype.num_integral); w64((uint64_t)s.u.dtype.num_boolean);
      w64((uint64_t)s.u.dtype.num_string);
      break;
    default: return set_error(DQ_E_STATE, "dq_state_to_bytes: bad op %d", s.op);
  }
  if (buf && cap >= n) std::memcpy(buf, tmp, (size_t)n);
  return n;
}

dq_status state_from_bytes(int32_t op, const uint8_t* buf, int64_t len, dq_state& o) {
  std::memset(&o, 0, sizeof(o));
  o.op = op;
  o.has_value[0] = o.has_value[1] = 1;
  auto need = [&](int64_t k) { return len == k; };
  int64_t p = 0;
  auto r64 = [&]() { uint64_t v = get_be64(buf + p); p += 8; return v; };
  switch (op) {
    case DQ_OP_SIZE:
      if (!need(8)) break;
      o.u.size.num_matches = (int64_t)r64(); return DQ_OK;
    case DQ_OP_COMPLETENESS:
    case DQ_OP_COMPLIANCE:
    case DQ_OP_PATTERN_MATCH:
      if (!need(16)) break;
      o.u.ratio.num_matches = (int64_t)r64(); o.u.ratio.count = (int64_t)r64(); return DQ_OK;
    case DQ_OP_SUM:
      if (!need(8)) break;
      o.u.sum.sum = bitsd(r64()); return DQ_OK;
    case DQ_OP_MEAN:
      if (!need(16)) break;
      o.u.mean.sum = bitsd(r64()); o.u.mean.count = (int64_t)r64(); return DQ_OK;
    case DQ_OP_MIN:
    case DQ_OP_MAX:
      if (!need(8)) break;
      o.u.minmax.value = bitsd(r64()); return DQ_OK;
    case DQ_OP_STDDEV:
      if (!need(24)) break;
      o.u.stddev.n = bitsd(r64()); o.u.stddev.avg = bitsd(r64()); o.u.stddev.m2 = bitsd(r64());
      return DQ_OK;
    case DQ_OP_CORRELATION:
      if (!need(48)) break;
      o.u.corr.n = bitsd(r64()); o.u.corr.x_avg = bitsd(r64()); o.u.corr.y_avg = bitsd(r64());
      o.u.corr.ck = bitsd(r64()); o.u.corr.x_mk = bitsd(r64()); o.u.corr.y_mk = bitsd(r64());
      return DQ_OK;
    case DQ_OP_APPROX_COUNT_DISTINCT: {
      if (len != 4 + 416) break;
      int32_t l = (int32_t)(((uint32_t)buf[0] << 24) | ((uint32_t)buf[1] << 16) | ((uint32_t)buf[2] << 8) | buf[3]);
      if (l != 416) break;  // wordsFromBytes: require(bytes.length == NUM_WORDS * 8)
      p = 4;
      for (int i = 0; i < kHllWords; ++i) o.u.hll.words[i] = (int64_t)r64();
      return DQ_OK;
    }
    case DQ_OP_DATATYPE: {
      if (len != 4 + 40) break;
      if (buf[0] != 0 || buf[1] != 0 || buf[2] != 0 || buf[3] != 40) break;  // fromBytes: require(length == 40)
      p = 4;
      o.u.dtype.num_null = (int64_t)r64(); o.u.dtype.num_fractional = (int64_t)r64();
      o.u.dtype.num_integral = (int64_t)r64(); o.u.dtype.num_boolean = (int64_t)r64();
      o.u.dtype.num_string = (int64_t)r64();
      return DQ_OK;
    }
    default:
      return set_error(DQ_E_STATE, "dq_state_from_bytes: bad op %d", op);
  }
  return set_error(DQ_E_STATE, "dq_state_from_bytes: bad image length %lld for op %d", (long long)len, op);
}

// scala.util.hashing.MurmurHash3.stringHash(s, 42) over UTF-16 code units.
static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static inline uint32_t mix_last(uint32_t h, uint32_t k) {
  k *= 0xCC9E2D51u; k = rotl32(k, 15); k *= 0x1B873593u; return h ^ k;
}
static inline uint32_t mix(uint32_t h, uint32_t k) {
  h = mix_last(h, k); h = rotl32(h, 13); return h * 5u + 0xE6546B64u;
}

int32_t murmur3_string_hash_utf8(const char* s, uint32_t seed) {
  // decode UTF-8 -> UTF-16 code units
  const unsigned char* p = (const unsigned char*)s;
  uint32_t units_buf[1024];
  uint32_t* units = units_buf;
  size_t len = std::strlen(s), cap = 1024, n = 0;
  uint32_t* heap = nullptr;
  if (len * 2 + 2 > cap) { heap = new uint32_t[len * 2 + 2]; units = heap; }
  size_t i = 0;
  while (i < len) {
    uint32_t cp;
    unsigned char c = p[i];
    if (c < 0x80) { cp = c; i += 1; }
    else if ((c >> 5) == 6 && i + 1 < len) { cp = ((c & 0x1Fu) << 6) | (p[i + 1] & 0x3Fu); i += 2; }
    else if ((c >> 4) == 14 && i + 2 < len) { cp = ((c & 0x0Fu) << 12) | ((p[i + 1] & 0x3Fu) << 6) | (p[i + 2] & 0x3Fu); i += 3; }
    else if (i + 3 < len) {
      cp = ((c & 0x07u) << 18) | ((p[i + 1] & 0x3Fu) << 12) | ((p[i + 2] & 0x3Fu) << 6) | (p[i + 3] & 0x3Fu);
      i += 4;
    } else { cp = 0xFFFD; i += 1; }
    if (cp >= 0x10000) { cp -= 0x10000; units[n++] = 0xD800 + (cp >> 10); units[n++] = 0xDC00 + (cp & 0x3FF); }
    else units[n++] = cp;
  }
  uint32_t h = seed;
  size_t k = 0;
  while (k + 1 < n) { h = mix(h, (units[k] << 16) + units[k + 1]); k += 2; }
  if (k < n) h = mix_last(h, units[k]);
  h ^= (uint32_t)n;
  h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
  delete[] heap;
  return (int32_t)h;
}

}  // namespace dq

// ---------------------------------------------------------------------------------------------
// C ABI wrappers
// ---------------------------------------------------------------------------------------------
extern "C" {

dq_status dq_state_merge(const dq_state* a, const dq_state* b, dq_state* out) {
  if (!a || !b || !out) return dq::set_error(DQ_E_INVALID, "dq_state_merge: null argument");
  dq_state tmp;
  dq_status st = dq::state_merge(*a, *b, tmp);
  if (st == DQ_OK) *out = tmp;
  return st;
}

dq_status dq_state_combine(const dq_state* a, const dq_state* b, dq_state* out) {
  if (!a || !b || !out) return dq::set_error(DQ_E_INVALID, "dq_state_combine: null argument");
  dq_state tmp;
  dq_status st = dq::state_combine(*a, *b, tmp);
  if (st == DQ_OK) *out = tmp;
  return st;
}

dq_status dq_state_merge_n(const dq_state* a, const dq_state* b, int32_t n, dq_state* out) {
  if (n < 0 || (n > 0 && (!a || !b || !out))) return dq::set_error(DQ_E_INVALID, "dq_state_merge_n: bad arguments");
  for (int32_t i = 0; i < n; ++i)
    if (dq_status st = dq_state_merge(a + i, b + i, out + i)) return st;
  return DQ_OK;
}

dq_status dq_state_combine_n(const dq_state* a, const dq_state* b, int32_t n, dq_state* out) {
  if (n < 0 || (n > 0 && (!a || !b || !out))) return dq::set_error(DQ_E_INVALID, "dq_state_combine_n: bad arguments");
  for (int32_t i = 0; i < n; ++i)
    if (dq_status st = dq_state_combine(a + i, b + i, out + i)) return st;
  return DQ_OK;
}

int32_t dq_state_is_defined(const dq_state* s) { return s ? dq::state_is_defined(*s) : 0; }

dq_status dq_state_metric(const dq_state* s, double* out) {
  if (!s || !out) return dq::set_error(DQ_E_INVALID, "dq_state_metric: null argument");
  return dq::state_metric(*s, *out);
}

dq_status dq_hll_estimate(const int64_t* words52, double* out) {
  if (!words52 || !out) return dq::set_error(DQ_E_INVALID, "dq_hll_estimate: null argument");
  *out = dq::hll_count(words52);
  return DQ_OK;
}

int64_t dq_state_to_bytes(const dq_state* s, uint8_t* buf, int64_t cap) {
  if (!s) return dq::set_error(DQ_E_INVALID, "dq_state_to_bytes: null state");
  return dq::state_to_bytes(*s, buf, cap);
}

dq_status dq_state_from_bytes(int32_t op, const uint8_t* buf, int64_t len, dq_state* out) {
  if (!buf || !out) return dq::set_error(DQ_E_INVALID, "dq_state_from_bytes: null argument");
  return dq::state_from_bytes(op, buf, len, *out);
}

int32_t dq_state_identifier(const char* s) { return s ? dq::murmur3_string_hash_utf8(s, 42u) : 0; }

}  // extern "C"
