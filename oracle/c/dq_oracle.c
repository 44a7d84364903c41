/*
 * dq_oracle.c -- CPU restatement of Deequ's scan semantics in C.  TEST INFRASTRUCTURE ONLY.
 *
 * Used by tests/ (parity at sizes the pure-Python oracle is too slow for) and by bench.py's
 * cpu_baseline leg.  Never linked into, called by, or shipped with the product library.
 * Compiled with -ffp-contract=off so every fp64 operation rounds exactly as the JVM's does.
 *
 * Semantics restated (reference paths relative to src/main/scala/com/amazon/deequ/):
 *   - Spark partial aggregation per partition + ordered final merge from the zero buffer:
 *       StandardDeviation -> CentralMomentAgg update/merge (analyzers/StandardDeviation.scala:37-44,
 *       analyzers/catalyst/StatefulStdDevPop.scala:24-34), Correlation -> Corr update/merge
 *       (analyzers/Correlation.scala:37-52, analyzers/catalyst/StatefulCorrelation.scala:24-49);
 *   - sum/count/min/max (analyzers/{Sum,Mean,Minimum,Maximum}.scala): integral sums wrap in
 *       int64, doubles summed sequentially, min/max with NaN ordered as the largest value;
 *   - HLL++ register update with XXH64 seed 42 (analyzers/catalyst/StatefulHyperloglogPlus.scala:89-115).
 * Same semantics as oracle/dq_oracle.py; tests check the two agree.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

enum { K_F64 = 1, K_I64 = 2, K_I32 = 3, K_UTF8 = 4, K_LARGE_UTF8 = 5,
       /* round 6: FloatType, ShortType, ByteType, BooleanType (LSB-first bit-packed values) */
       K_F32 = 6, K_I16 = 7, K_I8 = 8, K_BOOL = 9 };

#define P1 0x9E3779B185EBCA87ULL
#define P2 0xC2B2AE3D27D4EB4FULL
#define P3 0x165667B19E3779F9ULL
#define P4 0x85EBCA77C2B2AE63ULL
#define P5 0x27D4EB2F165667C5ULL

static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t fmix64(uint64_t h) {
  h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32; return h;
}
static inline uint64_t rd64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline uint32_t rd32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }

uint64_t dqo_xxh64_long(int64_t v, uint64_t seed) {
  uint64_t h = seed + P5 + 8;
  h ^= rotl64((uint64_t)v * P2, 31) * P1;
  h = rotl64(h, 27) * P1 + P4;
  return fmix64(h);
}

uint64_t dqo_xxh64_int(int32_t v, uint64_t seed) {
  uint64_t h = seed + P5 + 4;
  h ^= (uint64_t)(uint32_t)v * P1;
  h = rotl64(h, 23) * P2 + P3;
  return fmix64(h);
}

uint64_t dqo_xxh64_bytes(const uint8_t* p, int64_t n, uint64_t seed) {
  int64_t off = 0;
  uint64_t h;
  if (n >= 32) {
    uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    for (; off <= n - 32; off += 32) {
      v1 = rotl64(v1 + rd64(p + off) * P2, 31) * P1;
      v2 = rotl64(v2 + rd64(p + off + 8) * P2, 31) * P1;
      v3 = rotl64(v3 + rd64(p + off + 16) * P2, 31) * P1;
      v4 = rotl64(v4 + rd64(p + off + 24) * P2, 31) * P1;
    }
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    uint64_t vs[4] = {v1, v2, v3, v4};
    for (int i = 0; i < 4; ++i) {
      uint64_t v = rotl64(vs[i] * P2, 31) * P1;
      h ^= v;
      h = h * P1 + P4;
    }
  } else {
    h = seed + P5;
  }
  h += (uint64_t)n;
  for (; off <= n - 8; off += 8) {
    h ^= rotl64(rd64(p + off) * P2, 31) * P1;
    h = rotl64(h, 27) * P1 + P4;
  }
  if (off + 4 <= n) {
    h ^= (uint64_t)rd32(p + off) * P1;
    h = rotl64(h, 23) * P2 + P3;
    off += 4;
  }
  for (; off < n; ++off) {
    h ^= (uint64_t)p[off] * P5;
    h = rotl64(h, 11) * P1;
  }
  return fmix64(h);
}

static inline int bit(const uint8_t* bm, int64_t i) { return bm ? (bm[i >> 3] >> (i & 7)) & 1 : 1; }

static inline int is_float(int kind) { return kind == K_F64 || kind == K_F32; }
static inline int is_num(int kind) { return kind != K_UTF8 && kind != K_LARGE_UTF8 && kind != K_BOOL; }
/* an integral value widened to long (Spark's Sum of Byte / Short / Int / Long is a LongType sum) */
static inline int64_t as_long(int kind, const void* v, int64_t i) {
  switch (kind) {
    case K_I64: return ((const int64_t*)v)[i];
    case K_I16: return ((const int16_t*)v)[i];
    case K_I8: return ((const int8_t*)v)[i];
    case K_BOOL: return bit((const uint8_t*)v, i);
    default: return ((const int32_t*)v)[i];
  }
}
/* Cast(child, DoubleType): exact for every type here (a float widens exactly) */
static inline double as_double(int kind, const void* v, int64_t i) {
  switch (kind) {
    case K_F64: return ((const double*)v)[i];
    case K_F32: return (double)((const float*)v)[i];
    case K_I64: return (double)((const int64_t*)v)[i];
    default: return (double)as_long(kind, v, i);
  }
}

/* Spark's NaN-safe "a < b" (NaN is larger than every other double). */
static inline int nan_safe_lt(double a, double b) {
  int an = a != a, bn = b != b;
  if (an || bn) return !an && bn;
  return a < b;
}

typedef struct {
  int64_t count;      /* selected rows (non-null and where-true) */
  double sum_f64;     /* Spark sum for double columns (NaN-free order: sequential) */
  int64_t sum_i64;    /* Spark sum for integral columns (wrapping) */
  double n, avg, m2;  /* CentralMomentAgg buffer */
  double min, max;    /* valid iff count > 0 */
  int64_t imin, imax; /* integral min / max */
} dqo_col_stats;

static void stats_partial(int kind, const void* values, const uint8_t* validity, const uint8_t* mask,
                          int64_t lo, int64_t hi, dqo_col_stats* s) {
  memset(s, 0, sizeof(*s));
  int first = 1;
  for (int64_t i = lo; i < hi; ++i) {
    if (!bit(validity, i) || !bit(mask, i)) continue;
    double x = as_double(kind, values, i);
    s->count++;
    if (is_float(kind)) s->sum_f64 += x;
    else s->sum_i64 = (int64_t)((uint64_t)s->sum_i64 + (uint64_t)as_long(kind, values, i));
    /* CentralMomentAgg.updateExpressions */
    double newN = s->n + 1.0;
    double delta = x - s->avg;
    double deltaN = delta / newN;
    s->avg = s->avg + deltaN;
    s->m2 = s->m2 + delta * (delta - deltaN);
    s->n = newN;
    if (is_float(kind)) {
      if (first) { s->min = x; s->max = x; }
      else {
        if (nan_safe_lt(x, s->min)) s->min = x;
        if (nan_safe_lt(s->max, x)) s->max = x;
      }
    } else {
      int64_t iv = as_long(kind, values, i);
      if (first) { s->imin = iv; s->imax = iv; }
      else {
        if (iv < s->imin) s->imin = iv;
        if (iv > s->imax) s->imax = iv;
      }
    }
    first = 0;
  }
}

static void stats_merge(int kind, dqo_col_stats* a, const dqo_col_stats* b) {
  /* Spark final aggregate: CentralMomentAgg.mergeExpressions, sum/min/max merges */
  double n1 = a->n, n2 = b->n, newN = n1 + n2;
  double delta = b->avg - a->avg;
  double deltaN = newN == 0.0 ? 0.0 : delta / newN;
  a->avg = a->avg + deltaN * n2;
  a->m2 = a->m2 + b->m2 + delta * deltaN * n1 * n2;
  a->n = newN;
  if (b->count > 0) {
    if (a->count == 0) {
      a->sum_f64 = b->sum_f64; a->sum_i64 = b->sum_i64;
      a->min = b->min; a->max = b->max; a->imin = b->imin; a->imax = b->imax;
    } else {
      a->sum_f64 += b->sum_f64;
      a->sum_i64 = (int64_t)((uint64_t)a->sum_i64 + (uint64_t)b->sum_i64);
      if (is_float(kind)) {
        if (nan_safe_lt(b->min, a->min)) a->min = b->min;
        if (nan_safe_lt(a->max, b->max)) a->max = b->max;
      } else {
        if (b->imin < a->imin) a->imin = b->imin;
        if (b->imax > a->imax) a->imax = b->imax;
      }
    }
  }
  a->count += b->count;
}

static void stats_finish(int kind, dqo_col_stats* s) {
  if (!is_float(kind)) {
    s->sum_f64 = (double)s->sum_i64;
    s->min = (double)s->imin;
    s->max = (double)s->imax;
  }
}

static inline int64_t part_bound(int64_t n, int p, int nparts) {
  return (int64_t)(((__int128)n * p) / nparts);
}

void dqo_column_stats(int kind, const void* values, const uint8_t* validity, const uint8_t* mask,
                      int64_t n, int nparts, dqo_col_stats* out) {
  if (nparts < 1) nparts = 1;
  dqo_col_stats acc;
  memset(&acc, 0, sizeof(acc));
  for (int p = 0; p < nparts; ++p) {
    dqo_col_stats part;
    stats_partial(kind, values, validity, mask, part_bound(n, p, nparts), part_bound(n, p + 1, nparts), &part);
    stats_merge(kind, &acc, &part);
  }
  stats_finish(kind, &acc);
  *out = acc;
}

/* Corr: out = {n, xAvg, yAvg, ck, xMk, yMk} */
static void corr_partial(int kx, const void* x, const uint8_t* vx, int ky, const void* y, const uint8_t* vy,
                         const uint8_t* mask, int64_t lo, int64_t hi, double* s) {
  double n = 0, xAvg = 0, yAvg = 0, ck = 0, xMk = 0, yMk = 0;
  for (int64_t i = lo; i < hi; ++i) {
    if (!bit(vx, i) || !bit(vy, i) || !bit(mask, i)) continue;
    double xi = as_double(kx, x, i), yi = as_double(ky, y, i);
    double newN = n + 1.0;
    double dx = xi - xAvg, dxN = dx / newN;
    double dy = yi - yAvg, dyN = dy / newN;
    double newXAvg = xAvg + dxN, newYAvg = yAvg + dyN;
    ck = ck + dx * (yi - newYAvg);
    xMk = xMk + dx * (xi - newXAvg);
    yMk = yMk + dy * (yi - newYAvg);
    xAvg = newXAvg; yAvg = newYAvg; n = newN;
  }
  s[0] = n; s[1] = xAvg; s[2] = yAvg; s[3] = ck; s[4] = xMk; s[5] = yMk;
}

void dqo_corr_merge(double* a, const double* b) {
  double n1 = a[0], n2 = b[0], newN = n1 + n2;
  double dx = b[1] - a[1], dxN = newN == 0.0 ? 0.0 : dx / newN;
  double dy = b[2] - a[2], dyN = newN == 0.0 ? 0.0 : dy / newN;
  a[1] = a[1] + dxN * n2;
  a[2] = a[2] + dyN * n2;
  a[3] = a[3] + b[3] + dx * dyN * n1 * n2;
  a[4] = a[4] + b[4] + dx * dxN * n1 * n2;
  a[5] = a[5] + b[5] + dy * dyN * n1 * n2;
  a[0] = newN;
}

void dqo_corr(int kx, const void* x, const uint8_t* vx, int ky, const void* y, const uint8_t* vy,
              const uint8_t* mask, int64_t n, int nparts, double* out) {
  if (nparts < 1) nparts = 1;
  double acc[6] = {0, 0, 0, 0, 0, 0};
  for (int p = 0; p < nparts; ++p) {
    double part[6];
    corr_partial(kx, x, vx, ky, y, vy, mask, part_bound(n, p, nparts), part_bound(n, p + 1, nparts), part);
    dqo_corr_merge(acc, part);
  }
  memcpy(out, acc, sizeof(acc));
}

static inline uint64_t hash_row(int kind, const void* values, const void* offsets, int64_t i) {
  switch (kind) {
    case K_F64: {
      double d = ((const double*)values)[i];
      int64_t bits;
      if (d != d) bits = 0x7FF8000000000000LL;
      else memcpy(&bits, &d, 8);
      return dqo_xxh64_long(bits, 42);
    }
    case K_I64: return dqo_xxh64_long(((const int64_t*)values)[i], 42);
    case K_I32: case K_I16: case K_I8: case K_BOOL:  /* hashInt of the value widened to int (boolean: 1 / 0) */
      return dqo_xxh64_int((int32_t)as_long(kind, values, i), 42);
    case K_F32: {  /* hashInt(java.lang.Float.floatToIntBits(f)): every NaN as 0x7fc00000 */
      float f = ((const float*)values)[i];
      int32_t bits;
      if (f != f) bits = 0x7FC00000;
      else memcpy(&bits, &f, 4);
      return dqo_xxh64_int(bits, 42);
    }
    case K_UTF8: {
      const int32_t* o = (const int32_t*)offsets;
      return dqo_xxh64_bytes((const uint8_t*)values + o[i], o[i + 1] - o[i], 42);
    }
    default: {
      const int64_t* o = (const int64_t*)offsets;
      return dqo_xxh64_bytes((const uint8_t*)values + o[i], o[i + 1] - o[i], 42);
    }
  }
}

static inline void hll_add(uint8_t* regs, uint64_t x) {
  unsigned idx = (unsigned)(x >> 55);
  uint64_t w = (x << 9) | (1ULL << 8);
  uint8_t pw = (uint8_t)(__builtin_clzll(w) + 1);
  if (pw > regs[idx]) regs[idx] = pw;
}

void dqo_hll_registers(int kind, const void* values, const void* offsets, const uint8_t* validity,
                       const uint8_t* mask, int64_t n, uint8_t* regs /* [512], accumulated */) {
  for (int64_t i = 0; i < n; ++i) {
    if (!bit(validity, i) || !bit(mask, i)) continue;
    hll_add(regs, hash_row(kind, values, offsets, i));
  }
}

int64_t dqo_count_bits(const uint8_t* a, const uint8_t* b, int64_t n) {
  int64_t c = 0;
  for (int64_t i = 0; i < n; ++i) c += bit(a, i) & bit(b, i);
  return c;
}

/*
 * Profile scan (CPU baseline): for every column, count + moments + min/max + sum (numeric) and
 * HLL registers (all kinds), partitions folded in parallel, merged in partition order -- the
 * same work Spark local[N] does for ColumnProfiler passes 1-2 (profiles/ColumnProfiler.scala:200-235).
 */
void dqo_profile_scan(int ncols, const int* kinds, const void* const* values, const void* const* offsets,
                      const uint8_t* const* validity, int64_t n, int nparts, int nthreads,
                      dqo_col_stats* out_stats /* [ncols] */, uint8_t* out_regs /* [ncols*512] */) {
  if (nparts < 1) nparts = 1;
  dqo_col_stats* parts = (dqo_col_stats*)calloc((size_t)nparts * ncols, sizeof(dqo_col_stats));
  uint8_t* pregs = (uint8_t*)calloc((size_t)nparts * ncols, 512);
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int p = 0; p < nparts; ++p) {
    int64_t lo = part_bound(n, p, nparts), hi = part_bound(n, p + 1, nparts);
    for (int c = 0; c < ncols; ++c) {
      if (is_num(kinds[c]))
        stats_partial(kinds[c], values[c], validity[c], NULL, lo, hi, &parts[(size_t)p * ncols + c]);
      else {
        dqo_col_stats* s = &parts[(size_t)p * ncols + c];
        memset(s, 0, sizeof(*s));
        for (int64_t i = lo; i < hi; ++i) s->count += bit(validity[c], i);
      }
      uint8_t* r = pregs + ((size_t)p * ncols + c) * 512;
      for (int64_t i = lo; i < hi; ++i)
        if (bit(validity[c], i)) hll_add(r, hash_row(kinds[c], values[c], offsets[c], i));
    }
  }
  for (int c = 0; c < ncols; ++c) {
    dqo_col_stats acc;
    memset(&acc, 0, sizeof(acc));
    uint8_t* r = out_regs + (size_t)c * 512;
    memset(r, 0, 512);
    for (int p = 0; p < nparts; ++p) {
      if (is_num(kinds[c])) stats_merge(kinds[c], &acc, &parts[(size_t)p * ncols + c]);
      else acc.count += parts[(size_t)p * ncols + c].count;
      const uint8_t* pr = pregs + ((size_t)p * ncols + c) * 512;
      for (int i = 0; i < 512; ++i) if (pr[i] > r[i]) r[i] = pr[i];
    }
    if (is_num(kinds[c])) stats_finish(kinds[c], &acc);
    out_stats[c] = acc;
  }
  free(parts);
  free(pregs);
}

/*
 * Spark-order partials in parallel (full-scale parity checks): partition p of [0, n) folds its rows
 * sequentially (Spark's partial aggregate); the caller merges the partials in partition order from the
 * zero buffer (the final aggregate), so the result is bitwise that of dqo_column_stats / dqo_corr with
 * the same partition count -- only the partitions run on several threads.
 */
void dqo_column_stats_partials(int kind, const void* values, const uint8_t* validity, const uint8_t* mask,
                               int64_t n, int nparts, int nthreads, dqo_col_stats* out /* [nparts] */) {
  if (nparts < 1) nparts = 1;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int p = 0; p < nparts; ++p)
    stats_partial(kind, values, validity, mask, part_bound(n, p, nparts), part_bound(n, p + 1, nparts), &out[p]);
}

/* acc <- acc (+) part  (CentralMomentAgg / sum / min / max merge of the final aggregate), and the cast
   of integral sums / min / max to double at the end (dqo_stats_finish) */
void dqo_stats_merge(int kind, dqo_col_stats* acc, const dqo_col_stats* part) { stats_merge(kind, acc, part); }
void dqo_stats_finish(int kind, dqo_col_stats* s) { stats_finish(kind, s); }

void dqo_corr_partials(int kx, const void* x, const uint8_t* vx, int ky, const void* y, const uint8_t* vy,
                       const uint8_t* mask, int64_t n, int nparts, int nthreads, double* out /* [nparts][6] */) {
  if (nparts < 1) nparts = 1;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int p = 0; p < nparts; ++p)
    corr_partial(kx, x, vx, ky, y, vy, mask, part_bound(n, p, nparts), part_bound(n, p + 1, nparts), out + 6 * p);
}

/*
 * Near-exact references (SURVEY §7 "hard parts": which side carries the fp64 error at 1e9 rows).
 * Sums of (x - pivot) and (x - pivot)^2 -- and, for a pair, of the cross products -- accumulated in
 * double-double arithmetic (error-free TwoSum / TwoProd with fma, ~106-bit significand), so the
 * accumulated rounding error over 1e9 terms is ~1e-22 relative: far below the 1e-12 parity bar.  The
 * caller combines the per-chunk (hi, lo) pairs exactly (Python Fraction) and forms
 * mean = pivot + S1 / n, m2 = S2 - S1^2 / n, ck = Sxy - Sx Sy / n.
 */
typedef struct { double hi, lo; } dd_t;

static inline dd_t dd_two_sum(double a, double b) {
  double s = a + b, bb = s - a;
  dd_t r = {s, (a - (s - bb)) + (b - bb)};
  return r;
}
static inline dd_t dd_add_dd(dd_t a, dd_t b) {
  dd_t s = dd_two_sum(a.hi, b.hi);
  double lo = s.lo + a.lo + b.lo;
  return dd_two_sum(s.hi, lo);
}
static inline __attribute__((unused)) dd_t dd_add_d(dd_t a, double b) {
  dd_t s = dd_two_sum(a.hi, b);
  return dd_two_sum(s.hi, s.lo + a.lo);
}
static inline dd_t dd_prod(double a, double b) { /* exact product a * b = hi + lo */
  double p = a * b;
  dd_t r = {p, fma(a, b, -p)};
  return r;
}
static inline dd_t dd_mul(dd_t a, dd_t b) { /* (a.hi + a.lo)(b.hi + b.lo), dropping lo*lo */
  dd_t p = dd_prod(a.hi, b.hi);
  return dd_two_sum(p.hi, p.lo + (a.hi * b.lo + a.lo * b.hi));
}
static inline dd_t dd_diff(double x, double p) { return dd_two_sum(x, -p); } /* x - p exactly */

/* out = {count, S1.hi, S1.lo, S2.hi, S2.lo}: selected rows (valid & mask), finite values only */
void dqo_exact_moments(int kind, const void* values, const uint8_t* validity, const uint8_t* mask, int64_t n,
                       double pivot, int nthreads, double* out) {
  int nb = 1024;
  double* acc = (double*)calloc((size_t)nb * 5, sizeof(double));
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int b = 0; b < nb; ++b) {
    int64_t lo = part_bound(n, b, nb), hi = part_bound(n, b + 1, nb);
    dd_t s1 = {0, 0}, s2 = {0, 0};
    double cnt = 0;
    for (int64_t i = lo; i < hi; ++i) {
      if (!bit(validity, i) || !bit(mask, i)) continue;
      double x = as_double(kind, values, i);
      if (!isfinite(x)) continue;
      dd_t d = dd_diff(x, pivot);
      s1 = dd_add_dd(s1, d);
      s2 = dd_add_dd(s2, dd_mul(d, d));
      cnt += 1.0;
    }
    double* a = acc + 5 * b;
    a[0] = cnt; a[1] = s1.hi; a[2] = s1.lo; a[3] = s2.hi; a[4] = s2.lo;
  }
  dd_t s1 = {0, 0}, s2 = {0, 0};
  double cnt = 0;
  for (int b = 0; b < nb; ++b) {
    double* a = acc + 5 * b;
    cnt += a[0];
    s1 = dd_add_dd(s1, (dd_t){a[1], a[2]});
    s2 = dd_add_dd(s2, (dd_t){a[3], a[4]});
  }
  out[0] = cnt; out[1] = s1.hi; out[2] = s1.lo; out[3] = s2.hi; out[4] = s2.lo;
  free(acc);
}

/* out = {count, Sx, Sy, Sxy, Sxx, Syy} as (hi, lo) pairs -> 11 doubles; rows valid in both columns */
void dqo_exact_comoments(int kx, const void* x, const uint8_t* vx, int ky, const void* y, const uint8_t* vy,
                         const uint8_t* mask, int64_t n, double px, double py, int nthreads, double* out) {
  int nb = 1024;
  double* acc = (double*)calloc((size_t)nb * 11, sizeof(double));
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int b = 0; b < nb; ++b) {
    int64_t lo = part_bound(n, b, nb), hi = part_bound(n, b + 1, nb);
    dd_t sx = {0, 0}, sy = {0, 0}, sxy = {0, 0}, sxx = {0, 0}, syy = {0, 0};
    double cnt = 0;
    for (int64_t i = lo; i < hi; ++i) {
      if (!bit(vx, i) || !bit(vy, i) || !bit(mask, i)) continue;
      dd_t dx = dd_diff(as_double(kx, x, i), px), dy = dd_diff(as_double(ky, y, i), py);
      sx = dd_add_dd(sx, dx);
      sy = dd_add_dd(sy, dy);
      sxy = dd_add_dd(sxy, dd_mul(dx, dy));
      sxx = dd_add_dd(sxx, dd_mul(dx, dx));
      syy = dd_add_dd(syy, dd_mul(dy, dy));
      cnt += 1.0;
    }
    double* a = acc + 11 * b;
    a[0] = cnt;
    a[1] = sx.hi; a[2] = sx.lo; a[3] = sy.hi; a[4] = sy.lo; a[5] = sxy.hi; a[6] = sxy.lo;
    a[7] = sxx.hi; a[8] = sxx.lo; a[9] = syy.hi; a[10] = syy.lo;
  }
  dd_t s[5] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}};
  double cnt = 0;
  for (int b = 0; b < nb; ++b) {
    double* a = acc + 11 * b;
    cnt += a[0];
    for (int k = 0; k < 5; ++k) s[k] = dd_add_dd(s[k], (dd_t){a[1 + 2 * k], a[2 + 2 * k]});
  }
  out[0] = cnt;
  for (int k = 0; k < 5; ++k) { out[1 + 2 * k] = s[k].hi; out[2 + 2 * k] = s[k].lo; }
  free(acc);
}

/*
 * HLL registers of a large column on several threads (full-scale parity): partitions fold into private
 * registers, merged by max (order-free, so the result equals dqo_hll_registers).  Also counts the rows
 * that reach the GPU kernels' rare paths (test reporting only): paths[0] = selected rows whose hash has
 * bits 54..32 zero (the rank needs the low word: exact redo), paths[1] = selected strings longer than 28
 * bytes, paths[2] = selected strings whose 32-byte window (from the dword holding their first byte)
 * crosses the end of the chunk's string bytes (both take the general XXH64 loop).
 */
void dqo_hll_registers_mt(int kind, const void* values, const void* offsets, const uint8_t* validity,
                          const uint8_t* mask, int64_t n, int nthreads, uint8_t* regs /* [512], accumulated */,
                          int64_t* paths /* [3] */) {
  int nb = 1024;
  uint8_t* pr = (uint8_t*)calloc((size_t)nb, 512);
  int64_t* pc = (int64_t*)calloc((size_t)nb * 3, sizeof(int64_t));
  int64_t total = 0;
  if (kind == K_UTF8) total = ((const int32_t*)offsets)[n];
  if (kind == K_LARGE_UTF8) total = ((const int64_t*)offsets)[n];
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int b = 0; b < nb; ++b) {
    int64_t lo = part_bound(n, b, nb), hi = part_bound(n, b + 1, nb);
    uint8_t* r = pr + (size_t)b * 512;
    int64_t* c = pc + 3 * b;
    for (int64_t i = lo; i < hi; ++i) {
      if (!bit(validity, i) || !bit(mask, i)) continue;
      uint64_t h = hash_row(kind, values, offsets, i);
      hll_add(r, h);
      c[0] += ((h >> 32) & 0x7FFFFFu) == 0;
      if (kind == K_UTF8 || kind == K_LARGE_UTF8) {
        int64_t o0 = kind == K_UTF8 ? ((const int32_t*)offsets)[i] : ((const int64_t*)offsets)[i];
        int64_t o1 = kind == K_UTF8 ? ((const int32_t*)offsets)[i + 1] : ((const int64_t*)offsets)[i + 1];
        c[1] += o1 - o0 > 28;
        c[2] += o1 - o0 <= 28 && (o0 & ~(int64_t)3) + 32 > total;
      }
    }
  }
  paths[0] = paths[1] = paths[2] = 0;
  for (int b = 0; b < nb; ++b) {
    const uint8_t* r = pr + (size_t)b * 512;
    for (int i = 0; i < 512; ++i) if (r[i] > regs[i]) regs[i] = r[i];
    for (int k = 0; k < 3; ++k) paths[k] += pc[3 * b + k];
  }
  free(pr);
  free(pc);
}
