// dq_plan.cpp -- planner + scan driver behind the C ABI (include/dqscan.h).
//
// Replaces the body of AnalysisRunner.runScanningAnalyzers for the GPU-eligible analyzers
// (analyzers/runners/AnalysisRunner.scala:279-326): instead of building
// `aggregations = shareableAnalyzers.flatMap(_.aggregationFunctions())` and running
// `data.agg(...)`, the planner lowers the analyzers into column tasks, pair tasks and one
// predicate program, and dq_scan runs them over HBM-resident column chunks.  Identical analyzers
// are deduplicated (case-class equality, analyzers/AnalysisTest.scala:57-68) and shared
// sub-aggregates (count(*), the same column's moments, the same `where`) are computed once.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <iterator>
#include <limits>
#include <map>
#include <memory>
#include <string>
#include <tuple>
#include <vector>

#include "dq_device.h"
#include "dq_internal.h"
#include "dq_pred_jit.h"

// predicate-pass workgroups per chunk (A/B builds: -DDQ_PRED_WGS=...)
// rows per range at least this many: below it a launch's time goes to dispatching workgroups and to their
// fixed work (shift search, reductions, partial records), not to the rows -- a 10 M-row chunk (C1) otherwise
// ran 4-12 K workgroups of 2-4 K rows; every chunk of >= 16 K x 8192 rows is unaffected
#ifndef DQ_MIN_RANGE_ROWS
#define DQ_MIN_RANGE_ROWS 16384
#endif
// the validity-only pass (Completeness of a column): 8 KB of bitmap per 64 K rows, so its floor is higher (C1,
// 10 M rows: validity 21 -> 9-11 us, i64 moments 41 -> 31 us, finalize 13 -> 9 us; 256 K measured the same,
// profiles/r5_ab.txt r5i / r5j)
#ifndef DQ_MIN_VALIDITY_RANGE_ROWS
#define DQ_MIN_VALIDITY_RANGE_ROWS 65536
#endif
#ifndef DQ_F64_HLL_DIV
#define DQ_F64_HLL_DIV 2  // fp64 stats+HLL / HLL launches: ranges / 2 (see variant_div in dq_scan)
#endif
#ifndef DQ_PAIR_ONE_ROUND
#define DQ_PAIR_ONE_ROUND 1  // Correlation pass sized to one resident round (0: the column passes' ranges; A/B builds)
#endif
#ifndef DQ_PRED_WGS
#define DQ_PRED_WGS 2048
#endif
#include "dq_regex.h"

namespace dq {

hipError_t launch_pred_scan(const PredProgram* prog, const ScanCols& cols, const ScanBitmaps& bm, int64_t n_rows,
                            int64_t rows_per_range, int32_t nranges, PredPartial* acc, int32_t lds_bytes, hipStream_t st,
                            bool has_regex);
hipError_t launch_column_scan(int32_t variant, const ColTask* tasks, int32_t ntasks, int32_t part_base,
                              const ScanCols& cols, const ScanBitmaps& bm, int64_t n_rows, int64_t rows_per_range,
                              int32_t nranges, ColPartial* partials, uint32_t* hll_acc, bool long_str, hipStream_t st);
hipError_t launch_pair_scan(const PairWG* wgs, int32_t nwg, const ScanCols& cols, const ScanBitmaps& bm,
                            const uint32_t* ones, int64_t n_rows, int64_t rows_per_range, int32_t nranges,
                            CorrPartial* pair_part, ColPartial* col_part, int32_t* redo, bool all_f64, bool ring,
                            bool minmax, hipStream_t st);
hipError_t pair_scan_residency(bool all_f64, bool ring, bool minmax, int32_t* per_cu);
hipError_t launch_finalize(int32_t ncol, int32_t nranges_col, const ColPartial* col_part, ColPartial* col_acc,
                           int32_t npair, int32_t nranges_pair, const CorrPartial* pair_part, CorrPartial* pair_acc,
                           int32_t has_pred, int32_t nranges_pred, const PredPartial* pred_part, PredPartial* pred_acc, const FinRanges& fr, int64_t* rare_dev, int64_t* rare_host,
                           hipStream_t st);
hipError_t launch_init_acc(ColPartial* col_acc, int32_t ncol, CorrPartial* pair_acc, int32_t npair, int64_t* rare_dev,
                           hipStream_t st);

static thread_local char g_err[1024] = "";
// set with the error when a plan exceeds a fixed per-plan capacity (columns, predicates, counters, `where`
// bitmaps, column tasks, program length, regex LDS): dq_plan_create then splits the analyzers over several
// plans instead of failing (a spec that exceeds a capacity alone is a routing error, DQ_E_UNSUPPORTED)
static thread_local bool g_capacity = false;

dq_status set_error(dq_status code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

static dq_status cap_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  g_capacity = true;
  return DQ_E_UNSUPPORTED;
}

#define HIP_TRY(expr)                                                                              \
  do {                                                                                             \
    hipError_t e_ = (expr);                                                                        \
    if (e_ != hipSuccess)                                                                          \
      return set_error(e_ == hipErrorOutOfMemory ? DQ_E_OOM : DQ_E_HIP, "%s failed: %s (%s:%d)", \
                       #expr, hipGetErrorString(e_), __FILE__, __LINE__);                          \
  } while (0)

// Preconditions.isNumeric (Analyzer.scala:322-334): ByteType .. DoubleType and DecimalType
static bool is_numeric(int32_t t) {
  return t == DQ_TYPE_F64 || t == DQ_TYPE_I64 || t == DQ_TYPE_I32 || t == DQ_TYPE_F32 || t == DQ_TYPE_I16 ||
         t == DQ_TYPE_I8 || is_decimal(t);
}
static bool is_integral(int32_t t) { return t == DQ_TYPE_I64 || t == DQ_TYPE_I32 || t == DQ_TYPE_I16 || t == DQ_TYPE_I8; }
static bool is_floating(int32_t t) { return t == DQ_TYPE_F64 || t == DQ_TYPE_F32; }
static bool is_string(int32_t t) { return t == DQ_TYPE_UTF8 || t == DQ_TYPE_LARGE_UTF8; }
static int32_t kind_of(int32_t t) {
  switch (t) {
    case DQ_TYPE_F64: return CK_F64;
    case DQ_TYPE_I64: case DQ_TYPE_TIMESTAMP: return CK_I64;
    case DQ_TYPE_I32: case DQ_TYPE_DATE32: return CK_I32;
    case DQ_TYPE_F32: return CK_F32;
    case DQ_TYPE_I16: return CK_I16;
    case DQ_TYPE_I8: return CK_I8;
    case DQ_TYPE_BOOL: return CK_BOOL;
    case DQ_TYPE_UTF8: return CK_UTF8;
    case DQ_TYPE_LARGE_UTF8: return CK_LUTF8;
    default: return CK_D128;  // (type_valid: a DECIMAL128 code)
  }
}
// the Correlation pass's kind of a column: its ColKind, for a decimal CK_D128 | scale << 8 | (precision <= 18) << 16
// (dq_pair.hip casts it to double as it loads it)
static int32_t pair_kind(int32_t t) {
  if (!is_decimal(t)) return kind_of(t);
  return CK_D128 | DQ_DECIMAL_SCALE(t) << 8 | (DQ_DECIMAL_PRECISION(t) <= 18 ? 1 : 0) << 16;
}
// algorithmic bytes per row (x1000) of a column's value (or UTF8 offset) buffer
static int64_t value_bytes_x1000(int32_t t) {
  switch (t) {
    case DQ_TYPE_I32: case DQ_TYPE_F32: case DQ_TYPE_DATE32: case DQ_TYPE_UTF8: return 4000;
    case DQ_TYPE_I16: return 2000;
    case DQ_TYPE_I8: return 1000;
    case DQ_TYPE_BOOL: return 125;
    default: return is_decimal(t) ? 16000 : 8000;
  }
}
// (double)(float)v as Java's long -> float conversion rounds it (to nearest, ties to even)
static double int_as_float(int64_t v) { return (double)(float)v; }

// Where one analyzer's aggregation-result slots come from.
struct SpecOut {
  int32_t op = 0;
  int32_t col_task = -1;   // column task index
  int32_t pair_task = -1;  // pair task index
  int32_t ctr_a = -1;      // counter: (pred, where)  -- matches
  int32_t ctr_b = -1;      // counter: (where, none)  -- conditionalCount(where)
  int32_t col_type = 0;
  bool has_where = false;
};

// ------------------------------------------------------------------------------------------
// Predicate lowering: IR tree -> postfix program over three-valued atoms
// ------------------------------------------------------------------------------------------
struct Lit {  // exact literal: int / decimal (unscaled, scale) / double / null / bool
  enum K { INT, DEC, DBL, NUL, BOOL } k;
  int64_t i = 0;
  int32_t scale = 0;
  double d = 0.0;
};

static double lit_to_double(const Lit& l) {
  if (l.k == Lit::DBL) return l.d;
  if (l.k == Lit::INT || l.k == Lit::BOOL) return (double)l.i;
  // decimal -> correctly rounded double via its decimal text (Decimal.toDouble)
  char buf[64];
  long long u = (long long)l.i;
  bool neg = u < 0;
  unsigned long long a = neg ? (unsigned long long)(-(u + 1)) + 1ull : (unsigned long long)u;
  std::string digits = std::to_string(a);
  while ((int)digits.size() <= l.scale) digits = "0" + digits;
  std::string txt = (neg ? "-" : "") + digits.substr(0, digits.size() - l.scale) +
                    (l.scale ? "." + digits.substr(digits.size() - l.scale) : "");
  std::snprintf(buf, sizeof(buf), "%s", txt.c_str());
  return std::strtod(buf, nullptr);
}

static bool pow10_i64(int s, int64_t& out) {
  if (s < 0 || s > 18) return false;
  int64_t p = 1;
  for (int i = 0; i < s; ++i) p *= 10;
  out = p;
  return true;
}

// exact compare of two non-double literals: returns -1/0/1
static int exact_cmp(const Lit& a, const Lit& b) {
  int64_t pa = 1, pb = 1;
  pow10_i64(a.k == Lit::DEC ? a.scale : 0, pa);
  pow10_i64(b.k == Lit::DEC ? b.scale : 0, pb);
  __int128 x = (__int128)a.i * pb, y = (__int128)b.i * pa;
  return (x > y) - (x < y);
}

static int flip_cmp(int c) {
  switch (c) {
    case DQ_CMP_LT: return DQ_CMP_GT;
    case DQ_CMP_LE: return DQ_CMP_GE;
    case DQ_CMP_GT: return DQ_CMP_LT;
    case DQ_CMP_GE: return DQ_CMP_LE;
    default: return c;
  }
}

static bool cmp_holds(int c, int r) {
  switch (c) {
    case DQ_CMP_LT: return r < 0;
    case DQ_CMP_LE: return r <= 0;
    case DQ_CMP_GT: return r > 0;
    case DQ_CMP_GE: return r >= 0;
    case DQ_CMP_EQ: return r == 0;
    default: return r != 0;
  }
}

static int dbl_cmp(double a, double b) {  // Spark nanSafeCompare
  bool an = a != a, bn = b != b;
  if (an || bn) return (an && bn) ? 0 : (an ? 1 : -1);
  return (a > b) - (a < b);
}

// literal-vs-literal comparison under Spark coercion: any double -> double, else exact decimal
static int lit_cmp_result(int cmp, const Lit& a, const Lit& b) {  // returns NR_*
  if (a.k == Lit::NUL || b.k == Lit::NUL) return NR_NULL;
  int r = (a.k == Lit::DBL || b.k == Lit::DBL) ? dbl_cmp(lit_to_double(a), lit_to_double(b)) : exact_cmp(a, b);
  return cmp_holds(cmp, r) ? NR_TRUE : NR_FALSE;
}

static int to_cmpop(int c) {
  switch (c) {
    case DQ_CMP_LT: return C_LT;
    case DQ_CMP_LE: return C_LE;
    case DQ_CMP_GT: return C_GT;
    case DQ_CMP_GE: return C_GE;
    case DQ_CMP_EQ: return C_EQ;
    default: return C_NE;
  }
}

struct Lowering {
  const dq_pred_node* pool;
  int32_t n_pred;
  const std::vector<dq_column_desc>* schema;
  std::vector<PredInstr> out;
  const std::vector<std::string>* patterns = nullptr;
  std::vector<uint16_t>* regex_blob = nullptr;              // concatenated DFAs (dq_regex.h layout)
  std::map<std::pair<int64_t, int32_t>, int64_t> regex_at;  // (pattern, mode) -> blob word offset

  dq_status lit_of(int32_t idx, Lit& l) {
    const dq_pred_node& n = pool[idx];
    switch (n.kind) {
      case DQ_PRED_LIT_INT: l.k = Lit::INT; l.i = n.i64; return DQ_OK;
      case DQ_PRED_LIT_DECIMAL:
        if (n.cmp < 0 || n.cmp > 18) return set_error(DQ_E_UNSUPPORTED, "decimal literal scale %d unsupported", n.cmp);
        l.k = Lit::DEC; l.i = n.i64; l.scale = n.cmp; return DQ_OK;
      case DQ_PRED_LIT_DOUBLE: l.k = Lit::DBL; l.d = n.f64; return DQ_OK;
      case DQ_PRED_LIT_NULL: l.k = Lit::NUL; return DQ_OK;
      case DQ_PRED_LIT_BOOL: l.k = Lit::BOOL; l.i = n.i64 ? 1 : 0; return DQ_OK;
      default: return set_error(DQ_E_UNSUPPORTED, "node %d is not a literal", idx);
    }
  }
  bool is_lit(int32_t idx) const {
    int k = pool[idx].kind;
    return k >= DQ_PRED_LIT_INT && k <= DQ_PRED_LIT_BOOL;
  }
  dq_status check_idx(int32_t idx) {
    if (idx < 0 || idx >= n_pred) return set_error(DQ_E_INVALID, "predicate node index %d out of range", idx);
    return DQ_OK;
  }
  dq_status check_col(int32_t c) {
    if (c < 0 || c >= (int32_t)schema->size()) return set_error(DQ_E_INVALID, "predicate column %d out of range", c);
    return DQ_OK;
  }
  void push_const(int nr) {
    PredInstr p{};
    p.op = PO_CONST; p.null_res = nr; p.col_a = -1; p.col_b = -1;
    out.push_back(p);
  }

  // operand = column, or COALESCE(column, literal)
  struct Operand { int32_t col = -1; bool has_fallback = false; Lit fallback{}; };

  dq_status operand_of(int32_t idx, Operand& o) {
    const dq_pred_node& n = pool[idx];
    if (n.kind == DQ_PRED_COLUMN) {
      if (dq_status s = check_col(n.a)) return s;
      o.col = n.a;
      return DQ_OK;
    }
    if (n.kind == DQ_PRED_COALESCE) {
      if (dq_status s = check_idx(n.a)) return s;
      if (dq_status s = check_idx(n.b)) return s;
      if (pool[n.a].kind != DQ_PRED_COLUMN || !is_lit(n.b))
        return set_error(DQ_E_UNSUPPORTED, "COALESCE supported only as COALESCE(column, literal)");
      if (dq_status s = check_col(pool[n.a].a)) return s;
      o.col = pool[n.a].a;
      o.has_fallback = true;
      return lit_of(n.b, o.fallback);
    }
    return set_error(DQ_E_UNSUPPORTED, "unsupported comparison operand (node kind %d)", n.kind);
  }

  // DecimalType(p, s) column CMP an integer / decimal literal.  Spark 2.2 (DecimalPrecision) casts an integer
  // literal to DecimalType(10, 0) (an int) or (20, 0) (a long) and both sides to the wider decimal type
  // (max of the integer digits + max of the scales); while that fits 38 digits every cast is exact, so the
  // comparison is the exact rational one, rewritten here into a bound B on the unscaled value u: u CMP B.  Wider
  // types (Spark bounds them to 38 digits and can turn values NULL), double literals (the decimal is cast to
  // double) and boolean literals stay on the fallback.  Precision <= 18: one atom on the low word (the whole value,
  // |u| < 10^18); wider: the 128-bit comparison as atoms on the high word H and the low word L (compared unsigned),
  // e.g. u < B  <=>  H < Bh OR (H = Bh AND L <u Bl).
  dq_status emit_dec_lit(const Operand& o, int cmp, const Lit& lit, int32_t type) {
    const int prec = DQ_DECIMAL_PRECISION(type), sc = DQ_DECIMAL_SCALE(type);
    auto fits = [&](const Lit& l) {  // the wider decimal type of the column and the literal fits 38 digits
      if (l.k == Lit::NUL) return true;
      if (l.k != Lit::INT && l.k != Lit::DEC) return false;
      const int ls = l.k == Lit::DEC ? l.scale : 0;
      int lp;
      if (l.k == Lit::INT) lp = (l.i >= INT32_MIN && l.i <= INT32_MAX) ? 10 : 20;
      else {
        const uint64_t a = l.i < 0 ? (uint64_t)0 - (uint64_t)l.i : (uint64_t)l.i;
        lp = std::max((int)std::to_string(a).size(), ls);
      }
      return std::max(prec - sc, lp - ls) + std::max(sc, ls) <= kDecMaxPrecision;
    };
    if (!fits(lit) || (o.has_fallback && !fits(o.fallback)))
      return set_error(DQ_E_UNSUPPORTED, "decimal column %d compared with a %s literal", o.col,
                       lit.k == Lit::DBL || o.fallback.k == Lit::DBL ? "double" : "wider or boolean");
    const int nr = o.has_fallback ? lit_cmp_result(cmp, o.fallback, lit) : NR_NULL;
    if (lit.k == Lit::NUL) { push_const(NR_NULL); return DQ_OK; }
    // u / 10^sc CMP L / 10^t  ->  u CMP' B
    const int t = lit.k == Lit::DEC ? lit.scale : 0;
    int c2;
    i128 B;
    if (t <= sc) {
      i128 m = 1;
      for (int k = 0; k < sc - t; ++k) m *= 10;
      B = (i128)lit.i * m;  // (fits: the wider type has at most 38 digits)
      c2 = to_cmpop(cmp);
    } else {
      int64_t p10;
      pow10_i64(t - sc, p10);
      const int64_t u = lit.i;
      const int64_t fl = u >= 0 ? u / p10 : -((-u + p10 - 1) / p10);
      const bool exact = (u % p10) == 0;
      const int64_t ce = exact ? fl : fl + 1;
      switch (cmp) {
        case DQ_CMP_LT: c2 = C_LT; B = ce; break;
        case DQ_CMP_LE: c2 = C_LE; B = fl; break;
        case DQ_CMP_GT: c2 = C_GT; B = fl; break;
        case DQ_CMP_GE: c2 = C_GE; B = ce; break;
        case DQ_CMP_EQ: c2 = exact ? C_EQ : C_FALSE; B = fl; break;
        default: c2 = exact ? C_NE : C_TRUE; B = fl; break;
      }
    }
    auto atom = [&](int kind, int c, int64_t v) {
      PredInstr p{};
      p.op = PO_ATOM_CMP; p.col_a = o.col; p.col_b = -1; p.kind_a = kind; p.kind_b = 0;
      p.ctype = CT_INT; p.cmp = c; p.lit_i = v; p.null_res = nr;
      out.push_back(p);
    };
    auto logic = [&](int op) {
      PredInstr p{};
      p.op = op; p.col_a = p.col_b = -1;
      out.push_back(p);
    };
    if (c2 == C_TRUE || c2 == C_FALSE) { atom(CK_D128_LO, c2, 0); return DQ_OK; }
    if (prec <= 18) {
      if (B > (i128)INT64_MAX || B < (i128)INT64_MIN) {  // every |u| < 10^18 lies on one side of B
        const bool below = B > 0;  // u < B for every u
        const bool holds = c2 == C_LT || c2 == C_LE || c2 == C_NE ? below : (c2 == C_EQ ? false : !below);
        atom(CK_D128_LO, holds ? C_TRUE : C_FALSE, 0);
      } else {
        atom(CK_D128_LO, c2, (int64_t)B);
      }
      return DQ_OK;
    }
    const int64_t bh = (int64_t)(B >> 64);
    const int64_t bl = (int64_t)((uint64_t)B ^ (1ull << 63));  // (CK_D128_LOU flips the loaded low word the same way)
    if (c2 == C_EQ || c2 == C_NE) {
      atom(CK_D128_HI, c2, bh);
      atom(CK_D128_LOU, c2, bl);
      logic(c2 == C_EQ ? PO_AND : PO_OR);
      return DQ_OK;
    }
    const bool lt = c2 == C_LT || c2 == C_LE;
    atom(CK_D128_HI, lt ? C_LT : C_GT, bh);
    atom(CK_D128_HI, C_EQ, bh);
    atom(CK_D128_LOU, c2, bl);
    logic(PO_AND);
    logic(PO_OR);
    return DQ_OK;
  }

  // column CMP literal, with Spark 2.2 coercions (integral vs decimal exact, anything vs double in double)
  dq_status emit_col_lit(const Operand& o, int cmp, Lit lit) {
    const dq_column_desc& cd = (*schema)[o.col];
    if (is_decimal(cd.type)) return emit_dec_lit(o, cmp, lit, cd.type);
    const bool boolean = cd.type == DQ_TYPE_BOOL;
    if (!is_numeric(cd.type) && !boolean)
      return set_error(DQ_E_UNSUPPORTED, "comparison on a non-numeric column (%d)", o.col);
    PredInstr p{};
    p.op = PO_ATOM_CMP; p.col_a = o.col; p.col_b = -1; p.kind_a = kind_of(cd.type); p.kind_b = 0;
    Lit fb = o.fallback;
    if (boolean) {
      // BooleanType vs a boolean literal (Spark orders false < true); against a number Spark 2.2 rewrites
      // (BooleanEquality) or casts -- not restated here: the fallback
      if ((lit.k != Lit::BOOL && lit.k != Lit::NUL) || (o.has_fallback && fb.k != Lit::BOOL && fb.k != Lit::NUL))
        return set_error(DQ_E_UNSUPPORTED, "boolean column compared with a non-boolean literal");
      if (lit.k == Lit::BOOL) lit.k = Lit::INT;
      if (fb.k == Lit::BOOL) fb.k = Lit::INT;
    } else if (cd.type == DQ_TYPE_F32) {
      // FloatType vs an integral literal compares in FloatType (the literal cast to float: findTightestCommonType);
      // vs a decimal or double literal in DoubleType (DecimalPrecision: the decimal cast to double) -- the float
      // widens to double exactly, so every case is a double compare with the literal rounded accordingly.  A
      // COALESCE(col, lit) fallback takes the operand's widened type the same way.
      auto as_float_cmp = [](Lit& l) {
        if (l.k == Lit::INT || (l.k == Lit::DEC && l.scale == 0)) { l.d = int_as_float(l.i); l.k = Lit::DBL; }
        else if (l.k == Lit::DEC) { l.d = lit_to_double(l); l.k = Lit::DBL; }
      };
      as_float_cmp(lit);
      if (o.has_fallback) as_float_cmp(fb);
    }
    p.null_res = o.has_fallback ? lit_cmp_result(cmp, fb, lit) : NR_NULL;
    if (lit.k == Lit::NUL) { push_const(NR_NULL); return DQ_OK; }
    if (lit.k == Lit::BOOL) return set_error(DQ_E_UNSUPPORTED, "boolean literal compared with a number");
    if (is_floating(cd.type) || lit.k == Lit::DBL) {
      p.ctype = CT_DBL; p.cmp = to_cmpop(cmp); p.lit_d = lit_to_double(lit);
    } else if (lit.k == Lit::INT || (lit.k == Lit::DEC && lit.scale == 0)) {
      p.ctype = CT_INT; p.cmp = to_cmpop(cmp); p.lit_i = lit.i;
    } else {
      // integral column vs decimal literal v = u / 10^s: exact rewrite to integer bounds
      int64_t p10;
      pow10_i64(lit.scale, p10);
      int64_t u = lit.i;
      int64_t fl = u >= 0 ? u / p10 : -((-u + p10 - 1) / p10);  // floor
      bool integral = (u % p10) == 0;
      int64_t ce = integral ? fl : fl + 1;                      // ceil
      p.ctype = CT_INT;
      switch (cmp) {
        case DQ_CMP_LT: p.cmp = C_LT; p.lit_i = ce; break;      // x < v  <=> x < ceil(v)
        case DQ_CMP_LE: p.cmp = C_LE; p.lit_i = fl; break;      // x <= v <=> x <= floor(v)
        case DQ_CMP_GT: p.cmp = C_GT; p.lit_i = fl; break;      // x > v  <=> x > floor(v)
        case DQ_CMP_GE: p.cmp = C_GE; p.lit_i = ce; break;      // x >= v <=> x >= ceil(v)
        case DQ_CMP_EQ: p.cmp = integral ? C_EQ : C_FALSE; p.lit_i = fl; break;
        default: p.cmp = integral ? C_NE : C_TRUE; p.lit_i = fl; break;
      }
    }
    out.push_back(p);
    return DQ_OK;
  }

  dq_status lower(int32_t idx, int depth) {
    if (dq_status s = check_idx(idx)) return s;
    if (depth > 30) return set_error(DQ_E_UNSUPPORTED, "predicate nesting too deep");
    const dq_pred_node& n = pool[idx];
    switch (n.kind) {
      case DQ_PRED_AND:
      case DQ_PRED_OR: {
        if (dq_status s = lower(n.a, depth + 1)) return s;
        if (dq_status s = lower(n.b, depth + 1)) return s;
        PredInstr p{};
        p.op = n.kind == DQ_PRED_AND ? PO_AND : PO_OR; p.col_a = p.col_b = -1;
        out.push_back(p);
        return DQ_OK;
      }
      case DQ_PRED_NOT: {
        if (dq_status s = lower(n.a, depth + 1)) return s;
        PredInstr p{};
        p.op = PO_NOT; p.col_a = p.col_b = -1;
        out.push_back(p);
        return DQ_OK;
      }
      case DQ_PRED_REGEX: {  // PatternMatch.scala:48-49 / RLIKE on a string column
        if (dq_status s = check_idx(n.a)) return s;
        const dq_pred_node& c = pool[n.a];
        if (c.kind != DQ_PRED_COLUMN) return set_error(DQ_E_UNSUPPORTED, "regex on a non-column expression");
        if (dq_status s = check_col(c.a)) return s;
        const int32_t t = (*schema)[c.a].type;
        if (t != DQ_TYPE_UTF8 && t != DQ_TYPE_LARGE_UTF8)
          return set_error(DQ_E_UNSUPPORTED, "regex on a non-string column (%d)", c.a);
        if (n.cmp != DQ_REGEX_RLIKE && n.cmp != DQ_REGEX_EXTRACT_NONEMPTY && n.cmp != DQ_REGEX_FULL)
          return set_error(DQ_E_INVALID, "regex mode %d", n.cmp);
        if (!patterns || n.i64 < 0 || n.i64 >= (int64_t)patterns->size())
          return set_error(DQ_E_INVALID, "regex pattern index %lld out of range", (long long)n.i64);
        auto key = std::make_pair(n.i64, n.cmp);
        auto it = regex_at.find(key);
        int64_t off;
        if (it != regex_at.end()) {
          off = it->second;
        } else {
          RegexDfa d;
          if (dq_status s = regex_compile((*patterns)[n.i64].c_str(), n.cmp, d)) return s;
          off = (int64_t)regex_blob->size();
          regex_serialize(d, *regex_blob);
          regex_at[key] = off;
        }
        PredInstr p{};
        p.op = PO_ATOM_REGEX; p.col_a = c.a; p.col_b = -1; p.kind_a = kind_of(t);
        p.lit_i = off;
        p.null_res = n.cmp == DQ_REGEX_EXTRACT_NONEMPTY ? NR_FALSE : NR_NULL;
        out.push_back(p);
        return DQ_OK;
      }
      case DQ_PRED_IS_NULL:
      case DQ_PRED_IS_NOT_NULL: {
        if (dq_status s = check_idx(n.a)) return s;
        const dq_pred_node& c = pool[n.a];
        bool isnull = n.kind == DQ_PRED_IS_NULL;
        if (c.kind == DQ_PRED_COLUMN) {
          if (dq_status s = check_col(c.a)) return s;
          PredInstr p{};
          p.op = isnull ? PO_ATOM_ISNULL : PO_ATOM_NOTNULL; p.col_a = c.a; p.col_b = -1;
          out.push_back(p);
          return DQ_OK;
        }
        if (is_lit(n.a)) {
          bool lit_null = c.kind == DQ_PRED_LIT_NULL;
          push_const((lit_null == isnull) ? NR_TRUE : NR_FALSE);
          return DQ_OK;
        }
        if (c.kind == DQ_PRED_COALESCE && is_lit(c.b) && pool[c.b].kind != DQ_PRED_LIT_NULL) {
          push_const(isnull ? NR_FALSE : NR_TRUE);  // COALESCE(col, non-null literal) is never NULL
          return DQ_OK;
        }
        return set_error(DQ_E_UNSUPPORTED, "IS NULL over an unsupported expression");
      }
      case DQ_PRED_LIT_BOOL: push_const(n.i64 ? NR_TRUE : NR_FALSE); return DQ_OK;
      case DQ_PRED_LIT_NULL: push_const(NR_NULL); return DQ_OK;
      case DQ_PRED_COLUMN: {  // a BooleanType column as a predicate: its value (NULL stays NULL), i.e. col = TRUE
        if (dq_status s = check_col(n.a)) return s;
        if ((*schema)[n.a].type != DQ_TYPE_BOOL)
          return set_error(DQ_E_UNSUPPORTED, "column %d is not a boolean expression", n.a);
        PredInstr p{};
        p.op = PO_ATOM_CMP; p.col_a = n.a; p.col_b = -1; p.kind_a = CK_BOOL; p.kind_b = 0;
        p.null_res = NR_NULL; p.ctype = CT_INT; p.cmp = C_EQ; p.lit_i = 1;
        out.push_back(p);
        return DQ_OK;
      }
      case DQ_PRED_CMP: {
        if (dq_status s = check_idx(n.a)) return s;
        if (dq_status s = check_idx(n.b)) return s;
        int cmp = n.cmp;
        if (cmp < DQ_CMP_LT || cmp > DQ_CMP_NE) return set_error(DQ_E_INVALID, "bad comparison op %d", cmp);
        bool la = is_lit(n.a), lb = is_lit(n.b);
        if (la && lb) {
          Lit a, b;
          if (dq_status s = lit_of(n.a, a)) return s;
          if (dq_status s = lit_of(n.b, b)) return s;
          push_const(lit_cmp_result(cmp, a, b));
          return DQ_OK;
        }
        if (la || lb) {
          int32_t oi = la ? n.b : n.a, li = la ? n.a : n.b;
          if (la) cmp = flip_cmp(cmp);
          Operand o;
          Lit l;
          if (dq_status s = operand_of(oi, o)) return s;
          if (dq_status s = lit_of(li, l)) return s;
          return emit_col_lit(o, cmp, l);
        }
        // column vs column
        if (pool[n.a].kind != DQ_PRED_COLUMN || pool[n.b].kind != DQ_PRED_COLUMN)
          return set_error(DQ_E_UNSUPPORTED, "comparison of two non-column expressions");
        int32_t ca = pool[n.a].a, cb = pool[n.b].a;
        if (dq_status s = check_col(ca)) return s;
        if (dq_status s = check_col(cb)) return s;
        int32_t ta = (*schema)[ca].type, tb = (*schema)[cb].type;
        const bool bools = ta == DQ_TYPE_BOOL && tb == DQ_TYPE_BOOL;
        if (!bools && (!is_numeric(ta) || !is_numeric(tb)))
          return set_error(DQ_E_UNSUPPORTED, "comparison of non-numeric columns");
        if (is_decimal(ta) || is_decimal(tb))
          return set_error(DQ_E_UNSUPPORTED, "comparison of a decimal column with a column");
        // FloatType vs Int / LongType compares in FloatType (the integer rounded to float), which a double
        // compare does not restate for integers beyond 2^24: the fallback (ShortType / ByteType are exact)
        auto wide_int = [](int32_t t) { return t == DQ_TYPE_I32 || t == DQ_TYPE_I64; };
        if ((ta == DQ_TYPE_F32 && wide_int(tb)) || (tb == DQ_TYPE_F32 && wide_int(ta)))
          return set_error(DQ_E_UNSUPPORTED, "float column compared with an int / long column");
        PredInstr p{};
        p.op = PO_ATOM_CMP; p.col_a = ca; p.col_b = cb; p.kind_a = kind_of(ta); p.kind_b = kind_of(tb);
        p.null_res = NR_NULL; p.cmp = to_cmpop(cmp);
        p.ctype = bools || (is_integral(ta) && is_integral(tb)) ? CT_INT : CT_DBL;
        out.push_back(p);
        return DQ_OK;
      }
      default:
        return set_error(DQ_E_UNSUPPORTED, "predicate node kind %d is not a boolean expression", n.kind);
    }
  }
};

// canonical text of a predicate subtree (dedup of roots)
static std::string canon(const dq_pred_node* pool, int32_t n_pred, int32_t idx, int depth = 0) {
  if (idx < 0 || idx >= n_pred || depth > 64) return "?";
  const dq_pred_node& n = pool[idx];
  char buf[128];
  std::snprintf(buf, sizeof(buf), "(%d:%d:%lld:%a", n.kind, n.cmp, (long long)n.i64, n.f64);
  std::string s = buf;
  if (n.kind == DQ_PRED_COLUMN) s += ":c" + std::to_string(n.a);
  else {
    if (n.kind == DQ_PRED_CMP || n.kind == DQ_PRED_AND || n.kind == DQ_PRED_OR || n.kind == DQ_PRED_NOT ||
        n.kind == DQ_PRED_IS_NULL || n.kind == DQ_PRED_IS_NOT_NULL || n.kind == DQ_PRED_COALESCE ||
        n.kind == DQ_PRED_REGEX)
      s += canon(pool, n_pred, n.a, depth + 1);
    if (n.kind == DQ_PRED_CMP || n.kind == DQ_PRED_AND || n.kind == DQ_PRED_OR || n.kind == DQ_PRED_COALESCE)
      s += canon(pool, n_pred, n.b, depth + 1);
  }
  return s + ")";
}

}  // namespace dq

using namespace dq;

struct dq_plan {
  int32_t device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  std::vector<dq_column_desc> schema;
  std::vector<dq_analyzer_spec> specs;
  std::vector<SpecOut> outs;

  std::vector<ColTask> col_tasks;        // sorted by variant
  struct Group { int32_t variant, first, count; };
  std::vector<Group> groups;              // one column-scan launch per variant group
  std::vector<Group> pred_fused_groups;   // the predicate kernel's HLL tasks as column-pass launches (interpreter)
  std::vector<PairTask> pair_tasks;      // sorted by pair group
  std::vector<PairWG> pair_wgs;          // Correlation pass workgroup tasks (dq_pair.hip), moments fused
  int32_t n_fused = 0;                    // column tasks computed by the pair pass (sorted last)
  bool pair_all_f64 = true;               // every pair-group column is fp64 (the conversion-free instantiations)
  bool pair_minmax = false;               // a fused moments task feeds Minimum / Maximum
  PredProgram prog{};
  std::vector<std::string> patterns;      // DQ_PRED_REGEX patterns (dq_plan_create_ex)
  std::vector<uint16_t> regex_blob;       // their compiled DFAs
  uint16_t* d_regex = nullptr;
  int32_t n_hll = 0;
  bool has_pred = false;
  // the predicate pass compiled for this program (dq_pred_jit.cpp), or null: the interpreter runs it
  hipFunction_t pred_jit = nullptr;
  PredJitRef pred_jit_ref;                              // its compile, while it runs in the background (AUTO)
  std::vector<int32_t> pred_jit_cols;                   // its slots' plan columns
  std::vector<int32_t> pred_jit_hll_task, pred_jit_hll_slot;  // fused HLL tasks (post-sort index) / accumulators
  int32_t pred_fused_first = 0, pred_fused_count = 0;  // those tasks sort last (after the pair-fused ones)
  int32_t pair_fused_first = 0, pair_fused_count = 0;  // moments tasks the pair pass computes
  int32_t pair_resident[2] = {0, 0};  // pair-pass workgroups the device holds at once (ring / not), 0 = not asked
  std::string pred_jit_note;                            // why the interpreter runs, or the kernel's origin
  int32_t pred_pass = DQ_PRED_PASS_AUTO;                // dq_plan_options.pred_pass
  bool host_only = false;                               // dq_plan_explain: lower on the host, no device work
  bool probe = false;                                   // host-only capacity check: stop after the program
  std::string pred_jit_src;                             // the generated kernel source (host_only plans)
  double create_ms = 0.0, pred_jit_ms = 0.0;            // dq_plan_create_time

  // device memory
  ColTask* d_col_tasks = nullptr;
  PairTask* d_pair_tasks = nullptr;
  PairWG* d_pair_wgs = nullptr;
  int32_t* d_pair_redo = nullptr;         // [pair_wgs][kPairWaves][kMaxWG] ranges left to the checked fold
  char* h_stage = nullptr;                // pinned host copy of the accumulators (dq_finish: truly async D2H)
  // the string pass's variant per UTF8 HLL task: the string kernels count each task's rare-path rows since the
  // reset (d_rare_dev), the finalize kernel publishes them into mapped pinned memory (h_rare; d_rare its device
  // address), dq_scan reads them without waiting and runs the LONG variant for a task group once more than
  // 1 / 4096 of the rows took the rare path (the common variant redoes a whole 512-row block for one such row:
  // at 4.5 % of them it ran 5.86 ms per 1e8 rows x 4 columns against LONG's 2.44; on short strings alone
  // 1.80 against 2.34, profiles/r5_ab.txt r5aj)
  int64_t* d_rare_dev = nullptr;
  int64_t* h_rare = nullptr;
  int64_t* d_rare = nullptr;
  std::vector<uint8_t> str_long;  // per column task
  int32_t str_path = 0;           // DQ_STR_PATH: 0 auto, 1 fast variant only, 2 LONG variant only
  int64_t prev_rows = 0;          // rows of the scan before the last reset (its counts stay published until
                                  // this scan's first finalize)
  size_t h_stage_bytes = 0;
  PredProgram* d_prog = nullptr;
  ColPartial* d_col_part = nullptr;
  CorrPartial* d_pair_part = nullptr;
  PredPartial* d_pred_part = nullptr;
  ColPartial* d_col_acc = nullptr;
  uint32_t* d_hll_acc = nullptr;
  CorrPartial* d_pair_acc = nullptr;
  PredPartial* d_pred_acc = nullptr;
  uint64_t* d_where_bits[kMaxWhere] = {nullptr};
  int64_t where_cap_words = 0;
  uint32_t* d_ones = nullptr;  // all-ones bitmap (pair pass: columns without validity, groups without where)
  int64_t ones_cap_words = 0;

  int64_t total_rows = 0;
  int64_t next_chunk = 0;

  // optional per-kernel timing with hipEvents on the plan's stream (bench / profiling)
  bool timing = false;
  std::vector<hipEvent_t> ev_pool;
  struct Pending { int kernel; hipEvent_t a, b; };
  std::vector<Pending> pending;
  static constexpr int kTimers = 16 + kNumVariants;
  double kernel_ms[kTimers] = {0};       // 0 pred, 2 pair, 3 finalize, 16 + v column variant v
  int64_t kernel_launches[kTimers] = {0};
  int64_t bytes_per_row_x1000 = 0;
  int64_t pred_bytes_x1000 = 0, pair_bytes_x1000 = 0;
  int32_t launches_per_scan = 0;

  // composite plan: an analyzer set over one plan's capacity runs as several fused plans ("parts") over
  // disjoint spec subsets, each reading only its own columns; dq_scan runs every part on every chunk (in
  // part order, on this plan's stream) and dq_finish scatters their states back to the caller's spec order
  std::vector<dq_plan*> parts;
  std::vector<std::vector<int32_t>> part_specs;  // this plan's spec index of each part spec
  std::vector<std::vector<int32_t>> part_cols;   // this plan's column of each part column
};

static dq_status take_event(dq_plan* p, hipEvent_t* e) {
  if (!p->ev_pool.empty()) { *e = p->ev_pool.back(); p->ev_pool.pop_back(); return DQ_OK; }
  HIP_TRY(hipEventCreate(e));
  return DQ_OK;
}

static dq_status resolve_timing(dq_plan* p) {
  if (p->pending.empty()) return DQ_OK;
  HIP_TRY(hipStreamSynchronize(p->stream));
  for (auto& q : p->pending) {
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, q.a, q.b));
    p->kernel_ms[q.kernel] += ms;
    p->kernel_launches[q.kernel] += 1;
    p->ev_pool.push_back(q.a);
    p->ev_pool.push_back(q.b);
  }
  p->pending.clear();
  return DQ_OK;
}

// launch `fn` bracketed by timing events when enabled
template <typename F>
static dq_status timed(dq_plan* p, int kernel, hipStream_t st, F fn) {
  hipEvent_t a = nullptr, b = nullptr;
  if (p->timing) {
    if (dq_status s = take_event(p, &a)) return s;
    if (dq_status s = take_event(p, &b)) return s;
    HIP_TRY(hipEventRecord(a, st));
  }
  HIP_TRY(fn());
  if (p->timing) {
    HIP_TRY(hipEventRecord(b, st));
    p->pending.push_back({kernel, a, b});
  }
  return DQ_OK;
}

static dq_status free_plan_mem(dq_plan* p) {
  for (auto& q : p->pending) { p->ev_pool.push_back(q.a); p->ev_pool.push_back(q.b); }
  p->pending.clear();
  for (hipEvent_t e : p->ev_pool) (void)hipEventDestroy(e);
  p->ev_pool.clear();
  void* ptrs[] = {p->d_col_tasks, p->d_pair_tasks, p->d_pair_wgs, p->d_prog, p->d_col_part, p->d_pair_part,
                  p->d_pred_part, p->d_col_acc, p->d_hll_acc, p->d_pair_acc, p->d_pred_acc, p->d_regex, p->d_pair_redo,
                  p->d_rare_dev};
  for (void* q : ptrs)
    if (q) (void)hipFree(q);
  for (int i = 0; i < kMaxWhere; ++i)
    if (p->d_where_bits[i]) (void)hipFree(p->d_where_bits[i]);
  if (p->d_ones) (void)hipFree(p->d_ones);
  if (p->h_rare) (void)hipHostFree(p->h_rare);
  p->h_rare = p->d_rare = nullptr;
  if (p->h_stage) (void)hipHostFree(p->h_stage);
  p->h_stage = nullptr;
  p->h_stage_bytes = 0;
  return DQ_OK;
}

static dq_status reset_acc(dq_plan* p) {
  HIP_TRY(launch_init_acc(p->d_col_acc, (int32_t)p->col_tasks.size(), p->d_pair_acc, (int32_t)p->pair_tasks.size(),
                          p->d_rare_dev, p->stream));
  if (p->n_hll) HIP_TRY(hipMemsetAsync(p->d_hll_acc, 0, (size_t)p->n_hll * kHllCopies * 512 * sizeof(uint32_t), p->stream));
  if (p->has_pred) HIP_TRY(hipMemsetAsync(p->d_pred_acc, 0, kPredAccCopies * sizeof(PredPartial), p->stream));
  if (p->total_rows > 0) p->prev_rows = p->total_rows;
  p->total_rows = 0;
  p->next_chunk = 0;
  return DQ_OK;
}

template <typename T>
static dq_status dmalloc(T** ptr, size_t bytes) {
  if (bytes == 0) bytes = 16;
  HIP_TRY(hipMalloc((void**)ptr, bytes));
  return DQ_OK;
}

// Plan one pair group for the Correlation pass (dq_pair.hip): wave w's position p holds local column
// (p + w) % 8, so every pair of two distinct columns has exactly one (wave, slot) of the fixed pattern; the
// slot computes (position A, position B) and a pair whose first column sits at B swaps x / y on output.
// Each fusable moments column -- a stats-only column task of the group's columns and `where` -- goes to
// its even position (column c: wave c % 2, position c - c % 2).  Pairs the group cannot hold (x with
// itself, or (y, x) beside (x, y): one slot per unordered pair) become one- / two-column workgroup tasks of
// their own.
static void plan_pair_wgs(const dq_plan* p, const PairGroup& g, std::vector<PairWG>& out, std::vector<int>& fused) {
  auto blank = [&](const int32_t* lcols, int nl) {  // wave tasks over local columns lcols[0 .. nl)
    PairWG wg;
    std::memset(&wg, 0, sizeof(wg));
    for (int w = 0; w < kPairWaves; ++w) {
      PairWaveTask& t = wg.wave[w];
      t.where = g.where;
      for (int q = 0; q < kPairPos; ++q) {
        const int l = (q + w) % kPairPos;
        const int c = lcols[l < nl ? l : 0];  // an unused position repeats a used column (loaded, never read)
        t.cols[q] = g.cols[c];
        t.kinds[q] = g.kinds[c];
      }
      for (int q = 0; q < kPairSlots; ++q) t.pair_out[q] = -1;
      for (int k = 0; k < kPairMoments; ++k) t.mom_out[k] = -1;
    }
    return wg;
  };
  auto place = [&](PairWG& wg, int a, int b, int32_t pair) {  // local positions of the first / second column
    for (int w = 0; w < kPairWaves; ++w) {
      const int pa = (a - w + kPairPos) % kPairPos, pb = (b - w + kPairPos) % kPairPos;
      for (int q = 0; q < kPairSlots; ++q) {
        const bool fwd = kPairSlotA[q] == pa && kPairSlotB[q] == pb, rev = kPairSlotA[q] == pb && kPairSlotB[q] == pa;
        if (!fwd && !rev) continue;
        PairWaveTask& t = wg.wave[w];
        if ((t.pair_mask >> q) & 1u) return false;
        t.pair_mask |= 1u << q;
        if (rev) t.swap_mask |= 1u << q;
        t.pair_out[q] = pair;
        return true;
      }
    }
    return false;
  };
  int32_t ident[kPairPos];
  for (int c = 0; c < kPairPos; ++c) ident[c] = c;
  PairWG wg = blank(ident, g.ncols);
  std::vector<int> extra;
  for (int q = 0; q < g.npairs; ++q)
    if (g.pi[q] == g.pj[q] || !place(wg, g.pi[q], g.pj[q], g.first_pair + q)) extra.push_back(q);
  for (int c = 0; c < g.ncols; ++c)
    for (size_t t = 0; t < p->col_tasks.size(); ++t) {
      const ColTask& ct = p->col_tasks[t];
      if (ct.col == g.cols[c] && ct.where == g.where && !fused[t] &&
          (ct.variant == CV_F64_S || ct.variant == CV_I64_S || ct.variant == CV_I32_S || ct.variant == CV_F32_S ||
           ct.variant == CV_I16_S || ct.variant == CV_I8_S)) {
        PairWaveTask& w = wg.wave[c % 2];
        const int k = (c - c % 2) / 2;
        w.mom_mask |= 1u << k;
        w.mom_out[k] = (int32_t)t;
        fused[t] = 1;
        break;
      }
    }
  if (wg.wave[0].pair_mask | wg.wave[0].mom_mask | wg.wave[1].pair_mask | wg.wave[1].mom_mask) out.push_back(wg);
  for (int q : extra) {  // slot (0, 1) of wave 0 of a task holding the pair's column(s) at positions 0, 1
    const int32_t lc[2] = {g.pi[q], g.pj[q]};
    PairWG e = blank(lc, 2);
    PairWaveTask& t = e.wave[0];
    t.pair_mask = 1u;
    t.pair_out[0] = g.first_pair + q;
    out.push_back(e);
  }
}

static dq_status build_plan(dq_plan* p, const dq_pred_node* pool, int32_t n_pred) {
  const int32_t ncols = (int32_t)p->schema.size();
  std::map<std::string, int32_t> root_slot;          // canonical predicate text -> root slot
  std::vector<std::vector<PredInstr>> root_code;
  std::map<std::tuple<int32_t, int32_t, int32_t>, int32_t> col_task_of;  // (col, where bitmap, f64 DataType) -> task
  std::map<std::tuple<int32_t, int32_t, int32_t>, int32_t> pair_of; // (x, y, where bitmap) -> task
  std::map<std::pair<int32_t, int32_t>, int32_t> counter_of;      // (pred slot, where slot) -> counter
  std::map<int32_t, int32_t> bitmap_of;                             // where slot -> bitmap index
  struct Needs { bool stats = false, hll = false, dtype = false; };
  std::vector<Needs> col_task_needs;
  Lowering low{pool, n_pred, &p->schema, {}};
  low.patterns = &p->patterns;
  low.regex_blob = &p->regex_blob;

  auto root = [&](int32_t node, int32_t& slot) -> dq_status {
    if (node < 0 || node >= n_pred) return set_error(DQ_E_INVALID, "predicate root %d out of range", node);
    std::string key = canon(pool, n_pred, node);
    auto it = root_slot.find(key);
    if (it != root_slot.end()) { slot = it->second; return DQ_OK; }
    if ((int32_t)root_slot.size() >= kMaxRoots) return cap_error("more than %d distinct predicates", kMaxRoots);
    low.out.clear();
    if (dq_status s = low.lower(node, 0)) return s;
    slot = (int32_t)root_slot.size();
    root_slot[key] = slot;
    root_code.push_back(low.out);
    return DQ_OK;
  };
  auto notnull_root = [&](int32_t col, int32_t& slot) -> dq_status {
    std::string key = "notnull:" + std::to_string(col);
    auto it = root_slot.find(key);
    if (it != root_slot.end()) { slot = it->second; return DQ_OK; }
    if ((int32_t)root_slot.size() >= kMaxRoots) return cap_error("more than %d distinct predicates", kMaxRoots);
    PredInstr ins{};
    ins.op = PO_ATOM_NOTNULL; ins.col_a = col; ins.col_b = -1;
    slot = (int32_t)root_slot.size();
    root_slot[key] = slot;
    root_code.push_back({ins});
    return DQ_OK;
  };
  auto counter = [&](int32_t pred, int32_t where, int32_t& c) -> dq_status {
    auto key = std::make_pair(pred, where);
    auto it = counter_of.find(key);
    if (it != counter_of.end()) { c = it->second; return DQ_OK; }
    if ((int32_t)counter_of.size() >= kMaxCounters) return cap_error("more than %d predicate counters", kMaxCounters);
    c = (int32_t)counter_of.size();
    counter_of[key] = c;
    return DQ_OK;
  };
  auto bitmap = [&](int32_t where_slot, int32_t& b) -> dq_status {
    if (where_slot < 0) { b = -1; return DQ_OK; }
    auto it = bitmap_of.find(where_slot);
    if (it != bitmap_of.end()) { b = it->second; return DQ_OK; }
    if ((int32_t)bitmap_of.size() >= kMaxWhere) return cap_error("more than %d distinct where filters on value analyzers", kMaxWhere);
    b = (int32_t)bitmap_of.size();
    bitmap_of[where_slot] = b;
    return DQ_OK;
  };
  auto col_task = [&](int32_t col, int32_t bm, bool stats, bool hll, int32_t& t, bool dtype = false) -> dq_status {
    // a double / float / decimal column's DataType count is a variant of its own (CV_F64_D / CV_F32_D / CV_D128_D)
    auto key = std::make_tuple(col, bm, dtype && (is_floating(p->schema[col].type) || is_decimal(p->schema[col].type)) ? 1 : 0);
    auto it = col_task_of.find(key);
    if (it == col_task_of.end()) {
      if ((int32_t)p->col_tasks.size() >= kMaxColTasks) return cap_error("more than %d column tasks", kMaxColTasks);
      t = (int32_t)p->col_tasks.size();
      col_task_of[key] = t;
      ColTask ct{};
      ct.col = col; ct.where = bm; ct.hll_slot = -1; ct.variant = CV_VALIDITY;
      p->col_tasks.push_back(ct);
      col_task_needs.push_back(Needs{});
    } else {
      t = it->second;
    }
    col_task_needs[t].stats |= stats;
    col_task_needs[t].hll |= hll;
    col_task_needs[t].dtype |= dtype;
    return DQ_OK;
  };

  p->outs.resize(p->specs.size());
  for (size_t i = 0; i < p->specs.size(); ++i) {
    const dq_analyzer_spec& s = p->specs[i];
    SpecOut& o = p->outs[i];
    o.op = s.op;
    auto need_col = [&](int32_t c) -> dq_status {
      if (c < 0 || c >= ncols) return set_error(DQ_E_INVALID, "spec %zu: column %d out of range", i, c);
      return DQ_OK;
    };
    int32_t where_slot = -1;
    if (s.where_root >= 0) {
      if (dq_status st = root(s.where_root, where_slot)) return st;
      o.has_where = true;
    }
    switch (s.op) {
      case DQ_OP_SIZE:
        if (where_slot >= 0) {
          if (dq_status st = counter(where_slot, -1, o.ctr_b)) return st;
        }
        break;
      case DQ_OP_COMPLETENESS: {
        if (dq_status st = need_col(s.col_a)) return st;
        o.col_type = p->schema[s.col_a].type;
        if (where_slot >= 0) {
          int32_t nn;
          if (dq_status st = notnull_root(s.col_a, nn)) return st;
          if (dq_status st = counter(nn, where_slot, o.ctr_a)) return st;
          if (dq_status st = counter(where_slot, -1, o.ctr_b)) return st;
        } else if (p->schema[s.col_a].nullable) {
          if (dq_status st = col_task(s.col_a, -1, false, false, o.col_task)) return st;
        }
        break;
      }
      case DQ_OP_COMPLIANCE:
      case DQ_OP_PATTERN_MATCH: {  // PatternMatch = Compliance over the regexp_extract(...) != '' atom
        int32_t ps;
        if (s.pred_root < 0) return set_error(DQ_E_INVALID, "spec %zu: Compliance without predicate", i);
        if (s.op == DQ_OP_PATTERN_MATCH) {
          if (s.pred_root >= n_pred || pool[s.pred_root].kind != DQ_PRED_REGEX ||
              pool[s.pred_root].cmp != DQ_REGEX_EXTRACT_NONEMPTY)
            return set_error(DQ_E_INVALID, "spec %zu: PatternMatch needs a DQ_PRED_REGEX root (extract mode)", i);
        }
        if (dq_status st = root(s.pred_root, ps)) return st;
        if (dq_status st = counter(ps, where_slot, o.ctr_a)) return st;
        if (where_slot >= 0)
          if (dq_status st = counter(where_slot, -1, o.ctr_b)) return st;
        break;
      }
      case DQ_OP_SUM:
      case DQ_OP_MEAN:
      case DQ_OP_STDDEV:
      case DQ_OP_MIN:
      case DQ_OP_MAX:
      case DQ_OP_APPROX_COUNT_DISTINCT: {
        if (dq_status st = need_col(s.col_a)) return st;
        o.col_type = p->schema[s.col_a].type;
        bool hll = s.op == DQ_OP_APPROX_COUNT_DISTINCT;
        if (!hll && !is_numeric(o.col_type))  // Preconditions.isNumeric (Analyzer.scala:322-334)
          return set_error(DQ_E_TYPE, "spec %zu: column %d is not numeric", i, s.col_a);
        int32_t bm;
        if (dq_status st = bitmap(where_slot, bm)) return st;
        if (dq_status st = col_task(s.col_a, bm, !hll, hll, o.col_task)) return st;
        break;
      }
      case DQ_OP_DATATYPE: {  // DataType.scala:157-159: stateful_datatype(conditionalSelection(column, where))
        if (dq_status st = need_col(s.col_a)) return st;
        o.col_type = p->schema[s.col_a].type;
        int32_t bm;
        if (dq_status st = bitmap(where_slot, bm)) return st;
        // only floating-point, decimal and string values need classifying: an integral value's string always matches
        // INTEGRAL, a boolean's ("true" / "false") BOOLEAN, a date's / timestamp's ("2020-01-31 ...") STRING -- the
        // selected-row count suffices (dq_finish puts it in the type's class)
        const bool classify = is_floating(o.col_type) || is_string(o.col_type) || is_decimal(o.col_type);
        if (dq_status st = col_task(s.col_a, bm, false, false, o.col_task, classify)) return st;
        break;
      }
      case DQ_OP_CORRELATION: {
        if (dq_status st = need_col(s.col_a)) return st;
        if (dq_status st = need_col(s.col_b)) return st;
        if (!is_numeric(p->schema[s.col_a].type) || !is_numeric(p->schema[s.col_b].type))
          return set_error(DQ_E_TYPE, "spec %zu: Correlation needs numeric columns", i);
        int32_t bm;
        if (dq_status st = bitmap(where_slot, bm)) return st;
        auto key = std::make_tuple(s.col_a, s.col_b, bm);
        auto it = pair_of.find(key);
        if (it == pair_of.end()) {
          o.pair_task = (int32_t)p->pair_tasks.size();
          pair_of[key] = o.pair_task;
          PairTask pt{};
          pt.col_x = s.col_a; pt.col_y = s.col_b;
          pt.kind_x = pair_kind(p->schema[s.col_a].type); pt.kind_y = pair_kind(p->schema[s.col_b].type);
          pt.where = bm;
          p->pair_tasks.push_back(pt);
        } else {
          o.pair_task = it->second;
        }
        break;
      }
      default:
        return set_error(DQ_E_INVALID, "spec %zu: unknown op %d", i, s.op);
    }
  }

  // column task variants
  for (size_t t = 0; t < p->col_tasks.size(); ++t) {
    ColTask& ct = p->col_tasks[t];
    const bool stats = col_task_needs[t].stats, hll = col_task_needs[t].hll, dtype = col_task_needs[t].dtype;
    int32_t type = p->schema[ct.col].type;
    if (hll) ct.hll_slot = p->n_hll++;
    if (is_decimal(type)) ct.arg = DQ_DECIMAL_PRECISION(type) | DQ_DECIMAL_SCALE(type) << 8;
    if (dtype && type == DQ_TYPE_F64) ct.variant = CV_F64_D;
    else if (dtype && type == DQ_TYPE_F32) ct.variant = CV_F32_D;
    else if (dtype && is_decimal(type)) ct.variant = CV_D128_D;
    else if (!stats && !hll && !dtype) ct.variant = CV_VALIDITY;
    else if (is_decimal(type)) ct.variant = stats && hll ? CV_D128_SH : (stats ? CV_D128_S : CV_D128_H);
    else if (type == DQ_TYPE_UTF8) ct.variant = hll && dtype ? CV_UTF8_HD : (dtype ? CV_UTF8_D : CV_UTF8_H);
    else if (type == DQ_TYPE_LARGE_UTF8) ct.variant = hll && dtype ? CV_LUTF8_HD : (dtype ? CV_LUTF8_D : CV_LUTF8_H);
    else if (type == DQ_TYPE_BOOL) ct.variant = CV_BOOL;  // (HLL only: a boolean is not numeric)
    else {
      int base;
      switch (kind_of(type)) {
        case CK_F64: base = CV_F64_S; break;
        case CK_I64: base = CV_I64_S; break;  // (+ TimestampType: hashLong of the micros)
        case CK_F32: base = CV_F32_S; break;
        case CK_I16: base = CV_I16_S; break;
        case CK_I8: base = CV_I8_S; break;
        default: base = CV_I32_S; break;  // (+ DateType: hashInt of the days)
      }
      ct.variant = base + (stats && hll ? 1 : (stats ? 0 : 2));
    }
  }

  // predicate program: roots in slot order, each followed by STORE
  p->has_pred = !root_code.empty() && (!counter_of.empty() || !bitmap_of.empty());
  PredProgram& prog = p->prog;
  std::memset(&prog, 0, sizeof(prog));
  if (p->has_pred) {
    std::vector<PredInstr> code;
    for (size_t r = 0; r < root_code.size(); ++r) {
      for (const PredInstr& ins : root_code[r]) code.push_back(ins);
      PredInstr st{};
      st.op = PO_STORE; st.slot = (int32_t)r; st.col_a = st.col_b = -1;
      code.push_back(st);
    }
    if ((int32_t)code.size() > kMaxInstr) return cap_error("predicate program too long (%zu instructions, at most %d)", code.size(), kMaxInstr);
    int depth = 0, max_depth = 0;
    for (const PredInstr& ins : code) {
      depth += (ins.op == PO_AND || ins.op == PO_OR || ins.op == PO_STORE) ? -1 : (ins.op == PO_NOT ? 0 : 1);
      max_depth = std::max(max_depth, depth);
    }
    if (max_depth > kPredStack)
      return set_error(DQ_E_UNSUPPORTED, "predicate nesting needs a stack of %d (at most %d)", max_depth, kPredStack);
    prog.stack_depth = std::max(1, max_depth);
    prog.n_roots = (int32_t)root_code.size();
    prog.n_instr = (int32_t)code.size();
    std::copy(code.begin(), code.end(), prog.instr);
    for (int32_t i = 0; i < prog.n_instr; ++i)
      if (prog.instr[i].op == PO_ATOM_CMP || prog.instr[i].op == PO_ATOM_ISNULL || prog.instr[i].op == PO_ATOM_NOTNULL ||
          prog.instr[i].op == PO_ATOM_REGEX)
        prog.load_instr[prog.n_loads++] = (int16_t)i;
    prog.n_counters = (int32_t)counter_of.size();
    for (auto& kv : counter_of) prog.counters[kv.second] = PredCounter{kv.first.first, kv.first.second};
    prog.n_bitmaps = (int32_t)bitmap_of.size();
    for (auto& kv : bitmap_of) prog.bitmap_root[kv.second] = kv.first;
  }
  if (p->regex_blob.size() > (size_t)kMaxRegexWords)
    return cap_error("compiled patterns need %zu KB (LDS budget %d KB)", p->regex_blob.size() * 2 / 1024,
                     kMaxRegexWords * 2 / 1024);
  if (p->probe) {  // capacity probe (dq_plan_create's split): every capacity check is above
    // COMPILED: the generated kernel's own limits (<= 8 value columns, 16 counters, ...) are capacities too,
    // so the greedy split never grows a part past what pred_jit_eligible takes
    if (p->has_pred && p->pred_pass == DQ_PRED_PASS_COMPILED) {
      std::vector<int32_t> kinds(ncols);
      for (int c = 0; c < ncols; ++c) kinds[c] = kind_of(p->schema[c].type);
      if (!pred_jit_eligible(p->prog, kinds.data(), ncols, true))
        return cap_error("compiled predicate pass: program not eligible (regex / string atoms, > 8 columns, or > 16 "
                         "counters / 8 where bitmaps / 96 instructions)");
    }
    return DQ_OK;
  }

  // the predicate program compiled into its own kernel when the generator takes it; HLL-only tasks (no
  // `where`) on its columns are hashed there (fused = 2) instead of re-reading the column in the column pass
  std::vector<int> pred_fused(p->col_tasks.size(), 0);
  if (p->has_pred && p->pred_pass != DQ_PRED_PASS_INTERPRETER) {
    std::vector<int32_t> kinds(ncols);
    for (int c = 0; c < ncols; ++c) kinds[c] = kind_of(p->schema[c].type);
    if (pred_jit_eligible(p->prog, kinds.data(), ncols)) {
      std::vector<int32_t> slots;
      (void)pred_jit_source(p->prog, kinds.data(), slots, {});
      std::vector<PredJitHll> hll;
      std::vector<int32_t> tasks;
      for (size_t t = 0; t < p->col_tasks.size() && hll.size() < 8; ++t) {
        const ColTask& ct = p->col_tasks[t];
        if (ct.where >= 0 || (ct.variant != CV_F64_H && ct.variant != CV_I64_H && ct.variant != CV_I32_H)) continue;
        for (size_t i = 0; i < slots.size(); ++i)
          if (slots[i] == ct.col) {
            hll.push_back(PredJitHll{(int32_t)i});
            tasks.push_back((int32_t)t);
          }
      }
      const std::string src = pred_jit_source(p->prog, kinds.data(), slots, hll);
      std::string note = "generator declined the program";
      if (p->host_only) {
        p->pred_jit_src = src;
        note = src.empty() ? note : "host-only plan: kernel generated, not compiled";
      } else if (!src.empty()) {
        // AUTO: hipRTC on a background thread (a cold compile takes ~0.3 s); the scan starts on the interpreter
        // and switches to the compiled kernel between chunks once it is ready (dq_scan).  COMPILED: wait for it.
        const bool bg = p->pred_pass == DQ_PRED_PASS_AUTO;
        p->pred_jit_ref = pred_jit_request(src, p->device, bg, p->pred_jit_ms);
        p->pred_jit = pred_jit_poll(p->pred_jit_ref, bg ? 0 : -1, note);
        if (p->pred_jit || !pred_jit_pending(p->pred_jit_ref)) p->pred_jit_ref.reset();
      }
      p->pred_jit_note = note;
      // the fused arrangement (HLL tasks in the predicate kernel) whenever the kernel exists or is on its way;
      // until it is there, dq_scan runs those tasks in the column pass (pred_fused_groups)
      if (p->pred_jit || p->pred_jit_ref || (p->host_only && !p->pred_jit_src.empty())) {  // (explain: as compiled)
        p->pred_jit_cols = slots;
        p->pred_jit_hll_task = tasks;
        for (int32_t t : tasks) {
          pred_fused[t] = 2;
          p->pred_jit_hll_slot.push_back(p->col_tasks[t].hll_slot);
        }
      }
    } else {
      p->pred_jit_note = "program not eligible (regex / string atoms, > 8 columns, or > 16 counters / 8 where "
                         "bitmaps / 96 instructions)";
    }
    // (a capacity error: a program too large for the generated kernel splits into parts that fit it; a spec
    // whose program cannot be compiled even alone still fails, with the split's "spec i" message)
    if (!p->pred_jit && !(p->host_only && !p->pred_jit_src.empty()) && p->pred_pass == DQ_PRED_PASS_COMPILED)
      return cap_error("compiled predicate pass required: %s", p->pred_jit_note.c_str());
  } else if (p->has_pred) {
    p->pred_jit_note = "interpreter requested (DQ_PRED_PASS_INTERPRETER)";
  }

  // correlation pairs -> groups of <= kTileCols columns and one `where` (greedy), staged together
  std::vector<PairGroup> pair_groups;
  {
    std::vector<int32_t> order;
    std::vector<PairGroup> groups;
    std::vector<bool> taken(p->pair_tasks.size(), false);
    for (size_t a = 0; a < p->pair_tasks.size(); ++a) {
      if (taken[a]) continue;
      PairGroup g{};
      g.where = p->pair_tasks[a].where;
      g.first_pair = (int32_t)order.size();
      auto local = [&](int32_t col, int32_t kind) -> int32_t {
        for (int c = 0; c < g.ncols; ++c)
          if (g.cols[c] == col) return c;
        if (g.ncols == kTileCols) return -1;
        g.cols[g.ncols] = col;
        g.kinds[g.ncols] = kind;
        return g.ncols++;
      };
      for (size_t b = a; b < p->pair_tasks.size() && g.npairs < kTilePairs; ++b) {
        const PairTask& t = p->pair_tasks[b];
        if (taken[b] || t.where != g.where) continue;
        PairGroup save = g;
        int32_t x = local(t.col_x, t.kind_x), y = local(t.col_y, t.kind_y);
        if (x < 0 || y < 0) { g = save; continue; }
        g.pi[g.npairs] = (int8_t)x;
        g.pj[g.npairs] = (int8_t)y;
        g.npairs++;
        taken[b] = true;
        order.push_back((int32_t)b);
      }
      groups.push_back(g);
    }
    std::vector<PairTask> sorted(order.size());
    std::vector<int32_t> new_index(order.size());
    for (size_t k = 0; k < order.size(); ++k) {
      sorted[k] = p->pair_tasks[order[k]];
      new_index[order[k]] = (int32_t)k;
    }
    p->pair_tasks.swap(sorted);
    pair_groups.swap(groups);
    for (SpecOut& o : p->outs)
      if (o.pair_task >= 0) o.pair_task = new_index[o.pair_task];
  }

  // pair groups -> workgroup tasks of the Correlation pass (dq_pair.hip): the group's pairs and its
  // stats-only column tasks (Mean / StdDev / Sum / Min / Max of the same `where`) over two wave tasks
  std::vector<int> fused(pred_fused);
  for (const PairGroup& g : pair_groups) {
    plan_pair_wgs(p, g, p->pair_wgs, fused);
    for (int c = 0; c < g.ncols; ++c) p->pair_all_f64 = p->pair_all_f64 && g.kinds[c] == CK_F64;
  }

  // sort column tasks by (fused into the pair pass, variant) (stable), remap the analyzers' and lane tasks'
  // task indices, form one launch group per variant of the tasks the column pass still runs
  {
    std::vector<int32_t> order(p->col_tasks.size());
    for (size_t t = 0; t < order.size(); ++t) order[t] = (int32_t)t;
    std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
      if (fused[a] != fused[b]) return fused[a] < fused[b];
      return p->col_tasks[a].variant < p->col_tasks[b].variant;
    });
    std::vector<int32_t> new_index(order.size());
    std::vector<ColTask> sorted(order.size());
    for (size_t k = 0; k < order.size(); ++k) {
      sorted[k] = p->col_tasks[order[k]];
      new_index[order[k]] = (int32_t)k;
    }
    p->col_tasks.swap(sorted);
    for (SpecOut& o : p->outs)
      if (o.col_task >= 0) o.col_task = new_index[o.col_task];
    for (PairWG& wg : p->pair_wgs)
      for (PairWaveTask& w : wg.wave)
        for (int k = 0; k < kPairMoments; ++k)
          if ((w.mom_mask >> k) & 1u) {
            w.mom_out[k] = new_index[w.mom_out[k]];
            for (const SpecOut& o : p->outs)
              if (o.col_task == w.mom_out[k] && (o.op == DQ_OP_MIN || o.op == DQ_OP_MAX)) p->pair_minmax = true;
          }
    for (int32_t& t : p->pred_jit_hll_task) t = new_index[t];
    p->pred_fused_count = (int32_t)std::count(fused.begin(), fused.end(), 2);
    p->pred_fused_first = (int32_t)p->col_tasks.size() - p->pred_fused_count;
    p->pair_fused_count = (int32_t)std::count(fused.begin(), fused.end(), 1);
    p->pair_fused_first = p->pred_fused_first - p->pair_fused_count;
    for (int32_t k = 0; k < (int32_t)p->col_tasks.size(); ++k) {
      if (fused[order[k]]) break;  // fused tasks sort last: their partials come from the pair / predicate pass
      if (p->groups.empty() || p->groups.back().variant != p->col_tasks[k].variant)
        p->groups.push_back({p->col_tasks[k].variant, k, 0});
      p->groups.back().count++;
    }
    for (int32_t k = p->pred_fused_first; k < (int32_t)p->col_tasks.size(); ++k) {
      if (p->pred_fused_groups.empty() || p->pred_fused_groups.back().variant != p->col_tasks[k].variant)
        p->pred_fused_groups.push_back({p->col_tasks[k].variant, k, 0});
      p->pred_fused_groups.back().count++;
    }
    p->n_fused = (int32_t)std::count_if(fused.begin(), fused.end(), [](int f) { return f != 0; });
  }

  // algorithmic bytes per row: each (column, buffer) read once
  std::vector<int> need_values(ncols, 0), need_validity(ncols, 0);
  for (const ColTask& ct : p->col_tasks) {
    need_validity[ct.col] = 1;
    if (ct.variant != CV_VALIDITY) need_values[ct.col] = 1;
  }
  for (const PairTask& pt : p->pair_tasks) {
    need_values[pt.col_x] = need_values[pt.col_y] = 1;
    need_validity[pt.col_x] = need_validity[pt.col_y] = 1;
  }
  for (int i = 0; i < prog.n_instr; ++i) {
    const PredInstr& ins = prog.instr[i];
    if (ins.col_a >= 0) {
      need_validity[ins.col_a] = 1;
      if (ins.op == PO_ATOM_CMP || ins.op == PO_ATOM_REGEX) need_values[ins.col_a] = 1;  // regex: offsets
    }
    if (ins.col_b >= 0) { need_validity[ins.col_b] = 1; need_values[ins.col_b] = 1; }
  }
  int64_t b1000 = 0;
  for (int c = 0; c < ncols; ++c) {
    int32_t t = p->schema[c].type;
    if (need_values[c]) b1000 += value_bytes_x1000(t);  // value or offset bytes
    if (need_validity[c] && p->schema[c].nullable) b1000 += 125;
  }
  p->bytes_per_row_x1000 = b1000;
  // per-kernel algorithmic bytes: the predicate pass (its atoms' columns) and the pair pass (its columns)
  {
    auto bytes_of = [&](const std::vector<int>& vals, const std::vector<int>& valid) {
      int64_t b = 0;
      for (int c = 0; c < ncols; ++c) {
        int32_t t = p->schema[c].type;
        if (vals[c]) b += value_bytes_x1000(t);
        if (valid[c] && p->schema[c].nullable) b += 125;
      }
      return b;
    };
    std::vector<int> pv(ncols, 0), pn(ncols, 0), qv(ncols, 0), qn(ncols, 0);
    for (int i = 0; i < prog.n_instr; ++i) {
      const PredInstr& ins = prog.instr[i];
      if (ins.col_a >= 0) { pn[ins.col_a] = 1; if (ins.op == PO_ATOM_CMP || ins.op == PO_ATOM_REGEX) pv[ins.col_a] = 1; }
      if (ins.col_b >= 0) { pn[ins.col_b] = 1; pv[ins.col_b] = 1; }
    }
    for (const PairTask& pt : p->pair_tasks) { qv[pt.col_x] = qv[pt.col_y] = qn[pt.col_x] = qn[pt.col_y] = 1; }
    p->pred_bytes_x1000 = bytes_of(pv, pn);
    p->pair_bytes_x1000 = bytes_of(qv, qn);
  }
  p->launches_per_scan = (p->has_pred ? 1 : 0) + (int32_t)p->groups.size() + (p->pair_wgs.empty() ? 0 : 1) +
                         ((p->col_tasks.size() + p->pair_tasks.size()) ? 1 : 0);

  if (p->host_only) return DQ_OK;

  // device allocations
  const size_t nct = p->col_tasks.size(), npt = p->pair_tasks.size();
  if (dq_status s = dmalloc(&p->d_col_tasks, nct * sizeof(ColTask))) return s;
  if (dq_status s = dmalloc(&p->d_pair_tasks, npt * sizeof(PairTask))) return s;
  if (dq_status s = dmalloc(&p->d_pair_wgs, p->pair_wgs.size() * sizeof(PairWG))) return s;
  if (!p->pair_wgs.empty())
    HIP_TRY(hipMemcpyAsync(p->d_pair_wgs, p->pair_wgs.data(), p->pair_wgs.size() * sizeof(PairWG),
                           hipMemcpyHostToDevice, p->stream));
  if (dq_status s = dmalloc(&p->d_pair_redo, p->pair_wgs.size() * kPairWaves * kMaxWG * sizeof(int32_t))) return s;
  if (dq_status s = dmalloc(&p->d_prog, sizeof(PredProgram))) return s;
  if (dq_status s = dmalloc(&p->d_col_part, nct * kMaxWG * sizeof(ColPartial))) return s;
  if (dq_status s = dmalloc(&p->d_pair_part, npt * kMaxWG * sizeof(CorrPartial))) return s;
  if (dq_status s = dmalloc(&p->d_pred_part, sizeof(PredPartial))) return s;  // unused (kept for the finalize ABI)
  if (dq_status s = dmalloc(&p->d_col_acc, nct * sizeof(ColPartial))) return s;
  // counters [0, nct) (zeroed by every reset) and the values last published to h_rare [nct, 2 nct)
  if (dq_status s = dmalloc(&p->d_rare_dev, 2 * nct * sizeof(int64_t))) return s;
  if (nct) HIP_TRY(hipMemsetAsync(p->d_rare_dev, 0, 2 * nct * sizeof(int64_t), p->stream));
  p->str_long.assign(nct, 0);
  if (const char* e = std::getenv("DQ_STR_PATH")) p->str_path = std::strcmp(e, "fast") == 0 ? 1 : std::strcmp(e, "long") == 0 ? 2 : 0;
  if (nct && hipHostMalloc(reinterpret_cast<void**>(&p->h_rare), nct * sizeof(int64_t), hipHostMallocMapped) == hipSuccess) {
    std::memset(p->h_rare, 0, nct * sizeof(int64_t));
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, p->h_rare, 0) == hipSuccess) {
      p->d_rare = static_cast<int64_t*>(dp);
    } else {
      (void)hipHostFree(p->h_rare);
      p->h_rare = nullptr;
    }
  }
  (void)hipGetLastError();  // (no mapped memory: the fast variant throughout)
  if (dq_status s = dmalloc(&p->d_hll_acc, (size_t)p->n_hll * kHllCopies * 512 * sizeof(uint32_t))) return s;
  if (dq_status s = dmalloc(&p->d_pair_acc, npt * sizeof(CorrPartial))) return s;
  // (kPredAccCopies copies: the compiled predicate pass spreads its counter atomics over them; the host adds them)
  if (dq_status s = dmalloc(&p->d_pred_acc, kPredAccCopies * sizeof(PredPartial))) return s;
  if (nct) HIP_TRY(hipMemcpyAsync(p->d_col_tasks, p->col_tasks.data(), nct * sizeof(ColTask), hipMemcpyHostToDevice, p->stream));
  if (npt) HIP_TRY(hipMemcpyAsync(p->d_pair_tasks, p->pair_tasks.data(), npt * sizeof(PairTask), hipMemcpyHostToDevice, p->stream));
  if (!p->regex_blob.empty()) {
    if (dq_status s = dmalloc(&p->d_regex, p->regex_blob.size() * sizeof(uint16_t))) return s;
    HIP_TRY(hipMemcpyAsync(p->d_regex, p->regex_blob.data(), p->regex_blob.size() * sizeof(uint16_t),
                           hipMemcpyHostToDevice, p->stream));
  }
  p->prog.regex = p->d_regex;
  p->prog.regex_words = (int32_t)p->regex_blob.size();
  HIP_TRY(hipMemcpyAsync(p->d_prog, &p->prog, sizeof(PredProgram), hipMemcpyHostToDevice, p->stream));
  if (dq_status s = reset_acc(p)) return s;
  HIP_TRY(hipStreamSynchronize(p->stream));
  return DQ_OK;
}


// ------------------------------------------------------------------------------------------
// Splitting an analyzer set over one plan's capacity (composite plans)
// ------------------------------------------------------------------------------------------
// The reference fuses any number of scan-shareable analyzers into one data.agg
// (AnalysisRunner.scala:293-303).  One plan here has fixed capacities (kMaxCols columns, kMaxRoots distinct
// predicates, kMaxCounters counters, kMaxWhere `where` bitmaps, kMaxColTasks column tasks, kMaxInstr program
// instructions, kMaxRegexWords of DFAs); an analyzer set over any of them is planned as several fused plans
// over disjoint spec subsets.  Every part is one fused pass over the same chunks, merged in chunk order, so
// each analyzer's state is exactly the one a single plan would produce (the states of different analyzers
// are independent); a column shared by two parts is read once per part.

static void pred_columns(const dq_pred_node* pool, int32_t n_pred, int32_t idx, std::vector<int32_t>& cols,
                         int depth = 0) {
  if (idx < 0 || idx >= n_pred || depth > 64) return;
  const dq_pred_node& n = pool[idx];
  switch (n.kind) {
    case DQ_PRED_COLUMN: cols.push_back(n.a); return;
    case DQ_PRED_CMP: case DQ_PRED_AND: case DQ_PRED_OR: case DQ_PRED_COALESCE:
      pred_columns(pool, n_pred, n.a, cols, depth + 1);
      pred_columns(pool, n_pred, n.b, cols, depth + 1);
      return;
    case DQ_PRED_NOT: case DQ_PRED_IS_NULL: case DQ_PRED_IS_NOT_NULL: case DQ_PRED_REGEX:
      pred_columns(pool, n_pred, n.a, cols, depth + 1);
      return;
    default: return;
  }
}

// the schema columns a spec reads (sorted, unique; out-of-range indices are left to the part's own planning)
static std::vector<int32_t> spec_columns(const dq_analyzer_spec& s, const dq_pred_node* pool, int32_t n_pred,
                                         int32_t ncols) {
  std::vector<int32_t> c;
  if (s.op == DQ_OP_CORRELATION) { c.push_back(s.col_a); c.push_back(s.col_b); }
  else if (s.op != DQ_OP_SIZE && s.op != DQ_OP_COMPLIANCE) c.push_back(s.col_a);
  pred_columns(pool, n_pred, s.pred_root, c);
  pred_columns(pool, n_pred, s.where_root, c);
  c.erase(std::remove_if(c.begin(), c.end(), [&](int32_t x) { return x < 0 || x >= ncols; }), c.end());
  std::sort(c.begin(), c.end());
  c.erase(std::unique(c.begin(), c.end()), c.end());
  return c;
}

// one part's inputs: its specs and predicate pool with columns renumbered into its own schema
struct PartInput {
  std::vector<dq_analyzer_spec> specs;
  std::vector<dq_column_desc> schema;
  std::vector<dq_pred_node> pool;
};

static void make_part_input(const std::vector<dq_analyzer_spec>& specs, const std::vector<dq_column_desc>& schema,
                            const dq_pred_node* pool, int32_t n_pred, const std::vector<int32_t>& spec_idx,
                            const std::vector<int32_t>& cols, PartInput& in) {
  const int32_t ncols = (int32_t)schema.size();
  std::vector<int32_t> local(ncols, -1);
  in.schema.clear();
  for (size_t j = 0; j < cols.size(); ++j) {
    local[cols[j]] = (int32_t)j;
    in.schema.push_back(schema[cols[j]]);
  }
  auto map = [&](int32_t c) { return c >= 0 && c < ncols ? local[c] : -1; };
  in.specs.clear();
  for (int32_t i : spec_idx) {
    dq_analyzer_spec sp = specs[i];
    if (sp.col_a >= 0) sp.col_a = map(sp.col_a);
    if (sp.col_b >= 0) sp.col_b = map(sp.col_b);
    in.specs.push_back(sp);
  }
  in.pool.assign(pool, pool + n_pred);
  for (dq_pred_node& n : in.pool)
    if (n.kind == DQ_PRED_COLUMN) n.a = map(n.a);  // a column outside the part is not reachable from its roots
}

// host-only planning of one part (capacity probe, or the plan dq_plan_explain describes)
static dq_status plan_part_host(const dq_plan& parent, const dq_pred_node* pool, int32_t n_pred,
                                const std::vector<int32_t>& spec_idx, const std::vector<int32_t>& cols, bool probe,
                                dq_plan& q) {
  PartInput in;
  make_part_input(parent.specs, parent.schema, pool, n_pred, spec_idx, cols, in);
  q.host_only = true;
  q.probe = probe;
  q.schema = in.schema;
  q.specs = in.specs;
  q.patterns = parent.patterns;
  q.pred_pass = parent.pred_pass;
  g_capacity = false;
  return build_plan(&q, in.pool.data(), (int32_t)in.pool.size());
}

// Greedy split: specs in order of their lowest column (a column's analyzers -- ColumnProfiler emits them per
// column -- land in one part, so each column is read by as few parts as possible), each part grown while it
// fits.  Specs without predicates or `where` only add column tasks (at most one each); the others are checked
// by a host-only probe of the grown part.  A spec that does not fit a part by itself is an error (its own
// status: DQ_E_UNSUPPORTED routes it to the fallback set, DQ_E_INVALID / DQ_E_TYPE are spec errors).
static dq_status partition_specs(const dq_plan& parent, const dq_pred_node* pool, int32_t n_pred,
                                 std::vector<std::vector<int32_t>>& part_specs,
                                 std::vector<std::vector<int32_t>>& part_cols) {
  const int32_t ns = (int32_t)parent.specs.size(), ncols = (int32_t)parent.schema.size();
  std::vector<std::vector<int32_t>> sc(ns);
  std::vector<int32_t> order(ns);
  for (int32_t i = 0; i < ns; ++i) {
    sc[i] = spec_columns(parent.specs[i], pool, n_pred, ncols);
    order[i] = i;
  }
  std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
    return (sc[a].empty() ? -1 : sc[a][0]) < (sc[b].empty() ? -1 : sc[b][0]);
  });
  std::vector<int32_t> cur, cur_cols;
  int32_t cur_tasks = 0;
  auto probe = [&](const std::vector<int32_t>& idx, const std::vector<int32_t>& cols) {
    std::unique_ptr<dq_plan> q(new dq_plan());
    return plan_part_host(parent, pool, n_pred, idx, cols, true, *q);
  };
  auto start = [&](int32_t i) -> dq_status {
    if ((int32_t)sc[i].size() > kMaxCols)
      return set_error(DQ_E_UNSUPPORTED, "spec %d reads %zu columns (one plan reads at most %d)", i, sc[i].size(), kMaxCols);
    cur.assign(1, i);
    cur_cols = sc[i];
    cur_tasks = 1;
    if (dq_status st = probe(cur, cur_cols)) {
      std::string msg = g_err;
      return set_error(st, "spec %d: %s", i, msg.c_str());
    }
    return DQ_OK;
  };
  auto close = [&] {
    if (cur.empty()) return;
    part_specs.push_back(cur);
    part_cols.push_back(cur_cols);
    cur.clear();
    cur_cols.clear();
  };
  for (int32_t i : order) {
    if (cur.empty()) {
      if (dq_status st = start(i)) return st;
      continue;
    }
    std::vector<int32_t> u;
    std::set_union(cur_cols.begin(), cur_cols.end(), sc[i].begin(), sc[i].end(), std::back_inserter(u));
    bool fits = (int32_t)u.size() <= kMaxCols;
    const dq_analyzer_spec& s = parent.specs[i];
    if (fits && (s.pred_root >= 0 || s.where_root >= 0 || cur_tasks + 1 > kMaxColTasks)) {
      std::vector<int32_t> trial(cur);
      trial.push_back(i);
      dq_status st = probe(trial, u);
      if (st != DQ_OK && !g_capacity) {
        std::string msg = g_err;
        return set_error(st, "spec %d: %s", i, msg.c_str());
      }
      fits = st == DQ_OK;
    }
    if (fits) {
      cur.push_back(i);
      cur_cols.swap(u);
      ++cur_tasks;
    } else {
      close();
      if (dq_status st = start(i)) return st;
    }
  }
  close();
  return DQ_OK;
}

static int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// dq_plan_explain's description of one (host-only) plan
static std::string explain_text(const dq_plan& plan) {
  std::string t;
  char line[256];
  for (const auto& g : plan.groups) {
    std::snprintf(line, sizeof line, "column pass: variant %d, %d task(s)\n", g.variant, g.count);
    t += line;
  }
  std::snprintf(line, sizeof line, "pair pass: %zu pair(s), %zu workgroup task(s)\n", plan.pair_tasks.size(),
                plan.pair_wgs.size());
  t += line;
  if (plan.has_pred) {
    std::snprintf(line, sizeof line, "predicate program: %d instructions, %d roots, %d counters, %d bitmaps\n",
                  plan.prog.n_instr, plan.prog.n_roots, plan.prog.n_counters, plan.prog.n_bitmaps);
    t += line;
    t += "predicate pass: " + plan.pred_jit_note + "\n";
    if (!plan.pred_jit_src.empty()) t += "--- generated kernel source ---\n" + plan.pred_jit_src;
  }
  return t;
}

extern "C" {

int32_t dq_abi_version(void) { return DQ_ABI_VERSION; }
const char* dq_last_error(void) { return g_err; }

dq_status dq_plan_create(const dq_analyzer_spec* specs, int32_t n_specs, const dq_column_desc* schema, int32_t n_cols,
                         const dq_pred_node* pred_pool, int32_t n_pred, int32_t device, dq_plan** out) {
  return dq_plan_create_ex(specs, n_specs, schema, n_cols, pred_pool, n_pred, nullptr, 0, device, out);
}

dq_status dq_plan_create_ex(const dq_analyzer_spec* specs, int32_t n_specs, const dq_column_desc* schema,
                            int32_t n_cols, const dq_pred_node* pred_pool, int32_t n_pred,
                            const char* const* patterns, int32_t n_patterns, int32_t device, dq_plan** out) {
  return dq_plan_create_opts(specs, n_specs, schema, n_cols, pred_pool, n_pred, patterns, n_patterns, nullptr, device,
                             out);
}

// one plan over the whole spec set (the capacity flag tells dq_plan_create_opts to split instead)
static dq_status create_single(const std::vector<dq_analyzer_spec>& specs, const std::vector<dq_column_desc>& schema,
                               const dq_pred_node* pred_pool, int32_t n_pred, const std::vector<std::string>& patterns,
                               int32_t pred_pass, int32_t device, dq_plan** out) {
  g_capacity = false;
  if ((int32_t)schema.size() > kMaxCols) return cap_error("more than %d columns in one plan", kMaxCols);
  dq_plan* p = new dq_plan();
  p->device = device;
  p->schema = schema;
  p->specs = specs;
  p->patterns = patterns;
  hipError_t e = hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete p;
    return set_error(DQ_E_HIP, "hipStreamCreate: %s", hipGetErrorString(e));
  }
  p->own_stream = true;
  p->pred_pass = pred_pass;
  dq_status st = build_plan(p, pred_pool, n_pred);
  if (st != DQ_OK) {
    const bool cap = g_capacity;
    std::string msg = g_err;
    dq_plan_destroy(p);
    g_capacity = cap;
    return set_error(st, "%s", msg.c_str());
  }
  *out = p;
  return DQ_OK;
}

dq_status dq_plan_create_opts(const dq_analyzer_spec* specs, int32_t n_specs, const dq_column_desc* schema,
                              int32_t n_cols, const dq_pred_node* pred_pool, int32_t n_pred,
                              const char* const* patterns, int32_t n_patterns, const dq_plan_options* opts,
                              int32_t device, dq_plan** out) {
  const auto t0 = std::chrono::steady_clock::now();
  if (!out) return set_error(DQ_E_INVALID, "dq_plan_create: out is NULL");
  // options: the fields the caller's struct_size covers, defaults past it
  dq_plan_options o{};
  o.struct_size = (int32_t)sizeof(dq_plan_options);
  if (opts) {
    if (opts->struct_size < (int32_t)(2 * sizeof(int32_t)))
      return set_error(DQ_E_INVALID, "dq_plan_create: dq_plan_options.struct_size %d too small", opts->struct_size);
    std::memcpy(&o, opts, std::min((size_t)opts->struct_size, sizeof(o)));
  }
  if (o.pred_pass < DQ_PRED_PASS_AUTO || o.pred_pass > DQ_PRED_PASS_COMPILED)
    return set_error(DQ_E_INVALID, "dq_plan_create: unknown pred_pass %d", o.pred_pass);
  if (n_patterns < 0 || (n_patterns > 0 && !patterns)) return set_error(DQ_E_INVALID, "dq_plan_create: bad patterns");
  for (int32_t k = 0; k < n_patterns; ++k)
    if (!patterns[k]) return set_error(DQ_E_INVALID, "dq_plan_create: pattern %d is NULL", k);
  *out = nullptr;
  if (n_specs < 0 || (n_specs > 0 && !specs)) return set_error(DQ_E_INVALID, "dq_plan_create: bad specs");
  if (n_cols < 0 || n_cols > kMaxSchemaCols || (n_cols > 0 && !schema))
    return set_error(DQ_E_INVALID, "dq_plan_create: bad schema (at most %d columns)", kMaxSchemaCols);
  if (n_pred < 0 || (n_pred > 0 && !pred_pool)) return set_error(DQ_E_INVALID, "dq_plan_create: bad predicate pool");
  for (int32_t c = 0; c < n_cols; ++c)
    if (!type_valid(schema[c].type))
      return set_error(DQ_E_TYPE, "dq_plan_create: column %d has unknown type %d", c, schema[c].type);
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return set_error(DQ_E_INVALID, "dq_plan_create: device %d of %d", device, ndev);
  HIP_TRY(hipSetDevice(device));
  const std::vector<dq_analyzer_spec> vspecs(specs, specs + n_specs);
  const std::vector<dq_column_desc> vschema(schema, schema + n_cols);
  std::vector<std::string> vpat;
  for (int32_t k = 0; k < n_patterns; ++k) vpat.emplace_back(patterns[k]);
  dq_plan* p = nullptr;
  dq_status st = create_single(vspecs, vschema, pred_pool, n_pred, vpat, o.pred_pass, device, &p);
  if (st != DQ_OK && !g_capacity) return st;
  if (st != DQ_OK) {
    // over one plan's capacity: several fused plans on this plan's stream
    p = new dq_plan();
    p->device = device;
    p->schema = vschema;
    p->specs = vspecs;
    p->patterns = vpat;
    p->pred_pass = o.pred_pass;
    hipError_t e = hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
      delete p;
      return set_error(DQ_E_HIP, "hipStreamCreate: %s", hipGetErrorString(e));
    }
    p->own_stream = true;
    st = partition_specs(*p, pred_pool, n_pred, p->part_specs, p->part_cols);
    for (size_t k = 0; st == DQ_OK && k < p->part_specs.size(); ++k) {
      PartInput in;
      make_part_input(vspecs, vschema, pred_pool, n_pred, p->part_specs[k], p->part_cols[k], in);
      dq_plan* part = nullptr;
      st = create_single(in.specs, in.schema, in.pool.data(), (int32_t)in.pool.size(), vpat, o.pred_pass, device, &part);
      if (st == DQ_OK) {
        p->parts.push_back(part);
        st = dq_plan_set_stream(part, p->stream);
      } else {
        std::string msg = g_err;
        st = set_error(st, "part %zu of %zu: %s", k, p->part_specs.size(), msg.c_str());
      }
    }
    if (st != DQ_OK) {
      std::string msg = g_err;
      dq_plan_destroy(p);
      return set_error(st, "%s", msg.c_str());
    }
    for (dq_plan* q : p->parts) {
      p->pred_jit_ms += q->pred_jit_ms;
      p->launches_per_scan += q->launches_per_scan;
      p->bytes_per_row_x1000 += q->bytes_per_row_x1000;
      p->pred_bytes_x1000 += q->pred_bytes_x1000;
      p->pair_bytes_x1000 += q->pair_bytes_x1000;
    }
  }
  p->create_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  *out = p;
  return DQ_OK;
}

dq_status dq_plan_set_stream(dq_plan* p, void* hip_stream) {
  if (!p) return set_error(DQ_E_INVALID, "dq_plan_set_stream: plan is NULL");
  HIP_TRY(hipSetDevice(p->device));
  // a composite plan's parts launch on the parent's stream (they never own one): one sync of the old stream
  // covers their work too, then every part moves to the new stream before the old one may be destroyed
  HIP_TRY(hipStreamSynchronize(p->stream));
  for (dq_plan* q : p->parts) {
    if (q->stream != p->stream) HIP_TRY(hipStreamSynchronize(q->stream));  // (not reachable: parts share it)
    if (q->own_stream) (void)hipStreamDestroy(q->stream);
    q->stream = (hipStream_t)hip_stream;
    q->own_stream = false;
  }
  // NULL is the device's null stream (what torch's default stream reports), not "keep the plan's
  // own stream": the plan's own stream is non-blocking and would not wait for producers on it.
  if (p->own_stream) (void)hipStreamDestroy(p->stream);
  p->stream = (hipStream_t)hip_stream;
  p->own_stream = false;
  return DQ_OK;
}

}  // extern "C"

// dq_scan's contract for one column view (dqscan.h dq_column_view)
static dq_status check_view(const dq_column_desc& cd, const dq_column_view& v, int32_t c, int64_t n_rows) {
  const int32_t t = cd.type;
  if (v.reserved != 0) return set_error(DQ_E_INVALID, "dq_scan: column %d reserved field must be 0", c);
  if (n_rows > 0 && !v.values) return set_error(DQ_E_INVALID, "dq_scan: column %d has no values buffer", c);
  if (((uintptr_t)v.values & 15) != 0)
    return set_error(DQ_E_INVALID, "dq_scan: column %d values buffer must be 16-byte aligned", c);
  if (((uintptr_t)v.validity & 3) != 0)
    return set_error(DQ_E_INVALID, "dq_scan: column %d validity bitmap must be 4-byte aligned", c);
  if ((t == DQ_TYPE_UTF8 || t == DQ_TYPE_LARGE_UTF8) && n_rows > 0 && !v.offsets)
    return set_error(DQ_E_INVALID, "dq_scan: UTF8 column %d has no offsets", c);
  return DQ_OK;
}

extern "C" {

dq_status dq_scan(dq_plan* p, const dq_column_view* cols, int64_t n_rows, int64_t chunk_index) {
  if (!p) return set_error(DQ_E_INVALID, "dq_scan: plan is NULL");
  if (n_rows < 0) return set_error(DQ_E_INVALID, "dq_scan: n_rows < 0");
  if (n_rows >= (int64_t(1) << 31))
    return set_error(DQ_E_INVALID, "dq_scan: a chunk holds at most 2^31 - 1 rows (split larger inputs into chunks)");
  if (chunk_index != p->next_chunk)
    return set_error(DQ_E_INVALID, "dq_scan: chunk_index %lld out of order (expected %lld)", (long long)chunk_index,
                     (long long)p->next_chunk);
  const int32_t ncols = (int32_t)p->schema.size();
  if (ncols > 0 && !cols) return set_error(DQ_E_INVALID, "dq_scan: cols is NULL");
  HIP_TRY(hipSetDevice(p->device));
  if (!p->parts.empty()) {  // composite: every part over its own columns of this chunk, in part order
    // every view any part reads is checked before the first part scans: a rejected view must leave every
    // part's chunk count where it was (a partly scanned chunk could not be retried, and dq_finish would
    // merge states over different row sets)
    for (size_t k = 0; k < p->parts.size(); ++k) {
      for (int32_t c : p->part_cols[k])
        if (dq_status s = check_view(p->schema[c], cols[c], c, n_rows)) return s;
      if (p->parts[k]->next_chunk != chunk_index)
        return set_error(DQ_E_INVALID, "dq_scan: part %zu is at chunk %lld (expected %lld)", k,
                         (long long)p->parts[k]->next_chunk, (long long)chunk_index);
    }
    std::vector<dq_column_view> v;
    for (size_t k = 0; k < p->parts.size(); ++k) {
      v.resize(p->part_cols[k].size());
      for (size_t j = 0; j < v.size(); ++j) v[j] = cols[p->part_cols[k][j]];
      if (dq_status s = dq_scan(p->parts[k], v.data(), n_rows, chunk_index)) return s;
    }
    p->next_chunk++;
    p->total_rows += n_rows;
    return DQ_OK;
  }
  ScanCols sc{};
  for (int32_t c = 0; c < ncols; ++c)
    if (dq_status s = check_view(p->schema[c], cols[c], c, n_rows)) return s;
  for (int32_t c = 0; c < ncols; ++c) {
    const dq_column_view& v = cols[c];
    sc.values[c] = v.values;
    sc.validity[c] = p->schema[c].nullable ? reinterpret_cast<const uint32_t*>(v.validity) : nullptr;
    sc.offsets[c] = v.offsets;
  }
  p->next_chunk++;
  if (n_rows == 0) return DQ_OK;
  if (p->pred_jit_ref) {  // a background compile: take the compiled kernel from this chunk on once it is ready
    std::string note;
    if (hipFunction_t fn = pred_jit_poll(p->pred_jit_ref, 0, note)) {
      p->pred_jit = fn;
      p->pred_jit_note = note + " (compiled in the background; used from chunk " + std::to_string(chunk_index) + ")";
      p->pred_jit_ref.reset();
    } else if (!pred_jit_pending(p->pred_jit_ref)) {
      p->pred_jit_note = note;  // the compile failed: the interpreter stays
      p->pred_jit_ref.reset();
    }
  }
  // the launch groups of this scan: without the compiled kernel its HLL tasks run in the column pass
  std::vector<dq_plan::Group> groups(p->groups);
  if (!p->pred_jit) groups.insert(groups.end(), p->pred_fused_groups.begin(), p->pred_fused_groups.end());

  // where bitmaps (64 rows per word), grown on demand
  const int64_t words = ceil_div(n_rows, 64);
  if (p->prog.n_bitmaps > 0 && words > p->where_cap_words) {
    HIP_TRY(hipStreamSynchronize(p->stream));
    for (int b = 0; b < p->prog.n_bitmaps; ++b) {
      if (p->d_where_bits[b]) (void)hipFree(p->d_where_bits[b]);
      p->d_where_bits[b] = nullptr;
      if (dq_status s = dmalloc(&p->d_where_bits[b], (size_t)words * 8 + 64)) return s;
    }
    p->where_cap_words = words;
  }
  ScanBitmaps bm{};
  for (int b = 0; b < kMaxWhere; ++b) bm.where_bits[b] = p->d_where_bits[b];
  bm.rare_rows = p->d_rare_dev;
  // all-ones bitmap standing in for a missing validity / where bitmap in the pair pass and the compiled
  // predicate pass
  if ((!p->pair_wgs.empty() || p->pred_jit) && words + 1 > p->ones_cap_words) {
    HIP_TRY(hipStreamSynchronize(p->stream));
    if (p->d_ones) (void)hipFree(p->d_ones);
    p->d_ones = nullptr;
    if (dq_status s = dmalloc(&p->d_ones, (size_t)(words + 1) * 8)) return s;
    HIP_TRY(hipMemsetAsync(p->d_ones, 0xFF, (size_t)(words + 1) * 8, p->stream));
    p->ones_cap_words = words + 1;
  }

  // row ranges: column / pair passes in multiples of 2048 rows, predicate pass in multiples of 256
  // each variant (and the pair pass) is its own launch of (tasks x ranges) workgroups: size the ranges
  // so the smallest launch still has ~kTargetWGs workgroups (load balance over 256 CUs)
  int64_t min_launch = 0;
  for (const auto& g : groups) min_launch = min_launch ? std::min<int64_t>(min_launch, g.count) : g.count;
  if (!p->pair_wgs.empty()) {
    const int64_t wg = (int64_t)p->pair_wgs.size();
    min_launch = min_launch ? std::min<int64_t>(min_launch, wg) : wg;
  }
  const int64_t want = std::max<int64_t>(64, std::min<int64_t>(kMaxWG, kTargetWGs / std::max<int64_t>(1, min_launch)));
  // rows per range and range count for `want` ranges
  auto size_ranges = [&](int64_t w, int64_t& rpr, int32_t& nr, int64_t min_rows) {
    w = std::min<int64_t>(w, std::max<int64_t>(1, n_rows / min_rows));
    nr = (int32_t)std::min<int64_t>(w, ceil_div(n_rows, kRowsPerIter));
    rpr = ceil_div(ceil_div(n_rows, nr), kRowsPerIter) * kRowsPerIter;
    nr = (int32_t)ceil_div(n_rows, rpr);
  };
  int32_t nr_col;
  int64_t rpr_col;
  size_ranges(want, rpr_col, nr_col, DQ_MIN_RANGE_ROWS);
  // per-variant workgroup counts: the string hash balances better with twice the ranges (uneven string
  // lengths, deferred-round drains): utf8_hll 1.979 -> 1.949 ms per 125 M x 4 on the C5 headline (x3 1.963,
  // x4 1.965 ms); halving the fp64 hash's ranges measured no change
  auto variant_scale = [](int32_t v) -> int32_t {
    return v == CV_UTF8_H || v == CV_LUTF8_H || v == CV_UTF8_HD || v == CV_LUTF8_HD ? 2 : 1;
  };
  // and the fp64 hash with half the ranges: 1.437 -> 1.421 ms per 125 M rows x 8 (r5r; twice the ranges
  // 1.47 -> 1.52, r5q; the int64 hash: half 0.79 -> 0.79-0.80, a quarter 0.82)
  auto variant_div = [](int32_t v) -> int32_t { return v == CV_F64_SH || v == CV_F64_H ? DQ_F64_HLL_DIV : 1; };
  auto variant_min_rows = [](int32_t v) -> int64_t {
    return v == CV_VALIDITY ? DQ_MIN_VALIDITY_RANGE_ROWS : DQ_MIN_RANGE_ROWS;
  };
  FinRanges fr{};
  std::vector<std::pair<int64_t, int32_t>> vr(groups.size());  // (rows per range, ranges) per variant group
  for (size_t gi = 0; gi < groups.size(); ++gi) {
    const auto& g = groups[gi];
    const int32_t sc_v = variant_scale(g.variant);
    const int64_t min_rows = variant_min_rows(g.variant);
    const int32_t div_v = variant_div(g.variant);
    if (sc_v == 1 && div_v == 1 && min_rows == DQ_MIN_RANGE_ROWS) {
      vr[gi] = {rpr_col, nr_col};
      continue;
    }
    size_ranges(std::max<int64_t>(64, std::min<int64_t>(kMaxWG, want * sc_v / div_v)), vr[gi].first, vr[gi].second, min_rows);
    if (vr[gi].second == nr_col && vr[gi].first == rpr_col) continue;  // the default ranges after all
    if (fr.n >= kMaxFinRanges - 2) {  // (cannot happen: one entry per group) the default ranges
      vr[gi] = {rpr_col, nr_col};
      continue;
    }
    fr.first[fr.n] = g.first;
    fr.end[fr.n] = g.first + g.count;
    fr.nr[fr.n] = vr[gi].second;
    ++fr.n;
  }
  // predicate pass: ~2048 workgroups of whole 2048-row iterations (HBM-bound; counters leave by atomics;
  // 1024-16384 workgroups measured within 2 % on C3)
  int32_t nr_pred = (int32_t)std::min<int64_t>(
      DQ_PRED_WGS, std::min<int64_t>(ceil_div(n_rows, kRowsPerIter), std::max<int64_t>(1, n_rows / DQ_MIN_RANGE_ROWS)));
  int64_t rpr_pred = ceil_div(ceil_div(n_rows, nr_pred), kRowsPerIter) * kRowsPerIter;
  nr_pred = (int32_t)ceil_div(n_rows, rpr_pred);

  // the Correlation pass: one resident round -- as many ranges as leave every workgroup of the launch resident
  // at once (the occupancy API x CUs / pair workgroups).  Each workgroup ends with a heavy epilogue (the
  // butterfly sums of 70 accumulators per wave, a counts pass over the range's bitmaps), so the fewer,
  // longer ranges win -- but only while the launch fills the chip in one round: C4 (one pair group, 4
  // workgroups per CU) 1.523-1.528 ms per 125 M rows at 4096 ranges, 1.434-1.435 at 1024, 1.97 at 1365
  // (a partial second round), 2.28 at 512 (half the CUs' slots idle) -- profiles/r5_ab.txt r5t / r5u / r5w.
  // (The column passes, whose epilogue is light, measured slower at one round: fp64 hash 1.42 -> 1.50-1.51,
  // int64 0.79 -> 0.82-0.83, strings 1.94 -> 2.20 ms, r5w.)  Its fused moments tasks' partials follow its
  // range count.
  const bool pair_ring = [&] {
    if (p->pair_wgs.empty() || !p->pair_all_f64) return false;
    for (const PairWG& wg : p->pair_wgs)
      for (const PairWaveTask& t : wg.wave)
        for (int c = 0; c < kPairPos; ++c)
          if (((uintptr_t)sc.values[t.cols[c]] & 15u) != 0) return false;
    return true;
  }();
  int64_t rpr_pair = rpr_col;
  int32_t nr_pair = nr_col;
  if (!p->pair_wgs.empty() && DQ_PAIR_ONE_ROUND) {
    int32_t& res = p->pair_resident[pair_ring ? 1 : 0];
    if (res == 0) {
      int32_t per_cu = 0, cus = 0;
      HIP_TRY(pair_scan_residency(p->pair_all_f64, pair_ring, p->pair_minmax, &per_cu));
      HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, p->device));
      res = std::max<int32_t>(1, per_cu * cus);
    }
    const int64_t per_round = std::max<int64_t>(1, res / (int64_t)p->pair_wgs.size());
    size_ranges(std::min<int64_t>(kMaxWG, per_round), rpr_pair, nr_pair, DQ_MIN_RANGE_ROWS);
    if (nr_pair != nr_col && p->pair_fused_count > 0) {
      fr.first[fr.n] = p->pair_fused_first;
      fr.end[fr.n] = p->pair_fused_first + p->pair_fused_count;
      fr.nr[fr.n] = nr_pair;
      ++fr.n;
    }
  }
  // HLL tasks hashed by the compiled predicate pass: one partial per predicate-pass range
  if (p->pred_jit && p->pred_fused_count > 0) {  // (fr has room: the loop above leaves two entries)
    fr.first[fr.n] = p->pred_fused_first;
    fr.end[fr.n] = p->pred_fused_first + p->pred_fused_count;
    fr.nr[fr.n] = nr_pred;
    ++fr.n;
  }

  // every launch on the plan's stream, in order (the C5 variant launches spread over 2-3 streams measured the
  // same step time: each launch fills the chip)
  if (p->has_pred) {
    if (dq_status s = timed(p, 0, p->stream, [&] {
          if (p->pred_jit) {
            PredJitArgs a{};
            for (size_t i = 0; i < p->pred_jit_cols.size(); ++i) {
              a.values[i] = reinterpret_cast<const char*>(sc.values[p->pred_jit_cols[i]]);
              const uint32_t* vb = sc.validity[p->pred_jit_cols[i]];
              a.validity[i] = vb ? vb : reinterpret_cast<const uint32_t*>(p->d_ones);
            }
            for (int b = 0; b < kMaxWhere && b < 8; ++b) a.where_bits[b] = bm.where_bits[b];
            a.n_rows = n_rows;
            a.rows_per_range = rpr_pred;
            a.acc_t = reinterpret_cast<unsigned long long*>(p->d_pred_acc->t);
            a.acc_nn = reinterpret_cast<unsigned long long*>(p->d_pred_acc->nn);
            a.col_part = reinterpret_cast<char*>(p->d_col_part);
            a.hll_acc = p->d_hll_acc;
            for (size_t h = 0; h < p->pred_jit_hll_task.size(); ++h) {
              a.hll_task[h] = p->pred_jit_hll_task[h];
              a.hll_slot[h] = p->pred_jit_hll_slot[h];
            }
            return pred_jit_launch(p->pred_jit, a, nr_pred, p->stream);
          }
          const int32_t lds = kWaves * 128 * (p->prog.stack_depth + p->prog.n_roots + p->prog.n_counters) +
                              ((p->prog.regex_words * 2 + 15) & ~15);
          return launch_pred_scan(p->d_prog, sc, bm, n_rows, rpr_pred, nr_pred, p->d_pred_acc, lds, p->stream,
                                  p->prog.regex_words > 0);
        }))
      return s;
  }
  // the string pass's variant for a task group (see dq_plan::h_rare): the published rare-path rows are since the
  // reset and may be a chunk behind (read without waiting); the choice only changes speed, never the result
  auto str_long_of = [&](const dq_plan::Group& g) -> bool {
    if (g.variant != CV_UTF8_H && g.variant != CV_LUTF8_H && g.variant != CV_UTF8_HD && g.variant != CV_LUTF8_HD)
      return false;
    if (p->str_path != 0) return p->str_path == 2;
    const int64_t rows = p->total_rows > 0 ? p->total_rows : p->prev_rows;
    bool any = false;
    for (int32_t t = g.first; t < g.first + g.count; ++t) {
      if (p->h_rare && rows > 0) p->str_long[t] = __atomic_load_n(p->h_rare + t, __ATOMIC_RELAXED) * 4096 > rows;
      any = any || p->str_long[t];
    }
    return any;
  };
  for (size_t gi = 0; gi < groups.size(); ++gi) {
    const auto& g = groups[gi];
    if (dq_status s = timed(p, 16 + g.variant, p->stream, [&] {
          return launch_column_scan(g.variant, p->d_col_tasks + g.first, g.count, g.first, sc, bm, n_rows,
                                    vr[gi].first, vr[gi].second, p->d_col_part, p->d_hll_acc, str_long_of(g),
                                    p->stream);
        }))
      return s;
  }
  if (!p->pair_wgs.empty()) {
    // the LDS-ring path's 16-byte DMA needs 16-byte aligned fp64 columns (dq_scan's contract; checked above)
    const bool ring = pair_ring;
    if (dq_status s = timed(p, 2, p->stream, [&] {
          return launch_pair_scan(p->d_pair_wgs, (int32_t)p->pair_wgs.size(), sc, bm, p->d_ones, n_rows, rpr_pair,
                                  nr_pair, p->d_pair_part, p->d_col_part, p->d_pair_redo, p->pair_all_f64, ring,
                                  p->pair_minmax, p->stream);
        }))
      return s;
  }
  if (dq_status s = timed(p, 3, p->stream, [&] {
        return launch_finalize((int32_t)p->col_tasks.size(), nr_col, p->d_col_part, p->d_col_acc,
                               (int32_t)p->pair_tasks.size(), nr_pair, p->d_pair_part, p->d_pair_acc,
                               0 /* the predicate pass accumulates itself */, nr_pred, p->d_pred_part, p->d_pred_acc,
                               fr, p->d_rare_dev, p->d_rare, p->stream);
      }))
    return s;
  p->total_rows += n_rows;
  return DQ_OK;
}

dq_status dq_finish(dq_plan* p, dq_state* out) {
  if (!p) return set_error(DQ_E_INVALID, "dq_finish: plan is NULL");
  if (!out && !p->specs.empty()) return set_error(DQ_E_INVALID, "dq_finish: out is NULL");
  HIP_TRY(hipSetDevice(p->device));
  if (!p->parts.empty()) {
    std::vector<dq_state> tmp;
    for (size_t k = 0; k < p->parts.size(); ++k) {
      tmp.assign(p->part_specs[k].size(), dq_state{});
      if (dq_status s = dq_finish(p->parts[k], tmp.data())) return s;
      for (size_t j = 0; j < tmp.size(); ++j) out[p->part_specs[k][j]] = tmp[j];
    }
    return DQ_OK;
  }
  std::vector<ColPartial> col(p->col_tasks.size());
  std::vector<uint32_t> hll((size_t)p->n_hll * kHllCopies * 512);
  std::vector<CorrPartial> pair(p->pair_tasks.size());
  PredPartial pred{};
  std::vector<PredPartial> pred_copies(p->has_pred ? kPredAccCopies : 0);
  // the accumulators come back through one pinned staging buffer (copies to pageable memory are staged and
  // synchronous inside the runtime: 3-4 of them were ~10 us each of a 10 M-row scan's ~0.13 ms)
  const size_t b_col = col.size() * sizeof(ColPartial), b_hll = hll.size() * sizeof(uint32_t),
               b_pair = pair.size() * sizeof(CorrPartial), b_pred = pred_copies.size() * sizeof(PredPartial);
  const size_t o_hll = b_col, o_pair = o_hll + b_hll, o_pred = o_pair + b_pair, b_all = o_pred + b_pred;
  if (b_all > p->h_stage_bytes) {
    if (p->h_stage) (void)hipHostFree(p->h_stage);
    p->h_stage = nullptr;
    p->h_stage_bytes = 0;
    if (hipHostMalloc(reinterpret_cast<void**>(&p->h_stage), b_all, hipHostMallocDefault) == hipSuccess) {
      p->h_stage_bytes = b_all;
    } else {  // no pinned memory left: the copies go straight to the pageable vectors below
      (void)hipGetLastError();
      p->h_stage = nullptr;
    }
  }
  char* const hs = p->h_stage;
  void* const dst_col = hs ? (void*)hs : (void*)col.data();
  void* const dst_hll = hs ? (void*)(hs + o_hll) : (void*)hll.data();
  void* const dst_pair = hs ? (void*)(hs + o_pair) : (void*)pair.data();
  void* const dst_pred = hs ? (void*)(hs + o_pred) : (void*)pred_copies.data();
  if (b_col) HIP_TRY(hipMemcpyAsync(dst_col, p->d_col_acc, b_col, hipMemcpyDeviceToHost, p->stream));
  if (b_hll) HIP_TRY(hipMemcpyAsync(dst_hll, p->d_hll_acc, b_hll, hipMemcpyDeviceToHost, p->stream));
  if (b_pair) HIP_TRY(hipMemcpyAsync(dst_pair, p->d_pair_acc, b_pair, hipMemcpyDeviceToHost, p->stream));
  if (b_pred) HIP_TRY(hipMemcpyAsync(dst_pred, p->d_pred_acc, b_pred, hipMemcpyDeviceToHost, p->stream));
  HIP_TRY(hipStreamSynchronize(p->stream));
  if (hs) {
    if (b_col) std::memcpy(col.data(), hs, b_col);
    if (b_hll) std::memcpy(hll.data(), hs + o_hll, b_hll);
    if (b_pair) std::memcpy(pair.data(), hs + o_pair, b_pair);
    if (b_pred) std::memcpy(pred_copies.data(), hs + o_pred, b_pred);
  }
  for (const PredPartial& c : pred_copies)  // integer sums: the order of the copies does not matter
    for (int k = 0; k < kMaxCounters; ++k) {
      pred.t[k] += c.t[k];
      pred.nn[k] += c.nn[k];
    }
  // timed launches of this scan -> counters, their events back to the pool (no hipEventCreate in later scans)
  if (dq_status s = resolve_timing(p)) return s;

  const int64_t rows = p->total_rows;
  const double nan = std::numeric_limits<double>::quiet_NaN();
  const double inf = std::numeric_limits<double>::infinity();
  // Spark's sequential fp64 sum: the finite / NaN part plus the +-inf values kept out of the moments
  // (+inf and -inf together give NaN, as inf + -inf in any order)
  auto f64_sum = [&](const ColPartial& c) {
    double v = c.sum;
    if (c.pinf_count > 0) v += inf;
    if (c.ninf_count > 0) v += -inf;
    return v;
  };
  for (size_t i = 0; i < p->specs.size(); ++i) {
    const SpecOut& o = p->outs[i];
    dq_state& s = out[i];
    std::memset(&s, 0, sizeof(s));
    s.op = o.op;
    auto set1 = [&](bool v) { s.has_value[0] = s.has_value[1] = v ? 1 : 0; };
    const ColPartial* c = o.col_task >= 0 ? &col[o.col_task] : nullptr;
    switch (o.op) {
      case DQ_OP_SIZE:  // count(*) is never NULL; sum(cast(where as long)) is NULL if all where are NULL
        if (o.ctr_b >= 0) { s.u.size.num_matches = pred.t[o.ctr_b]; set1(pred.nn[o.ctr_b] > 0); }
        else { s.u.size.num_matches = rows; set1(true); }
        break;
      case DQ_OP_COMPLETENESS:
        if (o.has_where) {
          s.u.ratio.num_matches = pred.t[o.ctr_a];
          s.u.ratio.count = pred.t[o.ctr_b];
          s.has_value[0] = rows > 0;
          s.has_value[1] = pred.nn[o.ctr_b] > 0;
        } else {
          s.u.ratio.num_matches = c ? c->count : rows;
          s.u.ratio.count = rows;
          s.has_value[0] = rows > 0;  // sum over zero rows is NULL
          s.has_value[1] = 1;
        }
        break;
      case DQ_OP_COMPLIANCE:
      case DQ_OP_PATTERN_MATCH:
        s.u.ratio.num_matches = pred.t[o.ctr_a];
        s.has_value[0] = pred.nn[o.ctr_a] > 0;
        if (o.has_where) { s.u.ratio.count = pred.t[o.ctr_b]; s.has_value[1] = pred.nn[o.ctr_b] > 0; }
        else { s.u.ratio.count = rows; s.has_value[1] = 1; }
        break;
      case DQ_OP_SUM:  // Spark's Sum: LongType for integral children, DoubleType (each value cast) otherwise
        if (is_decimal(o.col_type)) {  // DecimalType: the exact decimal sum, cast at the end (state.integral 2)
          s.integral = 2;
          s.u.sum.dec_scale = DQ_DECIMAL_SCALE(o.col_type);
          s.u.sum.dec_digits = std::min(38, DQ_DECIMAL_PRECISION(o.col_type) + 10);  // Sum's result precision
          s.u.sum.partial = c->isum;
          s.u.sum.partial_hi = c->isum_hi;
          s.u.sum.guard = c->sum;
          if (!dec_sum_value(c->isum, c->isum_hi, c->sum, s.u.sum.dec_scale, s.u.sum.dec_digits, s.u.sum.sum))
            s.u.sum.sum = nan;
        } else {
          s.u.sum.sum = is_floating(o.col_type) ? f64_sum(*c) : (double)c->isum;
          s.integral = !is_floating(o.col_type);
          s.u.sum.partial = s.integral ? c->isum : 0;
        }
        set1(c->count > 0);
        break;
      case DQ_OP_MEAN:
        if (is_decimal(o.col_type)) {
          s.integral = 2;
          s.u.mean.dec_scale = DQ_DECIMAL_SCALE(o.col_type);
          s.u.mean.dec_digits = std::min(38, DQ_DECIMAL_PRECISION(o.col_type) + 10);  // Sum's result precision
          s.u.mean.partial = c->isum;
          s.u.mean.partial_hi = c->isum_hi;
          s.u.mean.guard = c->sum;
          if (!dec_sum_value(c->isum, c->isum_hi, c->sum, s.u.mean.dec_scale, s.u.mean.dec_digits, s.u.mean.sum))
            s.u.mean.sum = nan;
        } else {
          s.u.mean.sum = is_floating(o.col_type) ? f64_sum(*c) : (double)c->isum;
          s.integral = !is_floating(o.col_type);
          s.u.mean.partial = s.integral ? c->isum : 0;
        }
        s.u.mean.count = c->count;
        s.has_value[0] = c->count > 0;
        s.has_value[1] = 1;  // count(...) is never NULL
        break;
      case DQ_OP_STDDEV:
        s.u.stddev.n = c->n; s.u.stddev.avg = c->mean; s.u.stddev.m2 = c->m2;
        if (c->pinf_count + c->ninf_count > 0) {
          // an infinite value makes Spark's m2 NaN (delta * (x - avg) = inf * (inf - inf)) and its avg
          // inf or NaN depending on the row order; the metric sqrt(m2 / n) is NaN either way
          s.u.stddev.n = (double)c->count; s.u.stddev.avg = nan; s.u.stddev.m2 = nan;
        }
        set1(true);  // the struct is never NULL; n == 0 -> None (StandardDeviation.scala:46-47)
        break;
      case DQ_OP_MIN:
      case DQ_OP_MAX: {
        set1(c->count > 0);
        // fmin / fmax hold the min / max of the selected non-NaN values as doubles for every numeric
        // kind: for integral columns min(double(x)) == double(min(x)), Spark's CAST(min(col) AS DOUBLE),
        // because the int -> double cast is monotone.  nan_count is 0 for integral columns.
        {
          const bool all_nan = c->nan_count == c->count;
          if (o.op == DQ_OP_MIN) s.u.minmax.value = all_nan ? nan : c->fmin;
          else s.u.minmax.value = c->nan_count > 0 ? nan : c->fmax;  // NaN is the largest value
        }
        break;
      }
      case DQ_OP_CORRELATION: {
        const CorrPartial& q = pair[o.pair_task];
        s.u.corr.n = q.n; s.u.corr.x_avg = q.xa; s.u.corr.y_avg = q.ya;
        s.u.corr.ck = q.ck; s.u.corr.x_mk = q.xm; s.u.corr.y_mk = q.ym;
        set1(true);
        break;
      }
      case DQ_OP_DATATYPE: {  // StatefulDataType: NULL (incl. where-false), FRACTIONAL, INTEGRAL, BOOLEAN, STRING
        auto& d = s.u.dtype;
        d.num_null = rows - c->count;
        if (o.col_type == DQ_TYPE_UTF8 || o.col_type == DQ_TYPE_LARGE_UTF8) {
          d.num_fractional = c->isum;
          d.num_integral = c->nan_count;
          d.num_boolean = (int64_t)c->sum;
        } else if (is_floating(o.col_type)) {
          d.num_fractional = c->isum;
        } else if (is_decimal(o.col_type)) {  // BigDecimal.toString: plain (isum) or scientific; scale 0: integers
          if (DQ_DECIMAL_SCALE(o.col_type) == 0) d.num_integral = c->count;
          else d.num_fractional = c->isum;
        } else if (is_integral(o.col_type)) {
          d.num_integral = c->count;
        } else if (o.col_type == DQ_TYPE_BOOL) {
          d.num_boolean = c->count;
        }  // DateType / TimestampType: every value a STRING
        d.num_string = c->count - d.num_fractional - d.num_integral - d.num_boolean;
        set1(true);  // the UDAF result is never NULL
        break;
      }
      case DQ_OP_APPROX_COUNT_DISTINCT:
        {
          uint8_t regs[512];
          const uint32_t* r = hll.data() + (size_t)p->col_tasks[o.col_task].hll_slot * kHllCopies * 512;
          for (int k = 0; k < 512; ++k) {
            uint32_t v = 0;
            for (int c = 0; c < kHllCopies; ++c) v = std::max(v, r[c * 512 + k]);
            regs[k] = (uint8_t)v;
          }
          hll_registers_to_words(regs, s.u.hll.words);
        }
        set1(true);  // nullable = false (StatefulHyperloglogPlus.scala:59)
        break;
    }
  }
  return DQ_OK;
}

dq_status dq_plan_reset(dq_plan* p) {
  if (!p) return set_error(DQ_E_INVALID, "dq_plan_reset: plan is NULL");
  HIP_TRY(hipSetDevice(p->device));
  if (!p->parts.empty()) {
    for (dq_plan* q : p->parts)
      if (dq_status s = dq_plan_reset(q)) return s;
    p->total_rows = 0;
    p->next_chunk = 0;
    return DQ_OK;
  }
  return reset_acc(p);
}

void dq_plan_destroy(dq_plan* p) {
  if (!p) return;
  (void)hipSetDevice(p->device);
  for (dq_plan* q : p->parts) dq_plan_destroy(q);  // (parts launch on this plan's stream; they do not own it)
  p->parts.clear();
  if (p->stream) (void)hipStreamSynchronize(p->stream);
  free_plan_mem(p);
  if (p->own_stream && p->stream) (void)hipStreamDestroy(p->stream);
  delete p;
}

int64_t dq_plan_bytes_per_row_x1000(const dq_plan* p) { return p ? p->bytes_per_row_x1000 : 0; }

dq_status dq_plan_enable_timing(dq_plan* p, int32_t on) {
  if (!p) return set_error(DQ_E_INVALID, "dq_plan_enable_timing: plan is NULL");
  HIP_TRY(hipSetDevice(p->device));
  for (dq_plan* q : p->parts)
    if (dq_status s = dq_plan_enable_timing(q, on)) return s;
  if (dq_status s = resolve_timing(p)) return s;
  p->timing = on != 0;
  for (int k = 0; k < dq_plan::kTimers; ++k) { p->kernel_ms[k] = 0; p->kernel_launches[k] = 0; }
  return DQ_OK;
}

dq_status dq_plan_kernel_time(dq_plan* p, int32_t kernel, double* total_ms, int64_t* launches) {
  if (!p || kernel < 0 || kernel >= dq_plan::kTimers || !total_ms || !launches)
    return set_error(DQ_E_INVALID, "dq_plan_kernel_time: bad argument");
  HIP_TRY(hipSetDevice(p->device));
  if (!p->parts.empty()) {  // summed over the parts
    double ms = 0.0;
    int64_t n = 0;
    for (dq_plan* q : p->parts) {
      double m = 0.0;
      int64_t k = 0;
      if (dq_status s = dq_plan_kernel_time(q, kernel, &m, &k)) return s;
      ms += m;
      n += k;
    }
    *total_ms = ms;
    *launches = n;
    return DQ_OK;
  }
  if (dq_status s = resolve_timing(p)) return s;
  if (kernel == 1) {  // all column-scan variants
    double ms = 0;
    int64_t n = 0;
    for (int k = 16; k < dq_plan::kTimers; ++k) { ms += p->kernel_ms[k]; n += p->kernel_launches[k]; }
    *total_ms = ms;
    *launches = n;
  } else {
    *total_ms = p->kernel_ms[kernel];
    *launches = p->kernel_launches[kernel];
  }
  return DQ_OK;
}

int64_t dq_plan_variant_bytes_per_row_x1000(const dq_plan* p, int32_t variant) {
  if (!p) return 0;
  int64_t b = 0;
  for (const dq_plan* q : p->parts) b += dq_plan_variant_bytes_per_row_x1000(q, variant);
  const size_t n_run = p->col_tasks.size() - (size_t)p->n_fused;  // fused tasks run in the pair pass
  for (size_t i = 0; i < n_run; ++i) {
    const ColTask& t = p->col_tasks[i];
    if (t.variant != variant) continue;
    const dq_column_desc& cd = p->schema[t.col];
    if (t.variant != CV_VALIDITY) b += value_bytes_x1000(cd.type);
    if (cd.nullable) b += 125;
    if (t.where >= 0) b += 125;
  }
  return b;
}
int32_t dq_plan_num_launches(const dq_plan* p) { return p ? p->launches_per_scan : 0; }

dq_status dq_plan_create_time(const dq_plan* p, double* total_ms, double* pred_jit_ms) {
  if (!p) return set_error(DQ_E_INVALID, "dq_plan_create_time: plan is NULL");
  if (total_ms) *total_ms = p->create_ms;
  if (pred_jit_ms) *pred_jit_ms = p->pred_jit_ms;
  return DQ_OK;
}

int64_t dq_plan_explain(const dq_analyzer_spec* specs, int32_t n_specs, const dq_column_desc* schema, int32_t n_cols,
                        const dq_pred_node* pred_pool, int32_t n_pred, const char* const* patterns, int32_t n_patterns,
                        const dq_plan_options* opts, char* out, int64_t cap) {
  if (n_specs < 0 || (n_specs > 0 && !specs)) return set_error(DQ_E_INVALID, "dq_plan_explain: bad specs");
  if (n_cols < 0 || n_cols > kMaxSchemaCols || (n_cols > 0 && !schema))
    return set_error(DQ_E_INVALID, "dq_plan_explain: bad schema (at most %d columns)", kMaxSchemaCols);
  if (n_pred < 0 || (n_pred > 0 && !pred_pool)) return set_error(DQ_E_INVALID, "dq_plan_explain: bad predicate pool");
  if (n_patterns < 0 || (n_patterns > 0 && !patterns)) return set_error(DQ_E_INVALID, "dq_plan_explain: bad patterns");
  for (int32_t k = 0; k < n_patterns; ++k)
    if (!patterns[k]) return set_error(DQ_E_INVALID, "dq_plan_explain: pattern %d is NULL", k);
  for (int32_t c = 0; c < n_cols; ++c)
    if (!type_valid(schema[c].type))
      return set_error(DQ_E_TYPE, "dq_plan_explain: column %d has unknown type %d", c, schema[c].type);
  if (cap < 0 || (cap > 0 && !out)) return set_error(DQ_E_INVALID, "dq_plan_explain: bad output buffer");
  std::unique_ptr<dq_plan> holder(new dq_plan());
  dq_plan& plan = *holder;
  plan.host_only = true;
  plan.schema.assign(schema, schema + n_cols);
  plan.specs.assign(specs, specs + n_specs);
  for (int32_t k = 0; k < n_patterns; ++k) plan.patterns.emplace_back(patterns[k]);
  if (opts) {
    if (opts->struct_size < (int32_t)(2 * sizeof(int32_t))) return set_error(DQ_E_INVALID, "dq_plan_explain: bad options");
    if (opts->pred_pass < DQ_PRED_PASS_AUTO || opts->pred_pass > DQ_PRED_PASS_COMPILED)
      return set_error(DQ_E_INVALID, "dq_plan_explain: unknown pred_pass %d", opts->pred_pass);
    plan.pred_pass = opts->pred_pass;
  }
  std::string t;
  char line[256];
  g_capacity = false;
  dq_status st = n_cols <= kMaxCols ? build_plan(&plan, pred_pool, n_pred)
                                    : cap_error("more than %d columns in one plan", kMaxCols);
  if (st == DQ_OK) {
    std::snprintf(line, sizeof line, "plan: %d analyzers, %d columns, %d launches per scan\n", n_specs, n_cols,
                  plan.launches_per_scan);
    t += line;
    t += explain_text(plan);
  } else {
    if (!g_capacity) return st;
    // as dq_plan_create_opts: split into several fused plans
    std::string why = g_err;
    std::vector<std::vector<int32_t>> ps, pc;
    if (dq_status s2 = partition_specs(plan, pred_pool, n_pred, ps, pc)) return s2;
    std::snprintf(line, sizeof line, "plan: %d analyzers, %d columns, over one plan's capacity (%s): %zu fused plans\n",
                  n_specs, n_cols, why.c_str(), ps.size());
    t += line;
    for (size_t k = 0; k < ps.size(); ++k) {
      std::unique_ptr<dq_plan> q(new dq_plan());
      if (dq_status s2 = plan_part_host(plan, pred_pool, n_pred, ps[k], pc[k], false, *q)) return s2;
      std::snprintf(line, sizeof line, "--- part %zu: %zu analyzers, %zu columns, %d launches per scan\n", k,
                    ps[k].size(), pc[k].size(), q->launches_per_scan);
      t += line;
      t += "analyzers:";
      for (int32_t i : ps[k]) t += " " + std::to_string(i);
      t += "\ncolumns:";
      for (int32_t c : pc[k]) t += " " + std::to_string(c);
      t += "\n" + explain_text(*q);
    }
  }
  if (cap > 0) {
    const size_t n = std::min((size_t)cap - 1, t.size());
    std::memcpy(out, t.data(), n);
    out[n] = '\0';
  }
  return (int64_t)t.size() + 1;
}

int32_t dq_plan_pred_wait(dq_plan* p, int32_t timeout_ms) {
  if (!p) return set_error(DQ_E_INVALID, "dq_plan_pred_wait: plan is NULL");
  if (!p->parts.empty()) {
    int32_t all = 1, any_pred = 0;
    for (dq_plan* q : p->parts) {
      if (!q->has_pred) continue;
      any_pred = 1;
      const int32_t r = dq_plan_pred_wait(q, timeout_ms);
      if (r < 0) return r;
      all &= r;
    }
    return any_pred && all;
  }
  if (p->pred_jit_ref) {
    HIP_TRY(hipSetDevice(p->device));
    std::string note;
    if (hipFunction_t fn = pred_jit_poll(p->pred_jit_ref, timeout_ms, note)) {
      p->pred_jit = fn;
      p->pred_jit_note = note + " (compiled in the background; used from chunk " + std::to_string(p->next_chunk) + ")";
      p->pred_jit_ref.reset();
    } else if (!pred_jit_pending(p->pred_jit_ref)) {
      p->pred_jit_note = note;
      p->pred_jit_ref.reset();
    }
  }
  return p->pred_jit ? 1 : 0;
}

int32_t dq_plan_pred_compiled(const dq_plan* p, char* note, int32_t cap) {
  if (p && !p->parts.empty()) {  // composite: 1 iff every part with predicates runs compiled
    std::string n;
    int32_t all = 1, any_pred = 0;
    for (size_t k = 0; k < p->parts.size(); ++k) {
      const dq_plan* q = p->parts[k];
      if (!q->has_pred) continue;
      any_pred = 1;
      all &= dq_plan_pred_compiled(q, nullptr, 0);
      n += (n.empty() ? "" : "; ") + std::string("part ") + std::to_string(k) + ": " + q->pred_jit_note;
    }
    if (note && cap > 0) std::snprintf(note, (size_t)cap, "%s", any_pred ? n.c_str() : "no predicates");
    return any_pred && all;
  }
  if (note && cap > 0) {
    const std::string n = !p ? "plan is NULL" : (!p->has_pred ? "no predicates" : p->pred_jit_note);
    std::snprintf(note, (size_t)cap, "%s", n.c_str());
  }
  return p && p->pred_jit ? 1 : 0;
}

int64_t dq_plan_kernel_bytes_per_row_x1000(const dq_plan* p, int32_t kernel) {
  if (!p) return 0;
  if (kernel == 0) return p->pred_bytes_x1000;
  if (kernel == 2) return p->pair_bytes_x1000;
  if (kernel >= 16 && kernel < dq_plan::kTimers) return dq_plan_variant_bytes_per_row_x1000(p, kernel - 16);
  return 0;
}

}  // extern "C"
