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
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>
#include <map>
#include <string>
#include <tuple>
#include <vector>

#include "dq_device.h"
#include "dq_internal.h"
#include "dq_regex.h"

namespace dq {

hipError_t launch_pred_scan(const PredProgram* prog, const ScanCols& cols, const ScanBitmaps& bm, int64_t n_rows,
                            int64_t rows_per_range, int32_t nranges, PredPartial* acc, ColPartial* col_part,
                            uint32_t* hll_acc, int32_t lds_bytes, hipStream_t st, bool has_regex, bool has_hll);
hipError_t launch_column_scan(int32_t variant, const ColTask* tasks, int32_t ntasks, int32_t part_base,
                              const ScanCols& cols, const ScanBitmaps& bm, int64_t n_rows, int64_t rows_per_range,
                              int32_t nranges, ColPartial* partials, uint32_t* hll_acc, hipStream_t st);
hipError_t launch_pair_tile_scan(const PairGroup* groups, int32_t ngroups, const ScanCols& cols,
                                 const ScanBitmaps& bm, int64_t n_rows, int64_t rows_per_range, int32_t nranges,
                                 CorrPartial* partials, hipStream_t st);
hipError_t launch_pair_lane_scan(const PairWaveTask* tasks, int32_t ntasks, const ScanCols& cols,
                                 const ScanBitmaps& bm, const uint32_t* ones, int64_t n_rows, int64_t rows_per_range,
                                 int32_t nranges, CorrPartial* pair_part, ColPartial* col_part, bool all_f64,
                                 hipStream_t st);
hipError_t launch_pair_mfma_scan(const PairGroup* groups, int32_t ngroups, const ScanCols& cols,
                                 const ScanBitmaps& bm, const uint32_t* ones, int64_t n_rows, int64_t rows_per_range,
                                 int32_t nranges, CorrPartial* pair_part, ColPartial* col_part, bool all_f64,
                                 bool minmax, bool glds, hipStream_t st);
hipError_t launch_finalize(int32_t ncol, int32_t nranges_col, const ColPartial* col_part, ColPartial* col_acc,
                           int32_t npair, int32_t nranges_pair, const CorrPartial* pair_part, CorrPartial* pair_acc,
                           int32_t has_pred, int32_t nranges_pred, const PredPartial* pred_part, PredPartial* pred_acc, const FinRanges& fr,
                           hipStream_t st);
hipError_t launch_init_acc(ColPartial* col_acc, int32_t ncol, CorrPartial* pair_acc, int32_t npair, hipStream_t st);

static thread_local char g_err[1024] = "";

dq_status set_error(dq_status code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

#define HIP_TRY(expr)                                                                              \
  do {                                                                                             \
    hipError_t e_ = (expr);                                                                        \
    if (e_ != hipSuccess)                                                                          \
      return set_error(e_ == hipErrorOutOfMemory ? DQ_E_OOM : DQ_E_HIP, "%s failed: %s (%s:%d)", \
                       #expr, hipGetErrorString(e_), __FILE__, __LINE__);                          \
  } while (0)

static bool is_numeric(int32_t t) { return t == DQ_TYPE_F64 || t == DQ_TYPE_I64 || t == DQ_TYPE_I32; }
static bool is_integral(int32_t t) { return t == DQ_TYPE_I64 || t == DQ_TYPE_I32; }
static int32_t kind_of(int32_t t) {
  switch (t) {
    case DQ_TYPE_F64: return CK_F64;
    case DQ_TYPE_I64: return CK_I64;
    case DQ_TYPE_I32: return CK_I32;
    case DQ_TYPE_UTF8: return CK_UTF8;
    default: return CK_LUTF8;
  }
}

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

  // column CMP literal, with Spark 2.2 coercions (integral vs decimal exact, anything vs double in double)
  dq_status emit_col_lit(const Operand& o, int cmp, const Lit& lit) {
    const dq_column_desc& cd = (*schema)[o.col];
    if (!is_numeric(cd.type)) return set_error(DQ_E_UNSUPPORTED, "comparison on a non-numeric column (%d)", o.col);
    PredInstr p{};
    p.op = PO_ATOM_CMP; p.col_a = o.col; p.col_b = -1; p.kind_a = kind_of(cd.type); p.kind_b = 0;
    p.null_res = o.has_fallback ? lit_cmp_result(cmp, o.fallback, lit) : NR_NULL;
    if (lit.k == Lit::NUL) { push_const(NR_NULL); return DQ_OK; }
    if (lit.k == Lit::BOOL) return set_error(DQ_E_UNSUPPORTED, "boolean literal compared with a number");
    if (cd.type == DQ_TYPE_F64 || lit.k == Lit::DBL) {
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
        if (!is_numeric(ta) || !is_numeric(tb)) return set_error(DQ_E_UNSUPPORTED, "comparison of non-numeric columns");
        PredInstr p{};
        p.op = PO_ATOM_CMP; p.col_a = ca; p.col_b = cb; p.kind_a = kind_of(ta); p.kind_b = kind_of(tb);
        p.null_res = NR_NULL; p.cmp = to_cmpop(cmp);
        p.ctype = (is_integral(ta) && is_integral(tb)) ? CT_INT : CT_DBL;
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
  std::vector<PairTask> pair_tasks;      // sorted by pair group
  std::vector<PairGroup> pair_groups;     // <= 8 columns / <= 32 pairs / one where each (LDS-tile kernel)
  std::vector<PairWaveTask> lane_tasks;   // pair groups planned for the lane-per-row kernel (dq_pair.hip)
  int32_t n_fused = 0;                    // column tasks computed by the lane pair kernel (sorted last)
  bool lane_all_f64 = true;               // every lane task column is fp64 (the conversion-free instantiation)
  std::vector<PairGroup> mfma_groups;     // pair groups of the matrix-core Gram kernel (dq_pair.hip), moments fused
  bool mfma_all_f64 = true;
  bool mfma_minmax = false;               // a fused moments task feeds Minimum / Maximum
  int32_t concurrency = 1;                // HIP streams the variant launches are spread over
  std::vector<hipStream_t> side;          // concurrency - 1 extra streams
  std::vector<hipEvent_t> side_done;
  hipEvent_t fork_ev = nullptr;
  // DQ_PRED_CONCURRENT=1: the predicate pass on its own stream, concurrent with the column / pair
  // launches, when no `where` bitmap (the only thing those launches read from it) is produced.  Opt-in:
  // its waves (120 VGPRs, 4 per SIMD) can hold the SIMDs the hash passes need, so the gain depends on
  // dispatch order -- C3 29.17 -> 28.55 ms on one box, 35.1 ms on another
  hipStream_t pred_stream = nullptr;
  hipEvent_t pred_fork_ev = nullptr, pred_done_ev = nullptr;
  PredProgram prog{};
  std::vector<std::string> patterns;      // DQ_PRED_REGEX patterns (dq_plan_create_ex)
  std::vector<uint16_t> regex_blob;       // their compiled DFAs
  uint16_t* d_regex = nullptr;
  int32_t n_hll = 0;
  bool has_pred = false;

  // device memory
  ColTask* d_col_tasks = nullptr;
  PairTask* d_pair_tasks = nullptr;
  PairGroup* d_pair_groups = nullptr;
  PairWaveTask* d_lane_tasks = nullptr;
  PairGroup* d_mfma_groups = nullptr;
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
  uint32_t* d_ones = nullptr;  // all-ones bitmap (lane pair pass: columns without validity, tasks without where)
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
  if (p->pred_stream) (void)hipStreamDestroy(p->pred_stream);
  if (p->pred_fork_ev) (void)hipEventDestroy(p->pred_fork_ev);
  if (p->pred_done_ev) (void)hipEventDestroy(p->pred_done_ev);
  p->pred_stream = nullptr;
  p->pred_fork_ev = p->pred_done_ev = nullptr;
  for (hipStream_t st : p->side) (void)hipStreamDestroy(st);
  for (hipEvent_t ev : p->side_done) (void)hipEventDestroy(ev);
  if (p->fork_ev) (void)hipEventDestroy(p->fork_ev);
  p->side.clear();
  p->side_done.clear();
  for (auto& q : p->pending) { p->ev_pool.push_back(q.a); p->ev_pool.push_back(q.b); }
  p->pending.clear();
  for (hipEvent_t e : p->ev_pool) (void)hipEventDestroy(e);
  p->ev_pool.clear();
  void* ptrs[] = {p->d_col_tasks, p->d_pair_tasks, p->d_pair_groups, p->d_lane_tasks, p->d_mfma_groups, p->d_prog, p->d_col_part, p->d_pair_part,
                  p->d_pred_part, p->d_col_acc, p->d_hll_acc, p->d_pair_acc, p->d_pred_acc, p->d_regex};
  for (void* q : ptrs)
    if (q) (void)hipFree(q);
  for (int i = 0; i < kMaxWhere; ++i)
    if (p->d_where_bits[i]) (void)hipFree(p->d_where_bits[i]);
  if (p->d_ones) (void)hipFree(p->d_ones);
  return DQ_OK;
}

static dq_status reset_acc(dq_plan* p) {
  HIP_TRY(launch_init_acc(p->d_col_acc, (int32_t)p->col_tasks.size(), p->d_pair_acc, (int32_t)p->pair_tasks.size(),
                          p->stream));
  if (p->n_hll) HIP_TRY(hipMemsetAsync(p->d_hll_acc, 0, (size_t)p->n_hll * kHllCopies * 512 * sizeof(uint32_t), p->stream));
  if (p->has_pred) HIP_TRY(hipMemsetAsync(p->d_pred_acc, 0, sizeof(PredPartial), p->stream));
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

// Plan one pair group for the lane-per-row kernel (dq_pair.hip): cover its pairs with the fewest column
// subsets of kLaneCols local columns (one wave task each; every pair of 8 columns fits 4 subsets of 5), put
// each fusable moments column -- a stats-only column task of the group's columns and `where` -- at position
// 0 / 1 of a task holding it (extra moments-only tasks if the covers have no room), and hand every pair to
// the least-loaded task covering it.  Returns false when the group cannot be planned this way.
static bool plan_lane_tasks(const dq_plan* p, const PairGroup& g, std::vector<PairWaveTask>& out,
                            std::vector<int>& fused) {
  const int k = g.ncols;
  if (k < 2 || k > kTileCols || g.npairs < 1) return false;
  std::vector<int32_t> mom_task(k, -1);
  for (int c = 0; c < k; ++c)
    for (size_t t = 0; t < p->col_tasks.size(); ++t) {
      const ColTask& ct = p->col_tasks[t];
      if (ct.col == g.cols[c] && ct.where == g.where && !fused[t] &&
          (ct.variant == CV_F64_S || ct.variant == CV_I64_S || ct.variant == CV_I32_S))
        mom_task[c] = (int32_t)t;
    }
  auto pbit = [](int a, int b) { return a < b ? 1ull << (a * 8 + b) : 1ull << (b * 8 + a); };
  uint64_t need = 0;
  for (int q = 0; q < g.npairs; ++q) need |= pbit(g.pi[q], g.pj[q]);
  const int sz = std::min(k, kLaneCols);
  std::vector<uint32_t> subs;
  std::vector<uint64_t> cov;
  for (uint32_t m = 1; m < (1u << k); ++m) {
    if (__builtin_popcount(m) != sz) continue;
    uint64_t c = 0;
    for (int a = 0; a < k; ++a)
      for (int b = a + 1; b < k; ++b)
        if (((m >> a) & 1u) && ((m >> b) & 1u)) c |= pbit(a, b);
    if ((c & need) == 0) continue;
    subs.push_back(m);
    cov.push_back(c & need);
  }
  // moments matching: column -> one task holding it, at most kLaneMoments per task (augmenting paths)
  auto match = [&](const std::vector<uint32_t>& tasks, std::vector<int>& col_of_slot) {
    col_of_slot.assign(tasks.size() * kLaneMoments, -1);
    int matched = 0;
    for (int c = 0; c < k; ++c) {
      if (mom_task[c] < 0) continue;
      std::vector<char> seen(col_of_slot.size(), 0);
      std::function<bool(int)> aug = [&](int col) {
        for (size_t t = 0; t < tasks.size(); ++t) {
          if (!((tasks[t] >> col) & 1u)) continue;
          for (int sl = 0; sl < kLaneMoments; ++sl) {
            const size_t i = t * kLaneMoments + sl;
            if (seen[i]) continue;
            seen[i] = 1;
            if (col_of_slot[i] < 0 || aug(col_of_slot[i])) { col_of_slot[i] = col; return true; }
          }
        }
        return false;
      };
      if (aug(c)) ++matched;
    }
    return matched;
  };
  const int n_mom = (int)std::count_if(mom_task.begin(), mom_task.end(), [](int32_t t) { return t >= 0; });
  std::vector<uint32_t> best;
  std::vector<int> best_slots;
  int best_matched = -1;
  const int ns = (int)subs.size();
  for (int T = 1; T <= 4 && best.empty(); ++T) {
    std::vector<int> idx(T);
    for (int i = 0; i < T; ++i) idx[i] = i;
    while (T <= ns) {
      uint64_t c = 0;
      for (int i : idx) c |= cov[i];
      if ((c & need) == need) {
        std::vector<uint32_t> tasks;
        for (int i : idx) tasks.push_back(subs[i]);
        std::vector<int> slots;
        const int mt = match(tasks, slots);
        if (mt > best_matched) { best = tasks; best_slots = slots; best_matched = mt; }
        if (mt == n_mom) break;
      }
      int i = T - 1;  // next combination
      while (i >= 0 && idx[i] == ns - T + i) --i;
      if (i < 0) break;
      ++idx[i];
      for (int j = i + 1; j < T; ++j) idx[j] = idx[j - 1] + 1;
    }
  }
  if (best.empty()) return false;
  // position lists: matched moments columns first, then the rest of the subset
  std::vector<std::vector<int>> pos(best.size());
  std::vector<int> task_moms(best.size(), 0);
  for (size_t t = 0; t < best.size(); ++t) {
    for (int sl = 0; sl < kLaneMoments; ++sl)
      if (best_slots[t * kLaneMoments + sl] >= 0) { pos[t].push_back(best_slots[t * kLaneMoments + sl]); task_moms[t]++; }
    for (int c = 0; c < k; ++c)
      if (((best[t] >> c) & 1u) && std::find(pos[t].begin(), pos[t].end(), c) == pos[t].end()) pos[t].push_back(c);
  }
  std::vector<char> mom_done(k, 0);
  for (int v : best_slots)
    if (v >= 0) mom_done[v] = 1;
  for (int c = 0; c < k;) {  // unmatched moments columns: moments-only tasks
    if (mom_task[c] < 0 || mom_done[c]) { ++c; continue; }
    std::vector<int> ps{c};
    mom_done[c] = 1;
    for (int d = c + 1; d < k && (int)ps.size() < kLaneMoments; ++d)
      if (mom_task[d] >= 0 && !mom_done[d]) { ps.push_back(d); mom_done[d] = 1; }
    best.push_back(0);
    pos.push_back(ps);
    task_moms.push_back((int)ps.size());
  }
  std::vector<PairWaveTask> tasks(pos.size());
  std::vector<int> load(pos.size(), 0);
  for (size_t t = 0; t < pos.size(); ++t) {
    PairWaveTask& w = tasks[t];
    std::memset(&w, 0, sizeof(w));
    w.ncols = (int32_t)pos[t].size();
    w.where = g.where;
    for (int i = 0; i < kLaneCols; ++i) {  // unused positions repeat position 0 (loaded, never used)
      const int l = pos[t][i < w.ncols ? i : 0];
      w.cols[i] = g.cols[l];
      w.kinds[i] = g.kinds[l];
    }
    for (int i = 0; i < kLaneSlots; ++i) w.pair_out[i] = -1;
    for (int i = 0; i < kLaneMoments; ++i) w.mom_out[i] = -1;
    for (int i = 0; i < task_moms[t]; ++i) {
      w.mom_mask |= 1u << i;
      w.mom_out[i] = mom_task[pos[t][i]];
    }
    load[t] = 4 * task_moms[t] + w.ncols;
  }
  auto slot_of = [](int a, int b) {
    for (int i = 0; i < kLaneSlots; ++i)
      if (kLaneSlotA[i] == std::min(a, b) && kLaneSlotB[i] == std::max(a, b)) return i;
    return -1;
  };
  for (int q = 0; q < g.npairs; ++q) {
    int bt = -1, ba = -1, bb = -1;
    for (size_t t = 0; t < pos.size(); ++t) {
      auto ia = std::find(pos[t].begin(), pos[t].end(), (int)g.pi[q]);
      auto ib = std::find(pos[t].begin(), pos[t].end(), (int)g.pj[q]);
      if (ia == pos[t].end() || ib == pos[t].end()) continue;
      const int sl = slot_of((int)(ia - pos[t].begin()), (int)(ib - pos[t].begin()));
      if ((tasks[t].pair_mask >> sl) & 1u) continue;  // e.g. Correlation(a, b) and Correlation(b, a)
      if (bt < 0 || load[t] < load[bt]) { bt = (int)t; ba = (int)(ia - pos[t].begin()); bb = (int)(ib - pos[t].begin()); }
    }
    if (bt < 0) {  // no covering task with the slot free: a two-column task of its own
      PairWaveTask w;
      std::memset(&w, 0, sizeof(w));
      w.ncols = 2;
      w.where = g.where;
      for (int i = 0; i < kLaneCols; ++i) {
        const int l = i == 1 ? g.pj[q] : g.pi[q];
        w.cols[i] = g.cols[l];
        w.kinds[i] = g.kinds[l];
      }
      for (int i = 0; i < kLaneSlots; ++i) w.pair_out[i] = -1;
      for (int i = 0; i < kLaneMoments; ++i) w.mom_out[i] = -1;
      tasks.push_back(w);
      pos.push_back({(int)g.pi[q], (int)g.pj[q]});
      load.push_back(2);
      bt = (int)tasks.size() - 1;
      ba = 0;
      bb = 1;
    }
    const int slot = slot_of(ba, bb);
    if (slot < 0) return false;
    // the slot computes (position a, position b); a pair whose first column sits at b swaps x / y on output
    if (ba > bb) tasks[bt].swap_mask |= 1u << slot;
    tasks[bt].pair_mask |= 1u << slot;
    tasks[bt].pair_out[slot] = g.first_pair + q;
    load[bt] += 5;
  }
  for (size_t t = 0; t < pos.size(); ++t)
    for (int i = 0; i < kLaneMoments; ++i)
      if ((tasks[t].mom_mask >> i) & 1u) fused[tasks[t].mom_out[i]] = 1;
  out = tasks;
  return true;
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
    if ((int32_t)root_slot.size() >= kMaxRoots) return set_error(DQ_E_UNSUPPORTED, "more than %d distinct predicates", kMaxRoots);
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
    if ((int32_t)root_slot.size() >= kMaxRoots) return set_error(DQ_E_UNSUPPORTED, "more than %d distinct predicates", kMaxRoots);
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
    if ((int32_t)counter_of.size() >= kMaxCounters) return set_error(DQ_E_UNSUPPORTED, "more than %d predicate counters", kMaxCounters);
    c = (int32_t)counter_of.size();
    counter_of[key] = c;
    return DQ_OK;
  };
  auto bitmap = [&](int32_t where_slot, int32_t& b) -> dq_status {
    if (where_slot < 0) { b = -1; return DQ_OK; }
    auto it = bitmap_of.find(where_slot);
    if (it != bitmap_of.end()) { b = it->second; return DQ_OK; }
    if ((int32_t)bitmap_of.size() >= kMaxWhere) return set_error(DQ_E_UNSUPPORTED, "more than %d distinct where filters on value analyzers", kMaxWhere);
    b = (int32_t)bitmap_of.size();
    bitmap_of[where_slot] = b;
    return DQ_OK;
  };
  auto col_task = [&](int32_t col, int32_t bm, bool stats, bool hll, int32_t& t, bool dtype = false) -> dq_status {
    // a double column's DataType count is a variant of its own (CV_F64_D)
    auto key = std::make_tuple(col, bm, dtype && p->schema[col].type == DQ_TYPE_F64 ? 1 : 0);
    auto it = col_task_of.find(key);
    if (it == col_task_of.end()) {
      if ((int32_t)p->col_tasks.size() >= 256) return set_error(DQ_E_UNSUPPORTED, "too many column tasks");
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
        // integral columns: Long/Int.toString always matches INTEGRAL -> the selected-row count suffices
        if (dq_status st = col_task(s.col_a, bm, false, false, o.col_task, !is_integral(o.col_type))) return st;
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
          pt.kind_x = kind_of(p->schema[s.col_a].type); pt.kind_y = kind_of(p->schema[s.col_b].type);
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
    if (dtype && type == DQ_TYPE_F64) ct.variant = CV_F64_D;
    else if (!stats && !hll && !dtype) ct.variant = CV_VALIDITY;
    else if (type == DQ_TYPE_UTF8) ct.variant = hll && dtype ? CV_UTF8_HD : (dtype ? CV_UTF8_D : CV_UTF8_H);
    else if (type == DQ_TYPE_LARGE_UTF8) ct.variant = hll && dtype ? CV_LUTF8_HD : (dtype ? CV_LUTF8_D : CV_LUTF8_H);
    else {
      int base = type == DQ_TYPE_F64 ? CV_F64_S : (type == DQ_TYPE_I64 ? CV_I64_S : CV_I32_S);
      ct.variant = base + (stats && hll ? 1 : (stats ? 0 : 2));
    }
  }

  // correlation pairs -> groups sharing one LDS row tile (greedy, per where bitmap)
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
    p->pair_groups.swap(groups);
    for (SpecOut& o : p->outs)
      if (o.pair_task >= 0) o.pair_task = new_index[o.pair_task];
  }

  // pair groups -> the matrix-core Gram kernel (default) or lane-per-row wave tasks (dq_pair.hip), with the
  // groups' stats-only column tasks fused in; DQ_PAIR_KERNEL=lane|tile selects the older kernels (A/B tests)
  std::vector<int> fused(p->col_tasks.size(), 0);
  {
    const char* kern = std::getenv("DQ_PAIR_KERNEL");
    const bool tile_only = std::getenv("DQ_PAIR_TILE") != nullptr || (kern && std::strcmp(kern, "tile") == 0);
    const bool lane = kern && std::strcmp(kern, "lane") == 0;
    std::vector<PairGroup> tile_groups;
    for (PairGroup g : p->pair_groups) {
      std::vector<PairWaveTask> w;
      if (!tile_only && !lane && g.ncols >= 1) {
        for (int c = 0; c < kTileCols; ++c) g.mom_task[c] = -1;
        for (int c = 0; c < g.ncols; ++c)
          for (size_t t = 0; t < p->col_tasks.size(); ++t) {
            const ColTask& ct = p->col_tasks[t];
            if (ct.col == g.cols[c] && ct.where == g.where && !fused[t] &&
                (ct.variant == CV_F64_S || ct.variant == CV_I64_S || ct.variant == CV_I32_S)) {
              g.mom_task[c] = (int32_t)t;
              fused[t] = 1;
              break;
            }
          }
        for (int c = 0; c < g.ncols; ++c) p->mfma_all_f64 = p->mfma_all_f64 && g.kinds[c] == CK_F64;
        p->mfma_groups.push_back(g);
      } else if (!tile_only && plan_lane_tasks(p, g, w, fused)) {
        while (w.size() % kWaves) w.push_back(PairWaveTask{});  // idle padding: 4 tasks of one range per workgroup
        p->lane_tasks.insert(p->lane_tasks.end(), w.begin(), w.end());
      } else {
        tile_groups.push_back(g);
      }
    }
    p->pair_groups.swap(tile_groups);
    for (const PairWaveTask& w : p->lane_tasks)
      for (int c = 0; c < w.ncols; ++c) p->lane_all_f64 = p->lane_all_f64 && w.kinds[c] == CK_F64;
    // idle padding tasks still need valid column indices for nothing: they return before any load
  }

  // HLL-only column tasks (no `where`) of columns whose values an ATOM_CMP of the predicate program already
  // loads can be hashed inside the predicate pass (one read of the column for both).  Opt-in
  // (DQ_PRED_HLL=1): measured on C3 the fused pass takes 2.04 ms per 125 M rows against 0.99 + 0.66 ms for
  // the predicate pass plus the separate i64 HLL launch -- the interpreter's occupancy (3 waves/SIMD with
  // the hash registers) costs more than the second read of the columns saves.
  std::vector<int32_t> pred_hll_tasks;  // original task indices, in fusion order
  {
    const char* ph = std::getenv("DQ_PRED_HLL");
    const bool pred_used = !root_code.empty() && (!counter_of.empty() || !bitmap_of.empty());
    if (pred_used && ph && std::strcmp(ph, "1") == 0) {
      std::vector<char> loaded(ncols, 0);
      for (const auto& rc : root_code)
        for (const PredInstr& ins : rc)
          if (ins.op == PO_ATOM_CMP) {
            if (ins.col_a >= 0) loaded[ins.col_a] = 1;
            if (ins.col_b >= 0) loaded[ins.col_b] = 1;
          }
      for (size_t t = 0; t < p->col_tasks.size() && (int)pred_hll_tasks.size() < kMaxPredHll; ++t) {
        const ColTask& ct = p->col_tasks[t];
        if (fused[t] || ct.where >= 0 || !loaded[ct.col]) continue;
        if (ct.variant != CV_F64_H && ct.variant != CV_I64_H && ct.variant != CV_I32_H) continue;
        fused[t] = 2;
        pred_hll_tasks.push_back((int32_t)t);
      }
    }
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
    for (PairWaveTask& w : p->lane_tasks)
      for (int k = 0; k < kLaneMoments; ++k)
        if ((w.mom_mask >> k) & 1u) w.mom_out[k] = new_index[w.mom_out[k]];
    for (int32_t& t : pred_hll_tasks) t = new_index[t];
    for (PairGroup& g : p->mfma_groups)
      for (int c = 0; c < g.ncols; ++c)
        if (g.mom_task[c] >= 0) {
          g.mom_task[c] = new_index[g.mom_task[c]];
          for (const SpecOut& o : p->outs)
            if (o.col_task == g.mom_task[c] && (o.op == DQ_OP_MIN || o.op == DQ_OP_MAX)) p->mfma_minmax = true;
        }
    for (int32_t k = 0; k < (int32_t)p->col_tasks.size(); ++k) {
      if (fused[order[k]]) break;  // fused tasks sort last: their partials come from the pair pass
      if (p->groups.empty() || p->groups.back().variant != p->col_tasks[k].variant)
        p->groups.push_back({p->col_tasks[k].variant, k, 0});
      p->groups.back().count++;
    }
    p->n_fused = (int32_t)std::count_if(fused.begin(), fused.end(), [](int f) { return f != 0; });
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
    if ((int32_t)code.size() > kMaxInstr) return set_error(DQ_E_UNSUPPORTED, "predicate program too long (%zu)", code.size());
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
    for (int32_t t : pred_hll_tasks) {  // the first ATOM_CMP loading the column hashes it
      const ColTask& ct = p->col_tasks[(size_t)t];
      for (int32_t i = 0; i < prog.n_instr; ++i) {
        const PredInstr& ins = prog.instr[i];
        if (ins.op != PO_ATOM_CMP || (ins.col_a != ct.col && ins.col_b != ct.col)) continue;
        PredHll& e = prog.hll[prog.n_hll++];
        e.instr = i;
        e.operand = ins.col_a == ct.col ? 0 : 1;
        e.kind = ins.col_a == ct.col ? ins.kind_a : ins.kind_b;
        e.part = t;
        e.hll_slot = ct.hll_slot;
        e.pad = 0;
        break;
      }
    }
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
    if (need_values[c]) b1000 += (t == DQ_TYPE_I32 || t == DQ_TYPE_UTF8) ? 4000 : 8000;  // value or offset bytes
    if (need_validity[c] && p->schema[c].nullable) b1000 += 125;
  }
  p->bytes_per_row_x1000 = b1000;
  // per-kernel algorithmic bytes: the predicate pass (its atoms' columns) and the pair pass (its columns)
  {
    auto bytes_of = [&](const std::vector<int>& vals, const std::vector<int>& valid) {
      int64_t b = 0;
      for (int c = 0; c < ncols; ++c) {
        int32_t t = p->schema[c].type;
        if (vals[c]) b += (t == DQ_TYPE_I32 || t == DQ_TYPE_UTF8) ? 4000 : 8000;
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
  p->launches_per_scan = (p->has_pred ? 1 : 0) + (int32_t)p->groups.size() + (p->pair_groups.empty() ? 0 : 1) +
                         (p->lane_tasks.empty() ? 0 : 1) + (p->mfma_groups.empty() ? 0 : 1) +
                         ((p->col_tasks.size() + p->pair_tasks.size()) ? 1 : 0);

  // device allocations
  const size_t nct = p->col_tasks.size(), npt = p->pair_tasks.size();
  if (dq_status s = dmalloc(&p->d_col_tasks, nct * sizeof(ColTask))) return s;
  if (dq_status s = dmalloc(&p->d_pair_tasks, npt * sizeof(PairTask))) return s;
  if (dq_status s = dmalloc(&p->d_pair_groups, p->pair_groups.size() * sizeof(PairGroup))) return s;
  if (dq_status s = dmalloc(&p->d_lane_tasks, p->lane_tasks.size() * sizeof(PairWaveTask))) return s;
  if (dq_status s = dmalloc(&p->d_mfma_groups, p->mfma_groups.size() * sizeof(PairGroup))) return s;
  if (!p->mfma_groups.empty())
    HIP_TRY(hipMemcpyAsync(p->d_mfma_groups, p->mfma_groups.data(), p->mfma_groups.size() * sizeof(PairGroup),
                           hipMemcpyHostToDevice, p->stream));
  if (!p->lane_tasks.empty())
    HIP_TRY(hipMemcpyAsync(p->d_lane_tasks, p->lane_tasks.data(), p->lane_tasks.size() * sizeof(PairWaveTask),
                           hipMemcpyHostToDevice, p->stream));
  if (dq_status s = dmalloc(&p->d_prog, sizeof(PredProgram))) return s;
  if (dq_status s = dmalloc(&p->d_col_part, nct * kMaxWG * sizeof(ColPartial))) return s;
  if (dq_status s = dmalloc(&p->d_pair_part, npt * kMaxWG * sizeof(CorrPartial))) return s;
  if (dq_status s = dmalloc(&p->d_pred_part, sizeof(PredPartial))) return s;  // unused (kept for the finalize ABI)
  if (dq_status s = dmalloc(&p->d_col_acc, nct * sizeof(ColPartial))) return s;
  if (dq_status s = dmalloc(&p->d_hll_acc, (size_t)p->n_hll * kHllCopies * 512 * sizeof(uint32_t))) return s;
  if (dq_status s = dmalloc(&p->d_pair_acc, npt * sizeof(CorrPartial))) return s;
  if (dq_status s = dmalloc(&p->d_pred_acc, sizeof(PredPartial))) return s;
  if (nct) HIP_TRY(hipMemcpyAsync(p->d_col_tasks, p->col_tasks.data(), nct * sizeof(ColTask), hipMemcpyHostToDevice, p->stream));
  if (npt) HIP_TRY(hipMemcpyAsync(p->d_pair_tasks, p->pair_tasks.data(), npt * sizeof(PairTask), hipMemcpyHostToDevice, p->stream));
  if (!p->pair_groups.empty())
    HIP_TRY(hipMemcpyAsync(p->d_pair_groups, p->pair_groups.data(), p->pair_groups.size() * sizeof(PairGroup),
                           hipMemcpyHostToDevice, p->stream));
  if (p->regex_blob.size() > (size_t)kMaxRegexWords)
    return set_error(DQ_E_UNSUPPORTED, "compiled patterns need %zu KB (LDS budget %d KB)",
                     p->regex_blob.size() * 2 / 1024, kMaxRegexWords * 2 / 1024);
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
  // concurrency: DQ_COLUMN_STREAMS (default 1) streams for the variant launches
  if (const char* e = std::getenv("DQ_COLUMN_STREAMS")) p->concurrency = std::max(1, std::min(8, std::atoi(e)));
  p->concurrency = std::min<int32_t>(
      p->concurrency, std::max<int32_t>(1, (int32_t)p->groups.size() + (p->pair_groups.empty() ? 0 : 1) +
                                               (p->lane_tasks.empty() ? 0 : 1) + (p->mfma_groups.empty() ? 0 : 1)));
  HIP_TRY(hipEventCreateWithFlags(&p->fork_ev, hipEventDisableTiming));
  const char* pc = std::getenv("DQ_PRED_CONCURRENT");  // opt-in: see the plan field's note
  if (p->has_pred && p->prog.n_bitmaps == 0 && pc && pc[0] == '1') {
    HIP_TRY(hipStreamCreateWithFlags(&p->pred_stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&p->pred_fork_ev, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&p->pred_done_ev, hipEventDisableTiming));
  }
  for (int32_t k = 1; k < p->concurrency; ++k) {
    hipStream_t st;
    hipEvent_t ev;
    HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    p->side.push_back(st);
    p->side_done.push_back(ev);
  }
  return DQ_OK;
}

static int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

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
  if (!out) return set_error(DQ_E_INVALID, "dq_plan_create: out is NULL");
  if (n_patterns < 0 || (n_patterns > 0 && !patterns)) return set_error(DQ_E_INVALID, "dq_plan_create: bad patterns");
  for (int32_t k = 0; k < n_patterns; ++k)
    if (!patterns[k]) return set_error(DQ_E_INVALID, "dq_plan_create: pattern %d is NULL", k);
  *out = nullptr;
  if (n_specs < 0 || (n_specs > 0 && !specs)) return set_error(DQ_E_INVALID, "dq_plan_create: bad specs");
  if (n_cols < 0 || n_cols > kMaxCols || (n_cols > 0 && !schema))
    return set_error(DQ_E_INVALID, "dq_plan_create: bad schema (at most %d columns)", kMaxCols);
  if (n_pred < 0 || (n_pred > 0 && !pred_pool)) return set_error(DQ_E_INVALID, "dq_plan_create: bad predicate pool");
  for (int32_t c = 0; c < n_cols; ++c)
    if (schema[c].type < DQ_TYPE_F64 || schema[c].type > DQ_TYPE_LARGE_UTF8)
      return set_error(DQ_E_TYPE, "dq_plan_create: column %d has unknown type %d", c, schema[c].type);
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return set_error(DQ_E_INVALID, "dq_plan_create: device %d of %d", device, ndev);
  HIP_TRY(hipSetDevice(device));
  dq_plan* p = new dq_plan();
  p->device = device;
  p->schema.assign(schema, schema + n_cols);
  p->specs.assign(specs, specs + n_specs);
  for (int32_t k = 0; k < n_patterns; ++k) p->patterns.emplace_back(patterns[k]);
  hipError_t e = hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete p;
    return set_error(DQ_E_HIP, "hipStreamCreate: %s", hipGetErrorString(e));
  }
  p->own_stream = true;
  dq_status st = build_plan(p, pred_pool, n_pred);
  if (st != DQ_OK) {
    std::string msg = g_err;
    dq_plan_destroy(p);
    return set_error(st, "%s", msg.c_str());
  }
  *out = p;
  return DQ_OK;
}

dq_status dq_plan_set_stream(dq_plan* p, void* hip_stream) {
  if (!p) return set_error(DQ_E_INVALID, "dq_plan_set_stream: plan is NULL");
  HIP_TRY(hipSetDevice(p->device));
  HIP_TRY(hipStreamSynchronize(p->stream));
  // NULL is the device's null stream (what torch's default stream reports), not "keep the plan's
  // own stream": the plan's own stream is non-blocking and would not wait for producers on it.
  if (p->own_stream) (void)hipStreamDestroy(p->stream);
  p->stream = (hipStream_t)hip_stream;
  p->own_stream = false;
  return DQ_OK;
}

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
  ScanCols sc{};
  for (int32_t c = 0; c < ncols; ++c) {
    const dq_column_view& v = cols[c];
    int32_t t = p->schema[c].type;
    if (v.reserved != 0) return set_error(DQ_E_INVALID, "dq_scan: column %d reserved field must be 0", c);
    if (n_rows > 0 && !v.values) return set_error(DQ_E_INVALID, "dq_scan: column %d has no values buffer", c);
    if (((uintptr_t)v.values & 15) != 0)
      return set_error(DQ_E_INVALID, "dq_scan: column %d values buffer must be 16-byte aligned", c);
    if (((uintptr_t)v.validity & 3) != 0)
      return set_error(DQ_E_INVALID, "dq_scan: column %d validity bitmap must be 4-byte aligned", c);
    if ((t == DQ_TYPE_UTF8 || t == DQ_TYPE_LARGE_UTF8) && n_rows > 0 && !v.offsets)
      return set_error(DQ_E_INVALID, "dq_scan: UTF8 column %d has no offsets", c);
    sc.values[c] = v.values;
    sc.validity[c] = p->schema[c].nullable ? reinterpret_cast<const uint32_t*>(v.validity) : nullptr;
    sc.offsets[c] = v.offsets;
  }
  p->next_chunk++;
  if (n_rows == 0) return DQ_OK;

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
  // all-ones bitmap standing in for a missing validity / where bitmap in the lane pair pass
  if ((!p->lane_tasks.empty() || !p->mfma_groups.empty()) && words + 1 > p->ones_cap_words) {
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
  for (const auto& g : p->groups) min_launch = min_launch ? std::min<int64_t>(min_launch, g.count) : g.count;
  if (!p->pair_groups.empty())
    min_launch = min_launch ? std::min<int64_t>(min_launch, (int64_t)p->pair_groups.size()) : (int64_t)p->pair_groups.size();
  if (!p->lane_tasks.empty()) {  // workgroups of the lane pair launch per row range
    const int64_t wg = (int64_t)p->lane_tasks.size() / kWaves;
    min_launch = min_launch ? std::min<int64_t>(min_launch, wg) : wg;
  }
  if (!p->mfma_groups.empty()) {
    const int64_t wg = (int64_t)p->mfma_groups.size();
    min_launch = min_launch ? std::min<int64_t>(min_launch, wg) : wg;
  }
  static const int64_t target = [] {
    const char* e = std::getenv("DQ_TARGET_WGS");  // tuning override (diagnostic)
    return e ? std::max<int64_t>(256, std::atoll(e)) : (int64_t)kTargetWGs;
  }();
  const int64_t want = std::max<int64_t>(64, std::min<int64_t>(kMaxWG, target / std::max<int64_t>(1, min_launch)));
  // rows per range and range count for `want` ranges
  auto size_ranges = [&](int64_t w, int64_t& rpr, int32_t& nr) {
    nr = (int32_t)std::min<int64_t>(w, ceil_div(n_rows, kRowsPerIter));
    rpr = ceil_div(ceil_div(n_rows, nr), kRowsPerIter) * kRowsPerIter;
    nr = (int32_t)ceil_div(n_rows, rpr);
  };
  int32_t nr_col;
  int64_t rpr_col;
  size_ranges(want, rpr_col, nr_col);
  // per-variant workgroup counts: the string hash balances better with twice the ranges (uneven string
  // lengths, deferred-round drains): utf8_hll 1.979 -> 1.949 ms per 125 M x 4 on the C5 headline (A/B
  // twice, DQ_VARIANT_RANGES=0 for the common size); halving the fp64 hash's ranges measured no change.
  // scale > 0: want x scale ranges, < 0: want / -scale
  static const int32_t str_scale = [] {
    // tuning override (diagnostic); utf8_hll per 125 M x 4 on one box: x1 1.979, x2 1.951 / 1.956,
    // x3 1.963 / 1.964, x4 1.965 ms
    const char* e = std::getenv("DQ_STR_RANGE_SCALE");
    return e ? std::max(1, std::min(8, std::atoi(e))) : 2;
  }();
  auto variant_scale = [](int32_t v) -> int32_t {
    if (v == CV_UTF8_H || v == CV_LUTF8_H || v == CV_UTF8_HD || v == CV_LUTF8_HD) return str_scale;
    return 1;
  };
  static const bool per_variant = !(std::getenv("DQ_VARIANT_RANGES") && std::getenv("DQ_VARIANT_RANGES")[0] == '0');
  FinRanges fr{};
  std::vector<std::pair<int64_t, int32_t>> vr(p->groups.size());  // (rows per range, ranges) per variant group
  for (size_t gi = 0; gi < p->groups.size(); ++gi) {
    const auto& g = p->groups[gi];
    const int32_t sc_v = per_variant ? variant_scale(g.variant) : 1;
    if (sc_v == 1) {
      vr[gi] = {rpr_col, nr_col};
      continue;
    }
    const int64_t w = sc_v > 0 ? want * sc_v : want / -sc_v;
    size_ranges(std::max<int64_t>(64, std::min<int64_t>(kMaxWG, w)), vr[gi].first, vr[gi].second);
    if (fr.n < kNumVariants) {
      fr.first[fr.n] = g.first;
      fr.end[fr.n] = g.first + g.count;
      fr.nr[fr.n] = vr[gi].second;
      ++fr.n;
    }
  }
  // predicate pass: ~2048 workgroups of whole 2048-row iterations (HBM-bound; counters leave by atomics)
  static const int64_t pred_wgs = [] {
    // tuning override (diagnostic): 1024-16384 workgroups measured within 2 % of 2048 on C3 (0.954-0.978 ms)
    const char* e = std::getenv("DQ_PRED_WGS");
    return e ? std::max<int64_t>(64, std::min<int64_t>(65536, std::atoll(e))) : (int64_t)2048;
  }();
  int32_t nr_pred = (int32_t)std::min<int64_t>(pred_wgs, ceil_div(n_rows, kRowsPerIter));
  int64_t rpr_pred = ceil_div(ceil_div(n_rows, nr_pred), kRowsPerIter) * kRowsPerIter;
  nr_pred = (int32_t)ceil_div(n_rows, rpr_pred);

  // fused HLL tasks (counted by the predicate pass into range slot 0): empty partials for every range
  for (int32_t h = 0; h < p->prog.n_hll; ++h)
    HIP_TRY(hipMemsetAsync(p->d_col_part + (size_t)p->prog.hll[h].part * kMaxWG, 0, (size_t)nr_col * sizeof(ColPartial),
                           p->stream));
  if (p->has_pred) {
    hipStream_t pst = p->stream;
    if (p->pred_stream) {  // fork: the predicate pass beside the column / pair launches
      HIP_TRY(hipEventRecord(p->pred_fork_ev, p->stream));
      HIP_TRY(hipStreamWaitEvent(p->pred_stream, p->pred_fork_ev, 0));
      pst = p->pred_stream;
    }
    if (dq_status s = timed(p, 0, pst, [&] {
          const int32_t lds = kWaves * 128 * (p->prog.stack_depth + p->prog.n_roots + p->prog.n_counters) +
                              ((p->prog.regex_words * 2 + 15) & ~15);
          return launch_pred_scan(p->d_prog, sc, bm, n_rows, rpr_pred, nr_pred, p->d_pred_acc, p->d_col_part,
                                  p->d_hll_acc, lds, pst, p->prog.regex_words > 0, p->prog.n_hll > 0);
        }))
      return s;
    if (p->pred_stream) HIP_TRY(hipEventRecord(p->pred_done_ev, p->pred_stream));
  }
  // fork: variant launches (and the pair pass) round-robin over the plan stream + side streams
  const int32_t K = p->concurrency;
  if (K > 1) {
    HIP_TRY(hipEventRecord(p->fork_ev, p->stream));
    for (hipStream_t st : p->side) HIP_TRY(hipStreamWaitEvent(st, p->fork_ev, 0));
  }
  int32_t li = 0;
  auto stream_for = [&](int32_t i) { return (K > 1 && i % K) ? p->side[i % K - 1] : p->stream; };
  for (size_t gi = 0; gi < p->groups.size(); ++gi) {
    const auto& g = p->groups[gi];
    hipStream_t st = stream_for(li++);
    if (dq_status s = timed(p, 16 + g.variant, st, [&] {
          return launch_column_scan(g.variant, p->d_col_tasks + g.first, g.count, g.first, sc, bm, n_rows,
                                    vr[gi].first, vr[gi].second, p->d_col_part, p->d_hll_acc, st);
        }))
      return s;
  }
  if (!p->lane_tasks.empty()) {
    hipStream_t st = stream_for(li++);
    if (dq_status s = timed(p, 2, st, [&] {
          return launch_pair_lane_scan(p->d_lane_tasks, (int32_t)p->lane_tasks.size(), sc, bm, p->d_ones, n_rows, rpr_col,
                                       nr_col, p->d_pair_part, p->d_col_part, p->lane_all_f64, st);
        }))
      return s;
  }
  if (!p->mfma_groups.empty()) {
    hipStream_t st = stream_for(li++);
    // LDS-DMA staging of all-fp64 groups (dq_scan already requires 16-byte aligned value buffers; checked
    // again here since the kernel's DMA assumes it); DQ_PAIR_GLDS=0 selects the register-staged kernel
    const char* glds_env = std::getenv("DQ_PAIR_GLDS");
    bool glds = !(glds_env && glds_env[0] == '0') && p->mfma_all_f64;
    for (const PairGroup& g : p->mfma_groups)
      for (int c = 0; c < g.ncols && glds; ++c) glds = ((uintptr_t)sc.values[g.cols[c]] & 15u) == 0;
    if (dq_status s = timed(p, 2, st, [&] {
          return launch_pair_mfma_scan(p->d_mfma_groups, (int32_t)p->mfma_groups.size(), sc, bm, p->d_ones, n_rows,
                                       rpr_col, nr_col, p->d_pair_part, p->d_col_part, p->mfma_all_f64,
                                       p->mfma_minmax, glds, st);
        }))
      return s;
  }
  if (!p->pair_groups.empty()) {
    hipStream_t st = stream_for(li++);
    if (dq_status s = timed(p, 2, st, [&] {
          return launch_pair_tile_scan(p->d_pair_groups, (int32_t)p->pair_groups.size(), sc, bm, n_rows, rpr_col,
                                       nr_col, p->d_pair_part, st);
        }))
      return s;
  }
  if (K > 1) {  // join
    for (int32_t k = 1; k < K; ++k) {
      HIP_TRY(hipEventRecord(p->side_done[k - 1], p->side[k - 1]));
      HIP_TRY(hipStreamWaitEvent(p->stream, p->side_done[k - 1], 0));
    }
  }
  if (p->has_pred && p->pred_stream) HIP_TRY(hipStreamWaitEvent(p->stream, p->pred_done_ev, 0));
  if (dq_status s = timed(p, 3, p->stream, [&] {
        return launch_finalize((int32_t)p->col_tasks.size(), nr_col, p->d_col_part, p->d_col_acc,
                               (int32_t)p->pair_tasks.size(), nr_col, p->d_pair_part, p->d_pair_acc,
                               0 /* the predicate pass accumulates itself */, nr_pred, p->d_pred_part, p->d_pred_acc,
                               fr, p->stream);
      }))
    return s;
  p->total_rows += n_rows;
  return DQ_OK;
}

dq_status dq_finish(dq_plan* p, dq_state* out) {
  if (!p) return set_error(DQ_E_INVALID, "dq_finish: plan is NULL");
  if (!out && !p->specs.empty()) return set_error(DQ_E_INVALID, "dq_finish: out is NULL");
  HIP_TRY(hipSetDevice(p->device));
  std::vector<ColPartial> col(p->col_tasks.size());
  std::vector<uint32_t> hll((size_t)p->n_hll * kHllCopies * 512);
  std::vector<CorrPartial> pair(p->pair_tasks.size());
  PredPartial pred{};
  if (!col.empty()) HIP_TRY(hipMemcpyAsync(col.data(), p->d_col_acc, col.size() * sizeof(ColPartial), hipMemcpyDeviceToHost, p->stream));
  if (!hll.empty())
    HIP_TRY(hipMemcpyAsync(hll.data(), p->d_hll_acc, hll.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, p->stream));
  if (!pair.empty()) HIP_TRY(hipMemcpyAsync(pair.data(), p->d_pair_acc, pair.size() * sizeof(CorrPartial), hipMemcpyDeviceToHost, p->stream));
  if (p->has_pred) HIP_TRY(hipMemcpyAsync(&pred, p->d_pred_acc, sizeof(PredPartial), hipMemcpyDeviceToHost, p->stream));
  HIP_TRY(hipStreamSynchronize(p->stream));
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
      case DQ_OP_SUM:
        s.u.sum.sum = o.col_type == DQ_TYPE_F64 ? f64_sum(*c) : (double)c->isum;
        s.integral = o.col_type != DQ_TYPE_F64;
        s.u.sum.partial = s.integral ? c->isum : 0;
        set1(c->count > 0);
        break;
      case DQ_OP_MEAN:
        s.u.mean.sum = o.col_type == DQ_TYPE_F64 ? f64_sum(*c) : (double)c->isum;
        s.integral = o.col_type != DQ_TYPE_F64;
        s.u.mean.partial = s.integral ? c->isum : 0;
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
        } else if (o.col_type == DQ_TYPE_F64) {
          d.num_fractional = c->isum;
        } else {
          d.num_integral = c->count;
        }
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
  return reset_acc(p);
}

void dq_plan_destroy(dq_plan* p) {
  if (!p) return;
  (void)hipSetDevice(p->device);
  if (p->stream) (void)hipStreamSynchronize(p->stream);
  free_plan_mem(p);
  if (p->own_stream && p->stream) (void)hipStreamDestroy(p->stream);
  delete p;
}

int64_t dq_plan_bytes_per_row_x1000(const dq_plan* p) { return p ? p->bytes_per_row_x1000 : 0; }

dq_status dq_plan_enable_timing(dq_plan* p, int32_t on) {
  if (!p) return set_error(DQ_E_INVALID, "dq_plan_enable_timing: plan is NULL");
  HIP_TRY(hipSetDevice(p->device));
  if (dq_status s = resolve_timing(p)) return s;
  p->timing = on != 0;
  for (int k = 0; k < dq_plan::kTimers; ++k) { p->kernel_ms[k] = 0; p->kernel_launches[k] = 0; }
  return DQ_OK;
}

dq_status dq_plan_kernel_time(dq_plan* p, int32_t kernel, double* total_ms, int64_t* launches) {
  if (!p || kernel < 0 || kernel >= dq_plan::kTimers || !total_ms || !launches)
    return set_error(DQ_E_INVALID, "dq_plan_kernel_time: bad argument");
  HIP_TRY(hipSetDevice(p->device));
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
  const size_t n_run = p->col_tasks.size() - (size_t)p->n_fused;  // fused tasks run in the pair pass
  for (size_t i = 0; i < n_run; ++i) {
    const ColTask& t = p->col_tasks[i];
    if (t.variant != variant) continue;
    const dq_column_desc& cd = p->schema[t.col];
    if (t.variant != CV_VALIDITY) b += (cd.type == DQ_TYPE_I32 || cd.type == DQ_TYPE_UTF8) ? 4000 : 8000;
    if (cd.nullable) b += 125;
    if (t.where >= 0) b += 125;
  }
  return b;
}
int32_t dq_plan_num_launches(const dq_plan* p) { return p ? p->launches_per_scan : 0; }

int64_t dq_plan_kernel_bytes_per_row_x1000(const dq_plan* p, int32_t kernel) {
  if (!p) return 0;
  if (kernel == 0) return p->pred_bytes_x1000;
  if (kernel == 2) return p->pair_bytes_x1000;
  if (kernel >= 16 && kernel < dq_plan::kTimers) return dq_plan_variant_bytes_per_row_x1000(p, kernel - 16);
  return 0;
}

}  // extern "C"
