// dq_pred_compile.cpp -- Spark SQL predicate text -> the dq_pred_node IR (include/dqscan.h), on the host.
//
// Stands in for Spark's expr(...) parser at the C boundary: the predicate strings deequ builds
// (analyzers/Analyzer.scala:385-408 `where` filters; checks/Check.scala:538-548, 670-871 satisfies /
// isNonNegative / isContainedIn / isLessThan ...) are parsed here, so a JVM / JNI shim hands over the
// text and gets exactly the lowering the tests pin.  Grammar (the numeric subset the GPU evaluates with
// SQL three-valued logic, plus string equality / IN lists on string columns):
//
//     expr     := or
//     or       := and ( OR and )*
//     and      := not ( AND not )*
//     not      := NOT not | cmp
//     cmp      := operand ( (< | <= | > | >= | = | == | != | <>) operand | IS [NOT] NULL
//                           | [NOT] IN ('s', ...) )?
//     operand  := column | `column` | number | - number | NULL | TRUE | FALSE | 'string'
//               | COALESCE(operand, operand) | ( expr )
//
// Literal typing follows Spark 2.2: `3` integer, `3.0` exact decimal (unscaled int64 + scale), `3e0`
// double.  String (in)equality and IN lists compare the UTF-8 bytes of a string column with the literals:
// they lower to a whole-value DFA (DQ_PRED_REGEX, mode DQ_REGEX_FULL) over the escaped literals.  Anything
// else -- string ordering, numeric comparison of a string column, LIKE / RLIKE / BETWEEN, function calls,
// typed literal suffixes, backslash escapes in literals -- is DQ_E_UNSUPPORTED: the analyzer is routed to
// the fallback set, as a column type the plan does not cover.
#include <cerrno>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/dqscan.h"
#include "dq_internal.h"

struct dq_pred_pool {
  std::vector<std::string> names;
  std::vector<int32_t> types;
  std::unordered_map<std::string, int32_t> index;
  std::vector<dq_pred_node> nodes;
  std::vector<std::string> patterns;
  std::vector<const char*> pattern_ptrs;
};

namespace {

struct PredError {
  dq_status status;
  std::string msg;
};

[[noreturn]] void unsupported(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  throw PredError{DQ_E_UNSUPPORTED, buf};
}

enum TokKind { T_ID, T_STR, T_NUM, T_KW, T_OP, T_END };
struct Tok {
  TokKind kind;
  std::string text;
  bool operator==(const Tok& o) const { return kind == o.kind && text == o.text; }
};

const char* const kKeywords[] = {"AND", "OR", "NOT", "IS", "NULL", "COALESCE", "TRUE", "FALSE", "IN", "LIKE", "RLIKE",
                                 "BETWEEN"};

bool is_digit(char c) { return c >= '0' && c <= '9'; }
bool is_alpha(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (unsigned char)c >= 0x80; }
bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v'; }

std::string upper(const std::string& s) {
  std::string u = s;
  for (char& c : u)
    if (c >= 'a' && c <= 'z') c = (char)(c - 'a' + 'A');
  return u;
}

std::vector<Tok> tokenize(const std::string& s) {
  std::vector<Tok> toks;
  size_t i = 0;
  const char* q = s.c_str();
  while (i < s.size()) {
    const char c = s[i];
    if (is_space(c)) {
      ++i;
    } else if (c == '`') {
      const size_t j = s.find('`', i + 1);
      if (j == std::string::npos) unsupported("unterminated identifier in '%s'", q);
      toks.push_back({T_ID, s.substr(i + 1, j - i - 1)});
      i = j + 1;
    } else if (c == '\'' || c == '"') {
      const size_t j = s.find(c, i + 1);
      if (j == std::string::npos) unsupported("unterminated string literal in '%s'", q);
      const std::string body = s.substr(i + 1, j - i - 1);
      if (body.find('\\') != std::string::npos)  // Spark unescapes backslash sequences: not restated here
        unsupported("string literal with a backslash escape in '%s'", q);
      toks.push_back({T_STR, body});
      i = j + 1;
    } else if (is_digit(c) || (c == '.' && i + 1 < s.size() && is_digit(s[i + 1]))) {
      size_t j = i;
      while (j < s.size() && (is_digit(s[j]) || s[j] == '.')) ++j;
      if (j < s.size() && (s[j] == 'e' || s[j] == 'E')) {
        ++j;
        if (j < s.size() && (s[j] == '+' || s[j] == '-')) ++j;
        while (j < s.size() && is_digit(s[j])) ++j;
      }
      if (j < s.size() && std::strchr("dDlLsSyY", s[j]) && s[j] != '\0')  // typed literal suffixes (1.0D, 10L)
        unsupported("typed literal suffix in '%s'", q);
      toks.push_back({T_NUM, s.substr(i, j - i)});
      i = j;
    } else if (is_alpha(c) || c == '_') {
      size_t j = i;
      while (j < s.size() && (is_alpha(s[j]) || is_digit(s[j]) || s[j] == '_')) ++j;
      const std::string w = s.substr(i, j - i), u = upper(w);
      bool kw = false;
      for (const char* k : kKeywords) kw = kw || u == k;
      toks.push_back(kw ? Tok{T_KW, u} : Tok{T_ID, w});
      i = j;
    } else if (s.compare(i, 2, "<=") == 0 || s.compare(i, 2, ">=") == 0 || s.compare(i, 2, "!=") == 0 ||
               s.compare(i, 2, "<>") == 0 || s.compare(i, 2, "==") == 0) {
      toks.push_back({T_OP, s.substr(i, 2)});
      i += 2;
    } else if (std::strchr("<>=(),-", c) && c != '\0') {
      toks.push_back({T_OP, std::string(1, c)});
      ++i;
    } else {
      unsupported("unexpected character '%c' in '%s'", c, q);
    }
  }
  return toks;
}

int32_t cmp_of(const std::string& op) {
  if (op == "<") return DQ_CMP_LT;
  if (op == "<=") return DQ_CMP_LE;
  if (op == ">") return DQ_CMP_GT;
  if (op == ">=") return DQ_CMP_GE;
  if (op == "=" || op == "==") return DQ_CMP_EQ;
  if (op == "!=" || op == "<>") return DQ_CMP_NE;
  return 0;
}

// An operand: a node index, or (string literals) the literal text, valid only beside a string column.
struct Operand {
  int32_t node = -1;
  bool is_str = false;
  std::string str;
};

class Parser {
 public:
  Parser(dq_pred_pool& pool, const std::string& text) : P(pool), text(text), toks(tokenize(text)) {}

  int32_t parse() {
    const Operand r = parse_or();
    if (pos != toks.size()) unsupported("unsupported syntax near '%s' in '%s'", toks[pos].text.c_str(), text.c_str());
    if (r.is_str) unsupported("bare string literal in '%s'", text.c_str());
    return r.node;
  }

 private:
  dq_pred_pool& P;
  const std::string& text;
  std::vector<Tok> toks;
  size_t pos = 0;

  Tok peek() const { return pos < toks.size() ? toks[pos] : Tok{T_END, ""}; }
  Tok take() {
    Tok t = peek();
    ++pos;
    return t;
  }
  void expect(TokKind k, const char* v) {
    const Tok t = take();
    if (!(t.kind == k && t.text == v)) unsupported("expected '%s', got '%s' in '%s'", v, t.text.c_str(), text.c_str());
  }
  bool at(TokKind k, const char* v) const {
    const Tok t = peek();
    return t.kind == k && t.text == v;
  }
  int32_t add(int32_t kind, int32_t a = -1, int32_t b = -1, int32_t cmp = 0, int64_t i64 = 0, double f64 = 0.0) {
    P.nodes.push_back(dq_pred_node{kind, a, b, cmp, i64, f64});
    return (int32_t)P.nodes.size() - 1;
  }
  Operand node(int32_t n) {
    Operand o;
    o.node = n;
    return o;
  }
  int32_t need_node(const Operand& o) {
    if (o.is_str) unsupported("bare string literal in '%s'", text.c_str());
    return o.node;
  }

  Operand parse_or() {
    Operand a = parse_and();
    while (at(T_KW, "OR")) {
      take();
      const int32_t l = need_node(a);
      const int32_t r = need_node(parse_and());
      a = node(add(DQ_PRED_OR, l, r));
    }
    return a;
  }
  Operand parse_and() {
    Operand a = parse_not();
    while (at(T_KW, "AND")) {
      take();
      const int32_t l = need_node(a);
      const int32_t r = need_node(parse_not());
      a = node(add(DQ_PRED_AND, l, r));
    }
    return a;
  }
  Operand parse_not() {
    if (at(T_KW, "NOT")) {
      take();
      return node(add(DQ_PRED_NOT, need_node(parse_not())));
    }
    return parse_cmp();
  }

  // plan column of a COLUMN node or of COALESCE(column, ...); -1 otherwise
  int32_t column_of(int32_t n) const {
    const dq_pred_node& x = P.nodes[(size_t)n];
    if (x.kind == DQ_PRED_COLUMN) return x.a;
    if (x.kind == DQ_PRED_COALESCE && P.nodes[(size_t)x.a].kind == DQ_PRED_COLUMN) return P.nodes[(size_t)x.a].a;
    return -1;
  }
  bool is_string_col(int32_t col) const {
    return col >= 0 && (P.types[(size_t)col] == DQ_TYPE_UTF8 || P.types[(size_t)col] == DQ_TYPE_LARGE_UTF8);
  }

  Operand parse_cmp() {
    Operand a = parse_operand();
    const Tok t = peek();
    if (t.kind == T_OP && cmp_of(t.text)) {
      take();
      Operand b = parse_operand();
      if (a.is_str || b.is_str) {  // string (in)equality
        if (t.text != "=" && t.text != "==" && t.text != "!=" && t.text != "<>")
          unsupported("string ordering comparison in '%s'", text.c_str());
        const Operand& col = a.is_str ? b : a;
        const Operand& lit = a.is_str ? a : b;
        if (col.is_str) unsupported("comparison of two string literals in '%s'", text.c_str());
        const int32_t e = string_in(col.node, {lit.str});
        return node(t.text == "!=" || t.text == "<>" ? add(DQ_PRED_NOT, e) : e);
      }
      // numeric comparison: a string column operand is outside the grammar (Spark would cast it)
      for (int32_t side : {a.node, b.node}) {
        const int32_t c = column_of(side);
        if (is_string_col(c))
          unsupported("predicate compares string column '%s' in '%s'", P.names[(size_t)c].c_str(), text.c_str());
      }
      return node(add(DQ_PRED_CMP, a.node, b.node, cmp_of(t.text)));
    }
    if (!a.is_str && (at(T_KW, "IN") || at(T_KW, "NOT"))) {
      const size_t save = pos;
      const bool neg = at(T_KW, "NOT");
      take();
      if (neg && !at(T_KW, "IN")) {
        pos = save;
        return a;
      }
      if (neg) take();
      expect(T_OP, "(");
      std::vector<Tok> items{take()};
      while (at(T_OP, ",")) {
        take();
        items.push_back(take());
      }
      expect(T_OP, ")");
      std::vector<std::string> lits;
      for (const Tok& it : items) {
        if (it.kind != T_STR) unsupported("IN list of non-string literals in '%s'", text.c_str());
        lits.push_back(it.text);
      }
      const int32_t e = string_in(a.node, lits);
      return node(neg ? add(DQ_PRED_NOT, e) : e);
    }
    if (at(T_KW, "IS")) {
      take();
      bool neg = false;
      if (at(T_KW, "NOT")) {
        take();
        neg = true;
      }
      expect(T_KW, "NULL");
      return node(add(neg ? DQ_PRED_IS_NOT_NULL : DQ_PRED_IS_NULL, need_node(a)));
    }
    if (t.kind == T_KW && (t.text == "LIKE" || t.text == "RLIKE" || t.text == "BETWEEN"))
      unsupported("%s is not in the GPU predicate grammar: '%s'", t.text.c_str(), text.c_str());
    if (a.is_str) unsupported("bare string literal in '%s'", text.c_str());
    return a;
  }

  // col IN (literals) as one whole-value DFA (?:l1|l2|...) with every non-alphanumeric ASCII character
  // escaped (the DFA compiler reads `\` + such a character as the literal character)
  int32_t string_in(int32_t col_node, const std::vector<std::string>& lits) {
    const dq_pred_node cn = P.nodes[(size_t)col_node];
    if (cn.kind != DQ_PRED_COLUMN) unsupported("string comparison on a non-column expression in '%s'", text.c_str());
    if (!is_string_col(cn.a)) unsupported("string literal compared with a non-string column in '%s'", text.c_str());
    std::string pat = "(?:";
    for (size_t i = 0; i < lits.size(); ++i) {
      if (i) pat += '|';
      for (char ch : lits[i]) {
        const unsigned char u = (unsigned char)ch;
        if (!((u < 128 && (is_digit(ch) || (ch >= 'a' && ch <= 'z') || (ch >= 'A' && ch <= 'Z'))) || u >= 128))
          pat += '\\';
        pat += ch;
      }
    }
    pat += ')';
    if (col_node == (int32_t)P.nodes.size() - 1) P.nodes.pop_back();  // re-added by add_regex
    int32_t root = -1;
    const dq_status s = dq_pred_pool_add_regex(&P, cn.a, pat.c_str(), DQ_REGEX_FULL, &root);
    if (s != DQ_OK) throw PredError{s, dq_last_error()};
    return root;
  }

  Operand parse_operand() {
    const Tok t = take();
    if (t.kind == T_OP && t.text == "(") {
      Operand e = parse_or();
      expect(T_OP, ")");
      return e;
    }
    if (t.kind == T_OP && t.text == "-") {
      const Tok t2 = take();
      if (t2.kind != T_NUM) unsupported("unary minus on a non-literal in '%s'", text.c_str());
      return node(number("-" + t2.text));
    }
    if (t.kind == T_NUM) return node(number(t.text));
    if (t.kind == T_STR) {
      Operand o;
      o.is_str = true;
      o.str = t.text;
      return o;
    }
    if (t.kind == T_KW && t.text == "NULL") return node(add(DQ_PRED_LIT_NULL));
    if (t.kind == T_KW && (t.text == "TRUE" || t.text == "FALSE"))
      return node(add(DQ_PRED_LIT_BOOL, -1, -1, 0, t.text == "TRUE" ? 1 : 0));
    if (t.kind == T_KW && t.text == "COALESCE") {
      expect(T_OP, "(");
      const int32_t a = need_node(parse_operand());
      expect(T_OP, ",");
      const int32_t b = need_node(parse_operand());
      if (at(T_OP, ",")) unsupported("COALESCE with more than two arguments in '%s'", text.c_str());
      expect(T_OP, ")");
      return node(add(DQ_PRED_COALESCE, a, b));
    }
    if (t.kind == T_ID) {
      if (at(T_OP, "(")) unsupported("function call %s(...) in '%s'", t.text.c_str(), text.c_str());
      const auto it = P.index.find(t.text);
      if (it == P.index.end()) throw PredError{DQ_E_INVALID, "no such column: " + t.text};
      return node(add(DQ_PRED_COLUMN, it->second));
    }
    unsupported("unexpected token '%s' in '%s'", t.text.c_str(), text.c_str());
  }

  // Spark 2.2 literal typing: exponent -> double, '.' -> exact decimal (int64 unscaled, scale <= 18),
  // else a 64-bit integer
  int32_t number(const std::string& s) {
    const bool neg = !s.empty() && s[0] == '-';
    const std::string body = neg ? s.substr(1) : s;
    if (body.find_first_of("eE") != std::string::npos) {
      const size_t e = body.find_first_of("eE");
      const std::string mant = body.substr(0, e), ex = body.substr(e + 1);
      const size_t dot = mant.find('.');
      const bool mant_ok = !mant.empty() && mant.find('.', dot == std::string::npos ? 0 : dot + 1) == std::string::npos &&
                           mant != ".";
      const size_t ed = ex.find_first_not_of("+-") == std::string::npos ? ex.size() : ex.find_first_not_of("+-");
      if (!mant_ok || ed > 1 || ed >= ex.size()) unsupported("malformed number %s in '%s'", s.c_str(), text.c_str());
      errno = 0;
      char* end = nullptr;
      const double v = std::strtod(s.c_str(), &end);
      if (end != s.c_str() + s.size()) unsupported("malformed number %s in '%s'", s.c_str(), text.c_str());
      return add(DQ_PRED_LIT_DOUBLE, -1, -1, 0, 0, v);  // an overflow is +-inf, as float() / Double.parseDouble
    }
    const size_t dot = body.find('.');
    if (dot != std::string::npos) {
      const std::string ip = body.substr(0, dot), fp = body.substr(dot + 1);
      if (fp.find('.') != std::string::npos) unsupported("malformed number %s in '%s'", s.c_str(), text.c_str());
      uint64_t u = 0;
      for (char ch : ip + fp) {
        if (u > (UINT64_C(1) << 63) / 10) unsupported("decimal literal %s exceeds 64-bit precision", s.c_str());
        u = u * 10 + (uint64_t)(ch - '0');
      }
      if (u >= (UINT64_C(1) << 63) || fp.size() > 18)
        unsupported("decimal literal %s exceeds 64-bit precision", s.c_str());
      return add(DQ_PRED_LIT_DECIMAL, -1, -1, (int32_t)fp.size(), neg ? -(int64_t)u : (int64_t)u);
    }
    uint64_t u = 0;
    for (char ch : body) {
      if (u > UINT64_MAX / 10 || u * 10 > UINT64_MAX - (uint64_t)(ch - '0'))
        unsupported("integer literal %s out of range", s.c_str());
      u = u * 10 + (uint64_t)(ch - '0');
    }
    if (neg ? u > (UINT64_C(1) << 63) : u >= (UINT64_C(1) << 63)) unsupported("integer literal %s out of range", s.c_str());
    return add(DQ_PRED_LIT_INT, -1, -1, 0, neg ? (int64_t)(0 - u) : (int64_t)u);
  }
};

}  // namespace

extern "C" {

dq_status dq_pred_pool_create(const char* const* names, const int32_t* types, int32_t n_cols, dq_pred_pool** out) {
  if (!out || n_cols < 0 || (n_cols > 0 && (!names || !types)))
    return dq::set_error(DQ_E_INVALID, "dq_pred_pool_create: bad argument");
  dq_pred_pool* p = new dq_pred_pool();
  for (int32_t c = 0; c < n_cols; ++c) {
    if (!names[c]) {
      delete p;
      return dq::set_error(DQ_E_INVALID, "dq_pred_pool_create: NULL column name");
    }
    p->names.push_back(names[c]);
    p->types.push_back(types[c]);
    p->index.emplace(names[c], c);  // the first of duplicate names wins, as a resolver would fail later
  }
  *out = p;
  return DQ_OK;
}

dq_status dq_pred_pool_add(dq_pred_pool* pool, const char* sql, int32_t* root) {
  if (!pool || !sql || !root) return dq::set_error(DQ_E_INVALID, "dq_pred_pool_add: bad argument");
  const size_t n0 = pool->nodes.size(), np0 = pool->patterns.size();
  try {
    const std::string text(sql);
    Parser ps(*pool, text);
    *root = ps.parse();
    return DQ_OK;
  } catch (const PredError& e) {
    pool->nodes.resize(n0);  // the pool is unchanged by a failed add
    pool->patterns.resize(np0);
    pool->pattern_ptrs.resize(np0);
    return dq::set_error(e.status, "%s", e.msg.c_str());
  }
}

dq_status dq_pred_pool_add_regex(dq_pred_pool* pool, int32_t column, const char* pattern, int32_t mode, int32_t* root) {
  if (!pool || !pattern || !root || column < 0 || column >= (int32_t)pool->names.size())
    return dq::set_error(DQ_E_INVALID, "dq_pred_pool_add_regex: bad argument");
  if (dq_status s = dq_regex_info(pattern, mode, nullptr, nullptr)) return s;  // outside the DFA subset
  int32_t idx = -1;
  for (size_t i = 0; i < pool->patterns.size(); ++i)
    if (pool->patterns[i] == pattern) idx = (int32_t)i;
  if (idx < 0) {
    pool->patterns.push_back(pattern);
    pool->pattern_ptrs.clear();
    for (const std::string& q : pool->patterns) pool->pattern_ptrs.push_back(q.c_str());
    idx = (int32_t)pool->patterns.size() - 1;
  }
  pool->nodes.push_back(dq_pred_node{DQ_PRED_COLUMN, column, -1, 0, 0, 0.0});
  const int32_t col = (int32_t)pool->nodes.size() - 1;
  pool->nodes.push_back(dq_pred_node{DQ_PRED_REGEX, col, -1, mode, idx, 0.0});
  *root = (int32_t)pool->nodes.size() - 1;
  return DQ_OK;
}

int32_t dq_pred_pool_size(const dq_pred_pool* pool) { return pool ? (int32_t)pool->nodes.size() : 0; }
const dq_pred_node* dq_pred_pool_nodes(const dq_pred_pool* pool) {
  return pool && !pool->nodes.empty() ? pool->nodes.data() : nullptr;
}
int32_t dq_pred_pool_num_patterns(const dq_pred_pool* pool) { return pool ? (int32_t)pool->patterns.size() : 0; }
const char* const* dq_pred_pool_patterns(const dq_pred_pool* pool) {
  return pool && !pool->pattern_ptrs.empty() ? pool->pattern_ptrs.data() : nullptr;
}
void dq_pred_pool_destroy(dq_pred_pool* pool) { delete pool; }

}  // extern "C"
