// dq_regex.cpp -- host compiler of PatternMatch / RLIKE patterns into byte-level search DFAs.
//
// Reference: PatternMatch.aggregationFunctions (analyzers/PatternMatch.scala:46-55) counts the rows
// where Spark's `regexp_extract(col, pattern, 0) != ""`, i.e. java.util.regex Matcher.find() found
// a match and group 0 is non-empty; RLIKE is Matcher.find() alone.  For a pattern that cannot match
// the empty string both reduce to "some substring of the value (decoded as UTF-8 code points)
// is in the pattern's language", a regular property, so the pattern is compiled into a DFA over the
// UTF-8 bytes of the value that the GPU walks once per row (dq_kernels.hip, PO_ATOM_REGEX).
//
// Supported java.util.regex subset: literals (incl. non-ASCII), `.`, classes `[...]` / `[^...]`
// with ranges and \d \D \s \S \w \W \xhh \x{h..} \uhhhh \0ooo \t \n \r \f \a \e and escaped
// metacharacters, groups `(...)`, `(?:...)`, `(?<name>...)`, alternation, greedy and lazy
// quantifiers (* + ? {n} {n,} {n,m}; laziness does not change whether a match exists), a leading
// `^` and a trailing `$` on a pattern without top-level alternation.  Everything else
// (backreferences, look-around, \b, possessive / atomic groups, inline flags, class intersection,
// \p{..}) is DQ_E_UNSUPPORTED: the analyzer stays on the fallback path.
//
// Character semantics follow java.util.regex defaults: \d = [0-9], \s = [ \t\n\x0B\f\r],
// \w = [a-zA-Z_0-9]; `.` = any code point but \n \r \u0085 \u2028 \u2029; `$` (no MULTILINE) = end
// of input or before a final line terminator (\r\n \n \r \u0085 \u2028 \u2029).
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "dq_internal.h"
#include "dq_regex.h"

namespace dq {
namespace {

using Ranges = std::vector<std::pair<uint32_t, uint32_t>>;  // code point ranges, inclusive
constexpr uint32_t kMaxCp = 0x10FFFF;

Ranges normalize(Ranges r) {
  std::sort(r.begin(), r.end());
  Ranges o;
  for (auto& x : r) {
    if (!o.empty() && x.first <= o.back().second + 1) o.back().second = std::max(o.back().second, x.second);
    else o.push_back(x);
  }
  return o;
}
Ranges complement(const Ranges& in) {
  Ranges r = normalize(in), o;
  uint32_t next = 0;
  for (auto& x : r) {
    if (x.first > next) o.push_back({next, x.first - 1});
    next = x.second + 1;
  }
  if (next <= kMaxCp) o.push_back({next, kMaxCp});
  return o;
}
const Ranges kDigit = {{'0', '9'}};
const Ranges kSpace = {{'\t', '\r'}, {' ', ' '}};  // \t \n \x0B \f \r and space
const Ranges kWord = {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}};
Ranges dot_ranges() { return complement({{'\n', '\n'}, {'\r', '\r'}, {0x85, 0x85}, {0x2028, 0x2029}}); }

struct Node {
  enum Kind { EMPTY, SET, CAT, ALT, REP } k = EMPTY;
  Ranges set;
  std::vector<int> kids;
  int lo = 0, hi = 0;  // REP bounds, hi = -1: unbounded
};

struct Parser {
  std::vector<uint32_t> cp;  // pattern code points
  size_t i = 0;
  std::vector<Node> nodes;
  std::string err;
  bool anchored_start = false, anchored_end = false;

  int add(Node n) { nodes.push_back(std::move(n)); return (int)nodes.size() - 1; }
  bool fail(const char* what) {
    if (err.empty()) err = what;
    return false;
  }
  bool at_end() const { return i >= cp.size(); }
  uint32_t peek(size_t k = 0) const { return i + k < cp.size() ? cp[i + k] : 0xFFFFFFFFu; }

  static int hexval(uint32_t c) {
    if (c >= '0' && c <= '9') return (int)(c - '0');
    if (c >= 'a' && c <= 'f') return (int)(c - 'a' + 10);
    if (c >= 'A' && c <= 'F') return (int)(c - 'A' + 10);
    return -1;
  }

  // escape after '\\' (i at the escaped char): a set (class escapes) or one code point
  bool escape(Ranges& out, bool in_class) {
    if (at_end()) return fail("trailing backslash");
    uint32_t c = cp[i++];
    switch (c) {
      case 'd': out = kDigit; return true;
      case 'D': out = complement(kDigit); return true;
      case 's': out = kSpace; return true;
      case 'S': out = complement(kSpace); return true;
      case 'w': out = kWord; return true;
      case 'W': out = complement(kWord); return true;
      case 't': out = {{'\t', '\t'}}; return true;
      case 'n': out = {{'\n', '\n'}}; return true;
      case 'r': out = {{'\r', '\r'}}; return true;
      case 'f': out = {{'\f', '\f'}}; return true;
      case 'a': out = {{7, 7}}; return true;
      case 'e': out = {{27, 27}}; return true;
      case 'x': {
        uint32_t v = 0;
        if (peek() == '{') {
          ++i;
          int nd = 0;
          while (!at_end() && peek() != '}') {
            int h = hexval(cp[i++]);
            if (h < 0 || ++nd > 6) return fail("bad \\x{...} escape");
            v = v * 16 + (uint32_t)h;
          }
          if (at_end() || nd == 0) return fail("bad \\x{...} escape");
          ++i;
        } else {
          for (int k = 0; k < 2; ++k) {
            int h = at_end() ? -1 : hexval(cp[i++]);
            if (h < 0) return fail("bad \\x escape");
            v = v * 16 + (uint32_t)h;
          }
        }
        if (v > kMaxCp) return fail("\\x escape out of range");
        out = {{v, v}};
        return true;
      }
      case 'u': {
        uint32_t v = 0;
        for (int k = 0; k < 4; ++k) {
          int h = at_end() ? -1 : hexval(cp[i++]);
          if (h < 0) return fail("bad \\u escape");
          v = v * 16 + (uint32_t)h;
        }
        if (v >= 0xD800 && v <= 0xDFFF) return fail("surrogate \\u escape");
        out = {{v, v}};
        return true;
      }
      case '0': {  // \0n, \0nn, \0mnn (m <= 3)
        uint32_t v = 0;
        int nd = 0;
        while (nd < 3 && !at_end() && peek() >= '0' && peek() <= '7') {
          uint32_t nv = v * 8 + (peek() - '0');
          if (nv > 0377) break;
          v = nv;
          ++i;
          ++nd;
        }
        if (nd == 0) return fail("bad octal escape");
        out = {{v, v}};
        return true;
      }
      default:
        if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '1' && c <= '9'))
          return fail(in_class ? "unsupported escape in class" : "unsupported escape (backreference, \\b, \\p, \\Q, ...)");
        out = {{c, c}};  // escaped non-alphanumeric: the literal character
        return true;
    }
  }

  bool parse_class(int& node) {  // i just after '['
    bool neg = false;
    if (peek() == '^') { neg = true; ++i; }
    Ranges acc;
    bool first = true;
    while (true) {
      if (at_end()) return fail("unterminated class");
      uint32_t c = peek();
      if (c == ']' && !first) { ++i; break; }
      if (c == ']') return fail("empty class");
      if (c == '[') return fail("nested class / union");
      if (c == '&' && peek(1) == '&') return fail("class intersection");
      first = false;
      Ranges item;
      bool single = false;
      uint32_t lo = 0;
      if (c == '\\') {
        ++i;
        if (!escape(item, true)) return false;
        single = item.size() == 1 && item[0].first == item[0].second;
        lo = item[0].first;
      } else {
        ++i;
        item = {{c, c}};
        single = true;
        lo = c;
      }
      // range a-b ('-' before ']' is a literal)
      if (single && peek() == '-' && peek(1) != ']' && peek(1) != 0xFFFFFFFFu) {
        ++i;
        uint32_t hc = peek();
        uint32_t hi;
        if (hc == '\\') {
          ++i;
          Ranges h;
          if (!escape(h, true)) return false;
          if (h.size() != 1 || h[0].first != h[0].second) return fail("class escape as range bound");
          hi = h[0].first;
        } else if (hc == '[') {
          return fail("nested class / union");
        } else {
          ++i;
          hi = hc;
        }
        if (hi < lo) return fail("illegal character range");
        item = {{lo, hi}};
      }
      acc.insert(acc.end(), item.begin(), item.end());
    }
    Node n;
    n.k = Node::SET;
    n.set = neg ? complement(acc) : normalize(acc);
    node = add(std::move(n));
    return true;
  }

  bool parse_atom(int& node, int depth) {
    uint32_t c = peek();
    if (c == '(') {
      ++i;
      if (peek() == '?') {
        ++i;
        uint32_t d = peek();
        if (d == ':') {
          ++i;
        } else if (d == '<' && peek(1) != '=' && peek(1) != '!') {  // named group
          ++i;
          while (!at_end() && peek() != '>') ++i;
          if (at_end()) return fail("unterminated group name");
          ++i;
        } else {
          return fail("look-around, atomic group or inline flags");
        }
      }
      if (!parse_alt(node, depth + 1)) return false;
      if (peek() != ')') return fail("missing ')'");
      ++i;
      return true;
    }
    if (c == '[') { ++i; return parse_class(node); }
    Node n;
    n.k = Node::SET;
    if (c == '.') {
      ++i;
      n.set = dot_ranges();
    } else if (c == '\\') {
      ++i;
      if (!escape(n.set, false)) return false;
      n.set = normalize(n.set);
    } else if (c == '*' || c == '+' || c == '?' || c == '{') {
      return fail("dangling quantifier");
    } else if (c == '^' || c == '$') {
      return fail("anchor inside the pattern");
    } else {
      ++i;
      n.set = {{c, c}};
    }
    node = add(std::move(n));
    return true;
  }

  bool parse_int(int& v) {
    if (at_end() || peek() < '0' || peek() > '9') return false;
    v = 0;
    while (!at_end() && peek() >= '0' && peek() <= '9') {
      v = v * 10 + (int)(cp[i++] - '0');
      if (v > 1000) return fail("repetition bound above 1000");
    }
    return true;
  }

  bool parse_repeat(int& node, int depth) {
    if (!parse_atom(node, depth)) return false;
    while (true) {
      uint32_t c = peek();
      int lo, hi;
      if (c == '*') { lo = 0; hi = -1; ++i; }
      else if (c == '+') { lo = 1; hi = -1; ++i; }
      else if (c == '?') { lo = 0; hi = 1; ++i; }
      else if (c == '{') {
        ++i;
        if (!parse_int(lo)) return fail("bad repetition");
        hi = lo;
        if (peek() == ',') {
          ++i;
          if (peek() == '}') hi = -1;
          else if (!parse_int(hi)) return fail("bad repetition");
        }
        if (peek() != '}') return fail("bad repetition");
        ++i;
        if (hi >= 0 && hi < lo) return fail("bad repetition bounds");
      } else {
        return true;
      }
      if (peek() == '+') return fail("possessive quantifier");
      if (peek() == '?') ++i;  // lazy: same language
      Node r;
      r.k = Node::REP;
      r.kids = {node};
      r.lo = lo;
      r.hi = hi;
      node = add(std::move(r));
    }
  }

  bool parse_cat(int& node, int depth) {
    Node n;
    n.k = Node::CAT;
    while (!at_end() && peek() != '|' && peek() != ')') {
      if (depth == 0 && peek() == '$' && i + 1 == cp.size()) {  // trailing `$`
        anchored_end = true;
        ++i;
        break;
      }
      int a;
      if (!parse_repeat(a, depth)) return false;
      n.kids.push_back(a);
    }
    if (n.kids.empty()) n.k = Node::EMPTY;
    node = add(std::move(n));
    return true;
  }

  bool parse_alt(int& node, int depth) {
    Node n;
    n.k = Node::ALT;
    int a;
    if (!parse_cat(a, depth)) return false;
    n.kids.push_back(a);
    while (peek() == '|') {
      ++i;
      if (!parse_cat(a, depth)) return false;
      n.kids.push_back(a);
    }
    if (n.kids.size() == 1) { node = n.kids[0]; return true; }
    node = add(std::move(n));
    return true;
  }

  bool nullable(int k) const {
    const Node& n = nodes[k];
    switch (n.k) {
      case Node::EMPTY: return true;
      case Node::SET: return false;
      case Node::CAT:
        for (int c : n.kids) if (!nullable(c)) return false;
        return true;
      case Node::ALT:
        for (int c : n.kids) if (nullable(c)) return true;
        return false;
      case Node::REP: return n.lo == 0 || nullable(n.kids[0]);
    }
    return true;
  }
};

bool decode_utf8(const char* s, std::vector<uint32_t>& out) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(s);
  while (*p) {
    uint32_t c = *p;
    int n = c < 0x80 ? 0 : (c >> 5) == 6 ? 1 : (c >> 4) == 14 ? 2 : (c >> 3) == 30 ? 3 : -1;
    if (n < 0) return false;
    c &= n == 0 ? 0x7F : (0x3F >> n);
    ++p;
    for (int k = 0; k < n; ++k, ++p) {
      if ((*p & 0xC0) != 0x80) return false;
      c = (c << 6) | (*p & 0x3F);
    }
    out.push_back(c);
  }
  return true;
}

// ---- UTF-8 byte-range sequences of a code point range (the classic utf8-ranges split) ----
using ByteSeq = std::vector<std::pair<uint8_t, uint8_t>>;
int enc_utf8(uint32_t c, uint8_t* b) {
  if (c < 0x80) { b[0] = (uint8_t)c; return 1; }
  if (c < 0x800) { b[0] = (uint8_t)(0xC0 | (c >> 6)); b[1] = (uint8_t)(0x80 | (c & 0x3F)); return 2; }
  if (c < 0x10000) {
    b[0] = (uint8_t)(0xE0 | (c >> 12)); b[1] = (uint8_t)(0x80 | ((c >> 6) & 0x3F)); b[2] = (uint8_t)(0x80 | (c & 0x3F));
    return 3;
  }
  b[0] = (uint8_t)(0xF0 | (c >> 18)); b[1] = (uint8_t)(0x80 | ((c >> 12) & 0x3F));
  b[2] = (uint8_t)(0x80 | ((c >> 6) & 0x3F)); b[3] = (uint8_t)(0x80 | (c & 0x3F));
  return 4;
}
void utf8_split(uint32_t lo, uint32_t hi, std::vector<ByteSeq>& out) {
  if (lo > hi) return;
  static const uint32_t kBound[3] = {0x7F, 0x7FF, 0xFFFF};
  for (uint32_t b : kBound)
    if (lo <= b && hi > b) { utf8_split(lo, b, out); utf8_split(b + 1, hi, out); return; }
  if (hi <= 0x7F) { out.push_back({{(uint8_t)lo, (uint8_t)hi}}); return; }
  for (int k = 1; k < 4; ++k) {
    uint32_t m = (1u << (6 * k)) - 1;
    if ((lo & ~m) != (hi & ~m)) {
      if ((lo & m) != 0) { utf8_split(lo, lo | m, out); utf8_split((lo | m) + 1, hi, out); return; }
      if ((hi & m) != m) { utf8_split(lo, (hi & ~m) - 1, out); utf8_split(hi & ~m, hi, out); return; }
    }
  }
  uint8_t a[4], b[4];
  int n = enc_utf8(lo, a);
  enc_utf8(hi, b);
  ByteSeq s;
  for (int k = 0; k < n; ++k) s.push_back({a[k], b[k]});
  out.push_back(s);
}

// ---- Thompson NFA over bytes ----
struct Nfa {
  struct Edge { uint8_t lo, hi; int to; };
  std::vector<std::vector<int>> eps;
  std::vector<std::vector<Edge>> edges;
  int add() { eps.emplace_back(); edges.emplace_back(); return (int)eps.size() - 1; }
};
constexpr int kMaxNfa = 200000;
constexpr int kMaxDfa = 4096;

struct Builder {
  const Parser& P;
  Nfa& N;
  bool overflow = false;
  std::pair<int, int> build(int k) {
    if ((int)N.eps.size() > kMaxNfa) { overflow = true; int s = N.add(); return {s, s}; }
    const Node& n = P.nodes[k];
    switch (n.k) {
      case Node::EMPTY: { int s = N.add(); return {s, s}; }
      case Node::SET: {
        int s = N.add(), e = N.add();
        std::vector<ByteSeq> seqs;
        for (auto& r : n.set) utf8_split(r.first, r.second, seqs);
        for (auto& q : seqs) {
          int cur = s;
          for (size_t j = 0; j < q.size(); ++j) {
            int nx = j + 1 == q.size() ? e : N.add();
            N.edges[cur].push_back({q[j].first, q[j].second, nx});
            cur = nx;
          }
        }
        return {s, e};
      }
      case Node::CAT: {
        auto f = build(n.kids[0]);
        for (size_t j = 1; j < n.kids.size(); ++j) {
          auto g = build(n.kids[j]);
          N.eps[f.second].push_back(g.first);
          f.second = g.second;
        }
        return f;
      }
      case Node::ALT: {
        int s = N.add(), e = N.add();
        for (int c : n.kids) {
          auto g = build(c);
          N.eps[s].push_back(g.first);
          N.eps[g.second].push_back(e);
        }
        return {s, e};
      }
      case Node::REP: {
        int s = N.add(), cur = s;
        for (int j = 0; j < n.lo; ++j) {
          auto g = build(n.kids[0]);
          N.eps[cur].push_back(g.first);
          cur = g.second;
        }
        if (n.hi < 0) {  // star of one more copy
          auto g = build(n.kids[0]);
          int e = N.add();
          N.eps[cur].push_back(g.first);
          N.eps[cur].push_back(e);
          N.eps[g.second].push_back(g.first);
          N.eps[g.second].push_back(e);
          return {s, e};
        }
        int e = N.add();
        for (int j = n.lo; j < n.hi; ++j) {  // optional copies
          auto g = build(n.kids[0]);
          N.eps[cur].push_back(g.first);
          N.eps[cur].push_back(e);
          cur = g.second;
        }
        N.eps[cur].push_back(e);
        return {s, e};
      }
    }
    int s = N.add();
    return {s, s};
  }
};

void closure(const Nfa& N, std::vector<int>& set, std::vector<uint32_t>& mark, uint32_t stamp) {
  std::vector<int> stack(set.begin(), set.end());
  for (int s : set) mark[s] = stamp;
  while (!stack.empty()) {
    int s = stack.back();
    stack.pop_back();
    for (int t : N.eps[s])
      if (mark[t] != stamp) { mark[t] = stamp; set.push_back(t); stack.push_back(t); }
  }
  std::sort(set.begin(), set.end());
}

}  // namespace

dq_status regex_compile(const char* pattern, int32_t mode, RegexDfa& out) {
  if (!pattern) return set_error(DQ_E_INVALID, "NULL pattern");
  Parser P;
  if (!decode_utf8(pattern, P.cp)) return set_error(DQ_E_INVALID, "pattern is not valid UTF-8");
  const bool full = mode == DQ_REGEX_FULL;  // whole-value match: string = / IN
  if (full) P.anchored_start = true;
  else if (!P.cp.empty() && P.cp[0] == '^') { P.anchored_start = true; P.i = 1; }
  int root = -1;
  if (!P.parse_alt(root, 0) || !P.at_end()) {
    if (P.err.empty()) P.err = "unbalanced ')'";
    return set_error(DQ_E_UNSUPPORTED, "pattern /%s/: %s", pattern, P.err.c_str());
  }
  if (full) {
    if (P.anchored_end) return set_error(DQ_E_UNSUPPORTED, "pattern /%s/: `$` in a whole-value match", pattern);
    P.anchored_end = true;  // accepted at end of input only, no line-terminator allowance
  } else if ((P.anchored_start || P.anchored_end) && P.nodes[root].k == Node::ALT)
    return set_error(DQ_E_UNSUPPORTED, "pattern /%s/: anchor with top-level alternation", pattern);
  const bool can_be_empty = P.nullable(root);
  // regexp_extract(...) != "": an empty leftmost match counts as no match; which match Java's
  // backtracking prefers at a position is not a property of the language -> fallback
  if (mode == DQ_REGEX_EXTRACT_NONEMPTY && can_be_empty)
    return set_error(DQ_E_UNSUPPORTED, "pattern /%s/ matches the empty string", pattern);

  Nfa N;
  Builder B{P, N};
  const int s0 = N.add();
  if (!P.anchored_start) N.edges[s0].push_back({0, 255, s0});  // unanchored search: skip any prefix
  auto f = B.build(root);
  N.eps[s0].push_back(f.first);
  const int accept = N.add();
  if (full) {
    N.eps[f.second].push_back(accept);
  } else if (P.anchored_end) {  // R then an optional final line terminator, accepted at end of input only
    N.eps[f.second].push_back(accept);
    static const char* kTerm[] = {"\r\n", "\n", "\r", "\xC2\x85", "\xE2\x80\xA8", "\xE2\x80\xA9"};
    for (const char* t : kTerm) {
      int cur = f.second;
      for (size_t j = 0; t[j]; ++j) {
        int nx = t[j + 1] ? N.add() : accept;
        N.edges[cur].push_back({(uint8_t)t[j], (uint8_t)t[j], nx});
        cur = nx;
      }
    }
  } else {
    N.eps[f.second].push_back(accept);
  }
  if (B.overflow) return set_error(DQ_E_UNSUPPORTED, "pattern /%s/: NFA above %d states", pattern, kMaxNfa);

  // byte equivalence classes
  bool cut[257] = {false};
  cut[0] = true;
  for (auto& es : N.edges)
    for (auto& e : es) { cut[e.lo] = true; cut[e.hi + 1] = true; }
  int nc = 0;
  uint8_t cls[256];
  std::vector<int> rep;
  for (int b = 0; b < 256; ++b) {
    if (cut[b]) { rep.push_back(b); ++nc; }
    cls[b] = (uint8_t)(nc - 1);
  }

  // subset construction; 0 = dead, 1 = sticky accept (unanchored end), then discovered sets
  std::vector<uint32_t> mark(N.eps.size(), 0);
  uint32_t stamp = 0;
  std::map<std::vector<int>, int> id;
  std::vector<std::vector<int>> sets;
  std::vector<uint16_t> trans;
  std::vector<uint8_t> acc;
  auto intern = [&](std::vector<int>& s) -> int {
    if (s.empty()) return 0;
    const bool has_acc = std::binary_search(s.begin(), s.end(), accept);
    if (has_acc && !P.anchored_end) return 1;
    auto it = id.find(s);
    if (it != id.end()) return it->second;
    int k = (int)sets.size() + 2;
    id.emplace(s, k);
    sets.push_back(s);
    return k;
  };
  std::vector<int> start = {s0};
  closure(N, start, mark, ++stamp);
  const int start_id = intern(start);
  for (size_t q = 0; q < sets.size(); ++q) {
    if (sets.size() + 2 > (size_t)kMaxDfa)
      return set_error(DQ_E_UNSUPPORTED, "pattern /%s/: DFA above %d states", pattern, kMaxDfa);
    const std::vector<int> cur = sets[q];
    for (int c = 0; c < nc; ++c) {
      const uint8_t b = (uint8_t)rep[c];
      std::vector<int> nx;
      ++stamp;
      for (int s : cur)
        for (auto& e : N.edges[s])
          if (b >= e.lo && b <= e.hi && mark[e.to] != stamp) { mark[e.to] = stamp; nx.push_back(e.to); }
      closure(N, nx, mark, ++stamp);
      trans.push_back((uint16_t)intern(nx));
    }
  }
  const int ns = (int)sets.size() + 2;
  out.n_states = ns;
  out.n_classes = nc;
  out.start = start_id;
  out.end_anchored = P.anchored_end;
  std::memcpy(out.cls, cls, 256);
  out.acc_end.assign(ns, 0);
  out.acc_end[1] = 1;
  for (int k = 2; k < ns; ++k)
    out.acc_end[k] = std::binary_search(sets[k - 2].begin(), sets[k - 2].end(), accept) ? 1 : 0;
  out.trans.assign((size_t)ns * nc, 0);
  for (int c = 0; c < nc; ++c) out.trans[(size_t)1 * nc + c] = 1;
  std::copy(trans.begin(), trans.end(), out.trans.begin() + 2 * nc);
  return DQ_OK;
}

void regex_serialize(const RegexDfa& d, std::vector<uint16_t>& blob) {
  blob.push_back((uint16_t)d.n_states);
  blob.push_back((uint16_t)d.n_classes);
  blob.push_back((uint16_t)d.start);
  blob.push_back((uint16_t)(d.end_anchored ? 1 : 0));
  for (int b = 0; b < 256; ++b) blob.push_back(d.cls[b]);
  for (int s = 0; s < d.n_states; ++s) blob.push_back(d.acc_end[s]);
  blob.insert(blob.end(), d.trans.begin(), d.trans.end());
}

bool regex_run(const RegexDfa& d, const uint8_t* s, int64_t len) {
  int st = d.start;
  for (int64_t i = 0; i < len && st >= 2; ++i) st = d.trans[(size_t)st * d.n_classes + d.cls[s[i]]];
  return d.acc_end[st] != 0;
}

}  // namespace dq

extern "C" {

dq_status dq_regex_info(const char* pattern, int32_t mode, int32_t* n_states, int32_t* n_classes) {
  dq::RegexDfa d;
  if (dq_status s = dq::regex_compile(pattern, mode, d)) return s;
  if (n_states) *n_states = d.n_states;
  if (n_classes) *n_classes = d.n_classes;
  return DQ_OK;
}

dq_status dq_regex_match_host(const char* pattern, int32_t mode, const uint8_t* data, const int64_t* offsets,
                              int64_t n, uint8_t* out) {
  dq::RegexDfa d;
  if (dq_status s = dq::regex_compile(pattern, mode, d)) return s;
  if (n < 0 || (n > 0 && (!data || !offsets || !out))) return dq::set_error(DQ_E_INVALID, "bad arguments");
  for (int64_t r = 0; r < n; ++r) out[r] = dq::regex_run(d, data + offsets[r], offsets[r + 1] - offsets[r]) ? 1 : 0;
  return DQ_OK;
}

}  // extern "C"
