"""Spark-SQL predicate strings -> the C ABI predicate IR (dqscan.h, dq_pred_node).

Stands in for Spark's `expr(...)` parser at the boundary (analyzers/Analyzer.scala:385-408 and
the predicate strings checks/Check.scala builds at :676, :687, :705-760, :840, :867-868).  The
accepted grammar is the numeric subset the GPU evaluates with SQL three-valued logic:

    expr     := or
    or       := and ( OR and )*
    and      := not ( AND not )*
    not      := NOT not | cmp
    cmp      := operand ( (< | <= | > | >= | = | == | != | <>) operand | IS [NOT] NULL )?
    operand  := column | `column` | number | NULL | TRUE | FALSE | COALESCE(operand, operand)
              | ( expr ) | - number
    strcmp   := column (= | == | != | <>) 'string' | 'string' (= | ...) column
              | column [NOT] IN ('string', ...)

Literal typing follows Spark 2.2: `3` integer, `3.0` exact decimal, `3e0` double.  String
(in)equality and IN lists on a string column are byte-wise equality of the UTF-8 values; they lower to
a whole-value DFA (DQ_PRED_REGEX, mode DQ_REGEX_FULL) over the escaped literals.  Anything else
(string ordering, LIKE, RLIKE, functions, literals with backslash escapes) raises UnsupportedPredicate:
such an analyzer is routed to the fallback set, exactly like a type the GPU plan does not cover.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

from . import _lib as L


class UnsupportedPredicate(ValueError):
    pass


_KEYWORDS = {"AND", "OR", "NOT", "IS", "NULL", "COALESCE", "TRUE", "FALSE", "IN", "LIKE", "RLIKE", "BETWEEN"}


def _tokenize(s: str) -> List[Tuple[str, str]]:
    toks = []
    i = 0
    while i < len(s):
        c = s[i]
        if c.isspace():
            i += 1
        elif c == "`":
            j = s.find("`", i + 1)
            if j < 0:
                raise UnsupportedPredicate(f"unterminated identifier in {s!r}")
            toks.append(("id", s[i + 1:j]))
            i = j + 1
        elif c in "'\"":
            j = s.find(c, i + 1)
            if j < 0:
                raise UnsupportedPredicate(f"unterminated string literal in {s!r}")
            if "\\" in s[i + 1:j]:  # Spark unescapes backslash sequences: not restated here
                raise UnsupportedPredicate(f"string literal with a backslash escape in {s!r}")
            toks.append(("str", s[i + 1:j]))
            i = j + 1
        elif c.isdigit() or (c == "." and i + 1 < len(s) and s[i + 1].isdigit()):
            j = i
            while j < len(s) and (s[j].isdigit() or s[j] == "."):
                j += 1
            if j < len(s) and s[j] in "eE":
                j += 1
                if j < len(s) and s[j] in "+-":
                    j += 1
                while j < len(s) and s[j].isdigit():
                    j += 1
            if j < len(s) and s[j] in "dDlLsSyY":  # typed literal suffixes (1.0D, 10L, ...)
                raise UnsupportedPredicate(f"typed literal suffix in {s!r}")
            toks.append(("num", s[i:j]))
            i = j
        elif c.isalpha() or c == "_":
            j = i
            while j < len(s) and (s[j].isalnum() or s[j] == "_"):
                j += 1
            w = s[i:j]
            toks.append(("kw", w.upper()) if w.upper() in _KEYWORDS else ("id", w))
            i = j
        elif s.startswith(("<=", ">=", "!=", "<>", "=="), i):
            toks.append(("op", s[i:i + 2]))
            i += 2
        elif c in "<>=(),-":
            toks.append(("op", c))
            i += 1
        else:
            raise UnsupportedPredicate(f"unexpected character {c!r} in {s!r}")
    return toks


_CMP = {"<": L.CMP_LT, "<=": L.CMP_LE, ">": L.CMP_GT, ">=": L.CMP_GE, "=": L.CMP_EQ, "==": L.CMP_EQ,
        "!=": L.CMP_NE, "<>": L.CMP_NE}


class PredicatePool:
    """Accumulates IR nodes for several predicate roots of one plan."""

    def __init__(self, column_index: Dict[str, int]):
        self.column_index = column_index
        self.nodes: List[Tuple[int, int, int, int, int, float]] = []
        self.patterns: List[str] = []  # DQ_PRED_REGEX patterns (dq_plan_create_ex)

    def _add(self, kind, a=-1, b=-1, cmp=0, i64=0, f64=0.0) -> int:
        self.nodes.append((kind, a, b, cmp, i64, f64))
        return len(self.nodes) - 1

    def add_regex(self, column: int, pattern: str, mode: int) -> int:
        """A DQ_PRED_REGEX node on plan column `column`; raises UnsupportedPredicate when the pattern
        is outside the GPU regex subset (dq_regex_info), so the analyzer is routed to the fallback."""
        import ctypes

        if L.lib.dq_regex_info(pattern.encode("utf-8"), mode, None, None) != L.DQ_OK:
            raise UnsupportedPredicate(L.lib.dq_last_error().decode("utf-8", "replace"))
        if pattern not in self.patterns:
            self.patterns.append(pattern)
        col = self._add(L.PRED_COLUMN, column)
        return self._add(L.PRED_REGEX, col, -1, mode, self.patterns.index(pattern))

    def is_string_column(self, plan_col: int) -> bool:
        b = getattr(self.column_index, "b", None)
        if b is None:
            return False
        return b.by_name[b.columns[plan_col]][1] in ("utf8", "large_utf8")

    def patterns_ctypes(self):
        import ctypes

        arr = (ctypes.c_char_p * max(1, len(self.patterns)))(*[p.encode("utf-8") for p in self.patterns])
        return arr, len(self.patterns)

    def add(self, text: str) -> int:
        """Parse `text`; returns the root node index."""
        p = _Parser(_tokenize(text), text, self)
        root = p.parse_or()
        if p.pos != len(p.toks):
            raise UnsupportedPredicate(f"unsupported syntax near {p.toks[p.pos]} in {text!r}")
        return root

    def as_ctypes(self):
        arr = (L.PredNode * max(1, len(self.nodes)))()
        for i, (k, a, b, c, i64, f64) in enumerate(self.nodes):
            arr[i].kind, arr[i].a, arr[i].b, arr[i].cmp, arr[i].i64, arr[i].f64 = k, a, b, c, i64, f64
        return arr, len(self.nodes)


class _Parser:
    def __init__(self, toks, text, pool: PredicatePool):
        self.toks, self.text, self.pool, self.pos = toks, text, pool, 0

    def peek(self):
        return self.toks[self.pos] if self.pos < len(self.toks) else (None, None)

    def take(self):
        t = self.peek()
        self.pos += 1
        return t

    def expect(self, tok):
        t = self.take()
        if t != tok:
            raise UnsupportedPredicate(f"expected {tok[1]!r}, got {t[1]!r} in {self.text!r}")

    def parse_or(self):
        a = self.parse_and()
        while self.peek() == ("kw", "OR"):
            self.take()
            a = self.pool._add(L.PRED_OR, a, self.parse_and())
        return a

    def parse_and(self):
        a = self.parse_not()
        while self.peek() == ("kw", "AND"):
            self.take()
            a = self.pool._add(L.PRED_AND, a, self.parse_not())
        return a

    def parse_not(self):
        if self.peek() == ("kw", "NOT"):
            self.take()
            return self.pool._add(L.PRED_NOT, self.parse_not())
        return self.parse_cmp()

    def parse_cmp(self):
        a = self.parse_operand()
        k, v = self.peek()
        if k == "op" and v in _CMP:
            self.take()
            b = self.parse_operand()
            if isinstance(a, str) or isinstance(b, str):  # string (in)equality
                if v not in ("=", "==", "!=", "<>"):
                    raise UnsupportedPredicate(f"string ordering comparison in {self.text!r}")
                col, lit = (b, a) if isinstance(a, str) else (a, b)
                if isinstance(col, str):
                    raise UnsupportedPredicate(f"comparison of two string literals in {self.text!r}")
                e = self._string_in(col, [lit])
                return self.pool._add(L.PRED_NOT, e) if v in ("!=", "<>") else e
            return self.pool._add(L.PRED_CMP, a, b, _CMP[v])
        if (k, v) in (("kw", "IN"), ("kw", "NOT")) and not isinstance(a, str):
            neg = v == "NOT"
            save = self.pos
            self.take()
            if neg and self.peek() != ("kw", "IN"):
                self.pos = save
                return a
            if neg:
                self.take()
            self.expect(("op", "("))
            items = [self.take()]
            while self.peek() == ("op", ","):
                self.take()
                items.append(self.take())
            self.expect(("op", ")"))
            if any(t[0] != "str" for t in items):
                raise UnsupportedPredicate(f"IN list of non-string literals in {self.text!r}")
            e = self._string_in(a, [t[1] for t in items])
            return self.pool._add(L.PRED_NOT, e) if neg else e
        if (k, v) == ("kw", "IS"):
            self.take()
            neg = False
            if self.peek() == ("kw", "NOT"):
                self.take()
                neg = True
            self.expect(("kw", "NULL"))
            return self.pool._add(L.PRED_IS_NOT_NULL if neg else L.PRED_IS_NULL, a)
        if k == "kw" and v in ("LIKE", "RLIKE", "BETWEEN"):
            raise UnsupportedPredicate(f"{v} is not in the GPU predicate grammar: {self.text!r}")
        if isinstance(a, str):
            raise UnsupportedPredicate(f"bare string literal in {self.text!r}")
        return a

    def _string_in(self, col_node: int, literals):
        """col IN (literals) as one whole-value DFA: (?:l1|l2|...) with every non-alphanumeric
        ASCII character escaped (the DFA compiler reads `\\` + such a character as the literal)."""
        k, c = self.pool.nodes[col_node][0], self.pool.nodes[col_node][1]
        if k != L.PRED_COLUMN:
            raise UnsupportedPredicate(f"string comparison on a non-column expression in {self.text!r}")
        if not self.pool.is_string_column(c):
            raise UnsupportedPredicate(f"string literal compared with a non-string column in {self.text!r}")
        esc = ["".join(ch if (ch.isalnum() and ord(ch) < 128) or ord(ch) >= 128 else "\\" + ch for ch in lit)
               for lit in literals]
        pattern = "(?:" + "|".join(esc) + ")"
        if col_node == len(self.pool.nodes) - 1:
            self.pool.nodes.pop()  # the column node is re-added by add_regex
        return self.pool.add_regex(c, pattern, L.REGEX_FULL)

    def parse_operand(self):
        k, v = self.take()
        if (k, v) == ("op", "("):
            e = self.parse_or()
            self.expect(("op", ")"))
            return e
        if (k, v) == ("op", "-"):
            k2, v2 = self.take()
            if k2 != "num":
                raise UnsupportedPredicate(f"unary minus on a non-literal in {self.text!r}")
            return self._number("-" + v2)
        if k == "num":
            return self._number(v)
        if k == "str":
            return v  # a python str: only valid as one side of a string (in)equality / IN
        if (k, v) == ("kw", "NULL"):
            return self.pool._add(L.PRED_LIT_NULL)
        if k == "kw" and v in ("TRUE", "FALSE"):
            return self.pool._add(L.PRED_LIT_BOOL, i64=1 if v == "TRUE" else 0)
        if (k, v) == ("kw", "COALESCE"):
            self.expect(("op", "("))
            a = self.parse_operand()
            self.expect(("op", ","))
            b = self.parse_operand()
            if self.peek() == ("op", ","):
                raise UnsupportedPredicate(f"COALESCE with more than two arguments in {self.text!r}")
            self.expect(("op", ")"))
            return self.pool._add(L.PRED_COALESCE, a, b)
        if k == "id":
            if self.peek() == ("op", "("):
                raise UnsupportedPredicate(f"function call {v}(...) in {self.text!r}")
            if v not in self.pool.column_index:
                raise KeyError(v)
            return self.pool._add(L.PRED_COLUMN, self.pool.column_index[v])
        raise UnsupportedPredicate(f"unexpected token {v!r} in {self.text!r}")

    def _number(self, s: str) -> int:
        if "e" in s or "E" in s:
            return self.pool._add(L.PRED_LIT_DOUBLE, f64=float(s))
        if "." in s:
            neg = s.startswith("-")
            body = s[1:] if neg else s
            ip, fp = body.split(".", 1)
            unscaled = int((ip or "0") + fp) if (ip or fp) else 0
            if unscaled >= 1 << 63 or len(fp) > 18:
                raise UnsupportedPredicate(f"decimal literal {s} exceeds 64-bit precision")
            return self.pool._add(L.PRED_LIT_DECIMAL, cmp=len(fp), i64=-unscaled if neg else unscaled)
        v = int(s)
        if not -(1 << 63) <= v < (1 << 63):
            raise UnsupportedPredicate(f"integer literal {s} out of range")
        return self.pool._add(L.PRED_LIT_INT, i64=v)


def referenced_columns(text: str) -> Sequence[str]:
    """Column names a predicate references (for Preconditions.hasColumn-like checks)."""
    return [v for k, v in _tokenize(text) if k == "id"]
