"""PatternMatch / RLIKE pattern compiler (deequ_amd/csrc/dq_regex.cpp) vs the oracle, on the CPU.

The compiler turns a java.util.regex pattern into the byte-level search DFA the GPU walks
(dq_kernels.hip, pred_atom_regex).  dq_regex_match_host walks the same DFA on the host, so this
checks the compiler -- parser, UTF-8 range splitting, subset construction, `^` / `$` handling --
against the oracle's restatement of Spark's regexp_extract (Python's backtracking `re` with Java's
defaults, pinned by the reference's PatternMatch known answers in tests/golden/reference_kats.json).
The GPU walk itself is checked in tests/test_gpu_parity.py::test_pattern_match_vs_oracle.

Known, documented gap: a trailing `$` accepts "\\n" as the final terminator even when
the match ends with "\\r" (Java refuses to match between \\r and \\n); inputs here contain no "\\r".
"""
from __future__ import annotations

import ctypes
import zlib

import numpy as np
import pytest

from oracle import dq_oracle as O

PATTERNS = [
    r"\d", r"\d\.\d", r"^\d+$", r"^[a-z]+@", r"(?:ab|cd){2,3}x?", "é+", r"[^\s]+\s[^\s]+", ".{3}€",
    r"[à-ÿ]{2}", r"a.c", r"(?<g>x|y)z", r"[0-9]{2,4}-[a-z]*q", r"\x41é", "𝄞.", r"[^a-z]{3,}$",
    r"colou?r", r"\.\*\+", r"[\[\]]", r"\w+\W\w+", r"[-a]b", r"[a-]c", r"a}", r"\x{1D11E}", r"[^\x00-\x7f]",
    r"a+?b", r"(a|ab)(c|bcd)", r"\t|\n", "x.{0,2}y$", r"\0101", r"\e|\a", r"[\d\s]{4}", r"(?:(?:a|b)c)+d",
]
UNSUPPORTED = [
    r"\bab", r"(a)\1", r"(?=a)b", r"(?!a)b", r"(?<=a)b", r"(?i)ab", r"a++", r"(?>a)", r"[a&&b]", r"[[a]]",
    r"\p{Lu}", r"a^b", r"a$b", r"^a|b", r"a|b$", r"a*", r"(a|)", r"x?", r"\Qa\E", "(ab", "ab)", r"a{2,1}",
]


@pytest.fixture(scope="module")
def lib():
    import deequ_amd

    return deequ_amd


def _strings(seed: int, n: int):
    rng = np.random.default_rng(seed)
    alphabet = list("abcdxyzq@.-_:/ \t\n0123456789ABé€𝄞☺{}[]*+") + ["colour", "color", "ab", "cd", "http://",
                                                                 "someone@somewhere.org", "1.5", "àé", "\x1b"]
    out = ["", "a", "1", "ab", "é", "𝄞x", "\n", "12\n", "x1y", "xy"]
    for _ in range(n):
        k = int(rng.integers(0, 12))
        out.append("".join(alphabet[int(j)] for j in rng.integers(0, len(alphabet), k)))
    return [s.encode("utf-8") for s in out]


def _host_match(lib, pattern, mode, values):
    from deequ_amd import _lib as L

    data = b"".join(values)
    offs = np.zeros(len(values) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(v) for v in values])
    out = np.zeros(len(values), dtype=np.uint8)
    st = L.lib.dq_regex_match_host(pattern.encode("utf-8"), mode, ctypes.c_char_p(data),
                                   offs.ctypes.data_as(ctypes.c_void_p), len(values),
                                   out.ctypes.data_as(ctypes.c_void_p))
    return st, out.astype(bool)


def test_patterns_equal_reference(lib):
    import json
    import os

    kats = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))
    pats = {c["dataset"]: c["analyzer"][2] for c in kats["cases"] if c["analyzer"][0] == "PatternMatch"}
    assert pats["patternEmails"] == lib.Patterns.EMAIL and pats["patternUrls"] == lib.Patterns.URL
    assert pats["patternSsns"] == lib.Patterns.SOCIAL_SECURITY_NUMBER_US
    assert pats["patternCreditCards"] == lib.Patterns.CREDITCARD


@pytest.mark.parametrize("pattern", PATTERNS + ["EMAIL", "URL"])
def test_dfa_equals_oracle(lib, pattern):
    from deequ_amd import _lib as L

    pattern = getattr(lib.Patterns, pattern, pattern)
    values = _strings(zlib.crc32(pattern.encode()) & 0xFFFF, 400)
    st, got = _host_match(lib, pattern, L.REGEX_EXTRACT_NONEMPTY, values)
    assert st == L.DQ_OK, L.lib.dq_last_error()
    want = np.array([O.regexp_extract_nonempty(v, pattern) for v in values])
    bad = [(v, bool(g), bool(w)) for v, g, w in zip(values, got, want) if g != w]
    assert not bad, bad[:5]


def test_kat_strings_through_dfa(lib):
    """The reference's own PatternMatch rows (URL with non-ASCII hosts, emails) through the DFA."""
    import json
    import os

    from deequ_amd import _lib as L

    kats = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))
    checked = 0
    for c in kats["cases"]:
        if c["analyzer"][0] != "PatternMatch" or c["needs"]:
            continue
        _, col, pattern, _ = c["analyzer"]
        vals = [v.encode("utf-8") for v in kats["datasets"][c["dataset"]]["columns"][col][1]]
        st, got = _host_match(lib, pattern, L.REGEX_EXTRACT_NONEMPTY, vals)
        assert st == 0
        assert got.sum() / len(vals) == c["expected"], (c["source"], got)
        checked += 1
    assert checked == 5


@pytest.mark.parametrize("pattern", UNSUPPORTED)
def test_unsupported_patterns_are_refused(lib, pattern):
    from deequ_amd import _lib as L

    assert L.lib.dq_regex_info(pattern.encode("utf-8"), L.REGEX_EXTRACT_NONEMPTY, None, None) in (
        L.DQ_E_UNSUPPORTED, L.DQ_E_INVALID)
    assert L.lib.dq_last_error()


def test_rlike_mode_accepts_nullable(lib):
    """RLIKE is find(): a pattern that matches the empty string matches every value."""
    from deequ_amd import _lib as L

    values = _strings(5, 50)
    st, got = _host_match(lib, "x*", L.REGEX_RLIKE, values)
    assert st == 0 and got.all()
    st, got = _host_match(lib, "^ab*$", L.REGEX_RLIKE, values)
    assert st == 0
    import re

    want = [re.search(O.java_regex_to_python("^ab*$"), v.decode(), re.ASCII) is not None for v in values]
    assert list(got) == want


def test_fallback_routing(lib):
    """Patterns outside the subset and non-string columns route PatternMatch to the fallback set."""
    from deequ_amd.predicates import UnsupportedPredicate
    from deequ_amd.analyzers import PlanBuilder

    b = PlanBuilder([("s", "utf8", True), ("f", "f64", True)])
    for a in (lib.PatternMatch("s", lib.Patterns.SOCIAL_SECURITY_NUMBER_US), lib.PatternMatch("s", lib.Patterns.CREDITCARD),
              lib.PatternMatch("f", r"\d\.\d"), lib.PatternMatch("s", "a*")):
        with pytest.raises(UnsupportedPredicate):
            a._lower(b)
    op, ca, cb, root, where = lib.PatternMatch("s", lib.Patterns.EMAIL, "f > 0")._lower(b)
    assert root >= 0 and where >= 0 and b.pool.patterns == [lib.Patterns.EMAIL]


@pytest.mark.parametrize("lits", [["a"], ["1", "2"], [""], ["a.b", "c d", "é€", "x|y", "(z)", "q*"], ["ab", "abc", "a"]])
def test_string_in_full_match(lib, lits):
    """`col IN (...)` / `col = '...'` lower to a whole-value DFA over the escaped literals: byte
    equality with any literal, nothing else (no search, no trailing-terminator allowance)."""
    from deequ_amd import _lib as L
    from deequ_amd.analyzers import PlanBuilder

    b = PlanBuilder([("s", "utf8", True)])
    b.pred("s IN (" + ", ".join("'" + x + "'" for x in lits) + ")")
    pattern = b.pool.patterns[-1]
    values = [x.encode() for x in lits] + [x.encode() + b"\n" for x in lits] + [b"x" + x.encode() for x in lits] + \
        _strings(11, 200) + [b"", b"a", b"ab\n", b"c d", b"x|y"]
    st, got = _host_match(lib, pattern, L.REGEX_FULL, values)
    assert st == 0, L.lib.dq_last_error()
    want = [v in {x.encode() for x in lits} for v in values]
    assert list(got) == want


def test_string_predicate_grammar(lib):
    from deequ_amd.analyzers import PlanBuilder
    from deequ_amd.predicates import UnsupportedPredicate

    b = PlanBuilder([("s", "utf8", True), ("n", "i64", True)])
    for ok in ("s = 'x'", "'x' = s", "s != 'x'", "s <> 'x'", "s IN ('a', 'b')", "s NOT IN ('a')",
               "n > 0 AND s = 'q'", "NOT s IN ('a', \"b\")"):
        b.pred(ok)
    for bad in ("n = 'x'", "s < 'x'", "s LIKE 'a%'", "'a' = 'b'", "s = 'a\\\\b'", "s IN (1, 2)", "s RLIKE 'x'"):
        with pytest.raises(UnsupportedPredicate):
            b.pred(bad)
