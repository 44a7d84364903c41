"""Property fuzz of the host C++ that parses untrusted input, through the C ABI (CPU only).

* dq_pred_pool_add: arbitrary SQL-ish text (tokens of the predicate grammar mixed with garbage) returns
  OK / UNSUPPORTED / INVALID, never crashes, and a failed add leaves the pool unchanged (Check.scala's
  predicate strings; Spark's expr() parse is what it replaces);
* dq_state_from_bytes: arbitrary byte images of every state type (HdfsStateProvider formats,
  StateProvider.scala:176-294) are accepted or refused with DQ_E_STATE; an accepted image re-serialises
  to the same bytes;
* dq_regex_info / dq_regex_match_host: arbitrary patterns (PatternMatch regexes) and strings;
* dq_arrow_import: ArrowArray structures with random lengths, offsets, null counts and NULL buffers.

tests/test_sanitizers.py runs this file against the ASan + UBSan build of the library.
"""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

hyp = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

SETTINGS = settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.too_slow])
TOKENS = ["a", "b", "s", "`a`", "`b`", "zz", "(", ")", ",", ">", ">=", "<", "<=", "=", "==", "!=", "<>", "AND", "OR",
          "NOT", "IS", "NULL", "IN", "COALESCE", "TRUE", "FALSE", "LIKE", "BETWEEN", "0", "1", "-3", "2.5", "1e3",
          "1.0e-2", "9223372036854775807", "9223372036854775808", "-9223372036854775809", "0.000000000000000000001",
          "'x'", "'a.b'", "'it''s'", "'", "`", "\\", "1.2.3", "e5", ".5", "5.", "abs(", "+", "-", "*", " ", "\t"]


@pytest.fixture(scope="module")
def L():
    from deequ_amd import _lib

    return _lib


def _pool(L):
    cols = [("a", L.TYPE_F64), ("b", L.TYPE_I64), ("s", L.TYPE_UTF8)]
    names = (ctypes.c_char_p * 3)(*[n.encode() for n, _ in cols])
    types = (ctypes.c_int32 * 3)(*[t for _, t in cols])
    h = ctypes.c_void_p()
    assert L.lib.dq_pred_pool_create(names, types, 3, ctypes.byref(h)) == L.DQ_OK
    return h


@SETTINGS
@given(st.lists(st.sampled_from(TOKENS), min_size=0, max_size=24), st.binary(max_size=12))
def test_pred_pool_add_fuzz(L, toks, junk):
    h = _pool(L)
    try:
        size0 = L.lib.dq_pred_pool_size(h)
        text = " ".join(toks).encode() + (junk if len(junk) % 3 == 0 else b"")
        r = ctypes.c_int32(-7)
        rc = L.lib.dq_pred_pool_add(h, text.replace(b"\0", b" "), ctypes.byref(r))
        assert rc in (L.DQ_OK, L.DQ_E_UNSUPPORTED, L.DQ_E_INVALID, L.DQ_E_TYPE), (text, rc)
        n = L.lib.dq_pred_pool_size(h)
        if rc == L.DQ_OK:
            assert 0 <= r.value < n
            nodes = L.lib.dq_pred_pool_nodes(h)
            for i in range(n):  # child references point at earlier nodes
                k = nodes[i].kind
                if k in (L.PRED_CMP, L.PRED_AND, L.PRED_OR, L.PRED_COALESCE):
                    assert 0 <= nodes[i].a < i and 0 <= nodes[i].b < i
                elif k in (L.PRED_NOT, L.PRED_IS_NULL, L.PRED_IS_NOT_NULL, L.PRED_REGEX):
                    assert 0 <= nodes[i].a < i
        else:
            assert n == size0 and L.lib.dq_last_error()
    finally:
        L.lib.dq_pred_pool_destroy(h)


@SETTINGS
@given(st.integers(0, 13), st.binary(min_size=0, max_size=600))
def test_state_from_bytes_fuzz(L, op, img):
    s = L.State()
    rc = L.lib.dq_state_from_bytes(op, img, len(img), ctypes.byref(s))
    assert rc in (L.DQ_OK, L.DQ_E_STATE, L.DQ_E_INVALID), rc
    if rc == L.DQ_OK:
        buf = ctypes.create_string_buffer(1024)
        n = L.lib.dq_state_to_bytes(ctypes.byref(s), buf, 1024)
        assert n == len(img) and buf.raw[:n] == img


@SETTINGS
@given(st.integers(0, 13), st.sampled_from([4, 8, 16, 24, 48, 416, 420]), st.data())
def test_state_from_bytes_sized_images(L, op, size, data):
    """images of the lengths the formats use (so the parse goes past the length checks)"""
    img = data.draw(st.binary(min_size=size, max_size=size))
    if size == 420:  # an HLL image: int32 length 416 + 416 bytes
        img = (416).to_bytes(4, "big") + img[4:]
    s = L.State()
    rc = L.lib.dq_state_from_bytes(op, img, len(img), ctypes.byref(s))
    assert rc in (L.DQ_OK, L.DQ_E_STATE, L.DQ_E_INVALID)


REGEX_ATOMS = ["a", "b", ".", "\\d", "\\w", "\\s", "\\.", "[a-z]", "[^0-9]", "(", ")", "(?:", "|", "*", "+", "?", "{2}",
               "{1,3}", "^", "$", "\\b", "[", "]", "\\", "{", "}", "@", "-", "x{0}", "(?i)", "\\p{L}", "é"]


@SETTINGS
@given(st.lists(st.sampled_from(REGEX_ATOMS), max_size=14), st.integers(0, 2),
       st.lists(st.binary(max_size=12), min_size=1, max_size=6))
def test_regex_fuzz(L, atoms, mode, strings):
    pat = "".join(atoms).encode("utf-8")
    ns, nc = ctypes.c_int32(), ctypes.c_int32()
    rc = L.lib.dq_regex_info(pat, mode, ctypes.byref(ns), ctypes.byref(nc))
    assert rc in (L.DQ_OK, L.DQ_E_UNSUPPORTED, L.DQ_E_INVALID), (pat, rc)
    data = b"".join(strings)
    offs = np.zeros(len(strings) + 1, dtype=np.int64)
    np.cumsum([len(x) for x in strings], out=offs[1:])
    out = np.zeros(len(strings), dtype=np.uint8)
    rc2 = L.lib.dq_regex_match_host(pat, mode, ctypes.c_char_p(data + b"\0" * 8), offs.ctypes.data, len(strings),
                                    out.ctypes.data)
    assert (rc2 == L.DQ_OK) == (rc == L.DQ_OK)


@SETTINGS
@given(st.sampled_from(["g", "l", "i", "u", "U", "f", "", "ll"]), st.integers(0, 300), st.integers(0, 40),
       st.integers(-2, 400), st.lists(st.booleans(), min_size=3, max_size=3), st.integers(2, 3))
def test_arrow_import_fuzz(L, fmt, n, off, null_count, present, nbuf):
    from deequ_amd.ingest import ArrowArrayC, ArrowSchemaC, HostColumn, _bind

    lib = _bind()
    total = n + off + 1
    validity = np.full(total // 8 + 8, 0xFF, dtype=np.uint8)
    values = np.zeros(total * 8 + 16, dtype=np.uint8)
    offsets = np.arange(total + 1, dtype=np.int64 if fmt == "U" else np.int32) * 2
    data = np.zeros(2 * total + 16, dtype=np.uint8)
    str_ = fmt in ("u", "U")
    raw = [validity.ctypes.data if present[0] else None,
           (offsets.ctypes.data if str_ else values.ctypes.data) if present[1] else None,
           data.ctypes.data if present[2] else None]
    bufs = (ctypes.c_void_p * 3)(*raw)
    release_s = ArrowSchemaC._fields_[-2][1](lambda p: None)
    release_a = ArrowArrayC._fields_[-2][1](lambda p: None)
    sch = ArrowSchemaC()
    sch.format = fmt.encode()
    sch.release = release_s
    arr = ArrowArrayC()
    arr.length, arr.offset, arr.null_count, arr.n_buffers = n, off, null_count, nbuf
    arr.buffers = ctypes.cast(bufs, ctypes.POINTER(ctypes.c_void_p))
    arr.release = release_a
    out = HostColumn()
    rc = lib.dq_arrow_import(ctypes.byref(sch), ctypes.byref(arr), ctypes.byref(out))
    assert rc in (L.DQ_OK, L.DQ_E_UNSUPPORTED, L.DQ_E_INVALID), rc
    if rc == L.DQ_OK:
        assert out.n_rows == n and 0 <= out.validity_bit < 8


# ------------------------------------------------------------------------------------------------------
# random predicate programs through the planner and the predicate-kernel generator (dq_plan_explain: host
# only -- the plan is lowered and, for a numeric program, the compiled pass's kernel source generated from it,
# the path dq_plan_create takes before hipRTC; Check.scala:670-871 builds the strings)
# ------------------------------------------------------------------------------------------------------
_COLS = [("a", "f64"), ("b", "i64"), ("c", "i32"), ("s", "utf8")]
_NUM = ["a", "b", "c", "`a`", "`b`", "`c`"]
_LITS = ["0", "1", "-3", "2.5", "-0.0", "1e3", "1.0e-2", "9223372036854775807", "-9223372036854775808",
         "0.000000000000000000001", "NULL"]
_OPS = [">", ">=", "<", "<=", "=", "==", "!=", "<>"]


def _atom():
    num = st.sampled_from(_NUM)
    lit = st.sampled_from(_LITS)
    return st.one_of(
        st.builds(lambda x, o, y: f"{x} {o} {y}", num, st.sampled_from(_OPS), st.one_of(num, lit)),
        st.builds(lambda x, o, y: f"{y} {o} {x}", num, st.sampled_from(_OPS), lit),
        st.builds(lambda x, n: f"{x} IS {n}NULL", num, st.sampled_from(["", "NOT "])),
        st.builds(lambda x, d, o, y: f"COALESCE({x}, {d}) {o} {y}", num, st.sampled_from(["0", "1.5", "-2"]),
                  st.sampled_from(_OPS), lit),
        st.sampled_from(["TRUE", "FALSE", "NULL", "1 < 2", "s = 'x'", "s IN ('a', 'b')", "s IS NULL"]))


_PRED = st.recursive(_atom(), lambda e: st.one_of(
    st.builds(lambda x, y: f"({x}) AND ({y})", e, e), st.builds(lambda x, y: f"({x}) OR ({y})", e, e),
    st.builds(lambda x: f"NOT ({x})", e)), max_leaves=10)


@SETTINGS
@given(st.lists(_PRED, min_size=1, max_size=6), st.lists(st.booleans(), min_size=6, max_size=6),
       st.sampled_from([0, 1, 2]))
def test_pred_programs_through_planner_and_generator(L, preds, hll, pred_pass):
    names = (ctypes.c_char_p * 4)(*[n.encode() for n, _ in _COLS])
    tcode = {"f64": L.TYPE_F64, "i64": L.TYPE_I64, "i32": L.TYPE_I32, "utf8": L.TYPE_UTF8}
    types = (ctypes.c_int32 * 4)(*[tcode[t] for _, t in _COLS])
    h = ctypes.c_void_p()
    assert L.lib.dq_pred_pool_create(names, types, 4, ctypes.byref(h)) == L.DQ_OK
    try:
        roots = []
        for p in preds:
            r = ctypes.c_int32(-1)
            if L.lib.dq_pred_pool_add(h, p.encode(), ctypes.byref(r)) == L.DQ_OK:
                roots.append((p, r.value))
        if not roots:
            return
        specs = []
        for i, (_, r) in enumerate(roots):
            # Compliance of every accepted root; every second one also as a `where` of a Sum; fused-HLL
            # candidates: ApproxCountDistinct without `where` on the numeric columns
            specs.append((L.OP_COMPLIANCE, -1, -1, r, -1))
            if i % 2:
                specs.append((L.OP_SUM, 1, -1, -1, r))
        for c in range(3):
            if hll[c]:
                specs.append((L.OP_APPROX_COUNT_DISTINCT, c, -1, -1, -1))
        arr = (L.AnalyzerSpec * len(specs))(*[L.AnalyzerSpec(*x) for x in specs])
        sch = (L.ColumnDesc * 4)(*[L.ColumnDesc(tcode[t], 1) for _, t in _COLS])
        nodes = L.lib.dq_pred_pool_nodes(h)
        npred = L.lib.dq_pred_pool_size(h)
        npat = L.lib.dq_pred_pool_num_patterns(h)
        pats = L.lib.dq_pred_pool_patterns(h)
        opts = L.PlanOptions(ctypes.sizeof(L.PlanOptions), pred_pass)
        args = (arr, len(specs), sch, 4, nodes, npred, pats, npat, ctypes.byref(opts))
        n = L.lib.dq_plan_explain(*args, None, 0)
        if n < 0:  # planning limits (counters, roots, nesting) or a required compile the program cannot have
            assert n in (L.DQ_E_UNSUPPORTED, L.DQ_E_INVALID), (preds, n)
            assert n == L.DQ_E_UNSUPPORTED or L.lib.dq_last_error()
            return
        buf = ctypes.create_string_buffer(int(n))
        assert L.lib.dq_plan_explain(*args, buf, n) == n
        text = buf.value.decode()
        assert len(text) == n - 1 and text.startswith("plan: ")
        uses_string = any("s " in p or "s=" in p for p, _ in roots)
        if "--- generated kernel source ---" in text:
            assert pred_pass != 1 and "dq_pred_jit" in text and "__global__" in text
            assert not uses_string
        elif pred_pass == 2:
            raise AssertionError(("compiled pass required but no kernel generated", preds, text))
    finally:
        L.lib.dq_pred_pool_destroy(h)
