"""The drop-in boundary on the CPU: libdqscan.so loads, exports every symbol include/dqscan.h
declares, and its host-side state algebra (no device needed) equals the oracle's."""
from __future__ import annotations

import ctypes
import math
import os
import re

import numpy as np
import pytest

from oracle import dq_oracle as O
from tests.conftest import ROOT


@pytest.fixture(scope="module")
def dq():
    import deequ_amd

    return deequ_amd


def test_header_symbols_exported(dq):
    from deequ_amd import _lib as L

    hdr = open(os.path.join(ROOT, "include", "dqscan.h")).read()
    declared = set(re.findall(r"^\s*(?:dq_status|int32_t|int64_t|void|const char\* const\*|const char\*|const dq_\w+\*)"
                              r"\s+(dq_\w+)\s*\(", hdr, re.M))
    assert len(declared) >= 18
    for name in declared:
        assert hasattr(L.lib, name), name
    assert declared == set(L.EXPORTED)
    assert L.lib.dq_abi_version() == L.ABI_VERSION == 6


def test_struct_layouts(dq):
    from deequ_amd import _lib as L

    assert ctypes.sizeof(L.State) == 4 + 2 + 2 + 416
    assert ctypes.sizeof(L.PredNode) == 32
    assert ctypes.sizeof(L.ColumnView) == 32
    assert ctypes.sizeof(L.AnalyzerSpec) == 20


def _py(state):
    from deequ_amd import states as S

    m = {O.NumMatches: lambda s: S.NumMatches(s.numMatches),
         O.NumMatchesAndCount: lambda s: S.NumMatchesAndCount(s.numMatches, s.count),
         O.SumState: lambda s: S.SumState(s.sum_), O.MeanState: lambda s: S.MeanState(s.sum_, s.count),
         O.StandardDeviationState: lambda s: S.StandardDeviationState(s.n, s.avg, s.m2),
         O.MinState: lambda s: S.MinState(s.minValue), O.MaxState: lambda s: S.MaxState(s.maxValue),
         O.CorrelationState: lambda s: S.CorrelationState(s.n, s.xAvg, s.yAvg, s.ck, s.xMk, s.yMk),
         O.ApproxCountDistinctState: lambda s: S.ApproxCountDistinctState(tuple(s.words)),
         O.DataTypeHistogram: lambda s: S.DataTypeHistogram(*s.__dict__.values())}
    return m[type(state)](state)


def _rand_states(rng):
    words = lambda: tuple(O.registers_to_words(rng.integers(0, 20, 512).tolist()))
    return [
        (O.NumMatches(int(rng.integers(0, 1 << 40))), O.NumMatches(int(rng.integers(0, 1 << 40)))),
        (O.NumMatchesAndCount(3, 9), O.NumMatchesAndCount(5, 11)),
        (O.SumState(float(rng.normal())), O.SumState(float(rng.normal()))),
        (O.MeanState(float(rng.normal()), 4), O.MeanState(float(rng.normal()), 7)),
        (O.StandardDeviationState(5.0, 1.25, 3.5), O.StandardDeviationState(7.0, -2.0, 10.25)),
        (O.MinState(float(rng.normal())), O.MinState(float("nan"))),
        (O.MinState(-0.0), O.MinState(0.0)),
        (O.MaxState(0.0), O.MaxState(-0.0)),
        (O.MaxState(float(rng.normal())), O.MaxState(float(rng.normal()))),
        (O.CorrelationState(10.0, 1.0, 2.0, 3.0, 4.0, 5.0), O.CorrelationState(3.0, -1.0, 0.5, 0.25, 1.0, 2.0)),
        (O.ApproxCountDistinctState(words()), O.ApproxCountDistinctState(words())),
        (O.DataTypeHistogram(*rng.integers(0, 1 << 40, 5).tolist()), O.DataTypeHistogram(0, 1, 2, 3, 4)),
    ]


def _same(a, b):
    for x, y in zip(a.__dict__.values(), b.__dict__.values()):
        if isinstance(x, float):
            assert (math.isnan(x) and math.isnan(y)) or (x == y and math.copysign(1, x) == math.copysign(1, y)), (a, b)
        else:
            assert tuple(x) == tuple(y) if isinstance(x, tuple) else x == y


def test_state_sum_equals_oracle(dq):
    rng = np.random.default_rng(7)
    for a, b in _rand_states(rng):
        ref = a.sum(b)
        got = _py(a).sum(_py(b))
        _same(got, ref)
        if isinstance(ref, O.DataTypeHistogram):
            continue
        va, vb = ref.metricValue(), got.metricValue()
        assert (math.isnan(va) and math.isnan(vb)) or va == vb


def test_option_merge_semantics(dq):
    from deequ_amd.analyzers import merge

    s = dq.NumMatches(4)
    assert merge(None, s) == s and merge(s, None) == s and merge(None, None) is None
    assert merge(s, s, None, s) == dq.NumMatches(12)


def test_hll_estimate_equals_oracle(dq):
    from deequ_amd.states import hll_estimate

    rng = np.random.default_rng(3)
    for d in (0, 1, 5, 50, 399, 401, 1000, 2500, 10_000, 1_000_000):
        regs = O.np_hll_registers(O.np_xxh64_long(rng.integers(0, 1 << 62, d)))
        w = O.registers_to_words(regs.tolist())
        assert hll_estimate(w) == O.hll_count(w), d
    for m in (31, 32, 40, 56, 63):  # JVM Int shift quirk
        regs = [3] * 512
        regs[100] = m
        w = O.registers_to_words(regs)
        assert hll_estimate(w) == O.hll_count(w), m


def test_state_bytes_roundtrip_and_format(dq):
    from deequ_amd import _lib as L
    from deequ_amd.states import state_from_c, state_to_c

    rng = np.random.default_rng(5)
    ops = {O.NumMatches: L.OP_SIZE, O.NumMatchesAndCount: L.OP_COMPLIANCE, O.SumState: L.OP_SUM,
           O.MeanState: L.OP_MEAN, O.StandardDeviationState: L.OP_STDDEV, O.MinState: L.OP_MIN,
           O.MaxState: L.OP_MAX, O.CorrelationState: L.OP_CORRELATION,
           O.ApproxCountDistinctState: L.OP_APPROX_COUNT_DISTINCT, O.DataTypeHistogram: L.OP_DATATYPE}
    for a, _ in _rand_states(rng):
        op = ops[type(a)]
        c = state_to_c(_py(a), op)
        n = L.lib.dq_state_to_bytes(ctypes.byref(c), None, 0)
        buf = (ctypes.c_uint8 * n)()
        assert L.lib.dq_state_to_bytes(ctypes.byref(c), buf, n) == n
        assert bytes(buf) == O.state_to_bytes(a), type(a)
        back = L.State()
        L.check(L.lib.dq_state_from_bytes(op, bytes(buf), n, ctypes.byref(back)))
        _same(state_from_c(back), _py(a))
    bad = L.State()
    assert L.lib.dq_state_from_bytes(L.OP_SIZE, b"\0" * 7, 7, ctypes.byref(bad)) == L.DQ_E_STATE


def test_identifier_is_scala_murmur3(dq):
    from deequ_amd.state_provider import identifier

    for a in (dq.Size(), dq.Completeness("att1"), dq.Compliance("rule1", "att1 > 3", "att2 < 4"),
              dq.Correlation("a", "b"), dq.Mean("numericCol"), dq.ApproxCountDistinct("ü名"),
              dq.Completeness("att1", "item IN ('1', '2')"), dq.DataType("item")):
        assert int(identifier(a)) == O.murmur3_string_hash(str(a)), str(a)


def test_analyzer_tostring_and_equality(dq):
    # NullHandlingTests.scala:126-133 pins `Mean(numericCol,None)`
    assert str(dq.Mean("numericCol")) == "Mean(numericCol,None)"
    assert str(dq.Completeness("att1", "item IN ('1', '2')")) == "Completeness(att1,Some(item IN ('1', '2')))"
    assert str(dq.Compliance("rule1", "att1 > 3")) == "Compliance(rule1,att1 > 3,None)"
    assert dq.Size() == dq.Size() and len({dq.Size(), dq.Size(), dq.Size("x > 1")}) == 2


class _CPool:
    """dq_pred_pool_* straight through ctypes (what a JNI / cgo shim binds)."""

    def __init__(self, L, cols):
        names = (ctypes.c_char_p * len(cols))(*[n.encode() for n, _ in cols])
        types = (ctypes.c_int32 * len(cols))(*[t for _, t in cols])
        self.L, self.h = L, ctypes.c_void_p()
        assert L.lib.dq_pred_pool_create(names, types, len(cols), ctypes.byref(self.h)) == L.DQ_OK

    def add(self, text):
        r = ctypes.c_int32(-7)
        st = self.L.lib.dq_pred_pool_add(self.h, text.encode(), ctypes.byref(r))
        return st, r.value

    def nodes(self):
        n = self.L.lib.dq_pred_pool_size(self.h)
        p = self.L.lib.dq_pred_pool_nodes(self.h)
        return [(p[i].kind, p[i].a, p[i].b, p[i].cmp, p[i].i64, p[i].f64) for i in range(n)]

    def patterns(self):
        n = self.L.lib.dq_pred_pool_num_patterns(self.h)
        p = self.L.lib.dq_pred_pool_patterns(self.h)
        return [p[i].decode() for i in range(n)]

    def close(self):
        self.L.lib.dq_pred_pool_destroy(self.h)


def test_predicate_compiler_c_abi(dq):
    """dq_pred_pool_add: the Spark 2.2 literal typing and the grammar's routing decisions, via ctypes."""
    from deequ_amd import _lib as L

    P = _CPool(L, [("a", L.TYPE_F64), ("b", L.TYPE_I64), ("s", L.TYPE_UTF8)])
    st, r = P.add("`a` IS NULL OR (`a` >= 0.0 AND `a` <= 7.5)")
    nodes = P.nodes()
    assert st == L.DQ_OK and nodes[r][0] == L.PRED_OR
    dec = [n for n in nodes if n[0] == L.PRED_LIT_DECIMAL]
    assert [(d[4], d[3]) for d in dec] == [(0, 1), (75, 1)]  # 0.0 = 0 / 10^1, 7.5 = 75 / 10^1
    st, r = P.add("COALESCE(b, 1.0) > 0 AND a > -1.5e2 AND NOT b <> 3")
    nodes = P.nodes()
    assert st == L.DQ_OK
    assert [n[5] for n in nodes if n[0] == L.PRED_LIT_DOUBLE] == [-150.0]
    assert [n[4] for n in nodes if n[0] == L.PRED_LIT_INT] == [0, 3]
    assert any(n[0] == L.PRED_COALESCE for n in nodes) and any(n[3] == L.CMP_NE for n in nodes if n[0] == L.PRED_CMP)
    # 64-bit literal bounds (Spark: a literal beyond Long is a decimal / fails; the GPU takes int64 only)
    for text, want in (("b > 9223372036854775807", (1 << 63) - 1), ("b > -9223372036854775808", -(1 << 63))):
        st, r = P.add(text)
        assert st == L.DQ_OK and P.nodes()[P.nodes()[r][2]][4] == want
    # string equality / IN on the string column: one whole-value DFA node, literals escaped
    st, r = P.add("s IN ('a.b', 'c') OR s = 'd' OR s NOT IN ('e')")
    assert st == L.DQ_OK
    assert P.patterns() == [r"(?:a\.b|c)", "(?:d)", "(?:e)"]
    regex = [n for n in P.nodes() if n[0] == L.PRED_REGEX]
    assert len(regex) == 3 and all(n[3] == L.REGEX_FULL for n in regex)
    # outside the grammar: DQ_E_UNSUPPORTED, pool unchanged
    size = L.lib.dq_pred_pool_size(P.h)
    for bad in ("a IN (1, 2)", "a = 'x'", "abs(a) > 1", "a LIKE 'x%'", "1.0D > a", "s > 'x'", "s > 1",
                "COALESCE(s, 0) > 1", "a BETWEEN 1 AND 2", "'x' = 'y'", "a > 1e", "a > 1.2.3", "s = 'it\\'s'",
                "a > 9223372036854775808", "a > 0.1234567890123456789", "COALESCE(a, 1, 2) > 0", "a >", "(a > 1"):
        st, _ = P.add(bad)
        assert st == L.DQ_E_UNSUPPORTED, bad
        assert L.lib.dq_last_error(), bad
        assert L.lib.dq_pred_pool_size(P.h) == size, bad
    st, _ = P.add("zz > 1")
    assert st == L.DQ_E_INVALID and L.lib.dq_last_error() == b"no such column: zz"
    P.close()


def test_predicate_pool_python_mapping(dq):
    """The host wrapper re-indexes the C pool's table columns to plan columns (first reference order)."""
    from deequ_amd import _lib as L
    from deequ_amd.analyzers import PlanBuilder
    from deequ_amd.predicates import UnsupportedPredicate

    b = PlanBuilder([("x", "f64", True), ("y", "i64", False), ("t", "utf8", True)])
    r = b.pool.add("y > 2 AND x IS NOT NULL")
    assert b.columns == ["y", "x"]
    cols = [n[1] for n in b.pool.nodes if n[0] == L.PRED_COLUMN]
    assert cols == [0, 1] and b.pool.nodes[r][0] == L.PRED_AND
    b.pool.add("t = 'q'")
    assert b.columns == ["y", "x", "t"] and b.pool.patterns == ["(?:q)"]
    with pytest.raises(UnsupportedPredicate):
        b.pool.add("t > 'q'")
    with pytest.raises(KeyError):
        b.pool.add("zz > 1")


def test_plan_create_without_gpu_reports_error(dq):
    """On a host without a GPU the scan fails loudly (no CPU fallback)."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from deequ_amd import _lib as L

    specs = (L.AnalyzerSpec * 1)()
    specs[0].op, specs[0].col_a, specs[0].col_b, specs[0].pred_root, specs[0].where_root = L.OP_SIZE, -1, -1, -1, -1
    sch = (L.ColumnDesc * 1)()
    h = ctypes.c_void_p()
    rc = L.lib.dq_plan_create(specs, 1, sch, 0, None, 0, 0, ctypes.byref(h))
    assert rc != L.DQ_OK and L.lib.dq_last_error()


def test_combine_integral_with_double_partials(dq):
    """dq_state_combine of Sum / Mean slot sets: two fresh integral partials add as wrapping int64 (Spark's
    LongType partial buffers); a partial that is already a double (deserialized, or Analyzers.merge-d with a
    loaded state) combines with a fresh integral one by double addition instead of failing."""
    import ctypes

    from deequ_amd import _lib as L

    def mk(op, integral, partial, sum_, count=0):
        s = L.State()
        s.op = op
        s.has_value[0] = s.has_value[1] = 1
        s.integral = integral
        if op == L.OP_SUM:
            s.u.sum.sum, s.u.sum.partial = sum_, partial
        else:
            s.u.mean.sum, s.u.mean.partial, s.u.mean.count = sum_, partial, count
        return s

    big = (1 << 63) - 5
    for op in (L.OP_SUM, L.OP_MEAN):
        out = L.State()
        # two integral partials: the int64 sum wraps before the cast (Spark), not the doubles
        L.check(L.lib.dq_state_combine(ctypes.byref(mk(op, 1, big, float(big), 1)), ctypes.byref(mk(op, 1, 10, 10.0, 2)),
                                       ctypes.byref(out)))
        u = out.u.sum if op == L.OP_SUM else out.u.mean
        assert out.integral == 1 and u.partial == big + 10 - (1 << 64) and u.sum == float(big + 10 - (1 << 64))
        # integral + double (either order): double addition, the result is a double partial
        for a, b in ((mk(op, 1, 7, 7.0, 1), mk(op, 0, 0, 2.5, 1)), (mk(op, 0, 0, 2.5, 1), mk(op, 1, 7, 7.0, 1))):
            L.check(L.lib.dq_state_combine(ctypes.byref(a), ctypes.byref(b), ctypes.byref(out)))
            u = out.u.sum if op == L.OP_SUM else out.u.mean
            assert out.integral == 0 and u.sum == 9.5
            if op == L.OP_MEAN:
                assert out.u.mean.count == 2
        # a NULL side takes the other's partial and kind
        a = mk(op, 1, 4, 4.0, 1)
        nul = mk(op, 0, 0, 0.0, 0)
        nul.has_value[0] = 0
        L.check(L.lib.dq_state_combine(ctypes.byref(nul), ctypes.byref(a), ctypes.byref(out)))
        assert out.integral == 1 and (out.u.sum if op == L.OP_SUM else out.u.mean).partial == 4


def test_combine_decimal_partials(dq):
    """Sum / Mean states of a DecimalType column (integral = 2): row shards' exact 128-bit partials add before the
    cast (Spark's DecimalType partial buffers), the result is Decimal.toDouble of the exact sum, and a sum reaching
    10^dec_digits (Spark's sum-type overflow: NULL) leaves the state undefined -- host-only state algebra."""
    import ctypes
    from fractions import Fraction

    from deequ_amd import _lib as L

    mask = (1 << 64) - 1

    def mk(op, u, scale, digits, count=1):
        s = L.State()
        s.op = op
        s.has_value[0] = s.has_value[1] = 1
        s.integral = 2
        x = s.u.sum if op == L.OP_SUM else s.u.mean
        x.partial = ctypes.c_int64(u & mask).value
        x.partial_hi = ctypes.c_int64((u >> 64) & mask).value
        x.guard = float(Fraction(u, 10 ** scale))
        x.dec_scale, x.dec_digits = scale, digits
        x.sum = float(Fraction(u, 10 ** scale))
        if op == L.OP_MEAN:
            x.count = count
        return s

    rng = __import__("random").Random(6)
    for op in (L.OP_SUM, L.OP_MEAN):
        for _ in range(200):
            scale = rng.randint(0, 38)
            a, b = rng.randint(-(10 ** 37), 10 ** 37), rng.randint(-(10 ** 37), 10 ** 37)
            out = L.State()
            L.check(L.lib.dq_state_combine(ctypes.byref(mk(op, a, scale, 38)), ctypes.byref(mk(op, b, scale, 38)),
                                           ctypes.byref(out)))
            x = out.u.sum if op == L.OP_SUM else out.u.mean
            assert out.integral == 2 and ((x.partial_hi & mask) << 64 | (x.partial & mask)) == (a + b) & ((1 << 128) - 1)
            assert L.lib.dq_state_is_defined(ctypes.byref(out)) == 1
            assert x.sum == float(Fraction(a + b, 10 ** scale)), (a, b, scale)  # exact sum, one rounding
        # past the sum type's precision: Spark's NULL -> undefined; DecimalType(5, 2)'s sum type holds 15 digits
        out = L.State()
        L.check(L.lib.dq_state_combine(ctypes.byref(mk(op, 6 * 10 ** 37, 0, 38)), ctypes.byref(mk(op, 5 * 10 ** 37, 0, 38)),
                                       ctypes.byref(out)))
        assert L.lib.dq_state_is_defined(ctypes.byref(out)) == 0
        L.check(L.lib.dq_state_combine(ctypes.byref(mk(op, 6 * 10 ** 14, 2, 15)), ctypes.byref(mk(op, 4 * 10 ** 14, 2, 15)),
                                       ctypes.byref(out)))
        assert L.lib.dq_state_is_defined(ctypes.byref(out)) == 0
        L.check(L.lib.dq_state_combine(ctypes.byref(mk(op, 6 * 10 ** 14, 2, 15)), ctypes.byref(mk(op, -4 * 10 ** 14, 2, 15)),
                                       ctypes.byref(out)))
        assert L.lib.dq_state_is_defined(ctypes.byref(out)) == 1
        assert (out.u.sum if op == L.OP_SUM else out.u.mean).sum == 2e12
