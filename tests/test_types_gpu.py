"""Column types beyond DoubleType / LongType / IntegerType / StringType (round 6): FloatType, ShortType, ByteType,
BooleanType, DateType, TimestampType in the fused scan.

Reference: Preconditions.isNumeric accepts ByteType .. DoubleType (analyzers/Analyzer.scala:322-334); the checks'
own tests run isNonNegative / isPositive over every numeric type (checks/CheckTest.scala:478-489, 765-785) and
DataType over a FloatType column (analyzers/AnalyzerTests.scala:322-328) -- those KATs are in
tests/golden/reference_kats.json (test_gpu_parity.test_reference_kats_fused_and_single runs them on the GPU).

Semantics the oracle restates (oracle/dq_oracle.py): values cast to double as Spark's Cast(child, DoubleType)
(exact for every type here), Sum of an integral type = Spark's wrapping LongType sum, min / max with NaN largest,
ApproxCountDistinct with Spark 2.2's per-type XxHash64 (hashInt of floatToIntBits / of the widened byte, short,
days, of 1 / 0 for booleans; hashLong of timestamp micros), comparisons with Spark 2.2's coercions (a FloatType
column against an integer literal compares in float).  The per-type hash mapping is restated from Spark's
published HashExpression (Spark is not vendored in the reference): the XXH64 arithmetic is pinned by the
golden vectors, the mapping itself beyond the KATs above is "parity unpinned".

Tolerances: counts, min / max, compliance counts and HLL words bit-exact; fp64 moments 1e-12 relative.
"""
from __future__ import annotations

import math

import numpy as np
import pytest

from oracle import dq_oracle as O
from tests.helpers import host_column

pytestmark = pytest.mark.gpu

TYPES = ("f32", "i16", "i8", "bool", "date32", "timestamp")
SIZES = [0, 1, 63, 64, 65, 2047, 2049, 16_385, 65_537, 100_003]


@pytest.fixture(scope="module")
def dq():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    import deequ_amd

    return deequ_amd


def _values(dtype, n, rng, special=False):
    if dtype == "f32":
        v = (rng.normal(size=n) * 1000.0).astype(np.float32)
        if special and n:
            k = rng.integers(0, n, max(1, n // 50))
            v[k] = rng.choice(np.array([np.nan, np.inf, -np.inf, -0.0, 0.0, 1e-3, 1e7, 16777217.0], dtype=np.float32),
                              len(k))
        return v
    if dtype == "i16":
        return rng.integers(-32768, 32768, n).astype(np.int16)
    if dtype == "i8":
        return rng.integers(-128, 128, n).astype(np.int8)
    if dtype == "bool":
        return rng.random(n) < 0.3
    if dtype in ("date32", "i32"):
        return rng.integers(-50000, 50000, n).astype(np.int32)
    if dtype == "f64":
        return rng.normal(size=n) * 50.0 + 7.0
    return rng.integers(-(1 << 52), 1 << 52, n)  # timestamp micros (and i64)


def _table(dq, n, seed, null_frac, special=False, extra=()):
    from deequ_amd.table import column_from_numpy

    rng = np.random.default_rng(seed)
    cols, host = [], {}
    for t in TYPES + tuple(extra):
        v = _values(t, n, rng, special)
        valid = rng.random(n) >= null_frac
        cols.append(column_from_numpy(f"c_{t}", t, v, valid))
        host[f"c_{t}"] = O.OColumn(t, v, valid)
    return dq.Table(cols), host


def _profile(dq, schema):
    out = [dq.Size()]
    for name, t, _ in schema:
        out += [dq.Completeness(name), dq.ApproxCountDistinct(name), dq.DataType(name)]
        if t in ("f32", "i16", "i8", "f64", "i64", "i32"):
            out += [dq.Minimum(name), dq.Maximum(name), dq.Mean(name), dq.StandardDeviation(name), dq.Sum(name)]
    return out


def _spec(a):
    name = type(a).__name__
    if name == "Size":
        return ("Size", a.where)
    if name == "Compliance":
        return ("Compliance", a.instance, a.predicate, a.where)
    if name == "Correlation":
        return ("Correlation", a.firstColumn, a.secondColumn, a.where)
    return (name, a.column, a.where)


def _scale(host, a):
    """sum(|x|) over the column's valid finite values: the condition number of a floating-point sum (both sides
    round differently; the tolerance of Sum / Mean is 1e-12 of it)."""
    c = host.get(getattr(a, "column", None))
    if c is None or c.dtype not in ("f32", "f64"):
        return 1.0
    v = np.asarray(c.values, dtype=np.float64)[c.valid]
    v = v[np.isfinite(v)]
    return float(np.abs(v).sum()) + 1.0


def _check(states, analyzers, host, n):
    from tests.test_gpu_parity import assert_state_close

    for a in analyzers:
        ref = O.compute_state(_spec(a), host, n)
        assert_state_close(states[a], ref, scale=_scale(host, a)), a


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("null_frac", [0.0, 0.1, 1.0])
def test_profile_new_types_vs_oracle(dq, n, null_frac):
    from deequ_amd.runner import scan_states

    t, host = _table(dq, n, seed=3 * n + int(10 * null_frac), null_frac=null_frac)
    an = _profile(dq, t.schema)
    _check(scan_states(t, an), an, host, n)


@pytest.mark.parametrize("n", [2049, 65_537])
def test_float_non_finite_and_signed_zero(dq, n):
    """NaN / +-inf / -0.0 / the scientific-notation thresholds in a FloatType column: NaN hashed as
    floatToIntBits' canonical 0x7fc00000, NaN largest in min / max, +-inf in the sum, DataType's FRACTIONAL
    test on the exact float value."""
    from deequ_amd.runner import scan_states

    t, host = _table(dq, n, seed=n, null_frac=0.05, special=True)
    an = [a for a in _profile(dq, t.schema) if getattr(a, "column", "") == "c_f32"]
    _check(scan_states(t, an), an, host, n)


PREDICATES = [
    "c_f32 > 3", "c_f32 >= 16777217", "c_f32 < -2.5", "c_f32 = 0", "COALESCE(c_f32, 0.0) >= 0",
    "COALESCE(c_f32, 1.0) > 0", "COALESCE(c_f32, 5) < 100", "c_f32 > 1e2", "c_i16 > 2.5", "c_i16 <= -100",
    "COALESCE(c_i16, 0.0) >= 0", "c_i8 = 5", "c_i8 != 0", "COALESCE(c_i8, 1.0) > 0", "c_i8 < c_i16",
    "c_f32 < c_i16", "c_f32 >= c_i8", "c_bool", "NOT c_bool", "c_bool = false", "c_bool != true", "c_bool > false",
    "c_bool IS NULL", "c_date32 IS NOT NULL", "c_timestamp IS NULL", "c_bool OR c_i8 > 100",
    "(c_f32 > 0 AND c_bool) OR c_i16 IS NULL",
]


@pytest.mark.parametrize("n", [4097, 40_009])
def test_compliance_new_types_vs_oracle(dq, n):
    from deequ_amd.runner import scan_states

    t, host = _table(dq, n, seed=7 + n, null_frac=0.1)
    # values around 2^24 in the float column: the integer literal rounds to float (16777217 -> 16777216)
    f = host["c_f32"].values
    f[: n // 10] = np.float32(16777216.0)
    from deequ_amd.table import column_from_numpy

    t.columns["c_f32"] = column_from_numpy("c_f32", "f32", f, host["c_f32"].valid)
    an = [dq.Compliance(f"p{k}", p) for k, p in enumerate(PREDICATES)]
    an += [dq.Mean("c_f32", where="c_bool"), dq.Sum("c_i8", where="NOT c_bool"), dq.Size(where="c_i16 > 0"),
           dq.Completeness("c_date32", where="c_bool"), dq.ApproxCountDistinct("c_timestamp", where="c_f32 > 0")]
    _check(scan_states(t, an), an, host, n)
    _check(scan_states(t, an, "interpreter"), an, host, n)


@pytest.mark.parametrize("n", [4099, 100_003])
def test_correlation_new_types_vs_oracle(dq, n):
    """Correlation (Corr casts both children to double) over FloatType / ShortType / ByteType columns, alone and
    beside DoubleType ones, with the pair group's fused moments."""
    from deequ_amd.runner import scan_states

    t, host = _table(dq, n, seed=11 + n, null_frac=0.1, extra=("f64", "i32"))
    cols = ["c_f32", "c_i16", "c_i8", "c_f64", "c_i32"]
    an = [dq.Correlation(a, b) for i, a in enumerate(cols) for b in cols[i + 1:]]
    an += [dq.Mean(c) for c in cols] + [dq.StandardDeviation("c_f32"), dq.Maximum("c_i8"), dq.Sum("c_i16")]
    an += [dq.Correlation("c_f32", "c_i8", where="c_bool")]
    _check(scan_states(t, an), an, host, n)


def test_mixed_profile_chunks_vs_oracle(dq):
    """The new types fused with the existing ones in one AnalysisRunner pass over two chunks (chunk-order merge)."""
    from deequ_amd.table import column_from_numpy, utf8_column

    n, half = 30_011, 14_999
    rng = np.random.default_rng(5)
    data = []
    for t in TYPES + ("f64", "i64", "i32"):
        data.append((f"c_{t}", t, _values(t, n, rng), rng.random(n) >= 0.1))
    strs = [None if rng.random() < 0.1 else b"s%d" % int(rng.integers(0, 500)) for _ in range(n)]

    def chunk(lo, hi):
        cols = [column_from_numpy(name, t, v[lo:hi], m[lo:hi]) for name, t, v, m in data]
        return dq.Table(cols + [utf8_column("s", strs[lo:hi])])

    tables = [chunk(0, half), chunk(half, n)]
    an = _profile(dq, tables[0].schema)
    ctx = dq.AnalysisRunner.onData(tables).addAnalyzers(an).run()
    host = {name: O.OColumn(t, v, m) for name, t, v, m in data}
    host["s"] = O.OColumn("utf8", strs, np.array([x is not None for x in strs]))
    for a in an:
        ref = O.compute_state(_spec(a), host, n, 2)
        m = ctx.metric(a)
        if ref is None:
            assert m.value.isFailure, (a, m)
            continue
        if type(a).__name__ == "DataType":
            from deequ_amd.analyzers import toDistribution

            assert m.value.get() == toDistribution(dq.DataTypeHistogram(*ref.__dict__.values())), a
            continue
        want, got = ref.metricValue(), m.value.get()
        assert got == want or (math.isnan(got) and math.isnan(want)) or abs(got - want) <= 1e-12 * max(1.0, abs(want)), (
            a, got, want)


def test_non_numeric_preconditions(dq):
    """Mean / Maximum / Sum / ApproxQuantile over a BooleanType / DateType / TimestampType column fail their isNumeric
    precondition with the reference's WrongColumnTypeException text."""
    from deequ_amd.metrics import WrongColumnTypeException

    t, _ = _table(dq, 1000, seed=1, null_frac=0.0)
    an = [dq.Mean("c_bool"), dq.Maximum("c_date32"), dq.Sum("c_timestamp"), dq.ApproxQuantile("c_bool", 0.5)]
    ctx = dq.AnalysisRunner.onData(t).addAnalyzers(an).run()
    for a, spark in zip(an, ("BooleanType", "DateType", "TimestampType", "BooleanType")):
        err = ctx.metric(a).value.failed
        assert isinstance(err, WrongColumnTypeException) and f"but found {spark} instead" in str(err), err


def _group_data(n, seed):
    """Low-cardinality columns of the round-6 types (duplicates, NaN / -0.0 / 0.0 in the float column)."""
    rng = np.random.default_rng(seed)
    f = rng.choice(np.array([1.5, -2.25, 0.0, -0.0, np.nan, 3e9, 1e-5, 7.0], dtype=np.float32), n)
    h = rng.integers(-150, 150, n).astype(np.int16)
    c = rng.integers(-128, 128, n).astype(np.int8)
    b = rng.random(n) < 0.3
    d = rng.integers(18000, 18400, n).astype(np.int32)
    ts = rng.choice(np.array([0, 1_600_000_000_123_400, -86_400_000_001, 5_000_000], dtype=np.int64), n)
    out = {}
    for name, t, v in (("f", "f32", f), ("h", "i16", h), ("c", "i8", c), ("b", "bool", b), ("d", "date32", d),
                       ("t", "timestamp", ts)):
        out[name] = (t, v, rng.random(n) >= 0.1)
    return out


@pytest.mark.parametrize("n", [1, 4099, 70_001])
def test_grouping_and_histogram_new_types_vs_oracle(dq, n):
    """Uniqueness / Distinctness / CountDistinct / Entropy / MutualInformation / Histogram over the round-6 types:
    single columns grouped by their exact value (NaN canonical, -0.0 != 0.0), tuples by hash with the exact check;
    Histogram bins = the oracle's CAST-to-string frequencies (timestamps in UTC)."""
    from deequ_amd.table import column_from_numpy
    from tests.helpers import close

    data = _group_data(n, 13 + n)
    t = dq.Table([column_from_numpy(k, ty, v, m) for k, (ty, v, m) in data.items()])
    ocols = {k: O.OColumn(ty, v, m) for k, (ty, v, m) in data.items()}
    an = [dq.Uniqueness("f"), dq.Distinctness("h"), dq.CountDistinct("c"), dq.Entropy("b"), dq.Uniqueness("d"),
          dq.CountDistinct("t"), dq.Uniqueness(["f", "b"]), dq.CountDistinct(["h", "d", "t"]),
          dq.MutualInformation("b", "c"), dq.MutualInformation("f", "t")]
    ctx = dq.AnalysisRunner.onData(t).addAnalyzers(an).run()
    for a in an:
        spec = (type(a).__name__, a.columns[0] if type(a).__name__ == "Entropy" else a.columns)
        ref = O.compute_state(spec, ocols, n)
        m = ctx.metric(a)
        if ref is None:
            assert m.value.isFailure, (a, m)
            continue
        want, got = ref.metricValue(), m.value.get()
        ok = close(got, want, 1e-12, 1e-15) if type(a).__name__ in ("Entropy", "MutualInformation") else got == want
        assert ok, (a, got, want)
    for col in data:
        want = O.histogram(ocols, col, n)
        h = dq.Histogram(col).calculate(t).value.get()
        assert h.numberOfBins == len(want), (col, h.numberOfBins, len(want))
        for k, v in h.values.items():
            assert want[k] == v.absolute, (col, k, v.absolute, want.get(k))


@pytest.mark.parametrize("n", [1, 1000, 100_003])
@pytest.mark.parametrize("dtype", ["f32", "i16", "i8"])
def test_quantiles_new_types_vs_oracle(dq, n, dtype):
    """ApproxQuantile(s) over FloatType / ShortType / ByteType columns (widened exactly on the device, then the
    F64 / I32 select and digest): the exact order statistic of Spark's target rank, over two chunks."""
    from deequ_amd.table import column_from_numpy

    rng = np.random.default_rng(n + len(dtype))
    v = _values(dtype, n, rng, special=(dtype == "f32"))
    valid = rng.random(n) >= 0.1
    cut = n // 2
    chunks = [dq.Table([column_from_numpy("x", dtype, v[:cut], valid[:cut])]),
              dq.Table([column_from_numpy("x", dtype, v[cut:], valid[cut:])])]
    qs = [0.0, 0.1, 0.5, 0.9, 1.0]
    for err in (0.01, 0.0):
        want = O.approx_quantiles_exact(v, valid, qs, err)
        m = dq.ApproxQuantiles("x", qs, err).calculate(chunks)
        if want is None:
            assert m.value.isSuccess and m.value.get() == {}, m
            continue
        from deequ_amd.grouping import _java_double_to_string

        got = m.value.get()
        for q, w in zip(qs, want):
            g = got[_java_double_to_string(q)]
            assert g == w or (math.isnan(g) and math.isnan(w)), (dtype, n, err, q, g, w)
        single = dq.ApproxQuantile("x", 0.5, err).calculate(chunks).value.get()
        w = want[qs.index(0.5)]
        assert single == w or (math.isnan(single) and math.isnan(w))


NARROW_PREDICATES = [
    "c_f32 > 3", "c_f32 >= 16777217", "COALESCE(c_f32, 0.0) >= 0", "c_f32 < c_i16", "c_i16 > 2.5",
    "COALESCE(c_i16, 1.0) > 0", "c_i8 = 5", "c_i8 < c_i16", "c_i8 IS NULL OR c_f32 > 1e2", "NOT (c_i8 > 0)",
]


@pytest.mark.parametrize("n", [4097, 70_001])
def test_compiled_predicate_pass_narrow_types(dq, n):
    """The predicate kernel generated and compiled for a program over FloatType / ShortType / ByteType columns
    (4- / 2- / 1-byte loads, float widened exactly): DQ_PRED_PASS_COMPILED takes it, and its counters and `where`
    bitmaps equal the interpreter's and the oracle's."""
    from deequ_amd.runner import ScanPlan, scan_states

    t, host = _table(dq, n, seed=29 + n, null_frac=0.1)
    f = host["c_f32"].values
    f[: n // 10] = np.float32(16777216.0)
    from deequ_amd.table import column_from_numpy

    t.columns["c_f32"] = column_from_numpy("c_f32", "f32", f, host["c_f32"].valid)
    an = [dq.Compliance(f"q{k}", p) for k, p in enumerate(NARROW_PREDICATES)]
    an += [dq.Sum("c_i16", where="c_f32 > 0")]
    plan = ScanPlan(an, t.schema, pred_pass="compiled")
    ok, note = plan.pred_compiled()
    plan.close()
    assert ok, note
    comp = scan_states(t, an, "compiled")
    _check(comp, an, host, n)
    interp = scan_states(t, an, "interpreter")
    for a in an:
        assert comp[a] == interp[a], a
