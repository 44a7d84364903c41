"""DecimalType columns (Arrow decimal128, precision 1..38) in the fused scan, the predicate pass and the quantile
passes, against the oracle.

Reference: Preconditions.isNumeric accepts DecimalType (analyzers/Analyzer.scala:322-334); AnalyzerTests.scala:489-505
runs Minimum over a DecimalType.SYSTEM_DEFAULT = DecimalType(38, 18) column (in tests/golden/reference_kats.json,
run on the GPU by test_gpu_parity.test_reference_kats_fused_and_single); checks/ApplicabilityTest.scala:178-190 runs
Minimum / Maximum over DecimalType(38, 18), (5, 2) and (8, 4) columns.

Semantics restated by the oracle (oracle/dq_oracle.py, Spark 2.2 + java.math.BigDecimal): every numeric analyzer sees
Cast(child, DoubleType) = Decimal.toDouble, the correctly rounded double (Minimum / Maximum: min / max of the exact
decimals, cast -- the same double); Sum / Mean: the exact decimal sum in DecimalType(min(38, p + 10), s), NULL past
that precision, cast at the end; ApproxCountDistinct: hashLong of the unscaled long (p <= 18) or hashUnsafeBytes of
BigInteger.toByteArray (p > 18); DataType: the class of BigDecimal.toString ("0E-18" and "1.5E-7" are STRINGs);
comparisons with integer / decimal literals exact (DecimalPrecision's wider decimal type).  The decimal hash mapping
and the toString forms are restated from Spark / the JDK (neither is vendored in the reference): "parity unpinned"
beyond the KAT above.  Tolerances: counts, min / max, sums and HLL words bit-exact; moments 1e-12 relative.
"""
from __future__ import annotations

import math

import numpy as np
import pytest

from oracle import dq_oracle as O

pytestmark = pytest.mark.gpu

DECIMALS = [(5, 2), (8, 4), (18, 0), (18, 6), (19, 4), (28, 10), (38, 0), (38, 18), (38, 38)]


@pytest.fixture(scope="module")
def dq():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    import deequ_amd

    return deequ_amd


def dec_values(p: int, s: int, n: int, rng) -> list:
    """unscaled values of DecimalType(p, s): random digit counts 1..p, zeros, extremes (+-(10^p - 1)), values whose
    BigDecimal.toString is scientific (|u| < 10^(s - 6)), and for p >= 17 exact double-rounding ties."""
    out = []
    top = 10 ** p - 1
    for _ in range(n):
        r = rng.random()
        if r < 0.05:
            u = 0
        elif r < 0.08:
            u = top
        elif r < 0.14 and s > 6:
            u = int(rng.integers(1, 10 ** min(s - 6, 18)))
        elif r < 0.16 and p >= 17:
            u = 90071992547409925 * 10 ** (p - 17) if p - 17 <= s else 90071992547409925  # 2^53 + 0.5 (a tie)
        else:
            d = int(rng.integers(1, p + 1))
            u = int(rng.integers(0, 10 ** min(d, 18))) * 10 ** max(0, d - 18) + int(rng.integers(0, 10 ** max(0, min(d - 18, 18)) or 1))
        u = min(u, top)
        out.append(-u if rng.random() < 0.45 else u)
    return out


def _table(dq, n, seed, null_frac, decimals=DECIMALS):
    from deequ_amd.table import column_from_numpy

    rng = np.random.default_rng(seed)
    cols, host = [], {}
    for p, s in decimals:
        name, dt = f"d{p}_{s}", f"decimal({p},{s})"
        v = dec_values(p, s, n, rng)
        valid = rng.random(n) >= null_frac
        cols.append(column_from_numpy(name, dt, v, valid))
        host[name] = O.OColumn(dt, v, valid)
    iv = rng.integers(-1000, 1000, n)
    ivalid = rng.random(n) >= 0.1
    cols.append(column_from_numpy("i", "i64", iv, ivalid))
    host["i"] = O.OColumn("i64", iv, ivalid)
    return dq.Table(cols), host


def _spec(a):
    name = type(a).__name__
    if name == "Size":
        return ("Size", a.where)
    if name == "Compliance":
        return ("Compliance", a.instance, a.predicate, a.where)
    return (name, a.column, a.where)


def _check(states, analyzers, host, n):
    from tests.test_gpu_parity import assert_state_close

    for a in analyzers:
        ref = O.compute_state(_spec(a), host, n)
        c = host.get(getattr(a, "column", None))
        scale = 1.0
        if c is not None and O.decimal_ps(c.dtype):
            scale = float(sum(abs(x) for x in O._as_double_list(c))) + 1.0
        assert_state_close(states[a], ref, scale=scale), a


def _profile(dq, names):
    out = [dq.Size()]
    for name in names:
        out += [dq.Completeness(name), dq.ApproxCountDistinct(name), dq.DataType(name), dq.Minimum(name),
                dq.Maximum(name), dq.Mean(name), dq.StandardDeviation(name), dq.Sum(name)]
    return out


@pytest.mark.parametrize("n", [0, 1, 63, 65, 2049, 16_385])
@pytest.mark.parametrize("null_frac", [0.0, 0.1, 1.0])
def test_decimal_profile_vs_oracle(dq, n, null_frac):
    from deequ_amd.runner import scan_states

    t, host = _table(dq, n, seed=7 * n + int(10 * null_frac), null_frac=null_frac)
    an = _profile(dq, [f"d{p}_{s}" for p, s in DECIMALS])
    _check(scan_states(t, an), an, host, n)


def test_decimal_profile_large(dq):
    """100 003 rows of DecimalType(38, 18) and (18, 6), fused with an int64 column's profile, `where`-filtered."""
    from deequ_amd.runner import scan_states

    n = 100_003
    t, host = _table(dq, n, seed=1, null_frac=0.1, decimals=[(38, 18), (18, 6)])
    an = _profile(dq, ["d38_18", "d18_6", "i"])
    an += [dq.Sum("d38_18", where="i > 0"), dq.Minimum("d18_6", where="d38_18 > 0"), dq.Mean("i", where="d18_6 < 0")]
    _check(scan_states(t, an), an, host, n)


def test_decimal_sum_overflow_is_null(dq):
    """Sum of a DecimalType(38, 0) column past 10^38 is Spark 2.2's NULL (sum type DecimalType(38, 0)): no state,
    EmptyStateException; a DecimalType(5, 2) sum past 10^15 (DecimalType(15, 2)) likewise; below the bound exact."""
    from deequ_amd.metrics import EmptyStateException
    from deequ_amd.table import column_from_numpy

    big = [10 ** 37 * 9] * 12  # 1.08e39
    small = [5 * 10 ** 37, 4 * 10 ** 37, -3 * 10 ** 37] * 4  # 2.4e38 overall: past 10^38 as well
    t = dq.Table([column_from_numpy("a", "decimal(38,0)", big, np.ones(12, bool)),
                  column_from_numpy("b", "decimal(38,0)", small[:3] + [0] * 9, np.ones(12, bool)),
                  column_from_numpy("c", "decimal(38,0)", small, np.ones(12, bool))])
    for col, want in (("a", None), ("b", 6e37), ("c", None)):
        for a in (dq.Sum(col), dq.Mean(col)):
            m = a.calculate(t)
            if want is None:
                assert m.value.isFailure and isinstance(m.value.failed, EmptyStateException), (a, m)
            else:
                assert m.value.get() == (want if type(a).__name__ == "Sum" else want / 12), (a, m)
    v = [99999] * 100_000  # 999.99 x 1e5: unscaled 9.9999e9 < 10^15 (the sum type DecimalType(15, 2))
    assert dq.Sum("x").calculate(dq.Table([column_from_numpy("x", "decimal(5,2)", v, None)])).value.get() == 99999000.0


DEC_PREDICATES = [
    "d5_2 >= 0", "d5_2 < 12.345", "d5_2 = 1.5", "d5_2 != 0", "COALESCE(d5_2, 0) > 1", "d5_2 <= -999.99",
    "d18_6 <= -1.25", "d18_6 > 123456789", "d18_6 = 0.000001", "d18_6 >= 9999999999999", "d18_6 < 5000000000",
    "d38_18 >= 100", "d38_18 < 99.5", "d38_18 = 123.45", "d38_18 != 0", "d38_18 > -1234567890123456789",
    "d38_18 <= 0.000000000000000001", "COALESCE(d38_18, 1) >= 0", "COALESCE(d38_18, -1.5) < 0", "d38_18 IS NULL",
    "d38_0 < 5000000000", "d38_0 >= -99999999999999999", "d38_0 = 0", "d19_4 > 123.45678", "d19_4 <= -0.0001",
    "d38_18 IS NOT NULL AND d5_2 > 0", "NOT (d38_18 <= 0)", "d5_2 > 1 OR d38_18 < 0", "i > 0 AND d18_6 < 0",
]


@pytest.mark.parametrize("n", [4097, 30_011])
def test_decimal_compliance_vs_oracle(dq, n):
    """Comparisons of decimal columns with integer / decimal literals (exact bounds on the unscaled value; above
    precision 18 as atoms on the high and low words), COALESCE fallbacks, NULLs, `where` filters."""
    from deequ_amd.runner import scan_states
    from deequ_amd.table import column_from_numpy

    t, host = _table(dq, n, seed=13 + n, null_frac=0.1, decimals=[(5, 2), (18, 6), (38, 18), (38, 0), (19, 4)])
    # values sitting on the literals and one unit either side
    rng = np.random.default_rng(n)
    near = {"d5_2": [150, 149, 151, 1234, 1235, 0, 99999, -99999], "d18_6": [-1250000, -1250001, 1, 0, 2],
            "d38_18": [100 * 10 ** 18, 100 * 10 ** 18 - 1, 995 * 10 ** 17, 12345 * 10 ** 16, 1, 0, -1,
                       -1234567890123456789 * 10 ** 18, -1234567890123456789 * 10 ** 18 + 1],
            "d38_0": [5000000000, 4999999999, -99999999999999999, 0], "d19_4": [1234568, 1234567, -1, 0]}
    for name, vals in near.items():
        c = host[name]
        for k in range(n // 20):
            c.values[int(rng.integers(0, n))] = vals[k % len(vals)]
        t.columns[name] = column_from_numpy(name, c.dtype, c.values, c.valid)
    an = [dq.Compliance(f"p{k}", p) for k, p in enumerate(DEC_PREDICATES)]
    an += [dq.Mean("i", where="d38_18 > 0"), dq.Completeness("d5_2", where="d18_6 IS NOT NULL")]
    _check(scan_states(t, an), an, host, n)


def test_decimal_unsupported_routes(dq):
    """What stays on the fallback: a decimal compared with a double literal or a column, a literal whose wider
    decimal type exceeds 38 digits (DecimalType(38, 30) vs an int: 10 + 30 digits)."""
    from deequ_amd.metrics import UnsupportedOnGpuPathException

    t, _ = _table(dq, 1000, seed=2, null_frac=0.1, decimals=[(38, 18), (5, 2), (38, 30)])
    an = [dq.Compliance("dbl", "d38_18 > 1e0"), dq.Compliance("cols", "d5_2 < d38_18"),
          dq.Compliance("wide", "d38_30 > 1"), dq.Compliance("ok", "d38_18 > 1")]
    ctx = dq.AnalysisRunner.onData(t).addAnalyzers(an).run()
    for a in an[:-1]:
        m = ctx.metric(a)
        assert m.value.isFailure and isinstance(m.value.failed, UnsupportedOnGpuPathException), (a, m)
    assert ctx.metric(an[-1]).value.isSuccess


@pytest.mark.parametrize("n", [2, 4099, 100_003])
def test_decimal_correlation_vs_oracle(dq, n):
    """Correlation over decimal columns (Corr's inputs are the casts: each value converted as it is loaded by the
    pair pass), beside int64 columns, with a `where`; the same columns' Mean / Sum stay exact in the column pass."""
    from deequ_amd.runner import scan_states

    t, host = _table(dq, n, seed=17 + n, null_frac=0.1, decimals=[(38, 18), (18, 6), (5, 2), (28, 10)])
    cols = ["d38_18", "d18_6", "d5_2", "d28_10", "i"]
    an = [dq.Correlation(a, b) for k, a in enumerate(cols) for b in cols[k + 1:]]
    an += [dq.Correlation("d5_2", "d18_6", where="i > 0"), dq.Mean("d5_2"), dq.Sum("d38_18"), dq.StandardDeviation("d18_6")]
    states = scan_states(t, an)
    from tests.test_gpu_parity import assert_state_close

    for a in an:
        if type(a).__name__ == "Correlation":
            ref = O.compute_state(("Correlation", a.firstColumn, a.secondColumn, a.where), host, n)
            assert_state_close(states[a], ref), a
    _check(states, an[-3:], host, n)


@pytest.mark.parametrize("n", [1, 4099, 70_001])
def test_decimal_grouping_and_histogram_vs_oracle(dq, n):
    """Uniqueness / Distinctness / CountDistinct / Entropy / MutualInformation / Histogram over decimal columns:
    grouped by their exact unscaled value (hashed, checked word by word), Histogram bins rendered as
    BigDecimal.toString ("0E-18", "-1.5E-7", "123.450000000000000000")."""
    from deequ_amd.table import column_from_numpy
    from tests.helpers import close

    rng = np.random.default_rng(n + 3)
    pools = {"a": ("decimal(38,18)", [0, 123450000000000000000, -15 * 10 ** 10, 1, -(10 ** 38 - 1), 99 * 10 ** 18,
                                      2 ** 70, -(2 ** 64)]),
             "b": ("decimal(5,2)", [0, 150, -150, 99999, 5, -1]),
             "c": ("decimal(20,0)", [0, 10 ** 19, -(10 ** 19) + 7, 2 ** 63, -(2 ** 63) - 1, 42])}
    data = {k: (t, [int(x) for x in rng.choice(np.array(pool, dtype=object), n)], rng.random(n) >= 0.1)
            for k, (t, pool) in pools.items()}
    t = dq.Table([column_from_numpy(k, ty, v, m) for k, (ty, v, m) in data.items()])
    ocols = {k: O.OColumn(ty, v, m) for k, (ty, v, m) in data.items()}
    an = [dq.Uniqueness("a"), dq.Distinctness("b"), dq.CountDistinct("c"), dq.Entropy("a"),
          dq.Uniqueness(["a", "b"]), dq.CountDistinct(["b", "c"]), dq.MutualInformation("a", "c")]
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
@pytest.mark.parametrize("ps", [(5, 2), (38, 18)])
def test_decimal_quantiles_vs_oracle(dq, n, ps):
    """ApproxQuantile(s) of a decimal column: each value cast to double on the device (Decimal.toDouble), then the
    F64 select / digest -- the exact order statistic of Spark's target rank over the casts, two chunks."""
    from deequ_amd.grouping import _java_double_to_string
    from deequ_amd.table import column_from_numpy

    p, s = ps
    rng = np.random.default_rng(n + p)
    v = dec_values(p, s, n, rng)
    valid = rng.random(n) >= 0.1
    dt = f"decimal({p},{s})"
    cut = n // 2
    chunks = [dq.Table([column_from_numpy("x", dt, v[:cut], valid[:cut])]),
              dq.Table([column_from_numpy("x", dt, v[cut:], valid[cut:])])]
    x = np.array(O._as_double_list(O.OColumn(dt, v, valid)), dtype=np.float64)
    qs = [0.0, 0.1, 0.5, 0.9, 1.0]
    for err in (0.01, 0.0):
        want = O.approx_quantiles_exact(x, valid, qs, err)
        m = dq.ApproxQuantiles("x", qs, err).calculate(chunks)
        if want is None:
            assert m.value.isSuccess and m.value.get() == {}, m
            continue
        got = m.value.get()
        for q, w in zip(qs, want):
            assert got[_java_double_to_string(q)] == w, (ps, n, err, q)


def test_decimal_preconditions_and_type_names(dq):
    """DecimalType passes isNumeric; a WrongColumnTypeException names DecimalType(p,s) as the reference would."""
    from deequ_amd.analyzers import Preconditions, spark_type

    Preconditions.isNumeric("d")([("d", "decimal(38,18)", True)])
    assert spark_type("decimal(5,2)") == "DecimalType(5,2)"
