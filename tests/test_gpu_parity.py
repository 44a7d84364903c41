"""Parity of the MI355X path (libdqscan.so through the C ABI) with the CPU oracle.

Tolerances (BASELINE.json north_star): counts, min/max, compliance matches and HLL registers /
estimates bit-exact; fp64 sum / mean / stddev / correlation within 1e-12 relative (sums: relative
to sum(|x|), the condition number of a floating-point sum, since both sides round differently).
"""
from __future__ import annotations

import math

import numpy as np
import pytest

from oracle import dq_oracle as O
from oracle import dq_oracle_c as C
from tests.helpers import close, host_column, oracle_columns

pytestmark = pytest.mark.gpu

REL = 1e-12
GROUPING = ("Uniqueness", "Distinctness", "CountDistinct", "UniqueValueRatio", "Entropy", "MutualInformation")


@pytest.fixture(scope="module")
def dq():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    import deequ_amd

    return deequ_amd


def _device_table(dq, ds):
    data = {name: (t, vals) for name, (t, vals) in ds["columns"].items()}
    return dq.Table.from_pydict(data)


def _analyzer(dq, spec):
    op = spec[0]
    cls = getattr(dq, op)
    args = [a for a in spec[1:]]
    return cls(*args)


def assert_state_close(prod, ref, scale=None):
    """prod: deequ_amd state (or None); ref: oracle state (or None)."""
    if ref is None or prod is None:
        assert prod is None and ref is None, (prod, ref)
        return
    name = type(ref).__name__
    assert type(prod).__name__ == name
    if name in ("NumMatches", "NumMatchesAndCount", "MinState", "MaxState"):
        a, b = prod.__dict__, ref.__dict__
        for k in a:
            x, y = a[k], b[k]
            assert x == y or (isinstance(x, float) and math.isnan(x) and math.isnan(y)), (name, k, x, y)
    elif name == "DataTypeHistogram":
        assert tuple(prod.__dict__.values()) == tuple(ref.__dict__.values()), (prod, ref)
    elif name == "ApproxCountDistinctState":
        assert tuple(prod.words) == tuple(ref.words)
    elif name == "SumState":
        assert close(prod.sum_, ref.sum_, REL, REL * (scale or 0.0)), (prod, ref)
    elif name == "MeanState":
        assert prod.count == ref.count
        assert close(prod.sum_, ref.sum_, REL, REL * (scale or 0.0)), (prod, ref)
    elif name == "StandardDeviationState":
        assert prod.n == ref.n
        sd = math.sqrt(ref.m2 / ref.n) if ref.m2 >= 0 else 0.0
        assert close(prod.avg, ref.avg, REL, REL * (abs(ref.avg) + sd)), (prod, ref)
        assert close(prod.m2, ref.m2, REL, REL * ref.n * (sd * sd + 1e-300)), (prod, ref)
        assert close(prod.metricValue(), ref.metricValue(), REL), (prod.metricValue(), ref.metricValue())
    elif name == "CorrelationState":
        assert prod.n == ref.n
        for k in ("xAvg", "yAvg"):
            assert close(getattr(prod, k), getattr(ref, k), REL, REL * (abs(getattr(ref, k)) + math.sqrt(abs(ref.xMk) / ref.n + abs(ref.yMk) / ref.n))), k
        for k in ("xMk", "yMk"):
            assert close(getattr(prod, k), getattr(ref, k), REL, REL * abs(getattr(ref, k))), k
        assert close(prod.ck, ref.ck, REL, REL * math.sqrt(abs(ref.xMk * ref.yMk))), (prod.ck, ref.ck)
        a, b = prod.metricValue(), ref.metricValue()
        assert close(a, b, 0.0, 1e-12), (a, b)
    else:
        raise AssertionError(name)


# ---------------------------------------------------------------------------------------------
# 1. the reference's own known-answer tests, through AnalysisRunner (fused) and Analyzer.calculate
# ---------------------------------------------------------------------------------------------
def test_reference_kats_fused_and_single(dq, kats):
    from deequ_amd.metrics import EmptyStateException, UnsupportedOnGpuPathException

    by_ds = {}
    for case in kats["cases"]:
        by_ds.setdefault(case["dataset"], []).append(case)
    for ds_name, cases in by_ds.items():
        ds = kats["datasets"][ds_name]
        table = _device_table(dq, ds)
        analyzers = [_analyzer(dq, c["analyzer"]) for c in cases]
        ctx = dq.AnalysisRunner.onData(table).addAnalyzers(analyzers).run()
        for c, a in zip(cases, analyzers):
            for metric in (ctx.metric(a), a.calculate(table)):
                exp = c["expected"]
                if c["needs"]:  # string predicate / regex outside the GPU subset: Spark fallback set
                    assert metric.value.isFailure
                    assert isinstance(metric.value.failed, UnsupportedOnGpuPathException), metric
                    continue
                if isinstance(exp, dict):  # DataType -> HistogramMetric(column, Success(toDistribution(hist)))
                    from deequ_amd.analyzers import toDistribution

                    want = toDistribution(dq.DataTypeHistogram(*exp["DataTypeHistogram"]))
                    assert metric.value.get() == want, (c["source"], a, metric)
                elif exp == "EmptyState":
                    assert metric.value.isFailure and isinstance(metric.value.failed, EmptyStateException), (c, metric)
                elif exp == "NaN":
                    assert math.isnan(metric.value.get()), (c, metric)
                elif c["analyzer"][0] in ("Entropy", "MutualInformation"):  # device log vs the JVM's: fp64 tolerance
                    assert close(metric.value.get(), exp, REL), (c["source"], a, metric, exp)
                else:
                    assert metric.value.get() == exp, (c["source"], a, metric, exp)


def test_empty_state_message(dq, kats):
    # NullHandlingTests.scala:122-133
    table = _device_table(dq, kats["datasets"]["dataWithNullColumns"])
    m = dq.Mean("numericCol").calculate(table)
    assert str(m.value.failed) == "Empty state for analyzer Mean(numericCol,None), all input values were NULL."


def test_kat_states_match_oracle(dq, kats):
    """Every KAT analyzer's full state (not only the metric) equals the oracle's state."""
    for case in kats["cases"]:
        if case["needs"] or case["analyzer"][0] in GROUPING:  # grouping: metrics checked above / below
            continue
        ds = kats["datasets"][case["dataset"]]
        cols, n = oracle_columns(ds)
        ref = O.compute_state(tuple(case["analyzer"]), cols, n, ds.get("partitions", 1))
        table = _device_table(dq, ds)
        prod = _analyzer(dq, case["analyzer"]).computeStateFrom(table)
        assert_state_close(prod, ref, scale=1.0)


# ---------------------------------------------------------------------------------------------
# 2. randomised single-column parity vs the C oracle, edge sizes around the 2048-row block and the
#    rows-per-range floors of small chunks (16 K rows; 64 K for the validity-only pass: dq_plan.cpp)
# ---------------------------------------------------------------------------------------------
SIZES = [0, 1, 7, 63, 64, 65, 2047, 2048, 2049, 4097, 16_383, 16_385, 65_537, 100_003]


def _rand_table(dq, n, seed, null_frac):
    rng = np.random.default_rng(seed)
    valid = rng.random(n) >= null_frac
    f = rng.normal(1000.0, 7.5, n)
    i64 = rng.integers(-(1 << 40), 1 << 40, n)
    i32 = rng.integers(-50000, 50000, n).astype(np.int32)
    strs = [None if not valid[i] else (b"v%d-" % int(rng.integers(0, 5000))) * int(1 + i % 5) for i in range(n)]
    from deequ_amd.table import column_from_numpy, utf8_column

    t = dq.Table([column_from_numpy("f", "f64", f, valid), column_from_numpy("l", "i64", i64, valid),
                  column_from_numpy("i", "i32", i32, ~valid if null_frac < 1 else valid),
                  utf8_column("s", strs)])
    return t


def _profile(dq, t):
    from deequ_amd.synth import profile_analyzers

    return profile_analyzers(t)


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("null_frac", [0.0, 0.1, 1.0])
def test_profile_vs_oracle(dq, n, null_frac):
    t = _rand_table(dq, n, seed=n + int(null_frac * 10), null_frac=null_frac)
    analyzers = _profile(dq, t)
    from deequ_amd.runner import scan_states

    states = scan_states(t, analyzers)
    host = {name: host_column(c, n) for name, c in t.columns.items()}
    for a in analyzers:
        prod = states[a]
        if type(a).__name__ == "Size":
            assert prod.numMatches == n
            continue
        vals, valid, bm = host[a.column]
        dtype = t.columns[a.column].dtype
        ocol = O.OColumn(dtype, vals, valid)
        if type(a).__name__ in ("ApproxCountDistinct", "Completeness"):
            ref = O.compute_state((type(a).__name__, a.column, None), {a.column: ocol}, n)
            assert_state_close(prod, ref)
            continue
        s = C.column_stats(dtype, vals, bm, None, 1)
        name = type(a).__name__
        if s.count == 0:
            ref = None
        elif name == "Sum":
            ref = O.SumState(s.sum_f64)
        elif name == "Mean":
            ref = O.MeanState(s.sum_f64, s.count)
        elif name == "StandardDeviation":
            ref = O.StandardDeviationState(s.n, s.avg, s.m2)
        elif name == "Minimum":
            ref = O.MinState(s.min)
        else:
            ref = O.MaxState(s.max)
        scale = float(np.abs(np.asarray(vals, dtype=np.float64)[valid]).sum()) if len(vals) else 0.0
        assert_state_close(prod, ref, scale=scale)


UTF8_LENS = [0, 1, 3, 4, 7, 8, 9, 12, 15, 16, 17, 20, 23, 24, 25, 27, 28, 29, 31, 32, 33, 40, 63, 64, 65, 100]


@pytest.mark.parametrize("large", [False, True])
@pytest.mark.parametrize("n", [1, 5, 64, 513, 4099])
def test_utf8_hll_edge_lengths(dq, n, large):
    """HLL registers of strings of every round structure of the short hash (stripes, 4-byte and byte
    rounds), empty strings, the > 28-byte general path, arbitrary bytes (incl. 0x00 / 0xFF, invalid
    UTF-8) and both offset widths, with and without a `where` filter, vs the oracle."""
    from deequ_amd.runner import scan_states
    from deequ_amd.table import column_from_numpy, utf8_column

    rng = np.random.default_rng(1000 + n + int(large))
    strs = []
    for i in range(n):
        if rng.random() < 0.1:
            strs.append(None)
        else:
            ln = int(UTF8_LENS[int(rng.integers(0, len(UTF8_LENS)))])
            # a small alphabet keeps repeats (distinct counts well below n) next to unique values
            strs.append(bytes(rng.integers(0, 256, ln, dtype=np.uint8)) if rng.random() < 0.5
                        else bytes(rng.integers(0, 3, ln, dtype=np.uint8)))
    a = rng.integers(-5, 5, n).astype(np.int64)
    t = dq.Table([utf8_column("s", strs, large=large), column_from_numpy("a", "i64", a, np.ones(n, bool))])
    analyzers = [dq.ApproxCountDistinct("s"), dq.ApproxCountDistinct("s", "a > 0"), dq.Completeness("s")]
    got = scan_states(t, analyzers)
    valid = np.array([s is not None for s in strs])
    ocols = {"s": O.OColumn("utf8", strs, valid), "a": O.OColumn("i64", a, np.ones(n, bool))}  # (offset width: no effect on the hash)
    for an in analyzers:
        ref = O.compute_state((type(an).__name__, an.column, an.where), ocols, n)
        assert_state_close(got[an], ref)


@pytest.mark.parametrize("lens", [(24, 28), (23, 25), (8, 24)])
@pytest.mark.parametrize("n", [63, 4097, 100_003])
def test_utf8_hll_deferred_third_round(dq, n, lens):
    """The UTF8 pass defers a selected string of 24..28 bytes (third stripe round) to a per-wave LDS queue
    finished 64 at a time: every lane deferred (24..28 bytes: a drain per row group), a boundary mix, and
    C5's 8..24-byte lengths, with nulls and a `where`, vs the oracle's HLL registers."""
    from deequ_amd.runner import scan_states
    from deequ_amd.table import column_from_numpy, utf8_column

    rng = np.random.default_rng(77 + n + lens[0])
    strs = [None if rng.random() < 0.1 else bytes(rng.integers(0, 256, int(rng.integers(lens[0], lens[1] + 1)),
                                                              dtype=np.uint8)) for _ in range(n)]
    a = rng.integers(-5, 5, n).astype(np.int64)
    t = dq.Table([utf8_column("s", strs), column_from_numpy("a", "i64", a, np.ones(n, bool))])
    analyzers = [dq.ApproxCountDistinct("s"), dq.ApproxCountDistinct("s", "a > 0")]
    got = scan_states(t, analyzers)
    valid = np.array([s is not None for s in strs])
    ocols = {"s": O.OColumn("utf8", strs, valid), "a": O.OColumn("i64", a, np.ones(n, bool))}
    for an in analyzers:
        ref = O.compute_state((type(an).__name__, an.column, an.where), ocols, n)
        assert_state_close(got[an], ref)


def test_chunked_equals_single_scan(dq):
    """dq_scan over row chunks (chunk_index order) == one scan (PartitionedTableIntegrationTest analogue)."""
    from deequ_amd import synth
    from deequ_amd.runner import scan_states

    n = 3 * 65536 + 123
    whole = synth.c5_table(n, seed=3)
    parts = [synth.c5_table(65536, row0=r, seed=3) for r in (0, 65536, 131072)] + [synth.c5_table(n - 196608, row0=196608, seed=3)]
    analyzers = synth.profile_analyzers(whole)
    a = scan_states(whole, analyzers)
    b = scan_states(parts, analyzers)
    for an in analyzers:
        ref = a[an]
        got = b[an]
        if ref is None:
            assert got is None
            continue
        if hasattr(ref, "words"):
            assert got.words == ref.words
        elif type(ref).__name__ in ("NumMatches", "NumMatchesAndCount", "MinState", "MaxState"):
            assert got == ref
        else:
            assert close(got.metricValue(), ref.metricValue(), REL), (an, got, ref)


def test_nan_min_max_and_hash(dq):
    """Spark orders NaN above every double: max = NaN if any NaN; min ignores NaN unless all NaN."""
    from deequ_amd.runner import scan_states

    t = dq.Table.from_pydict({"x": ("f64", [1.0, float("nan"), -3.5, None, 2.0])})
    s = scan_states(t, [dq.Minimum("x"), dq.Maximum("x"), dq.ApproxCountDistinct("x")])
    assert s[dq.Minimum("x")].minValue == -3.5
    assert math.isnan(s[dq.Maximum("x")].maxValue)
    cols = {"x": O.OColumn("f64", np.array([1.0, float("nan"), -3.5, 0.0, 2.0]), np.array([1, 1, 1, 0, 1], bool))}
    assert s[dq.ApproxCountDistinct("x")].words == O.compute_state(("ApproxCountDistinct", "x", None), cols, 5).words
    t2 = dq.Table.from_pydict({"y": ("f64", [float("nan"), None, float("nan")])})
    s2 = scan_states(t2, [dq.Minimum("y"), dq.Maximum("y")])
    assert math.isnan(s2[dq.Minimum("y")].minValue) and math.isnan(s2[dq.Maximum("y")].maxValue)


@pytest.mark.parametrize("kinds", ["pinf", "ninf", "both", "nan_inf"])
@pytest.mark.parametrize("n", [1, 5, 300, 4099, 70_001])
def test_infinities_vs_oracle(dq, n, kinds):
    """+-inf values: Sum / Mean are Spark's sequential sum (+-inf, NaN with both signs or any NaN),
    Min / Max include them, StdDev's metric is NaN (its m2 is NaN in Spark; its avg is order-dependent:
    inf or NaN), counts and HLL registers stay exact."""
    from deequ_amd.runner import scan_states
    from deequ_amd.table import column_from_numpy

    rng = np.random.default_rng(4000 + n + len(kinds))
    x = rng.normal(10.0, 3.0, n)
    k = max(1, n // 500)
    pos = rng.choice(n, size=min(n, 3 * k), replace=False)
    specials = {"pinf": [np.inf], "ninf": [-np.inf], "both": [np.inf, -np.inf], "nan_inf": [np.inf, np.nan]}[kinds]
    x[pos] = np.array(specials)[rng.integers(0, len(specials), len(pos))]
    valid = rng.random(n) >= 0.1
    valid[pos[0]] = True
    t = dq.Table([column_from_numpy("x", "f64", x, valid)])
    an = [dq.Sum("x"), dq.Mean("x"), dq.Minimum("x"), dq.Maximum("x"), dq.StandardDeviation("x"),
          dq.ApproxCountDistinct("x"), dq.Completeness("x")]
    got = scan_states(t, an)
    cols = {"x": O.OColumn("f64", x, valid)}

    def same(a, b):
        return (math.isnan(a) and math.isnan(b)) or a == b

    for a in an:
        name = type(a).__name__
        ref = O.compute_state((name, "x", None), cols, n)
        g = got[a]
        if name == "StandardDeviation":
            assert g.n == ref.n and math.isnan(g.metricValue()) and math.isnan(ref.metricValue()), (g, ref)
        elif name in ("Sum", "Mean") and not math.isfinite(ref.sum_):
            assert same(g.sum_, ref.sum_), (a, g, ref)
            assert name == "Sum" or g.count == ref.count
        else:
            assert_state_close(g, ref, scale=float(np.abs(x[valid & np.isfinite(x)]).sum()))


# ---------------------------------------------------------------------------------------------
# 3. predicates (Compliance / where) vs the oracle's independent SQL evaluator
# ---------------------------------------------------------------------------------------------
PREDICATES = [
    "a > 3", "a >= 3.0", "a > 2.5", "a < -1.5", "a = 4", "a = 4.5", "a != 4.5", "a <> 7",
    "b <= 0.25", "b > 1e1", "a < b", "b >= a", "a = c", "c > a",
    "COALESCE(a, 0.0) >= 0", "COALESCE(b, 1.0) > 0", "COALESCE(a, 5) < 3",
    "`a` IS NULL OR (`a` >= 0.0 AND `a` <= 7.0)", "`b` IS NULL OR (`b` > -1.0 AND `b` < 8.0)",
    "a IS NOT NULL", "NOT (a > 2 AND b < 0.5)", "a > 2 OR b IS NULL", "NOT a > 2",
    "(a > 1 AND b > 0.1) OR (c < 0 AND a IS NULL)", "TRUE", "NULL", "a > NULL", "1 < 2", "1.5 > 2",
]


@pytest.fixture(scope="module")
def pred_data():
    rng = np.random.default_rng(11)
    n = 5000
    a = rng.integers(-8, 12, n).astype(np.int64)
    b = np.round(rng.normal(0.5, 2.0, n), 2)
    c = rng.integers(-5, 10, n).astype(np.int32)
    va, vb, vc = rng.random(n) > 0.15, rng.random(n) > 0.2, rng.random(n) > 0.1
    return n, {"a": ("i64", a, va), "b": ("f64", b, vb), "c": ("i32", c, vc)}


def _tables(dq, pred_data):
    from deequ_amd.table import column_from_numpy

    n, d = pred_data
    dev = dq.Table([column_from_numpy(k, t, v, m) for k, (t, v, m) in d.items()])
    ocols = {k: O.OColumn(t, v, m) for k, (t, v, m) in d.items()}
    return n, dev, ocols


def test_compliance_predicates_vs_oracle(dq, pred_data):
    n, dev, ocols = _tables(dq, pred_data)
    analyzers = [dq.Compliance(f"r{i}", p) for i, p in enumerate(PREDICATES)]
    from deequ_amd.runner import scan_states

    got = scan_states(dev, analyzers)
    for a in analyzers:
        ref = O.compute_state(("Compliance", a.instance, a.predicate, None), ocols, n)
        assert got[a] == (None if ref is None else dq.NumMatchesAndCount(ref.numMatches, ref.count)), (a.predicate, got[a], ref)


WHERES = ["a > 2", "b < 0.5", "c IS NULL", "COALESCE(a, 0.0) >= 0", "a > 100"]


def test_where_filters_vs_oracle(dq, pred_data):
    n, dev, ocols = _tables(dq, pred_data)
    analyzers = []
    for w in WHERES:
        analyzers += [dq.Size(w), dq.Completeness("b", w), dq.Compliance("w", "a < b", w), dq.Sum("a", w),
                      dq.Mean("b", w), dq.StandardDeviation("b", w), dq.Minimum("c", w), dq.Maximum("b", w),
                      dq.ApproxCountDistinct("a", w), dq.Correlation("a", "b", w)]
    from deequ_amd.runner import scan_states

    got = scan_states(dev, analyzers)
    for a in analyzers:
        name = type(a).__name__
        if name == "Size":
            spec = ("Size", a.where)
        elif name == "Compliance":
            spec = ("Compliance", a.instance, a.predicate, a.where)
        elif name == "Correlation":
            spec = ("Correlation", a.firstColumn, a.secondColumn, a.where)
        else:
            spec = (name, a.column, a.where)
        ref = O.compute_state(spec, ocols, n)
        prod = got[a]
        if ref is None:
            assert prod is None, (a, prod)
            continue
        conv = {"NumMatches": lambda r: dq.NumMatches(r.numMatches),
                "NumMatchesAndCount": lambda r: dq.NumMatchesAndCount(r.numMatches, r.count)}
        if type(ref).__name__ in conv:
            assert prod == conv[type(ref).__name__](ref), (a, prod, ref)
        else:
            assert_state_close(prod, ref, scale=float(np.abs(ocols["b"].values).sum() + np.abs(ocols["a"].values).sum()))


@pytest.mark.parametrize("n", [1, 31, 32, 33, 63, 64, 65, 511, 513, 2047, 2048, 2049, 4097, 100003])
def test_predicates_ragged_sizes(dq, n):
    """Row counts around the predicate pass's 32-row words, 64-row waves and 2048-row workgroup
    slices, with NaNs in the f64 column (Spark orders NaN above every number and NaN = NaN)."""
    from deequ_amd.runner import scan_states

    rng = np.random.default_rng(n)
    a = rng.integers(-8, 12, n).astype(np.int64)
    b = np.round(rng.normal(0.5, 2.0, n), 2)
    b[rng.random(n) < 0.05] = np.nan
    c = rng.integers(-5, 10, n).astype(np.int32)
    va, vb, vc = rng.random(n) > 0.15, rng.random(n) > 0.2, rng.random(n) > 0.1
    _, dev, ocols = _tables(dq, (n, {"a": ("i64", a, va), "b": ("f64", b, vb), "c": ("i32", c, vc)}))
    preds = ["a > 3", "b <= 0.25", "b = b", "b > 1e300", "a < b", "`b` IS NULL OR (`b` > -1.0 AND `b` < 8.0)",
             "NOT (a > 2 AND b < 0.5)", "(a > 1 AND b > 0.1) OR (c < 0 AND a IS NULL)"]
    analyzers = [dq.Compliance(f"r{i}", p) for i, p in enumerate(preds)]
    analyzers += [dq.Size("b > 0.5"), dq.Compliance("w", "a < c", "b >= 0"), dq.Sum("a", "c > 0"),
                  dq.Maximum("b", "a > 0")]
    got = scan_states(dev, analyzers)
    for an in analyzers:
        name = type(an).__name__
        if name == "Compliance":
            spec = ("Compliance", an.instance, an.predicate, an.where)
        elif name == "Size":
            spec = ("Size", an.where)
        else:
            spec = (name, an.column, an.where)
        ref = O.compute_state(spec, ocols, n)
        prod = got[an]
        if ref is None:
            assert prod is None, (an, prod)
        elif name == "Compliance":
            assert prod == dq.NumMatchesAndCount(ref.numMatches, ref.count), (an, prod, ref)
        elif name == "Size":
            assert prod == dq.NumMatches(ref.numMatches), (an, prod, ref)
        else:
            assert_state_close(prod, ref, scale=float(np.abs(a).sum()) + 1.0)


def test_unsupported_predicate_routes_to_fallback(dq, pred_data):
    from deequ_amd.metrics import UnsupportedOnGpuPathException

    n, dev, _ = _tables(dq, pred_data)
    good, bad = dq.Compliance("ok", "a > 1"), dq.Compliance("bad", "a IN (1, 2)")
    ctx = dq.AnalysisRunner.onData(dev).addAnalyzers([good, bad]).run()
    assert ctx.metric(good).value.isSuccess
    assert isinstance(ctx.metric(bad).value.failed, UnsupportedOnGpuPathException)


def test_missing_column_in_predicate_fails_whole_pass(dq, pred_data):
    """A predicate that cannot be analysed fails every shareable analyzer (AnalysisRunner.scala:310-313)."""
    n, dev, _ = _tables(dq, pred_data)
    ctx = dq.AnalysisRunner.onData(dev).addAnalyzers([dq.Size(), dq.Compliance("x", "nosuch > 3")]).run()
    assert all(m.value.isFailure for m in ctx.allMetrics)


# ---------------------------------------------------------------------------------------------
# 4. the benchmark configurations at reduced row counts vs the C oracle (Spark partition simulation)
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("cfg", ["c2", "c3", "c4", "c5"])
def test_configs_vs_oracle(dq, cfg):
    from deequ_amd import synth
    from deequ_amd.runner import scan_states

    # c3: the fused Compliance states are checked against the (pure-Python) oracle evaluator over every row
    n = 300_007 if cfg == "c3" else 1_000_003
    t = getattr(synth, f"{cfg}_table")(n, seed=5)
    if cfg == "c4":
        names = list(t.columns)
        analyzers = [dq.Correlation(names[i], names[j]) for i in range(8) for j in range(i + 1, 8)]
        analyzers += [dq.Mean(c) for c in names] + [dq.StandardDeviation(c) for c in names]
    elif cfg == "c3":
        analyzers = [dq.Size()] + [dq.ApproxCountDistinct(c) for c in t.columns]
        analyzers += [dq.Compliance("p0", "i0 >= 0"), dq.Compliance("p1", "`i1` IS NULL OR (`i1` >= 10.0 AND `i1` <= 1000.0)"),
                      dq.Compliance("p2", "i2 < i3"), dq.Compliance("p3", "COALESCE(i3, 0.0) >= 0")]
    else:
        analyzers = synth.profile_analyzers(t)
    got = scan_states(t, analyzers)
    host = {name: host_column(c, n) for name, c in t.columns.items()}
    nparts = 8
    errors = []
    for a in analyzers:
        try:
            _check_config_analyzer(dq, t, a, got[a], host, n, nparts)
        except AssertionError as e:
            errors.append(f"{a}: {e}")
    assert not errors, "\n".join(errors[:20]) + f"\n({len(errors)} mismatches)"


def _check_config_analyzer(dq, t, a, prod, host, n, nparts):
    name = type(a).__name__
    if name == "Size":
        assert prod.numMatches == n
    elif name == "Completeness":
        assert prod.numMatches == int(host[a.column][1].sum()) and prod.count == n
    elif name == "ApproxCountDistinct":
        vals, valid, bm = host[a.column]
        col = t.columns[a.column]
        if col.dtype == "utf8":
            offs = col.offsets.cpu().numpy()[: (n + 1) * 4].view(np.int32)
            data = np.frombuffer(col.values.cpu().numpy().tobytes(), dtype=np.uint8)
            regs = C.hll_registers("utf8", data, offs, bm, None, n)
        else:
            regs = C.hll_registers(col.dtype, vals, None, bm, None, n)
        assert prod.words == tuple(O.registers_to_words(regs.tolist())), "HLL words differ"
    elif name == "Compliance":
        # the state of the FUSED scan (HLL x 8 + 4 predicates in one plan) vs the oracle over all n rows
        cols = {k: O.OColumn(t.columns[k].dtype, host[k][0], host[k][1]) for k in ("i0", "i1", "i2", "i3")}
        ref = O.compute_state(("Compliance", a.instance, a.predicate, None), cols, n)
        assert prod == dq.NumMatchesAndCount(ref.numMatches, ref.count), (prod, ref)
    elif name == "Correlation":
        x, vx, bx = host[a.firstColumn]
        y, vy, by = host[a.secondColumn]
        r = C.corr("f64", x, bx, "f64", y, by, None, nparts)
        both = int((vx & vy).sum())
        assert r[0] == both, f"oracle n {r[0]} != numpy both-valid {both}"
        assert_state_close(prod, O.CorrelationState(*r))
    else:
        vals, valid, bm = host[a.column]
        dtype = t.columns[a.column].dtype
        s = C.column_stats(dtype, vals, bm, None, nparts)
        ref = {"Sum": lambda: O.SumState(s.sum_f64), "Mean": lambda: O.MeanState(s.sum_f64, s.count),
               "StandardDeviation": lambda: O.StandardDeviationState(s.n, s.avg, s.m2),
               "Minimum": lambda: O.MinState(s.min), "Maximum": lambda: O.MaxState(s.max)}[name]()
        assert_state_close(prod, ref, scale=float(np.abs(vals.astype(np.float64)[valid]).sum()))


def test_incremental_state_provider_roundtrip(dq, tmp_path):
    """persist -> load -> merge (IncrementalAnalysisTest / StateProviderTest analogue)."""
    from deequ_amd import synth

    t1 = synth.c5_table(50_000, seed=9)
    t2 = synth.c5_table(30_000, row0=50_016, seed=9)
    analyzers = synth.profile_analyzers(t1) + [dq.Correlation("c0", "c1")]
    for provider in (dq.InMemoryStateProvider(), dq.HdfsStateProvider(str(tmp_path / "state"), allowOverwrite=True)):
        dq.AnalysisRunner.onData(t1).addAnalyzers(analyzers).saveStatesWith(provider).run()
        inc = dq.AnalysisRunner.onData(t2).addAnalyzers(analyzers).aggregateWith(provider).run()
        both = dq.AnalysisRunner.onData([t1, t2]).addAnalyzers(analyzers).run()
        for a in analyzers:
            x, y = inc.metric(a).value.get(), both.metric(a).value.get()
            assert close(x, y, 1e-12), (a, x, y)


@pytest.mark.parametrize("cfg", ["c4", "c5"])
def test_deterministic_repeat(dq, cfg):
    """Fixed merge order everywhere: repeated scans are bitwise identical."""
    from deequ_amd import synth
    from deequ_amd.runner import scan_states

    t = getattr(synth, f"{cfg}_table")(700_001, seed=8)
    if cfg == "c4":
        names = list(t.columns)
        analyzers = [dq.Correlation(names[i], names[j]) for i in range(8) for j in range(i + 1, 8)]
        analyzers += [dq.StandardDeviation(c) for c in names]
    else:
        analyzers = synth.profile_analyzers(t)
    runs = [scan_states(t, analyzers) for _ in range(3)]
    for a in analyzers:
        assert repr(runs[0][a]) == repr(runs[1][a]) == repr(runs[2][a]), a


def test_scan_orders_after_producer_on_torch_stream(dq):
    """The plan launches on torch's current stream (the null stream by default): a column whose values
    are still being written by a queued kernel must be scanned after that kernel, not before."""
    import torch

    from deequ_amd.runner import scan_states
    from deequ_amd.table import Column

    n = 4_000_000
    for _ in range(3):
        raw = torch.zeros(n * 8 + 16, dtype=torch.uint8, device="cuda")
        torch.cuda._sleep(50_000_000)  # keep the stream busy so an unordered scan would read the zeros
        raw[: n * 8].view(torch.float64).fill_(1.5)
        t = dq.Table([Column("x", "f64", n, raw, None, None, nullable=False)])
        got = scan_states(t, [dq.Sum("x"), dq.Maximum("x")])
        assert got[dq.Sum("x")].sum_ == 1.5 * n
        assert got[dq.Maximum("x")].maxValue == 1.5


DT_ATOMS = [b"", b"-", b"+", b" ", b"- ", b"+ ", b"0", b"7", b"12", b"007", b".", b"..", b"1.5", b"-3.25", b"+ 0.",
            b"true", b"false", b"True", b"fals", b"truee", b"a", b"1e5", b"1 ", b" 1", b"--1", b"1\n", b"\xff",
            b"\xd9\xa1", b"\x00", b"/", b":", b"-", b"9" * 27 + b".", b"1" * 28, b"1" * 29, b"-" + b"2" * 40,
            b"3." + b"4" * 30, b"5" * 31 + b".6", b"12345678901234567890.1234567"]


def _dt_string(rng) -> bytes:
    k = rng.random()
    if k < 0.5:
        return DT_ATOMS[int(rng.integers(0, len(DT_ATOMS)))]
    # signed / spaced digit strings with 0-2 dots at random places, lengths 0..40
    sign = [b"", b"-", b"+", b"- ", b" "][int(rng.integers(0, 5))]
    body = bytearray(rng.choice(np.frombuffer(b"0123456789", np.uint8), int(rng.integers(0, 40))).tobytes())
    for _ in range(int(rng.integers(0, 3))):
        if body:
            body[int(rng.integers(0, len(body)))] = ord(".")
    if rng.random() < 0.05 and body:
        body[int(rng.integers(0, len(body)))] = int(rng.integers(0, 256))
    return sign + bytes(body)


@pytest.mark.parametrize("path", ["auto", "long"])
@pytest.mark.parametrize("large", [False, True])
@pytest.mark.parametrize("n", [1, 64, 513, 4099, 70_001])
def test_datatype_vs_oracle(dq, n, large, path, monkeypatch):
    """DataType (StatefulDataType.scala:36-67) on strings of every class and length (the <= 28-byte
    SWAR path and the byte path), alone and fused with ApproxCountDistinct, with and without `where`;
    on f64 values around the Double.toString boundaries (1e-3, 1e7, +-0, NaN, +-inf) and on integral
    columns -- bit-exact histograms vs the oracle.  path "long": the string HLL variants' LONG
    instantiation (DQ_STR_PATH; the one dq_scan picks for columns of long strings)."""
    from deequ_amd.runner import scan_states

    if path == "long":
        monkeypatch.setenv("DQ_STR_PATH", "long")
    from deequ_amd.table import column_from_numpy, utf8_column

    rng = np.random.default_rng(77 + n + int(large))
    strs = [None if rng.random() < 0.1 else _dt_string(rng) for _ in range(n)]
    pool = np.array([0.0, -0.0, 1e-3, np.nextafter(1e-3, 0), 9999999.999, 1e7, np.nextafter(1e7, 0), -5e-4,
                     float("nan"), float("inf"), -float("inf"), 1.5, -2.75e12, 3e-300])
    f = np.where(rng.random(n) < 0.5, pool[rng.integers(0, len(pool), n)], rng.normal(0, 1e4, n) * 10.0 ** rng.integers(-6, 9, n))
    fv = rng.random(n) >= 0.1
    a = rng.integers(-5, 5, n).astype(np.int64)
    i32 = rng.integers(-(1 << 31), 1 << 31, n).astype(np.int32)
    t = dq.Table([utf8_column("s", strs, large=large), utf8_column("u", strs, large=not large),
                  column_from_numpy("f", "f64", f, fv), column_from_numpy("a", "i64", a, rng.random(n) >= 0.2),
                  column_from_numpy("i", "i32", i32, np.ones(n, bool))])
    analyzers = [dq.DataType("s"), dq.ApproxCountDistinct("s"), dq.DataType("s", "a > 0"),
                 dq.DataType("u"),  # alone: the classify-only variant
                 dq.DataType("f"), dq.DataType("f", "a >= 0"), dq.Mean("f"), dq.DataType("a"), dq.DataType("i"),
                 dq.DataType("a", "a < 2")]
    got = scan_states(t, analyzers)
    host = {name: host_column(c, n) for name, c in t.columns.items()}
    ocols = {name: O.OColumn(t.columns[name].dtype.replace("large_", ""), host[name][0], host[name][1])
             for name in t.columns}
    for an in analyzers:
        ref = O.compute_state((type(an).__name__, an.column, an.where), ocols, n)
        if type(an).__name__ in ("DataType", "ApproxCountDistinct"):  # bit-exact histograms / registers
            norm = lambda st: [list(v) if isinstance(v, (list, tuple)) else v for v in st.__dict__.values()]
            assert norm(got[an]) == norm(ref), (an, got[an], ref)
        elif math.isfinite(ref.sum_):
            assert_state_close(got[an], ref, scale=float(np.abs(f[fv & np.isfinite(f)]).sum()))
        else:  # +-inf / NaN in the column: Spark's sum is +-inf or NaN
            g = got[an]
            assert g.count == ref.count and ((math.isnan(g.sum_) and math.isnan(ref.sum_)) or g.sum_ == ref.sum_)


# ---------------------------------------------------------------------------------------------
# PatternMatch (PatternMatch.scala:37-56): the search-DFA atom of the predicate pass
# ---------------------------------------------------------------------------------------------
def _pm_strings(rng, n):
    alphabet = list("abcdxyzq@.-_:/ \t0123456789é€𝄞☺") + ["someone@somewhere.org", "http://foo.com/x", "https://",
                                                           "1.5", "ftp://a.b", "x@y.io", "colour"]
    out = []
    for i in range(n):
        if rng.random() < 0.1:
            out.append(None)
            continue
        k = int(rng.integers(0, 9)) if i % 97 else int(rng.integers(20, 60))  # a few long values
        out.append("".join(alphabet[int(j)] for j in rng.integers(0, len(alphabet), k)).encode("utf-8"))
    return out


@pytest.mark.parametrize("large", [False, True])
@pytest.mark.parametrize("n", [0, 1, 513, 4099, 70_001])
def test_pattern_match_vs_oracle(dq, n, large):
    """PatternMatch on the GPU (alone, with `where`, fused with HLL / Completeness / Compliance) vs the
    oracle's regexp_extract restatement: NumMatchesAndCount bit-exact, incl. non-ASCII values, NULLs,
    empty values and values longer than a dword-loop's worth; int32 and int64 offsets."""
    from deequ_amd.runner import scan_states
    from deequ_amd.table import column_from_numpy, utf8_column

    rng = np.random.default_rng(1234 + n + int(large))
    strs = _pm_strings(rng, n)
    a = rng.integers(-3, 3, n).astype(np.int64)
    t = dq.Table([utf8_column("s", strs, large=large), column_from_numpy("a", "i64", a, rng.random(n) >= 0.2)])
    pats = [dq.Patterns.EMAIL, dq.Patterns.URL, r"\d\.\d", r"^\d+$", "é.", r"[^\s]{6,}", r"(?:ab|cd){2}"]
    analyzers = [dq.PatternMatch("s", p) for p in pats] + [
        dq.PatternMatch("s", dq.Patterns.EMAIL, "a > 0"), dq.PatternMatch("s", r"\d", "a >= 1"),
        dq.ApproxCountDistinct("s"), dq.Completeness("s"), dq.Compliance("c", "a < 2"), dq.Size()]
    got = scan_states(t, analyzers)
    host = {name: host_column(c, n) for name, c in t.columns.items()}
    ocols = {name: O.OColumn(t.columns[name].dtype.replace("large_", ""), host[name][0], host[name][1])
             for name in t.columns}
    for an in analyzers:
        kind = type(an).__name__
        if kind == "PatternMatch":
            spec = ("PatternMatch", an.column, an.pattern, an.where)
        elif kind == "Compliance":
            spec = ("Compliance", an.instance, an.predicate, an.where)
        elif kind == "Size":
            spec = ("Size", an.where)
        else:
            spec = (kind, an.column, an.where)
        ref = O.compute_state(spec, ocols, n)
        assert_state_close(got[an], ref)


def test_pattern_match_fallback_in_fused_run(dq):
    """A pattern outside the GPU subset fails only its own metric (routed to the fallback set); the
    rest of the fused pass is unaffected."""
    from deequ_amd.metrics import UnsupportedOnGpuPathException

    t = dq.Table.from_pydict({"s": ("utf8", ["111-05-1130", "x", None, "4111 1111 1111 1111"])})
    ssn, url = dq.PatternMatch("s", dq.Patterns.SOCIAL_SECURITY_NUMBER_US), dq.PatternMatch("s", dq.Patterns.URL)
    ctx = dq.AnalysisRunner.onData(t).addAnalyzers([ssn, url, dq.Size()]).run()
    assert isinstance(ctx.metric(ssn).value.failed, UnsupportedOnGpuPathException)
    assert ctx.metric(url).value.get() == 0.0 and ctx.metric(dq.Size()).value.get() == 4.0


@pytest.mark.parametrize("n", [1, 513, 70_001])
def test_string_predicates_vs_oracle(dq, n):
    """String (in)equality / IN / NOT IN on UTF8 columns (whole-value DFAs in the predicate pass) as
    Compliance predicates and as `where` filters of value analyzers, three-valued, vs the oracle."""
    from deequ_amd.runner import scan_states
    from deequ_amd.table import column_from_numpy, utf8_column

    rng = np.random.default_rng(99 + n)
    pool = ["a", "b", "ab", "", "é€", "a b", "a\n", "US", "DE"]
    strs = [None if rng.random() < 0.15 else pool[int(rng.integers(0, len(pool)))].encode() for _ in range(n)]
    x = rng.normal(10, 3, n)
    t = dq.Table([utf8_column("s", strs), utf8_column("t", strs[::-1], large=True),
                  column_from_numpy("x", "f64", x, rng.random(n) >= 0.1)])
    analyzers = [dq.Compliance("eq", "s = 'a'"), dq.Compliance("ne", "s != 'ab'"),
                 dq.Compliance("in", "s IN ('a', 'é€', '')"), dq.Compliance("nin", "t NOT IN ('US', 'DE')"),
                 dq.Compliance("mix", "x > 10 OR s = 'a b'"), dq.Mean("x", "s IN ('a', 'b')"),
                 dq.Maximum("x", "t != 'a'"), dq.Completeness("t", "s = 'DE'"), dq.Size("s <> 'US'"),
                 dq.ApproxCountDistinct("s", "t = 'b'")]
    got = scan_states(t, analyzers)
    host = {name: host_column(c, n) for name, c in t.columns.items()}
    ocols = {name: O.OColumn(t.columns[name].dtype.replace("large_", ""), host[name][0], host[name][1])
             for name in t.columns}
    for an in analyzers:
        kind = type(an).__name__
        if kind == "Compliance":
            spec = ("Compliance", an.instance, an.predicate, an.where)
        elif kind == "Size":
            spec = ("Size", an.where)
        else:
            spec = (kind, an.column, an.where)
        ref = O.compute_state(spec, ocols, n)
        assert_state_close(got[an], ref, scale=float(np.abs(x).sum()))



# ---------------------------------------------------------------------------------------------
# grouping analyzers: sort-based GROUP BY on the device (GroupingAnalyzers.scala:44-82)
# ---------------------------------------------------------------------------------------------
def _group_table(dq, n, seed, chunked=False):
    from deequ_amd.table import column_from_numpy, utf8_column

    rng = np.random.default_rng(seed)
    k = max(1, n // 3)
    f = rng.integers(0, k, n).astype(np.float64) / 4
    f[rng.random(n) < 0.02] = np.nan
    f[rng.random(n) < 0.02] = -0.0
    f[rng.random(n) < 0.02] = 0.0
    i64 = rng.integers(-k, k, n) * 1_000_003
    i32 = rng.integers(0, 7, n).astype(np.int32)
    strs = [None if rng.random() < 0.1 else ("v%d" % int(rng.integers(0, k))).encode() * int(1 + (i % 3) * 5)
            for i in range(n)]
    cols = lambda lo, hi: [column_from_numpy("f", "f64", f[lo:hi], rng.random(hi - lo) >= 0.1),
                           column_from_numpy("l", "i64", i64[lo:hi], np.ones(hi - lo, bool)),
                           column_from_numpy("i", "i32", i32[lo:hi], rng.random(hi - lo) >= 0.3),
                           utf8_column("s", strs[lo:hi]), utf8_column("t", strs[lo:hi][::-1], large=True)]
    if not chunked:
        return dq.Table(cols(0, n))
    cut = n // 3
    return [dq.Table(cols(0, cut)), dq.Table(cols(cut, n))]


@pytest.mark.parametrize("n,chunked", [(1, False), (700, False), (70_001, False), (50_000, True)])
def test_grouping_vs_oracle(dq, n, chunked):
    """Uniqueness / Distinctness / CountDistinct / UniqueValueRatio / Entropy over f64 (NaN, -0.0),
    i64, i32, UTF8, LARGE_UTF8 and multi-column keys, one or several chunks, vs the oracle's
    frequencies: counts bit-exact, entropy within 1e-12."""
    from deequ_amd.runner import _chunks

    data = _group_table(dq, n, 5 + n, chunked)
    analyzers = [dq.Uniqueness("f"), dq.Distinctness("l"), dq.CountDistinct("i"), dq.UniqueValueRatio("s"),
                 dq.Entropy("t"), dq.Entropy("f"), dq.Uniqueness(["s", "i"]), dq.CountDistinct(["l", "f", "t"]),
                 dq.Distinctness(["i"]), dq.MutualInformation("s", "i"), dq.MutualInformation("f", "l"),
                 dq.MutualInformation(["t", "t"]), dq.Size()]
    ctx = dq.AnalysisRunner.onData(data).addAnalyzers(analyzers).run()
    parts = _chunks(data)
    ocols, total = {}, 0
    for name in parts[0].columns:
        vals, valid = [], []
        for t in parts:
            v, ok, _ = host_column(t.columns[name], t.num_rows)
            vals.extend(list(v)) if isinstance(v, list) else vals.extend(v.tolist())
            valid.extend(ok.tolist())
        dt = parts[0].columns[name].dtype.replace("large_", "")
        arr = vals if dt == "utf8" else np.array(vals, dtype={"f64": np.float64, "i64": np.int64, "i32": np.int32}[dt])
        ocols[name] = O.OColumn(dt, arr, np.array(valid, bool))
    total = sum(t.num_rows for t in parts)
    for a in analyzers[:-1]:
        spec = (type(a).__name__, a.columns[0] if type(a).__name__ == "Entropy" else a.columns)
        ref = O.compute_state(spec, ocols, total)
        m = ctx.metric(a)
        if ref is None:
            assert m.value.isFailure, (a, m)
            continue
        want = ref.metricValue()
        got = m.value.get()
        assert close(got, want, REL, 1e-15) if type(a).__name__ in ("Entropy", "MutualInformation") else (got == want or (math.isnan(got) and math.isnan(want))), (a, got, want)


def test_grouping_state_merge_and_incremental(dq):
    """FrequenciesAndNumRows.sum (outer join adding counts) on the device: merging the states of two
    halves equals the state of the whole; aggregateWith / saveStatesWith through the runner."""
    from deequ_amd.grouping import build_frequencies

    a, b = _group_table(dq, 40_000, 3, chunked=True)
    for cols in (["l"], ["f"], ["s", "i"]):
        whole = build_frequencies([a, b], cols)
        merged = build_frequencies(a, cols).sum(build_frequencies(b, cols))
        assert merged == whole, cols
    prov = dq.InMemoryStateProvider()
    u = dq.Uniqueness("l")
    dq.AnalysisRunner.onData(a).addAnalyzer(u).saveStatesWith(prov).run()
    inc = dq.AnalysisRunner.onData(b).addAnalyzer(u).aggregateWith(prov).run().metric(u).value.get()
    assert inc == dq.AnalysisRunner.onData([a, b]).addAnalyzer(u).run().metric(u).value.get()


def test_grouping_merge_refuses_hash_collisions(dq, monkeypatch):
    """Two tables whose distinct string keys share the first tuple hash (forced by keeping none of its bits)
    must not merge silently: the per-group second hash catches it (DQ_E_UNSUPPORTED); equal tuples still
    merge; a merge of one table with itself adds counts."""
    from deequ_amd import _lib as L
    from deequ_amd.grouping import build_frequencies

    monkeypatch.setenv("DQ_TEST_GROUP_HASH_MASK", "0")  # every tuple's first hash is 0
    ta = dq.Table.from_pydict({"s": ("utf8", ["apple", "apple", None])})
    tb = dq.Table.from_pydict({"s": ("utf8", ["pear", None, "pear", "pear"])})
    tc = dq.Table.from_pydict({"s": ("utf8", ["apple"])})
    fa, fb, fc = (build_frequencies(t, ["s"]) for t in (ta, tb, tc))
    with pytest.raises(L.DQError) as e:
        fa.sum(fb)
    assert "collision" in str(e.value)
    same = fa.sum(fc)  # one group "apple": 2 + 1
    keys, counts = same.frequencies.export()
    assert list(counts) == [3]
    monkeypatch.delenv("DQ_TEST_GROUP_HASH_MASK")
    ok = build_frequencies(ta, ["s"]).sum(build_frequencies(tb, ["s"]))
    assert sorted(ok.frequencies.export()[1].tolist()) == [2, 3]


def test_histogram_reference_cases(dq, kats):
    """AnalyzerTests.scala:200-272: bins of a string column with NULLs, of a numeric column, top-N
    truncation, the maxDetailBins precondition, and a binning UDF (Spark-side, not on the GPU path)."""
    from deequ_amd.metrics import UnsupportedOnGpuPathException

    missing = _device_table(dq, kats["datasets"]["dfMissing"])
    h = dq.Histogram("att1").calculate(missing).value.get()
    assert h.numberOfBins == 3 and set(h.values) == {"a", "b", "NullValue"}
    assert h.values["a"].absolute == 4 and h.values["NullValue"].ratio == 6 / 12
    numeric = _device_table(dq, kats["datasets"]["dfWithNumericValues"])
    h = dq.Histogram("att2").calculate(numeric).value.get()
    assert h.numberOfBins == 4 and len(h.values) == 4 and h.values["0"].absolute == 3
    h = dq.Histogram("att1", None, 2).calculate(missing).value.get()
    assert h.numberOfBins == 3 and set(h.values) == {"a", "NullValue"}
    m = dq.Histogram("att1", None, 1001).calculate(_device_table(dq, kats["datasets"]["dfFull"]))
    assert str(m.value.failed) == "Cannot return histogram values for more than 1000 values"
    m = dq.Histogram("att1", lambda v: v).calculate(missing)
    assert isinstance(m.value.failed, UnsupportedOnGpuPathException)


@pytest.mark.parametrize("n", [1, 4099, 70_001])
def test_histogram_vs_oracle(dq, n):
    """Histogram of f64 (NaN, -0.0, scientific notation), i64, i32, UTF8 and LARGE_UTF8 columns with
    NULLs vs the oracle's CAST-to-string frequencies; with maxDetailBins below the number of bins the
    returned counts are the largest ones."""
    data = _group_table(dq, n, 11 + n)
    host = {name: host_column(c, n) for name, c in data.columns.items()}
    ocols = {name: O.OColumn(data.columns[name].dtype.replace("large_", ""), host[name][0], host[name][1])
             for name in data.columns}
    for col in ("f", "l", "i", "s", "t"):
        want = O.histogram(ocols, col, n)
        h = dq.Histogram(col).calculate(data).value.get()
        assert h.numberOfBins == len(want), (col, h.numberOfBins, len(want))
        top = sorted(want.values(), reverse=True)[:1000]
        assert sorted((v.absolute for v in h.values.values()), reverse=True) == top, col
        for k, v in h.values.items():
            assert want[k] == v.absolute and v.ratio == v.absolute / n, (col, k)
        h5 = dq.Histogram(col, None, 5).calculate(data).value.get()
        assert sorted((v.absolute for v in h5.values.values()), reverse=True) == top[:5], col
