"""ApproxQuantile / ApproxQuantiles (ApproxQuantile.scala:49-103, ApproxQuantiles.scala:30-105).

CPU: the oracle against the reference's own band tests (AnalyzerTests.scala:533-565) and the
parameter checks' messages (:567-600); the quantile state's digest (serializer layout and round trip as
StateProviderTest.scala:118-139 checks it, IncrementalAnalyzerTest.scala:176-199's merge, GK's rank bound).  GPU (`-m gpu`): dq_approx_quantiles through the C ABI
against the oracle's exact order statistic, bit-exact (it is a selection, no arithmetic), over f64
with NaN / +-inf / -0.0 / nulls, i64, i32, several chunks, all-null and ragged sizes.
"""
from __future__ import annotations

import math

import numpy as np
import pytest

from oracle import dq_oracle as O


def test_oracle_reference_bands():
    v = np.arange(-1000, 1000, dtype=np.int64)  # sparkContext.range(-1000L, 1000L)
    med, q1, q3 = O.approx_quantiles_exact(v, np.ones(len(v), bool), [0.5, 0.25, 0.75])
    assert -20 < med < 20 and -520 < q1 < -480 and 480 < q3 < 520


def test_oracle_order_and_ends():
    f = np.array([np.nan, -0.0, 0.0, -np.inf, np.inf, 1.5, -2.5])
    got = O.approx_quantiles_exact(f, np.ones(7, bool), [0.0, 0.3, 0.45, 0.6, 0.75, 1.0], 0.0)
    assert got[0] == -np.inf and math.copysign(1, got[1]) < 0 and got[1] == 0 and math.copysign(1, got[2]) > 0
    assert got[3] == 1.5 and got[4] == np.inf and math.isnan(got[5])
    # q <= relativeError -> min, q >= 1 - relativeError -> max (QuantileSummaries.query)
    assert O.approx_quantiles_exact(np.arange(100.0), np.ones(100, bool), [0.01, 0.995], 0.01) == [0.0, 99.0]
    assert O.approx_quantiles_exact(np.arange(3.0), np.zeros(3, bool), [0.5]) is None


@pytest.mark.parametrize("q,err,msg", [
    (0.5, 1.1, "Relative error parameter must be in the closed interval [0, 1]. Currently, the value is: 1.1!"),
    (0.5, -0.1, "Relative error parameter must be in the closed interval [0, 1]. Currently, the value is: -0.1!"),
    (-0.1, 0.01, "Quantile parameter must be in the closed interval [0, 1]. Currently, the value is: -0.1!"),
    (1.1, 0.01, "Quantile parameter must be in the closed interval [0, 1]. Currently, the value is: 1.1!"),
])
def test_param_checks(q, err, msg):
    from deequ_amd import ApproxQuantile, ApproxQuantiles
    from deequ_amd.analyzers import Preconditions

    schema = [("att1", "f64", True), ("s", "utf8", True)]
    for a in (ApproxQuantile("att1", q, err), ApproxQuantiles("att1", [0.5, q], err)):
        e = Preconditions.findFirstFailing(schema, a.preconditions())
        assert e is not None and str(e) == msg, (a, e)
    assert Preconditions.findFirstFailing(schema, ApproxQuantile("att1", 0.5).preconditions()) is None
    assert "Expected type of column s" in str(Preconditions.findFirstFailing(schema, ApproxQuantile("s", 0.5).preconditions()))
    assert str(ApproxQuantile("att1", 0.5)) == "ApproxQuantile(att1,0.5,0.01)"


# ---------------------------------------------------------------------------------------------
# GPU parity
# ---------------------------------------------------------------------------------------------
def _f64_data(rng, n):
    x = rng.normal(0, 1e3, n)
    x[rng.random(n) < 0.01] = np.nan
    x[rng.random(n) < 0.01] = np.inf
    x[rng.random(n) < 0.01] = -np.inf
    x[rng.random(n) < 0.02] = -0.0
    x[rng.random(n) < 0.02] = 0.0
    x[rng.random(n) < 0.05] = 12.5  # ties
    return x


QS = [0.0, 0.001, 0.01, 0.1, 0.25, 0.5, 0.75, 0.9, 0.99, 0.999, 1.0]


def _same(a, b):
    return (math.isnan(a) and math.isnan(b)) or (a == b and math.copysign(1, a) == math.copysign(1, b))


@pytest.fixture(scope="module")
def dq():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    import deequ_amd

    return deequ_amd


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 63, 1000, 70_001, 1_000_003])
@pytest.mark.parametrize("dtype", ["f64", "i64", "i32"])
def test_gpu_quantiles_vs_oracle(dq, n, dtype):
    from deequ_amd.table import column_from_numpy

    rng = np.random.default_rng(n * 7 + len(dtype))
    if dtype == "f64":
        v = _f64_data(rng, n)
    elif dtype == "i64":
        v = rng.integers(-(1 << 62), 1 << 62, n, dtype=np.int64)
        v[rng.random(n) < 0.1] = rng.integers(-5, 5)
    else:
        v = rng.integers(-(1 << 31), (1 << 31) - 1, n, dtype=np.int64).astype(np.int32)
    valid = rng.random(n) >= 0.1
    t = dq.Table([column_from_numpy("x", dtype, v, valid)])
    for err in (0.01, 0.0, 0.25):
        want = O.approx_quantiles_exact(v, valid, QS, err)
        m = dq.ApproxQuantiles("x", QS, err).calculate(t)
        if want is None:  # all NULL: ApproxQuantiles keeps Some(digest) -> an empty map (ApproxQuantiles.scala:64-72)
            assert m.value.isSuccess and m.value.get() == {}, m
            assert dq.ApproxQuantile("x", 0.5, err).calculate(t).value.isFailure
            continue
        got = m.value.get()
        for q, w in zip(QS, want):
            key = O_str(q)
            assert _same(got[key], w), (dtype, n, err, q, got[key], w)
        single = dq.ApproxQuantile("x", 0.5, err).calculate(t).value.get()
        assert _same(single, want[QS.index(0.5)])


def O_str(q):
    from deequ_amd.grouping import _java_double_to_string

    return _java_double_to_string(q)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["i64_small", "i32_small", "i64_const", "f64_one_binade", "f64_const", "i64_two"])
def test_gpu_quantiles_skip_equal_digits(dq, case):
    """Columns whose keys agree on whole digits (small-range integers, one binade, a constant): the select skips
    the passes over those digits (known from pass 0's AND / OR of the keys) and still answers every rank exactly,
    over several chunks with nulls."""
    from deequ_amd.table import column_from_numpy

    rng = np.random.default_rng(len(case))
    n = 250_003
    dtype = case.split("_")[0]
    if case == "i64_small":
        v = rng.integers(0, 1000, n, dtype=np.int64)
    elif case == "i32_small":
        v = rng.integers(0, 70_000, n, dtype=np.int64).astype(np.int32)
    elif case == "i64_const":
        v = np.full(n, -7, dtype=np.int64)
    elif case == "i64_two":
        v = rng.choice(np.array([1 << 40, (1 << 40) + 3], dtype=np.int64), n)
    elif case == "f64_one_binade":
        v = 1.0 + rng.random(n)
    else:
        v = np.full(n, 2.5)
    valid = rng.random(n) >= 0.1
    cuts = [0, 7, 100_000, n]
    parts = [dq.Table([column_from_numpy("x", dtype, v[a:b], valid[a:b])]) for a, b in zip(cuts, cuts[1:])]
    for err in (0.0, 0.01):
        want = O.approx_quantiles_exact(v, valid, QS, err)
        got = dq.ApproxQuantiles("x", QS, err).calculate(parts).value.get()
        for q, w in zip(QS, want):
            assert _same(got[O_str(q)], w), (case, err, q, got[O_str(q)], w)


@pytest.mark.gpu
def test_gpu_quantile_constraint_kat(dq):
    """constraints/ConstraintsTest.scala:73-77: approxQuantileConstraint("att1", 0.5, _ == 3.0) succeeds on
    getDfWithNumericValues (att1 = Int 1..6, utils/FixtureSupport.scala:137-148)."""
    from deequ_amd.table import column_from_numpy

    t = dq.Table([column_from_numpy("att1", "i32", np.arange(1, 7, dtype=np.int32), None)])
    assert dq.ApproxQuantile("att1", 0.5).calculate(t).value.get() == 3.0
    assert O.approx_quantiles_exact(np.arange(1, 7), np.ones(6, bool), [0.5], 0.01) == [3.0]


@pytest.mark.gpu
def test_gpu_quantiles_chunks_nulls_and_reference_bands(dq):
    from deequ_amd.table import column_from_numpy

    # AnalyzerTests.scala:533-565 on the device, through the runner
    v = np.arange(-1000, 1000, dtype=np.int64)
    t = dq.Table([column_from_numpy("att1", "i64", v, None)])
    ctx = dq.AnalysisRunner.onData(t).addAnalyzers(
        [dq.ApproxQuantile("att1", 0.5), dq.ApproxQuantile("att1", 0.25), dq.ApproxQuantile("att1", 0.75),
         dq.ApproxQuantile("att1", 1.1), dq.Size()]).run()
    assert -20 < ctx.metric(dq.ApproxQuantile("att1", 0.5)).value.get() < 20
    assert -520 < ctx.metric(dq.ApproxQuantile("att1", 0.25)).value.get() < -480
    assert 480 < ctx.metric(dq.ApproxQuantile("att1", 0.75)).value.get() < 520
    assert ctx.metric(dq.ApproxQuantile("att1", 1.1)).value.isFailure
    # several chunks == one table
    rng = np.random.default_rng(3)
    x = _f64_data(rng, 300_001)
    ok = rng.random(len(x)) >= 0.2
    cuts = [0, 1, 100_000, 100_000, 250_017, len(x)]
    parts = [dq.Table([column_from_numpy("x", "f64", x[a:b], ok[a:b])]) for a, b in zip(cuts, cuts[1:])]
    want = O.approx_quantiles_exact(x, ok, QS, 0.01)
    got = dq.ApproxQuantiles("x", QS).calculate(parts).value.get()
    assert all(_same(got[O_str(q)], w) for q, w in zip(QS, want))
    # all NULL: ApproxQuantile's state is None -> EmptyStateException (ApproxQuantile.scala:72-77), while
    # ApproxQuantiles keeps the digest and getPercentiles of an empty digest is empty -> Success(Map())
    t0 = dq.Table([column_from_numpy("x", "f64", x[:100], np.zeros(100, bool))])
    assert dq.ApproxQuantile("x", 0.5).calculate(t0).value.isFailure
    m = dq.ApproxQuantiles("x", [0.1, 0.5]).calculate(t0)
    assert m.value.isSuccess and m.value.get() == {}, m


# ---- ApproxQuantileState: the GK digest (Spark 2.2.2 QuantileSummaries / PercentileDigestSerializer restated;
# parity unpinned beyond the reference's StateProviderTest / IncrementalAnalyzerTest cases and GK's rank bound)

def _digest(values, valid, err):
    from deequ_amd.quantiles import PercentileDigest, QuantileSummaries, spark_relative_error

    n, sampled = O.gk_digest_exact(values, valid, err)
    return PercentileDigest(QuantileSummaries(10000, spark_relative_error(err), sampled, n))


def test_digest_serializer_layout_and_round_trip():
    from deequ_amd.quantiles import PercentileDigest

    d = _digest(np.array([3.0, -1.0, 2.5]), np.ones(3, bool), 0.01)
    img = d.serialize()
    # compressThreshold int, relativeError double, count long, length int, then (value double, g int, delta int)
    assert img[:4] == (10000).to_bytes(4, "big") and img[12:20] == (3).to_bytes(8, "big")
    assert img[20:24] == (3).to_bytes(4, "big") and len(img) == 24 + 3 * 16
    assert img[24:40] == bytes.fromhex("bff0000000000000") + (1).to_bytes(4, "big") + (0).to_bytes(4, "big")
    back = PercentileDigest.deserialize(img)  # StateProviderTest.assertCorrectlyApproxQuantileState
    s, c = d.quantileSummaries, back.quantileSummaries
    assert (s.compressThreshold, s.relativeError, s.count, s.sampled) == (c.compressThreshold, c.relativeError,
                                                                             c.count, c.sampled)
    with pytest.raises(ValueError):
        PercentileDigest.deserialize(img[:-1])


def test_incremental_merge_reference_case():
    # IncrementalAnalyzerTest.scala:176-199: median of first = (0, 1, 2) merged with second = (-2, -1) is 0.0,
    # the same as over the union
    first = _digest(np.array([0.0, 1.0, 2.0]), np.ones(3, bool), 0.01)
    second = _digest(np.array([-2.0, -1.0]), np.ones(2, bool), 0.01)
    union = _digest(np.array([0.0, 1.0, 2.0, -2.0, -1.0]), np.ones(5, bool), 0.01)
    assert first.merge(second).getPercentiles([0.5]) == [0.0] == union.getPercentiles([0.5])


@pytest.mark.parametrize("err", [0.01, 0.05, 0.2])
def test_digest_queries_within_gk_bound(err):
    rng = np.random.default_rng(int(err * 1000))
    x = rng.normal(size=20_000)
    srt = np.sort(x)
    parts = np.array_split(x, 5)
    single = _digest(x, np.ones(len(x), bool), err)
    merged = _digest(parts[0], np.ones(len(parts[0]), bool), err)
    for p in parts[1:]:
        merged = merged.merge(_digest(p, np.ones(len(p), bool), err))
    n = len(x)
    for q in np.linspace(0.0, 1.0, 41):
        target = min(n, max(1, math.ceil(q * n)))
        for dg, slack in ((single, math.ceil(err * n) + 1), (merged, 2 * math.ceil(err * n) + 1)):
            v = dg.getPercentiles([q])[0]
            lo, hi = np.searchsorted(srt, v, "left") + 1, np.searchsorted(srt, v, "right")
            assert lo - slack <= target <= hi + slack, (err, q, v, lo, hi, target)
    assert merged.quantileSummaries.count == n


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f64", "i64", "i32", "f64_skew"])
def test_gpu_digest_matches_exact_ranks(dq, dtype):
    """Every sample rank of the digest (dq_quantile_digest: splitters from a sample, per-bucket counts, the
    flagged buckets' keys sorted) equals the exact order statistic, over chunks incl. an empty one, with
    nulls; f64_skew puts 60 % of the rows on one value (one bucket far above its share) and the rest on a
    few specials, so the sample-chosen splitters are mostly equal."""
    from deequ_amd.quantiles import device_digest
    from deequ_amd.table import column_from_numpy

    rng = np.random.default_rng(11 + len(dtype))
    n = 123_457
    if dtype == "f64_skew":
        v = rng.choice(np.array([7.25, -0.0, 0.0, np.nan, np.inf, -np.inf, -3.0]), n,
                       p=[0.6, 0.05, 0.05, 0.05, 0.05, 0.05, 0.15])
        v[rng.random(n) < 0.05] = rng.normal(0, 1, n)[:1]  # a few more ties on one drawn value
        dtype = "f64"
    elif dtype == "f64":
        v = _f64_data(rng, n)
    elif dtype == "i64":
        v = rng.integers(-(1 << 40), 1 << 40, n, dtype=np.int64)
    else:
        v = rng.integers(-(1 << 31), (1 << 31) - 1, n, dtype=np.int64).astype(np.int32)
    valid = rng.random(n) >= 0.1
    cuts = [0, 50_000, 50_000, 99_999, n]
    parts = [dq.Table([column_from_numpy("x", dtype, v[a:b], valid[a:b])]) for a, b in zip(cuts, cuts[1:])]
    for err in (0.0, 1e-5, 0.001, 0.01, 0.1, 0.5):  # 0: every value sampled (one sort answers all ranks)
        got = device_digest(parts, "x", err).quantileSummaries
        cnt, want = O.gk_digest_exact(v, valid, err)
        assert got.count == cnt and len(got.sampled) == len(want)
        assert all(_same(a[0], b[0]) and a[1:] == b[1:] for a, b in zip(got.sampled, want)), (dtype, err)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 63, 513, 2049, 16_385, 16_387])
def test_gpu_digest_small_and_ragged(dq, n):
    """Sizes around the digest's sample (16 K rows) and bucket (2048) counts, one chunk and split into three
    (the last one ragged), with nulls: every sample rank equals the exact order statistic."""
    from deequ_amd.quantiles import device_digest
    from deequ_amd.table import column_from_numpy

    rng = np.random.default_rng(n)
    for dtype in ("f64", "i64"):
        v = _f64_data(rng, n) if dtype == "f64" else rng.integers(-50, 50, n, dtype=np.int64)
        valid = rng.random(n) >= 0.1
        valid[0] = True
        cuts = [0, n // 3, n - n // 5, n]
        whole = dq.Table([column_from_numpy("x", dtype, v, valid)])
        parts = [dq.Table([column_from_numpy("x", dtype, v[a:b], valid[a:b])]) for a, b in zip(cuts, cuts[1:])]
        for err in (0.0, 0.001, 0.01, 0.3):
            cnt, want = O.gk_digest_exact(v, valid, err)
            for data in (whole, parts):
                got = device_digest(data, "x", err).quantileSummaries
                assert got.count == cnt and len(got.sampled) == len(want), (dtype, n, err)
                assert all(_same(a[0], b[0]) and a[1:] == b[1:] for a, b in zip(got.sampled, want)), (dtype, n, err)


@pytest.mark.gpu
@pytest.mark.parametrize("budget", [700, 50_000])
def test_gpu_digest_bounded_batches(dq, monkeypatch, budget):
    """The digest's compaction runs in batches of at most DQ_DIGEST_CAND_BUDGET candidates (scratch bounded
    whatever the relative error): small budgets force many batches -- relativeError 1e-5 flags every bucket
    (m > 2048 samples), the skewed column's hot value is answered from its bucket's lower splitter -- and every
    sample rank is still the exact order statistic."""
    from deequ_amd.quantiles import device_digest
    from deequ_amd.table import column_from_numpy

    monkeypatch.setenv("DQ_DIGEST_CAND_BUDGET", str(budget))
    rng = np.random.default_rng(budget)
    n = 200_003
    for kind in ("f64", "skew", "i64"):
        if kind == "f64":
            v, dtype = _f64_data(rng, n), "f64"
        elif kind == "skew":
            v, dtype = rng.choice(np.array([7.25, -1.0, 3.5]), n, p=[0.9, 0.05, 0.05]), "f64"
            v[rng.random(n) < 0.02] = rng.normal(0, 1, n)[rng.random(n) < 0.02][:1]
        else:
            v, dtype = rng.integers(-1000, 1000, n, dtype=np.int64), "i64"
        valid = rng.random(n) >= 0.1
        t = dq.Table([column_from_numpy("x", dtype, v, valid)])
        for err in (1e-5, 0.001, 0.05):
            cnt, want = O.gk_digest_exact(v, valid, err)
            got = device_digest(t, "x", err).quantileSummaries
            assert got.count == cnt and len(got.sampled) == len(want), (kind, err)
            assert all(_same(a[0], b[0]) and a[1:] == b[1:] for a, b in zip(got.sampled, want)), (kind, err)


@pytest.mark.gpu
def test_gpu_digest_over_budget_bucket_falls_back(dq, monkeypatch):
    """One bucket with more distinct candidates than the budget: UnsupportedOnGpuPathException (the analyzer goes
    to the fallback set), not a bare DQError; and the device memory the digest held is returned (its pool keeps
    at most 256 MB; torch's own pool settings are untouched)."""
    import torch

    from deequ_amd import quantiles as Q
    from deequ_amd.metrics import UnsupportedOnGpuPathException
    from deequ_amd.table import column_from_numpy

    x = np.random.default_rng(5).normal(size=100_000)
    t = dq.Table([column_from_numpy("x", "f64", x, np.ones(len(x), bool))])
    monkeypatch.setenv("DQ_DIGEST_CAND_BUDGET", "10")
    with pytest.raises(UnsupportedOnGpuPathException):
        Q.device_digest(t, "x", 0.01)
    monkeypatch.delenv("DQ_DIGEST_CAND_BUDGET")
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    big = dq.Table([column_from_numpy("x", "f64", np.random.default_rng(6).normal(size=20_000_000),
                                      np.ones(20_000_000, bool))])
    free1 = torch.cuda.mem_get_info()[0]
    Q.device_digest(big, "x", 1e-6)  # every bucket flagged: ~20 M candidates (~0.5 GB of scratch)
    torch.cuda.synchronize()
    free2 = torch.cuda.mem_get_info()[0]
    assert free1 - free2 <= (256 << 20) + (64 << 20), (free0, free1, free2)


@pytest.mark.gpu
def test_gpu_digest_sample_limit(dq, monkeypatch):
    """relativeError 0 keeps every value (as Spark's GK does); past MAX_DIGEST_SAMPLES the GPU path refuses
    with UnsupportedOnGpuPathException (the analyzer goes to the Spark fallback) instead of building a digest
    the host cannot hold."""
    from deequ_amd import quantiles as Q
    from deequ_amd.metrics import UnsupportedOnGpuPathException
    from deequ_amd.table import column_from_numpy

    x = np.random.default_rng(3).normal(size=5000)
    t = dq.Table([column_from_numpy("x", "f64", x, np.ones(len(x), bool))])
    got = Q.device_digest(t, "x", 0.0).quantileSummaries
    assert got.count == len(x) and [s[0] for s in got.sampled] == sorted(x.tolist())
    monkeypatch.setattr(Q, "MAX_DIGEST_SAMPLES", 4096)
    with pytest.raises(UnsupportedOnGpuPathException):
        Q.device_digest(t, "x", 0.0)
    assert len(Q.device_digest(t, "x", 0.001).quantileSummaries.sampled) == 501


@pytest.mark.gpu
def test_gpu_quantile_state_persist_load_and_aggregate(dq, tmp_path):
    from deequ_amd.quantiles import ApproxQuantileState
    from deequ_amd.state_provider import HdfsStateProvider, InMemoryStateProvider
    from deequ_amd.table import column_from_numpy

    rng = np.random.default_rng(5)
    x = rng.normal(size=40_000)
    ok = rng.random(len(x)) >= 0.05
    a_t = dq.Table([column_from_numpy("price", "f64", x[:25_000], ok[:25_000])])
    b_t = dq.Table([column_from_numpy("price", "f64", x[25_000:], ok[25_000:])])
    an = dq.ApproxQuantile("price", 0.5)
    hdfs = HdfsStateProvider(str(tmp_path / "q"), allowOverwrite=True)
    mem = InMemoryStateProvider()
    for prov in (hdfs, mem):
        m_a = an.calculate(a_t, saveStatesWith=prov)
        st = prov.load(an)
        assert isinstance(st, ApproxQuantileState) and st == an.computeStateFrom(a_t)
        assert m_a.value.get() == st.percentileDigest.getPercentiles([0.5])[0]
        # the second batch aggregated with the first: the metric of the merged digest
        m_ab = an.calculate(b_t, aggregateWith=prov)
        merged = an.computeStateFrom(b_t).sum(st)
        assert m_ab.value.get() == merged.percentileDigest.getPercentiles([0.5])[0]
        srt = np.sort(x[ok])
        rank = np.searchsorted(srt, m_ab.value.get()) + 1
        assert abs(rank - math.ceil(0.5 * len(srt))) <= 2 * math.ceil(0.01 * len(srt)) + 1
    qs = dq.ApproxQuantiles("price", [0.1, 0.9])
    m = qs.calculate(a_t, saveStatesWith=mem)
    assert set(m.value.get()) == {"0.1", "0.9"} and isinstance(mem.load(qs), ApproxQuantileState)
    # all NULL: ApproxQuantile's state is None (EmptyStateException), ApproxQuantiles' an empty digest
    t0 = dq.Table([column_from_numpy("price", "f64", x[:10], np.zeros(10, bool))])
    assert an.calculate(t0, saveStatesWith=InMemoryStateProvider()).value.isFailure
    m0 = qs.calculate(t0, saveStatesWith=InMemoryStateProvider())
    assert m0.value.isSuccess and m0.value.get() == {}
