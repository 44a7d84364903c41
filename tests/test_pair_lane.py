"""The Correlation pass fused with the column moments (deequ_amd/csrc/dq_pair.hip): the VALU co-moment pass
(dq_pair_scan: per <= 8-column pair group two waves, a 14-slot pattern whose two rotations are the 28 pairs,
fp64 groups staged HBM -> LDS by global_load_lds in a ring of two-group slots) and its checked re-run of
non-finite ranges (dq_pair_redo).

Correlation co-moments (Correlation.scala:37-52) and the Mean / StandardDeviation / Sum / Minimum /
Maximum states of the same columns are computed in ONE read of each column.  Checked against the C
oracle (Spark partition order) on: nulls, `where` filters, f64 / i64 / i32 columns (the mixed-kind groups
take the register-staged fold), NaN / +-inf values, pairs in both orientations, ragged sizes around the
64-row groups and the two-group ring slots, columns drifting far from their first values (the per-range
shift), a complete 8-column pair set (C4's 28 correlations, bitwise deterministic across runs) plus pairs
on columns without moments.
"""
from __future__ import annotations

import math

import numpy as np
import pytest

from oracle import dq_oracle as O
from oracle import dq_oracle_c as C
from tests.helpers import close

pytestmark = pytest.mark.gpu
REL = 1e-12


@pytest.fixture(scope="module")
def dq():
    import torch

    assert torch.cuda.is_available()
    import deequ_amd

    return deequ_amd


def _data(n, seed, special=False):
    rng = np.random.default_rng(seed)
    cols = {}
    z0 = rng.normal(size=n)
    for c in range(6):
        x = 0.4 * z0 + rng.normal(size=n) + 100.0 * c
        cols[f"f{c}"] = ("f64", x, rng.random(n) > 0.1 * (c % 3))
    cols["l"] = ("i64", rng.integers(-(1 << 40), 1 << 40, n), rng.random(n) > 0.2)
    cols["i"] = ("i32", rng.integers(-50000, 50000, n).astype(np.int32), np.ones(n, bool))
    cols["w"] = ("i64", rng.integers(-3, 10, n), rng.random(n) > 0.05)
    if special and n > 10:
        f = cols["f1"][1]
        f[rng.integers(0, n, 3)] = np.nan
        f[rng.integers(0, n, 2)] = np.inf
        f[rng.integers(0, n, 1)] = -np.inf
    return cols


def _table(dq, cols):
    from deequ_amd.table import column_from_numpy

    return dq.Table([column_from_numpy(k, t, v, m, nullable=not m.all() or k != "i") for k, (t, v, m) in cols.items()])


def _bm(valid):
    return np.packbits(valid, bitorder="little")


def _analyzers(dq, where):
    names = [f"f{c}" for c in range(6)] + ["l", "i"]
    out = [dq.Correlation(names[i], names[j], where) for i in range(8) for j in range(i + 1, 8)]
    out += [dq.Correlation("f3", "f0", where), dq.Correlation("i", "f5", where)]  # reversed orientations
    for c in names:
        out += [dq.Mean(c, where), dq.StandardDeviation(c, where), dq.Minimum(c, where), dq.Maximum(c, where),
                dq.Sum(c, where)]
    return out


def _check(dq, cols, states, analyzers, n, where_mask):
    mask = None if where_mask is None else _bm(where_mask)
    for a in analyzers:
        got = states[a]
        name = type(a).__name__
        if name == "Correlation":
            (kx, x, vx), (ky, y, vy) = cols[a.firstColumn], cols[a.secondColumn]
            r = C.corr(kx, x, _bm(vx), ky, y, _bm(vy), mask, 4)
            if r[0] == 0:
                assert got is None or got.n == 0, (a, got)
                continue
            ref = O.CorrelationState(*r)
            assert got.n == ref.n, (a, got, ref)
            g, w = got.metricValue(), ref.metricValue()
            assert close(g, w, 0.0, 1e-12) or (math.isnan(g) and math.isnan(w)), (a, g, w)
            if math.isnan(w):  # a NaN / inf in the pair: the other state fields depend on Spark's row order
                continue
            for k in ("xAvg", "yAvg"):
                scale = abs(getattr(ref, k)) + math.sqrt(abs(ref.xMk) / ref.n + abs(ref.yMk) / ref.n)
                assert close(getattr(got, k), getattr(ref, k), REL, REL * scale), (a, k, got, ref)
            continue
        kind, v, valid = cols[a.column]
        s = C.column_stats(kind, v, _bm(valid), mask, 4)
        if s.count == 0:
            assert got is None, (a, got)
            continue
        fin = valid & (np.ones(len(v), bool) if where_mask is None else where_mask)
        scale = float(np.abs(v.astype(np.float64)[fin & np.isfinite(v.astype(np.float64))]).sum())
        if name == "Mean":
            assert got.count == s.count and close(got.sum_, s.sum_f64, REL, REL * scale), (a, got, s.sum_f64)
        elif name == "Sum":
            assert close(got.sum_, s.sum_f64, REL, REL * scale), (a, got, s.sum_f64)
        elif name == "StandardDeviation":
            assert got.n == s.n, (a, got.n, s.n)
            g, w = got.metricValue(), math.sqrt(s.m2 / s.n) if s.m2 == s.m2 else float("nan")
            assert close(g, w, REL) or (math.isnan(g) and math.isnan(w)), (a, g, w)
        elif name == "Minimum":
            assert got.metricValue() == s.min or (math.isnan(got.metricValue()) and math.isnan(s.min)), (a, got, s.min)
        elif name == "Maximum":
            assert got.metricValue() == s.max or (math.isnan(got.metricValue()) and math.isnan(s.max)), (a, got, s.max)


@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 127, 128, 129, 255, 256, 257, 511, 2047, 2049, 16_385, 100_003])
@pytest.mark.parametrize("where", [None, "w > 2"])
def test_pair_pass_vs_oracle(dq, n, where):
    from deequ_amd.runner import scan_states

    cols = _data(n, n * 3 + (where is not None), special=(n % 2 == 1))
    t = _table(dq, cols)
    an = _analyzers(dq, where)
    states = scan_states(t, an)
    wm = None
    if where is not None:
        wv, wvalid = cols["w"][1], cols["w"][2]
        wm = wvalid & (wv > 2)
    _check(dq, cols, states, an, n, wm)


def test_pair_pass_fuses_moments(dq):
    """The planner routes every pair group and its stats-only column tasks to the pair pass: one pair launch
    + finalize, no column pass; results vs the oracle."""
    from deequ_amd.runner import ScanPlan, scan_states

    n = 300_001
    cols = _data(n, 7)
    t = _table(dq, cols)
    an = _analyzers(dq, None)
    plan = ScanPlan(an, t.schema)
    launches = plan.num_launches()
    plan.close()
    assert launches == 2, launches  # the pair pass + finalize: moments fused, no column pass
    _check(dq, cols, scan_states(t, an), an, n, None)


def test_c4_complete_pair_set_deterministic(dq):
    from deequ_amd import synth
    from deequ_amd.runner import scan_results

    t = synth.c4_table(1_000_003, seed=21)
    names = list(t.columns)
    an = [dq.Correlation(names[i], names[j]) for i in range(8) for j in range(i + 1, 8)]
    an += [dq.Mean(c) for c in names] + [dq.StandardDeviation(c) for c in names]
    runs = [[bytes(s) for s in scan_results(t, an)] for _ in range(2)]
    assert runs[0] == runs[1]


def _f64_only(n, seed, special):
    rng = np.random.default_rng(seed)
    z0 = rng.normal(size=n)
    cols = {}
    for c in range(8):
        cols[f"f{c}"] = ("f64", 0.5 * z0 + rng.normal(size=n) + 10.0 * c, rng.random(n) > 0.1 * (c % 3))
    cols["w"] = ("i64", rng.integers(-3, 10, n), rng.random(n) > 0.05)
    if special and n > 10:
        for name, k in (("f2", 0), ("f6", 1)):
            f = cols[name][1]
            f[rng.integers(0, n, 2 + k)] = np.nan
            f[rng.integers(0, n, 1)] = np.inf
            f[rng.integers(0, n, 1 + k)] = -np.inf
    return cols


@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 255, 256, 257, 4095, 4097, 100_003])
@pytest.mark.parametrize("where", [None, "w > 2"])
def test_all_f64_pair_pass_vs_oracle(dq, n, where):
    """All-fp64 pair groups (the LDS-DMA staged pass) vs the oracle with NaN / +-inf, `where`, and sizes
    around the 64-row group and the 256-row tile."""
    from deequ_amd.runner import scan_states
    from deequ_amd.table import column_from_numpy

    cols = _f64_only(n, n * 5 + 11 + (where is not None), special=(n % 2 == 1))
    tbl = dq.Table([column_from_numpy(k, t, v, m) for k, (t, v, m) in cols.items()])
    names = [f"f{c}" for c in range(8)]
    an = [dq.Correlation(names[i], names[j], where) for i in range(8) for j in range(i + 1, 8)]
    for c in names:
        an += [dq.Mean(c, where), dq.StandardDeviation(c, where), dq.Minimum(c, where), dq.Maximum(c, where),
               dq.Sum(c, where)]
    states = scan_states(tbl, an)
    wm = None
    if where is not None:
        wm = cols["w"][2] & (cols["w"][1] > 2)
    _check(dq, cols, states, an, n, wm)


@pytest.mark.parametrize("n", [4097, 200_003])
def test_pair_pass_drift_and_offset_columns(dq, n):
    """Columns whose first rows are not representative of the rest: a linear trend around 1e9, a sorted
    column, a large offset with unit noise, and a first 64 / 128-row block far from everything after it (the
    pass's shifted sums take their shift from a range's first rows).  Correlation, Mean and StandardDeviation
    vs a double-double exact reference (oracle/c dqo_exact_*).  Mean: the north-star 1e-12.  Correlation and
    StandardDeviation: 1e-12, or the error of Spark's own algorithm on one partition (the oracle's row-by-row
    updates, StatefulCorrelation.scala:24-49, StandardDeviation.scala:37-44) where that is larger: both
    states keep the means (Correlation.scala:26-57), so a column far from zero relative to its spread loses
    digits in every merge of ranges / partitions (Chan, Correlation.scala:37-52) -- `offset` (1e12 + N(0, 1),
    ulp 1.2e-4 of the spread: ~1e-4 relative) and `trend` (1e9 + i at n = 4097: Spark's order is off by
    4e-11 on Correlation(trend, step128) and 8e-10 on its StandardDeviation) -- and the bar there is: no
    worse than the reference's own order."""
    import math
    from fractions import Fraction

    from deequ_amd.runner import scan_states
    from deequ_amd.table import column_from_numpy

    rng = np.random.default_rng(n)
    i = np.arange(n, dtype=np.float64)
    noise = rng.normal(size=n)
    cols = {"trend": 1e9 + i, "sorted": np.sort(rng.normal(0, 1000, n)), "offset": 1e12 + noise,
            "step64": np.where(i < 64, 0.0, 1e9 + noise), "step128": np.where(i < 128, -1e6, 3e8 + 0.5 * i + noise),
            "mixed": 0.5 * (1e9 + i) + 3.0 * noise}
    valid = {k: rng.random(n) > 0.05 for k in cols}
    tbl = dq.Table([column_from_numpy(k, "f64", v, valid[k]) for k, v in cols.items()])
    names = list(cols)
    an = [dq.Correlation(names[a], names[b]) for a in range(len(names)) for b in range(a + 1, len(names))]
    for c in names:
        an += [dq.Mean(c), dq.StandardDeviation(c)]
    got = scan_states(tbl, an)
    bm = {k: _bm(v) for k, v in valid.items()}
    piv = {k: float(v[np.argmax(valid[k])]) for k, v in cols.items()}

    def dd(p):
        return Fraction(p[0]) + Fraction(p[1])

    for a in an:
        st = got[a]
        if type(a).__name__ == "Correlation":
            x, y = a.firstColumn, a.secondColumn
            r = C.exact_comoments("f64", cols[x], bm[x], "f64", cols[y], bm[y], piv[x], piv[y], 8)
            m = r[0]
            sx, sy, sxy, sxx, syy = (dd(q) for q in r[1:])
            ck, xm, ym = sxy - sx * sy / m, sxx - sx * sx / m, syy - sy * sy / m
            exact = float(ck) / math.sqrt(float(xm) * float(ym))
            assert st.n == m
            o = C.corr("f64", cols[x], bm[x], "f64", cols[y], bm[y], None, 1)  # Spark's order, one partition
            bar = max(1e-12, abs(o[3] / math.sqrt(o[4] * o[5]) - exact))
            assert abs(st.metricValue() - exact) <= bar, (a, st.metricValue(), exact, bar)
        else:
            c = a.column
            m, s1, s2 = C.exact_moments("f64", cols[c], bm[c], piv[c], 8)
            mean = Fraction(piv[c]) + dd(s1) / m
            if type(a).__name__ == "Mean":
                assert st.count == m and abs(st.metricValue() - float(mean)) <= 1e-12 * abs(float(mean)), a
            else:
                sd = math.sqrt(float((dd(s2) - dd(s1) ** 2 / m) / m))
                o = C.column_stats("f64", cols[c], bm[c])  # Spark's order, one partition
                bar = max(1e-12 * sd, abs(math.sqrt(o.m2 / o.n) - sd))
                assert st.n == m and abs(st.metricValue() - sd) <= bar, (a, st.metricValue(), sd, bar)
