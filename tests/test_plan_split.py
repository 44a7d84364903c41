"""Analyzer sets over one plan's capacity (the reference fuses ANY number of scan-shareable
analyzers into one data.agg, AnalysisRunner.scala:293-303).

One dq_plan reads at most 64 columns and holds at most 32 distinct predicates, 32 predicate counters, 8 `where`
bitmaps, 256 column tasks and a 96-instruction program (deequ_amd/csrc/dq_device.h).  dq_plan_create splits a
larger set into several fused plans over the same chunks, so a wide ColumnProfiler pass
(ColumnProfiler.scala:112-151) or a VerificationSuite with many Compliance constraints (Check.scala:670-871)
gets every metric instead of a whole-pass failure.

CPU tests: the split as dq_plan_explain shows it (host only).  GPU tests: the split plans' states against the
oracle (bit-exact counts / HLL words / min / max, 1e-12 for fp64 moments).
"""
from __future__ import annotations

import re

import numpy as np
import pytest

import deequ_amd as dq
from deequ_amd import _lib as L
from deequ_amd.runner import explain, gpu_eligible


def _wide_schema(ncols):
    kinds = ["f64", "i64", "i32", "utf8"]
    return [(f"c{k}", kinds[k % 4], True) for k in range(ncols)]


def _profile(schema):
    out = [dq.Size()]
    for name, dtype, _ in schema:
        out += [dq.Completeness(name), dq.ApproxCountDistinct(name)]
        if dtype in ("f64", "i64", "i32"):
            out += [dq.Minimum(name), dq.Maximum(name), dq.Mean(name), dq.StandardDeviation(name), dq.Sum(name)]
    return out


def _compliance40():
    preds = []
    for k in range(40):
        c = f"c{(k % 8) * 4 + (k % 2)}"  # f64 / i64 columns
        preds.append(dq.Compliance(f"p{k}", [f"{c} >= {k - 20}", f"{c} < {3 * k}", f"COALESCE({c}, 0) > {k}",
                                              f"{c} IS NULL OR {c} <= {k * 7}"][k % 4]))
    return preds


def _where12():
    out = []
    for k in range(12):
        w = f"c1 > {k * 10 - 60}"
        out += [dq.Mean("c0", where=w), dq.Maximum(f"c{4 * (k % 3) + 1}", where=w), dq.Completeness("c3", where=w),
                dq.Size(where=w)]
    return out


def _corr_wide(schema):
    """Correlations over 75 numeric columns (f64 / i64 / i32 neighbours) with their Means: > 64 columns, so the
    pair groups land in several plans; each Correlation's two columns stay in one plan."""
    out = []
    for k in range(0, 100, 4):
        a, b, c = f"c{k}", f"c{k + 1}", f"c{k + 2}"
        out += [dq.Correlation(a, b), dq.Correlation(b, c), dq.Correlation(c, a), dq.Mean(a), dq.StandardDeviation(b)]
    return out


def _parts(text):
    m = re.search(r": (\d+) fused plans", text)
    return int(m.group(1)) if m else 1


def _part_members(text):
    return [list(map(int, m.split())) for m in re.findall(r"^analyzers:(.*)$", text, re.M)]


def _part_columns(text):
    return [list(map(int, m.split())) for m in re.findall(r"^columns:(.*)$", text, re.M)]


# ---------------------------------------------------------------------------------------------------------
# host-only: the split dq_plan_create performs, as dq_plan_explain reports it
# ---------------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("case", ["profile100", "compliance40", "where12", "corr100"])
def test_split_explain(case):
    schema = _wide_schema(36 if case in ("compliance40", "where12") else 100)
    analyzers = {"profile100": _profile, "compliance40": lambda s: _compliance40(),
                 "where12": lambda s: _where12(), "corr100": _corr_wide}[case](schema)
    text = explain(analyzers, schema)
    assert _parts(text) >= 2, text[:400]
    members = _part_members(text)
    assert len(members) == _parts(text)
    flat = sorted(i for m in members for i in m)
    assert flat == list(range(len(analyzers)))  # every analyzer in exactly one part
    for cols in _part_columns(text):
        assert 0 < len(cols) <= 64 or not cols
    if case == "profile100":
        # a column's analyzers share a part: each column is read by one part only
        seen = {}
        for k, cols in enumerate(_part_columns(text)):
            for c in cols:
                assert c not in seen, (c, seen.get(c), k)
                seen[c] = k


def test_fitting_set_stays_one_plan():
    schema = _wide_schema(16)
    text = explain(_profile(schema), schema)
    assert text.startswith("plan: ") and "fused plans" not in text


def test_over_deep_predicate_routes_to_fallback():
    """A predicate the device cannot hold by itself (a deeper stack than the predicate pass has) is a
    routing decision (fallback set), not a plan failure for the other analyzers."""
    schema = _wide_schema(8)
    deep = "c0 > 0"
    for k in range(20):
        deep = f"(c1 < {k}) OR ({deep})"
    bad = dq.Compliance("deep", deep)
    assert gpu_eligible(bad, schema) is not None
    assert gpu_eligible(dq.Compliance("ok", "c0 > 0"), schema) is None


# ---------------------------------------------------------------------------------------------------------
# GPU: split plans against the oracle
# ---------------------------------------------------------------------------------------------------------
def _wide_data(ncols, n, seed):
    rng = np.random.default_rng(seed)
    out = []
    for name, dtype, _ in _wide_schema(ncols):
        valid = rng.random(n) >= 0.1
        if dtype == "f64":
            vals = rng.normal(50.0, 30.0, n)
        elif dtype == "i64":
            vals = rng.integers(-100, 100, n)
        elif dtype == "i32":
            vals = rng.integers(-5000, 5000, n).astype(np.int32)
        else:
            vals = [None if not valid[i] else b"s%d" % int(rng.integers(0, 300)) for i in range(n)]
        out.append((name, dtype, vals, valid))
    return out


def _table(data, lo, hi):
    from deequ_amd.table import column_from_numpy, utf8_column

    cols = []
    for name, dtype, vals, valid in data:
        if dtype == "utf8":
            cols.append(utf8_column(name, vals[lo:hi]))
        else:
            cols.append(column_from_numpy(name, dtype, vals[lo:hi], valid[lo:hi]))
    return dq.Table(cols)


def _wide_table(ncols, n, seed):
    return _table(_wide_data(ncols, n, seed), 0, n)


def _oracle_cols(t, n):
    from oracle import dq_oracle as O
    from tests.helpers import host_column

    out = {}
    for name, c in t.columns.items():
        vals, valid, _ = host_column(c, n)
        out[name] = O.OColumn(c.dtype, vals, valid)
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


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["profile100", "compliance40", "where12", "corr100"])
def test_split_states_vs_oracle(case):
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from oracle import dq_oracle as O
    from tests.test_gpu_parity import assert_state_close
    from deequ_amd.runner import ScanPlan, scan_states

    n = 6000 if case in ("profile100", "corr100") else 20011
    data = _wide_data(36 if case in ("compliance40", "where12") else 100, n, seed=len(case))
    t = _table(data, 0, n)
    analyzers = {"profile100": _profile, "compliance40": lambda s: _compliance40(),
                 "where12": lambda s: _where12(), "corr100": _corr_wide}[case](t.schema)
    plan = ScanPlan(analyzers, t.schema)
    try:
        assert plan.num_launches() > 0
    finally:
        plan.close()
    # two chunks: the parts follow the chunk order like a single plan
    half = n // 2
    states = scan_states([_table(data, 0, half), _table(data, half, n)], analyzers)
    cols = _oracle_cols(t, n)
    for a in analyzers:
        ref = O.compute_state(_spec(a), cols, n)
        assert_state_close(states[a], ref, scale=1.0)


@pytest.mark.gpu
def test_split_runner_no_failures():
    """AnalysisRunner over a 100-column profile plus 40 Compliance constraints: every metric succeeds."""
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    t = _wide_table(100, 3000, seed=7)
    analyzers = _profile(t.schema) + _compliance40()
    ctx = dq.AnalysisRunner.onData(t).addAnalyzers(analyzers).run()
    for a in analyzers:
        m = ctx.metric(a)
        assert m is not None and m.value.isSuccess, (a, m)
    # the same values as each analyzer alone (Analyzer.calculate: one plan per analyzer)
    for a in analyzers[::17]:
        single = a.calculate(t).value.get()
        fused = ctx.metric(a).value.get()
        assert single == fused or (single != single and fused != fused), (a, single, fused)


@pytest.mark.gpu
def test_split_set_stream_twice_then_scan():
    """dq_plan_set_stream on a split plan moves every part to the new stream before the parent's own stream is
    destroyed (the parts never own one); setting it twice and scanning gives the oracle's states."""
    import ctypes

    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from oracle import dq_oracle as O
    from tests.test_gpu_parity import assert_state_close
    from deequ_amd.runner import ScanPlan

    n = 5003
    data = _wide_data(36, n, seed=41)
    t = _table(data, 0, n)
    analyzers = _compliance40()
    plan = ScanPlan(analyzers, t.schema)
    try:
        assert "fused plans" in explain(analyzers, t.schema)
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        L.check(L.lib.dq_plan_set_stream(plan.handle, ctypes.c_void_p(s1.cuda_stream)))
        L.check(L.lib.dq_plan_set_stream(plan.handle, ctypes.c_void_p(s2.cuda_stream)))
        torch.cuda.synchronize()  # the table's uploads, on torch's stream, are done before s2 reads them
        plan.scan(t)
        states = [a._from_result(r) for a, r in zip(analyzers, plan.finish())]
    finally:
        plan.close()
    cols = _oracle_cols(t, n)
    for a, s in zip(analyzers, states):
        assert_state_close(s, O.compute_state(_spec(a), cols, n), scale=1.0)


@pytest.mark.gpu
def test_split_scan_rejects_views_before_any_part_scans():
    """A column view that a later part of a split plan rejects fails dq_scan before any part has counted the
    chunk: the same chunk_index can then be scanned with good views, and the states are the oracle's."""
    import ctypes

    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from oracle import dq_oracle as O
    from tests.test_gpu_parity import assert_state_close
    from deequ_amd.runner import ScanPlan

    n = 4099
    data = _wide_data(100, n, seed=43)
    t = _table(data, 0, n)
    analyzers = _profile(t.schema)
    plan = ScanPlan(analyzers, t.schema)
    try:
        views = (L.ColumnView * len(plan.columns))()
        for i, name in enumerate(plan.columns):
            views[i] = t.columns[name].view()
        bad = len(plan.columns) - 1  # read by the last part only
        good = views[bad].values
        views[bad].values = good + 4  # not 16-byte aligned
        rc = L.lib.dq_scan(plan.handle, views, n, 0)
        assert rc == L.DQ_E_INVALID, rc
        views[bad].values = good
        L.check(L.lib.dq_scan(plan.handle, views, n, 0))
        states = [a._from_result(r) for a, r in zip(analyzers, plan.finish())]
    finally:
        plan.close()
    cols = _oracle_cols(t, n)
    for a, s in zip(analyzers, states):
        assert_state_close(s, O.compute_state(_spec(a), cols, n), scale=1.0)
