"""Check DSL / VerificationSuite over the GPU scan (checks/CheckTest.scala, VerificationSuite.scala) and
config C1 (the Item table of examples/entities.scala:19-25 through VerificationSuite).

CPU tests: constraint names, the reference's predicate strings and the status logic on hand-made metric
maps.  GPU tests: the CheckTest cases on the reference's fixtures, and C1 at 10M rows against the C oracle
(counts, min / max bit-exact; mean / stddev within 1e-12 relative).
"""
from __future__ import annotations

import math

import numpy as np
import pytest

from tests.helpers import close


@pytest.fixture(scope="module")
def dq():
    import deequ_amd

    return deequ_amd


def _ctx(dq, pairs):
    from deequ_amd.metrics import DoubleMetric, Entity, Failure, Success
    from deequ_amd.runner import AnalyzerContext

    m = {}
    for a, v in pairs:
        val = Failure(v) if isinstance(v, Exception) else Success(v)
        m[a] = DoubleMetric(Entity.Column, type(a).__name__, getattr(a, "instance", "*"), val)
    return AnalyzerContext(m)


def test_constraint_names_and_predicates(dq):
    """Constraint.scala:83-536 names; Check.scala:670-871 predicate strings (Scala Double.toString bounds)."""
    from deequ_amd.checks import Check, CheckLevel

    c = (Check(CheckLevel.Error, "d").hasSize(lambda n: n == 3).isComplete("att1").isNonNegative("x")
         .isPositive("y").isLessThan("a", "b").isContainedIn("z", 0, 7, includeLowerBound=False)
         .isContainedIn("s", ["a", "b'c"]).hasCorrelation("a", "b", lambda v: True).where("a > 1"))
    names = [str(k) for k in c.constraints]
    assert names == [
        "SizeConstraint(Size(None))",
        "CompletenessConstraint(Completeness(att1,None))",
        "ComplianceConstraint(Compliance(x is non-negative,COALESCE(x, 0.0) >= 0,None))",
        "ComplianceConstraint(Compliance(y is positive,COALESCE(y, 1.0) > 0,None))",
        "ComplianceConstraint(Compliance(a is less than b,a < b,None))",
        "ComplianceConstraint(Compliance(z between 0.0 and 7.0,`z` IS NULL OR (`z` > 0.0 AND `z` <= 7.0),None))",
        "ComplianceConstraint(Compliance(s contained in a,b'c,`s` IS NULL OR `s` IN ('a','b''c'),None))",
        "CorrelationConstraint(Correlation(a,b,Some(a > 1)))",
    ]
    assert len(c.requiredAnalyzers()) == 8


def test_check_status_logic(dq):
    """Check.evaluate (Check.scala:878-890) and AnalysisBasedConstraint messages (:75-111)."""
    from deequ_amd.checks import MISSING_ANALYSIS, Check, CheckLevel, CheckStatus, ConstraintStatus, VerificationSuite
    from deequ_amd.metrics import EmptyStateException

    comp = dq.Completeness("att2")
    ctx = _ctx(dq, [(dq.Completeness("att1"), 1.0), (comp, 0.75), (dq.Size(), 6.0),
                    (dq.Mean("m"), EmptyStateException("Empty state for analyzer Mean(m,None), all input values were NULL."))])
    c1 = Check(CheckLevel.Error, "g1").isComplete("att1").hasCompleteness("att1", lambda v: v == 1.0)
    c2 = Check(CheckLevel.Error, "g2").hasCompleteness("att2", lambda v: v > 0.8)
    c3 = Check(CheckLevel.Warning, "g3").hasCompleteness("att2", lambda v: v > 0.8, hint="too many nulls")
    c4 = Check(CheckLevel.Warning, "g4").hasSize(lambda n: n == 6)
    c5 = Check(CheckLevel.Error, "g5").hasMean("m", lambda v: v > 0)
    c6 = Check(CheckLevel.Error, "g6").hasMax("nosuch", lambda v: True)
    assert c1.evaluate(ctx).status == CheckStatus.Success
    assert c2.evaluate(ctx).status == CheckStatus.Error
    r3 = c3.evaluate(ctx)
    assert r3.status == CheckStatus.Warning
    assert r3.constraintResults[0].message == "Value: 0.75 does not meet the constraint requirement! too many nulls"
    assert c4.evaluate(ctx).status == CheckStatus.Success  # hasSize asserts on the Long value (valuePicker toLong)
    r5 = c5.evaluate(ctx).constraintResults[0]
    assert r5.status == ConstraintStatus.Failure and "all input values were NULL" in r5.message
    assert c6.evaluate(ctx).constraintResults[0].message == MISSING_ANALYSIS
    res = VerificationSuite._evaluate([c1, c3], ctx)
    assert res.status == CheckStatus.Warning
    assert VerificationSuite._evaluate([c1, c2, c3], ctx).status == CheckStatus.Error
    bad = Check(CheckLevel.Error, "g").hasSize(lambda n: 1 / 0)
    assert bad.evaluate(ctx).constraintResults[0].message.startswith("Can't execute the assertion: ")


# ---------------------------------------------------------------------------------------------
# GPU: CheckTest.scala cases on the reference's fixtures, through VerificationSuite
# ---------------------------------------------------------------------------------------------
def _table(dq, kats, name):
    ds = kats["datasets"][name]
    return dq.Table.from_pydict({k: (t, v) for k, (t, v) in ds["columns"].items()})


@pytest.mark.gpu
def test_checktest_cases_on_gpu(dq, kats):
    from deequ_amd.checks import Check, CheckLevel, CheckStatus, VerificationSuite
    from deequ_amd.metrics import UnsupportedOnGpuPathException

    E = CheckLevel.Error
    num = _table(dq, kats, "dfWithNumericValues")
    cases = [  # CheckTest.scala:156-273 (numeric constraints; the string-typed ones are the Spark fallback set)
        (Check(E, "group-1").satisfies("att1 > 0", "rule1"), CheckStatus.Success),
        (Check(E, "group-2-to-fail").satisfies("att1 > 3", "rule2"), CheckStatus.Error),
        (Check(E, "group-2-to-succeed").satisfies("att1 > 3", "rule3", lambda v: v == 0.5), CheckStatus.Success),
        (Check(E, "c1").satisfies("att1 < att2", "rule1").where("att1 > 3"), CheckStatus.Success),
        (Check(E, "c2").satisfies("att2 > 0", "rule2").where("att1 > 0"), CheckStatus.Error),
        (Check(E, "c3").satisfies("att2 > 0", "rule3", lambda v: v == 0.5).where("att1 > 0"), CheckStatus.Success),
        (Check(E, "a").isLessThan("att1", "att2"), CheckStatus.Error),
        (Check(E, "nr1").isContainedIn("att2", 0, 7), CheckStatus.Success),
        (Check(E, "nr2").isContainedIn("att2", 1, 7), CheckStatus.Error),
        (Check(E, "nr3").isContainedIn("att2", 0, 6), CheckStatus.Error),
        (Check(E, "nr4").isContainedIn("att2", 0, 7, includeLowerBound=False, includeUpperBound=False), CheckStatus.Error),
        (Check(E, "nr5").isContainedIn("att2", -1, 8, includeLowerBound=False, includeUpperBound=False), CheckStatus.Success),
        (Check(E, "nr6").isContainedIn("att2", 0, 7, includeLowerBound=True, includeUpperBound=False), CheckStatus.Error),
        (Check(E, "nr7").isContainedIn("att2", 0, 8, includeLowerBound=True, includeUpperBound=False), CheckStatus.Success),
        (Check(E, "nr8").isContainedIn("att2", 0, 7, includeLowerBound=False, includeUpperBound=True), CheckStatus.Error),
        (Check(E, "nr9").isContainedIn("att2", -1, 7, includeLowerBound=False, includeUpperBound=True), CheckStatus.Success),
        # CheckTest.scala:321-340 basic stats
        (Check(E, "s").hasMin("att1", lambda v: v == 1.0).hasMax("att1", lambda v: v == 6.0)
         .hasMean("att1", lambda v: v == 3.5).hasSum("att1", lambda v: v == 21.0)
         .hasStandardDeviation("att1", lambda v: v == 1.707825127659933)
         .hasApproxCountDistinct("att1", lambda v: v == 6.0), CheckStatus.Success),
    ]
    res = dq.VerificationSuite().onData(num).addChecks([c for c, _ in cases]).run()
    for c, want in cases:
        got = res.checkResults[c]
        assert got.status == want, (c.description, [(str(r.constraint), r.message) for r in got.constraintResults])
    assert res.status == CheckStatus.Error
    # one fused scan served every check: each analyzer appears once in the metrics
    assert len(res.metrics) == len({a for c, _ in cases for a in c.requiredAnalyzers()})
    # string-typed predicate (CheckTest.scala:205: isNonNegative("item") on a string column) -> Spark fallback
    r = dq.VerificationSuite().onData(num).addCheck(Check(E, "a").isNonNegative("item")).run()
    m = list(r.metrics.values())[0]
    assert isinstance(m.value.failed, UnsupportedOnGpuPathException)

    comp = _table(dq, {"datasets": {"d": {"columns": {"item": ["utf8", list("123456")],
                                                      "att1": ["utf8", list("abaaba")],
                                                      "att2": ["utf8", ["f", "d", None, "f", None, "f"]]}}}}, "d")
    c1 = Check(E, "group-1").isComplete("att1").hasCompleteness("att1", lambda v: v == 1.0)
    c2 = Check(E, "group-2-E").hasCompleteness("att2", lambda v: v > 0.8)
    c3 = Check(CheckLevel.Warning, "group-2-W").hasCompleteness("att2", lambda v: v > 0.8)
    sz = [Check(E, "S1").hasSize(lambda n: n == 6), Check(E, "E").hasSize(lambda n: n != 6),
          Check(CheckLevel.Warning, "W").hasSize(lambda n: 0 < n < 7)]
    r = dq.VerificationSuite().onData(comp).addChecks([c1, c2, c3] + sz).run()
    assert [r.checkResults[c].status for c in [c1, c2, c3] + sz] == [
        CheckStatus.Success, CheckStatus.Error, CheckStatus.Warning, CheckStatus.Success, CheckStatus.Error,
        CheckStatus.Success]
    # string IN list (CheckTest.scala:227-241) runs on the GPU (whole-value DFA)
    dv = dq.Table.from_pydict({"att1": ("utf8", ["a", "a", None, "b", "c", "c"])})
    rc = [Check(E, "r").isContainedIn("att1", ["a", "b", "c"]), Check(E, "i").isContainedIn("att1", ["a", "b"]),
          Check(E, "f").isContainedIn("att1", ["a"], lambda v: v == 0.5)]
    r = dq.VerificationSuite().onData(dv).addChecks(rc).run()
    assert [r.checkResults[c].status for c in rc] == [CheckStatus.Success, CheckStatus.Error, CheckStatus.Success]
    # correlation checks (CheckTest.scala:342-349)
    inf, uninf = _table(dq, kats, "dfWithConditionallyInformativeColumns"), _table(dq, kats, "dfWithConditionallyUninformativeColumns")
    ci = Check(E, "ci").hasCorrelation("att1", "att2", lambda v: v == 1.0)
    cu = Check(E, "cu").hasCorrelation("att1", "att2", math.isnan)
    assert dq.VerificationSuite().onData(inf).addCheck(ci).run().status == CheckStatus.Success
    assert dq.VerificationSuite().onData(uninf).addCheck(cu).run().status == CheckStatus.Success


@pytest.mark.gpu
def test_c1_item_table_verification_vs_oracle(dq):
    """Config C1: Size, isComplete x 5, Mean / StdDev / Min / Max on id and numViews of a 10M-row Item
    table via VerificationSuite, against the C oracle in Spark partition order."""
    from deequ_amd import synth
    from deequ_amd.checks import CheckStatus
    from oracle import dq_oracle_c as C
    from tests.helpers import host_column

    n = 10_000_000
    t = synth.item_table(n, seed=11)
    check = synth.item_checks()
    res = dq.VerificationSuite().onData(t).addCheck(check).run()
    assert res.status == CheckStatus.Error  # name / description / priority hold NULLs: isComplete fails
    statuses = {str(r.constraint): r.status.name for r in res.checkResults[check].constraintResults}
    assert statuses["CompletenessConstraint(Completeness(id,None))"] == "Success"
    assert statuses["CompletenessConstraint(Completeness(numViews,None))"] == "Success"
    assert statuses["CompletenessConstraint(Completeness(name,None))"] == "Failure"
    got = {(type(a).__name__, getattr(a, "column", None)): m.value.get() for a, m in res.metrics.items()}
    assert got[("Size", None)] == float(n)
    for col, frac in (("name", 0.10), ("description", 0.30), ("priority", 0.10)):
        bm = t.columns[col].validity.cpu().numpy()
        valid = np.unpackbits(bm, bitorder="little")[:n]
        assert got[("Completeness", col)] == float(valid.sum()) / n
        assert abs(got[("Completeness", col)] - (1 - frac)) < 2e-3
    for col in ("id", "numViews"):
        vals, valid, bm = host_column(t.columns[col], n)
        assert got[("Completeness", col)] == 1.0
        s = C.column_stats("i64", vals, bm, None, 16)
        assert got[("Minimum", col)] == s.min and got[("Maximum", col)] == s.max
        assert close(got[("Mean", col)], s.sum_f64 / s.count, 1e-12)
        assert close(got[("StandardDeviation", col)], math.sqrt(s.m2 / s.n), 1e-12)
    ids = host_column(t.columns["id"], n)[0]
    assert np.array_equal(ids, np.arange(n))
    pr = t.columns["priority"]
    offs = pr.offsets.cpu().numpy()[: (n + 1) * 4].view(np.int32)
    data = pr.values.cpu().numpy()[: offs[-1]].tobytes()
    assert {data[offs[i]:offs[i + 1]] for i in range(0, n, n // 1000)} == {b"high", b"low"}
