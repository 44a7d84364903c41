"""Check DSL + VerificationSuite over the GPU scan -- the callers of the hot path.

The reference's user entry point for config C1 is VerificationSuite().onData(df).addCheck(check).run()
(VerificationSuite.scala:42-130, VerificationRunBuilder.scala:28-149): the checks' analyzers are unioned
with the required ones, run through AnalysisRunner.doAnalysisRun (ONE fused scan: here dq_plan / dq_scan),
and every constraint's assertion is evaluated on the metrics (Check.scala:878-890,
AnalysisBasedConstraint.scala:42-122).  This module mirrors the constraint methods whose analyzers are on
the GPU path, with the reference's predicate strings (Check.scala:670-871), constraint names
(Constraint.scala:83-536) and failure messages, so a check runs unchanged on the MI355X path.  Grouping
constraints (isUnique, hasUniqueness, hasEntropy, ...) are the reference's grouping pass and are not
mirrored here.
"""
from __future__ import annotations

from enum import IntEnum
from typing import Callable, Dict, List, Optional, Sequence

from .analyzers import (Analyzer, ApproxCountDistinct, Completeness, Compliance, Correlation, Maximum, Mean, Minimum,
                        PatternMatch, Size, StandardDeviation, Sum)
from .grouping import _java_double_to_string
from .runner import AnalysisRunner, AnalyzerContext


class CheckLevel(IntEnum):  # Check.scala:30-32
    Error = 0
    Warning = 1


class CheckStatus(IntEnum):  # Check.scala:34-36 (Enumeration order: Success < Warning < Error)
    Success = 0
    Warning = 1
    Error = 2


class ConstraintStatus(IntEnum):  # Constraint.scala:25-27
    Success = 0
    Failure = 1


MISSING_ANALYSIS = "Missing Analysis, can't run the constraint!"          # AnalysisBasedConstraint.scala:117
PROBLEMATIC_METRIC_PICKER = "Can't retrieve the value to assert on"       # :118
ASSERTION_EXCEPTION = "Can't execute the assertion"                       # :119


class ConstraintResult:  # Constraint.scala:29-33
    def __init__(self, constraint, status: ConstraintStatus, message: Optional[str] = None, metric=None):
        self.constraint, self.status, self.message, self.metric = constraint, status, message, metric

    def __repr__(self):
        return f"ConstraintResult({self.constraint}, {self.status.name}, {self.message!r})"


class AnalysisBasedConstraint:  # AnalysisBasedConstraint.scala:42-111
    def __init__(self, analyzer: Analyzer, assertion: Callable, value_picker: Optional[Callable] = None,
                 hint: Optional[str] = None):
        self.analyzer, self.assertion, self.value_picker, self.hint = analyzer, assertion, value_picker, hint

    def evaluate(self, metric_map: Dict) -> ConstraintResult:
        metric = metric_map.get(self.analyzer)
        if metric is None:
            return ConstraintResult(self, ConstraintStatus.Failure, MISSING_ANALYSIS, None)
        if metric.value.isFailure:
            return ConstraintResult(self, ConstraintStatus.Failure, str(metric.value.failed), metric)
        value = metric.value.get()
        try:
            assert_on = self.value_picker(value) if self.value_picker else value
        except Exception as e:
            return ConstraintResult(self, ConstraintStatus.Failure, f"{PROBLEMATIC_METRIC_PICKER}: {e}!", metric)
        try:
            ok = bool(self.assertion(assert_on))
        except Exception as e:
            return ConstraintResult(self, ConstraintStatus.Failure, f"{ASSERTION_EXCEPTION}: {e}!", metric)
        if ok:
            return ConstraintResult(self, ConstraintStatus.Success, None, metric)
        shown = _java_double_to_string(assert_on) if isinstance(assert_on, float) else str(assert_on)
        msg = f"Value: {shown} does not meet the constraint requirement!"
        if self.hint:
            msg += f" {self.hint}"
        return ConstraintResult(self, ConstraintStatus.Failure, msg, metric)


class NamedConstraint:  # Constraint.scala:40-69 (ConstraintDecorator keeps the name in the result)
    def __init__(self, inner: AnalysisBasedConstraint, name: str):
        self.inner, self.name = inner, name

    def evaluate(self, metric_map: Dict) -> ConstraintResult:
        r = self.inner.evaluate(metric_map)
        r.constraint = self
        return r

    def __str__(self):
        return self.name

    __repr__ = __str__


def _named(analyzer, assertion, kind: str, picker=None, hint=None) -> NamedConstraint:
    return NamedConstraint(AnalysisBasedConstraint(analyzer, assertion, picker, hint), f"{kind}({analyzer})")


def _is_one(v) -> bool:  # Check.IsOne
    return v == 1.0


class CheckResult:  # Check.scala:39-42
    def __init__(self, check: "Check", status: CheckStatus, constraintResults: List[ConstraintResult]):
        self.check, self.status, self.constraintResults = check, status, constraintResults


class Check:  # Check.scala:59-902
    def __init__(self, level: CheckLevel, description: str, constraints: Sequence = ()):
        self.level, self.description, self.constraints = level, description, list(constraints)

    def addConstraint(self, constraint) -> "Check":
        return Check(self.level, self.description, self.constraints + [constraint])

    def _filterable(self, create: Callable[[Optional[str]], NamedConstraint]) -> "CheckWithLastConstraintFilterable":
        return CheckWithLastConstraintFilterable(self.level, self.description, self.constraints + [create(None)], create)

    # ---- constraints on GPU-path analyzers (Constraint.scala factories) ----------------------------
    def hasSize(self, assertion, hint=None):
        return self._filterable(lambda w: _named(Size(w), assertion, "SizeConstraint", lambda v: int(v), hint))

    def isComplete(self, column, hint=None):
        return self._filterable(lambda w: _named(Completeness(column, w), _is_one, "CompletenessConstraint", None, hint))

    def hasCompleteness(self, column, assertion, hint=None):
        return self._filterable(lambda w: _named(Completeness(column, w), assertion, "CompletenessConstraint", None, hint))

    def hasMin(self, column, assertion, hint=None):
        return self._filterable(lambda w: _named(Minimum(column, w), assertion, "MinimumConstraint", None, hint))

    def hasMax(self, column, assertion, hint=None):
        return self._filterable(lambda w: _named(Maximum(column, w), assertion, "MaximumConstraint", None, hint))

    def hasMean(self, column, assertion, hint=None):
        return self._filterable(lambda w: _named(Mean(column, w), assertion, "MeanConstraint", None, hint))

    def hasSum(self, column, assertion, hint=None):
        return self._filterable(lambda w: _named(Sum(column, w), assertion, "SumConstraint", None, hint))

    def hasStandardDeviation(self, column, assertion, hint=None):
        return self._filterable(
            lambda w: _named(StandardDeviation(column, w), assertion, "StandardDeviationConstraint", None, hint))

    def hasApproxCountDistinct(self, column, assertion, hint=None):
        return self._filterable(
            lambda w: _named(ApproxCountDistinct(column, w), assertion, "ApproxCountDistinctConstraint", None, hint))

    def hasCorrelation(self, columnA, columnB, assertion, hint=None):
        return self._filterable(
            lambda w: _named(Correlation(columnA, columnB, w), assertion, "CorrelationConstraint", None, hint))

    def hasPattern(self, column, pattern, assertion=_is_one, name=None, hint=None):  # Check.scala:560-575
        text = pattern if isinstance(pattern, str) else pattern.pattern

        def create(w):  # Constraint.patternMatchConstraint (Constraint.scala:290-312)
            c = AnalysisBasedConstraint(PatternMatch(column, pattern, w), assertion, None, hint)
            return NamedConstraint(c, name or f"PatternMatchConstraint({column}, {text})")
        return self._filterable(create)

    def satisfies(self, columnCondition, constraintName, assertion=_is_one, hint=None):  # Check.scala:538-548
        return self._filterable(lambda w: _named(Compliance(constraintName, columnCondition, w), assertion,
                                                 "ComplianceConstraint", None, hint))

    def isNonNegative(self, column, hint=None):  # Check.scala:670-677
        return self.satisfies(f"COALESCE({column}, 0.0) >= 0", f"{column} is non-negative", hint=hint)

    def isPositive(self, column):  # Check.scala:685-688
        return self.satisfies(f"COALESCE({column}, 1.0) > 0", f"{column} is positive")

    def isLessThan(self, columnA, columnB, hint=None):  # Check.scala:699-707
        return self.satisfies(f"{columnA} < {columnB}", f"{columnA} is less than {columnB}", hint=hint)

    def isLessThanOrEqualTo(self, columnA, columnB, hint=None):
        return self.satisfies(f"{columnA} <= {columnB}", f"{columnA} is less than or equal to {columnB}", hint=hint)

    def isGreaterThan(self, columnA, columnB, hint=None):
        return self.satisfies(f"{columnA} > {columnB}", f"{columnA} is greater than {columnB}", hint=hint)

    def isGreaterThanOrEqualTo(self, columnA, columnB, hint=None):
        return self.satisfies(f"{columnA} >= {columnB}", f"{columnA} is greater than or equal to {columnB}",
                              hint=hint)

    def isContainedIn(self, column, *args, **kw):
        """isContainedIn(column, allowedValues[, assertion][, hint]) (Check.scala:772-842) or
        isContainedIn(column, lowerBound, upperBound, includeLowerBound, includeUpperBound, hint) (:855-871)."""
        if args and isinstance(args[0], (list, tuple)):
            allowed = list(args[0])
            rest = list(args[1:])
            assertion = rest.pop(0) if rest and callable(rest[0]) else kw.get("assertion", _is_one)
            hint = rest.pop(0) if rest else kw.get("hint")
            values = ",".join("'" + v.replace("'", "''") + "'" for v in allowed)
            predicate = f"`{column}` IS NULL OR `{column}` IN ({values})"
            return self.satisfies(predicate, f"{column} contained in {','.join(allowed)}", assertion, hint)
        names = ["lowerBound", "upperBound", "includeLowerBound", "includeUpperBound", "hint"]
        vals = dict(zip(names, args))
        vals.update(kw)
        lo, hi = float(vals["lowerBound"]), float(vals["upperBound"])
        left = ">=" if vals.get("includeLowerBound", True) else ">"
        right = "<=" if vals.get("includeUpperBound", True) else "<"
        los, his = _java_double_to_string(lo), _java_double_to_string(hi)
        predicate = f"`{column}` IS NULL OR (`{column}` {left} {los} AND `{column}` {right} {his})"
        return self.satisfies(predicate, f"{column} between {los} and {his}", hint=vals.get("hint"))

    # ---- evaluation --------------------------------------------------------------------------------
    def evaluate(self, context: AnalyzerContext) -> CheckResult:  # Check.scala:878-890
        results = [c.evaluate(context.metricMap) for c in self.constraints]
        failed = any(r.status == ConstraintStatus.Failure for r in results)
        status = CheckStatus.Success
        if failed:
            status = CheckStatus.Error if self.level == CheckLevel.Error else CheckStatus.Warning
        return CheckResult(self, status, results)

    def requiredAnalyzers(self) -> List[Analyzer]:  # Check.scala:892-901
        out = []
        for c in self.constraints:
            inner = c.inner if isinstance(c, NamedConstraint) else c
            if isinstance(inner, AnalysisBasedConstraint) and inner.analyzer not in out:
                out.append(inner.analyzer)
        return out


class CheckWithLastConstraintFilterable(Check):  # CheckWithLastConstraintFilterable.scala:20-40
    def __init__(self, level, description, constraints, create):
        super().__init__(level, description, constraints)
        self._create = create

    def where(self, filter: str) -> Check:
        return Check(self.level, self.description, self.constraints[:-1] + [self._create(filter)])


class VerificationResult:  # VerificationResult.scala:33-36
    def __init__(self, status: CheckStatus, checkResults: Dict, metrics: Dict):
        self.status, self.checkResults, self.metrics = status, checkResults, metrics

    def successMetricsAsJson(self) -> str:
        return AnalyzerContext(self.metrics).successMetricsAsJson()


class VerificationSuite:  # VerificationSuite.scala:42-282
    def onData(self, data) -> "VerificationRunBuilder":
        return VerificationRunBuilder(data)

    @staticmethod
    def doVerificationRun(data, checks: Sequence[Check], requiredAnalyzers: Sequence[Analyzer] = (),
                          aggregateWith=None, saveStatesWith=None) -> VerificationResult:
        analyzers = list(requiredAnalyzers) + [a for c in checks for a in c.requiredAnalyzers()]
        context = AnalysisRunner.doAnalysisRun(data, analyzers, aggregateWith, saveStatesWith)
        return VerificationSuite._evaluate(checks, context)

    @staticmethod
    def _evaluate(checks, context: AnalyzerContext) -> VerificationResult:  # VerificationSuite.scala:263-281
        results = {c: c.evaluate(context) for c in checks}
        status = max((r.status for r in results.values()), default=CheckStatus.Success)
        return VerificationResult(CheckStatus(status), results, context.metricMap)


class VerificationRunBuilder:  # VerificationRunBuilder.scala:28-149
    def __init__(self, data):
        self.data = data
        self.checks: List[Check] = []
        self.required: List[Analyzer] = []
        self._aggregateWith = None
        self._saveStatesWith = None

    def addCheck(self, check: Check) -> "VerificationRunBuilder":
        self.checks.append(check)
        return self

    def addChecks(self, checks: Sequence[Check]) -> "VerificationRunBuilder":
        self.checks.extend(checks)
        return self

    def addRequiredAnalyzer(self, a: Analyzer) -> "VerificationRunBuilder":
        self.required.append(a)
        return self

    def addRequiredAnalyzers(self, analyzers: Sequence[Analyzer]) -> "VerificationRunBuilder":
        self.required.extend(analyzers)
        return self

    def aggregateWith(self, loader) -> "VerificationRunBuilder":
        self._aggregateWith = loader
        return self

    def saveStatesWith(self, persister) -> "VerificationRunBuilder":
        self._saveStatesWith = persister
        return self

    def run(self) -> VerificationResult:
        return VerificationSuite.doVerificationRun(self.data, self.checks, self.required, self._aggregateWith,
                                                   self._saveStatesWith)
