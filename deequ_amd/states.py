"""Analyzer states (sufficient statistics) -- the Scala State classes, backed by the C ABI.

Field names and `sum` semantics follow (paths relative to src/main/scala/com/amazon/deequ/):
NumMatches analyzers/Size.scala:23-33, NumMatchesAndCount analyzers/Analyzer.scala:220-234,
SumState analyzers/Sum.scala:25-34, MeanState analyzers/Mean.scala:25-34,
StandardDeviationState analyzers/StandardDeviation.scala:25-45, MinState/MaxState
analyzers/Minimum.scala:25-34 / analyzers/Maximum.scala:25-34, CorrelationState
analyzers/Correlation.scala:26-57, ApproxCountDistinctState analyzers/ApproxCountDistinct.scala:26-40,
DataTypeHistogram analyzers/DataType.scala:40-52.
`sum` and `metricValue` call dq_state_merge / dq_state_metric in libdqscan.so, so host-side
merges (StateLoader aggregation, incremental runs) use exactly the library's algebra.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional, Tuple

from . import _lib as L


class State:
    OP = 0

    def _to_c(self) -> L.State:
        s = L.State()
        s.op = self.OP
        s.has_value[0] = s.has_value[1] = 1
        self._fill(s.u)
        return s

    def _fill(self, u):  # pragma: no cover - abstract
        raise NotImplementedError

    def sum(self, other: "State") -> "State":
        if type(other) is not type(self):
            raise TypeError(f"cannot sum {type(self).__name__} with {type(other).__name__}")
        out = L.State()
        L.check(L.lib.dq_state_merge(ctypes.byref(self._to_c()), ctypes.byref(other._to_c()), ctypes.byref(out)))
        return state_from_c(out)

    __add__ = sum

    def metricValue(self) -> float:
        v = ctypes.c_double()
        L.check(L.lib.dq_state_metric(ctypes.byref(self._to_c()), ctypes.byref(v)))
        return v.value


@dataclass(frozen=True)
class NumMatches(State):
    numMatches: int
    OP = L.OP_SIZE

    def _fill(self, u):
        u.size.num_matches = self.numMatches


@dataclass(frozen=True)
class NumMatchesAndCount(State):
    numMatches: int
    count: int
    OP = L.OP_COMPLETENESS

    def _fill(self, u):
        u.ratio.num_matches = self.numMatches
        u.ratio.count = self.count


@dataclass(frozen=True)
class SumState(State):
    sum_: float
    OP = L.OP_SUM

    def _fill(self, u):
        u.sum.sum = self.sum_


@dataclass(frozen=True)
class MeanState(State):
    sum_: float
    count: int
    OP = L.OP_MEAN

    def _fill(self, u):
        u.mean.sum = self.sum_
        u.mean.count = self.count


@dataclass(frozen=True)
class StandardDeviationState(State):
    n: float
    avg: float
    m2: float
    OP = L.OP_STDDEV

    def __post_init__(self):
        if not self.n > 0.0:  # require(n > 0.0) (StandardDeviation.scala:31)
            raise ValueError("requirement failed: Standard deviation is undefined for n = 0.")

    def _fill(self, u):
        u.stddev.n, u.stddev.avg, u.stddev.m2 = self.n, self.avg, self.m2


@dataclass(frozen=True)
class MinState(State):
    minValue: float
    OP = L.OP_MIN

    def _fill(self, u):
        u.minmax.value = self.minValue


@dataclass(frozen=True)
class MaxState(State):
    maxValue: float
    OP = L.OP_MAX

    def _fill(self, u):
        u.minmax.value = self.maxValue


@dataclass(frozen=True)
class CorrelationState(State):
    n: float
    xAvg: float
    yAvg: float
    ck: float
    xMk: float
    yMk: float
    OP = L.OP_CORRELATION

    def __post_init__(self):
        if not self.n > 0.0:  # require(n > 0.0) (Correlation.scala:35)
            raise ValueError("requirement failed: Correlation undefined for n = 0.")

    def _fill(self, u):
        c = u.corr
        c.n, c.x_avg, c.y_avg, c.ck, c.x_mk, c.y_mk = self.n, self.xAvg, self.yAvg, self.ck, self.xMk, self.yMk


@dataclass(frozen=True)
class ApproxCountDistinctState(State):
    words: Tuple[int, ...]
    OP = L.OP_APPROX_COUNT_DISTINCT

    def _fill(self, u):
        for i, w in enumerate(self.words):
            u.hll.words[i] = w

    def __str__(self):
        return f"ApproxCountDistinctState({','.join(str(w) for w in self.words)})"


@dataclass(frozen=True)
class DataTypeHistogram(State):  # DataType.scala:40-52
    numNull: int
    numFractional: int
    numIntegral: int
    numBoolean: int
    numString: int
    OP = L.OP_DATATYPE

    def _fill(self, u):
        d = u.dtype
        d.num_null, d.num_fractional, d.num_integral = self.numNull, self.numFractional, self.numIntegral
        d.num_boolean, d.num_string = self.numBoolean, self.numString

    def metricValue(self) -> float:
        raise TypeError("DataTypeHistogram yields a Distribution (DataTypeHistogram.toDistribution), not a double")


_COMPLIANCE_LIKE = (L.OP_COMPLETENESS, L.OP_COMPLIANCE, L.OP_PATTERN_MATCH)


def state_from_c(s: L.State) -> Optional[State]:
    """fromAggregationResult: the Option[State] an analyzer builds from its Row slots."""
    if not L.lib.dq_state_is_defined(ctypes.byref(s)):
        return None
    u, op = s.u, s.op
    if op == L.OP_SIZE:
        return NumMatches(int(u.size.num_matches))
    if op in _COMPLIANCE_LIKE:
        return NumMatchesAndCount(int(u.ratio.num_matches), int(u.ratio.count))
    if op == L.OP_SUM:
        return SumState(u.sum.sum)
    if op == L.OP_MEAN:
        return MeanState(u.mean.sum, int(u.mean.count))
    if op == L.OP_STDDEV:
        return StandardDeviationState(u.stddev.n, u.stddev.avg, u.stddev.m2)
    if op == L.OP_MIN:
        return MinState(u.minmax.value)
    if op == L.OP_MAX:
        return MaxState(u.minmax.value)
    if op == L.OP_CORRELATION:
        c = u.corr
        return CorrelationState(c.n, c.x_avg, c.y_avg, c.ck, c.x_mk, c.y_mk)
    if op == L.OP_APPROX_COUNT_DISTINCT:
        return ApproxCountDistinctState(tuple(int(w) for w in u.hll.words))
    if op == L.OP_DATATYPE:
        d = u.dtype
        return DataTypeHistogram(int(d.num_null), int(d.num_fractional), int(d.num_integral), int(d.num_boolean),
                                 int(d.num_string))
    raise ValueError(f"unknown op {op}")


def state_to_c(state: State, op: int) -> L.State:
    s = state._to_c()
    s.op = op
    return s


def hll_estimate(words) -> float:
    arr = (ctypes.c_int64 * 52)(*words)
    v = ctypes.c_double()
    L.check(L.lib.dq_hll_estimate(arr, ctypes.byref(v)))
    return v.value
