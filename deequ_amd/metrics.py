"""Metric types and failure semantics.

Mirrors metrics/Metric.scala:21-68 (Entity, DoubleMetric), metrics/HistogramMetric.scala:21-61
(DistributionValue, Distribution, HistogramMetric) and
analyzers/runners/MetricCalculationException.scala:19-78 plus the EmptyStateException message
of analyzers/Analyzer.scala:420-422 (paths relative to src/main/scala/com/amazon/deequ/).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from enum import Enum
from typing import Dict, Optional


class Entity(Enum):  # Metric.scala:21-23 (the typo "Mutlicolumn" is the reference's)
    Dataset = "Dataset"
    Column = "Column"
    Mutlicolumn = "Mutlicolumn"


class MetricCalculationException(Exception):
    pass


class MetricCalculationRuntimeException(MetricCalculationException):
    pass


class MetricCalculationPreconditionException(MetricCalculationException):
    pass


class EmptyStateException(MetricCalculationRuntimeException):
    pass


class NoSuchColumnException(MetricCalculationPreconditionException):
    pass


class WrongColumnTypeException(MetricCalculationPreconditionException):
    pass


class NoColumnsSpecifiedException(MetricCalculationPreconditionException):
    pass


class NumberOfSpecifiedColumnsException(MetricCalculationPreconditionException):
    pass


class IllegalAnalyzerParameterException(MetricCalculationException):  # analyzers/Analyzer.scala (Histogram PARAM_CHECK)
    pass


class UnsupportedOnGpuPathException(MetricCalculationRuntimeException):
    """The analyzer (or its predicate) is outside the GPU-eligible set; a Spark shim keeps such
    analyzers on data.agg (fallback set).  This host has no Spark, so it surfaces as a
    failure metric instead of silently computing anything on the CPU."""


def wrap_if_necessary(e: BaseException) -> MetricCalculationException:
    """MetricCalculationException.wrapIfNecessary (MetricCalculationException.scala:69-76)."""
    if isinstance(e, MetricCalculationException):
        return e
    w = MetricCalculationRuntimeException(str(e))
    w.__cause__ = e
    return w


class Try:
    """scala.util.Try: Success(value) or Failure(exception)."""

    __slots__ = ("_value", "_error")

    def __init__(self, value=None, error: Optional[BaseException] = None):
        self._value = value
        self._error = error

    @property
    def isSuccess(self) -> bool:
        return self._error is None

    @property
    def isFailure(self) -> bool:
        return self._error is not None

    def get(self):
        if self._error is not None:
            raise self._error
        return self._value

    @property
    def failed(self) -> BaseException:
        if self._error is None:
            raise ValueError("Success.failed")
        return self._error

    def __eq__(self, other):
        if not isinstance(other, Try):
            return NotImplemented
        if self.isSuccess and other.isSuccess:
            a, b = self._value, other._value
            if isinstance(a, float) and isinstance(b, float) and math.isnan(a) and math.isnan(b):
                return False  # NaN != NaN, as for Scala Doubles inside Success
            return a == b
        if self.isFailure and other.isFailure:
            return type(self._error) is type(other._error) and str(self._error) == str(other._error)
        return False

    def __repr__(self):
        return f"Success({self._value!r})" if self.isSuccess else f"Failure({self._error!r})"


def Success(v) -> Try:
    return Try(value=v)


def Failure(e: BaseException) -> Try:
    return Try(error=e)


@dataclass(eq=True)
class DoubleMetric:  # Metric.scala:41-49
    entity: Entity
    name: str
    instance: str
    value: Try

    def flatten(self):
        return [self]


@dataclass(frozen=True)
class DistributionValue:  # HistogramMetric.scala:21
    absolute: int
    ratio: float


@dataclass(eq=True)
class Distribution:  # HistogramMetric.scala:23-35
    values: Dict[str, DistributionValue]
    numberOfBins: int

    def __getitem__(self, key: str) -> DistributionValue:
        return self.values[key]

    def argmax(self) -> str:
        return max(self.values.items(), key=lambda kv: kv[1].absolute)[0]


@dataclass(eq=True)
class HistogramMetric:  # HistogramMetric.scala:37-61
    column: str
    value: Try
    entity: Entity = Entity.Column
    name: str = "Histogram"

    @property
    def instance(self) -> str:
        return self.column

    def flatten(self):
        if self.value.isFailure:
            return [DoubleMetric(self.entity, f"{self.name}.bins", self.instance, self.value)]
        d = self.value.get()
        out = [DoubleMetric(self.entity, f"{self.name}.bins", self.instance, Success(float(d.numberOfBins)))]
        for key, v in d.values.items():
            out.append(DoubleMetric(self.entity, f"{self.name}.abs.{key}", self.instance, Success(float(v.absolute))))
            out.append(DoubleMetric(self.entity, f"{self.name}.ratio.{key}", self.instance, Success(v.ratio)))
        return out


@dataclass(eq=True)
class KeyedDoubleMetric:  # Metric.scala:51-63 (ApproxQuantiles: quantile.toString -> value)
    entity: Entity
    name: str
    instance: str
    value: Try

    def flatten(self):
        if self.value.isSuccess:
            return [DoubleMetric(self.entity, f"name-{k}", self.instance, Success(v))  # the reference's literal s"name-$key"
                    for k, v in self.value.get().items()]
        return [DoubleMetric(self.entity, "name", self.instance, self.value)]
