"""ApproxQuantile / ApproxQuantiles (ApproxQuantile.scala:49-103, ApproxQuantiles.scala:30-105) on the GPU.

The reference aggregates the column into Spark 2.2's ApproximatePercentile digest (Greenwald-Khanna,
order-dependent) and answers PercentileDigest.getPercentiles.  Here one device pass family
(dq_approx_quantiles: MSD radix select, six HBM-streaming histogram passes) returns the exact order
statistic of rank ceil(q * n) (min / max at the two ends, as QuantileSummaries.query), which lies inside
the error bound GK guarantees -- the property the reference's own tests check
(AnalyzerTests.scala:533-565).  The digest is not materialised as a state: aggregateWith /
saveStatesWith of a quantile analyzer are reported as failures of that metric.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Sequence

from . import _lib as L
from .analyzers import Analyzer, Preconditions, data_schema
from .grouping import _TYPES, _java_double_to_string
from .metrics import (DoubleMetric, EmptyStateException, Entity, Failure, IllegalAnalyzerParameterException,
                      KeyedDoubleMetric, Success, wrap_if_necessary)


def _param_msg(kind: str, v: float) -> str:  # MetricCalculationException.getApproxQuantileIllegal*Message
    return f"{kind} parameter must be in the closed interval [0, 1]. Currently, the value is: {_java_double_to_string(v)}!"


def device_quantiles(data, column: str, quantiles: Sequence[float], relative_error: float) -> List[float] | None:
    """dq_approx_quantiles over every chunk of `data`; None when all values are NULL."""
    import torch

    from .runner import _chunks

    chunks = _chunks(data)
    schema = {name: dt for name, dt, _ in chunks[0].schema}
    views = (L.ColumnView * max(1, len(chunks)))()
    rows = (ctypes.c_int64 * max(1, len(chunks)))()
    for k, t in enumerate(chunks):
        rows[k] = t.num_rows
        views[k] = t.columns[column].view()
    out: List[float] = []
    n_total = 0
    qs = list(quantiles)
    for lo in range(0, len(qs), 8):  # DQ_MAX_QUANTILES per call
        part = qs[lo:lo + 8]
        q = (ctypes.c_double * len(part))(*part)
        res = (ctypes.c_double * len(part))()
        cnt = ctypes.c_int64()
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        L.check(L.lib.dq_approx_quantiles(_TYPES[schema[column]], views, rows, len(chunks), q, len(part),
                                          float(relative_error), torch.cuda.current_device(), stream, res,
                                          ctypes.byref(cnt)))
        n_total = cnt.value
        if n_total == 0:
            return None
        out.extend(res[:len(part)])
    return out


class _QuantileBase(Analyzer):
    grouping = True  # not part of the fused dq_plan scan: its own device passes
    direct = True

    def _quantiles(self) -> List[float]:
        raise NotImplementedError

    def preconditions(self):
        def param_checks(schema):
            for q in self._quantiles():
                if q < 0.0 or q > 1.0:
                    raise IllegalAnalyzerParameterException(_param_msg("Quantile", q))
            if self.relativeError < 0.0 or self.relativeError > 1.0:
                raise IllegalAnalyzerParameterException(_param_msg("Relative error", self.relativeError))
        return [param_checks, Preconditions.hasColumn(self.column), Preconditions.isNumeric(self.column)]

    @property
    def instance(self):
        return self.column

    def _empty_exc(self):
        return EmptyStateException(f"Empty state for analyzer {self}, all input values were NULL.")

    def compute(self, data):
        raise NotImplementedError

    def calculate(self, data, aggregateWith=None, saveStatesWith=None):
        try:
            for cond in self.preconditions():
                cond(data_schema(data))
            if aggregateWith is not None or saveStatesWith is not None:
                raise NotImplementedError(f"incremental {type(self).__name__} needs the percentile digest as a state")
            return self.compute(data)
        except Exception as e:
            return self.toFailureMetric(e)


class ApproxQuantile(_QuantileBase):  # ApproxQuantile.scala:49-103
    name = "ApproxQuantile"

    def __init__(self, column: str, quantile: float, relativeError: float = 0.01):
        self.column, self.quantile, self.relativeError = column, float(quantile), float(relativeError)

    def _fields(self):
        return (self.column, self.quantile, self.relativeError)

    def _show(self):
        return (self.column, _java_double_to_string(self.quantile), _java_double_to_string(self.relativeError))

    def _quantiles(self):
        return [self.quantile]

    def compute(self, data) -> DoubleMetric:
        r = device_quantiles(data, self.column, [self.quantile], self.relativeError)
        if r is None:
            return self.toFailureMetric(self._empty_exc())
        return DoubleMetric(Entity.Column, self.name, self.column, Success(r[0]))

    def toFailureMetric(self, e: BaseException) -> DoubleMetric:
        return DoubleMetric(Entity.Column, self.name, self.column, Failure(wrap_if_necessary(e)))


class ApproxQuantiles(_QuantileBase):  # ApproxQuantiles.scala:30-105
    name = "ApproxQuantiles"

    def __init__(self, column: str, quantiles: Sequence[float], relativeError: float = 0.01):
        self.column, self.quantiles, self.relativeError = column, tuple(float(q) for q in quantiles), float(relativeError)

    def _fields(self):
        return (self.column, self.quantiles, self.relativeError)

    def _show(self):
        return (self.column, "List(" + ", ".join(_java_double_to_string(q) for q in self.quantiles) + ")",
                _java_double_to_string(self.relativeError))

    def _quantiles(self):
        return list(self.quantiles)

    def compute(self, data) -> KeyedDoubleMetric:
        if not self.quantiles:  # getPercentiles(Array()) -> an empty map
            return KeyedDoubleMetric(Entity.Column, self.name, self.column, Success({}))
        r = device_quantiles(data, self.column, self.quantiles, self.relativeError)
        if r is None:
            # all values NULL: the digest is still Some (ApproxQuantiles.scala:64-72, no isEmpty check as in
            # ApproxQuantile.scala:72-77) and Spark 2.2's PercentileDigest.getPercentiles returns an empty
            # array for count == 0, so quantiles.zip(...) is an empty map
            return KeyedDoubleMetric(Entity.Column, self.name, self.column, Success({}))
        vals: Dict[str, float] = {_java_double_to_string(q): v for q, v in zip(self.quantiles, r)}
        return KeyedDoubleMetric(Entity.Column, self.name, self.column, Success(vals))

    def toFailureMetric(self, e: BaseException) -> KeyedDoubleMetric:
        return KeyedDoubleMetric(Entity.Column, self.name, self.column, Failure(wrap_if_necessary(e)))
