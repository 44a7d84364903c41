"""ApproxQuantile / ApproxQuantiles (ApproxQuantile.scala:49-103, ApproxQuantiles.scala:30-105) on the GPU.

The reference aggregates the column into Spark 2.2's ApproximatePercentile digest (Greenwald-Khanna,
order-dependent) and answers PercentileDigest.getPercentiles.  Here one device pass family
(dq_approx_quantiles: MSD radix select, six HBM-streaming histogram passes) returns the exact order
statistic of rank ceil(q * n) (min / max at the two ends, as QuantileSummaries.query), which lies inside
the error bound GK guarantees -- the property the reference's own tests check
(AnalyzerTests.scala:533-565).

The state (ApproxQuantileState, ApproxQuantile.scala:28-35) is a PercentileDigest in Spark 2.2.2's
layout, for aggregateWith / saveStatesWith: a GK summary built from exact order statistics -- the values
at ranks 1, 1 + s, 1 + 2 s, ..., n with s = max(1, floor(2 e n)), g = the rank gaps, delta = 0 -- which
satisfies GK's invariants (sum g = n, g + delta <= 2 e n) with zero rank uncertainty.  QuantileSummaries'
merge / compress / query and the PercentileDigestSerializer byte layout are restated below from Spark
2.2.2 (catalyst/util/QuantileSummaries.scala, aggregate/ApproximatePercentile.scala), a dependency the
reference does not vendor: their parity is unpinned beyond the reference's own tests (StateProviderTest
round trip, IncrementalAnalyzerTest merge) and the GK rank bound.  With a state round trip the metric is
Spark's query over the (merged) summary; without one, the exact order statistic above.
"""
from __future__ import annotations

import ctypes
import math
import struct
from typing import Dict, List, Optional, Sequence, Tuple

from . import _lib as L
from .analyzers import Analyzer, Preconditions, data_schema
from .grouping import _gpu_type, _java_double_to_string
from .metrics import (DoubleMetric, EmptyStateException, Entity, Failure, IllegalAnalyzerParameterException,
                      KeyedDoubleMetric, Success, UnsupportedOnGpuPathException, wrap_if_necessary)
from .states import State


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
        L.check(L.lib.dq_approx_quantiles(_gpu_type(schema[column]), views, rows, len(chunks), q, len(part),
                                          float(relative_error), torch.cuda.current_device(), stream, res,
                                          ctypes.byref(cnt)))
        n_total = cnt.value
        if n_total == 0:
            return None
        out.extend(res[:len(part)])
    return out


Stats = Tuple[float, int, int]  # QuantileSummaries.Stats(value, g, delta): g / delta are Int in Spark 2.2


class QuantileSummaries:
    """Spark 2.2.2 QuantileSummaries (compressed: no head buffer), restated: merge, compressImmut, query."""

    defaultCompressThreshold = 10000

    def __init__(self, compressThreshold: int, relativeError: float, sampled: Sequence[Stats] = (), count: int = 0):
        self.compressThreshold, self.relativeError = int(compressThreshold), float(relativeError)
        self.sampled: List[Stats] = [(float(v), int(g), int(d)) for v, g, d in sampled]
        self.count = int(count)

    @staticmethod
    def _order(v: float):  # scala.math.Ordering.Double = java.lang.Double.compare: -0.0 < 0.0, NaN last
        if v != v:
            return (1, 0.0, 0)
        return (0, v, 0 if math.copysign(1.0, v) < 0 else 1)

    @staticmethod
    def _compress(samples: List[Stats], mergeThreshold: float) -> List[Stats]:
        """compressImmut: from the last sample down to index 1, merge a sample into the current head while
        g1 + head.g + head.delta < mergeThreshold; the first sample is kept if it is <= the head."""
        if not samples:
            return []
        res: List[Stats] = []
        head = samples[-1]
        i = len(samples) - 2
        while i >= 1:
            v1, g1, _ = samples[i]
            if g1 + head[1] + head[2] < mergeThreshold:
                head = (head[0], head[1] + g1, head[2])
            else:
                res.insert(0, head)
                head = samples[i]
            i -= 1
        res.insert(0, head)
        first = samples[0]
        if QuantileSummaries._order(first[0]) <= QuantileSummaries._order(head[0]) and len(samples) > 1:
            res.insert(0, first)
        return res

    def merge(self, other: "QuantileSummaries") -> "QuantileSummaries":
        if other.count == 0:
            return QuantileSummaries(self.compressThreshold, self.relativeError, self.sampled, self.count)
        if self.count == 0:
            return QuantileSummaries(other.compressThreshold, other.relativeError, other.sampled, other.count)
        # concatenation sorted by value (stable: this summary's samples first among equal values); the merge
        # threshold uses this summary's count, as Spark 2.2 does
        res = sorted(self.sampled + other.sampled, key=lambda st: self._order(st[0]))
        comp = self._compress(res, 2 * self.relativeError * self.count)
        return QuantileSummaries(other.compressThreshold, other.relativeError, comp, other.count + self.count)

    def query(self, quantile: float) -> float:
        if quantile < 0 or quantile > 1.0:
            raise ValueError("quantile should be in the range [0.0, 1.0]")
        if quantile <= self.relativeError:
            return self.sampled[0][0]
        if quantile >= 1 - self.relativeError:
            return self.sampled[-1][0]
        rank = int(math.ceil(quantile * self.count))
        target_error = math.ceil(self.relativeError * self.count)
        min_rank = 0
        i = 1
        while i < len(self.sampled) - 1:
            v, g, d = self.sampled[i]
            min_rank += g
            max_rank = min_rank + d
            if max_rank - target_error <= rank <= min_rank + target_error:
                return v
            i += 1
        return self.sampled[-1][0]

    def __eq__(self, other):
        return (isinstance(other, QuantileSummaries) and self.compressThreshold == other.compressThreshold
                and self.relativeError == other.relativeError and self.count == other.count
                and len(self.sampled) == len(other.sampled)
                and all(struct.pack(">dii", *a) == struct.pack(">dii", *b) for a, b in zip(self.sampled, other.sampled)))

    def __repr__(self):
        return (f"QuantileSummaries({self.compressThreshold},{self.relativeError},count={self.count},"
                f"sampled={len(self.sampled)})")


class PercentileDigest:
    """ApproximatePercentile.PercentileDigest over a compressed summary (getPercentiles, merge)."""

    def __init__(self, summaries: QuantileSummaries):
        self.quantileSummaries = summaries

    def merge(self, other: "PercentileDigest") -> "PercentileDigest":
        return PercentileDigest(self.quantileSummaries.merge(other.quantileSummaries))

    def getPercentiles(self, percentages: Sequence[float]) -> List[float]:
        s = self.quantileSummaries
        if s.count == 0 or len(percentages) == 0:
            return []
        return [s.query(p) for p in percentages]

    def __eq__(self, other):
        return isinstance(other, PercentileDigest) and self.quantileSummaries == other.quantileSummaries

    def serialize(self) -> bytes:
        """ApproximatePercentile.PercentileDigestSerializer (big-endian ByteBuffer): compressThreshold int,
        relativeError double, count long, sampled length int, then (value double, g int, delta int) each."""
        s = self.quantileSummaries
        out = [struct.pack(">idqi", s.compressThreshold, s.relativeError, s.count, len(s.sampled))]
        out += [struct.pack(">dii", v, g, d) for v, g, d in s.sampled]
        return b"".join(out)

    @staticmethod
    def deserialize(data: bytes) -> "PercentileDigest":
        if len(data) < 24:
            raise ValueError("percentile digest image too short")
        ct, rel, count, n = struct.unpack_from(">idqi", data, 0)
        if n < 0 or len(data) != 24 + 16 * n:
            raise ValueError("percentile digest image length does not match its sample count")
        sampled = [struct.unpack_from(">dii", data, 24 + 16 * k) for k in range(n)]
        return PercentileDigest(QuantileSummaries(ct, rel, sampled, count))


class ApproxQuantileState(State):
    """ApproxQuantile.scala:28-35: sum = PercentileDigest.merge."""

    def __init__(self, percentileDigest: PercentileDigest):
        self.percentileDigest = percentileDigest

    def sum(self, other: "ApproxQuantileState") -> "ApproxQuantileState":
        if not isinstance(other, ApproxQuantileState):
            raise TypeError(f"cannot sum ApproxQuantileState with {type(other).__name__}")
        return ApproxQuantileState(self.percentileDigest.merge(other.percentileDigest))

    __add__ = sum

    def __eq__(self, other):
        return isinstance(other, ApproxQuantileState) and self.percentileDigest == other.percentileDigest

    def __repr__(self):
        return f"ApproxQuantileState({self.percentileDigest.quantileSummaries!r})"


def spark_relative_error(relativeError: float) -> float:
    """StatefulApproxQuantile: accuracy = 1.0 / relativeError (DeequFunctions.scala:63-71), then
    relativeError = 1.0 / accuracy (createAggregationBuffer)."""
    if relativeError == 0.0:
        return 0.0
    return 1.0 / (1.0 / relativeError)


def digest_ranks(n: int, relativeError: float) -> List[int]:
    """Ranks (1-based) the state's summary samples: 1, 1 + s, ..., n with s = max(1, floor(2 e n))."""
    s = max(1, int(math.floor(2 * relativeError * n)))
    ranks = list(range(1, n + 1, s))
    if ranks[-1] != n:
        ranks.append(n)
    return ranks


# samples the state may hold: relativeError e keeps about 1 / (2 e) + 2 of them (52 at e = 0.01); e = 0 keeps
# every value, as Spark's GK summary does.  Past this, the Python digest (a list of samples) would not fit.
MAX_DIGEST_SAMPLES = 1 << 20


def device_digest(data, column: str, relativeError: float) -> PercentileDigest:
    """The column's digest from exact order statistics: dq_quantile_digest answers every sample rank in two
    passes over the column's non-null values on the device (per-bucket counts against sampled splitters, then
    the keys of the buckets that hold a sample rank compacted and sorted), whatever the number of samples; an
    empty digest (count 0) when every value is NULL."""
    rel = spark_relative_error(relativeError)
    n, ranks, values = _digest_samples(data, column, rel)
    if n == 0:
        return PercentileDigest(QuantileSummaries(QuantileSummaries.defaultCompressThreshold, rel))
    assert ranks == digest_ranks(n, rel)[:len(ranks)] and ranks[-1] == n
    sampled, prev = [], 0
    for r, v in zip(ranks, values):
        sampled.append((v, r - prev, 0))
        prev = r
    return PercentileDigest(QuantileSummaries(QuantileSummaries.defaultCompressThreshold, rel, sampled, n))


def _digest_samples(data, column: str, rel: float):
    """(n, sample ranks, sample values) of the column through dq_quantile_digest."""
    import torch

    from .runner import _chunks

    chunks = _chunks(data)
    schema = {name: dt for name, dt, _ in chunks[0].schema}
    views = (L.ColumnView * max(1, len(chunks)))()
    rows = (ctypes.c_int64 * max(1, len(chunks)))()
    total = 0
    for k, t in enumerate(chunks):
        rows[k] = t.num_rows
        views[k] = t.columns[column].view()
        total += t.num_rows
    # the sample count for n <= total values: (n - 1) / s + 2 at most, s = max(1, floor(2 rel n)), which peaks
    # near n = 1 / rel (s = 1 below it)
    cap = total + 1 if rel == 0.0 else min(total + 1, int(1.0 / rel) + 4)
    cap = min(cap, MAX_DIGEST_SAMPLES)
    vals = (ctypes.c_double * max(1, cap))()
    rks = (ctypes.c_int64 * max(1, cap))()
    m, cnt = ctypes.c_int64(), ctypes.c_int64()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rc = L.lib.dq_quantile_digest(_gpu_type(schema[column]), views, rows, len(chunks), rel, torch.cuda.current_device(),
                                  stream, vals, rks, cap, ctypes.byref(m), ctypes.byref(cnt))
    if rc == L.DQ_E_INVALID and m.value > cap:
        raise UnsupportedOnGpuPathException(
            f"a relativeError of {rel} over {cnt.value} values needs {m.value} samples in the quantile state "
            f"(at most {MAX_DIGEST_SAMPLES} on the GPU path)")
    if rc == L.DQ_E_UNSUPPORTED:  # a device limit of the digest (e.g. one bucket over the candidate budget)
        raise UnsupportedOnGpuPathException(
            f"ApproxQuantileState of {column} is outside the GPU path: {L.lib.dq_last_error().decode('utf-8', 'replace')}")
    L.check(rc)
    return cnt.value, list(rks[:m.value]), list(vals[:m.value])


def _rank_select(data, column: str):
    """qs -> (n, values): dq_approx_quantiles over every chunk of `data` with relative_error 0 (no end
    clamping: quantile q answers rank ceil(q * n))."""
    import torch

    from .runner import _chunks

    chunks = _chunks(data)
    schema = {name: dt for name, dt, _ in chunks[0].schema}
    views = (L.ColumnView * max(1, len(chunks)))()
    rows = (ctypes.c_int64 * max(1, len(chunks)))()
    for k, t in enumerate(chunks):
        rows[k] = t.num_rows
        views[k] = t.columns[column].view()

    def call(qs):
        q = (ctypes.c_double * len(qs))(*qs)
        res = (ctypes.c_double * len(qs))()
        cnt = ctypes.c_int64()
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        L.check(L.lib.dq_approx_quantiles(_gpu_type(schema[column]), views, rows, len(chunks), q, len(qs), 0.0,
                                          torch.cuda.current_device(), stream, res, ctypes.byref(cnt)))
        return cnt.value, list(res[:len(qs)])

    return call


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

    def computeStateFrom(self, data) -> Optional[ApproxQuantileState]:
        raise NotImplementedError

    def computeMetricFrom(self, state: Optional[ApproxQuantileState]):
        raise NotImplementedError

    def calculate(self, data, aggregateWith=None, saveStatesWith=None):
        """Without a state round trip: the exact order statistics.  With aggregateWith / saveStatesWith:
        load -> merge -> persist -> metric over the digest (Analyzer.scala:107-128)."""
        try:
            for cond in self.preconditions():
                cond(data_schema(data))
            if aggregateWith is None and saveStatesWith is None:
                return self.compute(data)
            from .analyzers import merge

            state = self.computeStateFrom(data)
            loaded = aggregateWith.load(self) if aggregateWith is not None else None
            merged = merge(state, loaded)
            if merged is not None and saveStatesWith is not None:
                saveStatesWith.persist(self, merged)
            return self.computeMetricFrom(merged)
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

    def computeStateFrom(self, data) -> Optional[ApproxQuantileState]:
        digest = device_digest(data, self.column, self.relativeError)
        if not digest.getPercentiles([self.quantile]):  # all values NULL (ApproxQuantile.scala:72-77)
            return None
        return ApproxQuantileState(digest)

    def computeMetricFrom(self, state: Optional[ApproxQuantileState]) -> DoubleMetric:
        if state is None:
            return self.toFailureMetric(self._empty_exc())
        return DoubleMetric(Entity.Column, self.name, self.column,
                            Success(state.percentileDigest.getPercentiles([self.quantile])[0]))

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

    def computeStateFrom(self, data) -> ApproxQuantileState:
        # no emptiness check (ApproxQuantiles.scala:61-72): an all-NULL column is a digest of count 0
        return ApproxQuantileState(device_digest(data, self.column, self.relativeError))

    def computeMetricFrom(self, state: Optional[ApproxQuantileState]) -> KeyedDoubleMetric:
        if state is None:
            return self.toFailureMetric(self._empty_exc())
        got = state.percentileDigest.getPercentiles(list(self.quantiles))
        vals: Dict[str, float] = {_java_double_to_string(q): v for q, v in zip(self.quantiles, got)}
        return KeyedDoubleMetric(Entity.Column, self.name, self.column, Success(vals))

    def toFailureMetric(self, e: BaseException) -> KeyedDoubleMetric:
        return KeyedDoubleMetric(Entity.Column, self.name, self.column, Failure(wrap_if_necessary(e)))
