"""Grouping analyzers on the GPU (analyzers/GroupingAnalyzers.scala and the frequency-based
analyzers): Uniqueness, Distinctness, CountDistinct, Entropy, UniqueValueRatio.

FrequencyBasedAnalyzer.computeFrequencies (GroupingAnalyzers.scala:44-82) becomes dq_freq_build: a
sort-based GROUP BY ... COUNT(*) over the rows whose grouping columns are all non-null, held on the
device as (key, count) groups.  The state is FrequenciesAndNumRows (frequencies + numRows) and sums
as the reference's outer join (:118-138) via dq_freq_merge; each metric is computed from the
summary (groups, groups of count 1, entropy) exactly as its aggregationFunctions prescribe.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Union

from . import _lib as L
from .analyzers import Analyzer, Preconditions, data_schema
from .metrics import DoubleMetric, EmptyStateException, Entity, Failure, Success, wrap_if_necessary
from .states import State

_TYPES = {"f64": L.TYPE_F64, "i64": L.TYPE_I64, "i32": L.TYPE_I32, "utf8": L.TYPE_UTF8,
          "large_utf8": L.TYPE_LARGE_UTF8}


class FreqTable:
    """Owner of a device dq_freq_table (sorted distinct keys + counts)."""

    def __init__(self, handle: ctypes.c_void_p, types: Sequence[int]):
        self.handle = handle
        self.types = tuple(types)

    def summary(self, num_rows: int) -> L.FreqSummary:
        s = L.FreqSummary()
        L.check(L.lib.dq_freq_summarize(self.handle, num_rows, ctypes.byref(s)))
        return s

    def merged(self, other: "FreqTable") -> "FreqTable":
        h = ctypes.c_void_p()
        L.check(L.lib.dq_freq_merge(self.handle, other.handle, ctypes.byref(h)))
        return FreqTable(h, self.types)

    def export(self):
        import numpy as np

        n = L.lib.dq_freq_num_groups(self.handle)
        keys = np.zeros(max(1, n), dtype=np.uint64)
        counts = np.zeros(max(1, n), dtype=np.int64)
        L.check(L.lib.dq_freq_export(self.handle, keys.ctypes.data_as(ctypes.c_void_p),
                                     counts.ctypes.data_as(ctypes.c_void_p), max(1, n)))
        return keys[:n], counts[:n]

    def __del__(self):
        try:
            if self.handle:
                L.lib.dq_freq_destroy(self.handle)
                self.handle = None
        except Exception:
            pass


def build_frequencies(data, columns: Sequence[str]) -> "FrequenciesAndNumRows":
    """computeFrequencies(data, columns) + numRows = data.count() on the GPU."""
    import torch

    from .runner import _chunks

    chunks = _chunks(data)
    schema = {name: dt for name, dt, _ in chunks[0].schema}
    types = (ctypes.c_int32 * len(columns))(*[_TYPES[schema[c]] for c in columns])
    views = (L.ColumnView * max(1, len(chunks) * len(columns)))()
    rows = (ctypes.c_int64 * max(1, len(chunks)))()
    for k, t in enumerate(chunks):
        rows[k] = t.num_rows
        for c, name in enumerate(columns):
            views[k * len(columns) + c] = t.columns[name].view()
    h = ctypes.c_void_p()
    dev = torch.cuda.current_device()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    L.check(L.lib.dq_freq_build(types, len(columns), views, rows, len(chunks), dev, stream, ctypes.byref(h)))
    return FrequenciesAndNumRows(FreqTable(h, list(types)), sum(t.num_rows for t in chunks))


class FrequenciesAndNumRows(State):
    """GroupingAnalyzers.scala:118-138 (the frequencies live on the device)."""

    OP = -1

    def __init__(self, frequencies: FreqTable, numRows: int):
        self.frequencies = frequencies
        self.numRows = int(numRows)

    def sum(self, other: "FrequenciesAndNumRows") -> "FrequenciesAndNumRows":
        return FrequenciesAndNumRows(self.frequencies.merged(other.frequencies), self.numRows + other.numRows)

    def __eq__(self, other):
        if not isinstance(other, FrequenciesAndNumRows) or self.numRows != other.numRows:
            return False
        a, b = self.frequencies.export(), other.frequencies.export()
        return a[0].tolist() == b[0].tolist() and a[1].tolist() == b[1].tolist()

    __hash__ = None

    def _to_c(self):
        raise TypeError("FrequenciesAndNumRows has no fixed-size dq_state (HdfsStateProvider stores it as parquet)")


class FrequencyBasedAnalyzer(Analyzer):
    """ScanShareableFrequencyBasedAnalyzer (GroupingAnalyzers.scala:84-116)."""

    grouping = True

    def __init__(self, columns: Union[str, Sequence[str]]):
        self.columns: List[str] = [columns] if isinstance(columns, str) else list(columns)

    def _fields(self):
        return (tuple(self.columns),)

    def __str__(self):
        return f"{type(self).__name__}(List({', '.join(self.columns)}))"

    __repr__ = __str__

    @property
    def entity(self):
        return Entity.Column if len(self.columns) == 1 else Entity.Mutlicolumn

    @property
    def instance(self):
        return ",".join(self.columns)

    def groupingColumns(self) -> List[str]:
        return list(self.columns)

    def preconditions(self):
        def at_least_one(schema):
            if not self.columns:
                raise ValueError("At least one column needs to be specified!")
        return [at_least_one] + [Preconditions.hasColumn(c) for c in self.columns]

    def computeStateFrom(self, data) -> Optional[FrequenciesAndNumRows]:
        return build_frequencies(data, self.columns)

    def _value(self, s: L.FreqSummary, num_rows: int) -> Optional[float]:
        raise NotImplementedError

    def computeMetricFrom(self, state: Optional[FrequenciesAndNumRows]) -> DoubleMetric:
        if state is None:
            return self._empty()
        v = self._value(state.frequencies.summary(state.numRows), state.numRows)
        if v is None:  # the SQL aggregate over an empty frequencies table is NULL
            return self._empty()
        return DoubleMetric(self.entity, self.name, self.instance, Success(v))

    def _empty(self) -> DoubleMetric:
        return self.toFailureMetric(EmptyStateException(
            f"Empty state for analyzer {self}, all input values were NULL."))

    def toFailureMetric(self, e: BaseException) -> DoubleMetric:
        return DoubleMetric(self.entity, self.name, self.instance, Failure(wrap_if_necessary(e)))

    def calculate(self, data, aggregateWith=None, saveStatesWith=None) -> DoubleMetric:
        try:
            for cond in self.preconditions():
                cond(data_schema(data))
            return self.calculateMetric(self.computeStateFrom(data), aggregateWith, saveStatesWith)
        except Exception as e:
            return self.toFailureMetric(e)


class Uniqueness(FrequencyBasedAnalyzer):  # Uniqueness.scala:24-36: sum(count == 1) / numRows
    name = "Uniqueness"

    def _value(self, s, n):
        return None if s.num_groups == 0 else s.num_unique / n


class Distinctness(FrequencyBasedAnalyzer):  # Distinctness.scala:26-38: sum(count >= 1) / numRows
    name = "Distinctness"

    def _value(self, s, n):
        return None if s.num_groups == 0 else s.num_groups / n


class CountDistinct(FrequencyBasedAnalyzer):  # CountDistinct.scala:22-38: count(*), never NULL
    name = "CountDistinct"

    def _value(self, s, n):
        return float(s.num_groups)


class UniqueValueRatio(FrequencyBasedAnalyzer):  # UniqueValueRatio.scala:22-43
    name = "UniqueValueRatio"

    def _value(self, s, n):
        # Row.getDouble of a NULL sum unboxes to 0.0 (no isNullAt check here): 0.0 / 0 -> NaN
        num_unique = float(s.num_unique) if s.num_groups else 0.0
        return num_unique / s.num_groups if s.num_groups else float("nan")


class Entropy(FrequencyBasedAnalyzer):  # Entropy.scala:26-44 (single column)
    name = "Entropy"

    def __init__(self, column: str):
        super().__init__([column])

    def __str__(self):
        return f"Entropy({self.columns[0]})"

    __repr__ = __str__

    def _value(self, s, n):
        return None if s.num_groups == 0 else s.entropy




class MutualInformation(FrequencyBasedAnalyzer):  # MutualInformation.scala:32-80
    """sum over the joint groups of (pxy/N) ln((pxy/N) / ((px/N)(py/N))), marginals summed from the joint
    counts (rows with both values), N = numRows -- computed in one device pass (dq_mutual_information).
    The joint frequencies are not materialised as a state here: aggregateWith / saveStatesWith of a
    MutualInformation are reported as failures of that metric."""
    name = "MutualInformation"
    direct = True

    def __init__(self, columnA, columnB: Optional[str] = None):
        super().__init__(list(columnA) if columnB is None else [columnA, columnB])

    @property
    def entity(self):
        return Entity.Mutlicolumn

    def preconditions(self):
        def exactly_two(schema):  # Preconditions.exactlyNColumns(columns, 2)
            if len(self.columns) != 2:
                raise ValueError(f"{self.columns} has {len(self.columns)} columns, but exactly 2 are required")
        return [exactly_two] + [Preconditions.hasColumn(c) for c in self.columns]

    def compute(self, data) -> DoubleMetric:
        import torch

        from .runner import _chunks

        chunks = _chunks(data)
        schema = {name: dt for name, dt, _ in chunks[0].schema}
        types = (ctypes.c_int32 * 2)(*[_TYPES[schema[c]] for c in self.columns])
        views = (L.ColumnView * max(1, 2 * len(chunks)))()
        rows = (ctypes.c_int64 * max(1, len(chunks)))()
        for k, t in enumerate(chunks):
            rows[k] = t.num_rows
            for c, name in enumerate(self.columns):
                views[2 * k + c] = t.columns[name].view()
        value, defined = ctypes.c_double(), ctypes.c_int32()
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        L.check(L.lib.dq_mutual_information(types, views, rows, len(chunks), sum(t.num_rows for t in chunks),
                                            torch.cuda.current_device(), stream, ctypes.byref(value),
                                            ctypes.byref(defined)))
        if not defined.value:
            return self._empty()
        return DoubleMetric(self.entity, self.name, self.instance, Success(value.value))

    def calculate(self, data, aggregateWith=None, saveStatesWith=None) -> DoubleMetric:
        try:
            for cond in self.preconditions():
                cond(data_schema(data))
            if aggregateWith is not None or saveStatesWith is not None:
                raise NotImplementedError("incremental MutualInformation needs the joint frequencies as a state")
            return self.compute(data)
        except Exception as e:
            return self.toFailureMetric(e)
