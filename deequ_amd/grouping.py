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
          "large_utf8": L.TYPE_LARGE_UTF8, "f32": L.TYPE_F32, "i16": L.TYPE_I16, "i8": L.TYPE_I8,
          "bool": L.TYPE_BOOL, "date32": L.TYPE_DATE32, "timestamp": L.TYPE_TIMESTAMP}


def _gpu_type(dtype: str) -> int:
    """The grouping / quantile kernels' column type code (a DecimalType's carries its precision / scale)."""
    from .table import decimal_ps

    ps = decimal_ps(dtype)
    if ps:
        return L.decimal_type(*ps)
    t = _TYPES.get(dtype)
    if t is None:
        from .metrics import UnsupportedOnGpuPathException

        raise UnsupportedOnGpuPathException(f"column type {dtype} is not a GPU column type")
    return t


def _java_decimal_to_string(u: int, scale: int) -> str:
    """java.math.BigDecimal.toString of unscaled u at scale >= 0 (Spark's CAST(decimal AS STRING)): plain notation
    unless the adjusted exponent digits - 1 - scale is below -6, then "1.5E-7" / "0E-18"."""
    sign = "-" if u < 0 else ""
    coeff = str(abs(u))
    adjusted = len(coeff) - 1 - scale
    if scale == 0:
        return sign + coeff
    if adjusted >= -6:
        if len(coeff) > scale:
            return f"{sign}{coeff[:-scale]}.{coeff[-scale:]}"
        return f"{sign}0.{'0' * (scale - len(coeff))}{coeff}"
    return f"{sign}{coeff[0]}{'.' + coeff[1:] if len(coeff) > 1 else ''}E{adjusted}"


def _java_float_to_string(f: float) -> str:
    """java.lang.Float.toString (CAST(float AS STRING)): Double.toString's forms with float's shortest digits."""
    import math

    import numpy as np

    if math.isnan(f) or math.isinf(f) or f == 0.0:
        return _java_double_to_string(f)
    if 1e-3 <= abs(f) < 1e7:
        r = np.format_float_positional(np.float32(f), unique=True)
        return r + "0" if r.endswith(".") else r
    m, e = np.format_float_scientific(np.float32(f), unique=True, exp_digits=1).split("e")
    return f"{m + '0' if m.endswith('.') else m}E{int(e)}"


def _render_fixed(dtype: str, key: int) -> str:
    """CAST(value AS STRING) of a fixed-width grouping key (value bits, integers sign-extended; timestamps in UTC
    as Spark's DateTimeUtils.timestampToString with the session zone UTC)."""
    import datetime

    import numpy as np

    v = int(np.uint64(key).astype(np.int64))
    if dtype == "f64":
        return _java_double_to_string(float(np.uint64(key).view(np.float64)))
    if dtype == "f32":
        return _java_float_to_string(float(np.uint32(key & 0xFFFFFFFF).view(np.float32)))
    if dtype == "bool":
        return "true" if v else "false"
    if dtype == "date32":
        return (datetime.date(1970, 1, 1) + datetime.timedelta(days=v)).isoformat()
    if dtype == "timestamp":
        t = datetime.datetime(1970, 1, 1) + datetime.timedelta(microseconds=v)
        frac = f"{t.microsecond:06d}".rstrip("0")
        return t.strftime("%Y-%m-%d %H:%M:%S") + ("." + frac if frac else "")
    return str(v)


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
    types = (ctypes.c_int32 * len(columns))(*[_gpu_type(schema[c]) for c in columns])
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
        types = (ctypes.c_int32 * 2)(*[_gpu_type(schema[c]) for c in self.columns])
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


def _java_double_to_string(d: float) -> str:
    """java.lang.Double.toString (Spark's CAST(double AS STRING)): plain decimal for 1e-3 <= |d| < 1e7,
    computerized scientific notation otherwise; digits from the shortest round-trip repr (Java 8 can
    print one more digit in rare cases)."""
    import math

    if math.isnan(d):
        return "NaN"
    if math.isinf(d):
        return "Infinity" if d > 0 else "-Infinity"
    if d == 0.0:
        return "-0.0" if math.copysign(1.0, d) < 0 else "0.0"
    if 1e-3 <= abs(d) < 1e7:
        r = repr(d)
        return r if "." in r else r + ".0"
    from decimal import Decimal

    t = Decimal(repr(abs(d))).as_tuple()  # the shortest round-trip digits
    digits = "".join(map(str, t.digits)).lstrip("0")
    exp10 = t.exponent + len(t.digits) - 1 - (len(t.digits) - len("".join(map(str, t.digits)).lstrip("0")))
    digits = digits.rstrip("0") or "0"
    mant = digits[0] + "." + (digits[1:] or "0")
    return f"{'-' if d < 0 else ''}{mant}E{exp10}"


class Histogram(Analyzer):  # Histogram.scala:33-99
    """Counts of the column's values cast to string (NULL -> "NullValue"): the maxDetailBins largest
    groups (ties in key order; Spark's rdd.top leaves them unspecified) with ratio count / numRows, and
    the number of bins.  The frequencies are the device table of build_frequencies; values are
    rendered on the host only for the returned bins."""
    name = "Histogram"
    grouping = True
    direct = True
    NullFieldReplacement = "NullValue"
    MaximumAllowedDetailBins = 1000

    def __init__(self, column: str, binningUdf=None, maxDetailBins: int = 1000):
        self.column = column
        self.binningUdf = binningUdf
        self.maxDetailBins = maxDetailBins

    def _fields(self):
        return (self.column, id(self.binningUdf) if self.binningUdf is not None else None, self.maxDetailBins)

    def __str__(self):
        return f"Histogram({self.column},{'None' if self.binningUdf is None else 'Some(udf)'},{self.maxDetailBins})"

    __repr__ = __str__

    @property
    def instance(self):
        return self.column

    def groupingColumns(self):
        return [self.column]

    def preconditions(self):
        from .metrics import IllegalAnalyzerParameterException

        def param_check(schema):
            if self.maxDetailBins > Histogram.MaximumAllowedDetailBins:
                raise IllegalAnalyzerParameterException(
                    f"Cannot return histogram values for more than {Histogram.MaximumAllowedDetailBins} values")
        return [param_check, Preconditions.hasColumn(self.column)]

    def toFailureMetric(self, e: BaseException):
        from .metrics import HistogramMetric

        return HistogramMetric(self.column, Failure(wrap_if_necessary(e)))

    def _render(self, data, dtype: str, key: int, rep: int) -> str:
        import numpy as np

        from .table import decimal_ps

        ps = decimal_ps(dtype)
        if dtype not in ("utf8", "large_utf8") and not ps:
            return _render_fixed(dtype, key)
        if rep == (1 << 64) - 1:
            raise NotImplementedError("Histogram of a merged string / decimal frequency table (no representative rows)")
        from .runner import _chunks

        col = _chunks(data)[rep >> 40].columns[self.column]
        r = rep & ((1 << 40) - 1)
        if ps:  # the representative row's 16-byte unscaled value, as Decimal.toString
            u = int.from_bytes(bytes(col.values[16 * r:16 * r + 16].cpu().numpy()), "little", signed=True)
            return _java_decimal_to_string(u, ps[1])
        width = 8 if col.dtype == "large_utf8" else 4
        o = col.offsets[r * width:(r + 2) * width].cpu().numpy().view(np.int64 if width == 8 else np.int32)
        return bytes(col.values[int(o[0]):int(o[1])].cpu().numpy()).decode("utf-8", "replace")

    def computeMetricFromState(self, state: "FrequenciesAndNumRows", data):
        from .metrics import Distribution, DistributionValue, HistogramMetric

        n = self.maxDetailBins
        keys = (ctypes.c_uint64 * max(1, n))()
        counts = (ctypes.c_int64 * max(1, n))()
        reps = (ctypes.c_uint64 * max(1, n))()
        got = ctypes.c_int32()
        L.check(L.lib.dq_freq_top(state.frequencies.handle, n, keys, counts, reps, ctypes.byref(got)))
        t0 = state.frequencies.types[0]
        dtype = ({v: k for k, v in _TYPES.items()}.get(t0) or
                 f"decimal({(t0 >> 8) & 0xFF},{(t0 >> 16) & 0xFF})")  # (a DQ_DECIMAL128 code carries p, s)
        bins = [(self._render(data, dtype, keys[i], reps[i]), int(counts[i])) for i in range(got.value)]
        summary = state.frequencies.summary(state.numRows)
        nulls = state.numRows - summary.num_values
        bin_count = summary.num_groups
        if nulls > 0:  # .na.fill("NullValue"): the NULLs are one more group
            merged = False
            for i, (k, c) in enumerate(bins):
                if k == Histogram.NullFieldReplacement:  # a literal "NullValue" string joins them
                    bins[i] = (k, c + nulls)
                    merged = True
            if not merged:
                bins.append((Histogram.NullFieldReplacement, nulls))
                bin_count += 1
            bins.sort(key=lambda kc: -kc[1])
            bins = bins[:n]
        values = {k: DistributionValue(c, c / state.numRows) for k, c in bins}
        return HistogramMetric(self.column, Success(Distribution(values, numberOfBins=bin_count)))

    def calculate(self, data, aggregateWith=None, saveStatesWith=None):
        try:
            for cond in self.preconditions():
                cond(data_schema(data))
            if self.binningUdf is not None:
                from .metrics import UnsupportedOnGpuPathException

                raise UnsupportedOnGpuPathException(f"{self}: a binning UDF runs in Spark, not on the GPU path")
            state = build_frequencies(data, [self.column])
            if aggregateWith is not None:
                prev = aggregateWith.load(self)
                if prev is not None:
                    state = state.sum(prev)
            if saveStatesWith is not None:
                saveStatesWith.persist(self, state)
            return self.computeMetricFromState(state, data)
        except Exception as e:
            return self.toFailureMetric(e)
