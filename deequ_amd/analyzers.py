"""The GPU-eligible ScanShareableAnalyzers, mirroring the Scala case classes.

Reference (paths relative to src/main/scala/com/amazon/deequ/analyzers/):
  Analyzer.calculate / calculateMetric      Analyzer.scala:88-128
  ScanShareableAnalyzer.computeStateFrom    Analyzer.scala:168-172
  StandardScanShareableAnalyzer             Analyzer.scala:190-216
  Preconditions.hasColumn / isNumeric       Analyzer.scala:315-334
  Size.scala, Completeness.scala, Compliance.scala, Sum.scala, Mean.scala, StandardDeviation.scala,
  Minimum.scala, Maximum.scala, Correlation.scala, ApproxCountDistinct.scala, DataType.scala

Instead of `aggregationFunctions(): Seq[Column]` each analyzer lowers itself into one
dq_analyzer_spec of the C ABI (`_lower`), and instead of `fromAggregationResult(row, offset)` it
receives the dq_state slot set libdqscan.so produced for that spec (`_from_result`).
"""
from __future__ import annotations

import math
from typing import Callable, List, Optional, Sequence

from . import _lib as L
from .metrics import (DoubleMetric, EmptyStateException, Entity, Failure, NoSuchColumnException, Success,
                      WrongColumnTypeException, wrap_if_necessary)
from .predicates import PredicatePool
from .states import State, state_from_c
from .table import decimal_ps, is_numeric

Schema = Sequence  # list of (name, dtype, nullable)
# the Spark SQL type each column dtype carries (WrongColumnTypeException text, Analyzer.scala:330-332)
SPARK_TYPE = {"f64": "DoubleType", "f32": "FloatType", "i64": "LongType", "i32": "IntegerType", "i16": "ShortType",
              "i8": "ByteType", "bool": "BooleanType", "date32": "DateType", "timestamp": "TimestampType",
              "utf8": "StringType", "large_utf8": "StringType"}


def spark_type(dtype: str) -> str:
    ps = decimal_ps(dtype)
    return f"DecimalType({ps[0]},{ps[1]})" if ps else SPARK_TYPE.get(dtype, dtype)


def _opt(x: Optional[str]) -> str:
    return "None" if x is None else f"Some({x})"


class Preconditions:
    @staticmethod
    def hasColumn(column: str) -> Callable:
        def check(schema):
            if column not in [c[0] for c in schema]:
                raise NoSuchColumnException(f"Input data does not include column {column}!")
        return check

    @staticmethod
    def isNumeric(column: str) -> Callable:
        def check(schema):
            t = dict((c[0], c[1]) for c in schema)[column]
            if not is_numeric(t):
                raise WrongColumnTypeException(
                    f"Expected type of column {column} to be one of (ByteType,ShortType,IntegerType,LongType,"
                    f"FloatType,DoubleType,DecimalType), but found {spark_type(t)} instead!")
        return check

    @staticmethod
    def findFirstFailing(schema, conditions) -> Optional[Exception]:
        for cond in conditions:
            try:
                cond(schema)
            except Exception as e:  # only exceptions, as the reference
                return e
        return None


class PlanBuilder:
    """Collects the specs, referenced columns and predicate pool of one fused plan."""

    def __init__(self, table_schema):
        self.table_schema = list(table_schema)
        self.by_name = {c[0]: c for c in self.table_schema}
        self.columns: List[str] = []
        self.pool = PredicatePool(self)
        self.specs: List[tuple] = []

    def col(self, name: str) -> int:
        if name not in self.by_name:
            raise NoSuchColumnException(f"Input data does not include column {name}!")
        if name not in self.columns:
            self.columns.append(name)
        return self.columns.index(name)

    def pred(self, text: Optional[str]) -> int:
        return -1 if text is None else self.pool.add(text)

    def schema_ctypes(self):
        arr = (L.ColumnDesc * max(1, len(self.columns)))()
        from .table import type_code

        for i, name in enumerate(self.columns):
            _, dt, nullable = self.by_name[name]
            arr[i].type = type_code(dt)
            arr[i].nullable = 1 if nullable else 0
        return arr


class Analyzer:
    """Common analyzer contract (Analyzer.scala:56-155)."""

    name = ""
    entity = Entity.Column

    # ---- identity: Scala case-class equality / toString ---------------------------------
    def _fields(self) -> tuple:
        raise NotImplementedError

    def __eq__(self, other):
        return type(self) is type(other) and self._fields() == other._fields()

    def __hash__(self):
        return hash((type(self).__name__,) + self._fields())

    def __str__(self):
        parts = [_opt(f[1]) if isinstance(f, tuple) and f and f[0] == "opt" else str(f) for f in self._show()]
        return f"{type(self).__name__}({','.join(parts)})"

    __repr__ = __str__

    def _show(self):
        return self._fields()

    @property
    def instance(self) -> str:
        raise NotImplementedError

    # ---- preconditions -------------------------------------------------------------------
    def additionalPreconditions(self) -> List[Callable]:
        return []

    def preconditions(self) -> List[Callable]:
        return self.additionalPreconditions()

    # ---- GPU lowering --------------------------------------------------------------------
    def _lower(self, b: PlanBuilder) -> tuple:
        """-> (op, col_a, col_b, pred_root, where_root)"""
        raise NotImplementedError

    def _from_result(self, c_state: L.State) -> Optional[State]:
        return state_from_c(c_state)

    def _lower_op(self) -> int:
        return self.OP

    # ---- metric computation --------------------------------------------------------------
    def computeStateFrom(self, data) -> Optional[State]:
        """Runs this analyzer's aggregation alone (ScanShareableAnalyzer.computeStateFrom)."""
        from .predicates import UnsupportedPredicate
        from .metrics import UnsupportedOnGpuPathException
        from .runner import scan_states

        try:
            return scan_states(data, [self])[self]
        except UnsupportedPredicate as e:
            raise UnsupportedOnGpuPathException(
                f"{self} is outside the GPU-eligible set ({e}); a Spark integration keeps it on data.agg") from e

    def computeMetricFrom(self, state: Optional[State]) -> DoubleMetric:
        if state is not None:
            return DoubleMetric(self.entity, self.name, self.instance, Success(state.metricValue()))
        return self.toFailureMetric(EmptyStateException(
            f"Empty state for analyzer {self}, all input values were NULL."))

    def toFailureMetric(self, e: BaseException) -> DoubleMetric:
        return DoubleMetric(self.entity, self.name, self.instance, Failure(wrap_if_necessary(e)))

    def calculate(self, data, aggregateWith=None, saveStatesWith=None) -> DoubleMetric:
        try:
            for cond in self.preconditions():
                cond(data_schema(data))
            state = self.computeStateFrom(data)
            return self.calculateMetric(state, aggregateWith, saveStatesWith)
        except Exception as e:
            return self.toFailureMetric(e)

    def calculateMetric(self, state, aggregateWith=None, saveStatesWith=None) -> DoubleMetric:
        """load -> merge -> persist -> metric (Analyzer.scala:107-128)."""
        loaded = aggregateWith.load(self) if aggregateWith is not None else None
        merged = merge(state, loaded)
        if merged is not None and saveStatesWith is not None:
            saveStatesWith.persist(self, merged)
        return self.computeMetricFrom(merged)

    def aggregateStateTo(self, sourceA, sourceB, target) -> None:
        a, b = sourceA.load(self), sourceB.load(self)
        agg = merge(a, b)
        if agg is not None:
            target.persist(self, agg)

    def loadStateAndComputeMetric(self, source) -> Optional[DoubleMetric]:
        s = source.load(self)
        return None if s is None else self.computeMetricFrom(s)


def merge(*states) -> Optional[State]:
    """Analyzers.merge (Analyzer.scala:343-362)."""
    acc = None
    for s in states:
        if acc is None:
            acc = s
        elif s is not None:
            acc = acc.sum(s)
    return acc


def data_schema(data):
    from .table import Table

    if isinstance(data, Table):
        return data.schema
    return data[0].schema  # list of chunks


# ------------------------------------------------------------------------------------------
class Size(Analyzer):  # Size.scala:36-48
    name = "Size"
    entity = Entity.Dataset
    OP = L.OP_SIZE

    def __init__(self, where: Optional[str] = None):
        self.where = where

    def _fields(self):
        return (self.where,)

    def _show(self):
        return (("opt", self.where),)

    @property
    def instance(self):
        return "*"

    def _lower(self, b):
        return (L.OP_SIZE, -1, -1, -1, b.pred(self.where))


class _ColumnAnalyzer(Analyzer):
    OP = 0
    numeric = True

    def __init__(self, column: str, where: Optional[str] = None):
        self.column = column
        self.where = where

    def _fields(self):
        return (self.column, self.where)

    def _show(self):
        return (self.column, ("opt", self.where))

    @property
    def instance(self):
        return self.column

    def additionalPreconditions(self):
        pre = [Preconditions.hasColumn(self.column)]
        if self.numeric:
            pre.append(Preconditions.isNumeric(self.column))
        return pre

    def _lower(self, b):
        return (self.OP, b.col(self.column), -1, -1, b.pred(self.where))


class Completeness(_ColumnAnalyzer):  # Completeness.scala:26-46
    name = "Completeness"
    OP = L.OP_COMPLETENESS
    numeric = False


class Sum(_ColumnAnalyzer):  # Sum.scala:36-52
    name = "Sum"
    OP = L.OP_SUM


class Mean(_ColumnAnalyzer):  # Mean.scala:36-54
    name = "Mean"
    OP = L.OP_MEAN


class StandardDeviation(_ColumnAnalyzer):  # StandardDeviation.scala:47-73
    name = "StandardDeviation"
    OP = L.OP_STDDEV


class Minimum(_ColumnAnalyzer):  # Minimum.scala:36-53
    name = "Minimum"
    OP = L.OP_MIN


class Maximum(_ColumnAnalyzer):  # Maximum.scala:36-53
    name = "Maximum"
    OP = L.OP_MAX


class ApproxCountDistinct(_ColumnAnalyzer):  # ApproxCountDistinct.scala:47-64
    name = "ApproxCountDistinct"
    OP = L.OP_APPROX_COUNT_DISTINCT
    numeric = False


class Compliance(Analyzer):  # Compliance.scala:37-53 (no additional preconditions)
    name = "Compliance"
    OP = L.OP_COMPLIANCE

    def __init__(self, instance: str, predicate: str, where: Optional[str] = None):
        self._instance = instance
        self.predicate = predicate
        self.where = where

    def _fields(self):
        return (self._instance, self.predicate, self.where)

    def _show(self):
        return (self._instance, self.predicate, ("opt", self.where))

    @property
    def instance(self):
        return self._instance

    def _lower(self, b):
        return (L.OP_COMPLIANCE, -1, -1, b.pred(self.predicate), b.pred(self.where))


class PatternMatch(_ColumnAnalyzer):  # PatternMatch.scala:37-56
    """Fraction of rows whose value contains a match of `pattern` (java.util.regex find()):
    sum(CASE WHEN where THEN (regexp_extract(column, pattern, 0) != '' ? 1 : 0) END) over
    conditionalCount(where).  A NULL value counts as 0; state NumMatchesAndCount.  The pattern is
    compiled into a byte-level search DFA walked on the GPU (deequ_amd/csrc/dq_regex.cpp)."""
    name = "PatternMatch"
    OP = L.OP_PATTERN_MATCH
    numeric = False

    def __init__(self, column: str, pattern, where: Optional[str] = None):
        super().__init__(column, where)
        self.pattern = pattern if isinstance(pattern, str) else pattern.pattern  # scala Regex / re.Pattern

    def _fields(self):
        return (self.column, self.pattern, self.where)

    def _show(self):
        return (self.column, self.pattern, ("opt", self.where))

    def _lower(self, b):
        from .predicates import UnsupportedPredicate
        from .table import type_code

        col = b.col(self.column)
        if type_code(b.by_name[self.column][1]) not in (L.TYPE_UTF8, L.TYPE_LARGE_UTF8):
            raise UnsupportedPredicate(f"PatternMatch on non-string column {self.column} (Spark casts it to string)")
        root = b.pool.add_regex(col, self.pattern, L.REGEX_EXTRACT_NONEMPTY)
        return (L.OP_PATTERN_MATCH, col, -1, root, b.pred(self.where))


class Patterns:  # PatternMatch.scala:58-74
    # http://emailregex.com
    EMAIL = (r"""(?:[a-z0-9!#$%&'*+/=?^_`{|}~-]+(?:\.[a-z0-9!#$%&'*+/=?^_`{|}~-]+)*|"(?:[\x01-\x08\x0b\x0c\x0e-\x1f\x21\x23-\x5b\x5d-\x7f]|\\[\x01-\x09\x0b\x0c\x0e-\x7f])*")"""
             r"""@(?:(?:[a-z0-9](?:[a-z0-9-]*[a-z0-9])?\.)+[a-z0-9](?:[a-z0-9-]*[a-z0-9])?|\[(?:(?:25[0-5]|2[0-4][0-9]|[01]?[0-9][0-9]?)\.){3}"""
             r"""(?:25[0-5]|2[0-4][0-9]|[01]?[0-9][0-9]?|[a-z0-9-]*[a-z0-9]:(?:[\x01-\x08\x0b\x0c\x0e-\x1f\x21-\x5a\x53-\x7f]|\\[\x01-\x09\x0b\x0c\x0e-\x7f])+)\])""")
    # https://mathiasbynens.be/demo/url-regex stephenhay
    URL = r"""(https?|ftp)://[^\s/$.?#].[^\s]*"""
    # look-ahead / backreference / \b: outside the GPU regex subset (UnsupportedPredicate -> fallback)
    SOCIAL_SECURITY_NUMBER_US = (r"""((?!219-09-9999|078-05-1120)(?!666|000|9\d{2})\d{3}-(?!00)\d{2}-(?!0{4})\d{4})|"""
                                 r"""((?!219 09 9999|078 05 1120)(?!666|000|9\d{2})\d{3} (?!00)\d{2} (?!0{4})\d{4})|"""
                                 r"""((?!219099999|078051120)(?!666|000|9\d{2})\d{3}(?!00)\d{2}(?!0{4})\d{4})""")
    CREDITCARD = (r"""\b(?:3[47]\d{2}([\ \-]?)\d{6}\1\d|(?:(?:4\d|5[1-5]|65)\d{2}|6011)([\ \-]?)\d{4}\2\d{4}\2)\d{4}\b""")


class Correlation(Analyzer):  # Correlation.scala:65-105
    name = "Correlation"
    entity = Entity.Mutlicolumn
    OP = L.OP_CORRELATION

    def __init__(self, firstColumn: str, secondColumn: str, where: Optional[str] = None):
        self.firstColumn = firstColumn
        self.secondColumn = secondColumn
        self.where = where

    def _fields(self):
        return (self.firstColumn, self.secondColumn, self.where)

    def _show(self):
        return (self.firstColumn, self.secondColumn, ("opt", self.where))

    @property
    def instance(self):
        return f"{self.firstColumn},{self.secondColumn}"

    def additionalPreconditions(self):
        return [Preconditions.hasColumn(self.firstColumn), Preconditions.isNumeric(self.firstColumn),
                Preconditions.hasColumn(self.secondColumn), Preconditions.isNumeric(self.secondColumn)]

    def _lower(self, b):
        return (L.OP_CORRELATION, b.col(self.firstColumn), b.col(self.secondColumn), -1, b.pred(self.where))


class DataTypeInstances:  # DataType.scala:32-38 (Enumeration: name -> id)
    Unknown = "Unknown"
    Fractional = "Fractional"
    Integral = "Integral"
    Boolean = "Boolean"
    String = "String"
    ALL = (Unknown, Fractional, Integral, Boolean, String)


def _ratio(count: int, total: int) -> float:
    # Long.toDouble / Long in the JVM: 0 / 0 -> NaN
    return count / total if total != 0 else (float("nan") if count == 0 else math.copysign(float("inf"), count))


def toDistribution(hist) -> "Distribution":
    """DataTypeHistogram.toDistribution (DataType.scala:98-114)."""
    from .metrics import Distribution, DistributionValue

    total = hist.numNull + hist.numString + hist.numBoolean + hist.numIntegral + hist.numFractional
    counts = {DataTypeInstances.Unknown: hist.numNull, DataTypeInstances.Fractional: hist.numFractional,
              DataTypeInstances.Integral: hist.numIntegral, DataTypeInstances.Boolean: hist.numBoolean,
              DataTypeInstances.String: hist.numString}
    return Distribution({k: DistributionValue(v, _ratio(v, total)) for k, v in counts.items()}, numberOfBins=5)


def determineType(dist) -> str:
    """DataTypeHistogram.determineType (DataType.scala:116-143)."""
    def ratio_of(key):
        v = dist.values.get(key)
        return 0.0 if v is None else v.ratio

    I = DataTypeInstances
    if ratio_of(I.Unknown) == 1.0:
        return I.Unknown
    if ratio_of(I.String) > 0.0 or (ratio_of(I.Boolean) > 0.0 and (ratio_of(I.Integral) > 0.0 or ratio_of(I.Fractional) > 0.0)):
        return I.String
    if ratio_of(I.Boolean) > 0.0:
        return I.Boolean
    if ratio_of(I.Fractional) > 0.0:
        return I.Fractional
    return I.Integral


class DataType(_ColumnAnalyzer):  # DataType.scala:152-183
    """stateful_datatype(conditionalSelection(column, where)): every row is NULL (null or `where` not
    TRUE), or its string form is classified FRACTIONAL / INTEGRAL / BOOLEAN / STRING
    (catalyst/StatefulDataType.scala:36-67).  The metric is a HistogramMetric."""
    name = "Histogram"
    OP = L.OP_DATATYPE
    numeric = False

    def computeMetricFrom(self, state):
        from .metrics import HistogramMetric, Success

        if state is not None:
            return HistogramMetric(self.column, Success(toDistribution(state)))
        return self.toFailureMetric(EmptyStateException(
            f"Empty state for analyzer {self}, all input values were NULL."))

    def toFailureMetric(self, e: BaseException):
        from .metrics import HistogramMetric

        return HistogramMetric(self.column, Failure(wrap_if_necessary(e)))
