"""deequ_amd -- MI355X-native replacement of Deequ's fused single-pass metric scan.

The hot path (AnalysisRunner.runScanningAnalyzers / ScanShareableAnalyzer aggregation) runs in
libdqscan.so: hand-written gfx950 HIP kernels behind the C ABI in include/dqscan.h.  This package
is the host-side mirror of the reference's analyzer / state / runner API over that ABI.
"""
from ._lib import DQError, lib  # noqa: F401  (fails loudly if libdqscan.so is missing)
from .checks import (Check, CheckLevel, CheckStatus, ConstraintStatus, VerificationResult,  # noqa: F401
                     VerificationSuite)
from .analyzers import (ApproxCountDistinct, Completeness, Compliance, Correlation, DataType,  # noqa: F401
                        DataTypeInstances, Maximum, Mean, Minimum, PatternMatch, Patterns, Size, StandardDeviation,
                        Sum)
from .grouping import (CountDistinct, Distinctness, Entropy, FrequenciesAndNumRows, Histogram,  # noqa: F401
                       MutualInformation, Uniqueness, UniqueValueRatio)
from .metrics import (DoubleMetric, Distribution, DistributionValue, Entity, HistogramMetric,  # noqa: F401
                      KeyedDoubleMetric)
from .quantiles import ApproxQuantile, ApproxQuantiles  # noqa: F401
from .runner import AnalysisRunner, AnalyzerContext  # noqa: F401
from .state_provider import HdfsStateProvider, InMemoryStateProvider  # noqa: F401
from .states import (ApproxCountDistinctState, CorrelationState, DataTypeHistogram, MaxState, MeanState,  # noqa: F401
                     MinState, NumMatches, NumMatchesAndCount, StandardDeviationState, SumState)
from .table import Column, Table  # noqa: F401
