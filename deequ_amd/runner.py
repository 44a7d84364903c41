"""AnalysisRunner: the drop-in replacement of the fused single-pass scan.

Mirrors analyzers/runners/AnalysisRunner.scala (paths relative to src/main/scala/com/amazon/deequ/):
  doAnalysisRun            :98-193   preconditions -> failure metrics, then the scan
  runScanningAnalyzers     :279-326  ONE fused pass for every scan-shareable analyzer; an
                                     aggregation failure fails every analyzer of the pass (:310-313)
  successOrFailureMetricFrom :330-343 per-analyzer decode failures stay local
and AnalyzerContext (analyzers/runners/AnalyzerContext.scala:29-105), AnalysisRunBuilder
(analyzers/runners/AnalysisRunBuilder.scala:25-186).

`data` is a deequ_amd.table.Table, or a list of Tables = row chunks of one dataset scanned in
order (dq_scan chunk_index 0, 1, ...), e.g. uploaded batches.
"""
from __future__ import annotations

import ctypes
import json
import math
from typing import Dict, Iterable, List, Optional, Sequence

from . import _lib as L
from .analyzers import Analyzer, PlanBuilder, Preconditions, data_schema
from .metrics import DoubleMetric, UnsupportedOnGpuPathException
from .predicates import UnsupportedPredicate
from .states import State
from .table import Table


def _chunks(data) -> List[Table]:
    return [data] if isinstance(data, Table) else list(data)


class ScanPlan:
    """One dq_plan: the fused scan of a set of analyzers over tables with a fixed schema.

    pred_pass (dq_plan_options.pred_pass): "auto" runs the predicate program as the kernel compiled for it
    when the generator takes it, else the interpreter; "interpreter" forces the interpreter; "compiled"
    requires the compiled kernel (plan creation fails with DQError DQ_E_UNSUPPORTED instead of falling back)."""

    def __init__(self, analyzers: Sequence[Analyzer], schema, device: Optional[int] = None, pred_pass: str = "auto"):
        import torch

        self.analyzers = list(analyzers)
        b = PlanBuilder(schema)
        specs = (L.AnalyzerSpec * max(1, len(self.analyzers)))()
        for i, a in enumerate(self.analyzers):
            op, ca, cb, pr, wr = a._lower(b)
            specs[i].op, specs[i].col_a, specs[i].col_b, specs[i].pred_root, specs[i].where_root = op, ca, cb, pr, wr
        self.columns = list(b.columns)
        sch = b.schema_ctypes()
        pool, npred = b.pool.as_ctypes()
        if device is None:
            device = torch.cuda.current_device()
        self.device = device
        self._specs, self._sch, self._pool = specs, sch, pool
        handle = ctypes.c_void_p()
        pats, npats = b.pool.patterns_ctypes()
        self._pats = pats
        opts = L.PlanOptions(ctypes.sizeof(L.PlanOptions), L.PRED_PASS[pred_pass])
        L.check(L.lib.dq_plan_create_opts(specs, len(self.analyzers), sch, len(self.columns), pool, npred, pats, npats,
                                          ctypes.byref(opts), device, ctypes.byref(handle)))
        self.handle = handle
        self.chunk = 0
        with torch.cuda.device(device):
            L.check(L.lib.dq_plan_set_stream(self.handle, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))

    def bytes_per_row(self) -> float:
        return L.lib.dq_plan_bytes_per_row_x1000(self.handle) / 1000.0

    def num_launches(self) -> int:
        return L.lib.dq_plan_num_launches(self.handle)

    def enable_timing(self, on: bool = True) -> None:
        L.check(L.lib.dq_plan_enable_timing(self.handle, 1 if on else 0))

    def variant_bytes_per_row(self, variant: int) -> float:
        return L.lib.dq_plan_variant_bytes_per_row_x1000(self.handle, variant) / 1000.0

    def pred_compiled(self):
        """(True, origin of the code object: "hiprtc" / "disk cache" / "process cache") when the predicate pass
        runs as the kernel compiled for this plan's program, else (False, the reason the interpreter runs it)
        -- dq_plan_pred_compiled."""
        buf = ctypes.create_string_buffer(2048)
        on = L.lib.dq_plan_pred_compiled(self.handle, buf, len(buf))
        return bool(on), buf.value.decode("utf-8", "replace")

    def pred_wait(self, timeout_ms: int = -1) -> bool:
        """Wait for a background compile of the predicate kernel (AUTO); True when the next scan runs it."""
        r = L.lib.dq_plan_pred_wait(self.handle, timeout_ms)
        if r < 0:
            L.check(r)
        return bool(r)

    def create_time(self):
        """(host ms dq_plan_create spent, of which ms obtaining the compiled predicate kernel)."""
        total, jit = ctypes.c_double(), ctypes.c_double()
        L.check(L.lib.dq_plan_create_time(self.handle, ctypes.byref(total), ctypes.byref(jit)))
        return total.value, jit.value

    def kernel_bytes_per_row(self, kernel: int) -> float:
        """Algorithmic bytes per row of timing kernel `kernel` (0 pred, 2 pair, 16+v variant v; no UTF8 data)."""
        return L.lib.dq_plan_kernel_bytes_per_row_x1000(self.handle, kernel) / 1000.0

    def kernel_time(self, kernel: int):
        """(total ms, launches) of kernel 0 pred / 1 column (all) / 2 pair / 3 finalize / 16+v column
        variant v, since enable_timing."""
        ms, n = ctypes.c_double(), ctypes.c_int64()
        L.check(L.lib.dq_plan_kernel_time(self.handle, kernel, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def scan(self, table: Table) -> None:
        views = (L.ColumnView * max(1, len(self.columns)))()
        for i, name in enumerate(self.columns):
            views[i] = table.columns[name].view()
        L.check(L.lib.dq_scan(self.handle, views, table.num_rows, self.chunk))
        self.chunk += 1

    def finish(self) -> List[L.State]:
        out = (L.State * max(1, len(self.analyzers)))()
        L.check(L.lib.dq_finish(self.handle, out))
        return [out[i] for i in range(len(self.analyzers))]

    def reset(self) -> None:
        L.check(L.lib.dq_plan_reset(self.handle))
        self.chunk = 0

    def close(self) -> None:
        if self.handle:
            L.lib.dq_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _lower_all(analyzers: Sequence[Analyzer], schema):
    b = PlanBuilder(schema)
    specs = (L.AnalyzerSpec * max(1, len(analyzers)))()
    for i, a in enumerate(analyzers):
        op, ca, cb, pr, wr = a._lower(b)
        specs[i].op, specs[i].col_a, specs[i].col_b, specs[i].pred_root, specs[i].where_root = op, ca, cb, pr, wr
    return b, specs


def _explain(b: PlanBuilder, specs, n_specs: int, pred_pass: str):
    """(status, text or dq_last_error) of dq_plan_explain over lowered specs (host only)."""
    sch = b.schema_ctypes()
    pool, npred = b.pool.as_ctypes()
    pats, npats = b.pool.patterns_ctypes()
    opts = L.PlanOptions(ctypes.sizeof(L.PlanOptions), L.PRED_PASS[pred_pass])
    args = (specs, n_specs, sch, len(b.columns), pool, npred, pats, npats, ctypes.byref(opts))
    n = L.lib.dq_plan_explain(*args, None, 0)
    if n < 0:
        return int(n), L.lib.dq_last_error().decode("utf-8", "replace")
    buf = ctypes.create_string_buffer(int(n))
    L.lib.dq_plan_explain(*args, buf, n)
    return L.DQ_OK, buf.value.decode("utf-8", "replace")


def explain(analyzers: Sequence[Analyzer], schema, pred_pass: str = "auto") -> str:
    """The plan dq_plan_create would build for these analyzers, lowered on the host only (dq_plan_explain: no
    GPU): launches per scan, column-pass variants, the predicate program and the generated predicate kernel;
    an analyzer set over one plan's capacity is shown as the fused plans dq_plan_create splits it into."""
    b, specs = _lower_all(analyzers, schema)
    rc, text = _explain(b, specs, len(analyzers), pred_pass)
    L.check(rc)
    return text


def scan_results(data, analyzers: Sequence[Analyzer], pred_pass: str = "auto") -> List[L.State]:
    """Fused scan of all chunks -> raw aggregation-result slot sets, one per analyzer."""
    chunks = _chunks(data)
    plan = ScanPlan(analyzers, chunks[0].schema, pred_pass=pred_pass)
    try:
        for t in chunks:
            plan.scan(t)
        return plan.finish()
    finally:
        plan.close()


def scan_states(data, analyzers: Sequence[Analyzer], pred_pass: str = "auto") -> Dict[Analyzer, Optional[State]]:
    res = scan_results(data, analyzers, pred_pass)
    return {a: a._from_result(r) for a, r in zip(analyzers, res)}


def gpu_eligible(analyzer: Analyzer, schema) -> Optional[Exception]:
    """None if the analyzer lowers into a GPU plan; else the reason (-> fallback set).

    Two checks, both on the host: the predicate compiler (SQL text outside the GPU grammar), then the planner
    on this analyzer alone (dq_plan_explain: e.g. a predicate nested deeper than the device stack).  Capacity
    limits of a plan are never a routing reason: dq_plan_create splits a set over them into several fused
    plans, so only what does not fit a plan by itself goes to the fallback."""
    try:
        b, specs = _lower_all([analyzer], schema)
    except UnsupportedPredicate as e:
        return e
    except Exception:
        return None  # a missing column etc. is an aggregation error, not a routing decision
    rc, msg = _explain(b, specs, 1, "auto")
    if rc == L.DQ_E_UNSUPPORTED:
        return UnsupportedPredicate(msg)
    return None


class AnalyzerContext:
    """analyzers/runners/AnalyzerContext.scala:29-105"""

    def __init__(self, metricMap: Optional[Dict[Analyzer, DoubleMetric]] = None):
        self.metricMap: Dict[Analyzer, DoubleMetric] = dict(metricMap or {})

    @staticmethod
    def empty() -> "AnalyzerContext":
        return AnalyzerContext()

    @property
    def allMetrics(self) -> List[DoubleMetric]:
        return list(self.metricMap.values())

    def metric(self, analyzer: Analyzer) -> Optional[DoubleMetric]:
        return self.metricMap.get(analyzer)

    def __add__(self, other: "AnalyzerContext") -> "AnalyzerContext":
        m = dict(self.metricMap)
        m.update(other.metricMap)
        return AnalyzerContext(m)

    def successMetricsAsJson(self) -> str:
        rows = []
        for m in (d for metric in self.allMetrics for d in metric.flatten()):  # AnalyzerContext.scala:90
            if m.value.isSuccess:
                rows.append({"entity": m.entity.value, "instance": m.instance, "name": m.name,
                             "value": m.value.get()})
        return json.dumps(rows)


class AnalysisRunner:
    @staticmethod
    def onData(data) -> "AnalysisRunBuilder":
        return AnalysisRunBuilder(data)

    @staticmethod
    def doAnalysisRun(data, analyzers: Sequence[Analyzer], aggregateWith=None, saveStatesWith=None) -> AnalyzerContext:
        if not analyzers:
            return AnalyzerContext.empty()
        all_analyzers = list(dict.fromkeys(analyzers))  # case-class equality dedup, order kept
        schema = data_schema(data)
        passed, failures = [], {}
        for a in all_analyzers:
            err = Preconditions.findFirstFailing(schema, a.preconditions())
            if err is None:
                passed.append(a)
            else:
                failures[a] = a.toFailureMetric(err)
        grouping = [a for a in passed if getattr(a, "grouping", False)]
        scanning = [a for a in passed if not getattr(a, "grouping", False)]
        ctx = AnalysisRunner.runScanningAnalyzers(data, scanning, aggregateWith, saveStatesWith)
        by_cols: Dict[tuple, List[Analyzer]] = {}
        for a in grouping:  # AnalysisRunner.scala:160-180: one frequency computation per column set
            if getattr(a, "direct", False):  # MutualInformation: its own device pass
                ctx = ctx + AnalyzerContext({a: a.calculate(data, aggregateWith, saveStatesWith)})
                continue
            by_cols.setdefault(tuple(a.groupingColumns()), []).append(a)
        for cols, group in by_cols.items():
            ctx = ctx + AnalysisRunner.runGroupingAnalyzers(data, list(cols), group, aggregateWith, saveStatesWith)
        return AnalyzerContext(failures) + ctx

    @staticmethod
    def runGroupingAnalyzers(data, columns, analyzers, aggregateWith=None, saveStatesWith=None) -> AnalyzerContext:
        """AnalysisRunner.scala:249-277 and runAnalyzersForParticularGrouping: frequencies once (GPU),
        the state of the first analyzer merged with a loaded one, persisted for every analyzer."""
        from .grouping import build_frequencies

        try:
            state = build_frequencies(data, columns)
            if aggregateWith is not None:
                prev = aggregateWith.load(analyzers[0])
                if prev is not None:
                    state = state.sum(prev)
        except Exception as e:
            return AnalyzerContext({a: a.toFailureMetric(e) for a in analyzers})
        metrics = {}
        for a in analyzers:
            try:
                if saveStatesWith is not None:
                    saveStatesWith.persist(a, state)
                metrics[a] = a.computeMetricFrom(state)
            except Exception as e:
                metrics[a] = a.toFailureMetric(e)
        return AnalyzerContext(metrics)

    @staticmethod
    def runScanningAnalyzers(data, analyzers: Sequence[Analyzer], aggregateWith=None,
                             saveStatesWith=None) -> AnalyzerContext:
        if not analyzers:
            return AnalyzerContext.empty()
        schema = data_schema(data)
        gpu, fallback = [], {}
        for a in analyzers:
            reason = gpu_eligible(a, schema)
            if reason is None:
                gpu.append(a)
            else:
                fallback[a] = a.toFailureMetric(UnsupportedOnGpuPathException(
                    f"{a} is outside the GPU-eligible set ({reason}); a Spark integration keeps it on data.agg"))
        metrics: Dict[Analyzer, DoubleMetric] = {}
        if gpu:
            try:
                results = scan_results(data, gpu)
                for a, r in zip(gpu, results):
                    metrics[a] = AnalysisRunner._success_or_failure(a, r, aggregateWith, saveStatesWith)
            except Exception as e:  # AnalysisRunner.scala:310-313: the whole pass fails
                metrics = {a: a.toFailureMetric(e) for a in gpu}
        metrics.update(fallback)
        return AnalyzerContext(metrics)

    @staticmethod
    def _success_or_failure(a: Analyzer, r: L.State, aggregateWith, saveStatesWith) -> DoubleMetric:
        try:
            return a.calculateMetric(a._from_result(r), aggregateWith, saveStatesWith)
        except Exception as e:
            return a.toFailureMetric(e)

    @staticmethod
    def runOnAggregatedStates(schema, analyzers: Sequence[Analyzer], stateLoaders: Sequence,
                              saveStatesWith=None) -> AnalyzerContext:
        """AnalysisRunner.scala:375-446: merge persisted states without touching data."""
        from .state_provider import InMemoryStateProvider

        if not analyzers or not stateLoaders:
            return AnalyzerContext.empty()
        agg = InMemoryStateProvider()
        metrics = {}
        for a in dict.fromkeys(analyzers):
            err = Preconditions.findFirstFailing(schema, a.preconditions())
            if err is not None:
                metrics[a] = a.toFailureMetric(err)
                continue
            try:
                for loader in stateLoaders:
                    a.aggregateStateTo(agg, loader, agg)
                m = a.loadStateAndComputeMetric(agg)
                if m is None:
                    m = a.computeMetricFrom(None)
                if saveStatesWith is not None:
                    s = agg.load(a)
                    if s is not None:
                        saveStatesWith.persist(a, s)
                metrics[a] = m
            except Exception as e:
                metrics[a] = a.toFailureMetric(e)
        return AnalyzerContext(metrics)


class AnalysisRunBuilder:
    def __init__(self, data):
        self.data = data
        self.analyzers: List[Analyzer] = []
        self._aggregateWith = None
        self._saveStatesWith = None

    def addAnalyzer(self, a: Analyzer) -> "AnalysisRunBuilder":
        self.analyzers.append(a)
        return self

    def addAnalyzers(self, analyzers: Iterable[Analyzer]) -> "AnalysisRunBuilder":
        self.analyzers.extend(analyzers)
        return self

    def aggregateWith(self, loader) -> "AnalysisRunBuilder":
        self._aggregateWith = loader
        return self

    def saveStatesWith(self, persister) -> "AnalysisRunBuilder":
        self._saveStatesWith = persister
        return self

    def run(self) -> AnalyzerContext:
        return AnalysisRunner.doAnalysisRun(self.data, self.analyzers, self._aggregateWith, self._saveStatesWith)
