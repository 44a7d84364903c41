"""Host-resident Arrow batches -> the fused GPU scan (libdqscan dq_arrow_import / dq_upload*).

The data path of a JVM-free drop-in: record batches arrive through the Arrow C Data Interface (Spark's
Arrow export, pyarrow, arrow-rs), are mapped without copying to host column buffers
(dq_arrow_import), copied by CPU threads into a pinned staging slot and DMA'd into a device slot on the
uploader's own stream (dq_upload), while the previous chunk scans (dq_upload_fence / dq_upload_release
order the plan's stream against the slot).  Reference seam: AnalysisRunner.runScanningAnalyzers'
data.agg over the DataFrame (analyzers/runners/AnalysisRunner.scala:279-326).
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Sequence

from . import _lib as L

_FORMAT_DTYPE = {"g": "f64", "l": "i64", "i": "i32", "u": "utf8", "U": "large_utf8", "f": "f32", "s": "i16",
                 "c": "i8", "b": "bool", "tdD": "date32"}  # + "tsu:<tz>" -> timestamp, "d:p,s" -> decimal(p,s)


class ArrowSchemaC(ctypes.Structure):
    pass


class ArrowArrayC(ctypes.Structure):
    pass


ArrowSchemaC._fields_ = [("format", ctypes.c_char_p), ("name", ctypes.c_char_p), ("metadata", ctypes.c_char_p),
                         ("flags", ctypes.c_int64), ("n_children", ctypes.c_int64),
                         ("children", ctypes.POINTER(ctypes.POINTER(ArrowSchemaC))),
                         ("dictionary", ctypes.POINTER(ArrowSchemaC)),
                         ("release", ctypes.CFUNCTYPE(None, ctypes.POINTER(ArrowSchemaC))),
                         ("private_data", ctypes.c_void_p)]
ArrowArrayC._fields_ = [("length", ctypes.c_int64), ("null_count", ctypes.c_int64), ("offset", ctypes.c_int64),
                        ("n_buffers", ctypes.c_int64), ("n_children", ctypes.c_int64),
                        ("buffers", ctypes.POINTER(ctypes.c_void_p)),
                        ("children", ctypes.POINTER(ctypes.POINTER(ArrowArrayC))),
                        ("dictionary", ctypes.POINTER(ArrowArrayC)),
                        ("release", ctypes.CFUNCTYPE(None, ctypes.POINTER(ArrowArrayC))),
                        ("private_data", ctypes.c_void_p)]


class HostColumn(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("nullable", ctypes.c_int32), ("n_rows", ctypes.c_int64),
                ("values", ctypes.c_void_p), ("validity", ctypes.c_void_p), ("offsets", ctypes.c_void_p),
                ("value_bytes", ctypes.c_int64), ("validity_bytes", ctypes.c_int64), ("offset_bytes", ctypes.c_int64),
                ("offset_base", ctypes.c_int64), ("validity_bit", ctypes.c_int32), ("reserved", ctypes.c_int32)]


def _bind():
    lib = L.lib
    if getattr(lib, "_dq_ingest_bound", False):
        return lib
    P = ctypes.POINTER
    lib.dq_arrow_import.restype = ctypes.c_int32
    lib.dq_arrow_import.argtypes = [P(ArrowSchemaC), P(ArrowArrayC), P(HostColumn)]
    lib.dq_uploader_create.restype = ctypes.c_int32
    lib.dq_uploader_create.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32,
                                       P(ctypes.c_void_p)]
    lib.dq_upload.restype = ctypes.c_int32
    lib.dq_upload.argtypes = [ctypes.c_void_p, P(HostColumn), ctypes.c_int32, P(L.ColumnView)]
    for f in ("dq_upload_fence", "dq_upload_release"):
        getattr(lib, f).restype = ctypes.c_int32
        getattr(lib, f).argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.dq_upload_sync.restype = ctypes.c_int32
    lib.dq_upload_sync.argtypes = [ctypes.c_void_p]
    lib.dq_uploader_destroy.restype = None
    lib.dq_uploader_destroy.argtypes = [ctypes.c_void_p]
    lib._dq_ingest_bound = True
    return lib


class ImportedArray:
    """One pyarrow array exported through the C Data Interface and mapped by dq_arrow_import; the
    exported structures are released by close() (the pyarrow array must outlive the upload)."""

    def __init__(self, arr):
        lib = _bind()
        self._arr = arr
        self.c_array, self.c_schema = ArrowArrayC(), ArrowSchemaC()
        arr._export_to_c(ctypes.addressof(self.c_array), ctypes.addressof(self.c_schema))
        self.host = HostColumn()
        st = lib.dq_arrow_import(ctypes.byref(self.c_schema), ctypes.byref(self.c_array), ctypes.byref(self.host))
        if st != L.DQ_OK:
            self.close()
            L.check(st)

    def close(self):
        for s in (self.c_array, self.c_schema):
            if s.release:
                s.release(ctypes.byref(s))


def arrow_schema(batch) -> List[tuple]:
    """(name, dtype, nullable) of a pyarrow RecordBatch / Table for ScanPlan."""
    import pyarrow as pa

    out = []
    for f in batch.schema:
        dt = {pa.float64(): "f64", pa.int64(): "i64", pa.int32(): "i32", pa.string(): "utf8",
              pa.large_string(): "large_utf8", pa.float32(): "f32", pa.int16(): "i16", pa.int8(): "i8",
              pa.bool_(): "bool", pa.date32(): "date32"}.get(f.type)
        if dt is None and pa.types.is_timestamp(f.type) and f.type.unit == "us":
            dt = "timestamp"
        if dt is None and pa.types.is_decimal128(f.type) and 1 <= f.type.precision <= 38 and 0 <= f.type.scale:
            dt = f"decimal({f.type.precision},{f.type.scale})"
        if dt is None:
            raise TypeError(f"column {f.name}: Arrow type {f.type} is not a GPU column type")
        out.append((f.name, dt, f.nullable))
    return out


class ArrowScanner:
    """Scan pyarrow record batches with a ScanPlan: upload chunk k + 1 while chunk k scans."""

    def __init__(self, plan, slot_bytes: int, n_slots: int = 2, host_threads: int = 0):
        import torch

        self.plan = plan
        self.lib = _bind()
        h = ctypes.c_void_p()
        L.check(self.lib.dq_uploader_create(plan.device, n_slots, slot_bytes, host_threads, ctypes.byref(h)))
        self.h = h
        self.stream = ctypes.c_void_p(torch.cuda.current_stream(plan.device).cuda_stream)

    def scan(self, batch) -> None:
        """Upload one batch (its columns in the plan's order) and enqueue its scan."""
        cols = [batch.column(batch.schema.get_field_index(n)) for n in self.plan.columns]
        cols = [c.combine_chunks() if hasattr(c, "combine_chunks") else c for c in cols]
        imported = [ImportedArray(c) for c in cols]
        try:
            hosts = (HostColumn * max(1, len(imported)))(*[i.host for i in imported])
            views = (L.ColumnView * max(1, len(imported)))()
            L.check(self.lib.dq_upload(self.h, hosts, len(imported), views))
        finally:
            for i in imported:
                i.close()
        L.check(self.lib.dq_upload_fence(self.h, self.stream))
        L.check(L.lib.dq_scan(self.plan.handle, views, batch.num_rows, self.plan.chunk))
        self.plan.chunk += 1
        L.check(self.lib.dq_upload_release(self.h, self.stream))

    def close(self) -> None:
        if self.h:
            self.lib.dq_uploader_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def scan_arrow(batches: Sequence, analyzers, slot_bytes: int = 0, n_slots: int = 2) -> List[L.State]:
    """Fused scan of host-resident Arrow record batches -> raw aggregation-result slot sets."""
    from .runner import ScanPlan

    batches = list(batches)
    plan = ScanPlan(analyzers, arrow_schema(batches[0]))
    if slot_bytes <= 0:
        slot_bytes = max(sum(b.get_total_buffer_size() for b in batches[:1]) * 2, 1 << 20)
    sc = ArrowScanner(plan, slot_bytes, n_slots)
    try:
        for b in batches:
            sc.scan(b)
        return plan.finish()
    finally:
        sc.close()
        plan.close()


def host_columns(batch) -> Dict[str, HostColumn]:
    """dq_arrow_import of every column of a batch (host only; for tests / diagnostics)."""
    out = {}
    for f in batch.schema:
        im = ImportedArray(batch.column(batch.schema.get_field_index(f.name)))
        out[f.name] = im.host
        im.close()
    return out
