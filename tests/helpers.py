"""Shared test helpers: build the same table for the oracle (host) and the product (device)."""
from __future__ import annotations

import math

import numpy as np

from oracle import dq_oracle as O


_INT_NP = {"i64": np.int64, "i32": np.int32, "i16": np.int16, "i8": np.int8, "date32": np.int32,
           "timestamp": np.int64}


def oracle_columns(ds: dict):
    """reference_kats dataset -> ({name: OColumn}, n)"""
    cols = {}
    n = 0
    for name, (t, vals) in ds["columns"].items():
        valid = np.array([v is not None for v in vals], dtype=bool)
        if t == "utf8":
            v = [None if x is None else x.encode("utf-8") for x in vals]
        elif t in ("f64", "f32"):
            v = np.array([0.0 if x is None else x for x in vals], dtype=np.float64 if t == "f64" else np.float32)
        elif t == "bool":
            v = np.array([False if x is None else bool(x) for x in vals], dtype=bool)
        elif O.decimal_ps(t):  # decimal text -> unscaled ints at the column's scale
            from deequ_amd.table import decimal_unscaled

            v = [0 if x is None else decimal_unscaled(x, O.decimal_ps(t)[1]) for x in vals]
        else:
            v = np.array([0 if x is None else x for x in vals], dtype=_INT_NP[t])
        cols[name] = O.OColumn(t, v, valid)
        n = len(vals)
    return cols, n


def close(a: float, b: float, rel: float = 1e-12, abs_: float = 0.0) -> bool:
    if isinstance(a, float) and isinstance(b, float) and math.isnan(a) and math.isnan(b):
        return True
    if a == b:
        return True
    return abs(a - b) <= max(rel * max(abs(a), abs(b)), abs_)


def host_column(col, n):
    """device Column -> (values ndarray or list[bytes], valid bool ndarray, validity bitmap uint8)"""
    bm = None if col.validity is None else col.validity.cpu().numpy()
    valid = np.ones(n, dtype=bool) if bm is None else np.unpackbits(bm, bitorder="little")[:n].astype(bool)
    raw = col.values.cpu().numpy()
    fixed = {"f64": np.float64, "i64": np.int64, "i32": np.int32, "f32": np.float32, "i16": np.int16, "i8": np.int8,
             "date32": np.int32, "timestamp": np.int64}
    if col.dtype in fixed:
        w = np.dtype(fixed[col.dtype]).itemsize
        return raw[: n * w].view(fixed[col.dtype]).copy(), valid, bm
    if col.dtype == "bool":
        return np.unpackbits(raw, bitorder="little")[:n].astype(bool), valid, bm
    if O.decimal_ps(col.dtype):  # 16-byte two's-complement unscaled values -> Python ints
        w = raw[: n * 16].view(np.uint64).reshape(-1, 2)
        return [int(lo) | int(hi) << 64 if hi < (1 << 63) else (int(lo) | int(hi) << 64) - (1 << 128)
                for lo, hi in w], valid, bm
    offs_raw = col.offsets.cpu().numpy()
    offs = offs_raw[: (n + 1) * (4 if col.dtype == "utf8" else 8)].view(np.int32 if col.dtype == "utf8" else np.int64)
    data = raw.tobytes()
    vals = [data[offs[i]:offs[i + 1]] if valid[i] else None for i in range(n)]
    return vals, valid, bm
