"""Shared test helpers: build the same table for the oracle (host) and the product (device)."""
from __future__ import annotations

import math

import numpy as np

from oracle import dq_oracle as O


def oracle_columns(ds: dict):
    """reference_kats dataset -> ({name: OColumn}, n)"""
    cols = {}
    n = 0
    for name, (t, vals) in ds["columns"].items():
        valid = np.array([v is not None for v in vals], dtype=bool)
        if t == "utf8":
            v = [None if x is None else x.encode("utf-8") for x in vals]
        elif t == "f64":
            v = np.array([0.0 if x is None else x for x in vals], dtype=np.float64)
        else:
            v = np.array([0 if x is None else x for x in vals], dtype=np.int64 if t == "i64" else np.int32)
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
    if col.dtype == "f64":
        return raw[: n * 8].view(np.float64).copy(), valid, bm
    if col.dtype == "i64":
        return raw[: n * 8].view(np.int64).copy(), valid, bm
    if col.dtype == "i32":
        return raw[: n * 4].view(np.int32).copy(), valid, bm
    offs_raw = col.offsets.cpu().numpy()
    offs = offs_raw[: (n + 1) * (4 if col.dtype == "utf8" else 8)].view(np.int32 if col.dtype == "utf8" else np.int64)
    data = raw.tobytes()
    vals = [data[offs[i]:offs[i + 1]] if valid[i] else None for i in range(n)]
    return vals, valid, bm
