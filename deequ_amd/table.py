"""HBM-resident columnar tables (Arrow physical layout) handed to the scan.

A Column owns device buffers (torch CUDA/HIP tensors are used purely as device allocations):
values (f64 / f32 / i64 / i32 / i16 / i8 / date32 / timestamp, decimal(p,s) as 16-byte two's-complement unscaled
integers, bit-packed bool, or UTF-8 bytes), an optional LSB-first validity bitmap, and int32
(utf8) / int64 (large_utf8) offsets.  Buffers are allocated with the padding dqscan.h requires:
values 16-byte aligned, bitmaps readable in whole 32-bit words, UTF-8 data readable up to the
next 4-byte boundary past the last string.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L

DTYPES = {"f64": L.TYPE_F64, "i64": L.TYPE_I64, "i32": L.TYPE_I32, "utf8": L.TYPE_UTF8,
          "large_utf8": L.TYPE_LARGE_UTF8, "f32": L.TYPE_F32, "i16": L.TYPE_I16, "i8": L.TYPE_I8,
          "bool": L.TYPE_BOOL, "date32": L.TYPE_DATE32, "timestamp": L.TYPE_TIMESTAMP}
# Preconditions.isNumeric (Analyzer.scala:322-334): ByteType .. DoubleType, and DecimalType ("decimal(p,s)")
NUMERIC = ("f64", "i64", "i32", "f32", "i16", "i8")


def decimal_ps(dtype: str) -> Optional[Tuple[int, int]]:
    """(precision, scale) of a "decimal(p,s)" dtype (DecimalType(p, s)), else None."""
    if not dtype.startswith("decimal(") or not dtype.endswith(")"):
        return None
    p, s = dtype[8:-1].split(",")
    return int(p), int(s)


def is_numeric(dtype: str) -> bool:
    return dtype in NUMERIC or decimal_ps(dtype) is not None


def type_code(dtype: str) -> int:
    ps = decimal_ps(dtype)
    return L.decimal_type(*ps) if ps else DTYPES[dtype]


def decimal_unscaled(v, scale: int) -> int:
    """A value as the unscaled integer of DecimalType(_, scale): an int is taken as the value itself, a
    decimal.Decimal / str / float through its exact decimal value, rounded HALF_UP to the scale (Spark's
    Decimal.changePrecision)."""
    import decimal

    d = v if isinstance(v, decimal.Decimal) else decimal.Decimal(str(v) if isinstance(v, float) else v)
    return int((d.scaleb(scale)).quantize(decimal.Decimal(1), rounding=decimal.ROUND_HALF_UP))
# fixed-width physical layouts (bool: bit-packed values; date32: int32 days since 1970-01-01; timestamp: int64 us)
_NP = {"f64": np.float64, "i64": np.int64, "i32": np.int32, "f32": np.float32, "i16": np.int16, "i8": np.int8,
       "date32": np.int32, "timestamp": np.int64}
FIXED = tuple(_NP) + ("bool",)


def _torch():
    import torch

    return torch


def _pad_u8(a: np.ndarray, mult: int, extra: int = 0) -> np.ndarray:
    n = len(a)
    total = ((n + mult - 1) // mult) * mult + extra
    out = np.zeros(max(total, mult), dtype=np.uint8)
    out[:n] = a
    return out


def pack_validity(valid: np.ndarray) -> np.ndarray:
    """bool[n] -> Arrow LSB-first bitmap padded to whole 64-bit words (+1 word)."""
    bits = np.packbits(np.asarray(valid, dtype=bool), bitorder="little")
    return _pad_u8(bits, 8, 8)


@dataclass
class Column:
    name: str
    dtype: str
    n_rows: int
    values: object                 # torch tensor on the device
    validity: Optional[object]     # torch uint8 tensor or None (no nulls)
    offsets: Optional[object] = None
    nullable: bool = True
    data_bytes: int = 0            # UTF-8 payload bytes (for traffic accounting)

    def view(self) -> L.ColumnView:
        v = L.ColumnView()
        v.values = self.values.data_ptr() if self.values is not None else None
        v.validity = self.validity.data_ptr() if self.validity is not None else None
        v.offsets = self.offsets.data_ptr() if self.offsets is not None else None
        v.reserved = 0
        return v

    @property
    def type_code(self) -> int:
        return type_code(self.dtype)


class Table:
    """An ordered set of equally long device columns (the scan input of one chunk / shard)."""

    def __init__(self, columns: Sequence[Column]):
        self.columns: Dict[str, Column] = {}
        n = None
        for c in columns:
            if n is None:
                n = c.n_rows
            elif c.n_rows != n:
                raise ValueError("columns differ in length")
            self.columns[c.name] = c
        self.num_rows = n or 0

    @property
    def schema(self) -> List[Tuple[str, str, bool]]:
        return [(c.name, c.dtype, c.nullable) for c in self.columns.values()]

    def count(self) -> int:
        return self.num_rows

    # -------------------------------------------------------------------- construction helpers
    @staticmethod
    def from_pydict(data: Dict[str, Tuple[str, Iterable]], device: str = "cuda", nullable: Optional[Dict[str, bool]] = None) -> "Table":
        """{"att1": ("i32", [1, None, 3]), "name": ("utf8", ["a", None])} -> device Table."""
        cols = []
        for name, (dtype, vals) in data.items():
            vals = list(vals)
            valid = np.array([v is not None for v in vals], dtype=bool)
            nl = True if nullable is None else nullable.get(name, True)
            if dtype == "bool":
                arr = np.array([False if v is None else bool(v) for v in vals], dtype=bool)
                cols.append(column_from_numpy(name, dtype, arr, valid, device=device, nullable=nl))
            elif dtype in FIXED:
                arr = np.array([0 if v is None else v for v in vals], dtype=_NP[dtype])
                cols.append(column_from_numpy(name, dtype, arr, valid, device=device, nullable=nl))
            elif decimal_ps(dtype):
                sc = decimal_ps(dtype)[1]
                u = [0 if v is None else decimal_unscaled(v, sc) for v in vals]
                cols.append(column_from_numpy(name, dtype, u, valid, device=device, nullable=nl))
            else:
                b = [None if v is None else (v.encode("utf-8") if isinstance(v, str) else bytes(v)) for v in vals]
                cols.append(utf8_column(name, b, device=device, large=(dtype == "large_utf8"), nullable=nl))
        return Table(cols)


def column_from_numpy(name: str, dtype: str, values: np.ndarray, valid: Optional[np.ndarray] = None,
                      device: str = "cuda", nullable: bool = True) -> Column:
    torch = _torch()
    if dtype == "bool":  # Arrow boolean: LSB-first bit-packed values, read as whole 32-bit words
        n = len(values)
        raw = pack_validity(np.asarray(values, dtype=bool))
        raw = _pad_u8(raw, 16, 16)
    elif decimal_ps(dtype):  # Arrow decimal128: the unscaled values (Python ints) as 16-byte little-endian
        p, _ = decimal_ps(dtype)
        L.decimal_type(p, 0)  # (validates the precision)
        n = len(values)
        mask = (1 << 64) - 1
        w = np.zeros((n, 2), dtype=np.uint64)
        if n:
            u = [int(v) for v in values]
            if any(abs(v) >= 10 ** p for v in u):
                raise ValueError(f"a value exceeds the precision of {dtype}")
            w[:, 0] = [v & mask for v in u]
            w[:, 1] = [(v >> 64) & mask for v in u]
        raw = _pad_u8(w.view(np.uint8).reshape(-1), 16, 16)
    else:
        values = np.ascontiguousarray(values, dtype=_NP[dtype])
        n = len(values)
        raw = _pad_u8(values.view(np.uint8), 16, 16)
    vt = torch.from_numpy(raw).to(device)
    bt = None
    if valid is not None and nullable:
        bt = torch.from_numpy(pack_validity(valid)).to(device)
    return Column(name, dtype, n, vt, bt, None, nullable=nullable and valid is not None)


def utf8_column(name: str, values: Sequence[Optional[bytes]], device: str = "cuda", large: bool = False,
                nullable: bool = True) -> Column:
    torch = _torch()
    n = len(values)
    valid = np.array([v is not None for v in values], dtype=bool)
    lens = np.array([0 if v is None else len(v) for v in values], dtype=np.int64)
    offs = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lens, out=offs[1:])
    if not large and offs[-1] >= 2 ** 31:
        raise ValueError("utf8 chunk exceeds 2 GiB; use large_utf8")
    data = b"".join(v for v in values if v is not None)
    raw = _pad_u8(np.frombuffer(data, dtype=np.uint8) if data else np.zeros(0, np.uint8), 16, 16)
    offs_np = offs if large else offs.astype(np.int32)
    ot = torch.from_numpy(_pad_u8(offs_np.view(np.uint8), 16, 16)).to(device)
    return Column(name, "large_utf8" if large else "utf8", n, torch.from_numpy(raw).to(device),
                  torch.from_numpy(pack_validity(valid)).to(device) if nullable else None, ot,
                  nullable=nullable, data_bytes=int(offs[-1]))
