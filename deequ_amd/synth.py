"""Seeded synthetic device tables for tests and bench.py (test/bench infrastructure, not the product).

Values are generated on the device by libdqsynth.so (counter-based RNG, so every chunk / shard is a
pure function of (seed, global row index)); see csrc/dq_synth.hip for the distributions.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Sequence

from .table import Column, Table, is_numeric

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(_HERE, "libdqsynth.so")
        if not os.path.exists(path):
            raise ImportError(f"{path} missing: run `make -C deequ_amd`")
        L = ctypes.CDLL(path)
        i64, u64, vp, d, i32 = ctypes.c_int64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_double, ctypes.c_int32
        L.dqs_f64.argtypes = [vp, i64, i64, u64, d, d, vp]
        L.dqs_corr.argtypes = [vp, i64, i64, u64, u64, d, d, d, vp]
        L.dqs_i64.argtypes = [vp, i64, i64, u64, u64, i64, vp]
        L.dqs_validity.argtypes = [vp, i64, i64, u64, d, vp]
        L.dqs_utf8_lengths.argtypes = [vp, i64, i64, u64, u64, i32, i32, vp]
        L.dqs_utf8_bytes.argtypes = [vp, vp, i64, i64, u64, u64, vp]
        L.dqs_i64_to_i32.argtypes = [vp, vp, i64, vp]
        _lib = L
    return _lib


def _stream():
    import torch

    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _check(rc):
    if rc != 0:
        raise RuntimeError(f"synth kernel launch failed: hipError {rc}")


def _alloc(nbytes: int):
    import torch

    n = ((nbytes + 15) // 16) * 16 + 16
    return torch.empty(n, dtype=torch.uint8, device="cuda")


def validity(n: int, seed: int, null_frac: float, row0: int = 0):
    if null_frac <= 0.0:
        return None
    assert row0 % 32 == 0
    buf = _alloc(((n + 63) // 64) * 8 + 8)
    _check(lib().dqs_validity(buf.data_ptr(), row0, n, seed, null_frac, _stream()))
    return buf


def f64_column(name, n, seed, mean=0.0, sd=1.0, null_frac=0.0, row0=0) -> Column:
    v = _alloc(n * 8)
    _check(lib().dqs_f64(v.data_ptr(), row0, n, seed, mean, sd, _stream()))
    bm = validity(n, seed ^ 0xABCDEF, null_frac, row0)
    return Column(name, "f64", n, v, bm, None, nullable=bm is not None)


def corr_column(name, n, seed, col_seed, a, b, offset, null_frac=0.0, row0=0) -> Column:
    v = _alloc(n * 8)
    _check(lib().dqs_corr(v.data_ptr(), row0, n, seed, col_seed, a, b, offset, _stream()))
    bm = validity(n, col_seed ^ 0x1234567, null_frac, row0)
    return Column(name, "f64", n, v, bm, None, nullable=bm is not None)


def i64_column(name, n, seed, distinct, base=0, null_frac=0.0, row0=0) -> Column:
    v = _alloc(n * 8)
    _check(lib().dqs_i64(v.data_ptr(), row0, n, seed, distinct, base, _stream()))
    bm = validity(n, seed ^ 0xABCDEF, null_frac, row0)
    return Column(name, "i64", n, v, bm, None, nullable=bm is not None)


def i32_column(name, n, seed, distinct, base=0, null_frac=0.0, row0=0) -> Column:
    import torch

    tmp = _alloc(n * 8)
    _check(lib().dqs_i64(tmp.data_ptr(), row0, n, seed, distinct, base, _stream()))
    v = _alloc(n * 4)
    _check(lib().dqs_i64_to_i32(v.data_ptr(), tmp.data_ptr(), n, _stream()))
    del tmp
    bm = validity(n, seed ^ 0xABCDEF, null_frac, row0)
    return Column(name, "i32", n, v, bm, None, nullable=bm is not None)


def utf8_column(name, n, seed, distinct, lmin=8, lmax=24, null_frac=0.0, row0=0, large=False,
                null_empty=False) -> Column:
    """null_empty: NULL rows get empty slots (offsets[r + 1] == offsets[r]), as Spark's and Arrow's writers
    emit them; otherwise the validity is drawn independently of the lengths (a NULL row keeps its bytes)."""
    import torch

    lens = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    lens[0] = 0
    _check(lib().dqs_utf8_lengths(lens[1:].data_ptr(), row0, n, seed, distinct, lmin, lmax, _stream()))
    bm = validity(n, seed ^ 0xABCDEF, null_frac, row0)
    if null_empty and bm is not None:
        r = torch.arange(n, device="cuda")
        lens[1:] *= ((bm[r >> 3].to(torch.int64) >> (r & 7)) & 1)
        del r
    offs = torch.cumsum(lens, 0)
    del lens
    total = int(offs[-1].item())
    if not large and total >= 2 ** 31:
        raise ValueError("utf8 chunk > 2 GiB: use large=True or smaller chunks")
    data = _alloc(total)
    _check(lib().dqs_utf8_bytes(data.data_ptr(), offs.data_ptr(), row0, n, seed, distinct, _stream()))
    if large:
        o = _alloc((n + 1) * 8)
        o[: (n + 1) * 8].copy_(offs.view(torch.uint8))
    else:
        o = _alloc((n + 1) * 4)
        _check(lib().dqs_i64_to_i32(o.data_ptr(), offs.data_ptr(), n + 1, _stream()))
    del offs
    return Column(name, "large_utf8" if large else "utf8", n, data, bm, o, nullable=bm is not None, data_bytes=total)


# ---------------------------------------------------------------------------------------------
# benchmark configurations
# ---------------------------------------------------------------------------------------------
INT_DISTINCT = [1000, 1_000_000, 100_000_000, 1 << 62]
STR_DISTINCT = [1000, 1_000_000, 100_000_000, 0]  # 0 = unique (a fresh id per row)


def c2_table(n, row0=0, seed=42, null_frac=0.10) -> Table:
    """8 fp64 columns, column c ~ N(1000 c, (1 + c)^2), 10% nulls."""
    return Table([f64_column(f"c{c}", n, seed + c, 1000.0 * c, 1.0 + c, null_frac, row0) for c in range(8)])


def c3_table(n, row0=0, seed=42, null_frac=0.10, null_empty=False) -> Table:
    cols = [i64_column(f"i{c}", n, seed + 100 + c, INT_DISTINCT[c], 0, null_frac, row0) for c in range(4)]
    cols += [utf8_column(f"s{c}", n, seed + 200 + c, STR_DISTINCT[c], 8, 24, null_frac, row0, null_empty=null_empty)
             for c in range(4)]
    return Table(cols)


def c4_table(n, row0=0, seed=42, null_frac=0.10) -> Table:
    cols = []
    for c in range(8):
        a, b = 0.3 + 0.1 * c, 1.0 - 0.05 * c
        cols.append(corr_column(f"x{c}", n, seed, seed + 300 + c, a, b, 1000.0 * c, null_frac, row0))
    return Table(cols)


def c5_table(n, row0=0, seed=42, null_frac=0.10, null_empty=False) -> Table:
    """16 mixed columns: C2's 8 fp64 + C3's 4 int64 + 4 UTF8 (null_empty: NULL string slots empty)."""
    return Table(list(c2_table(n, row0, seed, null_frac).columns.values()) +
                 list(c3_table(n, row0, seed, null_frac, null_empty).columns.values()))


def types_table(n, row0=0, seed=42, null_frac=0.10) -> Table:
    """The round-6 column types, one column each: FloatType ~ N(100, 30), ShortType / ByteType uniform, BooleanType
    (30 % true), DateType (days in [-50000, 50000)), TimestampType (micros in +-2^52), DecimalType(18, 2) and
    (38, 18); 10 % nulls (torch-generated on the device, seeded by row0 so chunks differ)."""
    import torch

    g = torch.Generator(device="cuda")
    g.manual_seed(seed * 1_000_003 + row0)
    cols = []

    def col(name, dtype, t, nbytes, k):
        v = _alloc(nbytes)
        v[:nbytes].copy_(t.contiguous().view(torch.uint8).reshape(-1)[:nbytes])
        bm = validity(n, seed + 7 * k, null_frac, row0)
        cols.append(Column(name, dtype, n, v, bm, None, nullable=bm is not None))

    col("f", "f32", torch.randn(n, device="cuda", generator=g) * 30.0 + 100.0, 4 * n, 1)
    col("h", "i16", torch.randint(-32768, 32768, (n,), device="cuda", generator=g, dtype=torch.int16), 2 * n, 2)
    col("c", "i8", torch.randint(-128, 128, (n,), device="cuda", generator=g, dtype=torch.int8), n, 3)
    bits = torch.rand(((n + 7) // 8) * 8, device="cuda", generator=g) < 0.3
    packed = (bits.view(-1, 8).to(torch.uint8) << torch.arange(8, device="cuda", dtype=torch.uint8)).sum(1, dtype=torch.uint8)
    col("b", "bool", packed, (n + 7) // 8, 4)
    col("d", "date32", torch.randint(-50000, 50000, (n,), device="cuda", generator=g, dtype=torch.int32), 4 * n, 5)
    col("t", "timestamp", torch.randint(-(1 << 52), 1 << 52, (n,), device="cuda", generator=g, dtype=torch.int64),
        8 * n, 6)
    # DecimalType: (18, 2) money amounts (|unscaled| < 10^12, high word the sign extension) and (38, 18) values of
    # up to 2^79 unscaled (~ +-6e5): 16-byte two's-complement (low word uniform, high word in [-2^15, 2^15))
    lo = torch.randint(-(10 ** 12), 10 ** 12, (n,), device="cuda", generator=g, dtype=torch.int64)
    col("m", "decimal(18,2)", torch.stack([lo, lo >> 63], 1), 16 * n, 7)
    lo = torch.randint(-(1 << 63), (1 << 63) - 1, (n,), device="cuda", generator=g, dtype=torch.int64)
    hi = torch.randint(-(1 << 15), 1 << 15, (n,), device="cuda", generator=g, dtype=torch.int64)
    col("q", "decimal(38,18)", torch.stack([lo, hi], 1), 16 * n, 8)
    return Table(cols)


def profile_analyzers(table: Table):
    """ColumnProfiler passes 1-2 minus DataType / ApproxQuantiles (profiles/ColumnProfiler.scala:200-235)."""
    from .analyzers import (ApproxCountDistinct, Completeness, Maximum, Mean, Minimum, Size, StandardDeviation,
                            Sum)

    out = [Size()]
    for name, dtype, _ in table.schema:
        out += [Completeness(name), ApproxCountDistinct(name)]
        if is_numeric(dtype):
            out += [Minimum(name), Maximum(name), Mean(name), StandardDeviation(name), Sum(name)]
    return out


def c3_analyzers(table: Table):
    """BASELINE config C3: Size + ApproxCountDistinct of every column + four Compliance predicates on i0..i3."""
    from .analyzers import ApproxCountDistinct, Compliance, Size

    out = [Size()] + [ApproxCountDistinct(c) for c in table.columns]
    out += [Compliance("p0", "i0 >= 0"), Compliance("p1", "`i1` IS NULL OR (`i1` >= 10.0 AND `i1` <= 1000.0)"),
            Compliance("p2", "i2 < i3"), Compliance("p3", "COALESCE(i3, 0.0) >= 0")]
    return out


def _device_i64_column(name, values, nullable=False) -> Column:
    """An int64 device column from a torch int64 tensor (padded as dqscan.h requires, no nulls)."""
    n = values.numel()
    buf = _alloc(n * 8)
    buf[: n * 8].copy_(values.view(__import__("torch").uint8))
    return Column(name, "i64", n, buf, None, None, nullable=nullable)


def _enum_utf8_column(name, n, seed, words, null_frac, row0=0) -> Column:
    """UTF8 column whose values are words[k] with k uniform (a counter hash of the row), on the device."""
    import torch

    k = torch.empty(n, dtype=torch.int64, device="cuda")
    _check(lib().dqs_i64(k.data_ptr(), row0, n, seed, len(words), 0, _stream()))
    wl = torch.tensor([len(w) for w in words], dtype=torch.int64, device="cuda")
    lens = wl[k]
    offs = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    torch.cumsum(lens, 0, out=offs[1:])
    total = int(offs[-1].item())
    width = max(len(w) for w in words)
    table = torch.zeros((len(words), width), dtype=torch.uint8)
    for i, w in enumerate(words):
        table[i, : len(w)] = torch.tensor(list(w), dtype=torch.uint8)
    table = table.cuda()
    row = torch.repeat_interleave(torch.arange(n, device="cuda"), lens)
    pos = torch.arange(total, device="cuda") - offs[row]
    data = _alloc(total)
    data[:total] = table[k[row], pos]
    o = _alloc((n + 1) * 4)
    _check(lib().dqs_i64_to_i32(o.data_ptr(), offs.data_ptr(), n + 1, _stream()))
    bm = validity(n, seed ^ 0xABCDEF, null_frac, row0)
    return Column(name, "utf8", n, data, bm, o, nullable=bm is not None, data_bytes=total)


def item_table(n, row0=0, seed=42) -> Table:
    """Config C1: the Item entity of examples/entities.scala:19-25 (id: Long, name, description, priority:
    String, numViews: Long).  id = row index and numViews uniform over [0, 10000] are non-nullable Scala
    Longs; name / description / priority have 10 % / 30 % / 10 % NULLs, priority in {high, low}
    (SURVEY §8d C1)."""
    import torch

    assert row0 % 32 == 0
    ids = torch.arange(row0, row0 + n, dtype=torch.int64, device="cuda")
    id_col = _device_i64_column("id", ids)
    views = i64_column("numViews", n, seed + 401, 10001, 0, 0.0, row0)
    views.nullable = False
    return Table([id_col,
                  utf8_column("name", n, seed + 402, 0, 8, 24, 0.10, row0),
                  utf8_column("description", n, seed + 403, 1_000_000, 16, 48, 0.30, row0),
                  _enum_utf8_column("priority", n, seed + 404, [b"high", b"low"], 0.10, row0),
                  views])


def item_checks():
    """The C1 verification: hasSize, isComplete x 5, hasMean / hasStandardDeviation / hasMin / hasMax on
    id and numViews, as one Check of the reference's DSL (checks/Check.scala)."""
    from .checks import Check, CheckLevel

    c = Check(CheckLevel.Error, "item table")
    c = c.hasSize(lambda n: n > 0)
    for col in ("id", "name", "description", "priority", "numViews"):
        c = c.isComplete(col)
    for col in ("id", "numViews"):
        c = (c.hasMean(col, lambda v: v >= 0).hasStandardDeviation(col, lambda v: v >= 0)
              .hasMin(col, lambda v: v >= 0).hasMax(col, lambda v: v >= 0))
    return c
