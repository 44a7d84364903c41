"""Arrow C Data Interface ingestion (deequ_amd/csrc/dq_ingest.cpp, deequ_amd/ingest.py).

CPU: dq_arrow_import maps pyarrow-exported arrays (zero-copy) to the host buffers dq_upload copies, and
rejects what a dq column cannot represent.  GPU: host-resident Arrow batches scanned through the pinned
double-buffered upload give bit-identical states to the same data scanned from device tables.
"""
from __future__ import annotations

import numpy as np
import pytest

pa = pytest.importorskip("pyarrow")


def _batch(n, seed):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=n) * 10 + 3
    xv = rng.random(n) > 0.1
    l = rng.integers(-(1 << 40), 1 << 40, n)
    lv = rng.random(n) > 0.2
    i = rng.integers(-50000, 50000, n).astype(np.int32)
    words = np.array([f"val{k:05d}-{'x' * (k % 17)}" for k in range(997)])
    s = words[rng.integers(0, len(words), n)]
    sv = rng.random(n) > 0.15
    return pa.record_batch([pa.array(x, mask=~xv), pa.array(l, mask=~lv), pa.array(i), pa.array(s, mask=~sv)],
                           names=["x", "l", "i", "s"]), (x, xv, l, lv, i, s, sv)


def test_arrow_import_maps_buffers():
    from deequ_amd import _lib as L
    from deequ_amd.ingest import ImportedArray

    b, _ = _batch(1000, 1)
    for name, t in (("x", L.TYPE_F64), ("l", L.TYPE_I64), ("i", L.TYPE_I32), ("s", L.TYPE_UTF8)):
        arr = b.column(b.schema.get_field_index(name))
        im = ImportedArray(arr)
        h = im.host
        bufs = arr.buffers()
        assert h.type == t and h.n_rows == 1000
        if name == "i":  # no nulls: no bitmap
            assert h.nullable == 0 and not h.validity
        else:
            assert h.nullable == 1 and h.validity == bufs[0].address and h.validity_bytes == 125
        if name == "s":
            assert h.offsets == bufs[1].address and h.offset_bytes == 4004 and h.values == bufs[2].address
            assert h.value_bytes == int(np.frombuffer(bufs[1], dtype=np.int32)[1000])
        else:
            assert h.values == bufs[1].address and h.value_bytes == 1000 * (4 if name == "i" else 8)
        im.close()
    # a slice at a byte boundary is a pointer offset; elsewhere dq_upload shifts the bitmap into place
    im = ImportedArray(b.column(0).slice(16, 100))
    assert im.host.validity == b.column(0).buffers()[0].address + 2 and im.host.n_rows == 100
    assert im.host.validity_bit == 0
    im.close()
    im = ImportedArray(b.column(0).slice(3, 100))
    assert im.host.validity == b.column(0).buffers()[0].address and im.host.validity_bit == 3
    assert im.host.values == b.column(0).buffers()[1].address + 3 * 8
    im.close()
    # a string slice: data from its first string, offsets rebased by o0
    s = b.column(3)
    o = np.frombuffer(s.buffers()[1], dtype=np.int32)
    im = ImportedArray(s.slice(21, 100))
    assert im.host.offset_base == o[21] and im.host.values == s.buffers()[2].address + int(o[21])
    assert im.host.value_bytes == int(o[121] - o[21]) and im.host.validity_bit == 5
    im.close()
    # an empty array maps to an empty column without touching its (possibly NULL) buffers
    im = ImportedArray(pa.array([], type=pa.string()))
    assert im.host.n_rows == 0 and im.host.value_bytes == 0 and not im.host.values
    im.close()
    with pytest.raises(L.DQError):
        ImportedArray(pa.array([1, 2], type=pa.uint32()))
    with pytest.raises(L.DQError):
        ImportedArray(pa.array([1, 2], type=pa.timestamp("ms")))  # not TimestampType's unit
    with pytest.raises(L.DQError):
        ImportedArray(pa.array(["a", "b"]).dictionary_encode())


def _typed_batch(n, seed):
    """One column of each round-6 type (FloatType, ShortType, ByteType, BooleanType, DateType, TimestampType)."""
    rng = np.random.default_rng(seed)
    f = (rng.normal(size=n) * 100).astype(np.float32)
    h = rng.integers(-30000, 30000, n).astype(np.int16)
    c = rng.integers(-128, 128, n).astype(np.int8)
    b = rng.random(n) > 0.4
    d = rng.integers(-20000, 30000, n).astype(np.int32)
    ts = rng.integers(-(1 << 50), 1 << 50, n)
    masks = [rng.random(n) > q for q in (0.1, 0.2, 0.0, 0.15, 0.3, 0.05)]
    arrs = [pa.array(f, mask=~masks[0]), pa.array(h, mask=~masks[1]), pa.array(c),
            pa.array(b, mask=~masks[3]), pa.array(d, type=pa.int32(), mask=~masks[4]).cast(pa.date32()),
            pa.array(ts, mask=~masks[5]).cast(pa.timestamp("us", tz="UTC"))]
    return pa.record_batch(arrs, names=["f", "h", "c", "b", "d", "t"]), (f, h, c, b, d, ts), masks


def test_arrow_import_round6_types():
    """dq_arrow_import maps float32 / int16 / int8 / bool / date32 / timestamp[us, tz] arrays; a boolean slice's
    value bits carry the slice's bit offset like its validity."""
    from deequ_amd import _lib as L
    from deequ_amd.ingest import ImportedArray, arrow_schema

    bt, _, _ = _typed_batch(1000, 3)
    assert [d for _, d, _ in arrow_schema(bt)] == ["f32", "i16", "i8", "bool", "date32", "timestamp"]
    want = {"f": (L.TYPE_F32, 4), "h": (L.TYPE_I16, 2), "c": (L.TYPE_I8, 1), "d": (L.TYPE_DATE32, 4),
            "t": (L.TYPE_TIMESTAMP, 8)}
    for name, (t, w) in want.items():
        arr = bt.column(bt.schema.get_field_index(name))
        im = ImportedArray(arr)
        assert im.host.type == t and im.host.values == arr.buffers()[1].address and im.host.value_bytes == 1000 * w
        im.close()
    arr = bt.column(3)
    im = ImportedArray(arr)
    assert im.host.type == L.TYPE_BOOL and im.host.values == arr.buffers()[1].address and im.host.value_bytes == 125
    im.close()
    im = ImportedArray(arr.slice(11, 300))
    assert im.host.values == arr.buffers()[1].address + 1 and im.host.validity_bit == 3 and im.host.value_bytes == 38
    im.close()


@pytest.mark.gpu
def test_arrow_ingest_vs_oracle_and_device_scan():
    """Host Arrow batches -- raw RecordBatch.slice chunks at odd row offsets (bitmap shifted, string
    offsets rebased by dq_upload) -- scanned through the pinned upload: every state equals the C / numpy
    oracle over the whole data (counts, min / max, HLL words, compliance bit-exact; fp64 within 1e-12)
    and the same data scanned from device tables."""
    import torch

    import deequ_amd as dq
    from deequ_amd.ingest import scan_arrow
    from deequ_amd.runner import scan_results
    from deequ_amd.states import state_from_c
    from deequ_amd.table import column_from_numpy, utf8_column
    from oracle import dq_oracle as O
    from oracle import dq_oracle_c as C
    from tests.helpers import close

    assert torch.cuda.is_available()
    n, parts = 300_000, [0, 100_003, 200_010, 300_000]
    b, (x, xv, l, lv, i, s, sv) = _batch(n, 7)
    an = [dq.Size(), dq.Completeness("x"), dq.Mean("x"), dq.StandardDeviation("x"), dq.Minimum("l"), dq.Maximum("l"),
          dq.Sum("i"), dq.ApproxCountDistinct("s"), dq.ApproxCountDistinct("l"), dq.Correlation("x", "i"),
          dq.Compliance("c", "x > 3 AND l IS NOT NULL"), dq.Completeness("s"), dq.Mean("i", "x > 0")]
    batches = [b.slice(parts[k], parts[k + 1] - parts[k]) for k in range(3)]
    got = scan_arrow(batches, an)
    # the oracle over the whole data (Spark partitions = the three chunks)
    bx, bl = np.packbits(xv, bitorder="little"), np.packbits(lv, bitorder="little")
    bs = np.packbits(sv, bitorder="little")
    enc = [v.encode() for v in s]
    offs = np.zeros(n + 1, dtype=np.int64)
    np.cumsum([len(e) for e in enc], out=offs[1:])
    data = np.frombuffer(b"".join(enc) + b"\0" * 8, dtype=np.uint8)
    st = {a: state_from_c(g) for a, g in zip(an, got)}
    assert st[an[0]].numMatches == n
    assert (st[an[1]].numMatches, st[an[1]].count) == (int(xv.sum()), n)
    assert (st[an[11]].numMatches, st[an[11]].count) == (int(sv.sum()), n)
    sx = C.column_stats("f64", x, bx, None, 3)
    assert st[an[2]].count == sx.count and close(st[an[2]].sum_, sx.sum_f64, 1e-12)
    assert st[an[3]].n == sx.n and close(st[an[3]].metricValue(), (sx.m2 / sx.n) ** 0.5, 1e-12)
    sl = C.column_stats("i64", l, bl, None, 3)
    assert st[an[4]].metricValue() == sl.min and st[an[5]].metricValue() == sl.max
    assert st[an[6]].metricValue() == float(int(i.astype(np.int64).sum()))
    regs = C.hll_registers("large_utf8", data, offs, bs, None, n)
    assert st[an[7]].words == tuple(O.registers_to_words(regs.tolist()))
    regs = C.hll_registers("i64", l, None, bl, None, n)
    assert st[an[8]].words == tuple(O.registers_to_words(regs.tolist()))
    r = C.corr("f64", x, bx, "i32", i, None, None, 3)
    assert st[an[9]].n == r[0] and close(st[an[9]].metricValue(), r[3] / (r[4] * r[5]) ** 0.5, 1e-12)
    t_, _ = O.NpPredicate("x > 3 AND l IS NOT NULL").eval_bool({"x": ("f64", x, xv), "l": ("i64", l, lv)}, n)
    assert (st[an[10]].numMatches, st[an[10]].count) == (int(t_.sum()), n)
    si = C.column_stats("i32", i, None, np.packbits(xv & (x > 0), bitorder="little"), 3)
    assert st[an[12]].count == si.count and st[an[12]].sum_ == si.sum_f64
    # and the same chunks from device tables
    tables = []
    for k in range(3):
        sl_ = slice(parts[k], parts[k + 1])
        strs = [v.encode() if ok else None for v, ok in zip(s[sl_], sv[sl_])]
        tables.append(dq.Table([column_from_numpy("x", "f64", x[sl_], xv[sl_]), column_from_numpy("l", "i64", l[sl_], lv[sl_]),
                                column_from_numpy("i", "i32", i[sl_], np.ones(len(i[sl_]), bool), nullable=False),
                                utf8_column("s", strs)]))
    want = scan_results(tables, an)
    for a, g, w in zip(an, got, want):
        assert bytes(g) == bytes(w), a


@pytest.mark.gpu
def test_arrow_ingest_round6_types_vs_device_scan():
    """Host Arrow batches of the round-6 types, sliced at odd row offsets (boolean value bits shifted like the
    validity by dq_upload), scanned through the pinned upload: the same states as the device tables, and the
    oracle's HLL words / counts."""
    import torch

    import deequ_amd as dq
    from deequ_amd.ingest import scan_arrow
    from deequ_amd.runner import scan_results
    from deequ_amd.states import state_from_c
    from deequ_amd.table import column_from_numpy
    from oracle import dq_oracle as O

    assert torch.cuda.is_available()
    n, parts = 200_000, [0, 70_001, 140_013, 200_000]
    bt, (f, h, c, b, d, ts), masks = _typed_batch(n, 9)
    an = [dq.Mean("f"), dq.StandardDeviation("h"), dq.Sum("c"), dq.Minimum("f"), dq.Maximum("h"),
          dq.ApproxCountDistinct("b"), dq.ApproxCountDistinct("d"), dq.ApproxCountDistinct("t"),
          dq.ApproxCountDistinct("f"), dq.Completeness("b"), dq.Compliance("bt", "b"), dq.Completeness("d"),
          dq.Correlation("f", "c"), dq.DataType("b"), dq.DataType("f")]
    batches = [bt.slice(parts[k], parts[k + 1] - parts[k]) for k in range(3)]
    got = scan_arrow(batches, an)
    tables = []
    for k in range(3):
        sl = slice(parts[k], parts[k + 1])
        cols = [column_from_numpy(name, dt, v[sl], m[sl]) for name, dt, v, m in
                zip("fhcbdt", ["f32", "i16", "i8", "bool", "date32", "timestamp"], (f, h, c, b, d, ts), masks)]
        cols[2] = column_from_numpy("c", "i8", c[sl], np.ones(parts[k + 1] - parts[k], bool), nullable=False)
        tables.append(dq.Table(cols))
    want = scan_results(tables, an)
    for a, g, w in zip(an, got, want):
        assert bytes(g) == bytes(w), a
    st = {a: state_from_c(g) for a, g in zip(an, got)}
    ocols = {"b": O.OColumn("bool", b, masks[3]), "d": O.OColumn("date32", d, masks[4]),
             "t": O.OColumn("timestamp", ts, masks[5]), "f": O.OColumn("f32", f, masks[0])}
    for a in (an[5], an[6], an[7], an[8]):
        assert st[a].words == O.compute_state(("ApproxCountDistinct", a.column, None), ocols, n).words, a
    assert (st[an[9]].numMatches, st[an[9]].count) == (int(masks[3].sum()), n)
    assert st[an[10]].numMatches == int((b & masks[3]).sum())


def _decimal_batch(n, seed):
    """DecimalType(38, 18) and (9, 2) columns as Arrow decimal128 (Spark's export of DecimalType)."""
    import decimal

    rng = np.random.default_rng(seed)
    u38 = [int(rng.integers(-(10 ** 18), 10 ** 18)) * 10 ** int(rng.integers(0, 15)) for _ in range(n)]
    u9 = [int(rng.integers(-(10 ** 9) + 1, 10 ** 9)) for _ in range(n)]
    m38, m9 = rng.random(n) > 0.1, rng.random(n) > 0.2
    a38 = pa.array([decimal.Decimal(u).scaleb(-18) if ok else None for u, ok in zip(u38, m38)], type=pa.decimal128(38, 18))
    a9 = pa.array([decimal.Decimal(u).scaleb(-2) if ok else None for u, ok in zip(u9, m9)], type=pa.decimal128(9, 2))
    return pa.record_batch([a38, a9], names=["d38", "d9"]), (u38, u9), (m38, m9)


def test_arrow_import_decimal128():
    """dq_arrow_import maps decimal128(p, s) arrays (format "d:p,s") to DECIMAL128 columns of 16-byte values; a
    decimal256 or a negative scale stays on the fallback."""
    from deequ_amd import _lib as L
    from deequ_amd.ingest import ImportedArray, arrow_schema

    bt, _, _ = _decimal_batch(1000, 5)
    assert [d for _, d, _ in arrow_schema(bt)] == ["decimal(38,18)", "decimal(9,2)"]
    for k, (p, s) in enumerate(((38, 18), (9, 2))):
        arr = bt.column(k)
        im = ImportedArray(arr)
        assert im.host.type == L.decimal_type(p, s) and im.host.values == arr.buffers()[1].address
        assert im.host.value_bytes == 16 * 1000
        im.close()
        im = ImportedArray(arr.slice(7, 100))
        assert im.host.values == arr.buffers()[1].address + 16 * 7 and im.host.validity_bit == 7
        im.close()
    with pytest.raises(L.DQError):
        ImportedArray(pa.array([1, 2], type=pa.decimal256(40, 2)))


@pytest.mark.gpu
def test_arrow_ingest_decimal_vs_device_scan():
    """Arrow decimal128 batches sliced at odd row offsets through the pinned upload: the same states as the device
    tables, and the oracle's (exact sums cast to double, Decimal.toDouble min / max, Spark's decimal hash)."""
    import torch

    import deequ_amd as dq
    from deequ_amd.ingest import scan_arrow
    from deequ_amd.runner import scan_results
    from deequ_amd.states import state_from_c
    from deequ_amd.table import column_from_numpy
    from oracle import dq_oracle as O

    assert torch.cuda.is_available()
    n, parts = 50_000, [0, 17_001, 33_333, 50_000]
    bt, (u38, u9), (m38, m9) = _decimal_batch(n, 11)
    an = [dq.Sum("d38"), dq.Minimum("d38"), dq.Maximum("d9"), dq.Mean("d9"), dq.StandardDeviation("d38"),
          dq.ApproxCountDistinct("d38"), dq.ApproxCountDistinct("d9"), dq.DataType("d38"), dq.Completeness("d9"),
          dq.Compliance("pos", "d38 > 0 AND d9 <= 100.5")]
    batches = [bt.slice(parts[k], parts[k + 1] - parts[k]) for k in range(3)]
    got = scan_arrow(batches, an)
    tables = []
    for k in range(3):
        sl = slice(parts[k], parts[k + 1])
        tables.append(dq.Table([column_from_numpy("d38", "decimal(38,18)", u38[sl], m38[sl]),
                                column_from_numpy("d9", "decimal(9,2)", u9[sl], m9[sl])]))
    want = scan_results(tables, an)
    for a, g, w in zip(an, got, want):
        assert bytes(g) == bytes(w), a
    ocols = {"d38": O.OColumn("decimal(38,18)", u38, m38), "d9": O.OColumn("decimal(9,2)", u9, m9)}
    st = {a: state_from_c(g) for a, g in zip(an, got)}
    for a in an[:4] + an[5:7]:
        ref = O.compute_state((type(a).__name__, a.column, None), ocols, n)
        assert ref is not None and st[a].metricValue() == ref.metricValue(), a
