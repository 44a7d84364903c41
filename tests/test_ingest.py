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
        ImportedArray(pa.array([1.5, 2.5], type=pa.float32()))
    with pytest.raises(L.DQError):
        ImportedArray(pa.array(["a", "b"]).dictionary_encode())


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
