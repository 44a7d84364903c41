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
    # a slice at a byte boundary is a pointer offset; elsewhere (with nulls) it must be re-sliced
    im = ImportedArray(b.column(0).slice(16, 100))
    assert im.host.validity == b.column(0).buffers()[0].address + 2 and im.host.n_rows == 100
    im.close()
    with pytest.raises(L.DQError):
        ImportedArray(b.column(0).slice(3, 100))
    with pytest.raises(L.DQError):  # string slice: offsets do not start at 0
        ImportedArray(b.column(3).slice(16, 100))
    with pytest.raises(L.DQError):
        ImportedArray(pa.array([1.5, 2.5], type=pa.float32()))
    with pytest.raises(L.DQError):
        ImportedArray(pa.array(["a", "b"]).dictionary_encode())


@pytest.mark.gpu
def test_arrow_ingest_equals_device_scan():
    import torch

    import deequ_amd as dq
    from deequ_amd.ingest import scan_arrow
    from deequ_amd.runner import scan_results
    from deequ_amd.table import column_from_numpy, utf8_column

    assert torch.cuda.is_available()
    n, parts = 300_000, [0, 100_000, 200_008, 300_000]
    b, (x, xv, l, lv, i, s, sv) = _batch(n, 7)
    an = [dq.Size(), dq.Completeness("x"), dq.Mean("x"), dq.StandardDeviation("x"), dq.Minimum("l"), dq.Maximum("l"),
          dq.Sum("i"), dq.ApproxCountDistinct("s"), dq.ApproxCountDistinct("l"), dq.Correlation("x", "i"),
          dq.Compliance("c", "x > 3 AND l IS NOT NULL"), dq.Completeness("s"), dq.Mean("i", "x > 0")]
    batches = [b.slice(parts[k], parts[k + 1] - parts[k]) for k in range(3)]
    # string slices must start their offsets at 0: rebuild those columns per chunk (as a batch producer would)
    batches = [pa.record_batch([c if c.type != pa.string() else pa.array(c.to_pylist()) for c in bt.columns],
                               names=bt.schema.names) for bt in batches]
    got = scan_arrow(batches, an)
    tables = []
    for k in range(3):
        sl = slice(parts[k], parts[k + 1])
        strs = [v.encode() if ok else None for v, ok in zip(s[sl], sv[sl])]
        tables.append(dq.Table([column_from_numpy("x", "f64", x[sl], xv[sl]), column_from_numpy("l", "i64", l[sl], lv[sl]),
                                column_from_numpy("i", "i32", i[sl], np.ones(len(i[sl]), bool), nullable=False),
                                utf8_column("s", strs)]))
    want = scan_results(tables, an)
    for a, g, w in zip(an, got, want):
        assert bytes(g) == bytes(w), a
