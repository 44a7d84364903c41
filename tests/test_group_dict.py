"""The dictionary form of GROUP BY (dq_group.hip dict_table): when an evenly spaced sample of the compacted keys
holds few distinct keys, every key is counted against them in one pass instead of being radix-sorted.  Its table
must equal the sort's -- the same group keys in the same (ascending) order, the same counts -- for strings, tuples
and wide numeric keys, over one chunk and several; a group the sample missed falls back to the sort; hash
collisions between distinct strings are still refused (the check runs in compaction order against each group's
sampled representative row).  DQ_GROUP_DICT=0 turns the form off, =1 lifts its size thresholds so that small
tables take it; the default takes it from 1 M keys whose sort would need more than 4 digit passes.
"""
from __future__ import annotations

import collections

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dq():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    import deequ_amd

    return deequ_amd


def _data(dq, n, distinct, seed, chunks=1, rare=0):
    """s: strings (t: the same, reversed per chunk, LARGE_UTF8), l: wide i64 keys (all 64 bits differ), f: f64 with NaN / -0.0 / 0.0, i: i32; NULLs in s and f.
    `rare` extra string and i64 values occur once each (groups an evenly spaced sample likely misses)."""
    from deequ_amd.table import Table, column_from_numpy, utf8_column

    rng = np.random.default_rng(seed)
    pick = rng.integers(0, distinct, n)
    spool = [f"key-{i:06d}-{'y' * (i % 29)}".encode() for i in range(distinct)]
    lpool = rng.integers(-(1 << 63), (1 << 63) - 1, distinct, dtype=np.int64)
    fpool = np.concatenate([[np.nan, -0.0, 0.0], rng.normal(size=max(1, distinct - 3)) * 1e6])[:distinct]
    s = [spool[j] for j in pick]
    lv = lpool[pick].copy()
    for r, at in enumerate(rng.choice(n, size=rare, replace=False)):
        s[at] = f"rare-{r}".encode()
        lv[at] = (1 << 62) + r
    s = [None if rng.random() < 0.1 else v for v in s]
    fv = fpool[pick]
    fok = rng.random(n) >= 0.1
    iv = (pick % 7).astype(np.int32)
    step = (n + chunks - 1) // chunks
    out = []
    for lo in range(0, n, step):
        hi = min(n, lo + step)
        out.append(Table([utf8_column("s", s[lo:hi]), utf8_column("t", s[lo:hi][::-1], large=True),
                          column_from_numpy("l", "i64", lv[lo:hi], np.ones(hi - lo, bool)),
                          column_from_numpy("f", "f64", fv[lo:hi], fok[lo:hi]),
                          column_from_numpy("i", "i32", iv[lo:hi], np.ones(hi - lo, bool))]))
    return out[0] if chunks == 1 else out, s, lv


def _table_of(data, cols):
    from deequ_amd.grouping import build_frequencies

    fr = build_frequencies(data, cols)
    keys, counts = fr.frequencies.export()
    return fr, np.asarray(keys).copy(), np.asarray(counts).copy()


def _both(monkeypatch, data, cols, mode="1"):
    monkeypatch.setenv("DQ_GROUP_DICT", "0")
    ref = _table_of(data, cols)
    monkeypatch.setenv("DQ_GROUP_DICT", mode)
    got = _table_of(data, cols)
    return ref, got


COLS = [["s"], ["t"], ["l"], ["f"], ["s", "i"], ["l", "f", "s"]]


@pytest.mark.parametrize("n,distinct,chunks", [(1, 1, 1), (3000, 7, 1), (20_000, 300, 3), (50_000, 2000, 2)])
def test_dictionary_equals_sort(dq, monkeypatch, n, distinct, chunks):
    data, s, lv = _data(dq, n, distinct, n + distinct, chunks)
    for cols in COLS:
        (fr0, k0, c0), (fr1, k1, c1) = _both(monkeypatch, data, cols)
        assert np.array_equal(k0, k1) and np.array_equal(c0, c1), cols
        assert fr0 == fr1, cols
        s0, s1 = fr0.frequencies.summary(fr0.numRows), fr1.frequencies.summary(fr1.numRows)
        assert (s0.num_groups, s0.num_unique, s0.num_values, s0.entropy) == (s1.num_groups, s1.num_unique,
                                                                              s1.num_values, s1.entropy), cols
    # counts against a host count of the same values
    _, _, c1 = _table_of(data, ["s"])
    assert sorted(c1.tolist()) == sorted(collections.Counter(v for v in s if v is not None).values())
    _, _, c1 = _table_of(data, ["l"])
    assert sorted(c1.tolist()) == sorted(collections.Counter(lv.tolist()).values())


def test_dictionary_sample_misses_groups(dq, monkeypatch):
    """40 values seen once among 60 000 rows of 50 frequent ones: the evenly spaced sample misses some of them
    (the dictionary pass sees a key outside it and the table is sorted instead) -- same table either way."""
    data, s, lv = _data(dq, 60_000, 50, 3, chunks=2, rare=40)
    for cols in (["s"], ["l"], ["s", "i"]):
        (fr0, k0, c0), (fr1, k1, c1) = _both(monkeypatch, data, cols)
        assert np.array_equal(k0, k1) and np.array_equal(c0, c1), cols
    _, _, c = _table_of(data, ["l"])
    assert sorted(c.tolist()) == sorted(collections.Counter(lv.tolist()).values())


@pytest.mark.parametrize("chunks", [1, 3])
@pytest.mark.parametrize("col", ["s", "t"])
def test_dictionary_refuses_collisions(dq, monkeypatch, chunks, col):
    from deequ_amd import _lib as L
    from deequ_amd.grouping import build_frequencies

    data, _, _ = _data(dq, 6000, 100, 11, chunks)
    monkeypatch.setenv("DQ_GROUP_DICT", "1")
    monkeypatch.setenv("DQ_TEST_GROUP_HASH_MASK", "f")  # 16 possible keys for 100 distinct strings
    with pytest.raises(L.DQError) as e:
        build_frequencies(data, [col])
    assert "collision" in str(e.value)


def test_string_check_same_length_strings(dq, monkeypatch):
    """Equal-length strings that differ in one byte at every position (first 8 bytes, the 8-byte steps, the
    4-byte step, the last bytes), colliding under the mask: refused; without the mask, exact counts."""
    from deequ_amd import _lib as L
    from deequ_amd.grouping import build_frequencies
    from deequ_amd.table import Table, utf8_column

    base = "abcdefghijklmnopqrstuvwxyz0123456789!"
    rng = np.random.default_rng(2)
    for cut in (3, 7, 9, 17, 29, 33, 37):
        b = base[:cut]
        pool = [b] + [b[:i] + "#" + b[i + 1:] for i in range(cut)]
        vals = [pool[i].encode() for i in rng.integers(0, len(pool), size=8000)]
        data = Table([utf8_column("s", vals)])
        monkeypatch.setenv("DQ_GROUP_DICT", "1")
        _, _, c = _table_of(data, ["s"])
        assert sorted(c.tolist()) == sorted(collections.Counter(vals).values()), cut
        monkeypatch.setenv("DQ_TEST_GROUP_HASH_MASK", "0")  # every string in one hash group
        with pytest.raises(L.DQError) as e:
            build_frequencies(data, ["s"])
        assert "collision" in str(e.value), cut
        monkeypatch.delenv("DQ_TEST_GROUP_HASH_MASK")


def test_dictionary_default_thresholds(dq, monkeypatch):
    """2 M rows of 1000 values: the default takes the dictionary form for strings and wide i64 keys (and
    keeps the sort for the i32 column's 3 bits); the tables equal the sort's."""
    data, _, _ = _data(dq, 2_000_000, 1000, 17, chunks=2)
    for cols in (["s"], ["l"], ["i"], ["f", "i"]):
        monkeypatch.delenv("DQ_GROUP_DICT", raising=False)
        (fr0, k0, c0), (fr1, k1, c1) = _both(monkeypatch, data, cols, mode="auto")
        assert np.array_equal(k0, k1) and np.array_equal(c0, c1), cols


def test_dictionary_histogram(dq, monkeypatch):
    """Histogram renders each bin's value from the group's representative row: the sampled row in the
    dictionary form, a sorted run's first row otherwise -- the same bins."""
    data, _, _ = _data(dq, 30_000, 40, 23)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("DQ_GROUP_DICT", mode)
        h = dq.Histogram("s").calculate(data).value.get()
        out[mode] = {k: v.absolute for k, v in h.values.items()}
    assert out["0"] == out["1"] and len(out["1"]) == 41  # 40 values + NullValue
