"""The exact check behind hashed GROUP BY (dq_group.hip): every group's rows must hold equal tuples, whatever the
64-bit tuple hash says.  Two forms: tables of few groups are checked in compaction order against each group's
representative row (verify_compacted: the group found by binary search of the row's key), others by equal-hash
neighbours in sorted order (verify_runs).
DQ_TEST_GROUP_HASH_MASK keeps only some bits of the hash, so distinct strings collide; both forms must refuse the
table (DQ_E_UNSUPPORTED, "collision"), over one chunk and several, and with the full hash the same tables group
exactly as the oracle counts them.
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


def _table(dq, values, chunks=1):
    from deequ_amd.table import Table, utf8_column

    values = [None if v is None else v.encode() for v in values]
    if chunks == 1:
        return Table([utf8_column("s", values)])
    step = (len(values) + chunks - 1) // chunks
    return [Table([utf8_column("s", values[i:i + step])]) for i in range(0, len(values), step)]


def _values(n_rows, n_distinct, seed):
    rng = np.random.default_rng(seed)
    pool = [f"value-{i:05d}-{'x' * (i % 23)}" for i in range(n_distinct)]
    vals = [pool[i] for i in rng.integers(0, n_distinct, size=n_rows)]
    for i in rng.choice(n_rows, size=n_rows // 10, replace=False):
        vals[i] = None
    return vals


@pytest.mark.parametrize("n_rows,n_distinct", [(5000, 100),    # <= 16 keys under the mask, 4500 rows: compaction order
                                               (100, 100)])    # 16 keys for ~90 rows: sorted neighbours
@pytest.mark.parametrize("chunks", [1, 3])
def test_collisions_refused(dq, monkeypatch, n_rows, n_distinct, chunks):
    from deequ_amd import _lib as L
    from deequ_amd.grouping import build_frequencies

    vals = _values(n_rows, n_distinct, n_rows + chunks)
    t = _table(dq, vals, chunks)
    monkeypatch.setenv("DQ_TEST_GROUP_HASH_MASK", "f")  # 16 possible keys for 100 distinct strings
    with pytest.raises(L.DQError) as e:
        build_frequencies(t, ["s"])
    assert "collision" in str(e.value)
    monkeypatch.delenv("DQ_TEST_GROUP_HASH_MASK")
    fr = build_frequencies(t, ["s"])
    _, counts = fr.frequencies.export()
    want = collections.Counter(v for v in vals if v is not None)
    assert sorted(counts.tolist()) == sorted(want.values())


def test_compaction_order_form_exact(dq):
    """Few groups (compaction-order form) with equal-length strings differing in one byte at every position."""
    from deequ_amd.grouping import build_frequencies

    base = "abcdefghijklmnopqrstuvwxyz0123456789"
    pool = [base] + [base[:i] + "#" + base[i + 1:] for i in range(len(base))]
    rng = np.random.default_rng(5)
    vals = [pool[i] for i in rng.integers(0, len(pool), size=20_000)]
    fr = build_frequencies(_table(dq, vals), ["s"])
    _, counts = fr.frequencies.export()
    assert sorted(counts.tolist()) == sorted(collections.Counter(vals).values())
