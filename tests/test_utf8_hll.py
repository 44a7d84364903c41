"""ApproxCountDistinct of string columns through the lock-step string hash (dq_kernels.hip utf8_range).

Lengths 0..40 around every round boundary of XXH64 (no / one / two / three stripe rounds, the 4-byte and
byte rounds, the deferred third round of 24..28-byte strings, > 28 bytes in the rare path: the 64-byte
register window up to 63 bytes, the byte-addressed loop beyond), NULL rows,
ragged sizes around the 64-row group and the 2048-row iteration, windows past the chunk's end, and 600 KB
strings whose 2048-row iteration spans more than a buffer resource.  Every case: the 52 HLL words bit-exact
against the oracle (XXH64 seed 42 over the UTF-8 bytes, StatefulHyperloglogPlus.scala:89-115), for int32
(UTF8) and int64 (LARGE_UTF8) offsets.  (Round 5 measured a compacted-stream variant of this pass against these
same cases; DESIGN.md section 7 records why it was not kept.)
"""
from __future__ import annotations

import numpy as np
import pytest

from oracle import dq_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dq():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    import deequ_amd

    return deequ_amd


def _words(dq, values, large):
    from deequ_amd.runner import scan_states
    from deequ_amd.table import utf8_column

    t = dq.Table([utf8_column("s", values, large=large)])
    a = dq.ApproxCountDistinct("s")
    return tuple(scan_states(t, [a])[a].words)


def _oracle(values):
    valid = np.array([v is not None for v in values], dtype=bool)
    return O.hll_words_for(O.OColumn("utf8", values, valid), valid)


def _strings(rng, n, lens, null_frac, distinct=None):
    out = []
    for i in range(n):
        if rng.random() < null_frac:
            out.append(None)
            continue
        ln = int(lens[i])
        if distinct is not None:  # a value drawn from `distinct` seeds (repeats: the HLL registers saturate less)
            r = np.random.default_rng(int(rng.integers(0, distinct)))
            out.append(r.integers(0, 256, ln, dtype=np.uint8).tobytes())
        else:
            out.append(rng.integers(0, 256, ln, dtype=np.uint8).tobytes())
    return out


@pytest.fixture(params=["fast", "long"])
def str_path(request, monkeypatch):
    """The string pass's two instantiations (DQ_STR_PATH; dq_scan otherwise picks one from the rare-path rows
    of the earlier chunks): the rare path redoing the whole block, or only its long rows from a register
    window."""
    monkeypatch.setenv("DQ_STR_PATH", request.param)
    return request.param


@pytest.mark.parametrize("large", [False, True])
@pytest.mark.parametrize("n", [1, 63, 64, 65, 2047, 2049, 70_001])
def test_every_length(dq, n, large, str_path):
    """Lengths 0..40 (none / one / two / three stripe rounds, the 4-byte and byte rounds, > 28 bytes) with
    12 % NULLs, ragged sizes around the 64-row group and the 2048-row iteration."""
    rng = np.random.default_rng(n + 7 * large)
    vals = _strings(rng, n, rng.integers(0, 41, n), 0.12)
    assert _words(dq, vals, large) == _oracle(vals)


@pytest.mark.parametrize("lo,hi", [(0, 7), (8, 15), (16, 23), (24, 28), (16, 28), (8, 24), (29, 40), (29, 63),
                                   (32, 48), (16, 48), (48, 63), (0, 140)])
@pytest.mark.parametrize("large", [False, True])
def test_one_length_band(dq, lo, hi, large, str_path):
    """One band of lengths per column: one stripe round, two, the deferred third, or none of them (> 28
    bytes: the rare path -- a 64-byte register window up to 63 bytes, one 32-byte stripe from 32 on, the
    byte-addressed loop beyond)."""
    rng = np.random.default_rng(lo * 100 + hi)
    n = 40_000
    vals = _strings(rng, n, rng.integers(lo, hi + 1, n), 0.05, distinct=30_000)
    assert _words(dq, vals, large) == _oracle(vals)


def test_variant_switch_across_chunks(dq, monkeypatch):
    """Automatic choice (DQ_STR_PATH unset): chunks of short strings, then long ones, then short ones again
    through one plan -- the string pass changes variant between chunks (from the rare-path rows the finalize
    publishes) and the registers stay bit-exact against the oracle over all chunks."""
    import torch

    from deequ_amd.runner import ScanPlan
    from deequ_amd.table import utf8_column

    monkeypatch.delenv("DQ_STR_PATH", raising=False)
    rng = np.random.default_rng(21)
    bands = [(8, 24), (30, 63), (30, 63), (30, 63), (0, 28), (8, 90), (8, 24)]
    chunks = [_strings(rng, 30_000, rng.integers(lo, hi + 1, 30_000), 0.08, distinct=50_000) for lo, hi in bands]
    a = dq.ApproxCountDistinct("s")
    t0 = dq.Table([utf8_column("s", chunks[0])])
    plan = ScanPlan([a], t0.schema)
    for rep in range(2):  # a second pass after reset starts from the published counts of the first
        plan.reset()
        for c in chunks:
            plan.scan(dq.Table([utf8_column("s", c)]))
            torch.cuda.synchronize()  # (the finalize has published the counts the next chunk's choice reads)
        got = tuple(a._from_result(plan.finish()[0]).words)
        allv = [v for c in chunks for v in c]
        assert got == _oracle(allv), rep
    plan.close()


def test_nulls_and_empty(dq, str_path):
    rng = np.random.default_rng(3)
    assert _words(dq, [None] * 5000, False) == _oracle([None] * 5000)
    vals = [b"" if i % 3 else None for i in range(10_000)]
    assert _words(dq, vals, False) == _oracle(vals)
    vals = _strings(rng, 30_000, rng.integers(0, 29, 30_000), 0.97)  # a few strings per group
    assert _words(dq, vals, True) == _oracle(vals)


@pytest.mark.parametrize("large", [False, True])
def test_strings_at_the_chunk_end(dq, large, str_path):
    """The last strings' 32-byte windows reach past the chunk's bytes: they take the general loop."""
    rng = np.random.default_rng(11)
    n = 4099
    vals = _strings(rng, n, rng.integers(0, 29, n), 0.1)
    vals[-40:] = [bytes([65 + k % 26]) * (k % 29) for k in range(40)]
    assert _words(dq, vals, large) == _oracle(vals)


@pytest.mark.parametrize("large", [False, True])
def test_huge_iteration_subranges(dq, large, str_path):
    """Every 8th row holds a 600 KB string: a 2048-row iteration spans ~150 MB of string bytes, so short
    strings far from their range's first byte take the general loop with the big ones."""
    import xxhash

    rng = np.random.default_rng(5)
    n = 4096
    big = rng.integers(0, 256, 600_000, dtype=np.uint8).tobytes()
    vals = []
    for i in range(n):
        if i % 8 == 0:
            vals.append(big[: 600_000 - i])  # distinct lengths: distinct values
        elif i % 13 == 0:
            vals.append(None)
        else:
            vals.append(rng.integers(0, 256, int(rng.integers(0, 29)), dtype=np.uint8).tobytes())
    got = _words(dq, vals, large)
    hashes = np.array([xxhash.xxh64_intdigest(v, seed=42) for v in vals if v is not None], dtype=np.uint64)
    want = tuple(O.registers_to_words(O.np_hll_registers(hashes).tolist()))
    assert got == want
