"""HLL registers of values whose XXH64 needs the exact-rank redo (StatefulHyperloglogPlus.scala:96-113).

The kernels take an HLL register's rank from the high word of the hash; when its bits 54..32 are all
zero (p = 2^-23 for random data) the rank needs the low word and the value is redone exactly
(dq_kernels.hip: the block redo of the numeric passes, the deferred-string drain, the general string
loop).  Random data reaches those paths about twice in the whole GPU suite, so these tests scan tables
built from constructed values (tests/golden/hll_redo_values.json, made by make_hll_redo_values.py) and
compare the registers bit-exactly with the C oracle.
"""
from __future__ import annotations

import json
import os
import struct

import numpy as np
import pytest

from oracle import dq_oracle as O
from oracle import dq_oracle_c as C

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def redo_values():
    with open(os.path.join(HERE, "golden", "hll_redo_values.json")) as f:
        d = json.load(f)
    f64 = np.array([int(b, 16) for b in d["f64_bits"]], dtype=np.uint64).view(np.float64)
    return np.array(d["i64"], dtype=np.int64), f64, [s.encode("ascii") for s in d["utf8"]]


def _rank_needs_low_word(h: int) -> bool:
    return (h >> 32) & 0x7FFFFF == 0


def test_fixture_values_take_the_redo_path(redo_values):
    """CPU: every fixture value's hash (oracle XXH64) has bits 54..32 zero, and the oracle's register
    for it is the exact rank computed from the full 64-bit hash (pw >= 24)."""
    i64, f64, strs = redo_values
    for v in i64:
        assert _rank_needs_low_word(C.lib().dqo_xxh64_long(int(v), 42))
    for x in f64:
        assert _rank_needs_low_word(C.lib().dqo_xxh64_long(struct.unpack("<q", struct.pack("<d", x))[0], 42))
    for s in strs:
        h = C.lib().dqo_xxh64_bytes(s, len(s), 42)
        assert _rank_needs_low_word(h) and O.xxh64_bytes(s) & ((1 << 64) - 1) == h
        idx, pw = O.hll_index_and_pw(h)
        assert pw >= 24


def _table(dq, redo_values, n, p_redo, seed):
    from deequ_amd.table import column_from_numpy, utf8_column

    i64r, f64r, strr = redo_values
    rng = np.random.default_rng(seed)
    valid = rng.random(n) >= 0.1
    pick = rng.random(n) < p_redo
    i64 = np.where(pick, i64r[rng.integers(0, len(i64r), n)], rng.integers(-(1 << 40), 1 << 40, n))
    f64 = np.where(pick, f64r[rng.integers(0, len(f64r), n)], rng.normal(5.0, 3.0, n))
    # the same with a few NaN / +-inf rows: the fp64 pass's rare non-finite block path
    fnf = f64.copy()
    special = rng.random(n) < 0.01
    fnf[special] = rng.choice(np.array([np.nan, np.inf, -np.inf]), int(special.sum()))
    strs = []
    for i in range(n):
        if not valid[i]:
            strs.append(None)
        elif pick[i]:
            strs.append(strr[int(rng.integers(0, len(strr)))])
        else:
            strs.append(bytes(rng.integers(65, 91, int(rng.integers(0, 40)), dtype=np.uint8)))
    a = rng.integers(-5, 5, n).astype(np.int64)
    t = dq.Table([column_from_numpy("l", "i64", i64, valid), column_from_numpy("f", "f64", f64, valid),
                  column_from_numpy("fn", "f64", fnf, valid), utf8_column("s", strs),
                  utf8_column("ls", strs, large=True), column_from_numpy("a", "i64", a, np.ones(n, bool))])
    return t, {"l": i64, "f": f64, "fn": fnf, "s": strs, "ls": strs, "a": a}, valid


@pytest.mark.gpu
@pytest.mark.parametrize("n,p_redo", [(64, 1.0), (4099, 1.0), (65_537, 1.0), (100_003, 0.05)])
def test_hll_exact_rank_redo_values(n, p_redo, redo_values):
    import deequ_amd as dq
    from deequ_amd.runner import scan_states

    t, host, valid = _table(dq, redo_values, n, p_redo, seed=n)
    cols = ["l", "f", "fn", "s", "ls"]
    # HLL-only variants, stats+HLL variants (Mean / StdDev share the pass), and a `where` filter
    plans = [[dq.ApproxCountDistinct(c) for c in cols],
             [a for c in cols for a in ([dq.ApproxCountDistinct(c)] +
                                        ([dq.StandardDeviation(c), dq.Minimum(c)] if c in ("l", "f", "fn") else []))],
             [dq.ApproxCountDistinct(c, "a > 0") for c in cols]]
    bm = np.packbits(valid, bitorder="little")
    where = np.packbits(host["a"] > 0, bitorder="little")
    for analyzers in plans:
        got = scan_states(t, analyzers)
        for an in analyzers:
            if type(an).__name__ != "ApproxCountDistinct":
                continue
            mask = where if an.where else None
            c = an.column
            if c in ("s", "ls"):
                strs = host[c]
                lens = np.array([0 if s is None else len(s) for s in strs], dtype=np.int64)
                offs = np.zeros(n + 1, dtype=np.int64)
                np.cumsum(lens, out=offs[1:])
                data = np.frombuffer(b"".join(s for s in strs if s is not None) + b"\0" * 8, dtype=np.uint8)
                regs = C.hll_registers("large_utf8", data, offs, bm, mask, n)
            else:
                regs = C.hll_registers("i64" if c == "l" else "f64", host[c], None, bm, mask, n)
            want = tuple(O.registers_to_words(regs.tolist()))
            assert got[an].words == want, (an, n, p_redo)
            # the redo values land in high registers: make sure the test exercised them
            if p_redo == 1.0 and not an.where and n >= 4099:
                assert int(regs.max()) >= 24
