"""The oracle itself, pinned before it is trusted (CPU only).

* the reference's own known-answer tests (tests/golden/reference_kats.json, transcribed from
  src/test/scala/com/amazon/deequ/**) must all reproduce;
* XXH64 seed 42 must equal the independent `xxhash` package vectors (hash_vectors.json);
* the C restatement (oracle/c) must agree bit-for-bit with the Python restatement.
"""
from __future__ import annotations

import math

import numpy as np
import pytest

from oracle import dq_oracle as O
from oracle import dq_oracle_c as C
from tests.helpers import oracle_columns


def test_reference_kats(kats):
    for case in kats["cases"]:
        ds = kats["datasets"][case["dataset"]]
        cols, n = oracle_columns(ds)
        st = O.compute_state(tuple(case["analyzer"]), cols, n, ds.get("partitions", 1))
        exp = case["expected"]
        if isinstance(exp, dict):  # DataType: the histogram state itself
            assert st == O.DataTypeHistogram(*exp["DataTypeHistogram"]), (case["source"], st)
            continue
        got = "EmptyState" if st is None else st.metricValue()
        if exp == "NaN":
            assert isinstance(got, float) and math.isnan(got), case
        else:
            assert got == exp, (case["source"], case["analyzer"], got, exp)


def test_state_aggregation_integration_kat(kats):
    """StateAggregationIntegrationTest.scala:56-104: merge of per-partition states == direct."""
    ds = kats["datasets"]["stateAggregation"]
    cols, n = oracle_columns(ds)
    parts = {}
    for mk in ("NA", "EU", "IN"):
        sel = np.array([v == mk for v in ds["columns"]["marketplace"][1]])
        sub = {k: O.OColumn(c.dtype, [v for v, s in zip(c.values, sel) if s] if c.dtype == "utf8" else c.values[sel],
                            c.valid[sel]) for k, c in cols.items()}
        parts[mk] = (sub, int(sel.sum()))
    for spec in (("Completeness", "origin", None), ("StandardDeviation", "sales", None)):
        merged = O.merge_states(*[O.compute_state(spec, p, m) for p, m in parts.values()])
        direct = O.compute_state(spec, cols, n, 2)
        assert merged.metricValue() == pytest.approx(direct.metricValue(), rel=1e-15)


def test_xxh64_vectors(hash_vectors):
    for v, h in hash_vectors["long"]:
        assert O.xxh64_long(v) == h
        assert O.to_i64(int(C.lib().dqo_xxh64_long(v, 42))) == h
    for v, h in hash_vectors["int"]:
        assert O.xxh64_int(v) == h
        assert O.to_i64(int(C.lib().dqo_xxh64_int(v, 42))) == h
    for _, bits, h in hash_vectors["double"]:
        assert O.xxh64_long(bits) == h
    for hx, h in hash_vectors["bytes"]:
        b = bytes.fromhex(hx)
        assert O.xxh64_bytes(b) == h
        assert O.to_i64(int(C.lib().dqo_xxh64_bytes(b, len(b), 42))) == h


def test_numpy_hash_forms_match_scalar():
    rng = np.random.default_rng(0)
    v = rng.integers(-(1 << 62), 1 << 62, 200)
    assert [O.to_i64(int(x)) for x in O.np_xxh64_long(v)] == [O.xxh64_long(int(x)) for x in v]
    w = rng.integers(-(1 << 31), 1 << 31, 200).astype(np.int32)
    assert [O.to_i64(int(x)) for x in O.np_xxh64_int(w)] == [O.xxh64_int(int(x)) for x in w]
    d = np.array([0.0, -0.0, float("nan"), 1.5, -2.25e100])
    assert list(O.np_double_to_long_bits(d)) == [O.double_to_long_bits(float(x)) for x in d]


def test_hll_word_update_equals_register_fold():
    rng = np.random.default_rng(1)
    vals = rng.integers(0, 10_000, 3000)
    words = [0] * O.NUM_WORDS
    for x in vals:
        O.hll_update_words(words, O.xxh64_long(int(x)))
    regs = O.np_hll_registers(O.np_xxh64_long(vals))
    assert words == O.registers_to_words(regs.tolist())
    assert O.words_to_registers(words) == regs.tolist()


def test_hll_jvm_int_shift_quirk():
    """count() computes 1.0 / (1 << Midx) with a JVM Int shift (StatefulHyperloglogPlus.scala:222)."""
    base = [5] * 512
    for m, contrib in ((31, 1.0 / -2147483648.0), (32, 1.0), (33, 0.5), (56, 1.0 / (1 << 24))):
        regs = list(base)
        regs[7] = m
        z = sum(1.0 / 2 ** 5 for _ in range(511)) + contrib
        e = (0.7213 / (1 + 1.079 / 512)) * 512 * 512 / z
        got = O.hll_count(O.registers_to_words(regs))
        assert got == float(O.java_math_round(e if e >= 5 * 512 else e - O._estimate_bias(e))), m


def test_hll_estimates_match_spark_ranges():
    """Linear counting below the p=9 threshold (400), bias-corrected raw estimate above."""
    for d in (10, 100, 300, 1000, 3000, 100_000):
        regs = O.np_hll_registers(O.np_xxh64_long(np.arange(d)))
        est = O.hll_count(O.registers_to_words(regs.tolist()))
        assert abs(est - d) / d < 0.2, (d, est)


def test_java_math_round():
    for a, r in ((0.5, 1), (-0.5, 0), (2.5, 3), (-2.5, -2), (0.49999999999999994, 0), (1e17 + 0.5, 100000000000000000)):
        assert O.java_math_round(a) == r, a


@pytest.mark.parametrize("nparts", [1, 3])
def test_c_oracle_equals_python_oracle(nparts):
    rng = np.random.default_rng(nparts)
    n = 3000
    x = rng.normal(50, 4, n)
    valid = rng.random(n) > 0.1
    vb = np.packbits(valid, bitorder="little")
    s = C.column_stats("f64", x, vb, None, nparts)
    col = {"c": O.OColumn("f64", x, valid)}
    st = O.compute_state(("StandardDeviation", "c", None), col, n, nparts)
    assert (s.n, s.avg, s.m2) == (st.n, st.avg, st.m2)
    assert s.sum_f64 == O.compute_state(("Sum", "c", None), col, n, nparts).sum_
    assert s.min == O.compute_state(("Minimum", "c", None), col, n).minValue
    assert s.max == O.compute_state(("Maximum", "c", None), col, n).maxValue
    iv = rng.integers(-(1 << 62), 1 << 62, n)
    si = C.column_stats("i64", iv, vb, None, nparts)
    ist = O.compute_state(("Sum", "c", None), {"c": O.OColumn("i64", iv, valid)}, n, nparts)
    assert si.sum_f64 == ist.sum_  # wrapping long sum, then cast
    y = 2 * x + rng.normal(0, 1, n)
    vy = rng.random(n) > 0.2
    r = C.corr("f64", x, vb, "f64", y, np.packbits(vy, bitorder="little"), None, nparts)
    cs = O.compute_state(("Correlation", "a", "b", None), {"a": O.OColumn("f64", x, valid), "b": O.OColumn("f64", y, vy)}, n, nparts)
    assert r == (cs.n, cs.xAvg, cs.yAvg, cs.ck, cs.xMk, cs.yMk)
    strs = [b"s%d" % i for i in rng.integers(0, 500, n)]
    data = b"".join(strs)
    offs = np.zeros(n + 1, dtype=np.int32)
    offs[1:] = np.cumsum([len(s) for s in strs])
    regs = C.hll_registers("utf8", np.frombuffer(data + b"\0" * 8, dtype=np.uint8), offs, vb, None, n)
    ref = O.compute_state(("ApproxCountDistinct", "s", None), {"s": O.OColumn("utf8", strs, valid)}, n)
    assert tuple(O.registers_to_words(regs.tolist())) == ref.words


def test_datatype_classes():
    """StatefulDataType.scala:36-38 patterns, whole-value match, first match wins."""
    cases = {b"": 2, b"-": 2, b"+ ": 2, b"- 12": 2, b"007": 2, b".": 1, b"-.5": 1, b"+ 3.": 1, b"1.2.3": 4,
             b"true": 3, b"false": 3, b"TRUE": 4, b"1\n": 4, b"1 ": 4, b" -1": 4, b"--1": 4, b"1e5": 4,
             "\u0661".encode(): 4, b"\xff": 4, b"tru": 4, b"falsee": 4}
    for v, k in cases.items():
        assert O.datatype_class(v) == k, v
    # Double.toString: plain decimal on [1e-3, 1e7) and for zero, else scientific / NaN / Infinity
    for d, k in ((0.0, 1), (-0.0, 1), (1e-3, 1), (0.000999, 4), (9999999.5, 1), (1e7, 4), (-2.5, 1),
                 (float("nan"), 4), (float("-inf"), 4), (1e300, 4)):
        assert O.datatype_class(O.java_double_to_string(d).encode()) == k, d


def test_state_bytes_and_identifier():
    # HdfsStateProvider images are Java DataOutputStream big-endian (StateProvider.scala:176-245)
    assert O.state_to_bytes(O.NumMatches(3)) == bytes.fromhex("0000000000000003")
    assert O.state_to_bytes(O.MeanState(1.0, 2))[:8] == bytes.fromhex("3ff0000000000000")
    img = O.state_to_bytes(O.ApproxCountDistinctState(tuple(range(52))))
    assert img[:4] == bytes.fromhex("000001a0") and len(img) == 420
    img = O.state_to_bytes(O.DataTypeHistogram(1, 2, 3, 4, 5))
    assert img[:4] == bytes.fromhex("00000028") and len(img) == 44 and img[-1] == 5
    # scala.util.hashing.MurmurHash3.stringHash("", 42) == avalanche(42 ^ 0)
    assert isinstance(O.murmur3_string_hash("Size(None)"), int)


def test_vectorised_predicates_match_the_row_evaluator():
    """NpPredicate (the full-scale runs' Compliance oracle) == OracleExpr row by row, incl. C3's predicates,
    decimal literals against int64 (exact), COALESCE, NULL logic, IN, doubles with NaN."""
    rng = np.random.default_rng(3)
    n = 4000
    i0 = rng.integers(-2000, 2000, n).astype(np.int64)
    i1 = rng.integers(-5, 1200, n).astype(np.int64)
    i1[::97] = (1 << 62) + 7
    f = rng.normal(0, 5, n)
    f[::53] = np.nan
    cols = {"i0": ("i64", i0, rng.random(n) > 0.1), "i1": ("i64", i1, rng.random(n) > 0.2),
            "i2": ("i64", rng.integers(-3, 3, n).astype(np.int64), rng.random(n) > 0.1),
            "i3": ("i64", rng.integers(-3, 3, n).astype(np.int64), rng.random(n) > 0.3),
            "f": ("f64", f, rng.random(n) > 0.1)}
    preds = ["i0 >= 0", "`i1` IS NULL OR (`i1` >= 10.0 AND `i1` <= 1000.0)", "i2 < i3", "COALESCE(i3, 0.0) >= 0",
             "i0 > 2.5", "i0 <= -3.5", "i0 = 7.0", "i0 != 7.5", "i1 < 4611686018427387911", "f >= 0.5",
             "f < i0", "NOT (i2 = i3) OR f IS NULL", "i0 IN (1, 2, 3.0)", "f > 1e0 AND i3 IS NOT NULL",
             "COALESCE(f, i0) > 0", "i2 >= NULL", "i0 < 1e30", "i0 > -99999999999999999999.5"]
    ocols = {k: O.OColumn(t, v, valid) for k, (t, v, valid) in cols.items()}
    for p in preds:
        t_ref, nn_ref = O.OracleExpr(p).eval_bool(ocols, n)
        t_np, nn_np = O.NpPredicate(p).eval_bool(cols, n)
        assert (t_ref == t_np).all() and (nn_ref == nn_np).all(), p
