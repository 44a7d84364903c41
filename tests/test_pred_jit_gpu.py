"""The compiled predicate pass (deequ_amd/csrc/dq_pred_jit.cpp) against the interpreter and the oracle.

Spark evaluates Compliance / `where` predicates by whole-stage code generation inside the one aggregation
pass (AnalysisRunner.scala:303, Compliance.scala:37-53); dq_plan_create does the same on the GPU, generating a
kernel for the plan's numeric predicate program and compiling it with hipRTC.  That kernel is a second product
implementation of A3 (Compliance / where) and -- for ApproxCountDistinct without `where` on a program column --
of A9 (HLL++ registers, StatefulHyperloglogPlus.scala:89-115).  These tests pin it:

* the plan of config C3 (and every numeric program below) runs the compiled kernel: dq_plan_create_opts with
  DQ_PRED_PASS_COMPILED fails instead of falling back, so a missing hipRTC fails the suite;
* the compiled kernel and the interpreter (DQ_PRED_PASS_INTERPRETER, the column pass hashing the HLL columns)
  give bit-identical states on the same plan, and both equal the oracle (counts, HLL registers);
* fused HLL on int32 and fp64 columns (NaN, -0.0, +-inf, and constructed values whose hash needs the exact-rank
  redo), at row counts that are not multiples of 64 / 512 / 2048;
* a predicate column that ends exactly at the end of its allocation (the next-block prefetch of the range's
  last block lies past it).
"""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

from oracle import dq_oracle as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def dq():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    import deequ_amd

    return deequ_amd


@pytest.fixture(scope="module")
def redo_values():
    with open(os.path.join(HERE, "golden", "hll_redo_values.json")) as f:
        d = json.load(f)
    f64 = np.array([int(b, 16) for b in d["f64_bits"]], dtype=np.uint64).view(np.float64)
    return np.array(d["i64"], dtype=np.int64), np.array(d["i32"], dtype=np.int32), f64


def _spec(a):
    name = type(a).__name__
    if name == "Compliance":
        return ("Compliance", a.instance, a.predicate, a.where)
    if name == "Size":
        return ("Size", a.where)
    if name == "Correlation":
        return ("Correlation", a.firstColumn, a.secondColumn, a.where)
    return (name, a.column, a.where)


def _check_vs_oracle(dq, states, analyzers, ocols, n):
    for a in analyzers:
        ref = O.compute_state(_spec(a), ocols, n)
        got = states[a]
        if ref is None:
            assert got is None, (a, got)
            continue
        name = type(ref).__name__
        if name == "NumMatchesAndCount":
            assert got == dq.NumMatchesAndCount(ref.numMatches, ref.count), (a, got, ref)
        elif name == "NumMatches":
            assert got == dq.NumMatches(ref.numMatches), (a, got, ref)
        elif name == "ApproxCountDistinctState":
            assert tuple(got.words) == tuple(ref.words), a
        else:
            raise AssertionError(name)


def _both_passes(dq, table, analyzers):
    """States of the compiled pass (required) and of the interpreter on the same analyzers; launch counts."""
    from deequ_amd.runner import ScanPlan, scan_states

    plan = ScanPlan(analyzers, table.schema, pred_pass="compiled")
    ok, origin = plan.pred_compiled()
    assert ok and origin in ("hiprtc", "disk cache", "process cache"), (ok, origin)
    total_ms, jit_ms = plan.create_time()
    assert 0.0 <= jit_ms <= total_ms
    fused_launches = plan.num_launches()
    plan.close()
    plan = ScanPlan(analyzers, table.schema, pred_pass="interpreter")
    assert plan.pred_compiled()[0] is False
    interp_launches = plan.num_launches()
    plan.close()
    return (scan_states(table, analyzers, "compiled"), scan_states(table, analyzers, "interpreter"),
            fused_launches, interp_launches)


def test_c3_plan_runs_the_compiled_pass(dq):
    """Config C3's plan (4 int64 Compliance predicates + HLL of i0..i3 and s0..s3): the default plan runs the
    compiled kernel, DQ_PRED_PASS_COMPILED accepts it, and the fused HLL tasks leave the column pass
    (one launch fewer than with the interpreter)."""
    from deequ_amd import synth
    from deequ_amd.runner import ScanPlan

    t = synth.c3_table(4099, seed=5)
    an = synth.c3_analyzers(t)
    plan = ScanPlan(an, t.schema)
    assert plan.pred_wait(), plan.pred_compiled()  # AUTO: a cold compile runs in the background
    ok, origin = plan.pred_compiled()
    assert ok, origin
    plan.close()
    c, i, fl, il = _both_passes(dq, t, an)
    assert fl < il, (fl, il)
    for a in an:
        assert c[a] == i[a] or (c[a] is None and i[a] is None), (a, c[a], i[a])


def test_large_program_stays_on_the_interpreter(dq):
    """A program of more than 16 counters (29 Compliance predicates) is not compiled -- LLVM's register
    allocation of the pinned counters fails past ~24 after up to a minute of hipRTC time -- and runs on the
    interpreter, equal to the oracle.  DQ_PRED_PASS_COMPILED treats the generated kernel's limits as plan
    capacities: the set splits into fused plans whose programs each fit the kernel, all compiled."""
    from deequ_amd.runner import ScanPlan, scan_states

    t, ocols = _abc_table(dq, 4097, 9)
    an = [dq.Compliance(f"r{i}", p) for i, p in enumerate(PREDICATES)]
    plan = ScanPlan(an, t.schema)
    ok, note = plan.pred_compiled()
    assert not ok and "16 counters" in note, note
    assert plan.create_time()[1] == 0.0
    plan.close()
    comp = ScanPlan(an, t.schema, pred_pass="compiled")
    ok, note = comp.pred_compiled()
    assert ok and note.count("part ") >= 2, note
    comp.close()
    _check_vs_oracle(dq, scan_states(t, an), an, ocols, 4097)
    _check_vs_oracle(dq, scan_states(t, an, "compiled"), an, ocols, 4097)


def test_compiled_requires_eligible_program(dq):
    """DQ_PRED_PASS_COMPILED on a program with a string atom fails plan creation (no silent interpreter)."""
    from deequ_amd._lib import DQ_E_UNSUPPORTED, DQError
    from deequ_amd.runner import ScanPlan

    t = dq.Table.from_pydict({"s": ("utf8", ["a", None, "b"]), "x": ("i64", [1, 2, None])})
    an = [dq.Compliance("eq", "s = 'a'"), dq.Compliance("gt", "x > 1")]
    with pytest.raises(DQError) as e:
        ScanPlan(an, t.schema, pred_pass="compiled")
    assert e.value.status == DQ_E_UNSUPPORTED and "not eligible" in e.value.message
    plan = ScanPlan(an, t.schema)
    assert plan.pred_compiled()[0] is False
    plan.close()


PREDICATES = [
    "a > 3", "a >= 3.0", "a > 2.5", "a < -1.5", "a = 4", "a = 4.5", "a != 4.5", "a <> 7",
    "b <= 0.25", "b > 1e1", "a < b", "b >= a", "a = c", "c > a", "b = b", "b > 1e300",
    "COALESCE(a, 0.0) >= 0", "COALESCE(b, 1.0) > 0", "COALESCE(a, 5) < 3",
    "`a` IS NULL OR (`a` >= 0.0 AND `a` <= 7.0)", "`b` IS NULL OR (`b` > -1.0 AND `b` < 8.0)",
    "a IS NOT NULL", "NOT (a > 2 AND b < 0.5)", "a > 2 OR b IS NULL", "NOT a > 2",
    "(a > 1 AND b > 0.1) OR (c < 0 AND a IS NULL)", "TRUE", "NULL", "a > NULL", "1 < 2", "1.5 > 2",
]
WHERES = ["a > 2", "b < 0.5", "c IS NULL", "COALESCE(a, 0.0) >= 0", "a > 100", "NOT (b > 0 OR c < 2)"]


def _abc_table(dq, n, seed):
    from deequ_amd.table import column_from_numpy

    rng = np.random.default_rng(seed)
    a = rng.integers(-8, 12, n).astype(np.int64)
    b = np.round(rng.normal(0.5, 2.0, n), 2)
    b[rng.random(n) < 0.05] = np.nan
    b[rng.random(n) < 0.01] = np.inf
    b[rng.random(n) < 0.01] = -np.inf
    b[rng.random(n) < 0.01] = -0.0
    c = rng.integers(-5, 10, n).astype(np.int32)
    va, vb, vc = rng.random(n) > 0.15, rng.random(n) > 0.2, rng.random(n) > 0.1
    d = {"a": ("i64", a, va), "b": ("f64", b, vb), "c": ("i32", c, vc)}
    t = dq.Table([column_from_numpy(k, ty, v, m) for k, (ty, v, m) in d.items()])
    return t, {k: O.OColumn(ty, v, m) for k, (ty, v, m) in d.items()}


@pytest.mark.parametrize("n", [1, 63, 65, 511, 513, 2047, 2049, 4097, 100_003])
def test_predicates_compiled_equals_interpreter_and_oracle(dq, n):
    """Every PREDICATES / WHERES program of the parity suite in one plan: compiled == interpreter == oracle,
    with NaN / +-inf / -0.0 in the fp64 column."""
    t, ocols = _abc_table(dq, n, 100 + n)
    wheres = []
    for w in WHERES:
        wheres += [dq.Size(w), dq.Compliance("w", "a < b", w), dq.ApproxCountDistinct("a", w),
                   dq.ApproxCountDistinct("b", w), dq.Completeness("c", w)]
    # plans of <= 16 counters (the compiled pass's limit; larger programs stay on the interpreter)
    preds = [dq.Compliance(f"r{i}", p) for i, p in enumerate(PREDICATES)]
    for an in (preds[:12], preds[12:24], preds[24:], wheres[:15], wheres[15:]):
        c, i, _, _ = _both_passes(dq, t, an)
        for a in an:
            assert c[a] == i[a] or (c[a] is None and i[a] is None), (a, c[a], i[a])
        _check_vs_oracle(dq, c, an, ocols, n)


@pytest.mark.parametrize("n", [1, 513, 4099, 300_007])
def test_fused_hll_i32_f64_i64_with_redo_values(dq, redo_values, n):
    """ApproxCountDistinct (no `where`) of the program's int64, int32 and fp64 columns is hashed by the
    compiled kernel (dq_pred_jit.cpp: int32 via hashInt, fp64 via doubleToLongBits with NaN canonical and
    -0.0 / +-inf as their bits), including values whose hash needs the exact-rank redo: registers equal the
    interpreter plan's column pass and the oracle bit for bit; the fused plan has fewer launches."""
    from deequ_amd.table import column_from_numpy

    i64r, i32r, f64r = redo_values
    rng = np.random.default_rng(7 + n)
    pick = rng.random(n) < 0.02
    a = np.where(pick, i64r[rng.integers(0, len(i64r), n)], rng.integers(-1000, 1000, n)).astype(np.int64)
    b = np.where(rng.random(n) < 0.02, i32r[rng.integers(0, len(i32r), n)], rng.integers(-50, 50, n)).astype(np.int32)
    x = np.where(rng.random(n) < 0.02, f64r[rng.integers(0, len(f64r), n)], rng.normal(size=n))
    special = np.array([np.nan, -np.nan, -0.0, 0.0, np.inf, -np.inf, np.float64("nan")])
    where_special = rng.random(n) < 0.05
    x[where_special] = special[rng.integers(0, len(special), int(where_special.sum()))]
    if n > 10:  # a non-canonical NaN bit pattern hashes as the canonical NaN (doubleToLongBits)
        x[3] = np.array([0x7FF00000DEADBEEF], dtype=np.uint64).view(np.float64)[0]
    va, vx = rng.random(n) > 0.1, rng.random(n) > 0.2
    t = dq.Table([column_from_numpy("a", "i64", a, va),
                  column_from_numpy("b", "i32", b, np.ones(n, bool), nullable=False),
                  column_from_numpy("x", "f64", x, vx)])
    an = [dq.Compliance("c1", "a > 0 AND b < 10"), dq.Compliance("c2", "x >= 0.5 OR a IS NULL"),
          dq.ApproxCountDistinct("a"), dq.ApproxCountDistinct("b"), dq.ApproxCountDistinct("x"),
          dq.Completeness("a"), dq.Completeness("x"), dq.Size()]
    c, i, fl, il = _both_passes(dq, t, an)
    assert fl < il, (fl, il)
    for k in an:
        assert c[k] == i[k] or (c[k] is None and i[k] is None), (k, c[k], i[k])
    ocols = {"a": O.OColumn("i64", a, va), "b": O.OColumn("i32", b, np.ones(n, bool)), "x": O.OColumn("f64", x, vx)}
    _check_vs_oracle(dq, c, an[:5], ocols, n)


def test_redo_only_table_through_compiled_pass(dq, redo_values):
    """A table made only of redo values (every selected row takes the exact-rank path of the compiled
    kernel, the rows past the last full row group included)."""
    from deequ_amd.table import column_from_numpy

    i64r, i32r, f64r = redo_values
    n = 3 * 2048 + 77
    rng = np.random.default_rng(3)
    a = i64r[rng.integers(0, len(i64r), n)]
    b = i32r[rng.integers(0, len(i32r), n)]
    x = f64r[rng.integers(0, len(f64r), n)]
    v = rng.random(n) > 0.05
    t = dq.Table([column_from_numpy("a", "i64", a, v), column_from_numpy("b", "i32", b, v),
                  column_from_numpy("x", "f64", x, v)])
    an = [dq.Compliance("p", "a > 0 OR b < 0 OR x > 0"), dq.ApproxCountDistinct("a"), dq.ApproxCountDistinct("b"),
          dq.ApproxCountDistinct("x")]
    c, i, _, _ = _both_passes(dq, t, an)
    for k in an:
        assert c[k] == i[k], (k, c[k], i[k])
    ocols = {"a": O.OColumn("i64", a, v), "b": O.OColumn("i32", b, v), "x": O.OColumn("f64", x, v)}
    _check_vs_oracle(dq, c, an, ocols, n)


@pytest.mark.parametrize("n", [100_002, 2048 * 64 + 1030])
def test_predicate_column_at_end_of_allocation(dq, n):
    """The predicate columns are the last bytes of their device allocations and n is not a multiple of the
    2048-row block: the compiled kernel's next-block prefetch in the range's last block lies past the
    column, and must read nothing from there (bounds-checked voffset); counts equal the interpreter's and
    the oracle's."""
    import torch

    from deequ_amd.table import Column, column_from_numpy, pack_validity

    rng = np.random.default_rng(n)
    a = rng.integers(-100, 100, n).astype(np.int64)
    x = rng.normal(size=n)
    va = rng.random(n) > 0.1

    def tail_column(name, dtype, values, valid):
        raw = values.view(np.uint8)
        seg = torch.empty(2 * 1024 * 1024 * ((len(raw) >> 21) + 1), dtype=torch.uint8, device="cuda")
        off = seg.numel() - len(raw)
        assert off % 16 == 0
        vt = seg[off:]
        vt.copy_(torch.from_numpy(raw))
        bt = torch.from_numpy(pack_validity(valid)).to("cuda")
        return Column(name, dtype, len(values), vt, bt, None, nullable=True)

    t = dq.Table([tail_column("a", "i64", a, va), tail_column("x", "f64", x, np.ones(n, bool)),
                  column_from_numpy("y", "i64", a[::-1].copy(), va)])
    an = [dq.Compliance("p", "a > 10 AND x < 0.5"), dq.Compliance("q", "a <= y"), dq.Size("x > 1.0")]
    c, i, _, _ = _both_passes(dq, t, an)
    for k in an:
        assert c[k] == i[k], (k, c[k], i[k])
    ocols = {"a": O.OColumn("i64", a, va), "x": O.OColumn("f64", x, np.ones(n, bool)),
             "y": O.OColumn("i64", a[::-1].copy(), va)}
    _check_vs_oracle(dq, c, an, ocols, n)


def _unique_predicates(tag):
    """Predicates no other test compiles (a fresh kernel source: neither cache has it)."""
    import time

    k = (time.time_ns() // 1000) % 1_000_003 + 17
    return [f"a > {k % 11 - 5}", f"COALESCE(b, {k}.0) < {k % 7}.5", f"a < c OR c = {tag}", f"b IS NULL OR a >= {k % 13}"]


def test_background_compile_switches_between_chunks(dq, tmp_path, monkeypatch):
    """AUTO with a kernel in neither cache: plan creation does not wait for hipRTC, the first chunk runs the
    interpreter, later chunks the compiled kernel (with the fused HLL tasks), and the states are bit-identical
    to the interpreter's and equal to the oracle."""
    from deequ_amd.runner import ScanPlan
    from deequ_amd.table import column_from_numpy

    monkeypatch.setenv("DQ_JIT_CACHE_DIR", str(tmp_path / "jit"))
    n, parts = 30011, 3
    t, ocols = _abc_table(dq, n, 77)
    an = [dq.Compliance(f"q{i}", p) for i, p in enumerate(_unique_predicates(1))]
    an += [dq.ApproxCountDistinct("a"), dq.ApproxCountDistinct("c"), dq.Size("a > 0"), dq.Completeness("b", "c > 1")]
    bounds = [0, 7001, 19000, n]
    chunks = []
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        chunks.append(dq.Table([column_from_numpy(k, ocols[k].dtype, ocols[k].values[lo:hi], ocols[k].valid[lo:hi])
                                for k in ("a", "b", "c")]))
    plan = ScanPlan(an, t.schema)
    total_ms, jit_ms = plan.create_time()
    ok, note = plan.pred_compiled()
    assert not ok and "background" in note, note
    assert total_ms < 100.0, total_ms  # no hipRTC inside plan creation
    plan.scan(chunks[0])
    assert plan.pred_wait(), plan.pred_compiled()
    for c in chunks[1:]:
        plan.scan(c)
    ok, note = plan.pred_compiled()
    assert ok and "used from chunk 1" in note, note
    got = {a: a._from_result(r) for a, r in zip(an, plan.finish())}
    plan.close()
    from deequ_amd.runner import scan_states

    ref = scan_states(chunks, an, "interpreter")
    for a in an:
        assert got[a] == ref[a] or (got[a] is None and ref[a] is None), (a, got[a], ref[a])
    _check_vs_oracle(dq, got, an, ocols, n)
    # the code object is now in the (private, keyed) disk cache
    files = list((tmp_path / "jit").glob("*.co"))
    assert files and files[0].read_bytes()[:8] == b"DQJITCO1"


def test_concurrent_plan_creation_does_not_serialize_on_hiprtc(dq, monkeypatch):
    """Two threads create plans with kernels in neither cache at once: both return without waiting for a
    compile (the process-wide lock is held for the map lookup only), and both kernels become ready."""
    import threading
    import time

    from deequ_amd.runner import ScanPlan

    monkeypatch.setenv("DQ_JIT_CACHE_DIR", "off")
    t, _ = _abc_table(dq, 1000, 3)
    plans, errs, times = [None, None], [], [0.0, 0.0]
    import torch

    def make(k):
        try:
            torch.cuda.set_device(0)
            t0 = time.perf_counter()
            plans[k] = ScanPlan([dq.Compliance(f"t{i}", p) for i, p in enumerate(_unique_predicates(k + 10))], t.schema)
            times[k] = time.perf_counter() - t0
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=make, args=(k,)) for k in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs
    # neither creation waited for a compile (one hipRTC compile of such a program takes ~0.3 s): the part of
    # dq_plan_create spent obtaining the kernel is a map lookup and a thread start; the wall time includes
    # the thread's first HIP calls
    assert all(p.create_time()[1] < 50.0 for p in plans), [p.create_time() for p in plans]
    assert max(times) < 0.3, times
    for p in plans:
        assert p.pred_wait(), p.pred_compiled()
        p.close()


def test_jit_cache_refuses_foreign_or_shared_dirs(dq, tmp_path, monkeypatch):
    """A cache directory writable by group / others is not used (a planted code object would run); the plan
    still compiles its kernel (no disk cache) and nothing is written there."""
    from deequ_amd.runner import ScanPlan

    d = tmp_path / "shared"
    d.mkdir()
    d.chmod(0o777)
    monkeypatch.setenv("DQ_JIT_CACHE_DIR", str(d))
    t, _ = _abc_table(dq, 100, 4)
    plan = ScanPlan([dq.Compliance("u", p) for p in _unique_predicates(99)], t.schema, pred_pass="compiled")
    ok, origin = plan.pred_compiled()
    assert ok and origin == "hiprtc", origin
    plan.close()
    assert not list(d.iterdir())
