"""Full-scale parity (TEST INFRASTRUCTURE): the GPU scan of configs C2 / C3 / C4 / C5 at up to 1e9 rows vs
the C oracle (Spark partition order) and, for fp64 results, a near-exact reference.

* Integer results are compared BIT-EXACTLY with the oracle: Size, Completeness and Compliance counts, HLL
  register words and estimates (StatefulHyperloglogPlus.scala:89-115, incl. how many rows reached the
  kernels' exact-rank redo and general-string paths), int64 Min / Max, and the wrapping int64 Sum / Mean
  partials (Spark's LongType sum, cast at the end).
* fp64 results: SURVEY §7 "hard parts" -- at 1e9 rows Spark's own sequential rounding approaches the 1e-12
  bar, so every mean / stddev / sum / moment / correlation is compared with a double-double reference
  (~1e-22 relative; oracle/c dqo_exact_*) and must be within the north-star 1e-12 STRICT relative error
  |v - exact| / |exact|; the Spark-order oracle's own error is reported beside it.
* Compliance (C3's four predicates) uses the oracle's vectorised evaluator (NpPredicate, checked against
  the per-row OracleExpr in tests/test_oracle.py).

The data is generated on the device chunk by chunk (125M rows per chunk), scanned, copied to the host
and folded by the oracle, so host memory holds one chunk at a time.

    python tests/fullscale_parity.py --cfg c2 c3 c4 c5 --rows 1000000000 --out profiles/r3_fullscale_parity.json

Spark order: every chunk is split into `parts` row partitions, each folded sequentially (the partial
aggregate), and ALL partitions are merged in row order from the zero buffer (the final aggregate).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from fractions import Fraction

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

STRICT = 1e-12
C3_PREDICATES = [("p0", "i0 >= 0"), ("p1", "`i1` IS NULL OR (`i1` >= 10.0 AND `i1` <= 1000.0)"),
                 ("p2", "i2 < i3"), ("p3", "COALESCE(i3, 0.0) >= 0")]


def _f(dd) -> Fraction:
    return Fraction(dd[0]) + Fraction(dd[1])


def _rel(v: float, exact: Fraction) -> float:
    if math.isnan(v):
        return math.inf
    if exact == 0:
        return abs(v)
    return float(abs(Fraction(v) - exact) / abs(exact))


def _wrap64(x: int) -> int:
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >= 1 << 63 else x


def _analyzers(dq, cfg, schema):
    names = [c[0] for c in schema]
    if cfg == "c2":  # Size + per column Completeness, Mean, StdDev, Min, Max (+ Sum)
        out = [dq.Size()]
        for c in names:
            out += [dq.Completeness(c), dq.Mean(c), dq.StandardDeviation(c), dq.Minimum(c), dq.Maximum(c), dq.Sum(c)]
        return out
    if cfg == "c3":  # Size + ApproxCountDistinct x 8 + Compliance x 4 (bench.py config_setup)
        return [dq.Size()] + [dq.ApproxCountDistinct(c) for c in names] + [dq.Compliance(i, p) for i, p in C3_PREDICATES]
    if cfg == "c5":  # ColumnProfiler passes 1-2 (synth.profile_analyzers)
        out = [dq.Size()]
        for name, dtype, _ in schema:
            out += [dq.Completeness(name), dq.ApproxCountDistinct(name)]
            if dtype in ("f64", "i64"):
                out += [dq.Minimum(name), dq.Maximum(name), dq.Mean(name), dq.StandardDeviation(name), dq.Sum(name)]
        return out
    out = [dq.Correlation(names[i], names[j]) for i in range(len(names)) for j in range(i + 1, len(names))]
    return out + [dq.Mean(c) for c in names] + [dq.StandardDeviation(c) for c in names]


def _host(col, m):
    """device Column -> dict of host arrays (values / offsets / data / bitmap / valid)"""
    bm = col.validity[: (m + 7) // 8 + 16].cpu().numpy() if col.validity is not None else None
    h = {"bm": bm}
    if col.dtype == "utf8":
        offs = col.offsets[: (m + 1) * 4].cpu().numpy().view(np.int32)
        h["offs"] = offs
        h["data"] = col.values[: int(offs[-1]) + 16].cpu().numpy()
    else:
        h["vals"] = col.values[: m * 8].cpu().numpy().view(np.float64 if col.dtype == "f64" else np.int64)
    return h


def run(cfg: str, rows: int, chunk: int = 125_000_000, parts: int = 16, nthreads: int = 16, seed: int = 42,
        log=print) -> dict:
    import torch

    import deequ_amd as dq
    from deequ_amd import synth
    from deequ_amd.runner import ScanPlan
    from oracle import dq_oracle as O
    from oracle import dq_oracle_c as C

    gen = {"c2": synth.c2_table, "c3": synth.c3_table, "c4": synth.c4_table, "c5": synth.c5_table}[cfg]
    t0 = gen(min(chunk, rows), 0, seed)
    schema = t0.schema
    names = [c[0] for c in schema]
    dtypes = {c[0]: c[1] for c in schema}
    analyzers = _analyzers(dq, cfg, schema)
    plan = ScanPlan(analyzers, schema)
    del t0
    moments = [c for c in names if dtypes[c] in ("f64", "i64") and cfg != "c3"]  # columns with moment analyzers
    hll = names if cfg in ("c3", "c5") else []
    col_parts = {c: [] for c in moments}
    pair_parts = {}
    pivots = {}
    exact = {c: [0, Fraction(0), Fraction(0)] for c in moments}
    regs = {c: np.zeros(512, dtype=np.uint8) for c in hll}
    paths = {c: {"redo": 0, "long": 0, "window": 0} for c in hll}
    valid_count = {c: 0 for c in names}
    comp = {i: 0 for i, _ in C3_PREDICATES}
    npreds = {i: O.NpPredicate(p) for i, p in C3_PREDICATES}
    pairs = [(names[i], names[j]) for i in range(len(names)) for j in range(i + 1, len(names))] if cfg == "c4" else []
    pexact = {p: [0] + [Fraction(0)] * 5 for p in pairs}
    timing = {"gpu_gen_scan_s": 0.0, "copy_s": 0.0, "oracle_s": 0.0, "exact_s": 0.0}
    r = 0
    k = 0
    while r < rows:
        m = min(chunk, rows - r)
        a = time.perf_counter()
        t = gen(m, r, seed)
        plan.scan(t)
        torch.cuda.synchronize()
        b = time.perf_counter()
        host = {c: _host(t.columns[c], m) for c in names}
        del t
        torch.cuda.empty_cache()
        c_ = time.perf_counter()
        for c in names:
            h = host[c]
            valid_count[c] += m if h["bm"] is None else C.lib().dqo_count_bits(h["bm"].ctypes.data, None, m)
        for c in moments:
            col_parts[c] += C.column_stats_partials(dtypes[c], host[c]["vals"], host[c]["bm"], parts, nthreads)
        for c in hll:
            h = host[c]
            if dtypes[c] == "utf8":
                _, pth = C.hll_registers_mt("utf8", h["data"], h["offs"], h["bm"], None, m, nthreads, regs[c])
            else:
                _, pth = C.hll_registers_mt(dtypes[c], h["vals"], None, h["bm"], None, m, nthreads, regs[c])
            for key in pth:
                paths[c][key] += pth[key]
        if cfg == "c3":
            pc = {c: (dtypes[c], host[c]["vals"], np.unpackbits(host[c]["bm"], bitorder="little")[:m].astype(bool))
                  for c in ("i0", "i1", "i2", "i3")}
            for i, _ in C3_PREDICATES:
                comp[i] += int(npreds[i].eval_bool(pc, m)[0].sum())
            del pc
        for (x, y) in pairs:
            pair_parts.setdefault((x, y), [])
            pair_parts[(x, y)] += C.corr_partials("f64", host[x]["vals"], host[x]["bm"], "f64", host[y]["vals"],
                                                  host[y]["bm"], parts, nthreads)
        d = time.perf_counter()
        for c in moments:
            vals, bm = host[c]["vals"], host[c]["bm"]
            if c not in pivots:  # pivot: the column's first selected value (any fixed double works)
                valid = np.unpackbits(bm[: 1024], bitorder="little")[: min(m, 8192)].astype(bool) if bm is not None else None
                pivots[c] = float(vals[np.argmax(valid)] if valid is not None else vals[0])
            cnt, s1, s2 = C.exact_moments(dtypes[c], vals, bm, pivots[c], nthreads)
            e = exact[c]
            e[0] += cnt
            e[1] += _f(s1)
            e[2] += _f(s2)
        for (x, y) in pairs:
            res = C.exact_comoments("f64", host[x]["vals"], host[x]["bm"], "f64", host[y]["vals"], host[y]["bm"],
                                    pivots[x], pivots[y], nthreads)
            e = pexact[(x, y)]
            e[0] += res[0]
            for q in range(5):
                e[1 + q] += _f(res[1 + q])
        del host
        e_ = time.perf_counter()
        timing["gpu_gen_scan_s"] += b - a
        timing["copy_s"] += c_ - b
        timing["oracle_s"] += d - c_
        timing["exact_s"] += e_ - d
        log(f"{cfg}: chunk {k} ({r + m}/{rows} rows) gpu {b - a:.1f}s copy {c_ - b:.1f}s oracle {d - c_:.1f}s "
            f"exact {e_ - d:.1f}s")
        r += m
        k += 1
    states = dict(zip(analyzers, [a._from_result(s) for a, s in zip(analyzers, plan.finish())]))
    plan.close()

    report = {"cfg": cfg, "rows": rows, "chunk_rows": chunk, "spark_partitions": parts * k, "threads": nthreads,
              "strict_bar": STRICT, "columns": {}, "pairs": {}, "integer_checks": 0, "timing": timing}
    worst = {"gpu": 0.0, "oracle": 0.0}
    failures = []

    def exact_eq(what, got, want):
        report["integer_checks"] += 1
        same = got == want or (isinstance(got, float) and isinstance(want, float) and math.isnan(got) and math.isnan(want))
        if not same:
            failures.append(f"{what}: gpu {got!r} != oracle {want!r}")

    def strict(rec, key, gval, oval, ex):
        ge, oe = _rel(gval, ex), _rel(oval, ex)
        rec["gpu_rel_err"][key], rec["oracle_rel_err"][key] = ge, oe
        worst["gpu"] = max(worst["gpu"], ge)
        worst["oracle"] = max(worst["oracle"], oe)
        if ge > STRICT:
            failures.append(f"{rec['name']}.{key}: gpu strict rel err {ge:.3g} > 1e-12 (oracle {oe:.3g})")

    size = states.get(dq.Size())
    if size is not None:
        exact_eq("Size", size.numMatches, rows)
    for c in names:
        rec = {"name": c, "dtype": dtypes[c], "gpu_rel_err": {}, "oracle_rel_err": {}}
        an = dq.Completeness(c)
        if an in states:
            exact_eq(f"Completeness({c})", (states[an].numMatches, states[an].count), (valid_count[c], rows))
        if c in hll:
            st = states[dq.ApproxCountDistinct(c)]
            want = tuple(O.registers_to_words(regs[c].tolist()))
            exact_eq(f"ApproxCountDistinct({c}).words", st.words, want)
            exact_eq(f"ApproxCountDistinct({c}).estimate", st.metricValue(), O.hll_count(want))
            rec["hll_estimate"] = O.hll_count(want)
            rec["rare_path_rows"] = paths[c]
        if c in moments:
            o = C.stats_fold(dtypes[c], col_parts[c])
            n_e, s1, s2 = exact[c]
            piv = Fraction(pivots[c])
            mean_e = piv + s1 / n_e
            m2_e = s2 - s1 * s1 / n_e
            sd_state = states[dq.StandardDeviation(c)]
            mean_state = states[dq.Mean(c)]
            exact_eq(f"StandardDeviation({c}).n", sd_state.n, float(o.count))
            exact_eq(f"Mean({c}).count", mean_state.count, o.count)
            rec["n"] = n_e
            if n_e != o.count:
                failures.append(f"{c}: exact reference count {n_e} != oracle {o.count}")
            strict(rec, "stddev", sd_state.metricValue(), math.sqrt(o.m2 / o.n), Fraction(math.sqrt(float(m2_e / n_e))))
            strict(rec, "avg_state", sd_state.avg, o.avg, mean_e)
            strict(rec, "m2_state", sd_state.m2, o.m2, m2_e)
            if dtypes[c] == "f64":
                sum_e = piv * n_e + s1
                strict(rec, "mean", mean_state.sum_ / mean_state.count, o.sum_f64 / o.count, mean_e)
                strict(rec, "sum", mean_state.sum_, o.sum_f64, sum_e)
            else:  # Spark LongType sum: wrapping int64, cast to double at the end -- bit-exact
                exact_eq(f"Mean({c}).sum", mean_state.sum_, o.sum_f64)
                rec["int64_sum_wrapped"] = int(o.sum_i64)
            an = dq.Sum(c)
            if an in states:
                if dtypes[c] == "f64":
                    strict(rec, "Sum", states[an].sum_, o.sum_f64, piv * n_e + s1)
                else:
                    exact_eq(f"Sum({c})", states[an].sum_, o.sum_f64)
            for an, want in ((dq.Minimum(c), o.min), (dq.Maximum(c), o.max)):
                if an in states:
                    exact_eq(str(an), states[an].metricValue(), want)
        report["columns"][c] = rec
    if cfg == "c3":
        for i, p in C3_PREDICATES:
            st = states[dq.Compliance(i, p)]
            exact_eq(f"Compliance({i})", (st.numMatches, st.count), (comp[i], rows))
        report["compliance_matches"] = comp
    for (x, y) in pairs:
        o = C.corr_fold(pair_parts[(x, y)])
        n_e, sx, sy, sxy, sxx, syy = pexact[(x, y)]
        px, py = Fraction(pivots[x]), Fraction(pivots[y])
        ck_e = sxy - sx * sy / n_e
        xm_e = sxx - sx * sx / n_e
        ym_e = syy - sy * sy / n_e
        corr_e = float(ck_e) / math.sqrt(float(xm_e) * float(ym_e))
        ex = {"corr": Fraction(corr_e), "ck": ck_e, "xMk": xm_e, "yMk": ym_e, "xAvg": px + sx / n_e,
              "yAvg": py + sy / n_e}
        st = states[dq.Correlation(x, y)]
        g = {"corr": st.metricValue(), "ck": st.ck, "xMk": st.xMk, "yMk": st.yMk, "xAvg": st.xAvg, "yAvg": st.yAvg}
        orc = {"corr": o[3] / math.sqrt(o[4] * o[5]), "ck": o[3], "xMk": o[4], "yMk": o[5], "xAvg": o[1], "yAvg": o[2]}
        rec = {"name": f"corr({x},{y})", "n": n_e, "gpu_rel_err": {}, "oracle_rel_err": {}}
        exact_eq(f"corr({x},{y}).n", st.n, o[0])
        if st.n != n_e:
            failures.append(f"corr({x},{y}) n: gpu {st.n} exact {n_e}")
        for key in ex:
            strict(rec, key, g[key], orc[key], ex[key])
        report["pairs"][f"{x},{y}"] = rec
    report["worst_strict_rel_err"] = worst
    report["gpu_within_1e-12_strict"] = worst["gpu"] <= STRICT
    report["rare_path_rows_total"] = {key: sum(p[key] for p in paths.values()) for key in ("redo", "long", "window")}
    report["failures"] = failures
    report["ok"] = not failures
    return report


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", nargs="+", default=["c2", "c3", "c4", "c5"])
    ap.add_argument("--rows", type=int, default=1_000_000_000)
    ap.add_argument("--chunk", type=int, default=125_000_000)
    ap.add_argument("--parts", type=int, default=16, help="Spark partitions per chunk")
    ap.add_argument("--threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16")))
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch

    torch.cuda.set_device(0)
    reports = []
    for cfg in args.cfg:
        rep = run(cfg, args.rows, args.chunk, args.parts, args.threads, log=lambda s: print(s, flush=True))
        print(json.dumps({"cfg": cfg, "ok": rep["ok"], "worst_strict_rel_err": rep["worst_strict_rel_err"],
                          "integer_checks": rep["integer_checks"], "rare_path_rows": rep["rare_path_rows_total"],
                          "failures": rep["failures"][:10]}), flush=True)
        reports.append(rep)
        if args.out:
            with open(args.out, "w") as f:
                json.dump(reports, f, indent=1)
    sys.exit(0 if all(r["ok"] for r in reports) else 1)


if __name__ == "__main__":
    main()
