"""Full-scale fp64 parity (TEST INFRASTRUCTURE): the GPU scan of configs C2 / C4 at up to 1e9 rows vs
(a) the C oracle in Spark partition order and (b) a near-exact reference, per column and per pair.

SURVEY §7 "hard parts": at 1e9 rows Spark's own sequential fp64 rounding can approach the 1e-12 bar, so
every fp64 result is compared with a double-double reference (~1e-22 relative; oracle/c dqo_exact_*)
and the STRICT relative error |v - exact| / |exact| of both the GPU and the Spark-order oracle is
reported, showing which side carries the error.  Counts and min / max are compared bit-exactly with the
oracle.  The data is generated on the device chunk by chunk (125M rows = 8 GB per C2/C4 chunk), scanned,
copied to the host and folded by the oracle, so host memory holds one chunk at a time.

    python tests/fullscale_parity.py --cfg c2 c4 --rows 1000000000 --out profiles/r2_fullscale_parity.json

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


def _f(dd) -> Fraction:
    return Fraction(dd[0]) + Fraction(dd[1])


def _rel(v: float, exact: Fraction) -> float:
    if math.isnan(v):
        return math.inf
    if exact == 0:
        return abs(v)
    return float(abs(Fraction(v) - exact) / abs(exact))


def _analyzers(dq, cfg, names):
    if cfg == "c2":  # Size + per column Completeness, Mean, StdDev, Min, Max (+ Sum)
        out = [dq.Size()]
        for c in names:
            out += [dq.Completeness(c), dq.Mean(c), dq.StandardDeviation(c), dq.Minimum(c), dq.Maximum(c), dq.Sum(c)]
        return out
    out = [dq.Correlation(names[i], names[j]) for i in range(len(names)) for j in range(i + 1, len(names))]
    return out + [dq.Mean(c) for c in names] + [dq.StandardDeviation(c) for c in names]


def run(cfg: str, rows: int, chunk: int = 125_000_000, parts: int = 16, nthreads: int = 16, seed: int = 42,
        log=print) -> dict:
    import torch

    import deequ_amd as dq
    from deequ_amd import synth
    from deequ_amd.runner import ScanPlan
    from oracle import dq_oracle_c as C

    gen = {"c2": synth.c2_table, "c4": synth.c4_table}[cfg]
    t0 = gen(min(chunk, rows), 0, seed)
    names = list(t0.columns)
    analyzers = _analyzers(dq, cfg, names)
    plan = ScanPlan(analyzers, t0.schema)
    del t0
    col_parts = {c: [] for c in names}
    pair_parts = {}
    pivots = {}
    exact = {c: [0, Fraction(0), Fraction(0)] for c in names}
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
        host = {}
        for c in names:
            col = t.columns[c]
            vals = col.values[: m * 8].cpu().numpy().view(np.float64)
            bm = col.validity.cpu().numpy() if col.validity is not None else None
            host[c] = (vals, bm)
        del t
        torch.cuda.empty_cache()
        c_ = time.perf_counter()
        for c in names:
            vals, bm = host[c]
            col_parts[c] += C.column_stats_partials("f64", vals, bm, parts, nthreads)
        for (x, y) in pairs:
            pair_parts.setdefault((x, y), [])
            pair_parts[(x, y)] += C.corr_partials("f64", host[x][0], host[x][1], "f64", host[y][0], host[y][1], parts,
                                                  nthreads)
        d = time.perf_counter()
        for c in names:
            vals, bm = host[c]
            if c not in pivots:  # pivot: the column's first selected value (any fixed double works)
                valid = np.unpackbits(bm[: 1024], bitorder="little")[: min(m, 8192)].astype(bool) if bm is not None else None
                pivots[c] = float(vals[np.argmax(valid)] if valid is not None else vals[0])
            cnt, s1, s2 = C.exact_moments("f64", vals, bm, pivots[c], nthreads)
            e = exact[c]
            e[0] += cnt
            e[1] += _f(s1)
            e[2] += _f(s2)
        for (x, y) in pairs:
            res = C.exact_comoments("f64", host[x][0], host[x][1], "f64", host[y][0], host[y][1], pivots[x], pivots[y],
                                    nthreads)
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
              "strict_bar": STRICT, "columns": {}, "pairs": {}, "timing": timing}
    worst = {"gpu": 0.0, "oracle": 0.0}
    failures = []
    for c in names:
        o = C.stats_fold("f64", col_parts[c])
        n_e, s1, s2 = exact[c]
        piv = Fraction(pivots[c])
        mean_e = piv + s1 / n_e
        m2_e = s2 - s1 * s1 / n_e
        sum_e = piv * n_e + s1
        sd_e = math.sqrt(float(m2_e / n_e))
        sd_state = states[dq.StandardDeviation(c)]
        mean_state = states[dq.Mean(c)]
        g = {"mean": mean_state.sum_ / mean_state.count, "stddev": sd_state.metricValue(),
             "avg_state": sd_state.avg, "m2_state": sd_state.m2, "sum": mean_state.sum_}
        orc = {"mean": o.sum_f64 / o.count, "stddev": math.sqrt(o.m2 / o.n), "avg_state": o.avg, "m2_state": o.m2,
               "sum": o.sum_f64}
        ex = {"mean": mean_e, "stddev": Fraction(sd_e), "avg_state": mean_e, "m2_state": m2_e, "sum": sum_e}
        rec = {"n": n_e, "exact": {k_: float(v) for k_, v in ex.items()}, "gpu_rel_err": {}, "oracle_rel_err": {}}
        if sd_state.n != o.n or mean_state.count != o.count or sd_state.n != n_e:
            failures.append(f"{c}: count gpu {sd_state.n} oracle {o.n} exact {n_e}")
        for key in ex:
            ge, oe = _rel(g[key], ex[key]), _rel(orc[key], ex[key])
            rec["gpu_rel_err"][key], rec["oracle_rel_err"][key] = ge, oe
            worst["gpu"] = max(worst["gpu"], ge)
            worst["oracle"] = max(worst["oracle"], oe)
            if ge > max(STRICT, oe):
                failures.append(f"{c}.{key}: gpu strict rel err {ge:.3g} > max(1e-12, oracle {oe:.3g})")
        if cfg == "c2":
            for an, want in ((dq.Minimum(c), o.min), (dq.Maximum(c), o.max)):
                got = states[an].metricValue()
                if got != want:
                    failures.append(f"{an}: gpu {got!r} != oracle {want!r}")
            comp = states[dq.Completeness(c)]
            if comp.numMatches != o.count or comp.count != rows:
                failures.append(f"Completeness({c}): {comp} vs oracle count {o.count}")
        report["columns"][c] = rec
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
        rec = {"n": n_e, "exact": {k_: float(v) for k_, v in ex.items()}, "gpu_rel_err": {}, "oracle_rel_err": {}}
        if st.n != o[0] or st.n != n_e:
            failures.append(f"corr({x},{y}) n: gpu {st.n} oracle {o[0]} exact {n_e}")
        for key in ex:
            ge, oe = _rel(g[key], ex[key]), _rel(orc[key], ex[key])
            rec["gpu_rel_err"][key], rec["oracle_rel_err"][key] = ge, oe
            worst["gpu"] = max(worst["gpu"], ge)
            worst["oracle"] = max(worst["oracle"], oe)
            if ge > max(STRICT, oe):
                failures.append(f"corr({x},{y}).{key}: gpu strict rel err {ge:.3g} > max(1e-12, oracle {oe:.3g})")
        report["pairs"][f"{x},{y}"] = rec
    report["worst_strict_rel_err"] = worst
    report["gpu_within_1e-12_strict"] = worst["gpu"] <= STRICT
    report["failures"] = failures
    report["ok"] = not failures
    return report


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", nargs="+", default=["c2", "c4"])
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
                          "failures": rep["failures"][:10]}), flush=True)
        reports.append(rep)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(reports, f, indent=1)
    sys.exit(0 if all(r["ok"] for r in reports) else 1)


if __name__ == "__main__":
    main()
