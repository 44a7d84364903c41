"""Kernel sweep (diagnostic, GPU): column-scan time and algorithmic GB/s for analyzer subsets on one
C5 chunk.  Usage: python tools/sweep.py [rows [case-filter]]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import deequ_amd as dq  # noqa: E402
from deequ_amd import synth  # noqa: E402
from deequ_amd.runner import ScanPlan  # noqa: E402


ONLY = sys.argv[2] if len(sys.argv) > 2 else ""  # optional case-name filter


def measure(name, table, analyzers, reps=5):
    if ONLY and ONLY not in name:
        return
    plan = ScanPlan(analyzers, table.schema)
    for _ in range(2):
        plan.reset(); plan.scan(table); plan.finish()
    plan.enable_timing(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        plan.reset(); plan.scan(table); plan.finish()
    wall = (time.perf_counter() - t0) / reps
    res = {}
    for k, kn in enumerate(("pred", "column", "pair", "finalize")):
        ms, nl = plan.kernel_time(k)
        if nl:
            res[kn] = ms / reps
    cols = set()
    for a in analyzers:
        for f in ("column", "firstColumn", "secondColumn"):
            if hasattr(a, f):
                cols.add(getattr(a, f))
    strb = sum(table.columns[c].data_bytes for c in cols if table.columns[c].dtype == "utf8" and
               any(type(a).__name__ in ("ApproxCountDistinct", "PatternMatch") and a.column == c for a in analyzers))
    nbytes = plan.bytes_per_row() * table.num_rows + strb
    main = res.get("column") or res.get("pair") or res.get("pred")
    out = {"case": name, "rows": table.num_rows, "GB": nbytes / 1e9, "kernel_ms": res, "wall_ms": wall * 1e3,
           "GBps_main_kernel": nbytes / (main / 1e3) / 1e9 if main else None}
    print(json.dumps(out), flush=True)
    plan.close()


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 62_500_000
    if not ONLY or not ONLY.startswith("corr"):
        t = synth.c5_table(n, seed=42)
        torch.cuda.synchronize()
        f = [c for c, d, _ in t.schema if d == "f64"]
        i = [c for c, d, _ in t.schema if d == "i64"]
        s = [c for c, d, _ in t.schema if d == "utf8"]
        stats = lambda cs: [A(c) for c in cs for A in (dq.Mean, dq.StandardDeviation, dq.Minimum, dq.Maximum, dq.Sum)]
        measure("completeness16", t, [dq.Completeness(c) for c, _, _ in t.schema])
        measure("f64x1_stats", t, stats(f[:1]))
        measure("f64x1_hll", t, [dq.ApproxCountDistinct(f[0])])
        measure("f64x8_stats", t, stats(f))
        measure("f64x8_hll", t, [dq.ApproxCountDistinct(c) for c in f])
        measure("f64x8_stats_hll", t, stats(f) + [dq.ApproxCountDistinct(c) for c in f])
        measure("i64x4_stats_hll", t, stats(i) + [dq.ApproxCountDistinct(c) for c in i])
        measure("utf8x1_hll", t, [dq.ApproxCountDistinct(s[0])])
        measure("utf8x4_hll", t, [dq.ApproxCountDistinct(c) for c in s])
        measure("profile16", t, synth.profile_analyzers(t))
        measure("compliance4", t, [dq.Compliance("p0", "i0 >= 0"), dq.Compliance("p1", "`i1` IS NULL OR (`i1` >= 10.0 AND `i1` <= 1000.0)"),
                                   dq.Compliance("p2", "i2 < i3"), dq.Compliance("p3", "COALESCE(i3, 0.0) >= 0")])
        measure("pattern_email_utf8x1", t, [dq.PatternMatch(s[0], dq.Patterns.EMAIL)])
        measure("pattern_url_utf8x1", t, [dq.PatternMatch(s[0], dq.Patterns.URL)])
        measure("pattern_email_utf8x4", t, [dq.PatternMatch(c, dq.Patterns.EMAIL) for c in s])
        measure("pattern_digit_utf8x4", t, [dq.PatternMatch(c, r"\d") for c in s])
    if ONLY and ONLY.startswith("group"):
        t = synth.c5_table(n, seed=42)
        from deequ_amd.grouping import build_frequencies
        for name, cols in (("group_i64_1e6", ["i1"]), ("group_i64_unique", ["i3"]), ("group_f64", ["c0"]),
                           ("group_utf8_1e6", ["s1"]), ("group_i64_utf8", ["i0", "s0"])):
            for _ in range(2):
                build_frequencies(t, cols)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            reps = 3
            for _ in range(reps):
                st = build_frequencies(t, cols)
                st.frequencies.summary(st.numRows)
            ms = (time.perf_counter() - t0) / reps * 1e3
            s = st.frequencies.summary(st.numRows)
            print(json.dumps({"case": name, "rows": n, "wall_ms": ms, "groups": s.num_groups,
                              "rows_per_s": n / ms * 1e3}), flush=True)
        return
    c4 = synth.c4_table(n // 2, seed=42)
    names = list(c4.columns)
    measure("corr28_half", c4, [dq.Correlation(names[a], names[b]) for a in range(8) for b in range(a + 1, 8)])


if __name__ == "__main__":
    main()
