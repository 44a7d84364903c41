"""Grouping analyzers on the device: dq_freq_build (sort-based GROUP BY) + Uniqueness / Entropy at 1e8 rows (diagnostic).

    python tools/group_bench.py [--rows 1e8] [--reps 3]
One i64 column at several cardinalities (device-generated, 10 % nulls) and the four C5 utf8 columns; ms per
build_frequencies and per Uniqueness + Distinctness + Entropy calculation (one shared build).
"""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    assert torch.cuda.is_available()
    import deequ_amd as dq
    from deequ_amd import synth
    from deequ_amd.grouping import build_frequencies
    from deequ_amd.table import Column
    from deequ_amd import _lib as L

    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1e8)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    n = int(a.rows)
    g = torch.Generator(device="cuda").manual_seed(5)
    valid = torch.randint(0, 256, ((n + 31) // 32 * 4,), device="cuda", dtype=torch.uint8, generator=g) | 0xEF

    def timed(label, fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            r = fn()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.reps * 1e3
        print(f"{label} rows={n:.3g} ms={ms:.3f} rows/s={n / (ms * 1e-3):.4g}", flush=True)
        return r

    for card in (1000, 1_000_000, n):
        vals = torch.randint(0, card, (n,), device="cuda", dtype=torch.int64, generator=g)
        t = dq.Table([Column("x", "i64", n, vals.view(torch.uint8), valid, None, nullable=True)])
        st = timed(f"freq_build i64 cardinality={card:.3g}", lambda: build_frequencies(t, ["x"]))
        print(f"   groups={L.lib.dq_freq_num_groups(st.frequencies.handle)}", flush=True)
        an = [dq.Uniqueness(["x"]), dq.Distinctness(["x"]), dq.Entropy("x")]
        timed(f"uniqueness+distinctness+entropy i64 cardinality={card:.3g}",
              lambda: dq.AnalysisRunner.onData(t).addAnalyzers(an).run())
        del vals, t, st
        torch.cuda.empty_cache()
    t5 = synth.c5_table(n, row0=0, seed=42)
    for k, sname in enumerate(c for c, col in t5.columns.items() if col.dtype == "utf8"):
        d = synth.STR_DISTINCT[k]
        st = timed(f"freq_build utf8 ({sname}, C5 strings, drawn from {d:.3g} values)" if d else
                   f"freq_build utf8 ({sname}, C5 strings, unique)", lambda: build_frequencies(t5, [sname]))
        print(f"   groups={L.lib.dq_freq_num_groups(st.frequencies.handle)}", flush=True)
        del st


if __name__ == "__main__":
    main()
