"""ApproxQuantile(s) on the device: rows/s and HBM rate of dq_approx_quantiles (diagnostic).

Reports rows/s and the column-read-equivalent rate (8 B value + 1/8 B validity per row, i.e. one read of
the column, the least any selection needs); the radix select reads the column 2-3 times (6 digit passes,
the later ones over a compacted candidate list), so the per-pass HBM rate is in the rocprof kernel trace.
    python tools/quantile_bench.py [--rows 1e9] [--reps 5]
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
    from deequ_amd.quantiles import device_quantiles
    from deequ_amd.table import Column

    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1e9)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--int-range", type=int, default=0, help="an i64 column uniform in [0, R) instead of the f64 one")
    a = ap.parse_args()
    n = int(a.rows)
    g = torch.Generator(device="cuda").manual_seed(7)
    if a.int_range:
        vals = torch.randint(0, a.int_range, (n,), device="cuda", dtype=torch.int64, generator=g)
    else:
        vals = torch.randn(n, device="cuda", dtype=torch.float64, generator=g) * 1e3
    valid = torch.randint(0, 256, ((n + 31) // 32 * 4,), device="cuda", dtype=torch.uint8, generator=g)
    valid |= 0xEF  # ~1/8 nulls
    col = Column("x", "i64" if a.int_range else "f64", n, vals.view(torch.uint8), valid, None, nullable=True)
    t = dq.Table([col])
    for qs in ([0.5], [0.25, 0.5, 0.75], [0.01, 0.1, 0.25, 0.5, 0.75, 0.9, 0.99, 0.999]):
        device_quantiles(t, "x", qs, 0.01)  # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            r = device_quantiles(t, "x", qs, 0.01)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.reps * 1e3
        gbs = (8 + 1 / 8) * n / (ms * 1e-3) / 1e9
        print(f"quantiles={len(qs)} rows={n:.3g} ms={ms:.3f} rows/s={n / (ms * 1e-3):.4g} "
              f"column-read-equivalent GB/s={gbs:.0f} first={r[0]:.6g}", flush=True)
    # ApproxQuantileState's digest: every 1 / (2 e) + 2 sample ranks in two passes (bucket counts against sampled
    # splitters, then the flagged buckets' keys compacted and sorted)
    from deequ_amd.quantiles import device_digest

    if n <= (1 << 31) - 1:
        for err in (0.01, 0.001):
            device_digest(t, "x", err)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                d = device_digest(t, "x", err)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / a.reps * 1e3
            print(f"digest relativeError={err} samples={len(d.quantileSummaries.sampled)} rows={n:.3g} ms={ms:.3f} "
                  f"rows/s={n / (ms * 1e-3):.4g}", flush=True)


if __name__ == "__main__":
    main()
