"""Strict fp64 parity at scale (north_star: within 1e-12 relative for mean / stddev / correlation).

The GPU scan of C2 (8 fp64 columns, moments) and C4 (28 correlations + moments) is compared with a
double-double reference; the strict relative error |gpu - exact| / |exact| of every mean, stddev, sum,
StandardDeviation / Correlation state field and correlation must be <= 1e-12, or no larger than the
Spark-order oracle's own error (the reference's CPU path cannot do better).  Counts and min / max are
bit-exact vs the oracle.  tests/fullscale_parity.py runs the same check at 1e9 rows
(profiles/r2_fullscale_parity.json).
"""
from __future__ import annotations

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg,rows,chunk", [("c2", 250_000_000, 62_500_000), ("c4", 100_000_000, 50_000_000)])
def test_strict_fp64_parity_at_scale(cfg, rows, chunk):
    import os

    from tests.fullscale_parity import run

    rep = run(cfg, rows, chunk, parts=8, nthreads=int(os.environ.get("OMP_NUM_THREADS", "16")), log=lambda s: None)
    assert rep["ok"], rep["failures"][:20]
    print(cfg, rep["worst_strict_rel_err"])
