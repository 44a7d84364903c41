"""Parity at scale (north_star: bit-exact integer results, fp64 within 1e-12 relative).

C2 (8 fp64 columns, moments) and C4 (28 correlations + moments): the strict relative error
|gpu - exact| / |exact| against a double-double reference of every mean, stddev, sum, StandardDeviation /
Correlation state field and correlation must be <= 1e-12.  C3 (4 int64 + 4 UTF8: HLL + four Compliance
predicates) and C5 (the 16-column profile): HLL register words and estimates, Compliance / Completeness /
Size counts, int64 min / max and wrapping int64 sums bit-exact vs the oracle, fp64 moments strict as above.
tests/fullscale_parity.py runs the same checks at 1e9 rows (profiles/r3_fullscale_parity.json).
"""
from __future__ import annotations

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg,rows,chunk", [("c2", 250_000_000, 62_500_000), ("c4", 100_000_000, 50_000_000),
                                             ("c3", 250_000_000, 62_500_000), ("c5", 250_000_000, 62_500_000)])
def test_parity_at_scale(cfg, rows, chunk):
    import os

    from tests.fullscale_parity import run

    rep = run(cfg, rows, chunk, parts=8, nthreads=int(os.environ.get("OMP_NUM_THREADS", "16")), log=lambda s: None)
    assert rep["ok"], rep["failures"][:20]
    print(cfg, rep["worst_strict_rel_err"], rep["integer_checks"], rep["rare_path_rows_total"])
