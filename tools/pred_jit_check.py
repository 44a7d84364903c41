"""Diagnostic (GPU): whether the C3 / C1-style predicate programs run as compiled kernels, and why not."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import deequ_amd as dq  # noqa: E402
from deequ_amd import synth  # noqa: E402
from deequ_amd.runner import ScanPlan  # noqa: E402

t = synth.c3_table(1 << 20, 0, 42)
an = [dq.Size()] + [dq.ApproxCountDistinct(c) for c in t.columns]
an += [dq.Compliance("p0", "i0 >= 0"), dq.Compliance("p1", "`i1` IS NULL OR (`i1` >= 10.0 AND `i1` <= 1000.0)"),
       dq.Compliance("p2", "i2 < i3"), dq.Compliance("p3", "COALESCE(i3, 0.0) >= 0")]
t0 = time.perf_counter()
plan = ScanPlan(an, t.schema)
print("plan create s", round(time.perf_counter() - t0, 3), "compiled:", plan.pred_compiled())
