"""Predicate-pass sweep (diagnostic, GPU): time of dq_pred_scan for predicate sets of growing size
on one C5 chunk.  Usage: python tools/pred_sweep.py [rows]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import deequ_amd as dq  # noqa: E402
from deequ_amd import synth  # noqa: E402
from deequ_amd.runner import ScanPlan  # noqa: E402


def measure(name, t, analyzers, reps=5):
    plan = ScanPlan(analyzers, t.schema)
    for _ in range(2):
        plan.reset(); plan.scan(t); plan.finish()
    plan.enable_timing(True)
    for _ in range(reps):
        plan.reset(); plan.scan(t); plan.finish()
    ms, nl = plan.kernel_time(0)
    print(json.dumps({"case": name, "pred_ms": ms / reps, "bytes_per_row": plan.bytes_per_row(),
                      "GBps": plan.bytes_per_row() * t.num_rows / (ms / reps * 1e-3) / 1e9}), flush=True)
    plan.close()


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 62_500_000
    t = synth.c5_table(n, seed=42)
    torch.cuda.synchronize()
    C = dq.Compliance
    measure("1cmp_i64", t, [C("p0", "i0 >= 0")])
    measure("1cmp_f64", t, [C("p0", "c0 >= 0")])
    measure("1isnull", t, [C("p0", "i0 IS NULL")])
    measure("2cmp_2cols", t, [C("p0", "i0 >= 0"), C("p1", "i1 >= 0")])
    measure("4cmp_4cols", t, [C("p%d" % k, "i%d >= 0" % k) for k in range(4)])
    measure("range_i1", t, [C("p1", "`i1` IS NULL OR (`i1` >= 10.0 AND `i1` <= 1000.0)")])
    measure("colcol", t, [C("p2", "i2 < i3")])
    measure("c3_4preds", t, [C("p0", "i0 >= 0"), C("p1", "`i1` IS NULL OR (`i1` >= 10.0 AND `i1` <= 1000.0)"),
                             C("p2", "i2 < i3"), C("p3", "COALESCE(i3, 0.0) >= 0")])


if __name__ == "__main__":
    main()
