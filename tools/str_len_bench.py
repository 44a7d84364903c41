"""String-length sweep of the UTF8 column passes (diagnostic): 4 UTF8 columns of N rows (10 % nulls) with lengths
uniform in [lmin, lmax], ApproxCountDistinct (and + DataType: the ColumnProfiler's string pair) per column; prints
the average launch of each column-pass variant per 1e8 rows and the rows/s of the scan.

usage: python tools/str_len_bench.py [--rows N] [--bands 8:24,16:48,32:64,64:128] [--steps K]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=25_000_000)
    ap.add_argument("--bands", default="8:24,16:48,24:40,32:64,64:128")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--dtype", action="store_true", help="also DataType per column (UTF8_HD variant)")
    ap.add_argument("--path", choices=["auto", "fast", "long"], default="auto",
                    help="DQ_STR_PATH: the string pass's instantiation (auto: dq_scan's choice)")
    args = ap.parse_args()
    if args.path != "auto":
        os.environ["DQ_STR_PATH"] = args.path
    import torch

    from deequ_amd import synth
    from deequ_amd.analyzers import ApproxCountDistinct, DataType
    from deequ_amd.runner import ScanPlan
    from deequ_amd.table import Table

    out = []
    for band in args.bands.split(","):
        lmin, lmax = (int(x) for x in band.split(":"))
        cols = [synth.utf8_column(f"s{c}", args.rows, 1000 + c, 50_000_000, lmin, lmax, 0.10) for c in range(4)]
        t = Table(cols)
        torch.cuda.synchronize()
        an = [ApproxCountDistinct(f"s{c}") for c in range(4)]
        if args.dtype:
            an += [DataType(f"s{c}") for c in range(4)]
        plan = ScanPlan(an, t.schema)
        plan.enable_timing(True)
        plan.reset(); plan.scan(t); plan.finish()  # warm-up
        plan.enable_timing(True)
        torch.cuda.synchronize()
        a = time.perf_counter()
        for _ in range(args.steps):
            plan.reset()
            plan.scan(t)
            plan.finish()
        torch.cuda.synchronize()
        sec = (time.perf_counter() - a) / args.steps
        ker = {}
        for v in range(0, 32):
            try:
                ms, n = plan.kernel_time(16 + v)
            except Exception:  # past the last variant
                break
            if n:
                ker[v] = round(ms / n * 1e8 / args.rows, 4)
        nbytes = sum(c.data_bytes for c in cols)
        rec = {"band": band, "path": args.path, "rows": args.rows, "ms_per_scan": round(sec * 1e3, 3), "rows_per_s": args.rows / sec,
               "string_GBps": nbytes / sec / 1e9, "variant_ms_per_1e8_rows": ker}
        print(json.dumps(rec), flush=True)
        out.append(rec)
        plan.close()
        del cols, t
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
