"""Benchmark: fused 16-column profile scan (BASELINE.json metric).

Per GPU: ROWS rows (default 1e9) x 16 columns (8 fp64 + 4 int64 + 4 UTF8, 10 % nulls, synthetic,
generated on the device), held in HBM as CHUNK-row chunks (UTF8 int32 offsets < 2 GiB per chunk).
One step = one fused scan of every chunk with the ColumnProfiler pass-1/2 analyzer set
(Size, Completeness x16, ApproxCountDistinct x16, Min/Max/Mean/StdDev/Sum x12), dq_finish, and for
N > 1 the RCCL allgather of the per-rank state blobs + fixed-order merge.  Rows shard across ranks
(weak scaling).  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md (HBM3E peak 8.0 TB/s)
# FETCH_SIZE summary of this round's kernels (tools/profile_round.sh -> tools/summarize_prof.py):
# per-dispatch HBM read bytes of each kernel at the default 125 M-row chunk, gfx950-corrected
PMC_FILE = os.path.join(ROOT, "profiles", "r1f_pmc.json")
DEFAULT_CHUNK = 125_000_000  # 8 chunks per 1e9 rows; a UTF8 chunk's bytes (~2.0e9) stay < 2 GiB


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--rows", type=int, default=1_000_000_000, help="rows per GPU")
    p.add_argument("--chunk", type=int, default=DEFAULT_CHUNK, help="rows per chunk")
    p.add_argument("--cpu-sample", type=int, default=62_500_000, help="rows timed on the CPU baseline (0 = skip)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="repeat the CPU sample for at least this long")
    p.add_argument("--cpu-threads", type=int, default=16)
    return p.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local % max(1, torch.cuda.device_count())))

    import deequ_amd as dq
    from deequ_amd import distributed, synth
    from deequ_amd.runner import ScanPlan

    n_total = args.rows
    chunk = min(args.chunk, n_total)
    row0 = rank * n_total
    chunks = []
    r = 0
    while r < n_total:
        m = min(chunk, n_total - r)
        chunks.append(synth.c5_table(m, row0=row0 + r, seed=42))
        r += m
    torch.cuda.synchronize()
    analyzers = synth.profile_analyzers(chunks[0])
    plan = ScanPlan(analyzers, chunks[0].schema)
    str_bytes = sum(c.data_bytes for t in chunks for c in t.columns.values() if c.dtype in ("utf8", "large_utf8"))
    algo_bytes_per_step = plan.bytes_per_row() * n_total + str_bytes  # each needed buffer once

    def step():
        plan.reset()
        for t in chunks:
            plan.scan(t)
        states = plan.finish()
        if world > 1:
            states = distributed.allgather_combine(states)
        return states

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    plan.enable_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        states = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    from deequ_amd import _lib as L

    per_variant = {}
    for v, name in L.VARIANT_NAMES.items():
        ms, nl = plan.kernel_time(16 + v)
        if nl:
            bpr = plan.variant_bytes_per_row(v)
            data = sum(c.data_bytes for t in chunks for c in t.columns.values()
                       if (v == 10 and c.dtype == "utf8") or (v == 11 and c.dtype == "large_utf8"))
            per_variant[name] = {"launches": nl, "ms_total": ms, "avg_ms": ms / nl,
                                 "bytes_per_launch": (bpr * n_total + data) / len(chunks)}
    for rec in per_variant.values():
        rec["GBps"] = rec["bytes_per_launch"] / (rec["avg_ms"] / 1e3) / 1e9
    col_ms, col_launches = plan.kernel_time(1)
    fin_ms, _ = plan.kernel_time(3)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    rows_all = n_total * world * args.steps
    value = rows_all / elapsed
    # roofline of the dominant kernel (largest total time): algorithmic bytes per launch / avg duration
    dom_name, dom = max(per_variant.items(), key=lambda kv: kv[1]["ms_total"])
    dom_v = {name: v for v, name in L.VARIANT_NAMES.items()}[dom_name]
    achieved = dom["GBps"]
    traffic = pmc_traffic(f"dq::dq_column_scan<{dom_v}>") if chunk == DEFAULT_CHUNK else None
    out = {
        "metric": "rows/sec (whole node) for fused 16-col profile scan; % of HBM peak BW",
        "value": value,
        "unit": "rows/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64+int64+utf8",
        "data": "synthetic (device-generated, seeded; SURVEY 8d C5 distributions)",
        "config": {"workload": "C5 fused 16-col profile scan (8 f64 + 4 i64 + 4 utf8, 10% nulls)",
                   "rows_per_gpu": n_total, "chunk_rows": chunk, "analyzers": len(analyzers),
                   "parallelism": f"row-shard x{world}"},
        "hbm_frac_of_step": (algo_bytes_per_step / (elapsed / args.steps)) / 1e9 / HBM_PEAK_GBS,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_source": os.path.relpath(PMC_FILE, ROOT) if traffic is not None else None,
                     "kernel": f"dq_column_scan<{dom_name}>", "bytes_per_launch": dom["bytes_per_launch"],
                     "avg_launch_ms": dom["avg_ms"], "launches": dom["launches"],
                     "column_pass_ms_per_step": col_ms / args.steps,
                     "finalize_ms_per_step": fin_ms / args.steps, "per_variant": per_variant},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        out["cpu_baseline"] = cpu_baseline(chunks[0], min(args.cpu_sample, chunks[0].num_rows), args.cpu_threads,
                                           args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    plan.close()
    if world > 1:
        dist.destroy_process_group()


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed FETCH_SIZE pass (None if not profiled)."""
    try:
        with open(PMC_FILE) as f:
            recs = json.load(f)["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    for r in recs:
        if r["kernel"] == kernel:
            return r["hbm_read_bytes_per_call_corrected"]
    return None


def cpu_baseline(table, n, threads, min_seconds=10.0):
    """The C restatement (oracle/, "port") of the same profile scan on the host cores."""
    import numpy as np

    from oracle import dq_oracle_c as C

    cols = []
    for c in table.columns.values():
        bm = c.validity[: (n + 7) // 8 + 16].cpu().numpy() if c.validity is not None else None
        if c.dtype in ("utf8", "large_utf8"):
            w = 4 if c.dtype == "utf8" else 8
            offs = c.offsets[: (n + 1) * w].cpu().numpy().view(np.int32 if w == 4 else np.int64)
            data = c.values[: int(offs[-1]) + 16].cpu().numpy()
            cols.append((c.dtype, data, offs, bm))
        else:
            w = 4 if c.dtype == "i32" else 8
            cols.append((c.dtype, c.values[: n * w].cpu().numpy().view({"f64": np.float64, "i64": np.int64,
                                                                       "i32": np.int32}[c.dtype]), None, bm))
    threads = max(1, min(threads, os.cpu_count() or 1))
    reps = 0
    t0 = time.perf_counter()
    while True:
        C.profile_scan(cols, n, nparts=threads * 4, nthreads=threads)
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= min_seconds:
            break
    return {"value": reps * n / dt, "unit": "rows/s", "cores": threads, "kind": "port",
            "sample": f"{reps} x {n} rows x 16 cols of the same C5 data (first chunk), profile scan in oracle/c "
                      f"(Spark partial/final aggregation order, per-row Welford + XXH64 HLL), {threads} OpenMP "
                      f"threads, {dt:.1f} s"}


if __name__ == "__main__":
    main()
