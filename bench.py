"""Benchmark: fused 16-column profile scan (BASELINE.json metric).

Per GPU: ROWS rows (default 1e9) x 16 columns (8 fp64 + 4 int64 + 4 UTF8, 10 % nulls, synthetic,
generated on the device), held in HBM as CHUNK-row chunks (UTF8 int32 offsets < 2 GiB per chunk).
One step = one fused scan of every chunk with the ColumnProfiler pass-1/2 analyzer set
(Size, Completeness x16, ApproxCountDistinct x16, Min/Max/Mean/StdDev/Sum x12), dq_finish, for N > 1 the
RCCL all-gather of the per-rank state slot sets + fixed rank-order merge, and the incremental StateLoader
append of C5 (the previous run's states merged in and persisted, Analyzer.scala:107-128).  Rows shard
across ranks (weak scaling).  Prints ONE JSON line on rank 0.

`--gpus N` with N > 1 and no RANK in the environment re-launches this script as N ranks
(torch.distributed.run, one process per GPU) before anything touches the GPU.

At N = 1 the line also carries the other BASELINE configs measured on this GPU ("configs": C1 Item table,
C2 moments, C3 HLL + Compliance, C4 correlations + moments, each at its BASELINE size) and the CPU
baselines (the oracle's C restatement on this host's CPU share).
"""
from __future__ import annotations

import argparse
import gc
import json
import re
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md (HBM3E peak 8.0 TB/s)
# FETCH_SIZE summary of this round's kernels (tools/profile_round.sh -> tools/summarize_prof.py):
# per-dispatch HBM read bytes of each kernel at the default 125 M-row chunk, gfx950-corrected
PMC_FILE = os.path.join(ROOT, "profiles", "r6u2_pmc.json")
# tools/clock_probe.sh: held clock per kernel, one file per probe box (boxes hold 1.87-1.98 GHz under the same
# kernels); the floor at the held clock takes the highest clock any probe saw (the conservative floor)
CLOCK_FILES = [os.path.join(ROOT, "profiles", f) for f in ("r3_clock.json", "r3z_clock.json", "r4z_clock.json",
                                                         "r4z_cfg_clock.json", "r5l_clock.json", "r5p_clock.json",
                                                         "r5x_clock.json", "r5fin_clock.json",
                                                         "r5fin3_clock.json", "r5fin5_clock.json",
                                                         "r6p_clock.json", "r6f_clock.json", "r6y_clock.json",
                                                         "r6q2_clock.json", "r6s2_clock.json",
                                                         "r6t2_clock.json", "r6u2_clock.json")]
DEFAULT_CHUNK = 125_000_000  # 8 chunks per 1e9 rows; a UTF8 chunk's bytes (~2.0e9) stay < 2 GiB


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--rows", type=int, default=1_000_000_000, help="rows per GPU")
    p.add_argument("--chunk", type=int, default=DEFAULT_CHUNK, help="rows per chunk")
    p.add_argument("--cpu-sample", type=int, default=62_500_000, help="rows timed on the CPU baseline (0 = skip)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="repeat the CPU sample for at least this long")
    p.add_argument("--cpu-threads", type=int, default=0, help="0 = this host's CPU share (see host_cpu_share)")
    p.add_argument("--configs", default="c1,c2,c3,c4,c5e,types",
                   help="other configs to measure at N=1 ('' = none): BASELINE C1-C4, c5e = C5 with empty NULL string "
                        "slots (Spark / Arrow writers), types = the round-6 column types")
    p.add_argument("--config-steps", type=int, default=5)
    p.add_argument("--config-rows", type=int, default=0, help="rows of C2-C4 (0 = BASELINE's 1e9; profiling runs)")
    p.add_argument("--skip-headline", action="store_true", help="profiling runs: only the --configs")
    p.add_argument("--ingest-rows", type=int, default=62_500_000,
                   help="rows of the host-resident Arrow C5 batch for the ingestion leg (0 = skip)")
    p.add_argument("--ingest-reps", type=int, default=4, help="uploads + scans of that batch timed end to end")
    p.add_argument("--no-plan-timing", dest="plan_timing", action="store_false",
                   help="skip the fresh-process plan-creation timing (C3 / C5, cold and warm JIT cache)")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="process group for N > 1 (nccl = RCCL over xGMI; gloo: launcher tests with ranks sharing a GPU)")
    return p.parse_args(argv)


def launch_ranks(args) -> int:
    """N fresh processes (one per GPU) through torch.distributed.run; the parent never touches the GPU."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# plan creation of C3 (whose predicate program becomes a kernel compiled with hipRTC) and C5 (no predicates), in a
# fresh process: dq_plan_create's host time and its JIT part, for a first and a second plan of the process
_PLAN_PROBE = r"""
import json, sys, time
sys.path.insert(0, %r)
import torch
from deequ_amd import synth
from deequ_amd.runner import ScanPlan
torch.cuda.set_device(0)
out = {}
for cfg, tab, an in (("c3", synth.c3_table, synth.c3_analyzers), ("c5", synth.c5_table, synth.profile_analyzers)):
    t = tab(4096, seed=1)
    torch.cuda.synchronize()
    rec = {}
    for k in ("first", "second"):
        a = time.perf_counter()
        plan = ScanPlan(an(t), t.schema)
        wall = (time.perf_counter() - a) * 1e3
        total, jit = plan.create_time()
        plan.pred_wait()
        ready = (time.perf_counter() - a) * 1e3
        rec[k] = {"wall_ms": round(wall, 3), "dq_plan_create_ms": round(total, 3), "pred_jit_ms": round(jit, 3),
                  "pred_kernel_ready_ms": round(ready, 3),
                  "pred_kernel": plan.pred_compiled()[1] if plan.pred_compiled()[0] else None}
        plan.close()
    out[cfg] = rec
print(json.dumps(out))
"""


def plan_create_timing() -> dict:
    """Plan-creation cost (deequ builds one plan per run, AnalysisRunner.scala:279-326): C3 / C5 plans created in
    fresh processes, first with an empty code-object cache (the predicate kernel compiled by hipRTC), then with
    the cache that run filled (loaded from disk); in each process a second plan hits the process cache.  Runs
    before this process touches the GPU."""
    import tempfile

    out = {}
    with tempfile.TemporaryDirectory(prefix="dq_jit_") as d:
        env = dict(os.environ, DQ_JIT_CACHE_DIR=d)
        for label in ("cold_cache", "warm_disk_cache"):
            try:
                r = subprocess.run([sys.executable, "-c", _PLAN_PROBE % ROOT], env=env, capture_output=True, text=True,
                                   timeout=300)
                out[label] = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else {
                    "error": r.stderr[-500:]}
            except (subprocess.TimeoutExpired, ValueError, IndexError) as e:
                out[label] = {"error": str(e)}
    return out


def host_cpu_share() -> tuple:
    """(threads, description): the CPUs this process may use -- affinity, the cgroup CPU quota and the
    pool's OMP_NUM_THREADS (the per-GPU CPU share on the GPU boxes) -- whichever is smallest."""
    aff = len(os.sched_getaffinity(0))
    n = aff
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
            n = min(n, quota)
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return n, f"affinity {aff} CPUs (os.cpu_count() {os.cpu_count()}), cgroup quota {quota}, OMP_NUM_THREADS {omp}"


def main():
    args = parse()
    if args.gpus > 1 and "RANK" not in os.environ:
        sys.exit(launch_ranks(args))
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} disagrees with WORLD_SIZE={world_env}")
    rank = int(os.environ.get("RANK", "0"))
    plan_ms = (plan_create_timing() if (rank == 0 and world_env == 1 and args.plan_timing and not args.skip_headline)
               else None)
    import torch
    import torch.distributed as dist

    world = world_env
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local % max(1, torch.cuda.device_count())))
        else:
            dist.init_process_group("gloo")

    from deequ_amd import _lib as L
    from deequ_amd import distributed, synth
    from deequ_amd.runner import ScanPlan

    if args.skip_headline:
        deferred_cpu = []
        out = {"configs": {cfg: run_config(cfg, args, deferred_cpu) for cfg in re.split(r"[,+]", args.configs) if cfg}}
        for run in deferred_cpu:
            run()
        print(json.dumps(out), flush=True)
        return
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
    persisted = [None]  # the StateLoader / StatePersister of C5's incremental append (in memory)
    host_ms = {"merge": 0.0, "append": 0.0}

    def step():
        plan.reset()
        for t in chunks:
            plan.scan(t)
        states = plan.finish()
        if world > 1:
            a = time.perf_counter()
            states = distributed.allgather_combine(states)
            host_ms["merge"] += (time.perf_counter() - a) * 1e3
        a = time.perf_counter()
        if persisted[0] is not None:  # load -> Analyzers.merge(state, loaded) -> persist
            states = distributed.merge_loaded(states, persisted[0])
        persisted[0] = states
        host_ms["append"] += (time.perf_counter() - a) * 1e3
        return states

    # timing on for the warm-up too, so its hipEvent pool is filled outside the timed region (events are created
    # only when the pool is empty); enabling again below zeroes the counters and keeps the pool
    # the collector runs (and is then switched off, as timeit does) before the warm-up, not between it and
    # the timed steps: a ~50 ms idle GPU there drops its clocks and the first timed step ran ~7 % slower
    plan.enable_timing(True)
    gc.collect()
    gc.disable()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    plan.enable_timing(True)
    host_ms.update(merge=0.0, append=0.0)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    gc.enable()
    kernels = kernel_report(plan, chunks, n_total)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    rows_all = n_total * world * args.steps
    value = rows_all / elapsed
    dom_name, dom = max(((k, v) for k, v in kernels.items() if k.startswith("dq_column_scan")),
                        key=lambda kv: kv[1]["ms_total"])
    traffic = pmc_traffic(dom["pmc_name"]) if chunk == DEFAULT_CHUNK else None
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
        "config": {"workload": "C5 fused 16-col profile scan (8 f64 + 4 i64 + 4 utf8, 10% nulls) + state merge "
                               "+ incremental StateLoader append",
                   "rows_per_gpu": n_total, "chunk_rows": chunk, "analyzers": len(analyzers),
                   "parallelism": f"row-shard x{world}",
                   "collective": (f"{args.dist_backend} all-gather of the state slot sets" if world > 1 else None)},
        "hbm_frac_of_step": (algo_bytes_per_step / (elapsed / args.steps)) / 1e9 / HBM_PEAK_GBS,
        "rank_merge_ms_per_step": host_ms["merge"] / args.steps if world > 1 else 0.0,
        "append_ms_per_step": host_ms["append"] / args.steps,
        "roofline": roofline(dom_name, dom, traffic, kernels),
        "cpu_baseline": None,
        "plan_create_ms": plan_ms,
    }
    if rank == 0 and world == 1:
        out["state_io"] = state_io_timing(analyzers, persisted[0])
    # the CPU baselines run after every GPU measurement (their host copies are taken now): OpenMP's worker
    # threads outlive a parallel region, and config steps timed after one showed 39-64 ms outliers among
    # 22.5 ms C3 steps (none with the baseline off or run last)
    deferred_cpu = []
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        n_cpu = min(args.cpu_sample, chunks[0].num_rows)
        cols_cpu = _host_cols(chunks[0], n_cpu)
        deferred_cpu.append(lambda: out.__setitem__("cpu_baseline", cpu_baseline(cols_cpu, n_cpu, args.cpu_threads,
                                                                                 args.cpu_seconds)))
    plan.close()
    del chunks
    torch.cuda.empty_cache()
    if rank == 0 and world == 1 and args.ingest_rows > 0:
        out["ingest"] = ingest_timing(args, analyzers)
        torch.cuda.empty_cache()
    if world == 1 and args.configs:
        out["configs"] = {}
        for cfg in [c for c in re.split(r"[,+]", args.configs) if c]:
            out["configs"][cfg] = run_config(cfg, args, deferred_cpu)
            torch.cuda.empty_cache()
    for run in deferred_cpu:
        run()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def kernel_report(plan, chunks, n_total) -> dict:
    """Per-kernel launches, average hipEvent duration and algorithmic bytes per launch (plan timing)."""
    from deequ_amd import _lib as L

    nch = len(chunks)
    out = {}
    pred_name = "dq_pred_jit" if plan.pred_compiled()[0] else "dq_pred_scan"  # the compiled kernel or the interpreter
    ids = [(0, pred_name), (2, "dq_pair_scan")] + [(16 + v, f"dq_column_scan<{nm}>") for v, nm in L.VARIANT_NAMES.items()]
    for kid, name in ids:
        ms, nl = plan.kernel_time(kid)
        if not nl:
            continue
        bpr = plan.kernel_bytes_per_row(kid)
        data = 0
        if kid >= 16:
            v = kid - 16
            data = sum(c.data_bytes for t in chunks for c in t.columns.values()
                       if (v in (10, 13) and c.dtype == "utf8") or (v in (11, 15) and c.dtype == "large_utf8"))
        per_launch = (bpr * n_total + data) / nch
        rec = {"launches": nl, "ms_total": ms, "avg_ms": ms / nl, "bytes_per_launch": per_launch,
               "GBps": per_launch / (ms / nl / 1e3) / 1e9,
               "pmc_name": f"dq::dq_column_scan<{kid - 16}>" if kid >= 16 else name}
        out[name] = rec
    fin_ms, fin_n = plan.kernel_time(3)
    if fin_n:
        out["dq_finalize"] = {"launches": fin_n, "ms_total": fin_ms, "avg_ms": fin_ms / fin_n, "bytes_per_launch": 0,
                              "GBps": 0.0, "pmc_name": "dq::dq_finalize"}
    return out


def config_setup(cfg, n, chunk):
    """(chunk tables, analyzers, description) of a BASELINE config."""
    import deequ_amd as dq
    from deequ_amd import synth

    gen = {"c1": synth.item_table, "c2": synth.c2_table, "c3": synth.c3_table, "c4": synth.c4_table,
           "c5e": lambda m, r, s: synth.c5_table(m, r, s, null_empty=True), "types": synth.types_table}[cfg]
    tables = []
    r = 0
    while r < n:
        m = min(chunk, n - r)
        tables.append(gen(m, r, 42))
        r += m
    names = list(tables[0].columns)
    if cfg == "c1":
        analyzers = synth.item_checks().requiredAnalyzers()
        desc = "C1 Item table (examples/entities.scala:19-25): Size, isComplete x5, Mean/StdDev/Min/Max on id, numViews"
    elif cfg == "c2":
        analyzers = [dq.Size()] + [a for c in names for a in (dq.Completeness(c), dq.Mean(c), dq.StandardDeviation(c),
                                                              dq.Minimum(c), dq.Maximum(c))]
        desc = "C2 8 x f64 (10% nulls): Size + Completeness/Mean/StdDev/Min/Max per column"
    elif cfg == "c3":
        analyzers = synth.c3_analyzers(tables[0])
        desc = "C3 4 x i64 + 4 x utf8 (10% nulls): Size + ApproxCountDistinct x8 + Compliance x4"
    elif cfg == "c5e":
        analyzers = synth.profile_analyzers(tables[0])
        desc = ("C5 with empty NULL string slots (Spark / Arrow writers emit no bytes for a NULL): the headline's "
                "columns and 93 analyzers, string payload of non-NULL rows only")
    elif cfg == "types":
        analyzers = synth.profile_analyzers(tables[0]) + [dq.DataType(c) for c in names]
        desc = ("round-6 column types (f32, i16, i8, bool, date32, timestamp, decimal(18,2), decimal(38,18); 10% nulls): "
                "Size + Completeness + "
                "ApproxCountDistinct + DataType per column, Min/Max/Mean/StdDev/Sum of the numeric ones")
    else:
        analyzers = [dq.Correlation(names[i], names[j]) for i in range(8) for j in range(i + 1, 8)]
        analyzers += [dq.Mean(c) for c in names] + [dq.StandardDeviation(c) for c in names]
        desc = "C4 8 x f64 correlated (10% nulls): 28 Correlations + Mean/StdDev per column"
    return tables, analyzers, desc


def run_config(cfg, args, deferred_cpu) -> dict:
    """One BASELINE config at its size on this GPU: rows/s, per-kernel roofline, HBM fraction of the step.
    Its CPU baseline (C1), if any, is appended to `deferred_cpu` and run after every GPU measurement."""
    import torch

    from deequ_amd.runner import ScanPlan

    n = 10_000_000 if cfg == "c1" else (args.config_rows or 1_000_000_000)
    tables, analyzers, desc = config_setup(cfg, n, DEFAULT_CHUNK)
    torch.cuda.synchronize()
    plan = ScanPlan(analyzers, tables[0].schema)
    # the steady state: a predicate kernel compiling in the background (AUTO) is waited for before the warm-up
    a = time.perf_counter()
    pred_compiled = plan.pred_wait()
    pred_wait_ms = (time.perf_counter() - a) * 1e3
    str_bytes = sum(c.data_bytes for t in tables for c in t.columns.values() if c.dtype in ("utf8", "large_utf8"))

    def step():
        plan.reset()
        for t in tables:
            plan.scan(t)
        return plan.finish()

    plan.enable_timing(True)  # warm-up steps fill the hipEvent pool (see main)
    gc.collect()
    gc.disable()
    for _ in range(2):  # kernels right after table generation / an idle GPU run ~7 % slower (clock ramp, C3 trace)
        step()
    torch.cuda.synchronize()
    plan.enable_timing(True)
    k = max(1, args.config_steps)
    step_ms = []
    t0 = time.perf_counter()
    for _ in range(k):
        a = time.perf_counter()
        step()  # finish() synchronizes the plan stream
        step_ms.append((time.perf_counter() - a) * 1e3)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / k
    gc.enable()
    kernels = kernel_report(plan, tables, n)
    # C1's string columns are read for Completeness only (validity bytes): exclude their payload
    algo = plan.bytes_per_row() * n + (str_bytes if cfg in ("c3", "c5e") else 0)
    dom_name, dom = max(kernels.items(), key=lambda kv: kv[1]["ms_total"])
    rec = {"workload": desc, "rows": n, "analyzers": len(analyzers), "ms_per_step": dt * 1e3, "rows_per_s": n / dt,
           "step_ms": [round(x, 3) for x in step_ms], "ms_per_step_median": sorted(step_ms)[len(step_ms) // 2],
           "hbm_frac_of_step": algo / dt / 1e9 / HBM_PEAK_GBS,
           "roofline": {"kernel": dom_name, "achieved": dom["GBps"], "frac": dom["GBps"] / HBM_PEAK_GBS,
                        "avg_launch_ms": dom["avg_ms"], "bytes_per_launch": dom["bytes_per_launch"]},
           "kernels": {k_: {kk: v[kk] for kk in ("launches", "avg_ms", "GBps")} for k_, v in kernels.items()}}
    if plan.pred_compiled()[1] != "no predicates":
        rec["pred_pass"] = {"compiled": pred_compiled, "note": plan.pred_compiled()[1],
                            "waited_ms_before_warmup": round(pred_wait_ms, 3)}
    if cfg == "c1" and args.cpu_sample > 0:
        data_c1 = c1_host_data(tables[0])
        deferred_cpu.append(lambda: rec.__setitem__("cpu_baseline", cpu_baseline_c1(data_c1, args.cpu_threads,
                                                                                    min(args.cpu_seconds, 5.0))))
    plan.close()
    del tables
    return rec


def _sha256(path):
    import hashlib

    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


_PMC_CACHE = {}


def pmc_file():
    """The committed PMC summary (FETCH_SIZE + SQ passes, tools/profile_round.sh) -- used only when it was taken
    from THIS library build (its recorded libdqscan.so sha256 equals the loaded library's), so a stale file
    cannot feed the line."""
    if "d" not in _PMC_CACHE:
        from deequ_amd import _lib as L

        d = None
        try:
            with open(PMC_FILE) as f:
                d = json.load(f)
            if d.get("library_sha256") != _sha256(L.LIB_PATH):
                d = None
        except (OSError, ValueError):
            d = None
        _PMC_CACHE["d"] = d
    return _PMC_CACHE["d"]


def _kname(name):
    """A kernel name without the string variants' second template argument (dq_column_scan<10, false> is the
    common instantiation the bench's short strings run; round-5 profiles name it so)."""
    return re.sub(r", (false|true)>", lambda m: ">" if m.group(1) == "false" else ", true>", name)


def pmc_record(kernel):
    """The PMC pass record of `kernel` (FETCH_SIZE bytes, SQ instruction counts per launch), or None."""
    d = pmc_file()
    for r in (d or {}).get("kernels", []):
        if _kname(r["kernel"]) == kernel:
            return r
    return None


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed FETCH_SIZE pass (None if not profiled)."""
    r = pmc_record(kernel)
    return r["hbm_read_bytes_per_call_corrected"] if r else None


# VALU issue model of the HLL kernels (tools/micro/valu_rate_probe.hip, round-1 tools/rates.hip): one wave64
# integer VALU instruction per 4 SIMD cycles, 1024 SIMDs at 2.4 GHz
VALU_CYCLES_PER_WAVE_INST = 4.0


def valu_bound(kernel, avg_ms):
    """VALU issue floor of `kernel` from the committed SQ pass: wave-instructions per launch x 4 cycles
    / (1024 SIMDs x 2.4 GHz), and the fraction of the measured launch it accounts for."""
    r = pmc_record(kernel)
    if not r or "SQ_INSTS_VALU_per_call" not in r:
        return None
    insts = r["SQ_INSTS_VALU_per_call"]
    floor_ms = insts * VALU_CYCLES_PER_WAVE_INST / (1024 * 2.4e9) * 1e3
    out = {"valu_insts_per_launch": insts, "issue_floor_ms": floor_ms, "frac_of_launch": floor_ms / avg_ms,
           "model": "4 SIMD cycles per wave64 VALU instruction, 1024 SIMDs x 2.4 GHz (nominal peak clock)",
           "source": os.path.relpath(PMC_FILE, ROOT), "pmc_commit": pmc_file().get("commit"),
           "pmc_library_sha256": pmc_file().get("library_sha256")}
    # the clock the chip holds under this kernel (GRBM_GUI_ACTIVE / 8 XCDs / duration, committed probe): the
    # issue floor at that clock is what the launch can reach with its instruction count
    clocks = {}
    for path in CLOCK_FILES:
        try:
            with open(path) as f:
                clk = {_kname(k): v for k, v in json.load(f).items()}.get("void " + kernel)
        except (OSError, ValueError):
            clk = None
        if clk:
            clocks[os.path.relpath(path, ROOT)] = clk["effective_clock_GHz"]
    if clocks:
        ghz = max(clocks.values())
        held_ms = insts * VALU_CYCLES_PER_WAVE_INST / (1024 * ghz * 1e9) * 1e3
        out.update(held_clock_GHz=ghz, issue_floor_ms_at_held_clock=held_ms, frac_at_held_clock=held_ms / avg_ms,
                   held_clock_by_probe=clocks)
    return out


def roofline(dom_name, dom, traffic, kernels) -> dict:
    """The dominant kernel against the HBM roofline: `achieved` = its algorithmic bytes per launch
    (§8d per-row bytes x the rows of one launch + its UTF8 payload) / its hipEvent-timed average launch, `frac`
    = achieved / 8 TB/s.  The HLL kernels are limited by VALU issue before HBM: `valu_issue` gives that floor
    (wave64 VALU instructions of the committed SQ pass of the same library build x 4 cycles / 1024 SIMDs, at the
    nominal 2.4 GHz and at the clock the chip held) and the fraction of the launch it accounts for."""
    valu = valu_bound(dom["pmc_name"], dom["avg_ms"])
    out = {"kernel": dom_name, "bound": "hbm", "achieved": dom["GBps"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": dom["GBps"] / HBM_PEAK_GBS, "traffic": traffic,
           "traffic_source": os.path.relpath(PMC_FILE, ROOT) if traffic is not None else None,
           "bytes_per_launch": dom["bytes_per_launch"], "avg_launch_ms": dom["avg_ms"], "launches": dom["launches"],
           "hbm_floor_ms": dom["bytes_per_launch"] / (HBM_PEAK_GBS * 1e9) * 1e3, "valu_issue": valu,
           "limiter": ("valu_issue" if valu is not None and valu.get("frac_at_held_clock", valu["frac_of_launch"]) >
                       dom["GBps"] / HBM_PEAK_GBS else "hbm")}
    out["kernels"] = kernels
    return out


def state_io_timing(analyzers, states) -> dict:
    """HdfsStateProvider round trip of the C5 state set (binary big-endian files): persist + load ms."""
    import tempfile

    from deequ_amd import HdfsStateProvider

    with tempfile.TemporaryDirectory() as d:
        prov = HdfsStateProvider(os.path.join(d, "c5"), allowOverwrite=True)
        objs = [(a, a._from_result(s)) for a, s in zip(analyzers, states)]
        t0 = time.perf_counter()
        for a, s in objs:
            if s is not None:
                prov.persist(a, s)
        t1 = time.perf_counter()
        for a, _ in objs:
            prov.load(a)
        t2 = time.perf_counter()
    return {"persist_ms": (t1 - t0) * 1e3, "load_ms": (t2 - t1) * 1e3, "states": len(objs)}


def _host_cols(table, n):
    import numpy as np

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
    return cols


def _arrow_batch(table, n):
    """The device table's columns as a host-resident pyarrow RecordBatch (zero-copy over numpy buffers)."""
    import numpy as np
    import pyarrow as pa

    arrays, names = [], []
    for name, c in table.columns.items():
        bm = c.validity[: (n + 7) // 8].cpu().numpy() if c.validity is not None else None
        vb = pa.py_buffer(bm) if bm is not None else None
        if c.dtype in ("utf8", "large_utf8"):
            w = 4 if c.dtype == "utf8" else 8
            offs = c.offsets[: (n + 1) * w].cpu().numpy()
            nbytes = int(offs.view(np.int32 if w == 4 else np.int64)[-1])
            data = c.values[:nbytes].cpu().numpy()
            arr = pa.Array.from_buffers(pa.string() if w == 4 else pa.large_string(), n,
                                        [vb, pa.py_buffer(offs), pa.py_buffer(data)], null_count=-1 if bm is not None else 0)
        else:
            w = 4 if c.dtype == "i32" else 8
            t = {"f64": pa.float64(), "i64": pa.int64(), "i32": pa.int32()}[c.dtype]
            arr = pa.Array.from_buffers(t, n, [vb, pa.py_buffer(c.values[: n * w].cpu().numpy())],
                                        null_count=-1 if bm is not None else 0)
        arrays.append(arr)
        names.append(name)
    return pa.record_batch(arrays, names=names)


def ingest_timing(args, analyzers) -> dict:
    """C5 from HOST-resident Arrow batches (Arrow C Data Interface -> pinned double-buffered upload ->
    dq_scan): upload GB/s (host memory -> HBM, CPU staging copy included) and end-to-end rows/s of upload
    + scan with the copy of chunk k + 1 overlapping the scan of chunk k.  The same host batch is fed
    --ingest-reps times (rows counted each time)."""
    import ctypes

    import torch

    from deequ_amd import _lib as L
    from deequ_amd import synth
    from deequ_amd.ingest import ArrowScanner, ImportedArray, arrow_schema
    from deequ_amd.runner import ScanPlan

    n = args.ingest_rows
    t = synth.c5_table(n, row0=0, seed=42)
    torch.cuda.synchronize()
    batch = _arrow_batch(t, n)
    del t
    torch.cuda.empty_cache()
    plan = ScanPlan(analyzers, arrow_schema(batch))
    hosts = [ImportedArray(batch.column(batch.schema.get_field_index(c))) for c in plan.columns]
    nbytes = sum(h.host.value_bytes + h.host.validity_bytes + h.host.offset_bytes for h in hosts)
    for h in hosts:
        h.close()
    slot = nbytes + 3 * 256 * len(plan.columns)
    sc = ArrowScanner(plan, slot, n_slots=2)
    # upload alone: host -> pinned -> HBM, synchronised
    sc.scan(batch)  # warm (pinned pages touched, plan allocated)
    plan.finish()
    plan.reset()
    imported = [ImportedArray(batch.column(batch.schema.get_field_index(c))) for c in plan.columns]
    hc = (type(imported[0].host) * len(imported))(*[i.host for i in imported])
    views = (L.ColumnView * len(imported))()
    lib = sc.lib
    t0 = time.perf_counter()
    for _ in range(args.ingest_reps):
        L.check(lib.dq_upload(sc.h, hc, len(imported), views))
        L.check(lib.dq_upload_release(sc.h, sc.stream))
    L.check(lib.dq_upload_sync(sc.h))
    t_up = time.perf_counter() - t0
    for i in imported:
        i.close()
    torch.cuda.synchronize()
    # end to end: upload k + 1 overlaps scan k
    plan.reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.ingest_reps):
        sc.scan(batch)
    plan.finish()
    torch.cuda.synchronize()
    t_e2e = time.perf_counter() - t0
    sc.close()
    plan.close()
    reps = args.ingest_reps
    return {"rows_per_batch": n, "batches": reps, "host_bytes_per_batch": nbytes,
            "upload_GBps": nbytes * reps / t_up / 1e9,
            "pcie_gen5_x16_GBps": 64.0,
            "e2e_rows_per_s": n * reps / t_e2e, "e2e_ms_per_batch": t_e2e / reps * 1e3,
            "note": "host Arrow batch (pageable numpy buffers) -> CPU threads -> pinned slot -> DMA -> HBM, "
                    "2 slots; e2e = upload + fused scan + finish, copy of batch k+1 overlapping scan of k"}


def cpu_baseline(cols, n, threads, min_seconds=10.0):
    """The C restatement (oracle/, "port") of the same profile scan on the host's CPU share; `cols` = the
    host copy of the sample's columns (_host_cols)."""
    from oracle import dq_oracle_c as C

    share, how = host_cpu_share()
    threads = threads or share
    reps = 0
    t0 = time.perf_counter()
    while True:
        C.profile_scan(cols, n, nparts=threads * 4, nthreads=threads)
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= min_seconds:
            break
    return {"value": reps * n / dt, "unit": "rows/s", "cores": threads, "kind": "port",
            "per_core_rows_per_s": reps * n / dt / threads,
            "sample": f"{reps} x {n} rows x 16 cols of the same C5 data (first chunk), profile scan in oracle/c "
                      f"(Spark partial/final aggregation order, per-row Welford + XXH64 HLL), {threads} OpenMP "
                      f"threads = this host's CPU share ({how}), {dt:.1f} s"}


def c1_host_data(table):
    """Host copies of the C1 columns its CPU path reads (the i64 columns, every validity bitmap)."""
    n = table.num_rows
    cols = [c for c in _host_cols(table, n) if c[0] == "i64"]
    bitmaps = [c.validity[: (n + 7) // 8].cpu().numpy() for c in table.columns.values() if c.validity is not None]
    return n, cols, bitmaps


def cpu_baseline_c1(data, threads, min_seconds):
    """C1's CPU path: the oracle's C restatement of the Item-table analyzers (count / moments / min / max of
    id and numViews, validity counts of the strings) on the host's CPU share."""
    from oracle import dq_oracle_c as C

    n, cols, bitmaps = data
    share, how = host_cpu_share()
    threads = threads or share
    import numpy as np

    reps = 0
    t0 = time.perf_counter()
    while True:
        for kind, vals, _, bm in cols:
            parts = C.column_stats_partials(kind, vals, bm, threads * 4, threads)
            C.stats_fold(kind, parts)
        for bm in bitmaps:  # Completeness of the string columns: popcount of their validity
            int(np.unpackbits(bm, bitorder="little")[:n].sum())
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= min_seconds:
            break
    return {"value": reps * n / dt, "unit": "rows/s", "cores": threads, "kind": "port",
            "sample": f"{reps} x {n} Item rows: Spark-order moments / min / max of id and numViews in oracle/c, "
                      f"{threads} OpenMP threads ({how}), {dt:.1f} s"}


if __name__ == "__main__":
    main()
