"""Multi-rank merge on CPU (gloo, world_size 2): each rank contributes the aggregation-result slot
sets of its row shard; deequ_amd.distributed all-gathers them and merges in rank order with
dq_state_combine.  The result must equal the oracle over the union of the shards -- including
SQL null skipping across shards (a shard with no non-null predicate value) and Spark's NaN ordering.
The GPU scan itself is covered by tests/test_gpu_parity.py; this covers the exchange + merge."""
from __future__ import annotations

import math
import os
import socket

import numpy as np
import pytest

from tests.conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dataset(n=4000, seed=3):
    rng = np.random.default_rng(seed)
    x = rng.normal(10, 3, n)
    x[rng.integers(0, n, 5)] = np.nan
    y = 0.5 * x + rng.normal(0, 1, n)
    k = rng.integers(0, 300, n).astype(np.int64)
    vx, vy, vk = rng.random(n) > 0.1, rng.random(n) > 0.1, rng.random(n) > 0.1
    vk[n // 2:] = False  # the second shard has no valid k -> NULL slots that must be skipped
    return n, {"x": ("f64", x, vx), "y": ("f64", y, vy), "k": ("i64", k, vk)}


SPECS = [("Size", None), ("Completeness", "k", None), ("Compliance", "c", "k > 100", None),
         ("Sum", "x", None), ("Mean", "k", None), ("StandardDeviation", "y", None), ("Minimum", "x", None),
         ("Maximum", "x", None), ("Minimum", "k", None), ("Correlation", "y", "x", None),
         ("ApproxCountDistinct", "k", None), ("Sum", "k", "x > 10"), ("Compliance", "d", "x > 12", "k < 50")]


def slots(spec, cols, n):
    """Oracle slot set (SQL values incl. NULL) of one analyzer on one shard -> dq_state."""
    from deequ_amd import _lib as L

    from oracle import dq_oracle as O

    s = L.State()
    op = spec[0]
    s.op = {"Size": L.OP_SIZE, "Completeness": L.OP_COMPLETENESS, "Compliance": L.OP_COMPLIANCE,
            "Sum": L.OP_SUM, "Mean": L.OP_MEAN, "StandardDeviation": L.OP_STDDEV, "Minimum": L.OP_MIN,
            "Maximum": L.OP_MAX, "Correlation": L.OP_CORRELATION, "ApproxCountDistinct": L.OP_APPROX_COUNT_DISTINCT}[op]
    where = spec[-1]
    wt, wn = O._where(cols, n, where)
    if op == "Size":
        s.u.size.num_matches = int(wt.sum())
        s.has_value[0] = s.has_value[1] = 1 if where is None or wn.any() else 0
    elif op in ("Completeness", "Compliance"):
        if op == "Completeness":
            t, nn = cols[spec[1]].valid & wt, np.ones(n, bool) & wt
            nonnull_rows = n > 0
        else:
            pt, pn = O.OracleExpr(spec[2]).eval_bool(cols, n)
            t, nonnull_rows = pt & wt, (pn & wt).any()
        s.u.ratio.num_matches = int(t.sum())
        s.has_value[0] = 1 if nonnull_rows else 0
        s.u.ratio.count = n if where is None else int(wt.sum())
        s.has_value[1] = 1 if (where is None or wn.any()) else 0
    elif op in ("Sum", "Mean"):
        c = cols[spec[1]]
        sel = c.valid & wt
        v = O.spark_sum(c, sel)
        if op == "Sum":
            s.u.sum.sum = 0.0 if v is None else v
            s.has_value[0] = s.has_value[1] = 0 if v is None else 1
        else:
            s.u.mean.sum = 0.0 if v is None else v
            s.u.mean.count = int(sel.sum())
            s.has_value[0], s.has_value[1] = (0 if v is None else 1), 1
    elif op == "StandardDeviation":
        c = cols[spec[1]]
        nn, avg, m2 = O.spark_stddev_buffer(O._as_double_list(c), c.valid & wt)
        s.u.stddev.n, s.u.stddev.avg, s.u.stddev.m2 = nn, avg, m2
        s.has_value[0] = s.has_value[1] = 1
    elif op in ("Minimum", "Maximum"):
        c = cols[spec[1]]
        v = O.spark_min(c, c.valid & wt, is_max=(op == "Maximum"))
        s.u.minmax.value = 0.0 if v is None else v
        s.has_value[0] = s.has_value[1] = 0 if v is None else 1
    elif op == "Correlation":
        a, b = cols[spec[1]], cols[spec[2]]
        r = O.spark_corr_buffer(O._as_double_list(a), O._as_double_list(b), a.valid & b.valid & wt)
        (s.u.corr.n, s.u.corr.x_avg, s.u.corr.y_avg, s.u.corr.ck, s.u.corr.x_mk, s.u.corr.y_mk) = r
        s.has_value[0] = s.has_value[1] = 1
    else:
        w = O.hll_words_for(cols[spec[1]], cols[spec[1]].valid & wt)
        for i in range(52):
            s.u.hll.words[i] = w[i]
        s.has_value[0] = s.has_value[1] = 1
    return s


def _shard(cols_np, lo, hi):
    from oracle import dq_oracle as O

    return {k: O.OColumn(t, v[lo:hi], m[lo:hi]) for k, (t, v, m) in cols_np.items()}, hi - lo


def _worker(rank, world, port, q):
    import sys

    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from deequ_amd import distributed
    from deequ_amd.states import state_from_c

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, cols_np = _dataset()
    lo, hi = n * rank // world, n * (rank + 1) // world
    cols, m = _shard(cols_np, lo, hi)
    mine = [slots(sp, cols, m) for sp in SPECS]
    merged = distributed.allgather_combine(mine)
    q.put((rank, [repr(state_from_c(s)) for s in merged]))
    dist.destroy_process_group()


def test_two_rank_allgather_merge_equals_oracle():
    import torch.multiprocessing as mp

    from deequ_amd.states import state_from_c

    from oracle import dq_oracle as O

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert res[0] == res[1]  # every rank holds the same merged result
    n, cols_np = _dataset()
    whole, _ = _shard(cols_np, 0, n)
    # reference: Spark with two partitions = the two shards, merged in order
    for spec, got in zip(SPECS, res[0]):
        ref = O.compute_state(spec, whole, n, n_partitions=2)
        ref_py = None if ref is None else state_from_c(slots(spec, whole, n))
        if ref is None:
            assert got == "None", (spec, got)
            continue
        if spec[0] in ("StandardDeviation", "Correlation", "Sum", "Mean"):
            # same Spark partial/final merge algebra -> same doubles up to the merge order, which is rank order
            g = eval_state(got)
            assert math.isclose(g.metricValue(), ref.metricValue(), rel_tol=1e-13) or (
                math.isnan(g.metricValue()) and math.isnan(ref.metricValue())), (spec, got, ref)
        else:
            assert got == repr(ref_py), (spec, got, ref_py)


def eval_state(text):
    import deequ_amd.states as S

    nan = float("nan")  # noqa: F841 - used by eval of repr
    return eval(text, {k: getattr(S, k) for k in dir(S)} | {"nan": float("nan")})


def _gpu_worker(rank, world, port, n_shard, q):
    """One rank on the (single) GPU: scan its row shard of the C5 table with the profile analyzers, then
    all-gather + merge the slot sets in rank order (gloo on this box; RCCL in bench.py)."""
    import sys

    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from deequ_amd import distributed, synth
    from deequ_amd.runner import scan_results
    from deequ_amd.states import state_from_c

    t = synth.c5_table(n_shard, row0=rank * n_shard, seed=13)
    analyzers = synth.profile_analyzers(t) + _extra(__import__("deequ_amd"))
    merged = distributed.allgather_combine(scan_results(t, analyzers))
    q.put((rank, [repr(state_from_c(s)) for s in merged]))
    dist.destroy_process_group()


def _extra(dq):
    return [dq.Correlation("c0", "c1"), dq.Compliance("p", "i0 >= 500"), dq.Sum("c2", "c3 > 3000")]


@pytest.mark.gpu
def test_two_rank_gpu_shards_equal_whole_table_scan():
    """AnalysisRunner.scala:303's partial -> final contract across processes: two ranks each dq_scan a
    different row shard on the GPU and merge through deequ_amd.distributed; the result equals ONE process
    scanning both shards (as two chunks) -- counts / min / max / HLL bit-exact, fp64 within 1e-12."""
    import torch.multiprocessing as mp

    import deequ_amd as dq
    from deequ_amd import synth
    from deequ_amd.runner import scan_states
    from tests.helpers import close

    n_shard = 300_032
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, 2, port, n_shard, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert res[0] == res[1]
    parts = [synth.c5_table(n_shard, row0=r * n_shard, seed=13) for r in range(2)]
    analyzers = synth.profile_analyzers(parts[0]) + _extra(dq)
    whole = scan_states(parts, analyzers)
    for a, got_txt in zip(analyzers, res[0]):
        got, want = eval_state(got_txt), whole[a]
        if want is None:
            assert got is None, a
            continue
        gv, wv = got.metricValue(), want.metricValue()
        if type(a).__name__ in ("Mean", "StandardDeviation", "Sum", "Correlation"):
            assert close(gv, wv, 1e-12), (a, gv, wv)
        else:
            assert gv == wv or (math.isnan(gv) and math.isnan(wv)), (a, got, want)
