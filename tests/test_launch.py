"""The multi-GPU plumbing of bench.py and deequ_amd.distributed (AnalysisRunner.scala:303's partial ->
final merge across ranks), executed for real:

* CPU: `bench.py --gpus N` re-launches itself as N ranks through torch.distributed.run before anything
  touches the GPU (the command it builds);
* GPU: two ranks sharing the box's one GPU run the whole bench (scan, all-gather + rank-order combine,
  StateLoader append) over gloo and print ONE line with n_gpus = 2 and a measured merge time;
* GPU: a world-size-1 "nccl" (RCCL) process group initialised with device_id exactly as bench.py does,
  so allgather_combine's device-tensor branch runs (RCCL needs distinct GPUs per rank, so one rank is
  what a one-GPU box can run).
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT


def test_bench_launcher_builds_torchrun_command(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench

    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 0

    monkeypatch.setattr(bench.subprocess, "call", fake_call)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    assert bench.launch_ranks(bench.parse(["--gpus", "4", "--steps", "3"])) == 0
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"] and cmd[-5].endswith("bench.py")
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


@pytest.mark.gpu
def test_bench_two_ranks_gloo_on_one_gpu():
    env = dict(os.environ)
    env.pop("RANK", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo", "--rows",
           "4000000", "--chunk", "2000000", "--steps", "2", "--warmup", "1", "--configs", "", "--cpu-sample", "0",
           "--ingest-rows", "0"]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["scaling"] == "weak"
    assert rec["rank_merge_ms_per_step"] > 0.0
    assert rec["value"] > 0 and rec["config"]["rows_per_gpu"] == 4_000_000


def _nccl_worker(port, q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    from deequ_amd import distributed, synth
    from deequ_amd.runner import scan_results
    from deequ_amd.states import state_from_c

    t = synth.c5_table(100_000, seed=21)
    analyzers = synth.profile_analyzers(t)
    res = scan_results(t, analyzers)
    merged = distributed.allgather_combine(res)  # device tensors through RCCL
    q.put(([repr(state_from_c(s)) for s in res], [repr(state_from_c(s)) for s in merged]))
    dist.destroy_process_group()


@pytest.mark.gpu
def test_nccl_world_size_one_allgather_combine():
    import torch.multiprocessing as mp

    from tests.test_distributed import _free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), q))
    p.start()
    before, after = q.get(timeout=180)
    p.join(60)
    assert p.exitcode == 0
    assert before == after  # one rank: the all-gather + combine is the identity on the slot set
