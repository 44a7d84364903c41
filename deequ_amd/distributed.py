"""Multi-GPU: rows shard across ranks (one process per GPU); the fixed-size aggregation-result slot
sets (dq_state, 424 B per analyzer) are exchanged with ONE all-gather (RCCL over xGMI when the
process group is "nccl", gloo on CPU) and merged on every rank in rank order 0..N-1 with
dq_state_combine -- Spark's partial-aggregate merge (AnalysisRunner.scala:303: partial per partition
-> Exchange(SinglePartition) -> final merge), so every rank holds the same, deterministic result.
"""
from __future__ import annotations

import ctypes
from typing import List, Sequence

from . import _lib as L


def pack(states: Sequence[L.State]) -> bytes:
    arr = (L.State * len(states))(*states)
    return ctypes.string_at(ctypes.addressof(arr), ctypes.sizeof(arr))


def unpack(blob: bytes, n: int) -> List[L.State]:
    arr = (L.State * n).from_buffer_copy(blob)
    return [arr[i] for i in range(n)]


def combine_in_order(per_rank: Sequence[Sequence[L.State]]) -> List[L.State]:
    merged = [L.State.from_buffer_copy(bytes(s)) for s in per_rank[0]]
    for other in per_rank[1:]:
        for i, s in enumerate(other):
            out = L.State()
            L.check(L.lib.dq_state_combine(ctypes.byref(merged[i]), ctypes.byref(s), ctypes.byref(out)))
            merged[i] = out
    return merged


def allgather_combine(states: Sequence[L.State], group=None) -> List[L.State]:
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    n = len(states)
    blob = pack(states)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    t = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t, group=group)
    per_rank = [unpack(o.cpu().numpy().tobytes(), n) for o in out]
    return combine_in_order(per_rank)
