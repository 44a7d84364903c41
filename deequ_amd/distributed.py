"""Multi-GPU: rows shard across ranks (one process per GPU); the fixed-size aggregation-result slot
sets (dq_state, 424 B per analyzer) are exchanged with ONE all-gather (RCCL over xGMI when the
process group is "nccl", gloo on CPU) and merged on every rank in rank order 0..N-1 with
dq_state_combine_n -- Spark's partial-aggregate merge (AnalysisRunner.scala:303: partial per partition
-> Exchange(SinglePartition) -> final merge), so every rank holds the same, deterministic result.
"""
from __future__ import annotations

import ctypes
from typing import List, Sequence

from . import _lib as L


def _array(states: Sequence[L.State]):
    return (L.State * max(1, len(states)))(*states)


def pack(states: Sequence[L.State]) -> bytes:
    arr = _array(states)
    return ctypes.string_at(ctypes.addressof(arr), ctypes.sizeof(L.State) * len(states))


def unpack(blob: bytes, n: int) -> List[L.State]:
    arr = (L.State * n).from_buffer_copy(blob)
    return [arr[i] for i in range(n)]


def combine_in_order(per_rank: Sequence[Sequence[L.State]]) -> List[L.State]:
    """Fold the ranks' slot sets in rank order with dq_state_combine_n (one C call per rank)."""
    n = len(per_rank[0])
    acc = _array(per_rank[0])
    for other in per_rank[1:]:
        L.check(L.lib.dq_state_combine_n(acc, _array(other), n, acc))
    return [acc[i] for i in range(n)]


def allgather_combine(states: Sequence[L.State], group=None) -> List[L.State]:
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    n = len(states)
    blob = pack(states)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    t = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
    out = torch.empty(world * t.numel(), dtype=torch.uint8, device=dev)  # rank r's blob at [r * size, ...)
    dist.all_gather_into_tensor(out, t, group=group)
    host = out.cpu().numpy().tobytes()
    size = len(blob)
    per_rank = [unpack(host[r * size:(r + 1) * size], n) for r in range(world)]
    return combine_in_order(per_rank)


def merge_loaded(fresh: Sequence[L.State], loaded: Sequence[L.State]) -> List[L.State]:
    """Analyzers.merge(state, loadedState) for a whole run (Analyzer.scala:113-117: the freshly computed
    state summed with the StateLoader's before it is persisted), one dq_state_merge_n call."""
    n = len(fresh)
    out = _array(fresh)
    L.check(L.lib.dq_state_merge_n(out, _array(loaded), n, out))
    return [out[i] for i in range(n)]
