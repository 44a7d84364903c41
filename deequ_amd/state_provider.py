"""StateLoader / StatePersister implementations (analyzers/StateProvider.scala:36-295).

InMemoryStateProvider keeps states keyed by analyzer (case-class equality).  HdfsStateProvider
writes the reference's binary images -- `<prefix>-<MurmurHash3.stringHash(analyzer.toString, 42)>.bin`,
Java DataOutputStream big-endian -- through dq_state_to_bytes / dq_state_from_bytes /
dq_state_identifier of libdqscan.so, on a local (or mounted) file system.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Dict, Optional

from . import _lib as L
from .states import State, state_from_c, state_to_c


class StateLoader:
    def load(self, analyzer) -> Optional[State]:
        raise NotImplementedError


class StatePersister:
    def persist(self, analyzer, state: State) -> None:
        raise NotImplementedError


class InMemoryStateProvider(StateLoader, StatePersister):
    def __init__(self):
        self._states: Dict[object, State] = {}
        self._lock = threading.Lock()

    def load(self, analyzer):
        with self._lock:
            return self._states.get(analyzer)

    def persist(self, analyzer, state):
        with self._lock:
            self._states[analyzer] = state

    def __str__(self):
        return "".join(f"{a} => {s}\n" for a, s in self._states.items())


def identifier(analyzer) -> str:
    return str(L.lib.dq_state_identifier(str(analyzer).encode("utf-8")))


class HdfsStateProvider(StateLoader, StatePersister):
    def __init__(self, locationPrefix: str, allowOverwrite: bool = False):
        self.locationPrefix = locationPrefix
        self.allowOverwrite = allowOverwrite

    def _path(self, analyzer) -> str:
        return f"{self.locationPrefix}-{identifier(analyzer)}.bin"

    def persist(self, analyzer, state):
        from .quantiles import ApproxQuantileState

        if isinstance(state, ApproxQuantileState):  # ApproximatePercentile.serializer (StateProvider.scala:126-129)
            buf = state.percentileDigest.serialize()
        else:
            c = state_to_c(state, analyzer._lower_op())
            n = L.lib.dq_state_to_bytes(ctypes.byref(c), None, 0)
            if n < 0:
                L.check(int(n))
            buf = (ctypes.c_uint8 * n)()
            L.lib.dq_state_to_bytes(ctypes.byref(c), buf, n)
        path = self._path(analyzer)
        if os.path.exists(path) and not self.allowOverwrite:
            raise FileExistsError(f"File {path} already exists!")  # DfsUtils.writeToFileOnDfs
        with open(path, "wb") as f:
            f.write(bytes(buf))

    def load(self, analyzer):
        path = self._path(analyzer)
        if not os.path.exists(path):
            return None
        with open(path, "rb") as f:
            data = f.read()
        from .quantiles import ApproxQuantileState, PercentileDigest, _QuantileBase

        if isinstance(analyzer, _QuantileBase):  # StateProvider.scala:165-167
            return ApproxQuantileState(PercentileDigest.deserialize(data))
        out = L.State()
        L.check(L.lib.dq_state_from_bytes(analyzer._lower_op(), data, len(data), ctypes.byref(out)))
        return state_from_c(out)
