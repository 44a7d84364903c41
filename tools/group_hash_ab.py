"""Prints a digest of dq_freq_build's exported group keys (tuple hashes) over string / LARGE_UTF8 / tuple columns of
every length 0..40 (the last strings of a chunk included); run once per library (DQ_LIB_PATH) to check that a change
to the tuple hash's code keeps the hash values (diagnostic)."""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    assert torch.cuda.is_available()
    from deequ_amd.grouping import build_frequencies
    from deequ_amd.table import Table, column_from_numpy, utf8_column

    rng = np.random.default_rng(1)
    vals = [bytes(rng.integers(0, 256, int(rng.integers(0, 41)), dtype=np.uint8)) for _ in range(20000)]
    vals += [b"x" * k for k in range(41)]  # short and long strings at the end of the bytes buffer
    ints = rng.integers(0, 5, len(vals)).astype(np.int64)
    h = hashlib.sha256()
    for chunks in (1, 3):
        step = (len(vals) + chunks - 1) // chunks
        data = [Table([utf8_column("s", vals[lo:lo + step]), utf8_column("t", vals[lo:lo + step], large=True),
                       column_from_numpy("i", "i64", ints[lo:lo + step], np.ones(len(ints[lo:lo + step]), bool))])
                for lo in range(0, len(vals), step)]
        for cols in (["s"], ["t"], ["s", "i"], ["i", "t", "s"]):
            keys, counts = build_frequencies(data if chunks > 1 else data[0], cols).frequencies.export()
            h.update(np.asarray(keys).tobytes())
            h.update(np.asarray(counts).tobytes())
    print("group keys digest", h.hexdigest())


if __name__ == "__main__":
    main()
