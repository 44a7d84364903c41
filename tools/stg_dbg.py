"""Diagnostic: HLL registers of one-row and few-row UTF8 tables of every string length 0..40 through the
library DQ_LIB_PATH names, against the oracle; prints the lengths whose registers differ.  GPU box only."""
import sys

import numpy as np

sys.path.insert(0, ".")
import deequ_amd as dq  # noqa: E402
from deequ_amd.runner import scan_states  # noqa: E402
from deequ_amd.table import utf8_column  # noqa: E402
from oracle import dq_oracle as O  # noqa: E402

bad = []
for n in (1, 5, 64, 200):
    for ln in range(0, 41):
        rng = np.random.default_rng(ln * 7 + n)
        strs = [bytes(rng.integers(97, 123, ln, dtype=np.uint8)) for _ in range(n)]
        t = dq.Table([utf8_column("s", strs)])
        a = dq.ApproxCountDistinct("s")
        got = scan_states(t, [a])[a]
        ref = O.compute_state(("ApproxCountDistinct", "s", None), {"s": O.OColumn("utf8", strs, np.ones(n, bool))}, n)
        if tuple(got.words) != tuple(ref.words):
            gi = [i for i, w in enumerate(got.words) if w]
            ri = [i for i, w in enumerate(ref.words) if w]
            bad.append((n, ln))
            if len(bad) < 12:
                print("n", n, "len", ln, "gpu words", gi[:4], "oracle words", ri[:4], flush=True)
print("mismatching (n, len):", bad)
