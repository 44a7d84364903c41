"""Diagnostic: c4 scan vs numpy (counts / means / correlation n), with table checksums before/after."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import deequ_amd as dq
from deequ_amd import synth
from deequ_amd.runner import scan_states

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_003
t = synth.c4_table(n, seed=5)
torch.cuda.synchronize()

def snap():
    out = {}
    for k, c in t.columns.items():
        out[k] = (c.values.cpu().numpy().copy(), None if c.validity is None else c.validity.cpu().numpy().copy())
    return out

before = snap()
names = list(t.columns)
for label, analyzers in [
    ("mean_only", [dq.Mean(c) for c in names]),
    ("corr_only", [dq.Correlation(names[i], names[j]) for i in range(8) for j in range(i + 1, 8)]),
    ("all", [dq.Correlation(names[i], names[j]) for i in range(8) for j in range(i + 1, 8)]
            + [dq.Mean(c) for c in names] + [dq.StandardDeviation(c) for c in names]),
]:
    got = scan_states(t, analyzers)
    torch.cuda.synchronize()
    after = snap()
    changed = [k for k in names if not (np.array_equal(before[k][0], after[k][0]) and
                                        np.array_equal(before[k][1], after[k][1]))]
    bad = []
    for a in analyzers:
        s = got[a]
        if type(a).__name__ in ("Mean", "StandardDeviation"):
            vals = before[a.column][0][: n * 8].view(np.float64)
            valid = np.unpackbits(before[a.column][1], bitorder="little")[:n].astype(bool)
            cnt = int(valid.sum())
            c_got = s.count if hasattr(s, "count") else s.n
            if int(c_got) != cnt:
                bad.append(f"{a}: count {c_got} vs {cnt}")
        else:
            vx = np.unpackbits(before[a.firstColumn][1], bitorder="little")[:n].astype(bool)
            vy = np.unpackbits(before[a.secondColumn][1], bitorder="little")[:n].astype(bool)
            both = int((vx & vy).sum())
            if int(s.n) != both:
                bad.append(f"{a}: n {s.n} vs {both} xa={s.xAvg} ya={s.yAvg}")
    print(label, "changed:", changed, "bad:", len(bad), flush=True)
    for b in bad[:6]:
        print("   ", b, flush=True)
