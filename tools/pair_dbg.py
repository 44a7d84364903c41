import json, sys
import os; sys_path = __import__("sys").path; sys_path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import deequ_amd as dq
from deequ_amd import synth
from deequ_amd.runner import scan_states
out = {}
for n in [2048 * 64, 2048 * 64 + 64, 2048 * 64 + 128 + 5, 1_000_003]:
    t = synth.c4_table(n, seed=5)
    names = list(t.columns)
    an = [dq.Correlation(names[i], names[j]) for i in range(8) for j in range(i + 1, 8)]
    an += [dq.Mean(c) for c in names]
    got = scan_states(t, an)
    out[n] = {str(a): [float(x) for x in (got[a].n, got[a].xAvg, got[a].yAvg, got[a].ck)] if hasattr(got[a], "ck") else [float(got[a].sum_), float(got[a].count)] for a in an}
json.dump(out, open(sys.argv[1], "w"))
