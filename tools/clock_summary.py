"""Per-kernel effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration) and VALU issue efficiency at that clock
from one rocprofv3 --kernel-trace --pmc run (tools/clock_probe.sh).  Usage: clock_summary.py DIR [out.json]"""
import collections
import csv
import glob
import json
import sys

d = sys.argv[1]
cc = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
rows = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
for r in csv.DictReader(open(cc)):
    key = r.get("Dispatch_Id") or r.get("Correlation_Id")
    rows[key][r["Counter_Name"]] += float(r["Counter_Value"])
    names[key] = r["Kernel_Name"]
dur = {}
if kt:
    for r in csv.DictReader(open(kt[0])):
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for key, c in rows.items():
    n = names[key]
    if "dq_" not in n or key not in dur or dur[key] < 3e-4:
        continue
    a = agg[n.split("(")[0]]
    a["launches"] += 1
    a["seconds"] += dur[key]
    for k, v in c.items():
        a[k] += v
out = {}
for n, a in agg.items():
    L = a["launches"]
    sec = a["seconds"] / L
    clk = a["GRBM_GUI_ACTIVE"] / L / 8 / sec
    valu = a["SQ_INSTS_VALU"] / L
    floor_nominal = valu * 4 / (1024 * 2.4e9)
    floor_held = valu * 4 / (1024 * clk)
    out[n] = {"launches": int(L), "avg_ms": sec * 1e3, "effective_clock_GHz": clk / 1e9, "valu_per_launch": valu,
              "issue_floor_ms_2.4GHz": floor_nominal * 1e3, "issue_floor_ms_at_clock": floor_held * 1e3,
              "issue_frac_at_clock": floor_held / sec, "issue_frac_2.4GHz": floor_nominal / sec}
print(json.dumps(out, indent=1))
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
