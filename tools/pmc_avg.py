"""Average rocprofv3 counters per kernel (diagnostic).  Usage: python tools/pmc_avg.py gpurun_out/pmc_<label>"""
import collections
import csv
import glob
import sys

path = sorted(glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True))[0]
per = collections.defaultdict(lambda: collections.defaultdict(float))
for row in csv.DictReader(open(path)):
    per[(row.get("Dispatch_Id") or row.get("Correlation_Id"), row["Kernel_Name"].split("(")[0])][row["Counter_Name"]] += float(row["Counter_Value"])
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for (_, k), cs in per.items():
    for c, v in cs.items():
        agg[k][c].append(v)
for k, cs in agg.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(cs.items())})
