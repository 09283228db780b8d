"""Average rocprofv3 --pmc counters per dispatch, grouped by kernel (substring match).

usage: python profiles/pmc_summary.py <pmc_counter_collection.csv>... [--kernels a,b]
"""
import csv
import sys
from collections import defaultdict

files = [f for f in sys.argv[1:] if not f.startswith("--")]
keys = None
for f in sys.argv[1:]:
    if f.startswith("--kernels="):
        keys = f.split("=", 1)[1].split(",")
agg = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for f in files:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        name = next((kk for kk in keys if kk in k), None) if keys else k.split("(")[0][-40:]
        if name is None:
            continue
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(name, f)].add(r["Dispatch_Id"])
for name, cs in agg.items():
    print(name)
    for c, v in sorted(cs.items()):
        n = max(len(d) for (nm, f), d in disp.items() if nm == name)
        print(f"  {c:32s} {v / n:12.4g}")
