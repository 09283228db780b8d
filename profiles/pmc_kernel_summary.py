"""Per-kernel means of rocprofv3 --pmc counter CSVs (one row per dispatch and counter).

usage: python profiles/pmc_kernel_summary.py counter_collection.csv [more.csv ...]
"""
import csv
import re
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        m = re.search(r"(\w+_kernel(<[^>]*>)?)", r["Kernel_Name"])
        k = m.group(1) if m else r["Kernel_Name"][:50]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v) / len(v):16.1f}  (n={len(v)})")
