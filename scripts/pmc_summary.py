#!/usr/bin/env python3
"""Mean per-dispatch PMC counter values by kernel from a rocprofv3 --pmc CSV directory:
pmc_summary.py DIR [name-substring ...]"""
import csv
import sys
from collections import defaultdict
from pathlib import Path

d = Path(sys.argv[1])
keep = sys.argv[2:]
f = next(d.rglob("*counter_collection.csv"))
acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if keep and not any(s in k for s in keep):
        continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
for k, cs in acc.items():
    n = len(disp[k])
    print(f"{k[:110]}  ({n} dispatches)")
    for c, v in sorted(cs.items()):
        print(f"    {c:28s} {v / n:16.4g}")
