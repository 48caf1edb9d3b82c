#!/usr/bin/env python3
"""Per-kernel totals over the LAST <ms> milliseconds of a rocprofv3 kernel trace (the timed
steps of a bench run, excluding graph build and warmup): prof_window.py DIR MS [TOP]."""
import csv
import sys
from collections import defaultdict
from pathlib import Path

d, win = Path(sys.argv[1]), float(sys.argv[2]) * 1e6
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
tr = next(d.rglob("*kernel_trace.csv"))
ks = list(csv.DictReader(open(tr)))
end = max(int(r["End_Timestamp"]) for r in ks)
t0 = end - win
tot, cnt = defaultdict(float), defaultdict(int)
for r in ks:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s >= t0:
        tot[r["Kernel_Name"]] += (e - s) / 1e6
        cnt[r["Kernel_Name"]] += 1
busy = sum(tot.values())
print(f"last {win/1e6:.0f} ms: kernel busy {busy:.1f} ms, {sum(cnt.values())} dispatches")
for k, v in sorted(tot.items(), key=lambda x: -x[1])[:top]:
    print(f"{v:9.1f} ms {cnt[k]:5d} x {v/cnt[k]:8.3f}  {k[:120]}")
