#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-stats CSV (+ timeline gaps from the kernel trace)."""
import csv
import sys
from pathlib import Path

d = Path(sys.argv[1])
stats = next(d.rglob("*kernel_stats.csv"))
rows = list(csv.DictReader(open(stats)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"kernel time total {tot/1e6:.1f} ms over {sum(int(r['Calls']) for r in rows)} dispatches")
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.1f} ms {int(r['Calls']):5d} x {float(r['AverageNs'])/1e6:8.3f} ms "
          f"{float(r['Percentage']):5.1f}%  {r['Name'][:110]}")
tr = list(d.rglob("*kernel_trace.csv"))
if tr:
    ks = sorted(csv.DictReader(open(tr[0])), key=lambda r: int(r["Start_Timestamp"]))
    end = None
    gap = 0
    for r in ks:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if end is not None and s > end:
            gap += s - end
        end = e if end is None else max(end, e)
    span = end - int(ks[0]["Start_Timestamp"])
    print(f"timeline span {span/1e6:.1f} ms, idle gaps {gap/1e6:.1f} ms")
