#!/usr/bin/env python3
"""Kernel sequence of the last <ms> milliseconds of a rocprofv3 kernel trace (start offset,
duration, stream-agnostic), for reading a step's schedule: prof_seq.py DIR MS [OUT]."""
import csv
import sys
from pathlib import Path

d, win = Path(sys.argv[1]), float(sys.argv[2]) * 1e6
tr = next(d.rglob("*kernel_trace.csv"))
ks = sorted(csv.DictReader(open(tr)), key=lambda r: int(r["Start_Timestamp"]))
end = max(int(r["End_Timestamp"]) for r in ks)
t0 = end - win
lines = [f"{(int(r['Start_Timestamp']) - t0) / 1e6:9.3f} "
         f"{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6:8.3f} "
         f"{r['Kernel_Name'][:80]}" for r in ks if int(r["Start_Timestamp"]) >= t0]
out = "\n".join(lines) + "\n"
if len(sys.argv) > 3:
    Path(sys.argv[3]).write_text(out)
else:
    sys.stdout.write(out)
