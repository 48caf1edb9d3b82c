#!/usr/bin/env python3
"""Timeline of the last step from a rocprofv3 --kernel-trace CSV directory: every dispatch
of the last WINDOW_MS ms with its start offset, duration, queue and stream, plus the
time per queue and the overlap between the comm-stream kernels (link_copy / copy_rows /
rccl) and the compute kernels.

    prof_timeline.py DIR WINDOW_MS [max_rows]
"""
import csv
import sys
from collections import defaultdict
from pathlib import Path

d = Path(sys.argv[1])
win_ms = float(sys.argv[2])
max_rows = int(sys.argv[3]) if len(sys.argv) > 3 else 200
f = next(d.rglob("*kernel_trace.csv"))
rows = []
for r in csv.DictReader(open(f)):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"]
    rows.append((s, e, name, r.get("Queue_Id", "?"), r.get("Stream_Id", "?")))
rows.sort()
t_end = max(e for _, e, *_ in rows)
t0 = t_end - int(win_ms * 1e6)
rows = [r for r in rows if r[1] > t0]


def short(n):
    n = n.replace("void dgraph::(anonymous namespace)::", "").replace("(anonymous namespace)::", "")
    return n[:70]


comm_kw = ("link_copy", "link_delay", "nccl", "rccl", "copy_rows")
per_q = defaultdict(float)
comm_iv, comp_iv = [], []
for s, e, n, q, st in rows:
    per_q[(q, st)] += (e - s) / 1e6
    (comm_iv if any(k in n for k in comm_kw) else comp_iv).append((max(s, t0), e))


def union(iv):
    iv = sorted(iv)
    out, tot = [], 0
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def total(iv):
    return sum(e - s for s, e in iv) / 1e6


cu, pu = union(comm_iv), union(comp_iv)
ov = 0
i = j = 0
while i < len(cu) and j < len(pu):
    a, b = max(cu[i][0], pu[j][0]), min(cu[i][1], pu[j][1])
    if b > a:
        ov += b - a
    if cu[i][1] < pu[j][1]:
        i += 1
    else:
        j += 1
print(f"window {win_ms} ms: {len(rows)} dispatches; compute busy {total(pu):.1f} ms, "
      f"comm-kernel busy {total(cu):.1f} ms, overlap {ov / 1e6:.1f} ms")
for (q, st), ms in sorted(per_q.items(), key=lambda kv: -kv[1]):
    print(f"  queue {q} stream {st}: {ms:.1f} ms")
print(f"{'start_ms':>9} {'dur_ms':>8} {'queue':>6} {'stream':>6}  kernel")
for s, e, n, q, st in rows[-max_rows:]:
    print(f"{(s - t0) / 1e6:9.2f} {(e - s) / 1e6:8.3f} {q:>6} {st:>6}  {short(n)}")
