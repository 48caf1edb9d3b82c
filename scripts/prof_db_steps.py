#!/usr/bin/env python3
"""Per-step kernel totals from a rocprofv3 rocpd database (prof_results.db): steps are
delimited by the optimizer's fused kernel (name contains ``--marker``, default
``FusedOpti``); averages the kernels of the last ``--steps`` complete steps.

    python scripts/prof_db_steps.py DB [--steps 5] [--skip-last 0] [--top 30]
"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="FusedOpti")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--skip-last", type=int, default=0,
                    help="ignore this many trailing steps (e.g. region-timing steps)")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--total-steps", type=int, default=0,
                    help="steps the traced program ran (warmup + timed + extra): markers per "
                         "step = markers / this (an optimizer may launch several per step)")
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    rows = cur.execute("select name, start, end, duration, stream_id from kernels "
                       "order by start").fetchall()
    ends = [r[2] for r in rows if a.marker in r[0]]
    k = max(1, round(len(ends) / a.total_steps)) if a.total_steps else 1
    ends = ends[k - 1::k]  # the last marker of every step
    if a.skip_last:
        ends = ends[:-a.skip_last]
    ends = ends[-(a.steps + 1):]
    n = len(ends) - 1
    t0, t1 = ends[0], ends[-1]
    win = [r for r in rows if r[1] >= t0 and r[2] <= t1]
    tot, cnt = collections.defaultdict(float), collections.Counter()
    for r in win:
        tot[r[0]] += r[3]
        cnt[r[0]] += 1
    busy = sum(tot.values()) / n / 1e6
    print(f"steps {n}: span {(t1 - t0) / n / 1e6:.3f} ms/step, kernel time {busy:.3f} ms/step "
          f"(summed over streams), {len(win) / n:.0f} kernels/step")
    for name, v in sorted(tot.items(), key=lambda x: -x[1])[:a.top]:
        print(f"{v / n / 1e6:8.3f} ms {cnt[name] / n:6.1f}x  {name[:120]}")


if __name__ == "__main__":
    main()
