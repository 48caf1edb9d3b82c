#!/usr/bin/env python3
"""Stacked-bar timing breakdown from TimingReport JSON dumps (A7).

Reads ``{log_dir}/{dataset}_timing_report_world{W}.json`` files (``{region: [ms, ...]}``,
written by :meth:`dgraph_amd.utils.timing.TimingReport.dump`), drops the first iteration
of every region (warm-up, as experiments/OGB/plot_timing_reports.py:50-51 does), and draws
one stacked bar per world size with the mean time of each region. Also prints the table.

    python scripts/plot_timing_reports.py --log-dir logs --dataset arxiv --out timing.png
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import re
import statistics


def load(log_dir: str, dataset: str):
    out = {}
    for path in glob.glob(os.path.join(log_dir, f"{dataset}_timing_report_world*.json")):
        m = re.search(r"world(\d+)\.json$", path)
        if not m:
            continue
        with open(path) as f:
            data = json.load(f)
        out[int(m.group(1))] = {k: statistics.fmean(v[1:] if len(v) > 1 else v)
                                for k, v in data.items() if v}
    return dict(sorted(out.items()))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-dir", default="logs")
    ap.add_argument("--dataset", default="arxiv")
    ap.add_argument("--out", default=None, help="image path (needs matplotlib)")
    ap.add_argument("--title", default=None)
    a = ap.parse_args(argv)
    rep = load(a.log_dir, a.dataset)
    if not rep:
        print(f"no timing reports for {a.dataset} in {a.log_dir}")
        return 1
    regions = sorted({r for v in rep.values() for r in v})
    print("world " + " ".join(f"{r:>14s}" for r in regions))
    for w, v in rep.items():
        print(f"{w:5d} " + " ".join(f"{v.get(r, 0.0):14.3f}" for r in regions))
    if a.out:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt

        fig, ax = plt.subplots(figsize=(1.6 * len(rep) + 3, 4))
        xs = [str(w) for w in rep]
        bottom = [0.0] * len(rep)
        for r in regions:
            vals = [rep[w].get(r, 0.0) for w in rep]
            ax.bar(xs, vals, bottom=bottom, label=r)
            bottom = [b + v for b, v in zip(bottom, vals)]
        ax.set_xlabel("ranks")
        ax.set_ylabel("mean time per iteration (ms)")
        ax.set_title(a.title or f"{a.dataset}: timing breakdown")
        ax.legend(fontsize=8)
        fig.tight_layout()
        fig.savefig(a.out, dpi=120)
        print("wrote", a.out)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
