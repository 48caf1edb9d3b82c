#!/usr/bin/env bash
# GraphCast step on one MI355X: reference graph (655 320 mesh edges) with the reference's
# 73 channels and the ERA5 37-level (227-channel) configuration, plus a per-op table
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/gc_runs.jsonl
: > $O
timeout -k 10 300 python -u benchmarks/bench_graphcast.py --mode step --profile-ops gpurun_out/gc_ops.txt > gpurun_out/gc_73.log 2>&1
grep '^{' gpurun_out/gc_73.log >> $O
timeout -k 10 300 python -u benchmarks/bench_graphcast.py --mode step --channel-config era5-37 > gpurun_out/gc_227.log 2>&1
grep '^{' gpurun_out/gc_227.log >> $O
cut -c1-400 $O
head -30 gpurun_out/gc_ops.txt | cut -c1-200
