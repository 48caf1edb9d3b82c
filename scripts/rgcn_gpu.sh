#!/usr/bin/env bash
# R-GCN (BASELINE config 4) on one MI355X: 1/8-scale MAG240M (the per-GPU share of the
# 8-GPU job) and rank 1 of the real 8-way partition (loopback exchange).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 ${TMO:-400} python benchmarks/bench_rgcn.py --scale 0.125 --steps ${STEPS:-5} \
  --warmup 2 --verbose ${EXTRA:-} > gpurun_out/rgcn_scale0125.log 2>&1
grep '^{' gpurun_out/rgcn_scale0125.log
if [ -n "${REHEARSE:-}" ]; then
  timeout -k 10 ${TMO:-400} python benchmarks/bench_rgcn.py --rehearse-world 8 \
    --rehearse-rank 1 --steps ${STEPS:-5} --warmup 2 --verbose ${EXTRA:-} \
    > gpurun_out/rgcn_rehearse_w8.log 2>&1
  grep '^{' gpurun_out/rgcn_rehearse_w8.log
fi
