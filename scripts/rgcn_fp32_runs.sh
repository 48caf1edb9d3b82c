#!/usr/bin/env bash
# R-GCN 1/8-scale MAG240M step (dropout fused into BN+ReLU) then the fp32-vs-bf16 runs.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u benchmarks/bench_rgcn.py --scale 0.125 --steps 5 --warmup 2 > gpurun_out/rgcn_eighth.log 2>&1
tail -3 gpurun_out/rgcn_eighth.log
bash scripts/fp32_runs.sh
