#!/usr/bin/env bash
# Per-rank compute/memory of a W-way papers100M partition, one rank at a time on ONE GPU
# (loopback halo exchange; communication not included). Stops at the first failure.
# GF=1.0 rehearses the structureless graph (bench.py's secondary measurement).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
GF=${GF:-0.05}
for w in ${WORLDS:-2 4 8}; do
  timeout -k 10 ${TMO:-300} python bench.py --steps ${STEPS:-3} --warmup 1 --verbose \
    --global-frac "$GF" --rehearse-world $w --rehearse-rank ${RANK_OF:-1} \
    > gpurun_out/rehearse_gf${GF}_w$w.log 2>&1
  grep '^{' gpurun_out/rehearse_gf${GF}_w$w.log
done
