#!/usr/bin/env bash
# hub-row split on an extreme power-law graph (quarter-scale papers100M entries)
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u benchmarks/bench_spmm.py --shape ogbn-papers100M --scale 0.25 --feats 128 --rounds 2 \
  --powerlaw ${ALPHA:-3} --variants ${VARIANTS:-4:0:128:256,4:0:128:4096,4:0:128} > gpurun_out/spmm_powerlaw.log 2>&1
grep -v '^{' gpurun_out/spmm_powerlaw.log
