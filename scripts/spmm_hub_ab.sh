#!/usr/bin/env bash
# hub-row split A/B on both graph localities (papers100M shape, F = 128 and 256) + tests
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hub_split.py -x -q --timeout 120 --timeout-method thread > gpurun_out/hub_tests.log 2>&1
tail -1 gpurun_out/hub_tests.log
for gf in 1.0 0.05; do
  timeout -k 10 400 python -u benchmarks/bench_spmm.py --shape ogbn-papers100M --feats 128,256 --rounds 3 \
    --global-frac $gf --variants 4:0:128,4:0:128:256,4:0:128:1024,4:0:256:256 > gpurun_out/spmm_hub_$gf.log 2>&1
  grep -v '^{' gpurun_out/spmm_hub_$gf.log
done
