#!/usr/bin/env bash
# SpMM sensitivity to neighbour-window size (L2 fit) plus L2 hit counters.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for w in ${WINDOWS:-16384 4096 1024}; do
  timeout -k 10 200 python benchmarks/bench_spmm.py --shape ogbn-papers100M --feats ${FEATS:-128} \
    --rounds 2 --variants ${VARIANTS:-2:2:128} --window $w > gpurun_out/spmm_w$w.log 2>&1
done
if [ -n "${PMC:-1}" ]; then
  for w in ${PMC_WINDOWS:-16384 4096}; do
    COUNTERS="TCC_HIT_sum TCC_MISS_sum" TAG=w$w TMO=200 bash scripts/pmc.sh python3 \
      benchmarks/bench_spmm.py --shape ogbn-papers100M --feats ${FEATS:-128} --rounds 1 \
      --variants ${VARIANTS:-2:2:128} --window $w
  done
fi
