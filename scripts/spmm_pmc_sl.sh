#!/usr/bin/env bash
# L2 / memory-side counters of the SpMM on the structureless papers100M graph and on the
# power-law graph (hub split on): one counter group per pass, kernel trace only.
set -eu
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
SL="benchmarks/bench_spmm.py --shape ogbn-papers100M --feats 128 --rounds 1 --global-frac 1.0 --variants 4:0:128:2048"
PL="benchmarks/bench_spmm.py --shape ogbn-papers100M --scale 0.25 --feats 128 --rounds 1 --powerlaw 3 --variants 4:0:128:2048"
for spec in sl pl; do
  if [ $spec = sl ]; then CMD=$SL; else CMD=$PL; fi
  COUNTERS="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" TAG=spmm_${spec}_tcc TMO=300 \
    bash scripts/pmc.sh python3 $CMD
  COUNTERS="FETCH_SIZE" TAG=spmm_${spec}_fetch TMO=300 bash scripts/pmc.sh python3 $CMD
done
