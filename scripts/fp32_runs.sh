#!/usr/bin/env bash
# fp32 (reference precision) measurements of the headline step at the shapes that fit:
# ogbn-products whole graph, and one rank of the 4-way papers100M partition (loopback);
# the bf16 runs of the same configs alongside for the ratio.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/fp32_runs.jsonl
: > $O
for dt in fp32 bf16; do
  timeout -k 10 300 python -u bench.py --shape ogbn-products --steps 10 --warmup 3 --no-extra --dtype $dt > gpurun_out/fp32_products_$dt.log 2>&1
  grep '^{' gpurun_out/fp32_products_$dt.log | sed "s/^{/{\"run\": \"products_$dt\", /" >> $O
  timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --rehearse-world 4 --rehearse-rank 1 --dtype $dt > gpurun_out/fp32_w4_$dt.log 2>&1
  grep '^{' gpurun_out/fp32_w4_$dt.log | sed "s/^{/{\"run\": \"papers100M_w4rank1_$dt\", /" >> $O
done
cut -c1-400 $O
