#!/usr/bin/env bash
# Every BASELINE config that fits one MI355X, one JSON line each (gpurun_out/benches.jsonl).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
O=gpurun_out/benches.jsonl
: > $O
run() { local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/bench_$name.log 2>&1
  grep '^{' gpurun_out/bench_$name.log | sed "s/^{/{\"bench\": \"$name\", /" >> $O
  tail -1 $O | cut -c1-300; }
run sage_papers100M 600 python bench.py --steps 5 --warmup 2
run sage_products 300 python bench.py --shape ogbn-products --steps 10 --warmup 3
run rgcn_mag_eighth 600 python benchmarks/bench_rgcn.py --scale 0.125 --steps 5 --warmup 2
run rgcn_mag_w8_rank1 600 python benchmarks/bench_rgcn.py --rehearse-world 8 --rehearse-rank 1 --steps 3 --warmup 2
run graphcast_step 600 python benchmarks/bench_graphcast.py --mode step
