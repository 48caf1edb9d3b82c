#!/usr/bin/env bash
# Link-model rehearsals of BASELINE configs 4 (R-GCN, MAG240M-shaped) and 5 (GraphCast):
# one rank of the 8-way partition on one GPU, every exchange a loopback behind the 153 GB/s
# link model (and instant, for the exposed-exchange difference). fp32.
# Output: gpurun_out/cfg45/*.log, all.jsonl
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/cfg45
O=gpurun_out/cfg45
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -E '^\{' "$O/$name.log" | tee -a $O/all.jsonl | cut -c1-1500
  if fatal $rc; then echo "FATAL at $name"; exit $rc; fi
}
GC="python -u benchmarks/bench_graphcast.py --dtype fp32 --steps 5 --warmup 2 --rehearse-world 8"
for spec in ${GC_RUNS:-0:153 0:0 7:153 7:0}; do
  r=${spec%%:*}; g=${spec#*:}
  run gc_w8r${r}_g$g 400 $GC --rehearse-rank $r --link-gbps $g
done
RG="python -u benchmarks/bench_rgcn.py --dtype fp32 --steps 3 --warmup 1 --rehearse-world 8"
for spec in ${RG_RUNS:-1:153 1:0}; do
  r=${spec%%:*}; g=${spec#*:}
  run rgcn_w8r${r}_g$g 600 $RG --rehearse-rank $r --link-gbps $g
done
