#!/bin/bash
# GraphCast W=8 with the aligned partition (every rank behind the 153 GB/s link model; the
# job's step is the slowest rank), then the full GPU suite + smoke on this tree.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r06/gc
O=gpurun_out/r06/gc
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() {
  local name=$1; shift
  timeout -k 10 300 python -u benchmarks/bench_graphcast.py --mode step --steps 20 --warmup 3 "$@" \
    > $O/$name.log 2>&1
  local rc=$?
  grep '^{' $O/$name.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$name', round(d['ms_per_step'],2), d.get('launch'), d.get('partition'), d.get('halo_rows'), d.get('local_grid'), d.get('local_mesh'))" || { echo "$name rc=$rc"; tail -3 $O/$name.log; }
  if fatal $rc; then exit $rc; fi
}
for r in 0 1 2 3 4 5 6 7; do
  run w8r${r}_aligned_g153_graph --partition aligned --rehearse-world 8 --rehearse-rank $r --link-gbps 153 --cuda-graph
done
run w8r0_aligned_g153_eager --partition aligned --rehearse-world 8 --rehearse-rank 0 --link-gbps 153
run w8r3_latitude_g153_graph --rehearse-world 8 --rehearse-rank 3 --link-gbps 153 --cuda-graph
bash scripts/gpu_suite.sh; rc=$?; case $rc in 124|134|137|139) exit $rc;; esac
bash scripts/gpu_r06_j.sh
