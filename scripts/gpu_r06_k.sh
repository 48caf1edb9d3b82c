#!/bin/bash
# GraphCast W=8 aligned partition with the fitted cost weights: every rank (graph replay,
# 153 GB/s link model).
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r06/gc
O=gpurun_out/r06/gc
for r in ${RANKS:-0 1 2 3 4 5 6 7}; do
  timeout -k 10 300 python -u benchmarks/bench_graphcast.py --mode step --steps 20 --warmup 3 \
    --partition aligned --rehearse-world 8 --rehearse-rank $r --link-gbps 153 --cuda-graph ${EXTRA:-} \
    > $O/w8r${r}_aligned${TAG:-2}_g153_graph.log 2>&1
  rc=$?
  grep '^{' $O/w8r${r}_aligned${TAG:-2}_g153_graph.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('r$r', round(d['ms_per_step'],2), d.get('halo_rows'), d.get('local_grid'), d.get('local_mesh'))" || { echo "r$r rc=$rc"; tail -3 $O/w8r${r}_aligned${TAG:-2}_g153_graph.log; }
  case $rc in 124|134|137|139) exit $rc;; esac
done
